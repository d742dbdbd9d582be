"""DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY pages — the string encodings parquet-mr's PARQUET_2_0
writer falls back to (bsp/ParquetWriter.java:66). Files are written here by
pyarrow (an independent implementation): multi-page chunks, v1 and v2 pages, nulls, empty strings,
values longer than k_dba_chars' LDS buffers, and LIST<STRING> leaves. The CPU test pins the oracle
to pyarrow's reading of the files; the GPU test compares the HIP path (through the C ABI) with the
oracle bit-exactly."""
import importlib.util
import os

import numpy as np
import pytest

from conftest import GOLDEN
from golden_util import assert_chunk_equal

ENC = {"dlba": "DELTA_LENGTH_BYTE_ARRAY", "dba": "DELTA_BYTE_ARRAY", "dba_long": "DELTA_BYTE_ARRAY",
       "l.list.element": "DELTA_LENGTH_BYTE_ARRAY", "ldba.list.element": "DELTA_BYTE_ARRAY"}
CASES = [("1.0", "none"), ("1.0", "snappy"), ("2.0", "snappy")]


def _make_golden():
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _table(n, seed):
    import pyarrow as pa
    rng = np.random.default_rng(seed)
    letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", np.uint8)

    def word(k):
        return letters[rng.integers(0, 26, k)].tobytes().decode()

    dlba = [None if rng.random() < 0.08 else word(int(rng.integers(0, 41))) for _ in range(n)]
    stems = ["apple", "applesauce", "apply", "band", "bandana", "", "zebra" * 7]
    dba = sorted(stems[int(rng.integers(0, len(stems)))] + str(int(rng.integers(0, 50000))) for _ in range(n))
    dba = [None if rng.random() < 0.05 else v for v in dba]
    base = word(6000)
    longv = []
    for i in range(n):   # long shared prefixes every 97th value (> 4 KiB and > 8 KiB values)
        longv.append(base[: 3000 + (i * 131) % 9000] + word(int(rng.integers(0, 12000 if i % 389 == 0 else 20)))
                     if i % 97 == 0 else word(int(rng.integers(0, 16))))
    lst = [None if rng.random() < 0.1 else [word(int(rng.integers(0, 12))) if rng.random() > 0.05 else None
                                            for _ in range(int(rng.integers(0, 5)))] for _ in range(n)]
    ldba = [None if rng.random() < 0.1 else sorted(word(3) + word(int(rng.integers(0, 5)))
                                                   for _ in range(int(rng.integers(0, 4)))) for _ in range(n)]
    return pa.table({"dlba": pa.array(dlba, pa.string()), "dba": pa.array(dba, pa.string()),
                     "dba_long": pa.array(longv, pa.string()),
                     "l": pa.array(lst, pa.list_(pa.string())), "ldba": pa.array(ldba, pa.list_(pa.string()))})


def _write(tmp_path, version, compression, n=30000, seed=11):
    import pyarrow.parquet as pq
    path = str(tmp_path / f"delta_{version}_{compression}.parquet")
    pq.write_table(_table(n, seed), path, compression=compression, use_dictionary=False, column_encoding=ENC,
                   data_page_version=version, data_page_size=64 << 10, row_group_size=n // 2)
    md = pq.ParquetFile(path).metadata
    for c in range(md.num_columns):
        encs = set(md.row_group(0).column(c).encodings)
        assert encs & {"DELTA_LENGTH_BYTE_ARRAY", "DELTA_BYTE_ARRAY"}, (md.row_group(0).column(c).path_in_schema, encs)
    return path


@pytest.mark.parametrize("version,compression", CASES)
def test_oracle_matches_pyarrow(oracle, tmp_path, version, compression):
    import pyarrow.parquet as pq
    mg = _make_golden()
    path = _write(tmp_path, version, compression)
    pf = pq.ParquetFile(path)
    with oracle.open(path) as of:
        for rg in range(pf.metadata.num_row_groups):
            tbl = pf.read_row_group(rg)
            for c in range(pf.metadata.num_columns):
                exp = mg.expected_for_column(tbl, pf.metadata, c)
                o = of.decode(rg, c)
                assert o["status"] == 0, (rg, c, o.get("error"))
                assert_chunk_equal(o, exp, f"oracle v{version} {compression} rg{rg} c{c}")


@pytest.mark.gpu
@pytest.mark.parametrize("version,compression", CASES)
def test_gpu_matches_oracle(oracle, tmp_path, version, compression):
    from pfloor.decoder import GpuDecoder, decode_file
    path = _write(tmp_path, version, compression)
    with GpuDecoder(0) as dec:
        got = decode_file(path, decoder=dec)
    with oracle.open(path) as of:
        for rg in range(of.num_row_groups):
            for c in range(of.num_columns):
                g = got[(rg, c)]
                assert g["status"] == 0, (rg, c, got["_error"])
                assert_chunk_equal(g, of.decode(rg, c), f"gpu v{version} {compression} rg{rg} c{c}")


@pytest.mark.gpu
def test_gpu_corrupt_delta_pages(oracle, tmp_path):
    """Byte damage inside uncompressed DLBA / DBA pages (length streams, prefixes, data): each chunk
    decodes bit-exactly like the oracle or reports an error; the GPU never faults."""
    from pfloor.decoder import GpuDecoder, decode_file
    from test_gpu_parity import _corrupt_variants
    import pyarrow.parquet as pq
    path = str(tmp_path / "delta_small.parquet")
    pq.write_table(_table(4000, 5), path, compression="none", use_dictionary=False, column_encoding=ENC,
                   data_page_version="1.0", data_page_size=8 << 10)
    data = open(path, "rb").read()
    rng = np.random.default_rng(9)
    agree = 0
    with GpuDecoder(0) as dec:
        for i, bad in enumerate(_corrupt_variants(data, rng, 12)):
            p = tmp_path / f"bad_{i}.parquet"
            p.write_bytes(bad)
            try:
                got = decode_file(str(p), decoder=dec)
            except Exception:
                continue   # metadata-level rejection on the host
            try:
                of = oracle.open(str(p))
            except Exception:
                of = None
            try:
                for k, v in got.items():
                    if not isinstance(k, tuple):
                        continue
                    assert v["status"] in (0, -2, -3, -6), v["status"]
                    o = of.decode(*k) if of is not None else {"status": -2}
                    if v["status"] == 0 and o["status"] == 0:
                        assert_chunk_equal(v, o, f"corrupt {i} {k}")
                        agree += 1
            finally:
                if of is not None:
                    of.close()
        assert decode_file(path, decoder=dec)["_status"] == 0   # still healthy afterwards
    assert agree > 0

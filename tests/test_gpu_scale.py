"""GPU parity at BASELINE config shapes beyond the golden miniatures, through the C ABI, bit-exact
against the CPU oracle:
  * config 4 at shape: 500 nullable INT32/FLOAT columns, 30 % nulls, per-column pools of 100,000
    values, 100,000 rows (dictionary pages larger than the 160 KiB of LDS), one batch of 500 chunks;
  * the serial Snappy kernel striding over many jobs: every third Snappy page of a lineitem-shaped
    row group forced onto k_snappy_serial (PF_DEBUG_FORCE_SERIAL), so jobs far past its 64-block
    grid are decoded by later iterations of the grid-stride loop;
  * config 3 (4,000,000-row row groups) sharded over two processes: see test_gpu_shard.py."""
import os

import numpy as np
import pytest

from golden_util import assert_chunk_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def decoder():
    from pfloor.decoder import GpuDecoder
    d = GpuDecoder(0)
    yield d
    d.close()


def _check_all(got, oracle, path, label):
    n = 0
    with oracle.open(path) as of:
        for key, g in got.items():
            if not isinstance(key, tuple):
                continue
            assert g["status"] == 0, (label, key, got["_error"])
            assert_chunk_equal(g, of.decode(*key), f"{label} rg{key[0]} c{key[1]}")
            n += 1
    return n


def test_wide_config4_shape(decoder, oracle, tmp_path):
    import pyarrow.parquet as pq
    from pfloor import datagen
    from pfloor.decoder import ParquetFile, decode_file
    path = str(tmp_path / "wide_100k.parquet")
    pq.write_table(datagen.wide_table(100_000, ncols=500, pool=100_000, null_frac=0.3, seed=4), path,
                   compression="snappy")
    with ParquetFile(path) as pf:
        assert pf.num_columns == 500
        biggest = 0
        for c in range(pf.num_columns):
            d = pf.chunk_desc(0, c, 0)
            for i in range(d.n_pages):
                if d.pages[i].page_type == 2:
                    biggest = max(biggest, d.pages[i].uncompressed_size)
        assert biggest > 160 * 1024, biggest        # dictionaries spill out of LDS (config 4's point)
    got = decode_file(path, decoder=decoder)
    assert got["_status"] == 0, got["_error"]
    assert _check_all(got, oracle, path, "wide") == 500
    # nulls really are ~30 %
    g = got[(0, 0)]
    valid = np.unpackbits(g["validity"], bitorder="little")[:g["num_slots"]]
    assert 0.25 < 1 - valid.mean() < 0.35


def test_serial_snappy_kernel_many_jobs(oracle, switches):
    import ctypes as C
    from pfloor import _native
    from pfloor.decoder import GpuDecoder, decode_file
    path = os.path.join(os.path.dirname(__file__), "golden", "c2_lineitem.parquet")
    with switches(PF_DEBUG_FORCE_SERIAL=3), GpuDecoder(0) as decoder:
        got = decode_file(path, decoder=decoder)
        assert got["_status"] == 0, got["_error"]
        L = _native.lib()
        L.pf_debug_snappy_fallback.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.c_int]
        nj = L.pf_debug_snappy_fallback(decoder.h, None, 0)
        assert nj > 3 * 64, nj                     # forced jobs reach far past the serial kernel's 64 blocks
        rec = (C.c_int * (5 * nj))()
        assert L.pf_debug_snappy_fallback(decoder.h, rec, nj) == nj
    forced = [j for j in range(nj) if rec[5 * j] == 3]
    assert len(forced) == nj // 3 and max(forced) >= 128
    assert _check_all(got, oracle, path, "forced-serial") > 0


def test_nested_config5_shape(decoder, oracle, tmp_path):
    """BASELINE config 5 at shape: 1,000,000 rows of l optional LIST<STRUCT<a INT64, b UTF8>>,
    `a` DELTA_BINARY_PACKED, `b` dictionary, v2 pages, Snappy (4 row groups; one batch). Values,
    validity, list offsets, list validity and the raw rep/def levels bit-exact against the oracle
    (the reference's own reader stops at "Unexpected repetition": ParquetReader.java:199-202)."""
    import pyarrow.parquet as pq
    from pfloor import datagen
    from pfloor.decoder import decode_file
    path = str(tmp_path / "nested_1m.parquet")
    pq.write_table(datagen.nested_table(1_000_000, seed=5), path, row_group_size=250_000, compression="snappy",
                   data_page_version="2.0", column_encoding={"l.list.element.a": "DELTA_BINARY_PACKED"},
                   use_dictionary=["l.list.element.b"])
    got = decode_file(path, decoder=decoder)
    assert got["_status"] == 0, got["_error"]
    assert _check_all(got, oracle, path, "nested") == 8
    g = got[(0, 0)]
    assert g["num_rows"] == 250_000 and g["num_entries"] > g["num_rows"]   # lists of 0-4 elements
    assert "list_offsets" in g and "rep_levels" in g


def test_flat_config1_shape_uncompressed(decoder, oracle, tmp_path):
    """BASELINE config 1 at shape: 1,000,000 rows (id INT64, x DOUBLE, n nullable INT32, s dictionary
    UTF8), uncompressed (pyarrow compression='NONE'), v1 pages; bit-exact against the oracle."""
    import pyarrow.parquet as pq
    from pfloor import datagen
    from pfloor.decoder import decode_file
    path = str(tmp_path / "flat_1m.parquet")
    pq.write_table(datagen.flat_table(1_000_000, seed=1), path, row_group_size=250_000, compression="NONE")
    got = decode_file(path, decoder=decoder)
    assert got["_status"] == 0, got["_error"]
    assert _check_all(got, oracle, path, "flat") == 16

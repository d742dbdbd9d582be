"""k_snappy_head's two shortcuts, bit-exact against the CPU oracle through the C ABI:
  * DIRECT_VALUES: PLAIN fixed-width pages with every level present are written by the Snappy
    executor straight into the column's values (v1 pages with the level section in the first
    literal, v2 pages, required columns); pages with nulls, BOOLEAN and dictionary pages are not;
  * DIRECT_INPLACE: data pages whose Snappy stream is one literal (incompressible dictionary ids)
    are read in place from the compressed input, with no parse or executor work;
  * direct pages whose executor run is rejected (PF_DEBUG_FORCE_REDO) are decoded from the
    redo's scratch body instead, still bit-exact.
Reference path: DecompressorStream.java:101-173 (Snappy) -> ParquetReader.java:146-161 (values)."""
import ctypes as C
import os

import numpy as np
import pytest

from golden_util import assert_chunk_equal

pytestmark = pytest.mark.gpu

DIRECT_NONE, DIRECT_VALUES, DIRECT_INPLACE = 0, 1, 2


@pytest.fixture(scope="module")
def decoder():
    from pfloor.decoder import GpuDecoder
    d = GpuDecoder(0)
    yield d
    d.close()


def _file(tmp_path, version):
    import pyarrow as pa
    import pyarrow.parquet as pq
    rng = np.random.default_rng(11)
    n = 300_000
    okey = np.sort(rng.integers(1, 4 * n, n)).astype(np.int64)        # compressible, sorted
    price = np.round(rng.uniform(900.0, 100000.0, n), 2)                # doubles, few repeats
    i32 = rng.integers(0, 1 << 20, n).astype(np.int32)
    f32 = rng.random(n).astype(np.float32)
    nul = rng.integers(0, 1 << 30, n).astype(np.int64)
    ids = rng.integers(0, 5000, n).astype(np.int64)                     # dictionary: random ids
    flags = rng.random(n) < 0.5
    t = pa.table({
        "okey": pa.array(okey),                                          # optional, no nulls
        "price": pa.array(price),
        "i32": pa.array(i32),
        "f32": pa.array(f32),
        "req": pa.array(okey + 7),                                       # required (max_def 0)
        "nul": pa.array(nul, mask=rng.random(n) < 0.1),                  # nulls: never direct
        "ids": pa.array(ids),
        "flag": pa.array(flags),                                         # BOOLEAN: never direct
    }, schema=pa.schema([pa.field("okey", pa.int64()), pa.field("price", pa.float64()),
                         pa.field("i32", pa.int32()), pa.field("f32", pa.float32()),
                         pa.field("req", pa.int64(), nullable=False), pa.field("nul", pa.int64()),
                         pa.field("ids", pa.int64()), pa.field("flag", pa.bool_())]))
    path = str(tmp_path / f"direct_{version}.parquet")
    pq.write_table(t, path, compression="snappy", data_page_version=version, row_group_size=150_000,
                   use_dictionary=["ids"])
    return path


def _direct(decoder):
    from pfloor import _native
    L = _native.lib()
    L.pf_debug_page_direct.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.c_int]
    n = L.pf_debug_page_direct(decoder.h, None, 0)
    out = (C.c_int * n)()
    assert L.pf_debug_page_direct(decoder.h, out, n) == n
    return list(out)


def _check(got, oracle, path, label):
    n = 0
    with oracle.open(path) as of:
        for key, g in got.items():
            if not isinstance(key, tuple):
                continue
            assert g["status"] == 0, (label, key, got["_error"])
            assert_chunk_equal(g, of.decode(*key), f"{label} rg{key[0]} c{key[1]}")
            n += 1
    return n


@pytest.mark.parametrize("version", ["1.0", "2.0"])
def test_direct_and_inplace_pages(decoder, oracle, tmp_path, version):
    from pfloor.decoder import decode_file
    path = _file(tmp_path, version)
    got = decode_file(path, decoder=decoder, row_groups=[0])
    assert got["_status"] == 0, got["_error"]
    assert _check(got, oracle, path, f"direct v{version}") == 8
    d = _direct(decoder)
    assert d.count(DIRECT_VALUES) >= 5, d      # okey / price / i32 / f32 / req pages
    if version == "1.0":   # random dictionary ids do not compress (v2: Arrow may store them uncompressed)
        assert d.count(DIRECT_INPLACE) >= 1, d


def test_direct_pages_through_the_redo_path(oracle, tmp_path, switches):
    from pfloor.decoder import GpuDecoder, decode_file
    path = _file(tmp_path, "1.0")
    with switches(PF_DEBUG_FORCE_REDO=2), GpuDecoder(0) as decoder:
        got = decode_file(path, decoder=decoder)
        assert got["_status"] == 0, got["_error"]
        assert _check(got, oracle, path, "forced redo") == 16
        from pfloor import _native
        L = _native.lib()
        L.pf_debug_snappy_fallback.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.c_int]
        nj = L.pf_debug_snappy_fallback(decoder.h, None, 0)
        rec = (C.c_int * (5 * nj))()
        L.pf_debug_snappy_fallback(decoder.h, rec, nj)
        d = _direct(decoder)
    redone = [rec[5 * j + 4] for j in range(nj) if rec[5 * j] == 2]
    assert any(d[p] == DIRECT_VALUES for p in redone)   # accepted as direct, then decoded from scratch


# Streams of literals only (k_snappy_head -> k_snappy_litcopy, no parse / executor): Snappy emits one
# literal per 64 KiB block of incompressible input, so a 400 KB dictionary of random values is ~7
# literals and a 160 KB data page of random doubles 3. Dictionary pages and data pages that did not
# compress are copied from the literal table; the result must equal the oracle's decode.
FB_LITCOPY = 5


@pytest.mark.parametrize("version", ["1.0", "2.0"])
def test_multi_literal_pages(decoder, oracle, tmp_path, version):
    import pyarrow as pa
    import pyarrow.parquet as pq
    from pfloor import _native
    from pfloor.decoder import decode_file
    rng = np.random.default_rng(23)
    n = 120_000
    pool = rng.integers(-2**31, 2**31, 100_000, dtype=np.int64).astype(np.int32)   # 400 KB dictionary
    t = pa.table({
        "dict_i32": pa.array(pool[rng.integers(0, len(pool), n)], mask=rng.random(n) < 0.3),
        "rnd_f64": pa.array(rng.random(n)),                                          # PLAIN, incompressible
        "rnd_nul": pa.array(rng.random(n), mask=rng.random(n) < 0.2),
    })
    path = str(tmp_path / f"lits_{version}.parquet")
    pq.write_table(t, path, compression="snappy", data_page_version=version, row_group_size=n,
                   use_dictionary=["dict_i32"], data_page_size=1 << 20)
    got = decode_file(path, decoder=decoder)
    assert got["_status"] == 0, got["_error"]
    assert _check(got, oracle, path, f"literals v{version}") == 3
    L = _native.lib()
    L.pf_debug_snappy_fallback.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.c_int]
    nj = L.pf_debug_snappy_fallback(decoder.h, None, 0)
    rec = (C.c_int * (5 * nj))()
    L.pf_debug_snappy_fallback(decoder.h, rec, nj)
    lit = [rec[5 * j + 2] for j in range(nj) if rec[5 * j] == FB_LITCOPY]
    assert any(d > 65536 for d in lit), [rec[5 * j:5 * j + 5] for j in range(nj)]   # multi-literal pages copied

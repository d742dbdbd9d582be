"""Nullable flat fixed-width pages (k_page_null, round 4): one workgroup per page does the level-run
parse, the present-bit scan, the dictionary-id extraction and the gathers of all its 4096-entry
blocks. Columns of every width it takes (INT32 / INT64 / FLOAT / DOUBLE), dictionary and PLAIN,
null fractions from none to all, pages of one block to 16 blocks with ragged tails, v1 / v2 pages,
decoded on the GPU and compared with the CPU oracle bit-exactly; the page-done flags show which
kernel took each page (pages past its limits fall back to k_lvl + k_flat_null). Reference path:
ParquetReader.java:139-177 (the column readers behind streamContent) over
RunLengthBitPackingHybridDecoder levels and dictionary ids."""
import ctypes as C

import numpy as np
import pytest

from golden_util import assert_chunk_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def page_null_on():
    """k_page_null is opt-in (a diagnostics-build option, PF_PAGE_NULL=1 read at pf_ctx_create): this
    module runs on the diagnostics build with it on."""
    import os
    from pfloor import _native
    old = os.environ.get("PF_PAGE_NULL")
    os.environ["PF_PAGE_NULL"] = "1"
    try:
        with _native.diagnostics():
            yield
    finally:
        if old is None:
            os.environ.pop("PF_PAGE_NULL", None)
        else:
            os.environ["PF_PAGE_NULL"] = old


@pytest.fixture(scope="module")
def decoder():
    from pfloor.decoder import GpuDecoder
    d = GpuDecoder(0)
    yield d
    d.close()


def _done(decoder):
    """(done flags, k_lvl fit word) per page of the decoder's last decode (pf_debug_page_done)."""
    from pfloor import _native
    L = _native.lib()
    L.pf_debug_page_done.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.c_int]
    n = L.pf_debug_page_done(decoder.h, None, 0)
    out = (C.c_int * (2 * n))()
    assert L.pf_debug_page_done(decoder.h, out, n) == n
    return [tuple(out[2 * i:2 * i + 2]) for i in range(n)]


TYPES = {"i32": np.int32, "i64": np.int64, "f32": np.float32, "f64": np.float64}


@pytest.mark.parametrize("typ", sorted(TYPES))
@pytest.mark.parametrize("dictionary", [True, False])
@pytest.mark.parametrize("null_frac", [0.0, 0.3, 0.97, 1.0])
@pytest.mark.parametrize("version", ["1.0", "2.0"])
def test_page_null(decoder, oracle, tmp_path, typ, dictionary, null_frac, version):
    import pyarrow as pa
    import pyarrow.parquet as pq
    from pfloor.decoder import decode_file
    rng = np.random.default_rng(hash((typ, dictionary, null_frac, version)) % 2**32)
    n = 70_000
    pool = rng.integers(-2**31, 2**31 - 1, 5000).astype(TYPES[typ]) if typ[0] == "i" else \
        rng.standard_normal(5000).astype(TYPES[typ])
    vals = pool[rng.integers(0, len(pool), n)]
    mask = rng.random(n) < null_frac
    # runs of nulls and of present values too (RLE level runs between bit-packed ones)
    mask[1000:3000] = True
    mask[5000:9000] = False
    t = pa.table({"c": pa.array(vals, mask=mask)})
    path = str(tmp_path / f"pn_{typ}_{dictionary}_{null_frac}_{version}.parquet")
    # pages of 20,000 rows (pyarrow's row limit: 5 blocks, the last ragged) and one small page size
    pq.write_table(t, path, compression="snappy", data_page_version=version, use_dictionary=dictionary,
                   row_group_size=n, data_page_size=64 << 10 if null_frac == 0.3 else 1 << 20)
    got = decode_file(path, decoder=decoder)
    assert got["_status"] == 0, got["_error"]
    with oracle.open(path) as of:
        assert_chunk_equal(got[(0, 0)], of.decode(0, 0), f"{typ} dict={dictionary} nulls={null_frac} v{version}")
    flags = _done(decoder)
    if 0 < null_frac < 1:   # data pages with nulls: k_page_null (DONE_NULL, no k_lvl table)
        taken = [f for f in flags if f[0] & 4 and f[1] == 0]
        assert taken, flags


def test_page_null_many_runs(decoder, oracle, tmp_path):
    """Alternating null / present runs of 8-16 entries: more level runs than k_page_null holds
    (PN_RUNS) on long pages -> those pages fall back; results identical either way."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from pfloor.decoder import decode_file
    rng = np.random.default_rng(7)
    n = 60_000
    lens = rng.integers(8, 17, n // 8)
    mask = np.repeat(np.arange(len(lens)) % 2 == 0, lens)[:n]
    vals = rng.integers(0, 100, n).astype(np.int64)
    t = pa.table({"c": pa.array(vals, mask=mask)})
    path = str(tmp_path / "pn_runs.parquet")
    pq.write_table(t, path, compression="snappy", row_group_size=n, data_page_size=1 << 20)
    got = decode_file(path, decoder=decoder)
    assert got["_status"] == 0, got["_error"]
    with oracle.open(path) as of:
        assert_chunk_equal(got[(0, 0)], of.decode(0, 0), "many level runs")


@pytest.mark.parametrize("page_null", ["0", "1"])
def test_null_blocks_staggered(oracle, tmp_path, switches, page_null):
    """Blocks after a page's first start only once it has finished (PF_DEBUG_NULL_STAGGER), with
    k_page_null off (every page through k_lvl + k_flat_null) and on: bit-exact vs the oracle. r04
    regression: a k_flat_null block skipped its page (values and count lost) once a sibling block
    had finished and set DONE_NULL -- under the bench's four streams most config-4 runs hit it;
    k_page_null now marks the pages it decodes DONE_PAGE and k_flat_null tests only that."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from pfloor.decoder import decode_file
    rng = np.random.default_rng(5)
    n = 60_000
    cols = {}
    for c, typ in enumerate((np.int32, np.int64, np.float64)):
        pool = rng.integers(-2**31, 2**31 - 1, 3000).astype(typ)
        cols[f"c{c}"] = pa.array(pool[rng.integers(0, len(pool), n)], mask=rng.random(n) < 0.3)
    cols["p"] = pa.array(rng.integers(0, 1 << 40, n), mask=rng.random(n) < 0.3)   # PLAIN (no dictionary)
    path = str(tmp_path / "stagger.parquet")
    pq.write_table(pa.table(cols), path, compression="snappy", row_group_size=n,
                   use_dictionary=["c0", "c1", "c2"])
    with switches(PF_PAGE_NULL=page_null, PF_DEBUG_NULL_STAGGER=100):
        got = decode_file(path)
    assert got["_status"] == 0, got["_error"]
    with oracle.open(path) as of:
        for c in range(4):
            assert_chunk_equal(got[(0, c)], of.decode(0, c), f"column {c} page_null={page_null}")


@pytest.mark.parametrize("stagger", ["0", "100"])
def test_null_fallback_queue(oracle, tmp_path, switches, stagger):
    """Pages k_flat_null does not take go to its fallback queue and the fallback queue (k_flat_all's last workgroups) decodes them (round 5:
    k_flat_all no longer walks the nullable blocks). PF_NULL_DCAP=16 leaves no room for any block's
    level bytes, so k_lvl refuses every nullable page (fit word 0) and all of them take that path;
    INT32 / INT64 / DOUBLE dictionary columns and a PLAIN INT64 one, 30 % nulls, bit-exact."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from pfloor.decoder import GpuDecoder, decode_file
    rng = np.random.default_rng(11)
    n = 50_000
    cols = {}
    for c, typ in enumerate((np.int32, np.int64, np.float64)):
        pool = rng.integers(-2**31, 2**31 - 1, 2000).astype(typ)
        cols[f"c{c}"] = pa.array(pool[rng.integers(0, len(pool), n)], mask=rng.random(n) < 0.3)
    cols["p"] = pa.array(rng.integers(0, 1 << 40, n), mask=rng.random(n) < 0.3)
    path = str(tmp_path / "fbq.parquet")
    pq.write_table(pa.table(cols), path, compression="snappy", row_group_size=n, use_dictionary=["c0", "c1", "c2"])
    with switches(PF_PAGE_NULL="0", PF_NULL_DCAP="16", PF_DEBUG_NULL_STAGGER=stagger):
        d = GpuDecoder(0)
        try:
            got = decode_file(path, decoder=d)
            flags = _done(d)
        finally:
            d.close()
    assert got["_status"] == 0, got["_error"]
    with oracle.open(path) as of:
        for c in range(4):
            assert_chunk_equal(got[(0, c)], of.decode(0, c), f"column {c} via the fallback queue")
    nullable = [f for f in flags if f[0] & 4 or f[1] != 0]
    assert not nullable, flags   # no page was taken by k_flat_null / k_page_null


@pytest.mark.parametrize("page_null", ["0", "1"])
def test_null_blocks_concurrent(tmp_path, page_null):
    """Two contexts decoding nullable multi-block pages at once, with k_page_null off (every page
    through k_lvl + k_flat_null) and on: bit-exact vs the oracle every time. r04 regression: a
    k_flat_null block skipped its page (values and count lost) when a sibling block of the same
    page had already finished and set DONE_NULL; k_page_null now marks its pages DONE_PAGE."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, PF_PAGE_NULL=page_null)
    w = os.path.join(os.path.dirname(os.path.abspath(__file__)), "null_race_worker.py")
    r = subprocess.run([sys.executable, w, str(tmp_path / "race.parquet")], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])

"""Nested pages decoded in segments (k_nest_lvl / k_count_seg / k_nest_scan / k_nest_ids /
k_nest_chars / k_decode_seg, pf_pages.hip): each segment of a page starts from checkpoints of the
rep, def and dictionary-id streams instead of walking the page from its first entry. PF_NEST_SEG
forces the segment path on every eligible nested page with short segments (runs cut mid-way, segments
without values, segment bounds off the 512-entry tiles), and the results must equal the oracle's,
the golden vectors and the whole-page path's, bit for bit; damaged pages must report the same
status either way. Reference path: ParquetReader.java:176-212 (repetition levels -> lists)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_files
from golden_util import assert_chunk_equal, load_expected

pytestmark = pytest.mark.gpu

SEGS = ["64", "500", "4096"]


def _decode(switches, path, seg, decoder=None):
    """Decode with the product library (seg None: default segments) or with a forced segment length
    (PF_NEST_SEG, the diagnostics build; a decoder of its own)."""
    from pfloor.decoder import decode_file
    if seg is None:
        return decode_file(path, decoder=decoder)
    with switches(PF_NEST_SEG=seg):
        return decode_file(path)


@pytest.fixture(scope="module")
def decoder():
    from pfloor.decoder import GpuDecoder
    d = GpuDecoder(0)
    yield d
    d.close()


@pytest.mark.parametrize("seg", SEGS)
def test_golden_files_in_segments(oracle, switches, seg):
    for name in golden_files():
        path = os.path.join(GOLDEN, name + ".parquet")
        exp = load_expected(name)
        got = _decode(switches, path, seg)
        with oracle.open(path) as of:
            for key, e in sorted(exp.items()):
                g = got[key]
                label = f"{name} rg{key[0]} c{key[1]} {e['path']} seg={seg}"
                assert g["status"] == 0, (label, got["_error"])
                assert_chunk_equal(g, e, label + " [golden]")
                assert_chunk_equal(g, of.decode(*key), label + " [oracle]")


def _nested_file(tmp_path, v2, rows=60000, seed=21):
    """LIST<INT32 dict>, LIST<UTF8 dict>, LIST<INT64 DBP>, LIST<DOUBLE PLAIN>, LIST<LIST<INT32>>,
    optional lists with null lists / elements / empty lists, runs of repeated lengths (RLE level
    runs) next to random ones (bit-packed), pages of ~20K entries."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    rng = np.random.default_rng(seed)
    lens = np.where(rng.random(rows) < 0.5, rng.integers(0, 6, rows), 3)
    lens[rows // 3: rows // 3 + 5000] = 0                    # a long stretch of empty lists
    null_list = rng.random(rows) < 0.08
    lens = np.where(null_list, 0, lens)
    m = int(lens.sum())
    offs = np.zeros(rows + 1, dtype=np.int32)
    offs[1:] = np.cumsum(lens)

    def lst(values, mask):
        return pa.ListArray.from_arrays(pa.array(offs), pa.array(values, mask=mask), mask=pa.array(null_list))

    ints = (rng.integers(0, 40, m)).astype(np.int32)
    vocab = np.array(["", "a", "bb", "ccc", "dddd-long-word", "e" * 40] + [f"w{i}" for i in range(300)])
    strs = vocab[rng.integers(0, len(vocab), m)]
    big = (np.arange(m, dtype=np.int64) * 13 + rng.integers(-5, 6, m)).astype(np.int64)
    dbl = rng.random(m)
    inner_lens = rng.integers(0, 4, m)
    inner_offs = np.zeros(m + 1, dtype=np.int32)
    inner_offs[1:] = np.cumsum(inner_lens)
    inner = pa.ListArray.from_arrays(pa.array(inner_offs), pa.array(rng.integers(-9, 9, int(inner_lens.sum())).astype(np.int32)),
                                     mask=pa.array(rng.random(m) < 0.1))
    t = pa.table({
        "li": lst(ints, rng.random(m) < 0.1),
        "ls": lst(strs, rng.random(m) < 0.1),
        "ld": lst(big, rng.random(m) < 0.05),
        "lf": lst(dbl, None),
        "ll": pa.ListArray.from_arrays(pa.array(offs), inner, mask=pa.array(null_list)),
    })
    path = str(tmp_path / f"nest_seg_{int(v2)}.parquet")
    pq.write_table(t, path, compression="snappy", row_group_size=rows // 2, data_page_version="2.0" if v2 else "1.0",
                   use_dictionary=["li.list.element", "ls.list.element"],
                   column_encoding={"ld.list.element": "DELTA_BINARY_PACKED"}, data_page_size=64 << 10)
    return path


@pytest.mark.parametrize("v2", [False, True])
@pytest.mark.parametrize("seg", [None, "300", "2048"])
def test_generated_nested_in_segments(decoder, oracle, switches, tmp_path, v2, seg):
    path = _nested_file(tmp_path, v2)
    got = _decode(switches, path, seg, decoder)
    with oracle.open(path) as of:
        for rg in range(of.num_row_groups):
            for c in range(of.num_columns):
                g = got[(rg, c)]
                assert g["status"] == 0, (rg, c, got["_error"])
                assert_chunk_equal(g, of.decode(rg, c), f"nest rg{rg} c{c} v2={v2} seg={seg}")


def test_damaged_nested_pages_same_status(decoder, switches, tmp_path):
    """Byte damage in nested page bodies: the segment path reports what the whole-page path
    reports (same status per chunk, same data when both decode) and never faults."""
    from pfloor.decoder import decode_file
    from test_gpu_parity import _corrupt_variants
    rng = np.random.default_rng(5)
    data = open(os.path.join(GOLDEN, "c5_nested.parquet"), "rb").read()
    for i, bad in enumerate(_corrupt_variants(data, rng, 8)):
        p = tmp_path / f"c5_bad_{i}.parquet"
        p.write_bytes(bad)
        res = {}
        for seg in ("0", "100"):
            try:
                res[seg] = _decode(switches, str(p), seg)
            except Exception as e:   # metadata-level rejection on the host
                res[seg] = repr(e)
        a, b = res["0"], res["100"]
        if isinstance(a, str) or isinstance(b, str):
            assert a == b
            continue
        for k in a:
            if not isinstance(k, tuple):
                continue
            assert a[k]["status"] == b[k]["status"], (i, k)
            if a[k]["status"] == 0:
                assert_chunk_equal(b[k], a[k], f"damaged {i} {k}")
    got = decode_file(os.path.join(GOLDEN, "ref_roundtrip.parquet"), decoder=decoder)
    assert got["_status"] == 0


def _nested_types_file(tmp_path, rows=30000, seed=33):
    """More leaf types under repetition: FIXED_LEN_BYTE_ARRAY(5), INT96 timestamps, FLOAT, BOOLEAN
    (BOOLEAN pages stay on k_count / k_decode), INT32 dictionary three lists deep, an optional struct
    field two levels down."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    rng = np.random.default_rng(seed)

    def offsets(n, hi, null_p):
        lens = rng.integers(0, hi, n)
        nulls = rng.random(n) < null_p
        lens = np.where(nulls, 0, lens)
        o = np.zeros(n + 1, dtype=np.int32)
        o[1:] = np.cumsum(lens)
        return o, nulls, int(o[-1])

    o, nl, m = offsets(rows, 5, 0.1)
    flba = pa.array([bytes(rng.integers(0, 256, 5, dtype=np.uint8)) for _ in range(m)], type=pa.binary(5),
                    mask=rng.random(m) < 0.1)
    ts = pa.array((rng.integers(0, 2**40, m) * 1000).astype("datetime64[ns]"), mask=rng.random(m) < 0.1)
    fl = pa.array(rng.random(m).astype(np.float32), mask=rng.random(m) < 0.2)
    bo = pa.array(rng.random(m) < 0.5, mask=rng.random(m) < 0.1)
    o2, nl2, m2 = offsets(m, 3, 0.05)
    o3, nl3, m3 = offsets(m2, 3, 0.05)
    deep_vals = pa.array(rng.integers(0, 20, m3).astype(np.int32), mask=rng.random(m3) < 0.1)
    deep = pa.ListArray.from_arrays(pa.array(o3), deep_vals, mask=pa.array(nl3))
    deep = pa.ListArray.from_arrays(pa.array(o2), deep, mask=pa.array(nl2))
    st = pa.StructArray.from_arrays([pa.array(rng.integers(-5, 5, m).astype(np.int64), mask=rng.random(m) < 0.3),
                                     pa.array(rng.random(m), mask=rng.random(m) < 0.3)], names=["x", "y"],
                                    mask=pa.array(rng.random(m) < 0.1))

    def lst(child):
        return pa.ListArray.from_arrays(pa.array(o), child, mask=pa.array(nl))

    t = pa.table({"f": lst(flba), "t": lst(ts), "fl": lst(fl), "b": lst(bo), "d": lst(deep), "s": lst(st)})
    path = str(tmp_path / "nest_types.parquet")
    pq.write_table(t, path, compression="snappy", row_group_size=rows, use_deprecated_int96_timestamps=True,
                   use_dictionary=["d.list.element.list.element.list.element"], data_page_size=32 << 10)
    return path


@pytest.mark.parametrize("seg", [None, "100", "777"])
def test_nested_leaf_types_in_segments(decoder, oracle, switches, tmp_path, seg):
    path = _nested_types_file(tmp_path)
    got = _decode(switches, path, seg, decoder)
    with oracle.open(path) as of:
        for rg in range(of.num_row_groups):
            for c in range(of.num_columns):
                g = got[(rg, c)]
                assert g["status"] == 0, (rg, c, got["_error"])
                assert_chunk_equal(g, of.decode(rg, c), f"types rg{rg} c{c} seg={seg}")


@pytest.mark.parametrize("v2", [False, True])
def test_nest_handover_timeout_whole_page(oracle, switches, tmp_path, v2):
    """A k_nest_lvl hand-over that never comes (a scheduling stall) sends the page to the whole-page
    path (seg_ok = 2: k_count / k_decode decode it) instead of failing the chunk.
    PF_DEBUG_NEST_TIMEOUT=1 makes every hand-over time out: the pages with more than one level
    window take that path, and every chunk is bit-exact vs the oracle."""
    from pfloor.decoder import GpuDecoder, decode_file
    from test_dbp_config import _paths
    path = _nested_file(tmp_path, v2)
    with switches(PF_DEBUG_NEST_TIMEOUT="1"), GpuDecoder(0) as d:
        got = decode_file(path, decoder=d)
        paths = _paths(d)
    assert any(p[2] == 2 for p in paths), paths
    with oracle.open(path) as of:
        for rg in range(of.num_row_groups):
            for c in range(of.num_columns):
                g = got[(rg, c)]
                assert g["status"] == 0, (rg, c, got["_error"])
                assert_chunk_equal(g, of.decode(rg, c), f"nest timeout rg{rg} c{c} v2={v2}")

"""PLAIN BYTE_ARRAY chars (k_flat's span copy, round 4): the chars of a page's values are its body
with the 4-byte length prefixes removed, copied in 64-byte output spans from one round of source
loads. Length mixes that exercise every branch — several values starting in one span, values of
0-3 bytes (two prefixes in one dword: per-chunk fallback), values longer than a span, tile and
block ends, v1 / v2 pages, nulls — decoded on the GPU and compared with the CPU oracle bit-exactly.
Reference path: BinaryPlainValuesReader behind ParquetReader.java:148-151 (getBinary)."""
import numpy as np
import pytest

from golden_util import assert_chunk_equal

pytestmark = pytest.mark.gpu

MIXES = {
    "comments": (10, 44),     # lineitem l_comment-like
    "tiny": (0, 4),           # empty and 1-3 byte values
    "mixed": (0, 120),
    "long": (60, 400),        # several spans per value
    "short": (4, 12),         # up to ~5 value starts per span
}


@pytest.fixture(scope="module")
def decoder():
    from pfloor.decoder import GpuDecoder
    d = GpuDecoder(0)
    yield d
    d.close()


@pytest.mark.parametrize("mix", sorted(MIXES))
@pytest.mark.parametrize("version", ["1.0", "2.0"])
@pytest.mark.parametrize("nulls", [False, True])
def test_plain_strings(decoder, oracle, tmp_path, mix, version, nulls):
    import pyarrow as pa
    import pyarrow.parquet as pq
    from pfloor.decoder import decode_file
    rng = np.random.default_rng(hash((mix, version, nulls)) % 2**32)
    n = 30_000
    lo, hi = MIXES[mix]
    lens = rng.integers(lo, hi, n)
    alphabet = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz ,.0123456789", np.uint8)
    chars = alphabet[rng.integers(0, len(alphabet), int(lens.sum()))].tobytes()
    offs = np.concatenate([[0], np.cumsum(lens)])
    vals = [chars[offs[i]:offs[i + 1]].decode() for i in range(n)]
    mask = (rng.random(n) < 0.2) if nulls else None
    t = pa.table({"s": pa.array(vals, type=pa.string(), mask=mask)})
    path = str(tmp_path / f"plain_{mix}_{version}_{nulls}.parquet")
    pq.write_table(t, path, compression="snappy", data_page_version=version, use_dictionary=False,
                   row_group_size=n, data_page_size=256 << 10)
    got = decode_file(path, decoder=decoder)
    assert got["_status"] == 0, got["_error"]
    with oracle.open(path) as of:
        assert_chunk_equal(got[(0, 0)], of.decode(0, 0), f"plain {mix} v{version} nulls={nulls}")


@pytest.mark.parametrize("version", ["1.0", "2.0"])
def test_plain_strings_rare_long(decoder, oracle, tmp_path, version):
    """Short values with a few long ones (page average under k_ba_tile's 48-byte limit, some values
    past its 124-byte halo): the fused walk cannot link those values, so k_ba_fallback re-links the
    job over its whole candidate bitmap (test_rare_long_values_relinked_not_walked); a second, all-long column in the same batch sends the batch to the round-3 walk
    kernels. Both columns bit-exact vs the oracle (k_ba_tile, round 4)."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from pfloor.decoder import decode_file
    rng = np.random.default_rng(17)
    n = 40_000
    alphabet = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz ,.0123456789", np.uint8)

    def strings(lens):
        chars = alphabet[rng.integers(0, len(alphabet), int(lens.sum()))].tobytes()
        offs = np.concatenate([[0], np.cumsum(lens)])
        return [chars[offs[i]:offs[i + 1]].decode() for i in range(len(lens))]

    short = rng.integers(8, 30, n)
    short[rng.random(n) < 0.01] = rng.integers(200, 900)
    t = pa.table({"a": pa.array(strings(short), type=pa.string()),
                  "b": pa.array(strings(rng.integers(100, 300, n // 8)) * 8, type=pa.string())})
    path = str(tmp_path / f"rare_long_{version}.parquet")
    pq.write_table(t, path, compression="snappy", data_page_version=version, use_dictionary=False,
                   row_group_size=n, data_page_size=256 << 10)
    for cols in ([0], [0, 1]):
        got = decode_file(path, columns=cols, decoder=decoder)
        assert got["_status"] == 0, got["_error"]
        with oracle.open(path) as of:
            for c in cols:
                assert_chunk_equal(got[(0, c)], of.decode(0, c), f"rare long v{version} col {c} of {cols}")


def test_rare_long_values_relinked_not_walked(oracle, tmp_path):
    """a PLAIN string page with a few values longer than k_ba_tile's halo fails the fused
    walk's chain check (BA_RELINK); k_ba_fallback must re-link it from the tiles' candidate words
    (ba_relink_wg), not drop to the exact serial walk -- which needs every tile to write its words even
    after another tile rejected the job. Diagnostics build counters (pf_debug_ba_counts)."""
    import ctypes as C

    import pyarrow as pa
    import pyarrow.parquet as pq
    from pfloor import _native
    from pfloor.decoder import GpuDecoder, decode_file
    rng = np.random.default_rng(23)
    n = 60_000
    alphabet = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz ,.0123456789", np.uint8)
    lens = rng.integers(8, 30, n)
    lens[rng.random(n) < 0.005] = rng.integers(200, 600)
    chars = alphabet[rng.integers(0, len(alphabet), int(lens.sum()))].tobytes()
    offs = np.concatenate([[0], np.cumsum(lens)])
    t = pa.table({"a": pa.array([chars[offs[i]:offs[i + 1]].decode() for i in range(n)], type=pa.string())})
    path = str(tmp_path / "relink.parquet")
    pq.write_table(t, path, compression="snappy", use_dictionary=False, row_group_size=n, data_page_size=1 << 20)
    with _native.diagnostics() as L:
        f = L.pf_debug_ba_counts
        f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
        buf = (C.c_ulonglong * 2)()
        with GpuDecoder(0) as dec:
            assert f(buf, 1) == 0
            got = decode_file(path, decoder=dec)
            assert f(buf, 1) == 0
        assert got["_status"] == 0, got["_error"]
        with oracle.open(path) as of:
            assert_chunk_equal(got[(0, 0)], of.decode(0, 0), "rare long relink")
        relinked, walked = int(buf[0]), int(buf[1])
        assert relinked >= 1 and walked == 0, (relinked, walked)


@pytest.mark.parametrize("nulls", [False, True])
def test_dict_strings_multi_pass_tiles(decoder, oracle, tmp_path, nulls):
    """Dictionary strings averaging ~40 chars: a 2048-value tile holds ~80 KiB of chars, more
    16-byte chunks than the chunk -> value table (CV_CAP), so the copy runs in several table passes
    (round 5; the per-chunk search before). Config 1's 8-24-char vocabulary straddles one pass."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from pfloor.decoder import decode_file
    rng = np.random.default_rng(29 + nulls)
    n = 50_000
    alphabet = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz ,.0123456789", np.uint8)
    vlens = rng.integers(8, 72, 700)
    vocab = [alphabet[rng.integers(0, len(alphabet), int(k))].tobytes().decode() for k in vlens]
    vals = [vocab[i] for i in rng.integers(0, len(vocab), n)]
    mask = (rng.random(n) < 0.15) if nulls else None
    t = pa.table({"s": pa.array(vals, type=pa.string(), mask=mask)})
    path = str(tmp_path / f"dict_long_{nulls}.parquet")
    pq.write_table(t, path, compression="snappy", use_dictionary=True, row_group_size=n)
    got = decode_file(path, decoder=decoder)
    assert got["_status"] == 0, got["_error"]
    with oracle.open(path) as of:
        assert_chunk_equal(got[(0, 0)], of.decode(0, 0), f"dict long nulls={nulls}")


def test_dict_strings_page_over_256_blocks(decoder, oracle, tmp_path):
    """One dictionary string page of 1.5M values: more than 256 blocks of 4096 entries, so
    k_count_flat scans the block chars in several passes of block_excl_scan64 (the
    scan's LDS totals must not be overwritten by a fast wave of the next pass). A required and a
    nullable column, each one data page, bit-exact vs the oracle."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from pfloor.decoder import decode_file
    rng = np.random.default_rng(41)
    n = 1_500_000
    vocab = np.array(["v%05d" % i + "x" * (i % 7) for i in range(40)], dtype=object)
    mask = rng.random(n) < 0.1
    t = pa.table({"s": pa.array(vocab[rng.integers(0, 40, n)], type=pa.string()),
                  "m": pa.array(vocab[rng.integers(0, 40, n)], type=pa.string(), mask=mask)})
    path = str(tmp_path / "dict_big_page.parquet")
    pq.write_table(t, path, compression="snappy", use_dictionary=True, row_group_size=n,
                   data_page_size=64 << 20, max_rows_per_page=n)
    with oracle.open(path) as of:
        for c in range(2):
            pages = of.chunk_pages(0, c)[2]
            assert max(p["num_values"] for p in pages) == n
    got = decode_file(path, decoder=decoder)
    assert got["_status"] == 0, got["_error"]
    with oracle.open(path) as of:
        for c in range(2):
            assert_chunk_equal(got[(0, c)], of.decode(0, c), f"dict big page col {c}")

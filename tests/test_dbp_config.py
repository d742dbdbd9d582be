"""DELTA_BINARY_PACKED block configurations parquet-mr 1.12.2 reads: its DeltaBinaryPackingConfig only
requires the miniblock size (block size / miniblocks) to be a multiple of 8; the format spec's
"block size multiple of 128, miniblock multiple of 32" is a writer rule. Pages written here by a
hand-rolled encoder with (block, miniblocks) = (128, 4), (64, 2), (32, 4), (8, 1) are decoded by the
oracle (CPU) and by the GPU path, bit-exact; (36, 4) (miniblock of 9) and (64, 3) are rejected by
both. Reference path: DeltaBinaryPackingValuesReader behind ParquetReader.java:146-161; the
parquet-mr rule itself is restated from its source (not in this image): parity unpinned beyond it.
The file is assembled with the product's host file writer (pf_writer_*, no GPU) around one
uncompressed v1 page of a REQUIRED INT64 column."""
import ctypes as C
import os

import numpy as np
import pytest


def _uvarint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _zz(v):
    return (v << 1) ^ (v >> 63)


def _wrap(v, bits):
    v &= (1 << bits) - 1
    return v - (1 << bits) if v >> (bits - 1) else v


def _dbp(values, block, nmini, junk_tail=False, bad_block=None, bits=64):
    """parquet-mr's DeltaBinaryPackingValuesWriter[ForLong] layout; bits=32 is the INT32 writer:
    deltas and (delta - min_delta) wrap mod 2^32, as its int arithmetic does."""
    vpm = block // nmini
    out = bytearray(_uvarint(block) + _uvarint(nmini) + _uvarint(len(values)) + _uvarint(_zz(int(values[0])) & (2**64 - 1)))
    deltas = [_wrap(int(values[i]) - int(values[i - 1]), bits) for i in range(1, len(values))]
    for b0 in range(0, len(deltas), block):
        d = deltas[b0:b0 + block]
        mn = min(d)
        out += _uvarint(_zz(mn) & (2**64 - 1))
        rel = [(x - mn) & ((1 << bits) - 1) for x in d]
        widths, data = [], bytearray()
        for m in range(nmini):
            chunk = rel[m * vpm:(m + 1) * vpm]
            w = max((x.bit_length() for x in chunk), default=0)
            if not chunk:
                widths.append(200 if junk_tail else 0)   # unconsumed miniblock: its width is never checked
                continue
            if bad_block is not None and b0 // block == bad_block and m == 0:
                w = bits + 1                                # a width no reader of this type accepts
            widths.append(w)
            if w > bits:
                data += bytes((vpm * 64 + 7) // 8)
                continue
            chunk = chunk + [0] * (vpm - len(chunk))
            acc = 0
            for i, x in enumerate(chunk):
                acc |= x << (i * w)
            data += acc.to_bytes((vpm * w + 7) // 8, "little")
        out += bytes(widths) + data
    return bytes(out)


def _ci32(fid_delta, v):   # compact i32 field: header (delta << 4 | 5) + zigzag varint
    return bytes([(fid_delta << 4) | 5]) + _uvarint((v << 1) ^ (v >> 31))


def _page(body, num_values):
    dph = _ci32(1, num_values) + _ci32(1, 5) + _ci32(1, 3) + _ci32(1, 3) + b"\x00"   # DataPageHeader
    hdr = _ci32(1, 0) + _ci32(1, len(body)) + _ci32(1, len(body)) + bytes([(2 << 4) | 12]) + dph + b"\x00"
    return hdr + body


def _levels(present):
    """v1 definition-level section (bit width 1): 4-byte length + one bit-packed run."""
    n = len(present)
    g = (n + 7) // 8
    bits = np.zeros(g * 8, np.uint8)
    bits[:n] = present
    run = _uvarint((g << 1) | 1) + np.packbits(bits, bitorder="little").tobytes()
    return len(run).to_bytes(4, "little") + run


def _write(path, values, block, nmini, ptype=2, present=None, **kw):
    """One uncompressed v1 page of a REQUIRED (present None) or OPTIONAL column of ptype (1 INT32,
    2 INT64); values are the non-null entries."""
    from pfloor import _native
    from pfloor.writer import EncodedChunk, WriteField
    L = _native.lib()
    body = _dbp(values, block, nmini, bits=32 if ptype == 1 else 64, **kw)
    n = len(values)
    if present is not None:
        body = _levels(present) + body
        n = len(present)
    page = _page(body, n)
    buf = C.create_string_buffer(page, len(page))
    ch = EncodedChunk()
    ch.bytes = C.cast(buf, C.c_void_p)
    ch.size = len(page)
    ch.total_uncompressed_size = len(page)
    ch.num_values = n
    ch.dictionary_page_offset = -1
    ch.data_page_offset = 0
    ch.n_data_pages = 1
    ch.data_encoding = 5
    ch.codec = 0
    fields = (WriteField * 1)(WriteField(b"v", ptype, int(present is not None), 0))
    w = C.c_void_p()
    assert L.pf_writer_open(path.encode(), C.cast(fields, C.c_void_p), 1, C.byref(w)) == 0
    assert L.pf_writer_add_chunk(w, 0, C.byref(ch)) == 0
    assert L.pf_writer_end_row_group(w, n) == 0
    assert L.pf_writer_close(w) == 0


CONFIGS_OK = [(128, 4), (64, 2), (32, 4), (8, 1), (256, 8)]
CONFIGS_BAD = [(36, 4), (64, 3)]


def _values(n=5000, seed=3):
    rng = np.random.default_rng(seed)
    return np.cumsum(rng.integers(-1000, 5000, n)).astype(np.int64)


@pytest.mark.parametrize("block,nmini", CONFIGS_OK + CONFIGS_BAD)
def test_oracle_dbp_configs(oracle, tmp_path, block, nmini):
    v = _values()
    path = str(tmp_path / f"dbp_{block}_{nmini}.parquet")
    _write(path, v, block, nmini)
    with oracle.open(path) as of:
        got = of.decode(0, 0)
        if (block, nmini) in CONFIGS_BAD:
            assert got["status"] != 0
        else:
            assert got["status"] == 0, got["error"]
            assert np.array_equal(np.frombuffer(got["values"].tobytes(), np.int64), v)


@pytest.mark.gpu
@pytest.mark.parametrize("block,nmini", CONFIGS_OK + CONFIGS_BAD)
def test_gpu_dbp_configs(tmp_path, block, nmini):
    from pfloor.decoder import decode_file
    v = _values()
    path = str(tmp_path / f"dbp_{block}_{nmini}.parquet")
    _write(path, v, block, nmini)
    got = decode_file(path, device=0)
    if (block, nmini) in CONFIGS_BAD:
        assert got["_status"] != 0
    else:
        assert got["_status"] == 0, got["_error"]
        assert np.array_equal(np.frombuffer(got[(0, 0)]["values"].tobytes(), np.int64), v)


# Pages of >= DBP_PAR_MIN (16384) entries take the block-parallel path (k_dbp_pos / k_dbp_blk /
# k_dbp_scan, pf_delta.hip); PF_DBP_PAR=0 sends them to the one-workgroup k_delta. Both must give
# the same values, accept junk widths of unconsumed trailing miniblocks and reject a bad width in a
# middle block (which the parallel path hands back to k_delta).
@pytest.mark.gpu
@pytest.mark.parametrize("block,nmini", CONFIGS_OK)
@pytest.mark.parametrize("par", ["1", "0"])
def test_gpu_dbp_large_pages(tmp_path, switches, block, nmini, par):
    from pfloor.decoder import decode_file
    v = _values(n=60001, seed=block + nmini)
    path = str(tmp_path / f"dbp_big_{block}_{nmini}.parquet")
    _write(path, v, block, nmini, junk_tail=True)
    if par == "1":   # the default: the product library
        got = decode_file(path, device=0)
    else:
        with switches(PF_DBP_PAR=par):
            got = decode_file(path, device=0)
    assert got["_status"] == 0, got["_error"]
    assert np.array_equal(np.frombuffer(got[(0, 0)]["values"].tobytes(), np.int64), v)


@pytest.mark.gpu
@pytest.mark.parametrize("par", ["1", "0"])
def test_gpu_dbp_large_page_bad_width(oracle, tmp_path, switches, par):
    from pfloor.decoder import decode_file
    v = _values(n=40000, seed=9)
    path = str(tmp_path / "dbp_big_bad.parquet")
    _write(path, v, 128, 4, bad_block=100)
    with oracle.open(path) as of:
        assert of.decode(0, 0)["status"] != 0
    if par == "1":
        assert decode_file(path, device=0)["_status"] != 0
    else:
        with switches(PF_DBP_PAR=par):
            assert decode_file(path, device=0)["_status"] != 0


def _paths(decoder):
    """{direct, dbp_ok, seg_ok} per page of the decoder's last decode (pf_debug_page_paths)."""
    from pfloor import _native
    L = _native.lib()
    L.pf_debug_page_paths.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.c_int]
    n = L.pf_debug_page_paths(decoder.h, None, 0)
    out = (C.c_int * (3 * n))()
    assert L.pf_debug_page_paths(decoder.h, out, n) == n
    return [tuple(out[3 * i:3 * i + 3]) for i in range(n)]


@pytest.fixture(scope="module")
def decoder():
    from pfloor.decoder import GpuDecoder
    d = GpuDecoder(0)
    yield d
    d.close()


def _i32_wrapping(n, seed):
    """INT32 values over the whole range: most deltas and (delta - min_delta) wrap mod 2^32."""
    rng = np.random.default_rng(seed)
    return rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)


@pytest.mark.parametrize("block,nmini", [(128, 4), (64, 2)])
def test_oracle_dbp_int32_wrap(oracle, tmp_path, block, nmini):
    v = _i32_wrapping(3000, block)
    path = str(tmp_path / "dbp_i32.parquet")
    _write(path, v, block, nmini, ptype=1)
    with oracle.open(path) as of:
        got = of.decode(0, 0)
        assert got["status"] == 0, got["error"]
        assert np.array_equal(np.frombuffer(got["values"].tobytes(), np.int32), v)


# The block-parallel path is asserted to be the one that ran (dbp_ok == 1), not a silent k_delta
# redo: INT32 whose deltas wrap mod 2^32 across block boundaries (block bases summed
# in 64 bits, truncated at the end; min_delta sign-extended from int32), and nullable pages whose
# DBP count (non-null values) is below the page's entry count.
@pytest.mark.gpu
@pytest.mark.parametrize("block,nmini", [(128, 4), (64, 2), (256, 8)])
def test_gpu_dbp_par_int32_wrap(decoder, oracle, tmp_path, block, nmini):
    from golden_util import assert_chunk_equal
    from pfloor.decoder import decode_file
    v = _i32_wrapping(50001, block + 1)
    path = str(tmp_path / f"dbp_i32_{block}.parquet")
    _write(path, v, block, nmini, ptype=1)
    got = decode_file(path, decoder=decoder)
    assert got["_status"] == 0, got["_error"]
    assert np.array_equal(np.frombuffer(got[(0, 0)]["values"].tobytes(), np.int32), v)
    assert [p[1] for p in _paths(decoder)] == [1]
    with oracle.open(path) as of:
        assert_chunk_equal(got[(0, 0)], of.decode(0, 0), "int32 wrap")


@pytest.mark.gpu
@pytest.mark.parametrize("ptype", [1, 2])
def test_gpu_dbp_par_nullable(decoder, oracle, tmp_path, ptype):
    from golden_util import assert_chunk_equal
    from pfloor.decoder import decode_file
    rng = np.random.default_rng(21 + ptype)
    present = (rng.random(70000) >= 0.3).astype(np.uint8)
    nv = int(present.sum())
    v = _i32_wrapping(nv, 5) if ptype == 1 else _values(n=nv, seed=6)
    path = str(tmp_path / f"dbp_null_{ptype}.parquet")
    _write(path, v, 128, 4, ptype=ptype, present=present)
    got = decode_file(path, decoder=decoder)
    assert got["_status"] == 0, got["_error"]
    assert [p[1] for p in _paths(decoder)] == [1]
    with oracle.open(path) as of:
        exp = of.decode(0, 0)
        assert exp["status"] == 0, exp["error"]
        assert_chunk_equal(got[(0, 0)], exp, "nullable dbp")
    vals = np.frombuffer(got[(0, 0)]["values"].tobytes(), np.int32 if ptype == 1 else np.int64)
    assert np.array_equal(vals[present.astype(bool)], v)


@pytest.mark.gpu
@pytest.mark.parametrize("block,nmini", CONFIGS_OK)
def test_gpu_dbp_large_pages_took_parallel_path(tmp_path, switches, block, nmini):
    from pfloor.decoder import GpuDecoder, decode_file
    v = _values(n=60001, seed=block + nmini)
    path = str(tmp_path / f"dbp_big_{block}_{nmini}.parquet")
    _write(path, v, block, nmini, junk_tail=True)
    for par, want in (("1", 1), ("0", 0)):
        with switches(PF_DBP_PAR=par), GpuDecoder(0) as decoder:
            got = decode_file(path, decoder=decoder)
            assert got["_status"] == 0, got["_error"]
            assert np.array_equal(np.frombuffer(got[(0, 0)]["values"].tobytes(), np.int64), v)
            assert [p[1] for p in _paths(decoder)] == [want], par

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


def _dbp(values, block, nmini, junk_tail=False, bad_block=None):
    vpm = block // nmini
    out = bytearray(_uvarint(block) + _uvarint(nmini) + _uvarint(len(values)) + _uvarint(_zz(int(values[0])) & (2**64 - 1)))
    deltas = [(int(values[i]) - int(values[i - 1])) for i in range(1, len(values))]
    for b0 in range(0, len(deltas), block):
        d = deltas[b0:b0 + block]
        mn = min(d)
        out += _uvarint(_zz(mn) & (2**64 - 1))
        rel = [x - mn for x in d]
        widths, data = [], bytearray()
        for m in range(nmini):
            chunk = rel[m * vpm:(m + 1) * vpm]
            w = max((x.bit_length() for x in chunk), default=0)
            if not chunk:
                widths.append(200 if junk_tail else 0)   # unconsumed miniblock: its width is never checked
                continue
            if bad_block is not None and b0 // block == bad_block and m == 0:
                w = 65                                      # a width no INT64 reader accepts
            widths.append(w)
            if w > 64:
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


def _write(path, values, block, nmini, **kw):
    from pfloor import _native
    from pfloor.writer import EncodedChunk, WriteField
    L = _native.lib()
    page = _page(_dbp(values, block, nmini, **kw), len(values))
    buf = C.create_string_buffer(page, len(page))
    ch = EncodedChunk()
    ch.bytes = C.cast(buf, C.c_void_p)
    ch.size = len(page)
    ch.total_uncompressed_size = len(page)
    ch.num_values = len(values)
    ch.dictionary_page_offset = -1
    ch.data_page_offset = 0
    ch.n_data_pages = 1
    ch.data_encoding = 5
    ch.codec = 0
    fields = (WriteField * 1)(WriteField(b"v", 2, 0, 0))
    w = C.c_void_p()
    assert L.pf_writer_open(path.encode(), C.cast(fields, C.c_void_p), 1, C.byref(w)) == 0
    assert L.pf_writer_add_chunk(w, 0, C.byref(ch)) == 0
    assert L.pf_writer_end_row_group(w, len(values)) == 0
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
def test_gpu_dbp_large_pages(tmp_path, monkeypatch, block, nmini, par):
    from pfloor.decoder import decode_file
    monkeypatch.setenv("PF_DBP_PAR", par)
    v = _values(n=60001, seed=block + nmini)
    path = str(tmp_path / f"dbp_big_{block}_{nmini}.parquet")
    _write(path, v, block, nmini, junk_tail=True)
    got = decode_file(path, device=0)
    assert got["_status"] == 0, got["_error"]
    assert np.array_equal(np.frombuffer(got[(0, 0)]["values"].tobytes(), np.int64), v)


@pytest.mark.gpu
@pytest.mark.parametrize("par", ["1", "0"])
def test_gpu_dbp_large_page_bad_width(oracle, tmp_path, monkeypatch, par):
    from pfloor.decoder import decode_file
    monkeypatch.setenv("PF_DBP_PAR", par)
    v = _values(n=40000, seed=9)
    path = str(tmp_path / "dbp_big_bad.parquet")
    _write(path, v, 128, 4, bad_block=100)
    with oracle.open(path) as of:
        assert of.decode(0, 0)["status"] != 0
    assert decode_file(path, device=0)["_status"] != 0

"""Dictionary-id streams made of very short runs (RLE runs of 1-3 values, 1-group bit-packed runs):
valid for parquet-mr's RunLengthBitPackingHybridDecoder, never written by parquet-mr or Arrow
(their RLE runs hold >= 8 repeats). A 1,024-entry tile of such a page needs far more runs than
the flat kernels' run table holds (RUN_CAP = 256): the tile shrinks to what one table window
covers and the next window continues (r02 reported these pages as corrupt; with 4,096-entry tiles
even writer-made pages could hit it). Pages are hand-built (REQUIRED INT32 / INT64 columns,
PLAIN dictionary page + RLE_DICTIONARY v1 data pages, uncompressed) and written with the product's
host file writer (pf_writer_*); the oracle (CPU) and the GPU path must agree bit-exactly.
Reference path: DictionaryValuesReader behind ParquetReader.java:151-161."""
import ctypes as C

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


def _ci32(fid_delta, v):
    return bytes([(fid_delta << 4) | 5]) + _uvarint((v << 1) ^ (v >> 31))


def _dict_page(values):
    body = values.tobytes()
    dph = _ci32(1, len(values)) + _ci32(1, 0) + b"\x00"                       # DictionaryPageHeader: n, PLAIN
    hdr = _ci32(1, 2) + _ci32(1, len(body)) + _ci32(1, len(body)) + bytes([(4 << 4) | 12]) + dph + b"\x00"
    return hdr + body


def _data_page(ids, bw, rng):
    """RLE_DICTIONARY body: <bit width><hybrid runs>: mostly RLE runs of 1-3 values, some 8-value
    bit-packed groups."""
    out = bytearray([bw])
    nb = (bw + 7) // 8
    i, n = 0, len(ids)
    while i < n:
        if rng.random() < 0.2 and i + 8 <= n:
            acc = 0
            for k in range(8):
                acc |= int(ids[i + k]) << (k * bw)
            out += _uvarint((1 << 1) | 1) + acc.to_bytes(bw, "little")
            i += 8
        else:
            c = min(int(rng.integers(1, 4)), n - i)
            out += _uvarint(c << 1) + int(ids[i]).to_bytes(nb, "little")
            ids[i:i + c] = ids[i]                                           # a run repeats its value
            i += c
    body = bytes(out)
    dph = _ci32(1, n) + _ci32(1, 8) + _ci32(1, 3) + _ci32(1, 3) + b"\x00"     # RLE_DICTIONARY
    hdr = _ci32(1, 0) + _ci32(1, len(body)) + _ci32(1, len(body)) + bytes([(2 << 4) | 12]) + dph + b"\x00"
    return hdr + body


def _write(path, ptype, dict_values, pages_ids, bw, rng):
    from pfloor import _native
    from pfloor.writer import EncodedChunk, WriteField
    L = _native.lib()
    dp = _dict_page(dict_values)
    body = bytearray(dp)
    for ids in pages_ids:
        body += _data_page(ids, bw, rng)
    buf = C.create_string_buffer(bytes(body), len(body))
    ch = EncodedChunk()
    ch.bytes = C.cast(buf, C.c_void_p)
    ch.size = len(body)
    ch.total_uncompressed_size = len(body)
    ch.num_values = sum(len(x) for x in pages_ids)
    ch.dictionary_page_offset = 0
    ch.data_page_offset = len(dp)
    ch.n_data_pages = len(pages_ids)
    ch.dict_entries = len(dict_values)
    ch.data_encoding = 8
    ch.codec = 0
    fields = (WriteField * 1)(WriteField(b"v", ptype, 0, 0))
    w = C.c_void_p()
    assert L.pf_writer_open(path.encode(), C.cast(fields, C.c_void_p), 1, C.byref(w)) == 0
    assert L.pf_writer_add_chunk(w, 0, C.byref(ch)) == 0
    assert L.pf_writer_end_row_group(w, ch.num_values) == 0
    assert L.pf_writer_close(w) == 0


def _case(tmp_path, ptype, seed):
    rng = np.random.default_rng(seed)
    dtype = np.int32 if ptype == 1 else np.int64
    nd = 1000
    dict_values = rng.integers(-2**30, 2**30, nd).astype(dtype)
    bw = int(nd - 1).bit_length()
    pages = [rng.integers(0, nd, 20000) for _ in range(3)] + [rng.integers(0, nd, 777)]
    path = str(tmp_path / f"short_runs_{ptype}_{seed}.parquet")
    _write(path, ptype, dict_values, pages, bw, rng)                        # (runs rewrite the id arrays)
    expect = np.concatenate([dict_values[p] for p in pages])
    return path, expect, dtype


@pytest.mark.parametrize("ptype", [1, 2])
def test_oracle_short_runs(oracle, tmp_path, ptype):
    path, expect, dtype = _case(tmp_path, ptype, 7)
    with oracle.open(path) as of:
        got = of.decode(0, 0)
    assert got["status"] == 0, got["error"]
    assert np.array_equal(np.frombuffer(got["values"].tobytes(), dtype), expect)


@pytest.mark.gpu
@pytest.mark.parametrize("ptype", [1, 2])
def test_gpu_short_runs(tmp_path, ptype):
    from pfloor.decoder import decode_file
    path, expect, dtype = _case(tmp_path, ptype, 7)
    got = decode_file(path, device=0)
    assert got["_status"] == 0, got["_error"]
    assert np.array_equal(np.frombuffer(got[(0, 0)]["values"].tobytes(), dtype), expect)

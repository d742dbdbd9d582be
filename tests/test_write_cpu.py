"""Write path, host side (no GPU): the file writer (pf_writer_*: "PAR1", FileMetaData footer in
Thrift compact) and the ctypes mirror of the write-path structs. A column chunk is built here by
hand (one uncompressed v2 PLAIN page with a Thrift compact PageHeader) and the file is read back
with pyarrow (an independent reader) and with the CPU oracle."""
import ctypes as C
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _uvarint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7f) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _zz(v):
    return _uvarint((v << 1) ^ (v >> 63))


def _page_header_v2(n, nulls, enc, def_bytes, values_bytes):
    """PageHeader{1 type=3, 2 uncompressed, 3 compressed, 8 DataPageHeaderV2{...}} (compact)."""
    size = def_bytes + values_bytes
    h = bytearray()
    h += bytes([0x15]) + _zz(3) + bytes([0x15]) + _zz(size) + bytes([0x15]) + _zz(size)
    h += bytes([0x5c])   # field 8 (delta 5), struct
    for fid, v in ((1, n), (2, nulls), (3, n), (4, enc), (5, def_bytes), (6, 0)):
        h += bytes([0x15]) + _zz(v)
    h += bytes([0x12])   # field 7 bool false (is_compressed)
    h += b"\x00\x00"
    return bytes(h)


@pytest.fixture(scope="module")
def W():
    from pfloor import writer
    writer.lib()
    return writer


def _chunk(W, body, n):
    c = W.EncodedChunk()
    buf = C.create_string_buffer(body, len(body))
    c.bytes = C.cast(buf, C.c_void_p)
    c.size = len(body)
    c.total_uncompressed_size = len(body)
    c.num_values = n
    c.dictionary_page_offset = -1
    c.data_page_offset = 0
    c.n_data_pages = 1
    c.data_encoding = 0
    c.codec = 0
    return c, buf


def test_writer_footer_read_by_pyarrow_and_oracle(W, oracle, tmp_path):
    pq = pytest.importorskip("pyarrow.parquet")
    n = 1000
    ids = np.arange(n, dtype=np.int64) * 3 - 7
    body_a = _page_header_v2(n, 0, 0, 0, 8 * n) + ids.tobytes()
    present = (np.arange(n) % 4) != 0
    vals = (np.arange(n, dtype=np.int32) * 5)[present]
    groups = (n + 7) // 8
    defl = _uvarint((groups << 1) | 1) + np.packbits(present, bitorder="little").tobytes()
    body_b = _page_header_v2(n, int((~present).sum()), 0, len(defl), 4 * len(vals)) + defl + vals.tobytes()
    fields = (W.WriteField * 2)(W.WriteField(b"id", W.INT64, 0, 0), W.WriteField(b"v", W.INT32, 1, 0))
    path = str(tmp_path / "h.parquet")
    w = C.c_void_p()
    L = W.lib()
    assert L.pf_writer_open(path.encode(), fields, 2, C.byref(w)) == 0
    ca, ka = _chunk(W, body_a, n)
    cb, kb = _chunk(W, body_b, n)
    assert L.pf_writer_add_chunk(w, 1, C.byref(cb)) != 0          # out of field order
    assert L.pf_writer_add_chunk(w, 0, C.byref(ca)) == 0
    assert L.pf_writer_end_row_group(w, n) != 0                  # a chunk is missing
    assert L.pf_writer_add_chunk(w, 1, C.byref(cb)) == 0
    assert L.pf_writer_end_row_group(w, n) == 0
    assert L.pf_writer_close(w) == 0
    t = pq.read_table(path)
    assert t.schema.field("id").nullable is False and t.schema.field("v").nullable is True
    assert np.array_equal(t.column("id").to_numpy(), ids)
    got = t.column("v").to_pylist()
    assert [g is not None for g in got] == list(present)
    assert [g for g in got if g is not None] == list(vals)
    with oracle.open(path) as of:
        a = of.decode(0, 0)
        assert np.array_equal(np.frombuffer(a["values"].tobytes(), np.int64), ids)


def test_writer_rejects_unsupported_types(W, tmp_path):
    fields = (W.WriteField * 1)(W.WriteField(b"x", 3, 0, 0))   # INT96: ParquetWriter.java:158-159
    w = C.c_void_p()
    assert W.lib().pf_writer_open(str(tmp_path / "x.parquet").encode(), fields, 1, C.byref(w)) == -7


def test_write_struct_layouts_match_header(W, tmp_path):
    import subprocess
    structs = {"pf_encode_column": W.EncodeColumn, "pf_encoded_chunk": W.EncodedChunk, "pf_write_field": W.WriteField}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "pfloor.h"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} SIZEOF %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = {}
    for ln in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        s, f, v = ln.split()
        got[(s, f)] = int(v)
    for cname, py in structs.items():
        assert got[(cname, "SIZEOF")] == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)


def test_record_buffer_follows_write_field(W):
    """SimpleWriteSupport.writeField (ParquetWriter.java:143-160): typed conversion, BINARY only
    as a string, unknown names rejected, REQUIRED fields must be written, OPTIONAL become null."""
    sch = W.MessageType("m", W.required(W.INT64).named("a"), W.optional(W.BINARY).as_string().named("s"),
                        W.required(W.BINARY).named("raw"))
    b = W._RowBuffer(sch)
    b.write("a", 5)
    with pytest.raises(NotImplementedError):
        b.write("raw", "x")
    with pytest.raises(KeyError):
        b.write("nope", 1)
    with pytest.raises(RuntimeError):
        b.end_record()     # required "raw" missing
    sch2 = W.MessageType("m", W.required(W.INT64).named("a"), W.optional(W.BINARY).as_string().named("s"))
    b2 = W._RowBuffer(sch2)
    b2.write("a", 1)
    b2.end_record()
    b2.write("a", 2)
    b2.write("s", "é")
    b2.end_record()
    cols, n = b2.take()
    assert n == 2 and cols[0] == [1, 2] and cols[1] == [None, "é".encode()]
    (offs, chars), val = W.column_arrays(sch2.fields[1], cols[1])
    assert list(offs) == [0, 0, 2] and chars.tobytes() == "é".encode() and list(np.unpackbits(val, bitorder="little")[:2]) == [0, 1]

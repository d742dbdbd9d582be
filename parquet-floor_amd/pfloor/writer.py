"""Host mirror of the reference's write API (src/main/java/blue/strategic/parquet/ParquetWriter.java,
Dehydrator.java, ValueWriter.java) over the GPU write path of libpfloor.so.

ParquetWriter.writeFile(schema, file, dehydrator) -> writer; writer.write(record); writer.close().
Like the reference (ParquetWriter.java:61-68) every column is SNAPPY-compressed with the
PARQUET_2_0 writer settings of parquet-mr 1.12.2: data pages v2 of 20,000 rows, dictionary
encoding with PLAIN fallback above the 1 MiB dictionary page size. Records are buffered per
row group on the host (dehydrated column by column, SimpleWriteSupport.writeField :143-160) and
each column chunk is encoded on the GPU (pf_encode_chunk: dictionary build, ids, PLAIN values,
Snappy), then appended with its page headers by the host file writer (pf_writer_*).

Differences that are allowed by the format and documented in DESIGN.md: the fallback encoding is
PLAIN (parquet-mr's v2 writer falls back to DELTA_* for ints / strings), ids are written as one
bit-packed run per page, no page / column statistics are written.
"""
import ctypes as C

import numpy as np

from . import _native
from ._native import PfError, check, lib

BOOLEAN, INT32, INT64, INT96, FLOAT, DOUBLE, BINARY, FIXED_LEN_BYTE_ARRAY = 0, 1, 2, 3, 4, 5, 6, 7
_WIDTH = {BOOLEAN: 1, INT32: 4, INT64: 8, FLOAT: 4, DOUBLE: 8}
_DTYPE = {BOOLEAN: np.uint8, INT32: np.int32, INT64: np.int64, FLOAT: np.float32, DOUBLE: np.float64}
_NAMES = {BOOLEAN: "BOOLEAN", INT32: "INT32", INT64: "INT64", INT96: "INT96", FLOAT: "FLOAT", DOUBLE: "DOUBLE",
          BINARY: "BINARY", FIXED_LEN_BYTE_ARRAY: "FIXED_LEN_BYTE_ARRAY"}


class EncodeColumn(C.Structure):
    _fields_ = [("physical_type", C.c_int32), ("max_def", C.c_int32), ("num_rows", C.c_int64),
                ("values", C.c_void_p), ("validity", C.c_void_p), ("offsets", C.c_void_p), ("chars", C.c_void_p),
                ("chars_len", C.c_int64), ("dictionary", C.c_int32), ("page_rows", C.c_int32),
                ("dict_page_limit", C.c_int32), ("codec", C.c_int32)]


class EncodedChunk(C.Structure):
    _fields_ = [("bytes", C.c_void_p), ("size", C.c_int64), ("total_uncompressed_size", C.c_int64),
                ("num_values", C.c_int64), ("dictionary_page_offset", C.c_int64), ("data_page_offset", C.c_int64),
                ("n_data_pages", C.c_int32), ("dict_entries", C.c_int32), ("data_encoding", C.c_int32),
                ("fallback", C.c_int32), ("codec", C.c_int32), ("snappy_ms", C.c_float), ("encode_ms", C.c_float),
                ("snappy_in", C.c_int64), ("snappy_out", C.c_int64)]


class WriteField(C.Structure):
    _fields_ = [("name", C.c_char_p), ("physical_type", C.c_int32), ("optional", C.c_int32), ("utf8", C.c_int32)]


class Field:
    """One primitive field of a flat MessageType (parquet-mr Types.required/optional(...).named)."""

    def __init__(self, name, physical_type, optional=False, string=False):
        self.name, self.physical_type, self.optional, self.string = name, physical_type, optional, string


class _Builder:
    def __init__(self, physical_type, optional):
        self.t, self.opt, self.string = physical_type, optional, False

    def as_string(self):
        self.string = True
        return self

    def named(self, name):
        return Field(name, self.t, self.opt, self.string)


def required(physical_type):
    return _Builder(physical_type, False)


def optional(physical_type):
    return _Builder(physical_type, True)


class MessageType:
    def __init__(self, name, *fields):
        self.name, self.fields = name, list(fields)
        self._index = {f.name: i for i, f in enumerate(self.fields)}

    def getFieldIndex(self, name):
        if name not in self._index:
            raise KeyError(f"{name} not found in {self.name}")   # parquet-mr InvalidRecordException
        return self._index[name]


class Dehydrator:
    """Dehydrator.java: dehydrate(record, valueWriter)."""

    def dehydrate(self, record, value_writer):
        raise NotImplementedError


class ValueWriter:
    """ValueWriter.java: write(name, value)."""

    def write(self, name, value):
        raise NotImplementedError


class _RowBuffer(ValueWriter):
    """SimpleWriteSupport.writeField (ParquetWriter.java:143-160) into per-column host buffers."""

    def __init__(self, schema):
        self.schema = schema
        self.cols = [[] for _ in schema.fields]
        self.rows = 0
        self._seen = [False] * len(schema.fields)

    def write(self, name, value):
        i = self.schema.getFieldIndex(name)
        f = self.schema.fields[i]
        t = f.physical_type
        if self._seen[i]:
            raise RuntimeError(f"field {name} written twice in one record")
        if t == INT32:
            v = int(value)
        elif t == INT64:
            v = int(value)
        elif t == DOUBLE:
            v = float(value)
        elif t == BOOLEAN:
            v = bool(value)
        elif t == FLOAT:
            v = float(value)
        elif t == BINARY:
            if not f.string:
                raise NotImplementedError("We don't support writing " + str(None))
            v = str(value).encode("utf-8")
        else:
            raise NotImplementedError("We don't support writing " + _NAMES.get(t, str(t)))
        self._seen[i] = True
        self.cols[i].append(v)

    def end_record(self):
        for i, f in enumerate(self.schema.fields):
            if not self._seen[i]:
                if not f.optional:
                    raise RuntimeError(f"required field {f.name} was not written")
                self.cols[i].append(None)
            self._seen[i] = False
        self.rows += 1

    def take(self):
        cols, self.cols, n = self.cols, [[] for _ in self.schema.fields], self.rows
        self.rows = 0
        return cols, n


def column_arrays(field, values):
    """Python values (None = null) -> (values | (offsets, chars), validity or None) numpy arrays."""
    n = len(values)
    present = np.fromiter((v is not None for v in values), dtype=bool, count=n)
    validity = np.packbits(present, bitorder="little") if (field.optional and not present.all()) else None
    if field.optional and validity is None:
        validity = np.packbits(np.ones(n, bool), bitorder="little")
    if field.physical_type == BINARY:
        lens = np.fromiter((len(v) if v is not None else 0 for v in values), dtype=np.int64, count=n)
        offsets = np.zeros(n + 1, np.int32)
        np.cumsum(lens, out=offsets[1:])
        chars = np.frombuffer(b"".join(v for v in values if v is not None), dtype=np.uint8)
        return (offsets, chars), validity
    dt = _DTYPE[field.physical_type]
    arr = np.fromiter((v if v is not None else 0 for v in values), dtype=dt, count=n)
    return arr, validity


class GpuColumnEncoder:
    """pf_encode_chunk on one context: numpy column -> pf_encoded_chunk (bytes stay in the ctx)."""

    def __init__(self, decoder):
        self.dec = decoder

    def encode(self, field, data, validity, n, dictionary=True, page_rows=0, dict_page_limit=0, codec=1):
        c = EncodeColumn()
        c.physical_type = field.physical_type
        c.max_def = 1 if field.optional else 0
        c.num_rows = n
        keep = []
        if field.physical_type == BINARY:
            offsets, chars = data
            offsets = np.ascontiguousarray(offsets, np.int32)
            chars = np.ascontiguousarray(chars, np.uint8)
            keep += [offsets, chars]
            c.offsets = offsets.ctypes.data
            c.chars = chars.ctypes.data if chars.size else None
            c.chars_len = chars.size
        else:
            arr = np.ascontiguousarray(data)
            if arr.dtype.itemsize != _WIDTH[field.physical_type]:
                raise ValueError(f"{field.name}: {arr.dtype} does not match {_NAMES[field.physical_type]}")
            keep.append(arr)
            c.values = arr.ctypes.data
        if validity is not None:
            v = np.ascontiguousarray(validity, np.uint8)
            keep.append(v)
            c.validity = v.ctypes.data
        c.dictionary = 1 if dictionary else 0
        c.page_rows = page_rows
        c.dict_page_limit = dict_page_limit
        c.codec = codec
        out = EncodedChunk()
        check(lib().pf_encode_chunk(self.dec.h, C.byref(c), 0, C.byref(out)), self.dec.h, "pf_encode_chunk")
        return out


class ParquetWriter:
    """bsp/ParquetWriter.java: writeFile(schema, file, dehydrator), write(record), close().
    row_group_rows bounds the rows buffered per row group (parquet-mr flushes by its 128 MiB
    block size; the bound here is in rows, the byte size of a row group is the caller's)."""

    def __init__(self, schema, path, dehydrator, row_group_rows=1 << 20, device=0, decoder=None, codec=1,
                 decoders=None):
        """decoders: several contexts (GpuDecoder) to encode the columns of a row group in parallel
        (one host thread each); chunks are still appended in schema order."""
        from .decoder import GpuDecoder
        self.schema, self.dehydrator = schema, dehydrator
        self.row_group_rows = row_group_rows
        self._own = decoder is None and not decoders
        self.dec = decoder or (decoders[0] if decoders else GpuDecoder(device))
        self.enc = GpuColumnEncoder(self.dec)
        self.encoders = [GpuColumnEncoder(d) for d in decoders] if decoders else [self.enc]
        self.kernel_ms = {"snappy": 0.0, "encode": 0.0, "snappy_in": 0, "snappy_out": 0}
        self.codec = codec
        self.buf = _RowBuffer(schema)
        self.last_chunks = []     # (dict_entries, data_encoding, fallback) of the last row group
        fields = (WriteField * len(schema.fields))()
        self._names = [f.name.encode() for f in schema.fields]
        for i, f in enumerate(schema.fields):
            fields[i] = WriteField(self._names[i], f.physical_type, 1 if f.optional else 0, 1 if f.string else 0)
        self.w = C.c_void_p()
        rc = lib().pf_writer_open(str(path).encode(), fields, len(schema.fields), C.byref(self.w))
        if rc != 0:
            if self._own:
                self.dec.close()
            raise PfError(rc, "pf_writer_open: " + (lib().pf_writer_last_error() or b"").decode(errors="replace"))

    @staticmethod
    def writeFile(schema, out, dehydrator, **kw):
        return ParquetWriter(schema, out, dehydrator, **kw)

    def write(self, record):
        self.dehydrator.dehydrate(record, self.buf)
        self.buf.end_record()
        if self.buf.rows >= self.row_group_rows:
            self._flush()

    def write_columns(self, columns, n):
        """Columnar fast path: {name: array | (offsets, chars) | (array, validity)} for n rows,
        one row group (buffered records are flushed first)."""
        self._flush()
        self.last_chunks = []
        work = []
        for f in self.schema.fields:
            d = columns[f.name]
            validity = None
            if isinstance(d, tuple) and len(d) == 2 and f.physical_type != BINARY:
                d, validity = d
            elif isinstance(d, tuple) and len(d) == 3:
                d, validity = (d[0], d[1]), d[2]
            if f.optional and validity is None:
                validity = np.packbits(np.ones(n, bool), bitorder="little")
            work.append((f, d, validity))
        if len(self.encoders) == 1:
            for i, (f, d, validity) in enumerate(work):
                self._encode_add(f, d, validity, n, i)
        else:
            self._encode_parallel(work, n)
        self._end_group(n)

    def _encode_parallel(self, work, n):
        """Columns encoded concurrently, one host thread per context (ctypes releases the GIL), biggest
        first; each chunk's bytes are copied out of its context before the context encodes again."""
        import threading
        size = [sum(np.asarray(x).nbytes for x in (d if isinstance(d, tuple) else (d,))) for _f, d, _v in work]
        order = sorted(range(len(work)), key=lambda i: -size[i])
        results = [None] * len(work)
        lock = threading.Lock()
        errs = []

        def worker(enc):
            try:
                while True:
                    with lock:
                        if not order:
                            return
                        i = order.pop(0)
                    f, d, validity = work[i]
                    out = enc.encode(f, d, validity, n, codec=self.codec)
                    keep = C.create_string_buffer(C.string_at(out.bytes, out.size), max(1, out.size))
                    cp = EncodedChunk.from_buffer_copy(out)
                    cp.bytes = C.cast(keep, C.c_void_p)
                    results[i] = (cp, keep)
            except Exception as e:   # reported after the join
                errs.append(e)

        ts = [threading.Thread(target=worker, args=(e,)) for e in self.encoders]
        [t.start() for t in ts]
        [t.join() for t in ts]
        if errs:
            raise errs[0]
        for i, (cp, _keep) in enumerate(results):
            self._add(cp, i)

    def _add(self, out, i):
        self.last_chunks.append((out.dict_entries, out.data_encoding, out.fallback))
        self.kernel_ms["snappy"] += out.snappy_ms
        self.kernel_ms["encode"] += out.encode_ms
        self.kernel_ms["snappy_in"] += out.snappy_in
        self.kernel_ms["snappy_out"] += out.snappy_out
        rc = lib().pf_writer_add_chunk(self.w, i, C.byref(out))
        if rc != 0:
            raise PfError(rc, "pf_writer_add_chunk: " + (lib().pf_writer_last_error() or b"").decode(errors="replace"))

    def _encode_add(self, f, data, validity, n, i):
        out = self.enc.encode(f, data, validity, n, codec=self.codec)
        self._add(out, i)
        return out

    def _end_group(self, n):
        rc = lib().pf_writer_end_row_group(self.w, n)
        if rc != 0:
            raise PfError(rc, "pf_writer_end_row_group: " + (lib().pf_writer_last_error() or b"").decode(errors="replace"))

    def _flush(self):
        if self.buf.rows == 0:
            return
        cols, n = self.buf.take()
        self.last_chunks = []
        for i, f in enumerate(self.schema.fields):
            data, validity = column_arrays(f, cols[i])
            self._encode_add(f, data, validity, n, i)
        self._end_group(n)

    def close(self):
        if not self.w:
            return
        try:
            self._flush()
        finally:
            rc = lib().pf_writer_close(self.w)
            self.w = C.c_void_p()
            if self._own:
                self.dec.close()
        if rc != 0:
            raise PfError(rc, "pf_writer_close: " + (lib().pf_writer_last_error() or b"").decode(errors="replace"))

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


__all__ = ["ParquetWriter", "MessageType", "Field", "Dehydrator", "ValueWriter", "required", "optional",
           "BOOLEAN", "INT32", "INT64", "FLOAT", "DOUBLE", "BINARY", "_native"]

"""Host-side driver of the HIP decoder: file metadata (pf_file_*) and GPU contexts (pf_ctx).

`ParquetFile` plays the role of parquet-mr's footer/PageHeader parse (ParquetReader.java:120,
:183); `GpuDecoder` owns one pf_ctx (one GPU, one HIP stream) and turns column chunks into
decoded columnar numpy arrays in the canonical layout of include/pfloor.h."""
import ctypes as C

import numpy as np

from ._native import ChunkDesc, ColumnInfo, ColumnMeta, ColumnOut, PageDesc, ScanChunk, ScanResult, check, lib

CONVERTED_UTF8, CONVERTED_ENUM, CONVERTED_JSON = 0, 4, 19
LOGICAL_STRING, LOGICAL_ENUM, LOGICAL_JSON = 1, 4, 12


class ColumnDescriptor:
    """The parts of parquet-mr's ColumnDescriptor the reference reads
    (getPath(), getMaxDefinitionLevel(), getPrimitiveType(); ParquetReader.java:126-146)."""

    def __init__(self, index, m: ColumnMeta):
        self.index = index
        self.path = m.path.decode().split(".")
        self.physical_type = m.physical_type
        self.type_length = m.type_length
        self.max_def = m.max_def
        self.max_rep = m.max_rep
        self.repeated_def = m.repeated_def
        self.list_null_def = m.list_null_def
        self.converted_type = m.converted_type
        self.logical_type = m.logical_type
        self.scale = m.scale
        self.precision = m.precision

    def getPath(self):
        return list(self.path)

    def getMaxDefinitionLevel(self):
        return self.max_def

    def getMaxRepetitionLevel(self):
        return self.max_rep

    @property
    def is_string(self):
        return (self.converted_type in (CONVERTED_UTF8, CONVERTED_ENUM, CONVERTED_JSON) or
                self.logical_type in (LOGICAL_STRING, LOGICAL_ENUM, LOGICAL_JSON))

    def __repr__(self):
        return f"ColumnDescriptor({'.'.join(self.path)}, type={self.physical_type}, def={self.max_def}, rep={self.max_rep})"


class ParquetFile:
    def __init__(self, path):
        L = lib()
        self.path = str(path)
        self.h = C.c_void_p()
        check(L.pf_file_open(self.path.encode(), C.byref(self.h)), None, f"open {self.path}")
        n = C.c_int()
        check(L.pf_file_num_row_groups(self.h, C.byref(n)))
        self.num_row_groups = n.value
        check(L.pf_file_num_columns(self.h, C.byref(n)))
        self.num_columns = n.value
        r = C.c_int64()
        check(L.pf_file_num_rows(self.h, C.byref(r)))
        self.num_rows = r.value
        self.columns = []
        for i in range(self.num_columns):
            m = ColumnMeta()
            check(L.pf_file_column_meta(self.h, i, C.byref(m)))
            self.columns.append(ColumnDescriptor(i, m))
        self.created_by = (L.pf_file_created_by(self.h) or b"").decode(errors="replace")

    def close(self):
        if self.h:
            lib().pf_file_close(self.h)
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def row_group_rows(self, rg):
        r = C.c_int64()
        check(lib().pf_file_row_group_rows(self.h, rg, C.byref(r)))
        return r.value

    def chunk_range(self, rg, col):
        s, n = C.c_uint64(), C.c_uint64()
        check(lib().pf_file_chunk_range(self.h, rg, col, C.byref(s), C.byref(n)))
        return s.value, n.value

    def chunk_desc(self, rg, col, offset_in_buffer):
        d = ChunkDesc()
        check(lib().pf_file_chunk_desc(self.h, rg, col, offset_in_buffer, C.byref(d)), None, f"pages rg{rg} c{col}")
        return d

    def read_into(self, offset, size, dst_ptr):
        check(lib().pf_file_read(self.h, offset, size, C.c_void_p(dst_ptr)))

    def plan(self, row_groups, columns, align=256):
        """Chunk byte ranges + descriptors laid out back to back in one buffer."""
        items = []
        off = 0
        for rg in row_groups:
            for col in columns:
                s, n = self.chunk_range(rg, col)
                items.append((rg, col, s, n, off))
                off += (n + align - 1) // align * align
        return items, off


class PinnedBuffer:
    def __init__(self, ctx, nbytes):
        self.ctx = ctx
        self.ptr = C.c_void_p()
        self.nbytes = max(1, int(nbytes))
        check(lib().pf_host_alloc(ctx, self.nbytes, C.byref(self.ptr)), ctx, "pf_host_alloc")

    def array(self, dtype=np.uint8, n=None):
        n = self.nbytes // np.dtype(dtype).itemsize if n is None else n
        return np.ctypeslib.as_array(C.cast(self.ptr, C.POINTER(C.c_uint8)), shape=(self.nbytes,)).view(dtype)[:n]

    def free(self):
        if self.ptr:
            lib().pf_host_free(self.ctx, self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class GpuDecoder:
    """One pf_ctx = one GPU + one HIP stream."""

    def __init__(self, device=0, share=None):
        """share: another GpuDecoder whose HIP stream this context enqueues onto
        (pf_ctx_create_shared: pipelined decodes of consecutive batches)."""
        L = lib()
        self.h = C.c_void_p()
        if share is not None:
            check(L.pf_ctx_create_shared(share.h, C.byref(self.h)), None, "pf_ctx_create_shared")
            device = share.device
        else:
            check(L.pf_ctx_create(device, C.byref(self.h)), None, f"pf_ctx_create({device})")
        self.device = device
        self._staging = None
        self.n_chunks = 0

    def close(self):
        if self.h:
            if self._staging:
                self._staging.free()
                self._staging = None
            lib().pf_ctx_destroy(self.h)
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def staging(self, nbytes):
        if self._staging is None or self._staging.nbytes < nbytes:
            if self._staging:
                self._staging.free()
            self._staging = PinnedBuffer(self.h, max(nbytes, 1 << 20))
        return self._staging

    def decode(self, descs, buf_ptr, nbytes, on_device=False):
        """descs: ChunkDesc list, or a prebuilt ctypes ChunkDesc array (no per-call copy)."""
        arr = descs if isinstance(descs, C.Array) else (ChunkDesc * max(1, len(descs)))(*descs)
        self._keep = arr
        check(lib().pf_decode_row_group(self.h, arr, len(descs), C.c_void_p(buf_ptr), nbytes, 1 if on_device else 0),
              self.h, "pf_decode_row_group")
        self.n_chunks = len(descs)

    def wait(self):
        return lib().pf_wait(self.h)

    def error(self):
        return (lib().pf_last_error(self.h) or b"").decode(errors="replace")

    def info(self, i):
        ci = ColumnInfo()
        check(lib().pf_column_info_get(self.h, i, C.byref(ci)), self.h, "pf_column_info_get")
        return ci

    def snappy_decompress(self, data: bytes, cap=None):
        """Raw Snappy buffer -> bytes on the GPU (K1 kernels). Returns (bytes, used_fallback)."""
        L = lib()
        src = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, np.uint8)
        out_len = C.c_size_t()
        cap = cap if cap is not None else max(1, 64 * len(data) + 64)
        dst = np.zeros(cap, dtype=np.uint8)
        rc = L.pf_snappy_decompress(self.h, src.ctypes.data, len(data), dst.ctypes.data, cap, C.byref(out_len))
        if rc != 0:
            return rc, None
        return dst[:out_len.value].tobytes(), L.pf_snappy_last_fallback(self.h)

    def scan_pages(self, data, chunks, verify_crc=False, page_cap=4096):
        """GPU page-header scan (pf_scan_pages) of column chunks in one host buffer.
        chunks: [(chunk_offset, chunk_size, num_values)]. Returns (rc, [(status, err_page, crc_pages,
        [page dicts])] per chunk)."""
        L = lib()
        buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
        n = len(chunks)
        sc = (ScanChunk * max(n, 1))()
        for i, (off, size, nv) in enumerate(chunks):
            sc[i] = ScanChunk(off, size, nv, i * page_cap, page_cap)
        pages = (PageDesc * max(1, n * page_cap))()
        res = (ScanResult * max(n, 1))()
        rc = L.pf_scan_pages(self.h, sc, n, buf.ctypes.data, len(data), 0, int(verify_crc), pages, res)
        out = []
        for i in range(n):
            r = res[i]
            pg = [{f: getattr(pages[i * page_cap + k], f) for f, _ in PageDesc._fields_} for k in range(r.n_pages)]
            out.append((r.status, r.err_page, r.crc_pages, pg))
        return rc, out

    def set_timing(self, on):
        check(lib().pf_ctx_set_timing(self.h, 1 if on else 0), self.h, "pf_ctx_set_timing")

    def timing(self):
        buf = (C.c_float * 16)()
        n = C.c_int()
        check(lib().pf_last_timing(self.h, buf, 16, C.byref(n)), self.h, "pf_last_timing")
        names = ["h2d", "snappy_parse", "snappy_exec", "dict", "delta", "levels", "count", "scan", "flat", "decode"]
        return dict(zip(names, list(buf)[:n.value]))

    def fetch_batch(self, chunk_types, pageable=False):
        """All chunks of the last decode with ONE D2H per output arena (pf_copy_batch_async), then
        per chunk the canonical arrays cut from the host copy (pf_column_info_host).
        chunk_types: [(physical_type, max_def, max_rep)] per chunk. pageable: an ordinary host array
        instead of a mapped pinned buffer (the library's SDMA copy path instead of its download kernel)."""
        L = lib()
        n = C.c_size_t()
        check(L.pf_batch_bytes(self.h, C.byref(n)), self.h, "pf_batch_bytes")
        if pageable:
            class _Host:   # (same interface as PinnedBuffer for the code below)
                def __init__(self, nbytes):
                    self.arr = np.zeros(nbytes + 256, np.uint8)
                    a = self.arr.ctypes.data
                    self.off = (-a) % 256
                    self.ptr = C.c_void_p(a + self.off)
                    self.nbytes = nbytes

                def array(self):
                    return self.arr[self.off:self.off + self.nbytes]

                def free(self):
                    self.arr = None
            buf = _Host(max(1, n.value))
        else:
            buf = PinnedBuffer(self.h, max(1, n.value))
        try:
            check(L.pf_copy_batch_async(self.h, buf.ptr, buf.nbytes), self.h, "pf_copy_batch_async")
            check(L.pf_sync(self.h), self.h, "pf_sync")
            host = buf.array()
            base = buf.ptr.value
            out = []
            for i, (ptype, max_def, max_rep) in enumerate(chunk_types):
                ci = ColumnInfo()
                check(L.pf_column_info_host(self.h, i, buf.ptr, C.byref(ci)), self.h, "pf_column_info_host")
                g = {"status": ci.status, "num_entries": ci.num_entries, "num_slots": ci.num_slots,
                     "num_values": ci.num_values, "num_rows": ci.num_rows, "num_chars": ci.num_chars, "width": ci.width}
                if ci.status == 0:
                    ns, nr, ne = ci.num_slots, ci.num_rows, ci.num_entries

                    def cut(ptr, nbytes, dtype=np.uint8):
                        if not ptr:
                            raise AssertionError("array missing from the batch copy")
                        o = ptr - base
                        return host[o:o + nbytes].copy().view(dtype)
                    if ptype == 6:
                        g["offsets"] = cut(ci.d_offsets, 4 * (ns + 1), np.int32)
                        g["chars"] = cut(ci.d_chars, ci.num_chars) if ci.num_chars else np.zeros(0, np.uint8)
                    else:
                        g["values"] = cut(ci.d_values, ns * ci.width) if ns * ci.width else np.zeros(0, np.uint8)
                    if max_def > 0:
                        g["validity"] = cut(ci.d_validity, (ns + 7) // 8)
                    if max_rep == 1:
                        g["list_offsets"] = cut(ci.d_list_offsets, 4 * (nr + 1), np.int32)
                        g["list_validity"] = cut(ci.d_list_validity, (nr + 7) // 8)
                    if max_rep > 0:
                        g["def_levels"] = cut(ci.d_def_levels, ne)
                        g["rep_levels"] = cut(ci.d_rep_levels, ne)
                out.append(g)
            return out
        finally:
            buf.free()

    def fetch(self, i, physical_type, max_def, max_rep):
        """Copy chunk i's decoded arrays to host numpy (canonical layout)."""
        ci = self.info(i)
        out = {"status": ci.status, "num_entries": ci.num_entries, "num_slots": ci.num_slots,
               "num_values": ci.num_values, "num_rows": ci.num_rows, "num_chars": ci.num_chars, "width": ci.width}
        if ci.status != 0:
            return out
        ns, nr, ne = ci.num_slots, ci.num_rows, ci.num_entries
        arrs = {}
        o = ColumnOut()

        def want(name, n, dtype=np.uint8):
            a = np.zeros(max(n, 0), dtype=dtype)
            arrs[name] = a
            setattr(o, name, a.ctypes.data if a.size else None)
            setattr(o, name + "_cap", a.nbytes)

        if physical_type == 6:
            want("offsets", ns + 1, np.int32)
            want("chars", ci.num_chars)
        else:
            want("values", ns * ci.width)
        if max_def > 0:
            want("validity", (ns + 7) // 8)
        if max_rep == 1:
            want("list_offsets", nr + 1, np.int32)
            want("list_validity", (nr + 7) // 8)
        if max_rep > 0:
            want("def_levels", ne)
            want("rep_levels", ne)
        check(lib().pf_copy_column(self.h, i, C.byref(o)), self.h, "pf_copy_column")
        out.update(arrs)
        return out


def decode_file(path, row_groups=None, columns=None, device=0, decoder=None):
    """Decode the selected chunks of a file on the GPU: {(rg, col): arrays}. One batch."""
    with ParquetFile(path) as pf:
        rgs = list(range(pf.num_row_groups)) if row_groups is None else list(row_groups)
        cols = list(range(pf.num_columns)) if columns is None else list(columns)
        dec = decoder or GpuDecoder(device)
        try:
            items, total = pf.plan(rgs, cols)
            buf = dec.staging(total)
            descs = []
            for rg, col, s, n, off in items:
                if n:
                    pf.read_into(s, n, buf.ptr.value + off)
                descs.append(pf.chunk_desc(rg, col, off))
            dec.decode(descs, buf.ptr.value, max(total, 1))
            rc = dec.wait()
            out = {}
            for i, (rg, col, *_r) in enumerate(items):
                c = pf.columns[col]
                out[(rg, col)] = dec.fetch(i, c.physical_type, c.max_def, c.max_rep)
            out["_status"] = rc
            out["_error"] = dec.error() if rc else ""
            return out
        finally:
            if decoder is None:
                dec.close()

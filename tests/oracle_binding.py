"""ctypes binding of the CPU oracle (oracle/pf_oracle.h). TEST INFRASTRUCTURE ONLY:
the oracle is the checker, never the product path."""
import ctypes as C

import numpy as np


class PfoColumn(C.Structure):
    _fields_ = [("status", C.c_int32), ("error", C.c_char * 256),
                ("physical_type", C.c_int32), ("type_length", C.c_int32), ("max_def", C.c_int32),
                ("max_rep", C.c_int32), ("repeated_def", C.c_int32), ("list_null_def", C.c_int32),
                ("width", C.c_int32),
                ("num_entries", C.c_int64), ("num_slots", C.c_int64), ("num_values", C.c_int64),
                ("num_rows", C.c_int64), ("num_chars", C.c_int64),
                ("values", C.POINTER(C.c_uint8)), ("validity", C.POINTER(C.c_uint8)),
                ("offsets", C.POINTER(C.c_int32)), ("chars", C.POINTER(C.c_uint8)),
                ("list_offsets", C.POINTER(C.c_int32)), ("list_validity", C.POINTER(C.c_uint8)),
                ("def_levels", C.POINTER(C.c_uint8)), ("rep_levels", C.POINTER(C.c_uint8))]


def _arr(ptr, n, dtype):
    if n <= 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).copy().view(dtype) if dtype != np.int32 else \
        np.ctypeslib.as_array(ptr, shape=(n,)).copy()


class Oracle:
    def __init__(self, path):
        self.lib = L = C.CDLL(path)
        L.pfo_open.argtypes = [C.c_char_p, C.POINTER(C.c_void_p), C.c_char_p, C.c_int]
        L.pfo_open_mem.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_void_p), C.c_char_p, C.c_int]
        L.pfo_close.argtypes = [C.c_void_p]
        for fn in ("pfo_num_row_groups", "pfo_num_columns"):
            getattr(L, fn).argtypes = [C.c_void_p]
        L.pfo_num_rows.argtypes = [C.c_void_p]; L.pfo_num_rows.restype = C.c_int64
        L.pfo_row_group_rows.argtypes = [C.c_void_p, C.c_int]; L.pfo_row_group_rows.restype = C.c_int64
        L.pfo_column_path.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_int]
        L.pfo_column_top_name.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_int]
        L.pfo_column_schema.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int32)]
        L.pfo_decode.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(PfoColumn)]
        L.pfo_free_column.argtypes = [C.POINTER(PfoColumn)]
        L.pfo_snappy_uncompress.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.pfo_snappy_uncompress.restype = C.c_int64
        L.pfo_snappy_uncompressed_length.argtypes = [C.c_char_p, C.c_size_t]
        L.pfo_snappy_uncompressed_length.restype = C.c_int64
        L.pfo_snappy_compress.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int]
        L.pfo_snappy_compress.restype = C.c_int64
        L.pfo_chunk_pages.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(PfoPage), C.c_int, C.c_int,
                                      C.POINTER(C.c_int)]
        L.pfo_crc32.argtypes = [C.c_char_p, C.c_size_t]
        L.pfo_crc32.restype = C.c_uint32

    def snappy_compress(self, data: bytes, mode=0):
        """Test-vector generator: mode 0 Google-style 64 KiB blocks, mode 1 cross-block copies."""
        cap = len(data) + len(data) // 6 + 64
        out = C.create_string_buffer(cap)
        n = self.lib.pfo_snappy_compress(data, len(data), out, cap, mode)
        assert n >= 0
        return out.raw[:n]

    def snappy_uncompress(self, data: bytes):
        n = self.lib.pfo_snappy_uncompressed_length(data, len(data))
        if n < 0:
            return None
        out = C.create_string_buffer(max(1, n))
        got = self.lib.pfo_snappy_uncompress(data, len(data), out, n)
        if got < 0:
            return got
        return out.raw[:got]

    def crc32(self, data: bytes):
        return self.lib.pfo_crc32(data, len(data))

    def open(self, path=None, data=None):
        return OracleFile(self, path, data)


class PfoPage(C.Structure):
    _fields_ = [("offset", C.c_uint64), ("compressed_size", C.c_int32), ("uncompressed_size", C.c_int32),
                ("page_type", C.c_int32), ("encoding", C.c_int32), ("num_values", C.c_int32), ("has_crc", C.c_int32),
                ("crc", C.c_uint32), ("crc_ok", C.c_int32)]


class OracleFile:
    def __init__(self, o, path=None, data=None):
        self.o = o
        self.h = C.c_void_p()
        err = C.create_string_buffer(256)
        if data is not None:
            rc = o.lib.pfo_open_mem(data, len(data), C.byref(self.h), err, 256)
        else:
            rc = o.lib.pfo_open(path.encode(), C.byref(self.h), err, 256)
        if rc != 0:
            raise IOError(err.value.decode())

    def close(self):
        if self.h:
            self.o.lib.pfo_close(self.h)
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def num_row_groups(self):
        return self.o.lib.pfo_num_row_groups(self.h)

    @property
    def num_columns(self):
        return self.o.lib.pfo_num_columns(self.h)

    def column_path(self, c):
        b = C.create_string_buffer(4096)
        self.o.lib.pfo_column_path(self.h, c, b, 4096)
        return b.value.decode()

    def top_name(self, c):
        b = C.create_string_buffer(4096)
        self.o.lib.pfo_column_top_name(self.h, c, b, 4096)
        return b.value.decode()

    def schema(self, c):
        a = (C.c_int32 * 7)()
        self.o.lib.pfo_column_schema(self.h, c, a)
        return dict(zip(("type", "type_length", "max_def", "max_rep", "repeated_def", "list_null_def",
                         "converted_type"), list(a)))

    def chunk_pages(self, rg, col, verify_crc=False, cap=100000):
        """(status or page count, err_page, [page dicts]) of the oracle's PageHeader walk."""
        out = (PfoPage * cap)()
        err = C.c_int(-1)
        n = self.o.lib.pfo_chunk_pages(self.h, rg, col, out, cap, int(verify_crc), C.byref(err))
        pages = [{f: getattr(out[i], f) for f, _ in PfoPage._fields_} for i in range(max(n, 0))]
        return n, err.value, pages

    def decode(self, rg, col):
        """Decoded chunk as a dict of numpy arrays in the canonical layout (pfloor.h)."""
        c = PfoColumn()
        rc = self.o.lib.pfo_decode(self.h, rg, col, C.byref(c))
        try:
            out = {"status": rc, "error": c.error.decode(errors="replace")}
            if rc != 0:
                return out
            ns, nr, ne = c.num_slots, c.num_rows, c.num_entries
            out.update(num_entries=ne, num_slots=ns, num_values=c.num_values, num_rows=nr,
                       num_chars=c.num_chars, width=c.width)
            if c.physical_type == 6:
                out["offsets"] = _arr(c.offsets, ns + 1, np.int32)
                out["chars"] = _arr(c.chars, c.num_chars, np.uint8)
            else:
                out["values"] = _arr(c.values, ns * c.width, np.uint8)
            if c.max_def > 0:
                out["validity"] = _arr(c.validity, (ns + 7) // 8, np.uint8)
            if c.max_rep == 1:
                out["list_offsets"] = _arr(c.list_offsets, nr + 1, np.int32)
                out["list_validity"] = _arr(c.list_validity, (nr + 7) // 8, np.uint8)
            if c.max_rep > 0:
                out["def_levels"] = _arr(c.def_levels, ne, np.uint8)
                out["rep_levels"] = _arr(c.rep_levels, ne, np.uint8)
            return out
        finally:
            self.o.lib.pfo_free_column(C.byref(c))

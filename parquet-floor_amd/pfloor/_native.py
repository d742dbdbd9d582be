"""ctypes binding of libpfloor.so (include/pfloor.h).

This is the Python analogue of the FFM binding a Java maintainer adds:
plain C structs, plain pointers, no torch types. Loading fails loudly if the in-tree
library is missing — there is no CPU fallback on the product path."""
import contextlib
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PFLOOR_LIB_PATH: diagnostics only (e.g. the stamp build from `make stamps`).
LIB_PATH = os.environ.get("PFLOOR_LIB_PATH") or os.path.join(_HERE, "libpfloor.so")
# The diagnostics build (`make -C parquet-floor_amd diag`): the same library compiled with -DPF_DIAG,
# which reads the PF_* switches (include/pfloor.h is unchanged) from the environment at pf_ctx_create.
DIAG_PATH = os.path.join(os.path.dirname(_HERE), "diag", "libpfloor_diag.so")

PF_OK = 0
STATUS = {0: "PF_OK", -1: "PF_ERR_INVALID_ARG", -2: "PF_ERR_CORRUPT_PAGE", -3: "PF_ERR_UNSUPPORTED_ENCODING",
          -4: "PF_ERR_UNSUPPORTED_CODEC", -5: "PF_ERR_HIP", -6: "PF_ERR_CAPACITY", -7: "PF_ERR_UNSUPPORTED_TYPE",
          -8: "PF_ERR_IO", -9: "PF_ERR_STATE"}

PHYSICAL = {0: "BOOLEAN", 1: "INT32", 2: "INT64", 3: "INT96", 4: "FLOAT", 5: "DOUBLE", 6: "BINARY",
            7: "FIXED_LEN_BYTE_ARRAY"}


class PageDesc(C.Structure):
    _fields_ = [("offset", C.c_uint64), ("compressed_size", C.c_uint32), ("uncompressed_size", C.c_uint32),
                ("page_type", C.c_int32), ("encoding", C.c_int32), ("def_encoding", C.c_int32),
                ("rep_encoding", C.c_int32), ("num_values", C.c_int32), ("num_nulls", C.c_int32),
                ("num_rows", C.c_int32), ("def_bytes", C.c_int32), ("rep_bytes", C.c_int32),
                ("is_compressed", C.c_int32)]


class ChunkDesc(C.Structure):
    _fields_ = [("physical_type", C.c_int32), ("type_length", C.c_int32), ("max_def", C.c_int32),
                ("max_rep", C.c_int32), ("repeated_def", C.c_int32), ("list_null_def", C.c_int32),
                ("codec", C.c_int32), ("n_pages", C.c_int32), ("pages", C.POINTER(PageDesc)),
                ("chunk_offset", C.c_uint64), ("chunk_size", C.c_uint64), ("num_rows", C.c_int64)]


class ColumnOut(C.Structure):
    _fields_ = [("values", C.c_void_p), ("values_cap", C.c_size_t),
                ("validity", C.c_void_p), ("validity_cap", C.c_size_t),
                ("offsets", C.c_void_p), ("offsets_cap", C.c_size_t),
                ("chars", C.c_void_p), ("chars_cap", C.c_size_t),
                ("list_offsets", C.c_void_p), ("list_offsets_cap", C.c_size_t),
                ("list_validity", C.c_void_p), ("list_validity_cap", C.c_size_t),
                ("def_levels", C.c_void_p), ("def_levels_cap", C.c_size_t),
                ("rep_levels", C.c_void_p), ("rep_levels_cap", C.c_size_t)]


class ColumnInfo(C.Structure):
    _fields_ = [("num_entries", C.c_int64), ("num_slots", C.c_int64), ("num_values", C.c_int64),
                ("num_rows", C.c_int64), ("num_chars", C.c_int64), ("width", C.c_int32), ("status", C.c_int32),
                ("d_values", C.c_void_p), ("d_validity", C.c_void_p), ("d_offsets", C.c_void_p),
                ("d_chars", C.c_void_p), ("d_list_offsets", C.c_void_p), ("d_list_validity", C.c_void_p),
                ("d_def_levels", C.c_void_p), ("d_rep_levels", C.c_void_p)]


class ColumnMeta(C.Structure):
    _fields_ = [("path", C.c_char_p), ("top_name", C.c_char_p), ("physical_type", C.c_int32),
                ("type_length", C.c_int32), ("max_def", C.c_int32), ("max_rep", C.c_int32),
                ("repeated_def", C.c_int32), ("list_null_def", C.c_int32), ("converted_type", C.c_int32),
                ("logical_type", C.c_int32), ("scale", C.c_int32), ("precision", C.c_int32)]


class ScanChunk(C.Structure):
    _fields_ = [("chunk_offset", C.c_uint64), ("chunk_size", C.c_uint64), ("num_values", C.c_int64),
                ("page_base", C.c_int32), ("page_cap", C.c_int32)]


class ScanResult(C.Structure):
    _fields_ = [("n_pages", C.c_int32), ("status", C.c_int32), ("err_page", C.c_int32), ("crc_pages", C.c_int32)]


class PfError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code


_lib = None
_loaded = {}


def lib():
    """Load libpfloor.so once. Raises if it has not been built (no fallback)."""
    global _lib
    if _lib is None:
        _lib = _load(LIB_PATH)
    return _lib


@contextlib.contextmanager
def diagnostics():
    """Route lib() to the diagnostics build for the duration of the block (tests that force rare paths
    with PF_* switches, A/B tools). Contexts created inside must be closed inside. Never used by the
    product path."""
    global _lib
    saved = lib()
    _lib = _load(DIAG_PATH)
    try:
        yield _lib
    finally:
        _lib = saved


def _load(path):
    if path in _loaded:
        return _loaded[path]
    if not os.path.exists(path):
        raise ImportError(f"{path} missing: build it with `make -C parquet-floor_amd` "
                          "(or __graft_entry__.build()); the HIP path has no CPU fallback")
    L = C.CDLL(path)
    vp, i32, i64p, sz = C.c_void_p, C.c_int, C.POINTER(C.c_int64), C.c_size_t
    sig = {
        "pf_abi_version": ([], C.c_int),
        "pf_last_error": ([vp], C.c_char_p),
        "pf_device_count": ([C.POINTER(C.c_int)], C.c_int),
        "pf_ctx_create": ([i32, C.POINTER(vp)], C.c_int),
        "pf_ctx_destroy": ([vp], C.c_int),
        "pf_ctx_create_shared": ([vp, C.POINTER(vp)], C.c_int),
        "pf_ctx_set_timing": ([vp, i32], C.c_int),
        "pf_host_alloc": ([vp, sz, C.POINTER(vp)], C.c_int),
        "pf_host_free": ([vp, vp], C.c_int),
        "pf_device_alloc": ([vp, sz, C.POINTER(vp)], C.c_int),
        "pf_device_free": ([vp, vp], C.c_int),
        "pf_memcpy_h2d": ([vp, vp, vp, sz], C.c_int),
        "pf_decode_row_group": ([vp, C.POINTER(ChunkDesc), i32, vp, sz, i32], C.c_int),
        "pf_wait": ([vp], C.c_int),
        "pf_column_info_get": ([vp, i32, C.POINTER(ColumnInfo)], C.c_int),
        "pf_copy_column": ([vp, i32, C.POINTER(ColumnOut)], C.c_int),
        "pf_copy_columns_async": ([vp, i32, C.POINTER(C.c_int), C.POINTER(ColumnOut)], C.c_int),
        "pf_sync": ([vp], C.c_int),
        "pf_batch_bytes": ([vp, C.POINTER(C.c_size_t)], C.c_int),
        "pf_copy_batch_async": ([vp, vp, sz], C.c_int),
        "pf_column_info_host": ([vp, i32, vp, C.POINTER(ColumnInfo)], C.c_int),
        "pf_last_timing": ([vp, C.POINTER(C.c_float), i32, C.POINTER(C.c_int)], C.c_int),
        "pf_snappy_decompress": ([vp, vp, sz, vp, sz, C.POINTER(C.c_size_t)], C.c_int),
        "pf_snappy_last_fallback": ([vp], C.c_int),
        "pf_scan_pages": ([vp, C.POINTER(ScanChunk), i32, vp, sz, i32, i32, C.POINTER(PageDesc),
                           C.POINTER(ScanResult)], C.c_int),
        "pf_file_open": ([C.c_char_p, C.POINTER(vp)], C.c_int),
        "pf_file_close": ([vp], C.c_int),
        "pf_file_num_row_groups": ([vp, C.POINTER(C.c_int)], C.c_int),
        "pf_file_num_columns": ([vp, C.POINTER(C.c_int)], C.c_int),
        "pf_file_num_rows": ([vp, i64p], C.c_int),
        "pf_file_column_meta": ([vp, i32, C.POINTER(ColumnMeta)], C.c_int),
        "pf_file_row_group_rows": ([vp, i32, i64p], C.c_int),
        "pf_file_chunk_range": ([vp, i32, i32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)], C.c_int),
        "pf_file_chunk_desc": ([vp, i32, i32, C.c_uint64, C.POINTER(ChunkDesc)], C.c_int),
        "pf_file_read": ([vp, C.c_uint64, C.c_uint64, vp], C.c_int),
        "pf_file_created_by": ([vp], C.c_char_p),
        "pf_file_last_error": ([], C.c_char_p),
        "pf_encode_chunk": ([vp, vp, i32, vp], C.c_int),
        "pf_snappy_compress": ([vp, vp, sz, vp, sz, C.POINTER(C.c_size_t)], C.c_int),
        "pf_writer_open": ([C.c_char_p, vp, i32, C.POINTER(vp)], C.c_int),
        "pf_writer_add_chunk": ([vp, i32, vp], C.c_int),
        "pf_writer_end_row_group": ([vp, C.c_int64], C.c_int),
        "pf_writer_close": ([vp], C.c_int),
        "pf_writer_last_error": ([], C.c_char_p),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _loaded[path] = L
    return L


def check(rc, ctx=None, what=""):
    if rc != PF_OK:
        L = lib()
        msg = (L.pf_last_error(ctx) if ctx is not None else L.pf_file_last_error() or L.pf_last_error(None)) or b""
        raise PfError(rc, f"{what}: {msg.decode(errors='replace')}")
    return rc

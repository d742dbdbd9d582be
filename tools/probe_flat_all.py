"""Diagnostic (stamps build: PFLOOR_LIB_PATH=parquet-floor_amd/diag/libpfloor_stamps.so): k_flat_all's
cycles per block (PSTAMP slots 0 / 1 of flat_fixed_block and flat_block) for each lineitem column of one
row group decoded alone, then for all 16 columns in one batch (the blocks then share the GPU)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd")]
import pyarrow.parquet as pq  # noqa: E402
from pfloor import _native, datagen  # noqa: E402
from pfloor.decoder import GpuDecoder, ParquetFile, decode_file  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1048576
path = os.path.join(ROOT, "gpurun_out", f"probe_lineitem_{rows}.parquet")
if not os.path.exists(path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    pq.write_table(datagen.lineitem_table(rows, seed=42), path, compression="snappy", row_group_size=1 << 20)
L = _native.lib()
f = L.pf_debug_pstamps
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
buf = (C.c_ulonglong * 16)()
with ParquetFile(path) as pf:
    names = [c.path[0] for c in pf.columns]
with GpuDecoder(0) as dec:
    for c, col in list(enumerate(names)) + [(None, "ALL")]:
        cols = None if c is None else [c]
        decode_file(path, row_groups=[0], columns=cols, decoder=dec)
        f(buf, 16, 1)
        got = decode_file(path, row_groups=[0], columns=cols, decoder=dec)
        f(buf, 16, 0)
        n = max(buf[0], 1)
        print(f"{col:16s} blocks {buf[0]:6d} | cycles per block {buf[1] / n:9.0f} | dict {buf[6]} binary {buf[7]} | "
              f"max binary {buf[8]} max fixed {buf[9]}", "status", got["_status"], flush=True)
        t = max(buf[3], 1)
        print(f"{'':16s} general body: prologue {buf[2] / n:9.0f} per block | per tile ({buf[3]} tiles): "
              f"levels+values+offsets {buf[4] / t:9.0f} chars+validity {buf[5] / t:9.0f}", flush=True)
        print(f"{'':16s} tile sub-phases: levels {buf[11] / t:7.0f} values {buf[12] / t:7.0f} scan {buf[13] / t:7.0f} "
              f"offsets {buf[14] / t:7.0f} chars {buf[15] / t:7.0f}", flush=True)

"""Diagnostic (stamps build: PFLOOR_LIB_PATH=parquet-floor_amd/diag/libpfloor_stamps.so): k_flat_null
phase cycles per 4096-entry block on config-4-shaped columns (1M rows, 30 % nulls, POOL-value
dictionaries), one column alone and NCOLS columns in one batch (loaded latency).
  python tools/probe_wide.py [pool] [ncols]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd")]
import pyarrow.parquet as pq  # noqa: E402
from pfloor import _native, datagen  # noqa: E402
from pfloor.decoder import decode_file  # noqa: E402

pool = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
ncols = int(sys.argv[2]) if len(sys.argv) > 2 else 64
path = f"/tmp/probe_wide_{pool}_{ncols}.parquet"
if not os.path.exists(path):
    pq.write_table(datagen.wide_table(1_000_000, ncols=ncols, pool=pool), path, compression="snappy",
                   row_group_size=1_000_000)
L = _native.lib()
f = L.pf_debug_pstamps
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
buf = (C.c_ulonglong * 16)()
for cols in ([0], [ncols - 1], list(range(ncols))):
    decode_file(path, row_groups=[0], columns=cols)
    f(buf, 16, 1)
    got = decode_file(path, row_groups=[0], columns=cols)
    f(buf, 16, 0)
    n = max(buf[0], 1)
    print(f"cols {len(cols):3d} k_flat_null blocks {buf[0]} | per block cycles: tables {buf[1] / n:.0f} stage {buf[2] / n:.0f} "
          f"levels+scan {buf[3] / n:.0f} gather+store {buf[4] / n:.0f} total {buf[5] / n:.0f}", "status", got["_status"])
    m = max(buf[8], 1)
    print(f"          k_lvl pages {buf[8]} runs/page {buf[6] / m:.0f} level bytes/page {buf[7] / m:.0f} | per page cycles: "
          f"stage {buf[9] / m:.0f} headers {buf[10] / m:.0f} chain {buf[11] / m:.0f} runs {buf[12] / m:.0f} "
          f"present {buf[13] / m:.0f} blocks {buf[14] / m:.0f} total {buf[15] / m:.0f}")

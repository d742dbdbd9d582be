"""Diagnostic (stamps build: PFLOOR_LIB_PATH=parquet-floor_amd/diag/libpfloor_stamps.so): k_flat phase
cycles per page for single columns of one lineitem row group (PSTAMP slots of flat_block)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd")]
import pyarrow.parquet as pq  # noqa: E402
from pfloor import _native, datagen  # noqa: E402
from pfloor.decoder import ParquetFile, decode_file  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1048576
path = os.path.join(ROOT, "gpurun_out", f"probe_lineitem_{rows}.parquet")
if not os.path.exists(path):
    pq.write_table(datagen.lineitem_table(rows, seed=42), path, compression="snappy", row_group_size=1 << 20)
L = _native.lib()
f = L.pf_debug_pstamps
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
buf = (C.c_ulonglong * 16)()
with ParquetFile(path) as pf:
    names = [c.path[0] for c in pf.columns]
for col in (sys.argv[2].split(",") if len(sys.argv) > 2 else ("l_comment", "l_shipmode", "l_orderkey", "l_shipdate")):
    c = names.index(col)
    decode_file(path, row_groups=[0], columns=[c])
    f(buf, 16, 1)
    got = decode_file(path, row_groups=[0], columns=[c])
    f(buf, 16, 0)
    pages = max(buf[0], 1)
    print(f"{col:12s} k_flat blocks {buf[0]} tiles {buf[3]} | per block: total {buf[1] / pages:.0f} runs {buf[2] / pages:.0f} "
          f"values {buf[4] / pages:.0f} chars+flush {buf[5] / pages:.0f} cycles | max {max(buf[8], buf[9])}", "status", got["_status"])

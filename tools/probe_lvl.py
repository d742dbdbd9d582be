"""Diagnostic (stamps build): k_lvl per-page phase cycles on the config-1 flat table (one row group)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd")]
import pyarrow.parquet as pq  # noqa: E402
from pfloor import _native, datagen  # noqa: E402
from pfloor.decoder import decode_file  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 250000
path = f"/tmp/probe_flat_{rows}.parquet"
if not os.path.exists(path):
    pq.write_table(datagen.flat_table(rows, seed=1), path, compression="NONE", row_group_size=rows)
L = _native.lib()
f = L.pf_debug_pstamps
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
buf = (C.c_ulonglong * 16)()
decode_file(path, row_groups=[0])
f(buf, 16, 1)
got = decode_file(path, row_groups=[0])
f(buf, 16, 0)
pages = max(buf[11], 1)
print(f"k_lvl pages {buf[11]} | per page cycles: stage+positions {buf[12] / pages:.0f} chain {buf[13] / pages:.0f} "
      f"runs+counts {buf[14] / pages:.0f} blocks {buf[15] / pages:.0f}", "status", got["_status"])

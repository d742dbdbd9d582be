"""Diagnostic (stamps build): k_flat per-page phase cycles for one row group of a lineitem file."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd")]
import pyarrow.parquet as pq  # noqa: E402
from pfloor import _native, datagen  # noqa: E402
from pfloor.decoder import decode_file  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1048576
path = f"/tmp/probe_lineitem_{rows}.parquet"
if not os.path.exists(path):
    pq.write_table(datagen.lineitem_table(rows, seed=42), path, compression="snappy", row_group_size=1 << 20)
L = _native.lib()
f = L.pf_debug_pstamps
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
buf = (C.c_ulonglong * 16)()
decode_file(path, row_groups=[0])
f(buf, 16, 1)
got = decode_file(path, row_groups=[0])
f(buf, 16, 0)
pages = max(buf[0], 1)
print(f"k_flat pages {buf[0]} (dict {buf[6]}, binary {buf[7]}) tiles {buf[3]} | per page: total {buf[1] / pages:.0f} "
      f"runs {buf[2] / pages:.0f} values {buf[4] / pages:.0f} chars+flush {buf[5] / pages:.0f} cycles | max binary {buf[8]} "
      f"max fixed {buf[9]} unsplit {buf[10]}", "status", got["_status"])

"""Diagnostic (stamps build): decode a lineitem-shaped file once and print the BYTE_ARRAY walk
counters of pf_pages.hip (calls, tiles, fallbacks and why, cycles)."""
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
f(buf, 16, 1)
got = decode_file(path, row_groups=[0])
f(buf, 16, 0)
names = ["calls", "tiles", "fallbacks", "walk_cyc", "serial_cyc", "cap", "ba_verify_fail", "chainbreak", "short", "ph_stage", "ph_cand", "ph_link", "ph_accept", "ph_check", "ba_count_mismatch", "ba_excess"]
print({k: int(buf[i]) for i, k in enumerate(names)}, "status", got["_status"])

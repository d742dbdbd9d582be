"""Diagnostic (stamps build: PFLOOR_LIB_PATH=parquet-floor_amd/diag/libpfloor_stamps.so): the Snappy parse
kernels' phase counters (pf_debug_cstamps, CSTAMP slots of pf_snappy_par.hip) for one lineitem row group
(all 16 columns in one batch): index pass per window, chain pass per page."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd")]
import pyarrow.parquet as pq  # noqa: E402
from pfloor import _native, datagen  # noqa: E402
from pfloor.decoder import GpuDecoder, decode_file  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1048576
path = os.path.join(ROOT, "gpurun_out", f"probe_lineitem_{rows}.parquet")
if not os.path.exists(path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    pq.write_table(datagen.lineitem_table(rows, seed=42), path, compression="snappy", row_group_size=1 << 20)
L = _native.lib()
f = L.pf_debug_cstamps
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
N = 24
buf = (C.c_ulonglong * N)()
with GpuDecoder(0) as dec:
    decode_file(path, row_groups=[0], decoder=dec)
    f(buf, N, 1)
    got = decode_file(path, row_groups=[0], decoder=dec)
    f(buf, N, 1)
b = list(buf)
w = max(b[0], 1)
pages = max(b[17], 1)
print(f"index: windows {b[0]} | per window cycles: spec parse {b[1] / w:.0f} store {b[3] / w:.0f} entry table {b[4] / w:.0f} "
      f"| no-conv {b[2]} slow-entry windows {b[5]} slow entries {b[6]}")
print(f"chain: pages {b[17]} windows {b[18]} | rounds {b[13]} exact parses {b[14]} ({b[16] / max(b[14], 1):.0f} cycles each) "
      f"deep walks {b[11]} ({b[12] / max(b[11], 1):.0f} cycles each) | per page {b[19] / pages:.0f} cycles, max {b[20]}")
print("raw", b, "status", got["_status"])

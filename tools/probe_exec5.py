"""Diagnostic (stamps build: PFLOOR_LIB_PATH=parquet-floor_amd/diag/libpfloor_stamps.so):
decompress the first PLAIN data page of some lineitem columns through pf_snappy_decompress and
print k_snappy_exec5's per-phase s_memtime cycle sums per piece (producer wave 0, consumer wave 1)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd")]
import pyarrow.parquet as pq  # noqa: E402
from pfloor import _native, datagen  # noqa: E402
from pfloor.decoder import GpuDecoder, ParquetFile  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1048576
path = f"/tmp/probe_lineitem_{rows}.parquet"
if not os.path.exists(path):
    pq.write_table(datagen.lineitem_table(rows, seed=42), path, compression="snappy", row_group_size=1 << 20)
L = _native.lib()
st = L.pf_debug_stamps
st.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
buf = (C.c_ulonglong * 16)()
st(buf, 16, 1)
dec = GpuDecoder(0)
# k_snappy_exec5 slots (its X5T marks): producer 0-4, consumer 6-10
names = ["P:enum", "P:decode", "P:far", "P:descr", "P:barrier", "-", "C:windows", "C:flush", "C:drain", "other",
         "C:barrier", "-", "batches", "pieces", "-"]
with ParquetFile(path) as pf:
    for col in range(pf.num_columns):
        cname = pf.columns[col].path[0] if hasattr(pf, "columns") else str(col)
        s, n = pf.chunk_range(0, col)
        b = np.zeros(n, np.uint8)
        pf.read_into(s, n, b.ctypes.data)
        d = pf.chunk_desc(0, col, 0)
        for i in range(d.n_pages):
            pg = d.pages[i]
            if pg.page_type == 2 or pg.encoding in (2, 8):
                continue
            body = b[pg.offset:pg.offset + pg.compressed_size].tobytes()
            dec.snappy_decompress(body)
            st(buf, 16, 1)
            for _ in range(3):
                dec.snappy_decompress(body)
            st(buf, 16, 1)
            w = max(buf[13], 1)
            print(f"{cname:16s} in {len(body)} pieces/run {w / 3:.0f} | " +
                  " ".join(f"{names[k]}={buf[k] / w:.0f}" for k in (0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 12)), flush=True)
            break

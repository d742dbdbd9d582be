"""Diagnostic (stamps build): Snappy index/chain pass counters for the pages of one row group of a
lineitem file, decompressed one page at a time (pf_snappy_decompress)."""
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
st = L.pf_debug_cstamps
st.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
buf = (C.c_ulonglong * 32)()
dec = GpuDecoder(0)
names = {0: "idx_windows", 1: "idx_parse_cyc", 2: "idx_noconv", 3: "idx_seq_store_cyc", 4: "idx_table_cyc",
         5: "idx_windows_with_slow", 6: "idx_slow_lanes", 7: "idx_rounds", 8: "idx_rewalks", 11: "ch_deep_walks", 12: "ch_deep_cyc",
         13: "ch_rounds", 14: "ch_exact", 16: "ch_exact_cyc", 17: "ch_pages", 18: "ch_nw",
         19: "ch_total_cyc", 20: "ch_max_cyc", 21: "wp_decode_cyc", 22: "wp_exits_cyc", 23: "wp_chain_cyc",
         24: "wp_walk_cyc"}
with ParquetFile(path) as pf:
    for col in range(pf.num_columns):
        cname = pf.columns[col].path[0] if hasattr(pf, "columns") else str(col)
        s, n = pf.chunk_range(0, col)
        b = np.zeros(n, np.uint8)
        pf.read_into(s, n, b.ctypes.data)
        d = pf.chunk_desc(0, col, 0)
        st(buf, 32, 1)
        for i in range(d.n_pages):
            pg = d.pages[i]
            dec.snappy_decompress(b[pg.offset:pg.offset + pg.compressed_size].tobytes())
        st(buf, 32, 1)
        print(f"{cname:16s} " + " ".join(f"{v}={buf[k]}" for k, v in names.items() if buf[k]), flush=True)

"""Diagnostic (stamps build: PFLOOR_LIB_PATH=parquet-floor_amd/diag/libpfloor_stamps.so):
decompress the first few pages of every lineitem column with pf_snappy_decompress and print the
workgroup executor's per-phase s_memtime cycles per piece (k_snappy_exec_wg, PF_STAMPS)."""
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
st = L.pf_debug_wstamps
st.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
buf = (C.c_ulonglong * 16)()
dec = GpuDecoder(0)
names = {0: "tokens", 1: "tiling", 2: "wpre", 3: "literals", 4: "b_init", 5: "b_chase+write", 13: "chase_steps/wave",
         14: "max_chase", 12: "batches", 11: "span", 10: "tokens_n", 9: "fast_copy"}
with ParquetFile(path) as pf:
    for col in range(pf.num_columns):
        cname = pf.columns[col].path[0]
        s, n = pf.chunk_range(0, col)
        b = np.zeros(n, np.uint8)
        pf.read_into(s, n, b.ctypes.data)
        d = pf.chunk_desc(0, col, 0)
        for kind in ("dict-ids", "plain"):
            for i in range(d.n_pages):
                pg = d.pages[i]
                if pg.page_type == 2:
                    continue
                if (pg.encoding in (2, 8)) != (kind == "dict-ids"):
                    continue
                body = b[pg.offset:pg.offset + pg.compressed_size].tobytes()
                dec.snappy_decompress(body)
                st(buf, 16, 1)
                for _ in range(3):
                    dec.snappy_decompress(body)
                st(buf, 16, 1)
                w = max(buf[15], 1)
                if buf[9]:
                    print(f"{cname:16s} {kind:8s} in {len(body):7d} single-literal pieces/run {buf[9] / 3:.0f}", flush=True)
                    break
                print(f"{cname:16s} {kind:8s} in {len(body):7d} pieces/run {w / 3:.0f} | " +
                      " ".join(f"{names[k]}={buf[k] / w:.0f}" for k in (0, 1, 2, 3, 4, 5, 12, 11, 10, 13)) +
                      f" max_chase={buf[14]}", flush=True)
                break

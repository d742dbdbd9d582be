"""Diagnostic (run under rocprofv3 --kernel-trace): decompress the first PLAIN data page of four
lineitem columns through pf_snappy_decompress, 3 times each, so the kernel trace holds per-page
executor durations (one wave per 64 KiB piece, nothing else on the GPU)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd")]
import pyarrow.parquet as pq  # noqa: E402
from pfloor import datagen  # noqa: E402
from pfloor.decoder import GpuDecoder, ParquetFile  # noqa: E402

rows = 1048576
path = f"/tmp/probe_lineitem_{rows}.parquet"
if not os.path.exists(path):
    pq.write_table(datagen.lineitem_table(rows, seed=42), path, compression="snappy", row_group_size=1 << 20)
dec = GpuDecoder(0)
with ParquetFile(path) as pf:
    for col in (0, 1, 5, 15):
        s, n = pf.chunk_range(0, col)
        b = np.zeros(n, np.uint8)
        pf.read_into(s, n, b.ctypes.data)
        d = pf.chunk_desc(0, col, 0)
        for i in range(d.n_pages):
            pg = d.pages[i]
            if pg.page_type == 2 or pg.encoding in (2, 8):
                continue
            body = b[pg.offset:pg.offset + pg.compressed_size].tobytes()
            for _ in range(3):
                out, fb = dec.snappy_decompress(body)
            print(pf.columns[col].path[0], len(body), len(out), fb, flush=True)
            break

"""Timing probe: PLAIN string pages of short values, with and without a few values longer
than k_ba_tile's 124-byte halo. Prints per column the decode's stage times (the data-page walk is in
the count stage) for the library PFLOOR_LIB_PATH names (default: the product library).
  python tools/probe_rare_long.py [rows] [reps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd")]
import pyarrow as pa  # noqa: E402
import pyarrow.parquet as pq  # noqa: E402
from pfloor.decoder import GpuDecoder, ParquetFile  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
out = os.path.join(ROOT, "gpurun_out")
os.makedirs(out, exist_ok=True)
path = os.path.join(out, f"rare_long_{rows}.parquet")
rng = np.random.default_rng(3)
alphabet = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz ,.0123456789", np.uint8)


def strings(lens):
    chars = alphabet[rng.integers(0, len(alphabet), int(lens.sum()))].tobytes()
    offs = np.concatenate([[0], np.cumsum(lens)])
    return pa.array([chars[offs[i]:offs[i + 1]].decode() for i in range(len(lens))], type=pa.string())


short = rng.integers(8, 40, rows)
rare = short.copy()
rare[rng.random(rows) < 0.001] = 300   # about 30 values of 300 bytes per 1 MB page
pq.write_table(pa.table({"short": strings(short), "rare_long": strings(rare)}), path, compression="snappy",
               use_dictionary=False, row_group_size=rows, data_page_size=1 << 20)
lib = os.environ.get("PFLOOR_LIB_PATH", "product")
with ParquetFile(path) as pf, GpuDecoder(0) as dec:
    for col in range(pf.num_columns):
        items, total = pf.plan([0], [col])
        buf = dec.staging(total)
        descs = []
        for rg, c, s, n, off in items:
            pf.read_into(s, n, buf.ptr.value + off)
            descs.append(pf.chunk_desc(rg, c, off))
        dec.set_timing(True)
        stages, walls = [], []
        for r in range(reps + 2):
            t0 = time.perf_counter()
            dec.decode(descs, buf.ptr.value, total)
            rc = dec.wait()
            walls.append(time.perf_counter() - t0)
            assert rc == 0, dec.error()
            if r >= 2:
                stages.append(dec.timing())
        med = {k: round(float(np.median([s[k] for s in stages])), 3) for k in stages[0] if np.median([s[k] for s in stages]) > 0.01}
        print(f"{os.path.basename(lib)} {pf.columns[col].name if hasattr(pf.columns[col], 'name') else col}: "
              f"wall {np.median(walls[2:]) * 1e3:.3f} ms  stages {med}", flush=True)

"""Diagnostic: decompress every Snappy page of a lineitem-shaped file one at a time through
pf_snappy_decompress and report, per (column, page kind), fallback count and time."""
import collections
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd"), os.path.join(ROOT, "tests")]
import pyarrow.parquet as pq  # noqa: E402  (diagnostics only; generates the input)

from oracle_binding import Oracle  # noqa: E402
from pfloor import datagen  # noqa: E402
from pfloor.decoder import GpuDecoder, ParquetFile  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 300000
path = f"/tmp/probe_lineitem_{rows}.parquet"
if not os.path.exists(path):
    pq.write_table(datagen.lineitem_table(rows, seed=42), path, compression="snappy", row_group_size=1 << 20)
o = Oracle(os.path.join(ROOT, "oracle", "libpf_oracle.so"))
dec = GpuDecoder(0)
from pfloor import _native  # noqa: E402
L = _native.lib()
stamps = getattr(L, "pf_debug_stamps", None) if os.environ.get("PFLOOR_LIB_PATH") else None
if stamps:
    stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
sbuf = (C.c_ulonglong * 16)()
sacc = collections.defaultdict(lambda: np.zeros(16))
stats = collections.defaultdict(lambda: [0, collections.Counter(), 0.0, 0, 0, 0])
with ParquetFile(path) as pf:
    for col in range(pf.num_columns):
        s, n = pf.chunk_range(0, col)
        buf = np.zeros(n, np.uint8)
        pf.read_into(s, n, buf.ctypes.data)
        d = pf.chunk_desc(0, col, 0)
        for i in range(d.n_pages):
            pg = d.pages[i]
            body = buf[pg.offset:pg.offset + pg.compressed_size].tobytes()
            kind = "dict" if pg.page_type == 2 else ("dictids" if pg.encoding in (2, 8) else "plain")
            if stamps:
                stamps(sbuf, 16, 1)
            t0 = time.perf_counter()
            got, fb = dec.snappy_decompress(body)
            print('PAGE', pf.columns[col].path[0], kind, len(body), flush=True)
            dt = time.perf_counter() - t0
            if stamps:
                stamps(sbuf, 16, 1)
                sacc[(pf.columns[col].path[0], kind)] += np.array(list(sbuf), dtype=float)
            ref = o.snappy_uncompress(body)
            st = stats[(pf.columns[col].path[0], kind)]
            st[0] += 1
            st[1][fb] += 1
            st[5] = max(st[5], len(body))
            st[2] += dt
            st[3] += len(body)
            st[4] += int(got != ref)
for k, v in sorted(stats.items()):
    line = (f"{k[0]:16s} {k[1]:8s} pages {v[0]:4d} paths {dict(v[1])} maxpage {v[5]} mismatch {v[4]} in {v[3] / 1e6:7.2f} MB "
            f"avg {v[2] / v[0] * 1e3:7.3f} ms")
    if stamps:
        s = sacc[k] / max(v[0], 1)
        line += " | fix/page: rounds %.1f steps %.0f reparse %.1f cyc total %.0fk lane0 %.0fk par %.0fk rep %.0fk splits %.0fk" % (
            s[0], s[1], s[2], s[3] / 1e3, s[6] / 1e3, s[7] / 1e3, s[8] / 1e3, s[9] / 1e3)
    print(line, flush=True)

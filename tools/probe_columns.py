"""Diagnostic: per-column stage times (HIP events on one context) for the SF1 bench file, each
column's 6 chunks decoded alone, device-resident. Usage: python tools/probe_columns.py [reps]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "parquet-floor_amd")]
import bench  # noqa: E402
from pfloor import _native  # noqa: E402
from pfloor.decoder import GpuDecoder  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
import argparse  # noqa: E402
from pfloor.decoder import ParquetFile  # noqa: E402
args = argparse.Namespace(workload="sf1", data_dir="/tmp/pfloor_bench")
path = bench.make_input(args)
pf = ParquetFile(path)
dec = GpuDecoder(0)
tot = {}
for col in range(pf.num_columns):
    bi = bench.BatchInput(pf, [(g, g, [col]) for g in range(pf.num_row_groups)], dec.h)
    bi.upload(dec)
    dd = bi.descs
    st = bench.page_stats(dd)
    acc = {}
    for r in range(reps + 1):
        dec.decode(dd, bi.dev.value, bi.nbytes, on_device=True)
        assert dec.wait() == 0, dec.error()
        if r:
            for k, v in dec.timing().items():
                acc[k] = acc.get(k, 0.0) + v / reps
    bi.free(dec)
    for k, v in acc.items():
        tot[k] = tot.get(k, 0.0) + v
    s = " ".join(f"{k}={v:.3f}" for k, v in acc.items() if k != "h2d" and v >= 0.005)
    print(f"{pf.columns[col].path[0]:16s} pages={st['pages']:4d} in={st['snappy_in'] / 1e6:6.1f}MB "
          f"out={st['snappy_out'] / 1e6:6.1f}MB sum={sum(v for k, v in acc.items() if k != 'h2d'):.3f} | {s}", flush=True)
print("TOTAL", " ".join(f"{k}={v:.3f}" for k, v in tot.items()), flush=True)

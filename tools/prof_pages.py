"""Diagnostic: per-page Snappy kernel durations. Run tools/probe_pages.py under
rocprofv3 --kernel-trace --output-format csv, then feed the kernel_trace.csv here: the i-th
dispatch of each Snappy kernel belongs to the i-th page probe_pages.py decompressed (column
order, row group 0). Prints per (column, page kind) mean/max duration of each kernel."""
import collections
import csv
import sys

trace, probe_list = sys.argv[1], sys.argv[2]
pages = [ln.split() for ln in open(probe_list) if ln.startswith("PAGE ")]
per = collections.defaultdict(list)
with open(trace) as f:
    for r in csv.DictReader(f):
        name = r["Kernel_Name"].split("(")[0].replace("pf::", "").replace("void ", "")
        if name.startswith("k_snappy"):
            per[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for name, durs in per.items():
    if name == "k_snappy_exec":      # two launches per page (pieces, whole-page redo)
        durs = [a + b for a, b in zip(durs[0::2], durs[1::2])]
    for (_, col, kind, size), d in zip(pages, durs):
        agg[(col, kind)][name].append((d, int(size)))
for key in sorted(agg):
    parts = []
    for name in ("k_snappy_index", "k_snappy_chain", "k_snappy_exec", "k_snappy_serial"):
        v = agg[key].get(name, [])
        if v:
            ds = [d for d, _ in v]
            parts.append(f"{name[8:]} mean {sum(ds) / len(ds) / 1e3:8.1f} max {max(ds) / 1e3:8.1f}us")
    print(f"{key[0]:16s} {key[1]:8s} n={len(agg[key]['k_snappy_chain']):3d} " + " | ".join(parts))

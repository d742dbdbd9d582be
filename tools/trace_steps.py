"""Per stream, every decode of a rocprofv3 kernel trace: start, length (first to last kernel of the
decode), and the idle gap since the previous decode ended — shows whether a stream waits for its
host thread (gaps) or is busy back to back (pipelined steps).
  python tools/trace_steps.py run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
t00 = min(int(r["Start_Timestamp"]) for r in rows)
for s in sorted({r["Stream_Id"] for r in rows}):
    rs = sorted((r for r in rows if r["Stream_Id"] == s), key=lambda r: int(r["Start_Timestamp"]))
    # a decode starts at its k_snappy_head (first kernel after the metadata upload / memsets)
    # decodes start at their metadata upload: k_copy_words launches alternate upload / results
    # download (zero-copy default); older traces: the Snappy index / head kernel
    cw = [i for i, r in enumerate(rs) if "k_copy_words" in r["Kernel_Name"]]
    starts = cw[0::2] if cw else [i for i, r in enumerate(rs) if "k_snappy_index" in r["Kernel_Name"] or
                                  "k_snappy_head" in r["Kernel_Name"]]
    if not starts:
        continue
    print(f"stream {s}: {len(starts)} decodes")
    prev_end = None
    for k, i0 in enumerate(starts):
        i1 = starts[k + 1] if k + 1 < len(starts) else len(rs)
        seg = [r for r in rs[i0:i1] if not r["Kernel_Name"].startswith("__amd")]
        a = int(seg[0]["Start_Timestamp"])
        b = max(int(r["End_Timestamp"]) for r in seg)
        gap = (a - prev_end) / 1e3 if prev_end is not None else 0.0
        print(f"  #{k:2d} start {(a - t00) / 1e3:10.1f} us  busy {(b - a) / 1e3:8.1f} us  idle before {gap:8.1f} us")
        prev_end = b

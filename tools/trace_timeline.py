"""Timeline of one stream's decode from a rocprofv3 kernel trace: per kernel launch, start/end
relative to the decode's first kernel, and the gaps in between (host enqueue latency, waits).
  python tools/trace_timeline.py run_kernel_trace.csv [stream_id] [which_decode]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sid = sys.argv[2] if len(sys.argv) > 2 else None
which = int(sys.argv[3]) if len(sys.argv) > 3 else -4
streams = sorted({r["Stream_Id"] for r in rows})
print("streams:", streams)
for s in ([sid] if sid else streams):
    rs = sorted((r for r in rows if r["Stream_Id"] == s), key=lambda r: int(r["Start_Timestamp"]))
    # a decode starts at the fillBuffer (bits memset) or the first k_snappy_index after a gap
    # decodes start at their metadata upload: k_copy_words launches alternate upload / results
    # download (zero-copy default); older traces: the Snappy index / head kernel
    up = [i for i, r in enumerate(rs) if "k_upload" in r["Kernel_Name"]]   # r05: the upload kernel
    cw = [i for i, r in enumerate(rs) if "k_copy_words" in r["Kernel_Name"]]
    starts = up if up else cw[0::2] if cw else [i for i, r in enumerate(rs) if "k_snappy_index" in r["Kernel_Name"] or
                                  "k_snappy_head" in r["Kernel_Name"]]
    if not starts:
        continue
    i0 = starts[which] if -len(starts) <= which < len(starts) else starts[-1]
    i1 = starts[starts.index(i0) + 1] if starts.index(i0) + 1 < len(starts) else len(rs)
    t0 = int(rs[i0]["Start_Timestamp"])
    prev_end = t0
    print(f"stream {s}: decode #{starts.index(i0)} of {len(starts)}")
    for r in rs[i0:i1]:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"  {(a - t0) / 1e3:8.1f} {(b - t0) / 1e3:8.1f}  dur {(b - a) / 1e3:7.1f}  gap {(a - prev_end) / 1e3:6.1f}  {r['Kernel_Name'].split('(')[0]}")
        prev_end = b

"""Per-launch durations from a rocprofv3 kernel trace of bench.py: for each kernel, the average of
its launches in the timed steps (both contexts, overlapped) and of the last ROOF_PASSES launches
(bench.py's isolated roofline passes, context 0 alone). Launches under 100 us of k_snappy_exec
are the whole-page redo launch and are listed apart.
  python tools/trace_launches.py gpurun_out/<tag>/prof/run_kernel_trace.csv [passes]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 3
per = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("pf::", "").replace("void ", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if n.startswith("k_snappy_exec") and d < 100:
        n += "_redo"
    per[n].append(d)
print(f"{'kernel':24s} {'launches':>8s} {'avg_us':>10s} {'avg_last%d_us' % passes:>14s}")
for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    last = v[-passes:]
    print(f"{n:24s} {len(v):8d} {sum(v) / len(v):10.1f} {sum(last) / len(last):14.1f}")
# the dominant kernel's last launches one by one (start relative to the first of them, queue, duration)
dom = max(per, key=lambda k: sum(per[k]))
rows_d = [r for r in rows if r["Kernel_Name"].split("(")[0].replace("pf::", "").replace("void ", "") == dom]
tail = rows_d[-3 * passes:]
if tail:
    t0 = int(tail[0]["Start_Timestamp"])
    print(f"\nlast {len(tail)} launches of {dom}: start_us queue dur_us")
    for r in tail:
        print(f"  {(int(r['Start_Timestamp']) - t0) / 1e3:10.1f} {r.get('Queue_Id', r.get('Stream_Id', '?')):>4s} "
              f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:8.1f}")

"""E2E leg timeline from a rocprofv3 --kernel-trace --memory-copy-trace run of bench.py: over the last
`window_ms` of activity (the streamed E2E passes), the busy time of H2D copies, downloads (k_download
kernels or D2H copies) and decode kernels, their overlaps, and the idle link time.
  python tools/e2e_timeline.py OUTDIR [window_ms]"""
import csv
import glob
import os
import sys

out = sys.argv[1]
win = float(sys.argv[2]) if len(sys.argv) > 2 else 100.0


def rows(pat):
    fs = glob.glob(os.path.join(out, "**", pat), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


kt = rows("*kernel_trace.csv")
mt = rows("*memory_copy_trace.csv")
ev = []   # (start, end, cat, stream)
for r in kt:
    n = r["Kernel_Name"]
    cat = "dl" if "k_download" in n else "kern"
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), cat, r.get("Stream_Id", "?")))
for r in mt:
    d = r.get("Direction", "")
    cat = "h2d" if "HOST_TO_DEVICE" in d.upper() else ("d2h" if "DEVICE_TO_HOST" in d.upper() else "copy")
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), cat, "?"))
if not ev:
    sys.exit("no trace rows")
t1 = max(e[1] for e in ev)
t0 = t1 - int(win * 1e6)
ev = [(max(a, t0), b, c, s) for a, b, c, s in ev if b > t0]


def union(iv):
    iv = sorted(iv)
    tot, cur = 0, None
    for a, b in iv:
        if cur is None or a > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur:
        tot += cur[1] - cur[0]
    return tot


cats = sorted({e[2] for e in ev})
print(f"window {win:.0f} ms; events {len(ev)}")
for c in cats:
    iv = [(a, b) for a, b, cc, _ in ev if cc == c]
    print(f"  {c:5s} busy {union(iv) / 1e6:7.2f} ms  ({len(iv)} events, sum {sum(b - a for a, b in iv) / 1e6:.2f} ms)")
dl = [(a, b) for a, b, c, _ in ev if c in ("dl", "d2h")]
h2d = [(a, b) for a, b, c, _ in ev if c == "h2d"]
print(f"  link busy (any H2D or download) {union(dl + h2d) / 1e6:.2f} ms; download-or-D2H busy {union(dl) / 1e6:.2f} ms")
# downloads one by one: duration and the gap since the previous download ended (any stream)
dls = sorted((a, b, s) for a, b, c, s in ev if c == "dl")
if dls:
    durs = [(b - a) / 1e3 for a, b, _ in dls]
    gaps, last = [], None
    for a, b, _ in dls:
        if last is not None and a > last:
            gaps.append((a - last) / 1e3)
        last = b if last is None else max(last, b)
    print(f"  downloads: {len(dls)}, duration us min {min(durs):.0f} avg {sum(durs) / len(durs):.0f} max {max(durs):.0f}; "
          f"idle gaps between downloads {len(gaps)}, total {sum(gaps) / 1e3:.2f} ms, max {max(gaps) if gaps else 0:.0f} us")
    conc = sum(1 for i in range(1, len(dls)) if dls[i][0] < dls[i - 1][1])
    print(f"  downloads starting while the previous one runs: {conc}")

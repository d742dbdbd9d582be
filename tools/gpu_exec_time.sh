#!/bin/bash
# Per-page executor kernel durations (rocprofv3 kernel trace of tools/probe_exec_time.py).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/${1:-xt}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for X in ${2:-2}; do for NS in ${3:-4}; do
PF_NSUB=$NS PF_EXEC=$X timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/x$X$NS" -o run -- python3 "$ROOT/tools/probe_exec_time.py" > "$OUT/x$X$NS.log" 2>&1 || { tail -20 "$OUT/x$X$NS.log"; exit 1; }
f=$(find "$OUT/x$X$NS" -name '*kernel_trace.csv' | head -1)
python3 - "$f" "$X" "$NS" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_snappy_exec" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
# two executor launches per call (pieces, whole-page redo): keep the piece launches
print("PF_EXEC", sys.argv[2], "NSUB", sys.argv[3], "piece-launch us:", [round(x, 1) for x in d[0::2]])
PY
done; done

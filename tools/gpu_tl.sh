#!/bin/bash
# Per-stream timeline of the SF1 step: a rocprofv3 kernel trace of a short bench (timed steps,
# four streams), then the kernels of one decode per stream.   tools/gpu_tl.sh TAG [bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/${1:-tl}"; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-pmc --no-e2e --no-parity --no-write "$@" > "$OUT/prof.log" 2>&1 || { tail -30 "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
python3 "$ROOT/tools/trace_timeline.py" "$f" "" ${WHICH:--12} > "$OUT/timeline.txt"
s=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
cp "$s" "$OUT/kernel_stats.csv"
head -c 400 "$OUT/prof.log" | tail -c 200
tail -3 "$OUT/timeline.txt"

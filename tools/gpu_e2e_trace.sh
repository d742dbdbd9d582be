#!/bin/bash
# rocprofv3 kernel + memory-copy trace of bench.py's E2E leg (a short device-resident part first).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/${1:-e2e_trace}"; shift; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-pmc --no-write --no-parity "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 "$ROOT/tools/e2e_timeline.py" "$OUT/tr" 110 | tee "$OUT/timeline.txt"

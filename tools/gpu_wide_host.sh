#!/bin/bash
# Config 4 (wide): host planning per batch (PF_DEBUG_PLAN=1) and a kernel trace of the pipelined
# steps with each stream's idle gaps between decodes (tools/trace_steps.py).
#   tools/gpu_wide_host.sh TAG [bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-wide_host}"; shift
mkdir -p "$OUT"
B="--workload wide --no-cpu-baseline --no-pmc --no-e2e --no-write"
PF_DEBUG_PLAN=1 timeout -k 10 300 python -u bench.py $B --steps 20 --warmup 2 "$@" > "$OUT/plan.json" 2> "$OUT/plan.err" || { tail -30 "$OUT/plan.err"; exit 1; }
grep '\[pf plan\]' "$OUT/plan.err" | tail -12
python3 -c "import json; d=json.load(open('$OUT/plan.json')); print(d['ms_per_step'], d.get('host_enqueue_ms_per_batch'), {k: round(v,3) for k,v in d['stage_ms'].items()})"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" $B --steps 10 --warmup 1 --no-parity "$@" > "$OUT/prof.log" 2>&1 || { tail -30 "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
python3 "$ROOT/tools/trace_steps.py" "$f" > "$OUT/steps.txt"
python3 "$ROOT/tools/trace_launches.py" "$f" 3 > "$OUT/launches.txt"
tail -16 "$OUT/steps.txt"; head -20 "$OUT/launches.txt"
rm -rf "$OUT/prof"

#!/bin/bash
# Interleaved A/B of bench.py argument sets (same library): each variant REPS times, round-robin.
#   tools/gpu_ab_args.sh TAG REPS "args A" "args B" ...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-abargs}"; REPS=${2:-2}; shift 2
mkdir -p "$OUT"
for rep in $(seq 1 $REPS); do
  i=0
  for A in "$@"; do
    i=$((i+1))
    timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write $A > "$OUT/bench_v${i}_$rep.json" 2>> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_v${i}_$rep.json')); print('v$i [$A]', d['ms_per_step'], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
  done
done

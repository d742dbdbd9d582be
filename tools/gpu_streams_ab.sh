#!/bin/bash
# SF1 step vs number of decode streams (contexts) per GPU.  tools/gpu_streams_ab.sh TAG S1 S2 ...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-streams}"; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for S in "$@"; do
    timeout -k 10 300 python -u bench.py --steps 50 --warmup 3 --streams $S --no-cpu-baseline --no-pmc --no-e2e --no-write --no-parity > "$OUT/b_${S}_$rep.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${S}_$rep.json')); print('streams $S', d['ms_per_step'], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()})"
  done
done

#!/bin/bash
# SF1 plan: LPT chunk cost + row_cost bytes per row (--row-cost 0 / 0.5 / 1 / 2), interleaved.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-rowcost}"; mkdir -p "$OUT"
for i in 1 2; do
  for rc in 0 0.5 1 2; do
    timeout -k 10 200 python -u bench.py --row-cost $rc --steps 80 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/b_${rc}_$i.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${rc}_$i.json')); print('row_cost $rc', d['ms_per_step'], d['parity']['bit_exact'])"
  done
done

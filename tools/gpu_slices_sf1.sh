#!/bin/bash
# SF1 column-slice granularity (--slice-mult 1 / 2 / 3), three interleaved rounds.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-slices_sf1}"; mkdir -p "$OUT"
for i in 1 2 3; do
  for m in 1 2 3; do
    timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --slice-mult $m --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/b_${m}_$i.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${m}_$i.json')); print('slice x$m', d['ms_per_step'], d['parity']['bit_exact'])"
  done
done

#!/bin/bash
# SF1 decode streams per GPU (3 / 4 / 5) with the default plan, interleaved.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-streams_sf1}"; mkdir -p "$OUT"
for i in 1 2; do
  for S in 4 3 5; do
    timeout -k 10 200 python -u bench.py --streams $S --steps 60 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/b_${S}_$i.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${S}_$i.json')); print('streams $S', d['ms_per_step'], d['parity']['bit_exact'])"
  done
done

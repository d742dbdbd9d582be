#!/bin/bash
# SF1 plan variants on top of slice x2 (the default), interleaved.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-plan_sf1b}"; mkdir -p "$OUT"
run() {
  local n=$1; shift
  timeout -k 10 200 python -u bench.py "$@" --steps 100 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/b_$n.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', d['ms_per_step'], d['parity']['bit_exact'])"
}
for i in 1 2; do
  run def_$i
  run sw075_$i --string-weight 0.75
  run sw15_$i --string-weight 1.5
  run dec_$i --lpt-cost decompressed
done

#!/bin/bash
# Column-slice granularity (bench --slice-mult) on the column-split workloads, interleaved.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-slices}"; mkdir -p "$OUT"
run() {
  local n=$1; shift
  timeout -k 10 200 python -u bench.py "$@" --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/b_$n.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', d['ms_per_step'], d['parity']['bit_exact'])"
}
for i in 1 2; do
  run nest1_$i --workload nested --steps 100
  run nest2_$i --workload nested --steps 100 --slice-mult 2
  run nest4_$i --workload nested --steps 100 --slice-mult 4
  run flat2_$i --workload flat --steps 100 --slice-mult 2
  run sf1_1_$i --steps 60
  run sf1_2_$i --steps 60 --slice-mult 2
done

#!/bin/bash
# Stream-plan variants of the latency-bound workloads, interleaved.   tools/gpu_plan.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-plan}"; mkdir -p "$OUT"
run() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 200 python -u bench.py "$@" --steps 100 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/b_$n.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', d['ms_per_step'], d['parity']['bit_exact'], d['config']['parallelism'][-90:])"
}
for i in 1 2; do
  run flat_def_$i --workload flat
  run flat_sw3_$i --workload flat --string-weight 3
  run flat_sw6_$i --workload flat --string-weight 6
  run flat_dec_$i --workload flat --lpt-cost decompressed
  run nest_def_$i --workload nested
  run nest_dec_$i --workload nested --lpt-cost decompressed
  run nest_kinds_$i --workload nested --split kinds --string-ctx 2
done

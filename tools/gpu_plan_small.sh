#!/bin/bash
# Configs 1 / 5: column split (default) vs one row group per batch, interleaved.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-plan_small}"; mkdir -p "$OUT"
run() {
  local n=$1; shift
  timeout -k 10 200 python -u bench.py "$@" --steps 100 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/b_$n.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', d['ms_per_step'], d['parity']['bit_exact'])"
}
for i in 1 2; do
  run nest_def_$i --workload nested
  run nest_rg_$i --workload nested --split rowgroups --rg-batch 1
  run flat_def_$i --workload flat
  run flat_rg_$i --workload flat --split rowgroups --rg-batch 1
done

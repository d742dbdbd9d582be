#!/bin/bash
# Stage ablation (diagnostics build, results wrong by design): SF1 step with each PF_DEBUG_SKIP bit alone,
# interleaved with the unskipped diag library.  tools/gpu_ablate.sh TAG [ROUNDS] [bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-ablate}"; mkdir -p "$OUT"
export PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_diag.so
for i in $(seq 1 ${2:-2}); do
  for b in none parse exec ba levels count flat decode; do
    f="$OUT/b_skip${b}_$i.json"
    if [ $b == none ]; then unset PF_DEBUG_SKIP; else export PF_DEBUG_SKIP=$b; fi
    timeout -k 10 300 python -u bench.py ${3:-} --steps 100 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write --no-parity > "$f" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    python -c "import json; d=json.load(open('$f')); print('skip $b', d['ms_per_step'])"
  done
done

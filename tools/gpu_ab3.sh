#!/bin/bash
# Three interleaved rounds of SF1 bench lines: the product library against diag/libpfloor_<name>.so variants.
#   tools/gpu_ab3.sh TAG name...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-ab3}"; shift; mkdir -p "$OUT"
for i in 1 2 3; do
  for r in base "$@"; do
    if [ $r == base ]; then unset PFLOOR_LIB_PATH; else export PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_$r.so; fi
    timeout -k 10 200 python -u bench.py ${BARGS:-} --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/b_${r}_$i.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${r}_$i.json')); print('$r', d['ms_per_step'], d['parity']['bit_exact'])"
  done
done

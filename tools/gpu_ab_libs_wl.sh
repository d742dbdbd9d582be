#!/bin/bash
# Interleaved A/B of library variants (parquet-floor_amd/diag/libpfloor_<name>.so) on one workload:
#   tools/gpu_ab_libs_wl.sh TAG "bench args" name...   (parity checked in every bench line)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-libswl}"; shift
BARGS=$1; shift
mkdir -p "$OUT"
for i in 1 2; do
  for r in base "$@" base_end; do
    if [ ${r%_end} == base ]; then unset PFLOOR_LIB_PATH; else export PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_$r.so; fi
    timeout -k 10 300 python -u bench.py $BARGS --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/b_${r}_$i.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_${r}_$i.json')); print('$r', d['ms_per_step'], {k: round(v,3) for k,v in d['stage_ms'].items() if v > 0.02}, d['parity']['bit_exact'])"
  done
done

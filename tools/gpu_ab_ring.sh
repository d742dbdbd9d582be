#!/bin/bash
# A/B of the executor ring size: parity tests per variant, then interleaved bench runs.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-ring}"
mkdir -p "$OUT"
for r in 8192 16384; do
  PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_ring$r.so timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_$r.log" 2>&1 || { tail -30 "$OUT/pytest_$r.log"; exit 1; }
  tail -1 "$OUT/pytest_$r.log"
done
for i in 1 2; do
  for r in base 8192 16384; do
    if [ $r == base ]; then unset PFLOOR_LIB_PATH; else export PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_ring$r.so; fi
    timeout -k 10 300 python -u bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/b_${r}_$i.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_${r}_$i.json')); print('$r', d['ms_per_step'], d['roofline']['launch_ms'], round(d['stage_ms']['snappy_exec'],3), d['parity']['bit_exact'])"
  done
done

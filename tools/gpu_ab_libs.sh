#!/bin/bash
# A/B of library variants in parquet-floor_amd/diag/libpfloor_<name>.so: parity tests per variant,
# then interleaved bench runs with the default library ("base").  tools/gpu_ab_libs.sh TAG name...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-libs}"; shift
mkdir -p "$OUT"
for r in "$@"; do
  [ -n "$NOTEST" ] && continue
  PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_$r.so timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_$r.log" 2>&1 || { echo "$r FAILED"; tail -30 "$OUT/pytest_$r.log"; exit 1; }
  echo "$r $(tail -1 $OUT/pytest_$r.log)"
done
for i in 1 2; do
  for r in base "$@" base_end; do   # base first and last: the first run of a round is not favoured
    if [ ${r%_end} == base ]; then unset PFLOOR_LIB_PATH; else export PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_$r.so; fi
    timeout -k 10 300 python -u bench.py ${BARGS:-} --steps ${STEPS:-200} --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/b_${r}_$i.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_${r}_$i.json')); print('$r', d['ms_per_step'], d['roofline']['kernel'][:14], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items() if k in ('snappy_exec','flat','count','snappy_parse')}, d['parity']['bit_exact'])"
  done
done

#!/bin/bash
# Interleaved A/B of environment variants of the default library (e.g. PF_EXEC=2 vs the default):
#   tools/gpu_ab_env.sh TAG ROUNDS "bench args" VAR=VAL[,VAR=VAL] ...   ("base" = no extra variables)
# Each variant first passes the Snappy / parity tests; then ROUNDS passes over all variants.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-abenv}"; shift
R=${1:-2}; shift
BARGS=$1; shift
mkdir -p "$OUT"
run_env() {   # run_env "A=1,B=2" cmd...
  local spec=$1; shift
  if [ "$spec" == base ]; then "$@"; else env $(echo "$spec" | tr ',' ' ') "$@"; fi
}
for v in "$@"; do
  [ "$v" == base ] && continue
  [ -n "$NOTEST" ] && continue
  run_env "$v" timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_parity.py tests/test_gpu_direct.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_${v//[=,]/_}.log" 2>&1 || { echo "$v FAILED"; tail -30 "$OUT/pytest_${v//[=,]/_}.log"; exit 1; }
  echo "$v $(tail -1 $OUT/pytest_${v//[=,]/_}.log)"
done
for i in $(seq 1 $R); do
  for v in "$@"; do
    f="$OUT/b_${v//[=,]/_}_$i.json"
    run_env "$v" timeout -k 10 300 python -u bench.py $BARGS --no-cpu-baseline --no-pmc --no-e2e --no-write > "$f" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    python -c "import json; d=json.load(open('$f')); print('$v', d['ms_per_step'], d['roofline']['kernel'][:14], d['roofline'].get('launch_ms'), {k: round(v,3) for k,v in d['stage_ms'].items()}, d.get('parity', {}).get('bit_exact'))"
  done
done

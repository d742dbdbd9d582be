#!/bin/bash
# Executor A/B: Snappy / direct / parity GPU tests on the default executor, then interleaved SF1
# bench lines with the default executor and PF_EXEC=5.   tools/gpu_x6.sh TAG [pairs] [bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-x6}"; shift
N=${1:-2}; shift
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_direct.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" "$OUT/pytest.log" | head -30; tail -40 "$OUT/pytest.log"; exit 1; }
for i in $(seq 1 $N); do
  for v in 6 5; do
    PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_diag.so PF_EXEC=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-pmc --no-e2e "$@" > "$OUT/bench_${v}_$i.json" 2>> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$i.json')); print('exec$v', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
  done
done

#!/bin/bash
# A/B of environment settings on the SF1 bench (parity checked every run), after the GPU tests.
#   tools/gpu_ab_env.sh TAG "ENV1" "ENV2" ...   e.g. "PF_EXEC=2" "PF_NSUB=2"
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-ab}"; shift
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_delta_bytes.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { tail -60 "$OUT/pytest.log"; exit 1; }
i=0
for rep in 1 2; do
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-pmc --no-e2e > "$OUT/bench_$i.json" 2>> "$OUT/bench.err" || { echo "FAIL $E"; tail -30 "$OUT/bench.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$i.json')); print('$E', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
done
done

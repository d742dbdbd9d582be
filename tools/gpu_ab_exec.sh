#!/bin/bash
# Executor A/B on the gpurun box: GPU tests with the default executor, then the SF1 bench with
# PF_EXEC=1 (token-serial) and the default (byte-lane v2), interleaved.  tools/gpu_ab_exec.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-abx}"
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_delta_bytes.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { tail -50 "$OUT/pytest.log"; exit 1; }
for i in 1 2; do
  for X in 1 2; do
    PF_EXEC=$X timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-pmc --no-e2e > "$OUT/bench_x${X}_$i.json" 2>> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
    python -c "import json,sys; d=json.load(open('$OUT/bench_x${X}_$i.json')); print('X=$X', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['launch_ms'], d['stage_ms'].get('snappy_exec'), d['parity']['bit_exact'])"
  done
done

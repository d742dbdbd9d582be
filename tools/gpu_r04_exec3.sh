#!/bin/bash
# r04: the 4-wave executor (PF_EXEC=3): Snappy / parity / direct / scale GPU tests, then an A/B of
# exec2 vs exec3 on SF1 (interleaved).  tools/gpu_r04_exec3.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
OUT=$PWD/gpurun_out/${1:-exec3}; mkdir -p $OUT
export PF_EXEC=3
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py -m gpu -x -v --timeout 60 --timeout-method thread > $OUT/pytest_snappy.log 2>&1
rc=$?; tail -3 $OUT/pytest_snappy.log; [ $rc -eq 0 ] || { tail -40 $OUT/pytest_snappy.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_direct.py tests/test_gpu_scale.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -40 $OUT/pytest.log; exit 1; }
B="--no-cpu-baseline --no-pmc --no-e2e --no-write --steps 100 --warmup 5"
for i in 1 2; do
  for e in 2 3; do
    PF_EXEC=$e timeout -k 10 200 python -u bench.py $B > $OUT/b$e.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b$e.json')); print('exec$e', d['ms_per_step'], d['roofline']['kernel'][:20], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
  done
done

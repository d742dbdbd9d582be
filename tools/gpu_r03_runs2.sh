#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
OUT=gpurun_out/r03_runs2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -60 $OUT/pytest.log; exit 1; }
PFLOOR_LIB_PATH=$PWD/parquet-floor_amd/diag/libpfloor_ft4096.so timeout -k 10 300 python -u -m pytest tests/test_short_runs.py tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -q --timeout 150 --timeout-method thread > $OUT/pytest_ft4096.log 2>&1
rc=$?; echo "ft4096 rc=$rc"; tail -3 $OUT/pytest_ft4096.log
exit 0

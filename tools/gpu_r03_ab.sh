#!/bin/bash
# full GPU tests of the in-tree build, then interleaved SF1 A/B of diag/libpfloor_base.so vs diag/libpfloor_new.so
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
OUT=gpurun_out/${1:-r03_ab}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -60 $OUT/pytest.log; exit 1; }
tools/gpu_ab_libs2.sh ${1:-r03_ab} ${2:-3} parquet-floor_amd/diag/libpfloor_base.so parquet-floor_amd/diag/libpfloor_new.so

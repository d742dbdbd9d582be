#!/bin/bash
# ba_cand A/B: full tests with the current build, interleaved bench of the two builds, and a kernel trace.
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
OUT=gpurun_out/r03_cand; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -60 $OUT/pytest.log; exit 1; }
tools/gpu_ab_libs2.sh r03_cand 2 parquet-floor_amd/diag/libpfloor_cand1.so parquet-floor_amd/diag/libpfloor_cand2.so || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-e2e --no-parity --no-write > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/prof.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/$OUT/prof -name '*kernel_trace.csv' | head -1)
python3 $GRAFT_REPO_ROOT/tools/trace_launches.py "$f" 3 > $GRAFT_REPO_ROOT/$OUT/launches.txt; head -20 $GRAFT_REPO_ROOT/$OUT/launches.txt

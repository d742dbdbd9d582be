#!/bin/bash
# r04: k_page_null (one workgroup per nullable flat page): its tests, the whole GPU suite, then
# wide / flat / SF1 lines with and without it (PF_PAGE_NULL=0).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
OUT=$PWD/gpurun_out/${1:-r04_o}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_page_null.py -x -q --timeout 150 --timeout-method thread > $OUT/pytest_pn.log 2>&1
rc=$?; tail -2 $OUT/pytest_pn.log; [ $rc -eq 0 ] || { tail -60 $OUT/pytest_pn.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -40 $OUT/pytest.log; exit 1; }
PFLOOR_LIB_PATH=$PWD/parquet-floor_amd/diag/libpfloor_stamps.so timeout -k 10 300 python -u tools/probe_flat_cols.py > $OUT/probe_flat.log 2>&1 || { tail -20 $OUT/probe_flat.log; exit 1; }
cat $OUT/probe_flat.log
B="--no-cpu-baseline --no-pmc --no-e2e --no-write --steps 50 --warmup 5"
one() { local tag=$1 pn=$2; shift 2
  PF_PAGE_NULL=$pn timeout -k 10 400 python -u bench.py $B "$@" > $OUT/b_$tag.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['kernel'][:30], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"; }
one wide 1 --workload wide && one wide_off 0 --workload wide && one wide1k 1 --workload wide --pool 1000 && \
one flat 1 --workload flat && one flat_off 0 --workload flat && one sf1 1

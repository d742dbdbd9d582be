#!/bin/bash
# r04: k_flat_null gathers issued back to back (global loads), zero-copy metadata / results by
# default: tests, wide stamps, wide / SF1 / flat lines.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
OUT=$PWD/gpurun_out/${1:-r04_n}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -40 $OUT/pytest.log; exit 1; }
PFLOOR_LIB_PATH=$PWD/parquet-floor_amd/diag/libpfloor_stamps.so timeout -k 10 300 python -u tools/probe_wide.py 100000 64 > $OUT/probe_wide.log 2>&1 || { tail -20 $OUT/probe_wide.log; exit 1; }
cat $OUT/probe_wide.log
B="--no-cpu-baseline --no-pmc --no-e2e --no-write --steps 50 --warmup 5"
one() { local tag=$1; shift
  timeout -k 10 400 python -u bench.py $B "$@" > $OUT/b_$tag.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['kernel'][:30], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"; }
one wide --workload wide && one wide_b --workload wide && one wide1k --workload wide --pool 1000 && one sf1 && one flat --workload flat

#!/bin/bash
# r04: multi-literal litcopy + k_flat_null LDS dictionaries: GPU tests, SF1 line, wide pool lines
# (1K with / without the LDS dictionary, 16K, 100K).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
OUT=$PWD/gpurun_out/${1:-r04_e}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_snappy.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -40 $OUT/pytest.log; exit 1; }
B="--no-cpu-baseline --no-pmc --no-e2e --no-write --steps 50 --warmup 5"
one() { local tag=$1; shift
  timeout -k 10 400 python -u bench.py $B "$@" > $OUT/b_$tag.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$tag.json')); print('$tag', d['ms_per_step'], d.get('host_enqueue_ms_per_batch'), d['roofline']['kernel'][:30], d['roofline']['launch_ms'], d['roofline']['frac'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"; }
one sf1
one sf1_lptcomp --lpt-cost compressed
one sf1b
one wide100k --workload wide
one wide1k --workload wide --pool 1000
PF_NULL_DICT_LDS=0 one wide1k_nolds --workload wide --pool 1000
one wide16k --workload wide --pool 16000

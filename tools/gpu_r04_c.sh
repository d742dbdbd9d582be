#!/bin/bash
# r04: wide-window executor (PF_EXEC=4) GPU tests, A/B against exec2 with 4 / 8 / 16 KiB rings,
# and a kernel trace of the wide workload (config 4).  tools/gpu_r04_c.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
OUT=$PWD/gpurun_out/${1:-r04_c}; mkdir -p $OUT
PF_EXEC=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py -m gpu -x -v --timeout 60 --timeout-method thread > $OUT/pytest_snappy.log 2>&1
rc=$?; tail -3 $OUT/pytest_snappy.log; [ $rc -eq 0 ] || { tail -40 $OUT/pytest_snappy.log; exit 1; }
PF_EXEC=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_direct.py tests/test_gpu_scale.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -40 $OUT/pytest.log; exit 1; }
for r in 8 16; do
  PF_EXEC=4 PFLOOR_LIB_PATH=$PWD/parquet-floor_amd/diag/libpfloor_x4r$r.so timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_direct.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_r$r.log 2>&1
  rc=$?; tail -1 $OUT/pytest_r$r.log; [ $rc -eq 0 ] || { tail -40 $OUT/pytest_r$r.log; exit 1; }
done
B="--no-cpu-baseline --no-pmc --no-e2e --no-write --steps 100 --warmup 5"
one() { local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py $B > $OUT/b_$tag.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"; }
for i in 1 2; do
  one exec2 PF_EXEC=2
  one x4r4 PF_EXEC=4
  one x4r8 PF_EXEC=4 PFLOOR_LIB_PATH=$PWD/parquet-floor_amd/diag/libpfloor_x4r8.so
  one x4r16 PF_EXEC=4 PFLOOR_LIB_PATH=$PWD/parquet-floor_amd/diag/libpfloor_x4r16.so
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload wide --steps 5 --warmup 1 --warmup-s 0 --no-cpu-baseline --no-pmc --no-e2e --no-parity --no-write > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
python3 $GRAFT_REPO_ROOT/tools/trace_timeline.py "$f" > $OUT/wide_timeline.txt 2>&1
python3 $GRAFT_REPO_ROOT/tools/trace_launches.py "$f" 3 > $OUT/wide_launches.txt 2>&1
rm -rf $OUT/prof
head -50 $OUT/wide_timeline.txt

#!/bin/bash
# r04: where does the 20-step line lose to the 300-step line?  tools/gpu_r04_steps.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
OUT=$PWD/gpurun_out/${1:-steps}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_dbp_config.py tests/test_gpu_nest_seg.py tests/test_gpu_scale.py -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -40 $OUT/pytest.log; exit 1; }
B="--no-cpu-baseline --no-pmc --no-e2e --no-write --no-parity"
run() { timeout -k 10 200 python -u bench.py $B "$@" > $OUT/b.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
        python3 -c "import json,sys; d=json.load(open('$OUT/b.json')); print(sys.argv[1:], d['ms_per_step'])" "$@"; }
run --steps 20 --warmup 5
run --steps 20 --warmup 5
run --steps 300 --warmup 5
run --steps 20 --warmup 100
run --steps 20 --warmup 5
run --steps 100 --warmup 100
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-e2e --no-parity --no-write > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
python3 $GRAFT_REPO_ROOT/tools/trace_timeline.py "$f" > $OUT/timeline.txt 2>&1
python3 $GRAFT_REPO_ROOT/tools/trace_launches.py "$f" 3 > $OUT/launches.txt 2>&1
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof

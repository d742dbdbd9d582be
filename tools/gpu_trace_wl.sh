#!/bin/bash
# Kernel trace of a short bench of one workload; per-stream timeline of one decode.
#   tools/gpu_trace_wl.sh TAG [bench args]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
OUT=$PWD/gpurun_out/${1:-trace}; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-e2e --no-parity --no-write "$@" > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
python3 $GRAFT_REPO_ROOT/tools/trace_launches.py "$f" 3 > $OUT/launches.txt; head -24 $OUT/launches.txt
python3 $GRAFT_REPO_ROOT/tools/trace_timeline.py "$f" > $OUT/timeline.txt 2>&1

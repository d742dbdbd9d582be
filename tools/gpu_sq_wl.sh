#!/bin/bash
# SQ counters (wave cycles, instruction mix) per kernel for one workload at 1 stream.
#   tools/gpu_sq_wl.sh TAG KREGEX [bench args]
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
TAG=$1; K=$2; shift 2
KREGEX="$K" tools/gpu_pmc_sq.sh $TAG "$@" || exit 1
f=$(find gpurun_out/$TAG/sq -name '*counter_collection.csv' | head -1)
python3 tools/sq_summary.py $f > gpurun_out/$TAG/summary.txt && cat gpurun_out/$TAG/summary.txt

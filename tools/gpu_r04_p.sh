#!/bin/bash
# r04: kernel traces of config 5 (nested) and config 1 (flat), one stream and four: per-kernel
# launch times and one decode's timeline per stream.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
tools/gpu_trace_wl.sh ${1:-r04_p}/nested1 --workload nested --streams 1 && \
tools/gpu_trace_wl.sh ${1:-r04_p}/nested4 --workload nested && \
tools/gpu_trace_wl.sh ${1:-r04_p}/flat1 --workload flat --streams 1 && \
tools/gpu_trace_wl.sh ${1:-r04_p}/flat4 --workload flat && \
for d in nested1 nested4 flat1 flat4; do rm -rf gpurun_out/${1:-r04_p}/$d/prof; done

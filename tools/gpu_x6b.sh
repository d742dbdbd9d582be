#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/p6b
PFLOOR_LIB_PATH=$PWD/parquet-floor_amd/diag/libpfloor_stamps.so timeout -k 10 300 python -u tools/probe_exec6.py > gpurun_out/p6b/probe.log 2>&1 || { tail -20 gpurun_out/p6b/probe.log; exit 1; }
tail -5 gpurun_out/p6b/probe.log
bash tools/gpu_x6.sh x6b 1

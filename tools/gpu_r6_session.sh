#!/bin/bash
# Round-6 session: executor tests + probes + A/B (tools/gpu_exec_ab.sh), then the PCIe duplex probe.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
TAG=${1:-r6}
mkdir -p gpurun_out/$TAG
PROBE_FIRST=1 tools/gpu_exec_ab.sh $TAG || exit 1
timeout -k 10 120 python -u tools/probe_link.py 512 > gpurun_out/$TAG/link.txt 2>&1 || { cat gpurun_out/$TAG/link.txt; exit 1; }
HSA_ENABLE_SDMA=0 timeout -k 10 120 python -u tools/probe_link.py 512 >> gpurun_out/$TAG/link.txt 2>&1 || { cat gpurun_out/$TAG/link.txt; exit 1; }
cat gpurun_out/$TAG/link.txt

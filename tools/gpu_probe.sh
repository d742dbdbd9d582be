#!/bin/bash
# Per-page Snappy kernel durations on the gpurun box (tools/prof_pages.py reads the result).
#   tools/gpu_probe.sh TAG [rows]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-pp}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/tools/probe_pages.py" "${2:-1048576}" > "$OUT/probe.log" 2>&1

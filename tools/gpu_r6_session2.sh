#!/bin/bash
# Round-6 session: executor tests + stamps + A/B vs variants, then one full bench line (E2E included).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
TAG=${1:-r6}; shift
mkdir -p gpurun_out/$TAG
tools/gpu_exec_ab.sh $TAG "$@" || exit 1
timeout -k 10 600 python -u bench.py --steps 100 > gpurun_out/$TAG/bench_full.json 2> gpurun_out/$TAG/bench_full.err || { tail -20 gpurun_out/$TAG/bench_full.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/$TAG/bench_full.json')); print(d['ms_per_step'], d.get('e2e'))"

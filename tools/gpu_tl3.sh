#!/bin/bash
# Per-stream timelines of the flat (config 1), nested (config 5) and wide (config 4) workloads.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
for wl in flat nested wide; do
  bash tools/gpu_tl.sh tl_$wl --workload $wl > /dev/null 2>&1 || { echo "$wl failed"; tail -20 gpurun_out/tl_$wl/prof.log; exit 1; }
  timeout -k 10 200 python -u bench.py --workload $wl --steps 30 --warmup 3 --no-cpu-baseline --no-pmc --no-e2e --no-write > gpurun_out/tl_$wl/bench.json 2> gpurun_out/tl_$wl/bench.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/tl_$wl/bench.json')); print('$wl', d['ms_per_step'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
done

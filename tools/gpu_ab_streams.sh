#!/bin/bash
# A/B of hardware-queue / decode-stream settings on the SF1 bench (parity checked every run).
#   tools/gpu_ab_streams.sh TAG "ENV|STREAMS" ...   e.g. "GPU_MAX_HW_QUEUES=8|6"
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-abs}"; shift
mkdir -p "$OUT"
i=0
for rep in 1 2; do
for C in "$@"; do
  i=$((i+1))
  E="${C%%|*}"; S="${C##*|}"
  env $E timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --streams $S --no-cpu-baseline --no-pmc --no-e2e > "$OUT/bench_$i.json" 2>> "$OUT/bench.err" || { echo "FAIL $C"; tail -30 "$OUT/bench.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$i.json')); print('$C', d['ms_per_step'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
done
done

#!/bin/bash
# SF1 step vs decode streams and hardware queues (GPU_MAX_HW_QUEUES), interleaved.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-hwq}"; mkdir -p "$OUT"
B="--steps 150 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write"
for i in 1 2; do
  for cfg in "4 4" "8 4" "8 5" "8 6" "8 8" "4 4"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 300 python -u bench.py $B --streams $2 > "$OUT/q$1_s$2_$i.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/q$1_s$2_$i.json')); print('q$1 s$2', d['ms_per_step'], d['parity']['bit_exact'])"
  done
done

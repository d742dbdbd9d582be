#!/bin/bash
# Stream plan A/B: --string-weight (LPT cost multiplier of BYTE_ARRAY chunks) on the latency-bound
# workloads, interleaved.   tools/gpu_sw.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-sw}"; mkdir -p "$OUT"
for i in 1 2; do
  for wl in flat nested; do
    for sw in 1 2 4 8; do
      timeout -k 10 200 python -u bench.py --workload $wl --string-weight $sw --steps 100 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/b_${wl}_${sw}_$i.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/b_${wl}_${sw}_$i.json')); print('$wl sw=$sw', d['ms_per_step'], d['parity']['bit_exact'])"
    done
  done
done

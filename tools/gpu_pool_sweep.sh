#!/bin/bash
# SURVEY 8(d) config-4 pool sweep: one --workload wide bench line (roofline + PMC traffic) per pool size.
#   tools/gpu_pool_sweep.sh TAG [pools...]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-pool}"; shift
POOLS=${*:-1000 16000 32000 64000 100000}
mkdir -p "$OUT"
for P in $POOLS; do
  timeout -k 10 500 python -u bench.py --workload wide --pool $P --steps 30 --warmup 3 --no-cpu-baseline --no-e2e --no-write > "$OUT/wide_pool$P.json" 2>> "$OUT/bench.err" || { echo "FAIL pool $P"; tail -30 "$OUT/bench.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/wide_pool$P.json')); r=d['roofline']; print($P, d['ms_per_step'], d['value'], r['kernel'], r['launch_ms'], r['frac'], r['traffic'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
done

#!/bin/bash
# Bench lines of configs 1 (flat), 5 (nested), 4 (wide) and 3 (sf100) with stage times.  tools/gpu_cfgs.sh TAG [workloads]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-cfgs}"; shift
mkdir -p "$OUT"
for w in ${@:-flat nested wide}; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/b_$w.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$w.json')); print('$w', d['ms_per_step'], d['value'], d['roofline'].get('kernel','')[:30], d['roofline'].get('frac'), {k: round(v,3) for k,v in d['stage_ms'].items() if v > 0.01}, d.get('parity',{}).get('bit_exact'))"
done

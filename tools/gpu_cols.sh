#!/bin/bash
# SF1 step per column subset (bench --columns): what each column costs alone at 4 streams.
#   tools/gpu_cols.sh TAG "0 1 5 15 0,1,5 ..." [bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-cols}"; shift
SETS=$1; shift
mkdir -p "$OUT"
for c in $SETS; do
  f="$OUT/c_${c//,/_}.json"
  timeout -k 10 200 python -u bench.py --columns $c --steps 50 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write --no-parity "$@" > "$f" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
  python -c "import json; d=json.load(open('$f')); print('$c', d['ms_per_step'], d['value'], {k: round(v,3) for k,v in d['stage_ms'].items() if v > 0.02})"
done

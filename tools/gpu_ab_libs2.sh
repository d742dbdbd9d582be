#!/bin/bash
# Interleaved SF1 bench A/B over library builds (no tests; parity checked by every bench run).
#   tools/gpu_ab_libs2.sh TAG REPS LIB1 LIB2 ... [-- bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-ablibs}"; REPS=${2:-2}; shift 2
LIBS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done; [ "$1" == "--" ] && shift
mkdir -p "$OUT"
for rep in $(seq 1 $REPS); do
  for L in "${LIBS[@]}"; do
    tag=$(basename $L .so)
    PFLOOR_LIB_PATH=$ROOT/$L timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write "$@" > "$OUT/bench_${tag}_$rep.json" 2>> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_${tag}_$rep.json')); print('$tag', d['ms_per_step'], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
  done
done

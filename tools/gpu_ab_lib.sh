#!/bin/bash
# Quick GPU tests of the current build, then interleaved SF1 bench A/B against a saved library.
#   tools/gpu_ab_lib.sh TAG OTHER_LIB [REPS] [bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-ablib}"; OTHER=$2; REPS=${3:-2}; shift 3
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { tail -60 "$OUT/pytest.log"; exit 1; }
for rep in $(seq 1 $REPS); do
  for L in "$OTHER" ""; do
    tag=cur; [ -n "$L" ] && tag=other
    PFLOOR_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write "$@" > "$OUT/bench_${tag}_$rep.json" 2>> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_${tag}_$rep.json')); print('$tag', d['ms_per_step'], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
  done
done

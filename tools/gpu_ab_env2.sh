#!/bin/bash
# Full GPU tests, then interleaved A/B of environment settings (bench parity checked every run).
#   tools/gpu_ab_env2.sh TAG REPS "ENV1" "ENV2" ... [-- bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-abenv}"; REPS=${2:-2}; shift 2
ENVS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do ENVS+=("$1"); shift; done; [ "$1" == "--" ] && shift
mkdir -p "$OUT"
if [ -z "$NO_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { tail -60 "$OUT/pytest.log"; exit 1; }
fi
for rep in $(seq 1 $REPS); do
  i=0
  for E in "${ENVS[@]}"; do
    i=$((i+1))
    env $E timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write "$@" > "$OUT/bench_e${i}_$rep.json" 2>> "$OUT/bench.err" || { echo "FAIL $E"; tail -30 "$OUT/bench.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_e${i}_$rep.json')); print('[$E]', d['ms_per_step'], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
  done
done

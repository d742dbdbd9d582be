#!/bin/bash
# All GPU tests, then N short SF1 bench runs (parity on).  tools/gpu_quick2.sh TAG [N] [bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-q2}"; shift
N=${1:-2}; shift
mkdir -p "$OUT"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { tail -50 "$OUT/pytest.log"; exit 1; }
for i in $(seq 1 $N); do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write "$@" > "$OUT/bench_$i.json" 2>> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$i.json')); print(d['ms_per_step'], d['value'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
done

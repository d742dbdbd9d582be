#!/bin/bash
# GPU tests, then interleaved A/B of pipelined (default) vs --no-pipeline SF1 steps.
#   tools/gpu_ab_pipe.sh TAG [skip-tests]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-abpipe}"
mkdir -p "$OUT"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { tail -60 "$OUT/pytest.log"; exit 1; }
fi
for i in 1 2; do
  for v in pipe nopipe; do
    extra=""; [ $v == nopipe ] && extra="--no-pipeline"
    timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e $extra > "$OUT/bench_${v}_$i.json" 2>> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$i.json')); print('$v', d['ms_per_step'], d['value'], d['host_enqueue_ms_per_batch'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
  done
done

#!/bin/bash
# Quick GPU check: Snappy + parity tests, then N bench runs (SF1, parity on).  tools/gpu_quick.sh TAG [N] [bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-quick}"; shift
N=${1:-2}; shift
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_delta_bytes.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { tail -50 "$OUT/pytest.log"; exit 1; }
for i in $(seq 1 $N); do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-pmc --no-e2e "$@" > "$OUT/bench_$i.json" 2>> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$i.json')); print(d['ms_per_step'], d.get('host_enqueue_ms_per_batch'), d['roofline']['kernel'], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
done

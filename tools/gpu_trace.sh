#!/bin/bash
# Quick GPU check + per-kernel launch times: Snappy/parity tests, one bench run (parity on), then a
# rocprofv3 kernel trace of a short bench whose isolated roofline passes give context-0 launch times.
#   tools/gpu_trace.sh TAG [bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-trace}"; shift
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { tail -50 "$OUT/pytest.log"; exit 1; }
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-pmc --no-e2e "$@" > "$OUT/bench.json" 2>> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-e2e --no-parity "$@" > "$OUT/prof.log" 2>&1 || { tail -30 "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
python3 "$ROOT/tools/trace_launches.py" "$f" 3 | head -24

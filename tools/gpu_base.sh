#!/bin/bash
# Round baseline: full GPU tests, a bench line, a rocprofv3 kernel trace of a short bench (per-stream timeline).
#   tools/gpu_base.sh TAG [skip-tests] [bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-base}"; shift
SKIP=""; if [ "$1" == "skip-tests" ]; then SKIP=1; shift; fi
mkdir -p "$OUT"
if [ -z "$SKIP" ]; then
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { tail -60 "$OUT/pytest.log"; exit 1; }
fi
timeout -k 10 400 python -u bench.py --steps 100 --warmup 5 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-e2e --no-parity --no-write "$@" > "$OUT/prof.log" 2>&1 || { tail -30 "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
python3 "$ROOT/tools/trace_timeline.py" "$f" > "$OUT/timeline.txt" 2>&1
python3 "$ROOT/tools/trace_launches.py" "$f" 3 > "$OUT/launches.txt" 2>&1
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
exit 0

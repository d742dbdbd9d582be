#!/bin/bash
# One GPU session on the gpurun box: parity tests, bench line, rocprofv3 kernel summary.
# Every GPU step has its own time limit; the script stops at the first failing step.
#   tools/gpu_round.sh TAG [skip-tests] [bench args...]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
TAG=${1:-run}
shift
SKIP=""
if [ "$1" == "skip-tests" ]; then SKIP=1; shift; fi
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
if [ -z "$SKIP" ]; then
    timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
        > "$OUT/pytest.log" 2>&1
    rc=$?
    tail -5 "$OUT/pytest.log"
    [ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; tail -60 "$OUT/pytest.log"; exit 1; }
fi
timeout -k 10 600 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
cat "$OUT/bench.json"
[ $rc -eq 0 ] || { echo "bench failed rc=$rc"; tail -40 "$OUT/bench.err"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-e2e --no-parity --no-write > "$OUT/prof.log" 2>&1
rc=$?
[ $rc -eq 0 ] || { echo "rocprof failed rc=$rc"; tail -40 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cat {} \;
exit 0

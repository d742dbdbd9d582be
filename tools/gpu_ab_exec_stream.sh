#!/bin/bash
# A/B of PF_EXEC_STREAM (executor on its own low-priority stream): GPU tests with it on, then
# bench lines off/on/off/on. Every GPU step has its own time limit; stops at the first failure.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/abx"
mkdir -p "$OUT"
PF_EXEC_STREAM=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_on.log" 2>&1 || { tail -30 "$OUT/pytest_on.log"; exit 1; }
tail -2 "$OUT/pytest_on.log"
for v in 0 1 0 1; do
    PF_EXEC_STREAM=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline \
        > "$OUT/bench_x$v.json" 2> "$OUT/bench_x$v.err" || { tail -20 "$OUT/bench_x$v.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], d['stage_ms'])" \
        "$OUT/bench_x$v.json" "x$v" | tee -a "$OUT/summary.txt"
done

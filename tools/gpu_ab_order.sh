#!/bin/bash
# A/B of PF_PIECE_ORDER (executor pieces dispatched most-compressed-bytes first): GPU tests with it
# on, then bench lines off/on interleaved. Every GPU step has its own time limit.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/abo"
mkdir -p "$OUT"
PF_PIECE_ORDER=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_on.log" 2>&1 || { tail -30 "$OUT/pytest_on.log"; exit 1; }
tail -2 "$OUT/pytest_on.log"
for r in 1 2 3; do
  for v in 0 1; do
    PF_PIECE_ORDER=$v timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline \
        > "$OUT/bench_o${v}_r$r.json" 2> "$OUT/bench_o${v}_r$r.err" || { tail -20 "$OUT/bench_o${v}_r$r.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], d['stage_ms']['snappy_exec'], d['roofline']['launch_ms'])" \
        "$OUT/bench_o${v}_r$r.json" "order=$v run=$r" | tee -a "$OUT/summary.txt"
  done
done

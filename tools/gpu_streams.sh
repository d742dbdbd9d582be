#!/bin/bash
# Decode contexts (streams) per GPU: bench lines for 2 / 3 / 4 contexts, twice each, interleaved.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/streams"
mkdir -p "$OUT"
for r in ${RUNS:-1 2}; do
  for s in ${STREAMS:-2 3 4}; do
    timeout -k 10 240 python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --streams $s \
        > "$OUT/bench_s${s}_r$r.json" 2> "$OUT/bench_s${s}_r$r.err" || { tail -20 "$OUT/bench_s${s}_r$r.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'])" \
        "$OUT/bench_s${s}_r$r.json" "streams=$s run=$r" | tee -a "$OUT/summary.txt"
  done
done

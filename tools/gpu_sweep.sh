#!/bin/bash
# Bench sweep over decode contexts per GPU: tools/gpu_sweep.sh TAG "1 2 3 4"
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/$1"
mkdir -p "$OUT"
for s in $2; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --streams $s --no-cpu-baseline \
        > "$OUT/bench_s$s.json" 2> "$OUT/bench_s$s.err" || { echo "bench s=$s failed"; tail -20 "$OUT/bench_s$s.err"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('streams',sys.argv[2],d['ms_per_step'],d['value'])" "$OUT/bench_s$s.json" $s
done

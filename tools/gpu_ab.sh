#!/bin/bash
# A/B of library variants (tools/var/lib_*.so): bench at 2 streams + per-column probe each.
#   tools/gpu_ab.sh TAG "head x10d3 ..."
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/$1"
mkdir -p "$OUT"
for v in $2; do
    export PFLOOR_LIB_PATH="$ROOT/tools/var/lib_$v.so"
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" \
        || { echo "bench $v failed"; tail -20 "$OUT/bench_$v.err"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['ms_per_step'],d['stage_ms'])" "$OUT/bench_$v.json" $v
    if [ -n "$3" ]; then
        timeout -k 10 300 python -u tools/probe_columns.py 3 > "$OUT/cols_$v.log" 2>&1 || { echo "probe $v failed"; tail "$OUT/cols_$v.log"; exit 1; }
    fi
done

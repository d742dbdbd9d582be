#!/bin/bash
# Round-6 baseline session: GPU suite, SF1 bench line, SQ counters of the executor (one stream).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-r6a}"; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-e2e --no-write > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['roofline'], d.get('stage_ms'))"
KREGEX='k_snappy_exec' timeout -k 10 300 tools/gpu_pmc_sq.sh ${1:-r6a}/sq || exit 1
f=$(find "$OUT/sq" -name '*counter_collection.csv' | head -1) && python3 tools/sq_summary.py $f > "$OUT/sq_summary.txt" && cat "$OUT/sq_summary.txt"

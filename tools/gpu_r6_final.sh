#!/bin/bash
# Round-6 final measurements of this tree: part A = GPU suite, smoke, the default SF1 bench
# line (CPU baselines, PMC traffic, E2E, write), the per-config lines; part B = SF1 kernel trace and
# per-launch times, parse-pass phase stamps (needs `make -C parquet-floor_amd stamps` first), SQ counters of every kernel.
#   tools/gpu_r6_final.sh TAG A|B
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
TAG=${1:-r6f}; PART=${2:-A}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
if [ "$PART" == A ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  tail -2 "$OUT/smoke.log"
  timeout -k 10 600 python -u bench.py --steps 300 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('sf1', d['ms_per_step'], d['value'], d['roofline']['frac'], d.get('e2e', {}).get('value'), d['parity'])"
  for w in flat nested wide; do
    timeout -k 10 300 python -u bench.py --workload $w --steps 100 --warmup 5 --no-cpu-baseline --no-e2e --no-write > "$OUT/bench_$w.json" 2>> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_$w.json')); print('$w', d['ms_per_step'], d['value'], d['roofline']['frac'])"
  done
  timeout -k 10 600 python -u bench.py --workload sf100 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-write > "$OUT/bench_sf100.json" 2>> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_sf100.json')); print('sf100', d['ms_per_step'], d['value'], d['roofline']['frac'])"
else
  tools/gpu_prof.sh $TAG || exit 1
  f=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1) && python3 tools/trace_launches.py "$f" > "$OUT/launches.txt" || exit 1
  PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_stamps.so timeout -k 10 200 python3 tools/probe_parse_sf1.py > "$OUT/parse.txt" 2>&1 || { tail -20 "$OUT/parse.txt"; exit 1; }
  PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_stamps.so timeout -k 10 300 python3 tools/probe_exec5.py > "$OUT/stamps_exec.txt" 2>&1 || { tail -20 "$OUT/stamps_exec.txt"; exit 1; }
  KREGEX=k_ timeout -k 10 300 tools/gpu_pmc_sq.sh $TAG/sq || exit 1
  f=$(find "$OUT/sq/sq" -name '*counter_collection.csv' | head -1) && python3 tools/sq_summary.py "$f" > "$OUT/sq_summary.txt" || exit 1
  rm -rf "$OUT/prof" "$OUT/sq/sq" "$ROOT"/gpurun_out/probe_lineitem_*.parquet
  head -12 "$OUT/launches.txt"; cat "$OUT/parse.txt" | head -2
fi
exit 0

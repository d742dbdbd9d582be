#!/bin/bash
# Bench lines of configs 3 (sf100) and 4 (wide) at HEAD.  tools/gpu_configs.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-cfg}"
mkdir -p "$OUT"
timeout -k 10 500 python -u bench.py --workload wide --steps 20 --warmup 3 --no-cpu-baseline --no-write > "$OUT/bench_wide.json" 2> "$OUT/wide.err" || { tail -20 "$OUT/wide.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_wide.json')); print('wide', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'], d['parity']['bit_exact'])"
timeout -k 10 600 python -u bench.py --workload sf100 --steps 5 --warmup 1 --no-cpu-baseline --no-write --no-pmc > "$OUT/bench_sf100.json" 2> "$OUT/sf100.err" || { tail -20 "$OUT/sf100.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_sf100.json')); print('sf100', d['ms_per_step'], d['value'], d['roofline']['frac'], d['parity']['bit_exact'])"

#!/bin/bash
# Bench line with the write leg, then a rocprofv3 kernel summary of a short bench (write kernels included).
#   tools/gpu_write_prof.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-wprof}"
mkdir -p "$OUT"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pmc --no-e2e > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['parity']['bit_exact'], json.dumps(d.get('write')))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-e2e --no-parity > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
grep -E "k_enc|compress|Radix|radix|Scan|scan|Sort" "$OUT/prof/run_kernel_stats.csv" | cut -c1-220
exit 0

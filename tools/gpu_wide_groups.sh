#!/bin/bash
# Config 4: column batches per stream (--wide-groups 1 / 2 / 3), interleaved.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-wide_groups}"; mkdir -p "$OUT"
for i in 1 2; do
  for G in 1 2 3; do
    timeout -k 10 300 python -u bench.py --workload wide --wide-groups $G --steps 30 --warmup 3 --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/b_${G}_$i.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${G}_$i.json')); print('groups x$G', d['ms_per_step'], d['parity']['bit_exact'])"
  done
done

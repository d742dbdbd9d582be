#!/bin/bash
# E2E with the library's copy stream at the highest stream priority (diagnostics build, PF_DL_PRIO=1)
# against the product library, interleaved.   tools/gpu_e2e_prio.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-e2eprio}"; mkdir -p "$OUT"
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-pmc --no-write --no-parity"
for i in 1 2 3; do
  for g in base prio; do
    if [ "$g" == base ]; then
      timeout -k 10 300 python -u bench.py $ARGS > "$OUT/e_${g}_$i.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    else
      PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_diag.so PF_DL_PRIO=1 \
        timeout -k 10 300 python -u bench.py $ARGS > "$OUT/e_${g}_$i.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    fi
    python3 -c "import json; d=json.load(open('$OUT/e_${g}_$i.json')); e=d['e2e']; print('$g', e['value'], e['ms_per_pass'], e['file']['value'], d['ms_per_step'])"
  done
done

#!/bin/bash
# E2E with the upload by a kernel of G workgroups (diagnostics build, PF_H2D_KERNEL=1 PF_H2D_GRID=G) against
# the product library's SDMA upload, interleaved: a slower upload beside the downloads.
#   tools/gpu_e2e_h2d.sh TAG G...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-e2eh2d}"; shift; mkdir -p "$OUT"
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-pmc --no-write --no-parity"
for i in 1 2; do
  for g in base "$@"; do
    if [ "$g" == base ]; then
      timeout -k 10 300 python -u bench.py $ARGS > "$OUT/e_${g}_$i.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    else
      PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_diag.so PF_H2D_KERNEL=1 PF_H2D_GRID=$g \
        timeout -k 10 300 python -u bench.py $ARGS > "$OUT/e_${g}_$i.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    fi
    python3 -c "import json; d=json.load(open('$OUT/e_${g}_$i.json'))['e2e']; print('$g', d['value'], d['ms_per_pass'], d['file']['value'], d['frac_of_measured_d2h'])"
  done
done

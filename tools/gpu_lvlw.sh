#!/bin/bash
# k_lvl block-table A/B: level parity tests on the product library, the stamps probe for the saved
# (diag/libpfloor_sthead.so) and current stamps builds, then interleaved config 4 / config 1 lines
# against diag/libpfloor_head.so.   tools/gpu_lvlw.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
TAG=${1:-lvlw}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_page_null.py tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_short_runs.py tests/test_gpu_runs.py -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$OUT/pytest.log" | head -20; exit 1; }
for v in sthead stamps; do
  PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_$v.so timeout -k 10 300 python -u tools/probe_wide.py 100000 125 > "$OUT/probe_$v.log" 2>&1 || { tail -20 "$OUT/probe_$v.log"; exit 1; }
  echo "$v"; tail -4 "$OUT/probe_$v.log"
done
for wl in wide flat; do
  NOTEST=1 STEPS=${STEPS:-60} BARGS="--workload $wl" tools/gpu_ab_libs.sh "$TAG/$wl" head || exit 1
done

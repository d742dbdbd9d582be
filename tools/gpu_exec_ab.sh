#!/bin/bash
# Executor change: Snappy / direct / parity / string GPU tests on the product library, exec5 phase stamps
# (this tree's stamps build vs diag/libpfloor_stamps_<PREF>.so), an interleaved SF1 A/B against the
# diag/libpfloor_<variant>.so builds, and SQ counters of k_snappy_exec5 (product vs the first variant).
#   PREF=tpl1 tools/gpu_exec_ab.sh TAG variant...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
TAG=${1:-exec_ab}; shift
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_direct.py tests/test_gpu_parity.py tests/test_gpu_strings.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
if [ -n "$PREF" ]; then timeout -k 10 400 tools/gpu_probe_x5.sh $TAG/probe $PREF || exit 1; fi
NOTEST=1 STEPS=${STEPS:-100} timeout -k 10 900 tools/gpu_ab_libs.sh $TAG/ab "$@" || exit 1
if [ -z "$NOSQ" ]; then
  KREGEX='k_snappy_exec5' timeout -k 10 300 tools/gpu_pmc_sq.sh $TAG/sq_new || exit 1
  PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_$1.so KREGEX='k_snappy_exec5' timeout -k 10 300 tools/gpu_pmc_sq.sh $TAG/sq_ref || exit 1
  for v in sq_new sq_ref; do
    f=$(find "$OUT/$v/sq" -name '*counter_collection.csv' | head -1) && python3 tools/sq_summary.py $f > "$OUT/$v.txt" && echo "== $v" && cat "$OUT/$v.txt"
  done
fi
exit 0

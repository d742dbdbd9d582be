#!/bin/bash
# k_flat_null block groups: nullable-page tests with a group size, then an interleaved wide-workload A/B (diag lib).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-ngroup}"; mkdir -p "$OUT"
export PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_diag.so
PF_NULL_GROUP=${TESTG:-4} timeout -k 10 400 python -u -m pytest tests/test_gpu_page_null.py tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_runs.py -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$OUT/pytest.log" | head -20; exit 1; }
NOTEST=1 tools/gpu_ab_env.sh "${1:-ngroup}/ab" ${ROUNDS:-2} "--workload wide --steps 30 --warmup 3" ${VARIANTS:-PF_NULL_GROUP=1 PF_NULL_GROUP=2 PF_NULL_GROUP=4 PF_NULL_GROUP=8}

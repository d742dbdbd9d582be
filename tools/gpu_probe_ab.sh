#!/bin/bash
# String-path check: string / parity GPU tests, the k_flat_all stamps probe (diag/libpfloor_stamps.so),
# then an interleaved SF1 A/B against the given variants (diag/libpfloor_<name>.so).
#   tools/gpu_probe_ab.sh TAG name...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
TAG=${1:-pab}; shift
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_strings.py tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$OUT/pytest.log" | head -20; exit 1; }
PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_stamps.so timeout -k 10 300 python -u tools/probe_flat_all.py > "$OUT/probe.log" 2>&1 || { tail -20 "$OUT/probe.log"; exit 1; }
grep -A2 -E "returnflag|shipinstruct|l_comment|ALL" "$OUT/probe.log"
[ $# -gt 0 ] || exit 0
NOTEST=1 STEPS=${STEPS:-60} tools/gpu_ab_libs.sh "$TAG/ab" "$@"

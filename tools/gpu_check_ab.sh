#!/bin/bash
# Full GPU suite, then an interleaved A/B of the given library variants (diag/libpfloor_<name>.so) against
# the product library on a workload:  BARGS="--workload wide" tools/gpu_check_ab.sh TAG name...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
TAG=${1:-chk}; shift
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$OUT/pytest.log" | head -20; exit 1; }
[ $# -gt 0 ] || exit 0
NOTEST=1 STEPS=${STEPS:-30} tools/gpu_ab_libs.sh "$TAG/ab" "$@"

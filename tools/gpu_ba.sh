#!/bin/bash
# BYTE_ARRAY walk: string tests, then the rare-long timing probe for the product library and HEAD's.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-ba}"; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_strings.py tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$OUT/pytest.log" | head -20; exit 1; }
timeout -k 10 300 python -u tools/probe_rare_long.py 1000000 20 2>&1 | tee "$OUT/probe_new.log" || exit 1
[ -f parquet-floor_amd/diag/libpfloor_head.so ] && PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_head.so timeout -k 10 300 python -u tools/probe_rare_long.py 1000000 20 2>&1 | tee "$OUT/probe_head.log"

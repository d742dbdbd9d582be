#!/bin/bash
# exec5 phase stamps (tools/probe_exec5.py) of the stamps builds of this tree and a reference tree.
#   tools/gpu_probe_x5.sh TAG [ref=r05]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-x5probe}"; mkdir -p "$OUT"; REF=${2:-r05}
PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_stamps.so timeout -k 10 300 python -u tools/probe_exec5.py > "$OUT/new.txt" 2>&1 || { tail -20 "$OUT/new.txt"; exit 1; }
PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_stamps_$REF.so timeout -k 10 300 python -u tools/probe_exec5.py > "$OUT/ref.txt" 2>&1 || { tail -20 "$OUT/ref.txt"; exit 1; }
echo "== new"; cat "$OUT/new.txt"; echo "== $REF"; cat "$OUT/ref.txt"

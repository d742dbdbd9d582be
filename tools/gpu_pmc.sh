#!/bin/bash
# HBM traffic of the dominant kernel (k_snappy_exec) on the gpurun box: one rocprofv3 --pmc pass
# per counter (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), bench at 1 stream so the
# dispatches are not overlapped. tools/pmc_summary.py turns the CSVs into per-launch bytes.
#   tools/gpu_pmc.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/${1:-pmc}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex 'k_snappy_exec|k_flat|k_snappy_index' \
        --output-format csv -d "$OUT/$C" -o run -- \
        python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-e2e --no-parity --streams 1 > "$OUT/$C.log" 2>&1 || exit 1
done
exit 0

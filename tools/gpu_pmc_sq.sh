#!/bin/bash
# Where k_snappy_exec's wave time goes: one rocprofv3 --pmc pass of SQ counters (wave cycles split
# into parked / issue-stalled / issuing, instruction mix), bench at 1 stream.
#   tools/gpu_pmc_sq.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/${1:-pmcsq}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
    --kernel-include-regex 'k_snappy_exec|k_flat|k_snappy_index|k_snappy_chain' \
    --output-format csv -d "$OUT/sq" -o run -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-e2e --no-parity --streams 1 > "$OUT/sq.log" 2>&1 || exit 1
exit 0

#!/bin/bash
# Where a kernel's wave time goes: rocprofv3 --pmc passes of SQ counters (wave cycles split into
# parked / issue-stalled / issuing, instruction mix), TA/TCP busy and TCC traffic, bench at 1 stream.
#   tools/gpu_pmc_sq.sh TAG [bench args]      (KREGEX selects the kernels, default exec/flat/index/chain)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/${1:-pmcsq}"; shift
KRE="${KREGEX:-k_snappy_exec|k_flat|k_snappy_index|k_snappy_chain}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() {
    local name="$1"; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" --output-format csv -d "$OUT/$name" -o run -- \
        python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-e2e --no-parity --streams 1 $BENCH_ARGS \
        > "$OUT/$name.log" 2>&1
}
BENCH_ARGS="$*"
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU || exit 1
if [ -n "$PMC_MORE" ]; then
    pass sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH || exit 1
    pass ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum || exit 1
    pass tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum || exit 1
fi
exit 0

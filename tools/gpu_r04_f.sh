#!/bin/bash
# r04: SQ counters of every kernel (SF1, one stream) + k_flat phase stamps per column.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
OUT=$PWD/gpurun_out/${1:-r04_f}; mkdir -p $OUT
PFLOOR_LIB_PATH=$PWD/parquet-floor_amd/diag/libpfloor_stamps.so timeout -k 10 300 python -u tools/probe_flat_cols.py > $OUT/probe_flat.log 2>&1 || { tail -20 $OUT/probe_flat.log; exit 1; }
cat $OUT/probe_flat.log
KREGEX='k_' tools/gpu_pmc_sq.sh ${1:-r04_f}/pmc || exit 1
f=$(find $OUT/pmc/sq -name '*counter_collection.csv' | head -1)
python3 tools/sq_summary.py $f > $OUT/sq_summary.txt && cat $OUT/sq_summary.txt
rm -rf $OUT/pmc/sq

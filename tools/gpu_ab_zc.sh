#!/bin/bash
# A/B: H2D copies on the k_copy_words kernels (PF_ZC=1) vs SDMA copies (PF_ZC=0), per
# workload, interleaved; GPU tests first.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
OUT=$PWD/gpurun_out/${1:-ab_zc}; mkdir -p $OUT
PF_ZC=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -40 $OUT/pytest.log; exit 1; }
B="--no-cpu-baseline --no-pmc --no-e2e --no-write --steps 50 --warmup 5"
one() { local tag=$1 up=$2; shift 2
  PF_ZC=$up timeout -k 10 400 python -u bench.py $B "$@" > $OUT/b_$tag.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"; }
for wl in sf1 wide nested flat; do
  one ${wl}_off 0 --workload $wl && one ${wl}_on 1 --workload $wl && one ${wl}_off2 0 --workload $wl && one ${wl}_on2 1 --workload $wl || exit 1
done
PFLOOR_LIB_PATH=$PWD/parquet-floor_amd/diag/libpfloor_stamps.so timeout -k 10 300 python -u tools/probe_wide.py 100000 64 > $OUT/probe_wide.log 2>&1 || { tail -20 $OUT/probe_wide.log; exit 1; }
cat $OUT/probe_wide.log

#!/bin/bash
# r04 second GPU call: (1) the 20- vs 300-step gap with the round-3 bench (fresh threads per run,
# 5-pass warmup) against this round's (persistent threads, >= 0.3 s warmup); (2) executor phase
# stamps (stamps build); (3) the wide (config 4) host plan breakdown.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
OUT=$PWD/gpurun_out/${1:-r04_b}; mkdir -p $OUT
B="--no-cpu-baseline --no-pmc --no-e2e --no-write --no-parity"
run() { local f=$1; shift; timeout -k 10 200 python -u $f $B "$@" > $OUT/b.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
        python3 -c "import json,sys; d=json.load(open('$OUT/b.json')); print(sys.argv[1:], d['ms_per_step'])" $f "$@"; }
run bench_r03.py --steps 20 --warmup 5
run bench.py --steps 20 --warmup 5 --warmup-s 0
run bench_r03.py --steps 20 --warmup 5
run bench.py --steps 20 --warmup 5 --warmup-s 0
run bench_r03.py --steps 300 --warmup 5
run bench.py --steps 20 --warmup 5
PFLOOR_LIB_PATH=$PWD/parquet-floor_amd/diag/libpfloor_stamps.so timeout -k 10 200 python -u tools/probe_exec.py > $OUT/probe_exec.log 2>&1 || { tail -20 $OUT/probe_exec.log; exit 1; }
cat $OUT/probe_exec.log
PF_DEBUG_PLAN=1 timeout -k 10 300 python -u bench.py --workload wide $B --steps 10 --warmup 2 --warmup-s 0 > $OUT/wide.json 2> $OUT/wide_plan.log || { tail -20 $OUT/wide_plan.log; exit 1; }
grep "pf plan" $OUT/wide_plan.log | tail -8
python3 -c "import json; d=json.load(open('$OUT/wide.json')); print('wide', d['ms_per_step'], d['host_enqueue_ms_per_batch'], {k: round(v,3) for k,v in d['stage_ms'].items()})"

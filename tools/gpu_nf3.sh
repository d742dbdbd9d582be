#!/bin/bash
# the k_flat_null block race: staggered regression test with the racy library (expect a failure),
# the whole GPU suite with the fixed one, config 4 (k_page_null now opt-in)
cd $GRAFT_REPO_ROOT
PFLOOR_LIB_PATH=$GRAFT_REPO_ROOT/parquet-floor_amd/diag/libpfloor_bug.so timeout -k 10 300 python -u -m pytest tests/test_gpu_page_null.py -k "staggered" -q --timeout 280 --timeout-method thread > gpurun_out/nf3_old.log 2>&1; echo "racy lib: rc=$? $(tail -1 gpurun_out/nf3_old.log)"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/nf3_new.log 2>&1; rc=$?; echo "fixed lib: rc=$rc $(tail -1 gpurun_out/nf3_new.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/nf3_new.log; exit 1; }
run() { timeout -k 10 200 python -u bench.py --workload wide --steps 50 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write $2 > gpurun_out/nf3_$1.json 2> gpurun_out/nf3_$1.err; echo "[$1] rc=$? $(tail -1 gpurun_out/nf3_$1.err)"; python -c "import json; d=json.load(open('gpurun_out/nf3_$1.json')); print(d['ms_per_step'], {k: round(v,3) for k,v in d['stage_ms'].items() if v > 0.01})"; }
run def
PF_PAGE_NULL=1 run pn1
run def2

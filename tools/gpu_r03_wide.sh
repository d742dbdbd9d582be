#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
OUT=gpurun_out/r03_wide; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -60 $OUT/pytest.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write > $OUT/sf1.json 2> $OUT/sf1.err || { tail -20 $OUT/sf1.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/sf1.json')); print('sf1', d['ms_per_step'], d['host_enqueue_ms_per_batch'], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
PF_DEBUG_PLAN=1 timeout -k 10 300 python -u bench.py --workload wide --steps 30 --warmup 3 --no-cpu-baseline --no-pmc --no-e2e --no-write > $OUT/wide.json 2> $OUT/wide.err || { tail -20 $OUT/wide.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/wide.json')); print('wide', d['ms_per_step'], d['host_enqueue_ms_per_batch'], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
grep "pf plan" $OUT/wide.err | tail -4
tools/gpu_pool_sweep.sh r03_pool

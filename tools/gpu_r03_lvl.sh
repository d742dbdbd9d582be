#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
OUT=gpurun_out/r03_lvl; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -60 $OUT/pytest.log; exit 1; }
for w in wide sf1; do
timeout -k 10 300 python -u bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write > $OUT/$w.json 2> $OUT/$w.err || { tail -20 $OUT/$w.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/$w.json')); print('$w', d['ms_per_step'], d['host_enqueue_ms_per_batch'], d['roofline']['kernel'], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
done
tools/gpu_sq_wl.sh r03_sq_wide2 'k_lvl|k_flat_null|k_snappy_chain|k_runs' --workload wide

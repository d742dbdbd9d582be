#!/bin/bash
# Round-end measurement: GPU tests, the default bench line (PMC traffic, E2E, write leg, CPU
# baselines), rocprofv3 kernel trace + stats of a short bench, the other workloads' lines.
#   tools/gpu_final.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
TAG=${1:-final}; OUT=$PWD/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -60 $OUT/pytest.log; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('sf1', d['ms_per_step'], d['value'], d['roofline']['launch_ms'], d['roofline']['frac'], d['roofline']['traffic'], d['e2e']['value'], d['write']['value'], d['cpu_baseline']['value'], d['parity']['bit_exact'])"
for w in nested flat sf100; do
  timeout -k 10 500 python -u bench.py --workload $w --steps 30 --warmup 3 --no-cpu-baseline --no-write --no-e2e > $OUT/bench_$w.json 2>> $OUT/bench_w.err || { tail -20 $OUT/bench_w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$w.json')); r=d['roofline']; print('$w', d['ms_per_step'], d['value'], r['kernel'], r['launch_ms'], r['frac'], r['traffic'], d['parity']['bit_exact'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-e2e --no-parity --no-write > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
python3 $GRAFT_REPO_ROOT/tools/trace_launches.py "$f" 3 > $OUT/launches.txt; head -12 $OUT/launches.txt
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
[ -n "$SKIP_POOL" ] || (cd $GRAFT_REPO_ROOT && tools/gpu_pool_sweep.sh ${TAG}_pool)

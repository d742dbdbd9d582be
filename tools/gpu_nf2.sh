#!/bin/bash
# config 4 with k_page_null off (2 streams): failure rate, previous library vs head, mismatch details
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 200 python -u bench.py --workload wide --steps 5 --warmup 2 --no-cpu-baseline --no-pmc --no-e2e --no-write --streams 2 > gpurun_out/nf2_$1.json 2> gpurun_out/nf2_$1.err; echo "[$1] rc=$? $(tail -1 gpurun_out/nf2_$1.err)"; python -c "import json; d=json.load(open('gpurun_out/nf2_$1.json')); print(str(d.get('parity'))[:1500])" 2>/dev/null; }
for i in 1 2; do
PF_PAGE_NULL=0 run head$i
PFLOOR_LIB_PATH=$GRAFT_REPO_ROOT/parquet-floor_amd/diag/libpfloor_prev.so run prev$i
done

#!/bin/bash
# GPU parity tests, k_flat phase probe (stamps build), then 2 bench runs.  tools/gpu_flat_ab.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-flatab}"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_delta_bytes.py tests/test_gpu_scale.py tests/test_gpu_write.py -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { tail -50 "$OUT/pytest.log"; exit 1; }
PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_stamps.so timeout -k 10 200 python -u tools/probe_flat.py > "$OUT/probe.log" 2>&1 || { tail -20 "$OUT/probe.log"; exit 1; }
tail -1 "$OUT/probe.log"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/bench_$i.json" 2>> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$i.json')); print(d['ms_per_step'], d['value'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
done

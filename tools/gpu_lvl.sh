#!/bin/bash
# k_lvl check: parity tests over nullable pages, the stamps probe, then config 4 / 1 / 2 bench lines.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-lvl}"; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_page_null.py tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_short_runs.py tests/test_gpu_runs.py -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$OUT/pytest.log" | head -20; exit 1; }
if [ -f parquet-floor_amd/diag/libpfloor_stamps.so ]; then
  PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_stamps.so timeout -k 10 300 python -u tools/probe_wide.py 100000 125 > "$OUT/probe.log" 2>&1 || { tail -20 "$OUT/probe.log"; exit 1; }
  tail -2 "$OUT/probe.log"
fi
for wl in wide flat sf1; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 30 --warmup 3 --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/b_$wl.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$wl.json')); print('$wl', d['ms_per_step'], {k: round(v,3) for k,v in d['stage_ms'].items() if v > 0.02}, d['parity']['bit_exact'])"
done

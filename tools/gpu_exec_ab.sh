#!/bin/bash
# Snappy / parity GPU tests, the executor stamps probe, then SF1 bench A/B of two libraries
# (current build vs a saved one).  tools/gpu_exec_ab.sh TAG [OTHER_LIB]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-xab}"; OTHER=$2
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_delta_bytes.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { tail -60 "$OUT/pytest.log"; exit 1; }
PFLOOR_LIB_PATH=parquet-floor_amd/diag/libpfloor_stamps.so timeout -k 10 200 python -u tools/probe_exec.py > "$OUT/probe_exec.log" 2>&1 && cat "$OUT/probe_exec.log"
for rep in 1 2; do
  for L in "" "$OTHER"; do
    [ -z "$L" ] && [ "$rep" = "x" ] && continue
    tag=${L:+other}; tag=${tag:-cur}
    PFLOOR_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-pmc --no-e2e --no-write > "$OUT/bench_${tag}_$rep.json" 2>> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_${tag}_$rep.json')); print('$tag', d['ms_per_step'], d['roofline']['launch_ms'], {k: round(v,3) for k,v in d['stage_ms'].items()}, d['parity']['bit_exact'])"
    [ -z "$OTHER" ] && break
  done
done

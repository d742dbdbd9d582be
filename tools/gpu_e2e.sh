#!/bin/bash
# E2E variants (bench.py's e2e leg): decode streams 2 / 4 (--e2e-streams), batches per row group
# (--e2e-split), and the diagnostics build with the download on the decode stream (PF_DL_STREAM=0) or by
# SDMA (PF_DL_KERNEL=0).   tools/gpu_e2e.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-e2e}"; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "batch_copy or multi_device" -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
B="--steps 5 --warmup 2 --no-cpu-baseline --no-pmc --no-write --no-parity"
DIAG=$ROOT/parquet-floor_amd/diag/libpfloor_diag.so
one() {   # name, extra bench args (env via ENV=...)
  local name=$1; shift
  env $ENVV timeout -k 10 300 python -u bench.py $B "$@" > "$OUT/$name.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; return 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json'))['e2e']; print('$name', d.get('value'), d.get('ms_per_pass'), d.get('frac_of_measured_d2h'), d.get('file'), d.get('error'))"
}
ENVV="" one s2 --e2e-streams 2 &&
ENVV="" one s4 --e2e-streams 4 &&
ENVV="" one s2_rg1 --e2e-streams 2 --e2e-rg-batch 1 &&
ENVV="PFLOOR_LIB_PATH=$DIAG PF_H2D_KERNEL=0" one s2_h2dsdma --e2e-streams 2 &&
ENVV="PFLOOR_LIB_PATH=$DIAG PF_DL_KERNEL=0 PF_DL_STREAM=0 PF_H2D_KERNEL=0" one s4_r05style --e2e-streams 4

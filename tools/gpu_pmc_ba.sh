#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per k_ba_* launch of an l_comment-only decode (tools/probe_ba_stream.py), one
# rocprofv3 --pmc pass per counter.  tools/gpu_pmc_ba.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/${1:-pmc_ba}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
python3 "$ROOT/tools/probe_ba_stream.py" 1 > "$OUT/prep.log" 2>&1 || { tail -20 "$OUT/prep.log"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'k_ba_|k_snappy_exec5|k_flat_all' --output-format csv -d "$OUT/$C" -o run -- \
      python3 "$ROOT/tools/probe_ba_stream.py" 3 > "$OUT/$C.log" 2>&1 || { tail -20 "$OUT/$C.log"; exit 1; }
done
head -2 "$OUT/FETCH_SIZE.log"
python3 "$ROOT/tools/pmc_kernel.py" "$OUT/FETCH_SIZE" "$OUT/WRITE_SIZE"

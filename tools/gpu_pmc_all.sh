#!/bin/bash
# FETCH_SIZE (x2, gfx950) and WRITE_SIZE of every kernel of a one-row-group SF1 decode, MB per decode.
#   tools/gpu_pmc_all.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/${1:-pmc_all}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
python3 "$ROOT/tools/probe_rg_decode.py" 1 > "$OUT/prep.log" 2>&1 || { tail -20 "$OUT/prep.log"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'k_' --output-format csv -d "$OUT/$C" -o run -- \
      python3 "$ROOT/tools/probe_rg_decode.py" 3 > "$OUT/$C.log" 2>&1 || { tail -20 "$OUT/$C.log"; exit 1; }
done
head -1 "$OUT/prep.log"
python3 - "$OUT" <<'PY'
import collections, csv, glob, os, sys
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(os.path.join(out, c, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("pf::", "").replace("void ", "")
            acc[k][c] += float(r["Counter_Value"]) * 1024.0 * (2.0 if c == "FETCH_SIZE" else 1.0) / 3.0   # 3 decodes
for k, v in sorted(acc.items(), key=lambda kv: -(kv[1]["FETCH_SIZE"] + kv[1]["WRITE_SIZE"])):
    print(f"{k:28s} fetch x2 {v['FETCH_SIZE'] / 1e6:9.2f} MB  write {v['WRITE_SIZE'] / 1e6:9.2f} MB per decode")
PY

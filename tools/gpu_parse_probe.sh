#!/bin/bash
# Parse-pass counters (stamps build) over row group 0 of a lineitem file, one page at a time.
#   tools/gpu_parse_probe.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out/${1:-pp}"
mkdir -p "$OUT"
PFLOOR_LIB_PATH=$ROOT/parquet-floor_amd/diag/libpfloor_stamps.so timeout -k 10 300 python -u tools/probe_parse.py > "$OUT/probe.log" 2>&1 || { tail -20 "$OUT/probe.log"; exit 1; }
python3 - "$OUT/probe.log" <<'PY'
import re, sys
for line in open(sys.argv[1]):
    d = {k: int(v) for k, v in re.findall(r'(\w+)=(\d+)', line)}
    w = d.get('idx_windows', 1)
    calls = w + d.get('ch_exact', 0)
    print(f"{line.split()[0]:16s} win {w:5d} idx_parse/w {d.get('idx_parse_cyc', 0) // w:7d} table/w {d.get('idx_table_cyc', 0) // w:6d} "
          + " ".join(f"{k[3:-4]}={d[k] // calls}" for k in d if k.startswith('wp_'))
          + f" rounds/w {d.get('idx_rounds', 0) / w:.2f} rewalks/w {d.get('idx_rewalks', 0) / w:.1f}"
          + f" ch_max {d.get('ch_max_cyc', 0)} ch_exact {d.get('ch_exact', 0)}")
PY

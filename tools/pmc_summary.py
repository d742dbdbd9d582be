"""Per-launch HBM traffic from tools/gpu_pmc.sh output (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one
pass each). FETCH_SIZE and WRITE_SIZE are in KB; on gfx950 FETCH_SIZE counts half the bytes of
wide coalesced reads (MI355X_MICROARCH.md, HBM section), so fetch is reported raw and doubled.
  python tools/pmc_summary.py gpurun_out/pmc1 > profiles/<round>/pmc_traffic.json"""
import collections
import csv
import json
import sys

d = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(list))
seen = collections.Counter()
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    with open(f"{d}/{c}/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("pf::", "").replace("void ", "")
            if name == "k_snappy_exec":   # launched twice per step: pieces, then the whole-page redo
                seen[c] += 1
                if seen[c] % 2 == 0:
                    name = "k_snappy_exec_redo"
            per[name][c].append(float(r["Counter_Value"]) * 1024.0)
out = {}
for k, v in per.items():
    f = sum(v["FETCH_SIZE"]) / max(len(v["FETCH_SIZE"]), 1)
    w = sum(v["WRITE_SIZE"]) / max(len(v["WRITE_SIZE"]), 1)
    out[k] = {"launches": len(v["FETCH_SIZE"]), "fetch_bytes_raw": round(f), "fetch_bytes_x2": round(2 * f),
              "write_bytes": round(w), "traffic_bytes": round(2 * f + w)}
print(json.dumps(out, indent=1))

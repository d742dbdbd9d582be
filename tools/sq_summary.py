"""Summarise a rocprofv3 --pmc SQ_* pass (tools/gpu_pmc_sq.sh): per kernel, waves per dispatch,
cycles per wave, parked / stalled / active split and instructions per wave."""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("pf::", "").replace("void ", "")
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k, c in sorted(acc.items()):
    w = max(c["SQ_WAVES"], 1)
    cyc = c["SQ_WAVE_CYCLES"]
    print(f"{k:22s} dispatches={len(disp[k])} waves/dispatch={w / len(disp[k]):.0f} cycles/wave={cyc / w:.0f} "
          f"parked={c['SQ_WAIT_ANY'] / max(cyc, 1):.2f} stall={c['SQ_WAIT_INST_ANY'] / max(cyc, 1):.2f} "
          f"active={c['SQ_ACTIVE_INST_ANY'] / max(cyc, 1):.2f} valu={c['SQ_INSTS_VALU'] / w:.0f} "
          f"lds={c['SQ_INSTS_LDS'] / w:.0f} salu={c['SQ_INSTS_SALU'] / w:.0f} "
          f"| per dispatch: valu={c['SQ_INSTS_VALU'] / len(disp[k]) / 1e6:.2f}M lds={c['SQ_INSTS_LDS'] / len(disp[k]) / 1e6:.2f}M "
          f"salu={c['SQ_INSTS_SALU'] / len(disp[k]) / 1e6:.2f}M")

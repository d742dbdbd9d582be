"""Per-kernel sums of every counter in rocprofv3 --pmc csv files (tools/gpu_pmc_sq.sh), per dispatch.
python tools/pmc_kernel.py DIR..."""
import collections
import csv
import glob
import os
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("pf::", "").replace("void ", "")
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add((f, r["Dispatch_Id"]))
for k, c in sorted(acc.items()):
    print(k)
    for n, v in sorted(c.items()):
        nd = max(len(disp[(k, n)]), 1)
        print(f"    {n:36s} per-dispatch {v / nd:16.1f}")

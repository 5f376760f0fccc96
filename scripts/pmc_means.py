"""Per-dispatch counter means of the GEMM kernels (or, with --kernel NAME, of kernels whose name holds NAME) in
rocprofv3 --pmc output dirs:  python scripts/pmc_means.py [--kernel NAME] gpurun_out/pmc_cold/*/"""
import csv
import glob
import os
import sys
from collections import defaultdict

args = sys.argv[1:]
only = None
if args and args[0] == "--kernel":
    only, args = args[1], args[2:]
for root in args:
    for cc in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        acc = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        with open(cc) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"]
                if (only is None and "gemm_sk_kernel" not in k and "Cijk" not in k) or (only and only not in k):
                    continue
                k = k.split("(")[0][:48]
                d = r.get("Dispatch_Id") or r.get("Correlation_Id")
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(d)
        for k, cs in acc.items():
            n = max(1, len(disp[k]))
            print(os.path.basename(os.path.normpath(root)), k, " ".join(f"{c}={v / n:.4g}" for c, v in sorted(cs.items())))

"""Print per-kernel averages of the PMC passes of tools/gpu_sq.sh: python tools/pmc_report.py <tag>"""
import collections
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
vals = collections.defaultdict(list)
for path in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", tag, "p*", "p_counter_collection.csv"))):
    for r in csv.DictReader(open(path)):
        if "conv2d_tp" not in r["Kernel_Name"]:
            continue
        vals[(r["Kernel_Name"][:70], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(vals.items()):
    print("%-70s %-26s %14.4g" % (k, c, sum(v) / len(v)))

"""Summarize rocprofv3 PMC csv files: per kernel, mean of each counter over dispatches."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else "jt_"
acc = defaultdict(list)
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(f"{k:28s} mean {sum(v) / len(v):16.1f}  n={len(v)}")

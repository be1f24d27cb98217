"""Mean per-launch values of SQ counters of one kernel from rocprofv3 --pmc passes (JSON on stdout).
usage: pmc_sq.py <dir> <kernel substring>   (every *counter_collection.csv under <dir>)
Per dispatch rocprofv3 writes one row per counter (summed over the dimensions); launches are averaged."""
import csv
import glob
import json
import sys
from collections import defaultdict

root, key = sys.argv[1], sys.argv[2]
per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> value
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"]:
            per[(f, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
out = defaultdict(list)
for d in per.values():
    for c, v in d.items():
        out[c].append(v)
print(json.dumps({"kernel": key, "launches": max((len(v) for v in out.values()), default=0),
                  "per_launch": {c: sum(v) / len(v) for c, v in sorted(out.items())}}, indent=1))

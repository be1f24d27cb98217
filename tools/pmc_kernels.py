"""Per-kernel calibrated FETCH_SIZE + WRITE_SIZE (bytes per launch) from tools/profile_round.sh's
munin_* / pc5_* passes, corrected with the calibration of tools/pmc_traffic.sh (traffic/cal_*)."""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

root = sys.argv[1]


def per_kernel(prefix, counter):
    acc = defaultdict(list)
    for f in glob.glob(f"{root}/{prefix}_{counter}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0]
                acc[name.replace("void ", "")].append(float(r["Counter_Value"]))
    return acc


def calib(counter):
    vals = []
    for f in glob.glob(f"{root}/traffic/cal_{counter}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "copy8" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return (512 << 20) / (sum(vals) / len(vals) * 1024.0) if vals else None


out = {}
for prefix in ("munin", "pc5"):
    res = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = calib(c)
        for k, v in per_kernel(prefix, c).items():
            d = res.setdefault(k, {"launches": len(v)})
            d[c + "_bytes_total"] = sum(v) * 1024.0 * (f or 1.0)
    out[prefix] = res
print(json.dumps(out, indent=1))

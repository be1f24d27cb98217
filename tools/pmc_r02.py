"""Summarize tools/profile_r02.sh: per kernel and per launch (JT) / per PC run (config 5) -- kernel
time (kernel trace), calibrated fabric bytes (FETCH_SIZE x calibration + WRITE_SIZE) and VALU
instructions -- as JSON on stdout.  Calibration: tools/micro/calib_rw's copy8 kernel moves
512 MiB each way with 8-B/lane accesses (MI355X_MICROARCH.md: FETCH_SIZE reads half the bytes of
wide streaming reads on gfx950)."""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

root = sys.argv[1]


def clean(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name).replace("void ", "")
    return name.split("(")[0]


def counters(prefix):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{root}/{prefix}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[clean(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


cal = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    v = counters(f"cal_{c}").get("copy8", {}).get(c)
    cal[c] = (512 << 20) / (sum(v) / len(v) * 1024.0) if v else 1.0


def kernel_times(prefix):
    out = {}
    for f in glob.glob(f"{root}/{prefix}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            out[clean(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                     "total_ns": float(r["TotalDurationNs"])}
    return out


res = {"calibration": cal, "note": "bytes = rocprofv3 kB x 1024 x calibration; FETCH+WRITE = L2<->fabric traffic"}
for prefix, per, div in (("alarm", "launch", None), ("munin", "launch", None), ("pc5", "run", 3)):
    ks = defaultdict(dict)
    for c in ("FETCH_SIZE", "WRITE_SIZE", "VALU"):
        for k, d in counters(f"{prefix}_{c}").items():
            for cn, vals in d.items():
                if div:  # per PC run: sum over the run's launches (3 runs profiled)
                    ks[k][cn] = sum(vals) / div
                    ks[k]["launches_per_run"] = len(vals) / div
                else:  # per launch: mean over launches
                    ks[k][cn] = sum(vals) / len(vals)
    for k, d in ks.items():
        if "FETCH_SIZE" in d:
            d["fetch_bytes"] = d["FETCH_SIZE"] * 1024 * cal["FETCH_SIZE"]
        if "WRITE_SIZE" in d:
            d["write_bytes"] = d["WRITE_SIZE"] * 1024 * cal["WRITE_SIZE"]
    res[prefix] = {"per": per, "kernels": ks}
tr = kernel_times("pc5_trace")
for k, t in tr.items():
    if k in res["pc5"]["kernels"]:
        res["pc5"]["kernels"][k]["time_ns_per_run"] = t["total_ns"] / 3
res["stats_bench"] = kernel_times("stats")
print(json.dumps(res, indent=1))

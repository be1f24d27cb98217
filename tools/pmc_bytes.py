"""Calibrated HBM bytes per launch of one kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.
usage: pmc_bytes.py <root> <prefix> <kernel substring> [units per launch]   (JSON on stdout)
<root>/<prefix>_<COUNTER> and <root>/cal_<COUNTER> hold the kernel's and the copy8 calibration's
counter_collection.csv (tools/micro/calib_rw: 512 MiB read and written with 8-B lanes)."""
import csv
import glob
import json
import sys

root, prefix, key = sys.argv[1], sys.argv[2], sys.argv[3]
units = float(sys.argv[4]) if len(sys.argv) > 4 else None


def mean(counter, pre, k):
    vals = []
    for f in glob.glob(f"{root}/{pre}_{counter}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if k in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


cal_bytes = 512 << 20
out = {"kernel": key, "units_per_launch": units,
       "unit_note": "rocprofv3 FETCH_SIZE / WRITE_SIZE (kB) in separate --pmc passes, corrected by the copy8 "
                    "calibration (tools/micro/calib_rw: 8 B/lane loads and stores, 512 MiB each way)"}
tot = 0.0
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    cal, _ = mean(c, "cal", "copy8")
    raw, n = mean(c, prefix, key)
    factor = cal_bytes / (cal * 1024.0) if cal else None
    b = raw * 1024.0 * factor if (raw is not None and factor) else None
    out[c] = {"raw_kB": raw, "launches": n, "calib_raw_kB": cal, "calib_factor": factor, "bytes_per_launch": b}
    tot = tot + b if (b is not None and tot is not None) else None
out["hbm_bytes_per_launch"] = tot
if tot is not None and units:
    out["bytes_per_unit"] = tot / units
print(json.dumps(out, indent=1))

"""Summarize tools/pmc_traffic.sh output: calibrated HBM bytes per JT launch (JSON on stdout)."""
import csv
import glob
import json
import sys

root = sys.argv[1]


def mean(counter, prefix, key):
    vals = []
    for f in glob.glob(f"{root}/{prefix}_{counter}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if key in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None


cal_bytes = 512 << 20
out = {"cases_per_launch": 100000, "unit_note": "rocprofv3 FETCH_SIZE/WRITE_SIZE are kB; corrected by the copy8 calibration "
                    "(8 B/lane loads+stores, 512 MiB each way)"}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    cal = mean(c, "cal", "copy8")
    jt = mean(c, "jt", "fbn_jt_gen")
    factor = cal_bytes / (cal * 1024.0) if cal else None
    out[c] = {"jt_raw_kB": jt, "calib_raw_kB": cal, "calib_factor": factor,
              "jt_bytes_per_launch": jt * 1024.0 * factor if (jt and factor) else None}
f, w = out["FETCH_SIZE"]["jt_bytes_per_launch"], out["WRITE_SIZE"]["jt_bytes_per_launch"]
out["hbm_bytes_per_launch"] = (f + w) if (f is not None and w is not None) else None
print(json.dumps(out, indent=1))

"""profiles/{jt_traffic,munin_traffic,jt_valu}.json (read by bench.py) from a tools/pmc_r02.py summary of
tools/profile_r02.sh: calibrated FETCH + WRITE bytes and SQ_INSTS_VALU per launch of the ALARM
specialized kernel (fbn_jt_gen, 100k cases) and the Munin-like streamed kernel (jt_virt_kernel, 125k
cases).  usage: python tools/profile_jsons.py <pmc.json> <source label>"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = json.load(open(sys.argv[1]))
label = sys.argv[2] if len(sys.argv) > 2 else sys.argv[1]
cal = src["calibration"]


def kern(prefix, key):
    ks = src[prefix]["kernels"]
    name = next(k for k in ks if k.startswith(key))
    return name, ks[name]


name, a = kern("alarm", "fbn_jt_gen")
jt = {"cases_per_launch": 100000,
      "unit_note": "rocprofv3 FETCH_SIZE/WRITE_SIZE are kB; corrected by the copy8 calibration "
                   "(8 B/lane loads+stores, 512 MiB each way)",
      "FETCH_SIZE": {"jt_raw_kB": a["FETCH_SIZE"], "calib_factor": cal["FETCH_SIZE"], "jt_bytes_per_launch": a["fetch_bytes"]},
      "WRITE_SIZE": {"jt_raw_kB": a["WRITE_SIZE"], "calib_factor": cal["WRITE_SIZE"], "jt_bytes_per_launch": a["write_bytes"]},
      "hbm_bytes_per_launch": a["fetch_bytes"] + a["write_bytes"], "source": label}
mname, m = kern("munin", "jt_virt_kernel")
mu = {"cases_per_launch": 125000, "kernel": f"{mname} (variant 4, Munin-like 1041 vars)", "source": label,
      "unit_note": "rocprofv3 FETCH_SIZE / WRITE_SIZE in separate --pmc passes, kB, corrected with the copy8 "
                   "calibration (FETCH x2 on gfx950, WRITE exact)",
      "FETCH_bytes_per_launch": m["fetch_bytes"], "WRITE_bytes_per_launch": m["write_bytes"],
      "hbm_bytes_per_launch": m["fetch_bytes"] + m["write_bytes"]}
va = {"source": f"{label} (SQ_INSTS_VALU per launch)",
      "peak_note": "MI355X fp64 vector peak 78.6 TFLOP/s = 256 CUs x 4 SIMDs x 16 lanes x 2.4 GHz FMA lane-ops: a "
                   "wave64 VALU instruction occupies its SIMD 4 cycles",
      "alarm": {"kernel": f"{name} (variant 3)", "cases_per_launch": 100000, "valu_insts_per_launch": a["SQ_INSTS_VALU"]},
      "munin": {"kernel": f"{mname} (variant 4)", "cases_per_launch": 125000, "valu_insts_per_launch": m["SQ_INSTS_VALU"]}}
for fn, obj in (("jt_traffic", jt), ("munin_traffic", mu), ("jt_valu", va)):
    json.dump(obj, open(os.path.join(REPO, "profiles", fn + ".json"), "w"), indent=1)
    print("wrote profiles/%s.json" % fn)

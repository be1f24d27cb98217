"""profiles/pc5_kernels.json from a tools/pmc_r02.py summary of tools/pc5_profile.sh: per CI kernel and
PC run (config 5), launches, time, VALU lane-ops (SQ_INSTS_VALU x 64) and calibrated L2<->fabric
bytes (FETCH + WRITE), with their rates against the int32 VALU and HBM peaks.
usage: python tools/pc5_kernels_json.py <pmc.json> [out.json]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VALU_PEAK = 256 * 4 * 32 * 2.4e9  # lane-ops/s: a wave64 int32 VALU op issues in 2 cycles per SIMD
HBM = 8e12

src = json.load(open(sys.argv[1]))
dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "profiles", "pc5_kernels.json")
ks, tot_t, tot_ops, tot_fab = {}, 0.0, 0.0, 0.0
for k, d in sorted(src["pc5"]["kernels"].items()):
    if "time_ns_per_run" not in d:
        continue
    t = d["time_ns_per_run"] * 1e-9
    ops = d.get("SQ_INSTS_VALU", 0.0) * 64
    fab = d.get("fetch_bytes", 0.0) + d.get("write_bytes", 0.0)
    ks[k] = {"launches_per_run": d.get("launches_per_run"), "time_ms_per_run": t * 1e3,
             "valu_lane_ops_per_run": ops, "valu_Tops": ops / t / 1e12 if t else None,
             "valu_frac": ops / t / VALU_PEAK if t else None, "fabric_bytes_per_run": fab,
             "fabric_GBs": fab / t / 1e9 if t else None, "fabric_frac": fab / t / HBM if t else None}
    if k not in ("ci_cols_check", "ci_bits_build", "ci_bits_rowcount"):
        tot_t += t
        tot_ops += ops
        tot_fab += fab
out = {"source": "tools/pc5_profile.sh + tools/pmc_r02.py + tools/pc5_kernels_json.py on one MI355X: rocprofv3 kernel "
                 "trace of tools/pc5_timing.py (3 PC-stable runs of config 5) and separate --pmc passes "
                 "(FETCH_SIZE, WRITE_SIZE, SQ_INSTS_VALU); bytes calibrated with tools/micro/calib_rw",
       "calibration": src.get("calibration"),
       "peaks": {"int32_valu_lane_ops_per_s": VALU_PEAK, "hbm_Bps": HBM,
                 "note_valu": "256 CUs x 4 SIMD32 x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md)"},
       "per_run": {"ci_kernel_time_ms": tot_t * 1e3, "valu_lane_ops": tot_ops, "fabric_bytes": tot_fab},
       "kernels": ks}
json.dump(out, open(dst, "w"), indent=1)
print("wrote", dst, "kernels", len(ks), "time/run %.3f ms" % (tot_t * 1e3))

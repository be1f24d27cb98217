"""Assemble the committed roofline inputs bench.py reads (profiles/r05/) from a
tools/profile_r05_final.sh output directory:
  jt_valu.json      fp64 / all VALU instructions per launch of the ALARM and Munin-like kernels
  jt_traffic.json   ALARM kernel's calibrated FETCH + WRITE bytes per launch
  munin_traffic.json, pmc_pc_small_traffic.json, pc5_kernels.json
usage: r05_roofline_json.py <profile dir> [profiles/r05]"""
import json
import os
import shutil
import sys

src = sys.argv[1]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "profiles", "r05")
os.makedirs(dst, exist_ok=True)
F64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")


def load(p):
    with open(os.path.join(src, p)) as f:
        return json.load(f)


def valu(sq, cases, kernel, note):
    pl = sq["per_launch"]
    return {"kernel": kernel, "cases_per_launch": cases, "valu_insts_per_launch": pl["SQ_INSTS_VALU"],
            "f64_insts_per_launch": sum(pl[c] for c in F64), "f64_by_kind": {c: pl[c] for c in F64},
            "salu_insts_per_launch": pl.get("SQ_INSTS_SALU"), "lds_insts_per_launch": pl.get("SQ_INSTS_LDS"),
            "source": note}


out = {"source": "tools/profile_r05_final.sh (rocprofv3 --pmc, one counter group per pass) + tools/r05_roofline_json.py",
       "peak_note": "MI355X fp64 vector peak = 256 CUs x 4 SIMDs x 16 lanes x 2.4 GHz lane-ops: a wave64 fp64 VALU "
                    "instruction occupies its SIMD 4 cycles",
       "alarm": valu(load("alarm/alarm_sq.json"), 100000, "fbn_jt_gen (variant 3, fast arithmetic order)",
                     "alarm/alarm_sq.json"),
       "munin": valu(load("tile_sq.json"), 125000, "jt_tile_kernel (variant 5)", "tile_sq.json")}
json.dump(out, open(os.path.join(dst, "jt_valu.json"), "w"), indent=1)
a = load("alarm/alarm_traffic.json")
json.dump({"cases_per_launch": 100000, "kernel": "fbn_jt_gen (variant 3, fast arithmetic order)", **a,
           "source": "tools/profile_r05.sh"}, open(os.path.join(dst, "jt_traffic.json"), "w"), indent=1)
t = load("tile_traffic.json")
json.dump({"cases_per_launch": 125000, **t, "source": "tools/profile_r05_final.sh (munin_once.py 125000 5)"},
          open(os.path.join(dst, "munin_traffic.json"), "w"), indent=1)
shutil.copy(os.path.join(src, "pc_small_traffic.json"), os.path.join(dst, "pmc_pc_small_traffic.json"))
shutil.copy(os.path.join(src, "pc5_kernels.json"), os.path.join(dst, "pc5_kernels.json"))
print("wrote", dst)

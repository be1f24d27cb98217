"""Assemble the committed roofline inputs bench.py reads (profiles/r06/) from a tools/profile_r06.sh
output directory:
  jt_valu.json      fp64 / all VALU instructions per launch: the ALARM kernel (variable-major build,
                    measured this round) and the Munin-like tiled kernel (unchanged: profiles/r05)
  jt_traffic.json   ALARM kernel's calibrated FETCH + WRITE bytes per launch (variable-major), with
                    the case-major build's beside it
  pmc_pc_small_traffic.json, pc5_kernels.json
usage: r06_roofline_json.py <profile dir> [profiles/r06]"""
import json
import os
import shutil
import sys

src = sys.argv[1]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "profiles", "r06")
os.makedirs(dst, exist_ok=True)
F64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")


def load(p):
    with open(os.path.join(src, p)) as f:
        return json.load(f)


sq = load("alarm_sq.json")["per_launch"]
r05 = json.load(open(os.path.join(REPO, "profiles", "r05", "jt_valu.json")))
out = {"source": "tools/profile_r06.sh (rocprofv3 --pmc, one counter group per pass) + tools/r06_roofline_json.py; "
                 "munin: profiles/r05/jt_valu.json (kernel unchanged in round 6)",
       "peak_note": r05["peak_note"],
       "alarm": {"kernel": "fbn_jt_gen (variant 3, fast arithmetic order, variable-major marginals)",
                 "cases_per_launch": 100000, "valu_insts_per_launch": sq["SQ_INSTS_VALU"],
                 "f64_insts_per_launch": sum(sq[c] for c in F64), "f64_by_kind": {c: sq[c] for c in F64},
                 "salu_insts_per_launch": sq.get("SQ_INSTS_SALU"), "lds_insts_per_launch": sq.get("SQ_INSTS_LDS"),
                 "source": "alarm_sq.json"},
       "munin": r05["munin"]}
json.dump(out, open(os.path.join(dst, "jt_valu.json"), "w"), indent=1)
a, cm = load("alarm_traffic.json"), load("alarm_cm_traffic.json")
json.dump({"cases_per_launch": 100000, "kernel": "fbn_jt_gen (variant 3, fast order, variable-major marginals)", **a,
           "case_major_build": {k: cm[k] for k in ("FETCH_SIZE", "WRITE_SIZE", "hbm_bytes_per_launch")},
           "source": "tools/profile_r06.sh"}, open(os.path.join(dst, "jt_traffic.json"), "w"), indent=1)
shutil.copy(os.path.join(src, "pc_small_traffic.json"), os.path.join(dst, "pmc_pc_small_traffic.json"))
shutil.copy(os.path.join(src, "pc5_kernels.json"), os.path.join(dst, "pc5_kernels.json"))
print("wrote", dst)

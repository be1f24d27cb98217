"""Write profiles/r06/munin_traffic.json and the "munin" entry of profiles/r06/jt_valu.json from a
tools/profile_r06_munin.sh output directory (the Munin-like tiled kernel re-measured after round 6's
branch-free factor loads).  usage: r06_munin_json.py <profile dir> [profiles/r06]"""
import json
import os
import sys

src = sys.argv[1]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "profiles", "r06")
os.makedirs(dst, exist_ok=True)
F64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")


def load(p):
    with open(os.path.join(src, p)) as f:
        return json.load(f)


t = load("tile_traffic.json")
json.dump({"cases_per_launch": 125000, **t, "source": "tools/profile_r06_munin.sh (munin_once.py 125000 5)"},
          open(os.path.join(dst, "munin_traffic.json"), "w"), indent=1)
pl = load("tile_sq.json")["per_launch"]
pl2 = load("tile_sq2.json")["per_launch"]
vj = os.path.join(dst, "jt_valu.json")
v = json.load(open(vj))
v["munin"] = {"kernel": "jt_tile_kernel (variant 5, branch-free factor loads)", "cases_per_launch": 125000,
              "valu_insts_per_launch": pl["SQ_INSTS_VALU"], "f64_insts_per_launch": sum(pl[c] for c in F64),
              "f64_by_kind": {c: pl[c] for c in F64}, "salu_insts_per_launch": pl.get("SQ_INSTS_SALU"),
              "lds_insts_per_launch": pl.get("SQ_INSTS_LDS"), "wait": pl2,
              "source": "tools/profile_r06_munin.sh: tile_sq.json, tile_sq2.json"}
v["source"] = v["source"].split("; munin:")[0] + "; munin: tools/profile_r06_munin.sh + tools/r06_munin_json.py"
json.dump(v, open(vj, "w"), indent=1)
print("wrote", dst)

"""List the loops of a gfx950 assembly file (backward branches) with instruction-class counts.
asm_loops.py file.s [min_len]"""
import re
import sys
from collections import Counter

lines = open(sys.argv[1]).read().split("\n")
minlen = int(sys.argv[2]) if len(sys.argv) > 2 else 20
labels = {}
for i, l in enumerate(lines):
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        labels[m.group(1)] = i
for i, l in enumerate(lines):
    m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\w+)|\s+s_branch\s+(\.LBB\w+)", l)
    if not m:
        continue
    tgt = m.group(1) or m.group(2)
    j = labels.get(tgt)
    if j is None or j >= i:
        continue
    body = [x.strip().split()[0] for x in lines[j + 1:i + 1] if x.strip() and not x.strip().startswith((".", ";"))
            and not x.strip().endswith(":")]
    if len(body) < minlen:
        continue
    c = Counter()
    for ins in body:
        if ins.startswith("v_") and ("readlane" in ins or "writelane" in ins):
            c["v_lane"] += 1
        elif ins.startswith("v_"):
            c["valu"] += 1
        elif ins.startswith("s_load") or ins.startswith("s_buffer_load"):
            c["smem"] += 1
        elif ins.startswith("s_waitcnt"):
            c["wait"] += 1
        elif ins.startswith("s_"):
            c["salu"] += 1
        elif ins.startswith("buffer_load") or ins.startswith("global_load"):
            c["vmem_rd"] += 1
        elif ins.startswith("buffer_store") or ins.startswith("global_store"):
            c["vmem_wr"] += 1
        elif ins.startswith("ds_"):
            c["lds"] += 1
        else:
            c[ins] += 1
    print(f"{tgt} lines {j}-{i} n={len(body)} {dict(c)}")

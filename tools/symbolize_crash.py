"""Symbolize the frames of a glog-style crash report ('@ 0x... (unknown)' lines, as rocprofv3's
signal handler prints them) against a /proc/<pid>/maps dump of the same process (tools/exit_probe.py):
library + offset, then llvm-symbolizer on that library.  Runs on the host (no GPU).
usage: python tools/symbolize_crash.py <crash.log> <exit_maps_pid.txt>"""
import re
import subprocess
import sys


def main(log, maps):
    regions = []
    for ln in open(maps):
        t = ln.split()
        if len(t) < 6 or not t[5].startswith("/"):
            continue
        a, b = (int(x, 16) for x in t[0].split("-"))
        regions.append((a, b, int(t[2], 16), t[5]))
    for ln in open(log):
        m = re.search(r"(?:@|PC:\s*@)\s+0x([0-9a-f]+)", ln)
        if not m:
            continue
        addr = int(m.group(1), 16)
        hit = [(a, b, off, path) for a, b, off, path in regions if a <= addr < b]
        if not hit:
            print("0x%x  ?" % addr)
            continue
        a, b, off, path = hit[0]
        base = min(r[0] - r[2] for r in regions if r[3] == path)  # load base of that object
        rel = addr - base
        sym = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-symbolizer", "--obj=" + path, "0x%x" % rel],
                             capture_output=True, text=True).stdout.split("\n")[0]
        print("0x%x  %s+0x%x  %s" % (addr, path, rel, sym))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

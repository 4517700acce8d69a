"""Summarise tools/rf_trace.py output: per tick, block 0's phase stamps (us) and the builder blocks' end."""
import re
import sys

grp = []
for l in open(sys.argv[1]):
    l = l.strip()
    if l.startswith("RFTRACE") or l.startswith("RFBUILD"):
        grp.append(l)
        continue
    if not l.startswith("TICK"):
        continue
    tr = [g for g in grp if g.startswith("RFTRACE")]
    grp_b = [g for g in grp if g.startswith("RFBUILD")]
    grp = []
    if not tr:
        continue
    m = re.search(r"ts=(\d+) (.*)", tr[0])
    base = int(m.group(1))
    st = [int(x) / 100 for x in m.group(2).split()]
    ends = [(int(dict(x.split("=") for x in g.split()[1:])["end"]) - base) / 100 for g in grp_b]
    head = re.search(r"fuse=(\d) total=(\d+).*grid=(\d+)", tr[0])
    print(f"{l:16s} fuse={head.group(1)} total={head.group(2):3s} grid={head.group(3):3s} block0 "
          + " ".join(f"{x:6.2f}" for x in st if x < 1e6)
          + (f"  builders end {max(ends):6.2f}" if ends else ""))

#!/usr/bin/env python3
"""Mean of the last K launch times of each library in an ab_*.sh log (frontend_probe lines), per round.
usage: scripts/ab_summary.py <log> [K=4]"""
import re
import sys

k = int(sys.argv[2]) if len(sys.argv) > 2 else 4
d = {}
name = None
for line in open(sys.argv[1]).read().split("\n"):
    if line.startswith("=="):
        name = line.split()[1]
    m = re.search(r"ms \[(.*)\]", line)
    if m and name:
        v = [float(x.strip("' ")) for x in m.group(1).split(",")]
        d.setdefault(name, []).append(sum(v[-k:]) / len(v[-k:]))
for n, v in d.items():
    print("%-28s %s" % (n, " ".join("%.3f" % x for x in v)))

#!/usr/bin/env python3
"""VALU and SALU instructions per basic block of a kernel's hot loop (hipcc -S listing), with the
branches between blocks: which blocks a tracked lane/wave executes and what each costs.

usage: scripts/loop_blocks2.py <file.s> <kernel-substring>
"""
import re
import sys

lines = open(sys.argv[1]).read().splitlines()
st = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % sys.argv[2], l))
en = next(i for i in range(st, len(lines)) if lines[i].strip().startswith("s_endpgm"))
body = [l.strip() for l in lines[st:en]]
hdr = next(i for i, l in enumerate(body) if 'Inner Loop Header' in l)
lab = body[hdr].split(':')[0]
end = max(i for i, l in enumerate(body)
          if re.search(r's_cbranch\w*\s+%s$' % re.escape(lab), l) or re.search(r's_branch\s+%s$' % re.escape(lab), l))
cur, v, s = lab, 0, 0
for l in body[hdr + 1:end + 1]:
    if re.match(r'^\.LBB\S+:', l):
        print("%-14s VALU %4d SALU %3d" % (cur, v, s))
        cur, v, s = l.split(':')[0], 0, 0
    elif l.startswith('v_'):
        v += 1
    elif l.startswith('s_'):
        s += 1
        if l.startswith('s_cbranch') or l.startswith('s_branch'):
            print("%-14s VALU %4d SALU %3d   -> %s" % (cur, v, s, l))
            cur, v, s = cur + "'", 0, 0
print("%-14s VALU %4d SALU %3d" % (cur, v, s))

#!/usr/bin/env python3
"""VALU instructions per basic block of a kernel's hot loop in a hipcc -S listing (which blocks a
tracked lane executes: the fallback bodies sit behind s_cbranch_execz).

usage: scripts/loop_blocks.py <file.s> <kernel-substring>
"""
import re,collections,sys
lines=open(sys.argv[1]).read().splitlines()
name=sys.argv[2]
st=next(i for i,l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:"%name,l))
en=next(i for i in range(st,len(lines)) if lines[i].strip().startswith("s_endpgm"))
body=lines[st:en]
hdr=next(i for i,l in enumerate(body) if 'Inner Loop Header' in l)
lab=body[hdr].split(':')[0]
end=max(i for i,l in enumerate(body) if re.search(r's_cbranch\w*\s+%s$'%re.escape(lab),l.strip()) or re.search(r's_branch\s+%s$'%re.escape(lab),l.strip()))
blk=lab; cnt=collections.Counter(); order=[lab]
for l in body[hdr+1:end+1]:
    s=l.strip()
    if re.match(r'^\.LBB\S+:',s):
        blk=s.split(':')[0]; order.append(blk)
    elif s.startswith('v_'):
        cnt[blk]+=1
    elif s.startswith('s_cbranch') or s.startswith('s_branch'):
        order.append('   '+s)
        # the fall-through after a conditional branch is a block of its own (it may be the rare side)
        blk = (blk.split('+')[0] + '+%d' % (len(order))); order.append(blk)
for o in order:
    print(o, cnt.get(o,'') if not o.startswith(' ') else '')

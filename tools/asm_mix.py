"""Instruction mix per basic block (blocks holding MFMAs) of one kernel in a
hipcc -S listing.  usage: asm_mix.py <file.s> <mangled-name substring>"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
i = s.index(sys.argv[2])
i = s.index(":\n", i)
j = s.index(".Lfunc_end", i)
blocks, cur, lab = [], [], "entry"
for line in s[i:j].split("\n"):
    t = line.strip()
    if re.match(r"^\.LBB\S+:", t):
        blocks.append((lab, cur))
        lab, cur = t, []
    elif t and not t.startswith(";") and not t.startswith("."):
        cur.append(t)
blocks.append((lab, cur))
print("total", sum(len(b) for _, b in blocks))
for lab, ins in blocks:
    c = Counter(x.split()[0] for x in ins)
    if c.get("v_mfma_i32_32x32x32_i8") or len(ins) > 150:
        print(lab[:60], len(ins), sorted(c.items(), key=lambda x: -x[1])[:20])

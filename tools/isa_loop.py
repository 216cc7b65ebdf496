#!/usr/bin/env python3
"""tools/isa_loop.py FILE.s KERNEL_SUBSTR — instruction mix of a kernel's
outermost loop in a hipcc -S device listing (diagnostic): finds the loop
header with the most lines up to its back-edge, counts instruction classes
and lists every s_waitcnt in it, plus the kernel's VGPR/SGPR/occupancy."""
import re
import sys
from collections import Counter

src, name = sys.argv[1], sys.argv[2]
L = open(src).read().split("\n")
st = next(i for i, l in enumerate(L) if l.startswith("_Z") and name in l and l.rstrip().endswith(name.split()[-1]) or (l.startswith("_Z") and name in l and ":" in l))
en = next(i for i in range(st + 1, len(L)) if L[i].startswith(".Lfunc_end"))
F = L[st:en]
best = None
for i, l in enumerate(F):
    m = re.match(r"^(\.LBB\d+_\d+):.*Loop Header: Depth=1", l)
    if m:
        lab = m.group(1)
        ends = [j for j in range(i, len(F)) if re.search(r"s_(cbranch_\w+|branch) " + re.escape(lab) + r"$", F[j])]
        if ends and (best is None or ends[-1] - i > best[1] - best[0]):
            best = (i, ends[-1])
a, b = best
c, v = Counter(), Counter()
waits = []
for l in F[a:b + 1]:
    t = l.strip().split()
    if not t or t[0].startswith((";", ".")):
        continue
    op = t[0]
    if op.startswith("s_waitcnt"):
        waits.append(l.strip()); cls = "waitcnt"
    elif op.startswith("v_"):
        cls = "VALU"; v[op] += 1
    elif op.startswith("s_"):
        cls = "SALU"
    elif op.startswith("ds_"):
        cls = "LDS"
    elif op.startswith(("global_load", "buffer_load")):
        cls = "VMEM_RD"
    elif op.startswith(("global_store", "global_atomic", "buffer_store")):
        cls = "VMEM_WR"
    elif op.startswith("flat_"):
        cls = "FLAT"
    else:
        cls = op
    c[cls] += 1
print("loop lines", a, b, dict(c))
print("top VALU", v.most_common(25))
print("waits", Counter(waits).most_common())
for l in L[en:en + 80]:
    if re.search(r"NumVgprs|NumSgprs|Occupancy|ScratchSize|SGPRBlocks|spill", l):
        print(l.strip())

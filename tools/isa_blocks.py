"""Basic blocks of one kernel in a --save-temps .s file: VALU / SALU /
memory instruction counts per block and its branches (loop bodies stand out).
usage: python tools/isa_blocks.py file.s mangled_prefix"""
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r"^(" + re.escape(sys.argv[2]) + r"\S*):", s, re.M)
i = m.start()
j = s.index(".Lfunc_end", i)
body = s[i:j]
blocks, cur = [], None
for l in body.split("\n"):
    m = re.match(r"^(\.LBB\S+):", l)
    if m:
        cur = [m.group(1), 0, 0, 0, []]
        blocks.append(cur)
        continue
    if cur is None:
        continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    op = t.split()[0]
    cur[4].append(t)
    if op.startswith("v_"):
        cur[1] += 1
    elif op.startswith("s_"):
        cur[2] += 1
    else:
        cur[3] += 1
for b in blocks:
    br = [o for o in b[4] if o.startswith("s_cbranch") or o.startswith("s_branch")]
    print(b[0], "valu", b[1], "salu", b[2], "mem", b[3], br[-2:])

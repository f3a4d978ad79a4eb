"""Instruction mix of one kernel in a hipcc -S listing, with its basic blocks:
   python tools/isa_mix.py FILE.s SYMBOL_SUBSTRING [blocks]"""
import collections
import sys

lines = open(sys.argv[1]).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.split(";")[0].strip().endswith(":") and sys.argv[2] in l and not l.startswith("."))
body = []
for l in lines[start + 1:]:
    if "s_endpgm" in l:
        break
    body.append(l)
ins = [l.strip().split()[0] for l in body if l.strip() and not l.strip().startswith((".", ";")) and not l.strip().endswith(":")]
c = collections.Counter(ins)
print(len(ins), "instructions")
for k, v in c.most_common(40):
    print(f"{v:5d} {k}")
if len(sys.argv) > 3:
    blk, n = None, 0
    for l in body:
        t = l.strip()
        t = t.split(";")[0].strip()
        if t.endswith(":") and not t.startswith("."):
            if blk:
                print(blk, n)
            blk, n = t, 0
        elif t and not t.startswith((".", ";")):
            n += 1
    print(blk, n)

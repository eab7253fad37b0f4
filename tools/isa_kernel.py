"""Print (part of) one kernel's gfx950 assembly from a hipcc -S output.
   python3 tools/isa_kernel.py <file.s> <mangled-name-substring> [from] [to] [--grep re]"""
import re
import sys

s = open(sys.argv[1]).read()
names = [m.group(1) for m in re.finditer(r"^(\S+):\s*(?:;.*)?$", s, re.M) if sys.argv[2] in m.group(1) and not m.group(1).startswith(".")]
name = names[0]
i = s.index(name + ":")
e = s.index(".Lfunc_end", i)
body = s[i:e].split("\n")
argv = sys.argv[3:]
if "--grep" in argv:
    k = argv.index("--grep")
    argv = argv[:k] + argv[k + 2:]
args = [a for a in argv if not a.startswith("--")]
lo = int(args[0]) if args else 0
hi = int(args[1]) if len(args) > 1 else len(body)
g = None
if "--grep" in sys.argv:
    g = re.compile(sys.argv[sys.argv.index("--grep") + 1])
print(name, len(body), "lines")
for n in range(lo, min(hi, len(body))):
    if g is None or g.search(body[n]):
        print(n, body[n].rstrip()[:110])

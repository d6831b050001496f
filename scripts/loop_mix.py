"""Instruction mix of a kernel's largest loop (hipcc -save-temps .s): the span between a label and the
furthest backward branch to it. usage: python scripts/loop_mix.py <file.s> <kernel substring> [steps]"""
import collections
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l.split(":")[0])
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", l)}
best = None
for i, l in enumerate(body):
    m = re.match(r"\s+s_(?:c)?branch\w* (\.LBB\d+_\d+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        if best is None or i - labels[m.group(1)] > best[1] - best[0]:
            best = (labels[m.group(1)], i)
c = collections.Counter()
for l in body[best[0]:best[1] + 1]:
    m = re.match(r"\s+([a-z_0-9]+)", l)
    if m:
        c[m.group(1)] += 1
cls = collections.Counter()
for k, v in c.items():
    cls["nop" if k == "s_nop" else "cbranch" if "cbranch" in k else "waitcnt" if k == "s_waitcnt" else
        k.split("_")[0]] += v
print(f"loop {best[1] - best[0]} lines; per step ({steps}):", {k: round(v / steps, 1) for k, v in sorted(cls.items())})

"""Every backward-branch loop of a kernel in hipcc -save-temps output, with its instruction-class mix.
usage: python scripts/loops_all.py <file.s> <kernel symbol substring> [min lines]"""
import collections, re, sys

path, sym = sys.argv[1], sys.argv[2]
minl = int(sys.argv[3]) if len(sys.argv) > 3 else 50
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l.split(":")[0])
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", l)}
for i, l in enumerate(body):
    m = re.match(r"\s+s_(?:c)?branch\w* (\.LBB\d+_\d+)", l)
    if not (m and m.group(1) in labels and labels[m.group(1)] < i):
        continue
    a = labels[m.group(1)]
    if i - a < minl:
        continue
    c = collections.Counter()
    for x in body[a:i + 1]:
        mm = re.match(r"\s+([a-z_0-9]+)", x)
        if mm and not x.strip().startswith(";") and not x.strip().startswith("."):
            k = mm.group(1)
            c["nop" if k == "s_nop" else "cbranch" if "cbranch" in k else "waitcnt" if k == "s_waitcnt" else
              k.split("_")[0]] += 1
    print(f"{m.group(1)} lines {a}-{i} ({i - a}):", dict(sorted(c.items())))

import re, sys, collections
path, sym, must = sys.argv[1], sys.argv[2], [int(x) for x in sys.argv[3].split(",")]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l.split(":")[0])
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", l)}
files = {}
for l in lines:
    m = re.match(r'\s+\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
    if m: files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
def locs(a, b):
    s = set()
    for l in body[a:b+1]:
        m = re.match(r"\s+\.loc\s+(\d+)\s+(\d+)", l)
        if m and files.get(m.group(1)) == "rio_snappy.hip": s.add(int(m.group(2)))
    return s
cands = []
for i, l in enumerate(body):
    m = re.match(r"\s+s_(?:c)?branch\w* (\.LBB\d+_\d+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        a = labels[m.group(1)]
        if all(x in locs(a, i) for x in must): cands.append((i - a, a, i))
cands.sort()
_, a, b = cands[0]
cur = None; kinds = collections.defaultdict(collections.Counter)
for l in body[a:b+1]:
    m = re.match(r"\s+\.loc\s+(\d+)\s+(\d+)", l)
    if m: cur = (files.get(m.group(1), m.group(1)), int(m.group(2))); continue
    m = re.match(r"\s+([a-z_0-9]+)", l)
    if m and not l.strip().startswith("."):
        k = m.group(1); c = "v" if k.startswith("v_") else "s" if k.startswith("s_") else k.split("_")[0]
        kinds[cur][c] += 1
tot = collections.Counter()
for k, v in kinds.items(): tot.update(v)
print("loop lines", b - a, "total", dict(tot))
byl = sorted(kinds.items(), key=lambda kv: (kv[0][0], kv[0][1]))
for k, v in byl: print(k, dict(v))

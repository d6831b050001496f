"""Instruction mix of a kernel's largest loop (the decode step loop), from hipcc -save-temps output.

usage: python scripts/loop_isa.py <file.s> <kernel-symbol-substring> [steps-per-iteration]
Prints the loop length and the count of VALU / SALU / DS / global instructions; with
steps-per-iteration (k_snappy_pipe unrolls 4 steps) also VALU per step.
"""
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    per = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l and l.rstrip().endswith(":") or
                 (l.startswith("_Z") and sym in l.split(":")[0]))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end + 1]
    labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", l)}
    best = None
    for i, l in enumerate(body):
        m = re.match(r"\s+s_cbranch_\w+ (\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            span = i - labels[m.group(1)]
            if not best or span > best[0]:
                best = (span, labels[m.group(1)], i)
    _, a, b = best
    cnt = {}
    for l in body[a:b + 1]:
        m = re.match(r"\s+([a-z_0-9]+)", l)
        if not m or l.strip().startswith(";") or l.strip().startswith("."):
            continue
        k = m.group(1)
        cls = k.split("_")[0] if k.split("_")[0] in ("ds", "global", "buffer", "flat") else k[:2]
        cnt[cls] = cnt.get(cls, 0) + 1
    print(f"loop lines {b - a}: {cnt}; VALU per step {cnt.get('v_', 0) / per:.1f}, "
          f"SALU per step {cnt.get('s_', 0) / per:.1f}")


if __name__ == "__main__":
    main()

"""Summarise rocprofv3 counter CSVs: per kernel (substring match), mean counter value per dispatch, and the mean
over the real launches (the smallest dispatch dropped when there are 3 or more: bench.py's decode runs one
capacity-probe dispatch of ~no work before its timed launches).
usage: python scripts/pmc_summary.py <dir> [kernel-substring ...]"""
import collections, csv, glob, sys

root = sys.argv[1]
pats = sys.argv[2:] or ["k_snappy_ring", "k_decode_copy", "k_walk", "k_place"]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"]
        for p in pats:
            if p in name:
                acc[p][row["Counter_Name"]].append(float(row["Counter_Value"]))
for p, ctrs in acc.items():
    print(p)
    print(f"  {'counter':32s} {'mean':>16s} {'real-launch mean':>18s}")
    for c, v in sorted(ctrs.items()):
        real = sorted(v)[1:] if len(v) >= 3 else v
        print(f"  {c:32s} {sum(v) / len(v):16.4g} {sum(real) / len(real):18.4g}  (n={len(v)})")

"""Summarise rocprofv3 counter CSVs: per kernel (substring match), mean counter value per dispatch.
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
    for c, v in sorted(ctrs.items()):
        print(f"  {c:32s} {sum(v) / len(v):16.4g}  (n={len(v)})")

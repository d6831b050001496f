"""Mean per-dispatch counter values of one kernel from rocprofv3 --pmc csv passes.
usage: python scripts/pmc_print.py <dir with pmc*/run_counter_collection.csv> <kernel substring>"""
import collections, csv, glob, os, sys
d, k = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if k in r["Kernel_Name"]:
            agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, v in agg.items():
        vals = list(v.values())
        print(f"{os.path.basename(os.path.dirname(f))} {c:24s} {sum(vals) / len(vals):14.4g}  ({len(vals)} dispatches)")

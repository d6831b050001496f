"""Per-launch kernel durations from a rocprofv3 --kernel-trace CSV, probe dispatches excluded.

rocprofv3 --stats averages every dispatch of a kernel. bench.py's first decode of each file is a
capacity probe (the kernels launch, find nothing to do and return in a few microseconds), so the
--stats average of a decode kernel sits below its real launch time. This script reports, per kernel,
every dispatch ("all") and the dispatches that did work ("timed": longer than 5 % of the kernel's
longest dispatch), so profiles/README.md can quote the per-launch figure of the timed launches.

usage: python scripts/kstats.py <kernel_trace.csv or a directory holding one> [out.json] [substring ...]
"""
import csv
import glob
import json
import os
import sys


def load(path):
    if os.path.isdir(path):
        hits = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        if not hits:
            raise SystemExit(f"no kernel_trace.csv under {path}")
        path = hits[0]
    per = {}
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"]
        ns = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        per.setdefault(name, []).append(ns)
    return path, per


def summary(durs):
    top = max(durs)
    timed = [d for d in durs if d > 0.05 * top]
    return {"calls": len(durs), "avg_ms_all": round(sum(durs) / len(durs) / 1e6, 5),
            "timed_calls": len(timed), "avg_ms_timed": round(sum(timed) / len(timed) / 1e6, 5),
            "min_ms_timed": round(min(timed) / 1e6, 5), "max_ms": round(top / 1e6, 5)}


def main():
    src, out = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None
    subs = sys.argv[3:] or ["rio::"]
    path, per = load(src)
    doc = {"trace": os.path.basename(path),
           "rule": "timed = dispatches longer than 5 % of the kernel's longest (drops the capacity-probe dispatch)",
           "kernels": {}}
    for name, durs in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        if any(s in name for s in subs):
            doc["kernels"][name.split("(")[0].replace("void ", "")] = summary(durs)
    text = json.dumps(doc, indent=1)
    if out:
        open(out, "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()

"""Summarise rocprofv3 counter_collection CSVs: per-dispatch averages of every counter, per kernel."""
import collections
import csv
import glob
import sys


def summarise(paths, prefix=("void as::", "as::")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            if not k.startswith(prefix):
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    out = {}
    for k, v in agg.items():
        out[k] = {c: x / max(len(disp[(k, c)]), 1) for c, x in v.items()}
    return out


if __name__ == "__main__":
    root = sys.argv[1]
    res = summarise(sorted(glob.glob(f"{root}/**/run_counter_collection.csv", recursive=True)))
    for k, v in res.items():
        print(k)
        for c, x in sorted(v.items()):
            print(f"    {c:34s} {x:18.1f}")

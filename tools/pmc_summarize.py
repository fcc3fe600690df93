"""Summarise rocprofv3 --pmc output directories: per kernel (name filter), the mean of every counter per dispatch.

    python tools/pmc_summarize.py <dir> [substring ...]
"""
import collections
import csv
import glob
import os
import sys


def main():
    root, subs = sys.argv[1], sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", "")
                if subs and not any(s in name for s in subs):
                    continue
                short = name[:90]
                acc[short][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[short].add(r.get("Dispatch_Id", ""))
    for k in sorted(acc):
        n = max(1, len(disp[k]))
        vals = "  ".join(f"{c}={v / n:.4g}" for c, v in sorted(acc[k].items()))
        print(f"{k}  [{n} dispatches]  {vals}")


if __name__ == "__main__":
    main()

"""Sum rocprofv3 counter_collection.csv values per (kernel, counter) and print per-dispatch
averages for kernels matching a substring.   python tools/pmc_summary.py DIR [substr ...]"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    pats = sys.argv[2:] or [""]
    tot = defaultdict(float)
    disp = defaultdict(set)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if not any(p in k for p in pats):
                continue
            short = k.split("(")[0][-70:]
            tot[(short, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[short].add(r["Dispatch_Id"])
    for (k, c), v in sorted(tot.items()):
        n = len(disp[k])
        print(f"{k:72s} {c:24s} per-dispatch {v / n:14.4g}  (n={n})")


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Per-kernel averages of the counters tools/pmc_passes.sh collected (engine kernels only)."""
import collections
import csv
import glob
import sys


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "anonymous namespace)::" not in k or "at::" in k:
                continue
            k = k.split("::")[1].split("(")[0]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    for d in sys.argv[1:]:
        main(d)

#!/usr/bin/env python
"""Print the engine kernels' per-call averages from a rocprofv3 --stats CSV directory."""
import csv
import sys

for d in sys.argv[1:]:
    tot = 0.0
    print(d)
    for r in csv.DictReader(open(f"{d}/run_kernel_stats.csv")):
        if "anonymous namespace)::" in r["Name"] and "at::" not in r["Name"]:
            us = float(r["AverageNs"]) / 1e3
            tot += us
            print(f"  {r['Name'].split('::')[1].split('(')[0]:45s} {r['Calls']:>5} {us:9.1f} us")
    print(f"  {'sum':45s} {'':5} {tot:9.1f} us")

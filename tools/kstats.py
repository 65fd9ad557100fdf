#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv as (name, calls, mean us, share)."""
import csv
import sys

for x in csv.DictReader(open(sys.argv[1])):
    print(f"{x['Name'][:80]:80s} {x['Calls']:>5s} {float(x['AverageNs']) / 1e3:9.1f} us {float(x['Percentage']):6.2f}%")

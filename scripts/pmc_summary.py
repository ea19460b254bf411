#!/usr/bin/env python3
"""mean per-launch counter values by kernel from rocprofv3 counter_collection.csv files
usage: python scripts/pmc_summary.py gpurun_out/pmclat/*/*counter_collection.csv"""
import collections
import csv
import sys

per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sys.argv[1:]:
    agg = collections.defaultdict(float)
    name = {}
    for r in csv.DictReader(open(f)):
        key = (r['Dispatch_Id'], r['Counter_Name'])
        agg[key] += float(r['Counter_Value'])
        name[r['Dispatch_Id']] = r['Kernel_Name'].split('(')[0].replace('void ntc::', '')
    for (d, c), v in agg.items():
        per[name[d]][c].append(v)
for k, cs in per.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"  {c:34s} {sum(v) / len(v):.4e}  (n={len(v)})")

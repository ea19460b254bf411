#!/usr/bin/env python3
"""Per-arm kernel durations and counters from scripts/ab_sq.sh output."""
import collections, csv, glob, os, sys
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
for i in range(1, 20):
    if not os.path.exists(f"{d}/arm{i}.json"):
        break
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in glob.glob(f"{d}/pmc{i}/*counter_collection.csv") + glob.glob(f"{d}/tcc{i}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"].split("(")[0].replace("ntc::", "")
            agg[kn][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if "pmc" in f:
                dur[kn].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    print(f"arm{i}: {open(f'{d}/arm{i}.json').read()[:0]}")
    for kn, cs in agg.items():
        row = {c: sum(v) / len(v) for c, v in cs.items()}
        hit = row.get("TCC_HIT_sum"), row.get("TCC_MISS_sum")
        hr = hit[0] / (hit[0] + hit[1]) if None not in hit and sum(hit) else None
        print(f"  {kn:10s} {sum(dur[kn])/max(1,len(dur[kn])):7.3f} ms  VALU {row.get('SQ_INSTS_VALU',0):.3g}  "
              f"RDREQ {row.get('TCC_EA0_RDREQ_sum',0):.3g}  L2hit {hr if hr is None else round(hr,3)}")

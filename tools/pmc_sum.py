"""Aggregate a rocprofv3 counter_collection.csv per kernel: python tools/pmc_sum.py <csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r.get("Kernel_Name", r.get("Kernel-Name", "?"))[:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, d in sorted(agg.items(), key=lambda kv: -max(kv[1].values())):
    n = max(c for (kk, _), c in cnt.items() if kk == k)
    print(k, f"(dispatches {n})")
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v:.4g}")

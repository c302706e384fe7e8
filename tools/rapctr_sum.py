"""Sum the per-dispatch counters of tools/gpurun_rapctr.sh by kernel family (RAP numeric
SpGEMM kernels per template, and the long-row SpMV): one table row per kernel, the L2 hit
rate, LDS bank-conflict share, and where the waves spend their cycles.
usage: python tools/rapctr_sum.py <dir>"""
import collections
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(os.path.join(d, "pass*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"])[:60]
        tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add((f, r.get("Dispatch_Id", "")))
keys = sorted(tot, key=lambda k: -tot[k].get("SQ_BUSY_CYCLES", 0))
print(f"{'kernel':60s} {'L2hit':>6s} {'LDSconf/LDSact':>14s} {'wait/wave':>9s} {'instwait/wave':>13s} {'LDS/VALU':>8s} {'VMEMrd':>10s}")
for k in keys:
    t = tot[k]
    h, m = t.get("TCC_HIT_sum", 0), t.get("TCC_MISS_sum", 0)
    hit = h / (h + m) if h + m else float("nan")
    lc = t.get("SQ_LDS_BANK_CONFLICT", 0) / t["SQ_LDS_IDX_ACTIVE"] if t.get("SQ_LDS_IDX_ACTIVE") else float("nan")
    wv = t.get("SQ_WAVE_CYCLES", 0)
    wa = t.get("SQ_WAIT_ANY", 0) / wv if wv else float("nan")
    wi = t.get("SQ_WAIT_INST_ANY", 0) / wv if wv else float("nan")
    lv = t.get("SQ_INSTS_LDS", 0) / t["SQ_INSTS_VALU"] if t.get("SQ_INSTS_VALU") else float("nan")
    print(f"{k:60s} {hit:6.3f} {lc:14.3f} {wa:9.3f} {wi:13.3f} {lv:8.3f} {t.get('SQ_INSTS_VMEM_RD', 0):10.3g}")
print()
print("raw sums per kernel:")
for k in keys:
    print(k, {c: f"{v:.4g}" for c, v in sorted(tot[k].items())})

"""Sum tools/gpurun_mvctr.sh's per-dispatch counters per kernel and print the ratios:
TA busy share (TA_TA_BUSY over 256 CUs x the kernel's cycles, GRBM_GUI_ACTIVE / 8 XCDs), TA address / data stalls on
the cache, L1 cache-line accesses and L2 requests per load wavefront, UTCL1 misses.
usage: python tools/mvctr_sum.py <dir>"""
import collections
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.path.join(d, "pass*", "**", "*counter_collection.csv"), recursive=True):
    p = re.search(r"pass(\d+)", f).group(1)
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"])[:64]
        c = r["Counter_Name"]
        if c == "GRBM_GUI_ACTIVE":
            c = f"GRBM_GUI_ACTIVE@{p}"
        tot[name][c] += float(r["Counter_Value"])
CU = 256
XCD = 8      # GRBM_GUI_ACTIVE comes summed over the 8 XCDs: per-dispatch cycles x 8


def q(t, a, b, s=1.0):
    return t.get(a, 0) / (s * t[b]) if t.get(b) else float("nan")


print(f"{'kernel':64s} {'TAbusy':>6s} {'TAaddrSt':>8s} {'TAdataSt':>8s} {'lines/wf':>8s} {'L2req/wf':>8s} "
      f"{'TLBmiss':>7s} {'pendSt':>7s}")
for k in sorted(tot, key=lambda k: -tot[k].get("GRBM_GUI_ACTIVE@1", 0)):
    t = tot[k]
    g1, g2 = t.get("GRBM_GUI_ACTIVE@1", 0) / XCD, t.get("GRBM_GUI_ACTIVE@2", 0) / XCD
    ta = t.get("TA_TA_BUSY_sum", 0) / (CU * g1) if g1 else float("nan")
    sa = t.get("TA_ADDR_STALLED_BY_TC_CYCLES_sum", 0) / (CU * g2) if g2 else float("nan")
    sd = t.get("TA_DATA_STALLED_BY_TC_CYCLES_sum", 0) / (CU * g2) if g2 else float("nan")
    lw = q(t, "TCP_TOTAL_CACHE_ACCESSES_sum", "TA_FLAT_READ_WAVEFRONTS_sum")
    rw = q(t, "TCP_TCC_READ_REQ_sum", "TA_FLAT_READ_WAVEFRONTS_sum")
    tm = q(t, "TCP_UTCL1_TRANSLATION_MISS_sum", "TCP_UTCL1_REQUEST_sum")
    ps = t.get("TCP_PENDING_STALL_CYCLES_sum", 0) / (CU * g1) if g1 else float("nan")
    print(f"{k:64s} {ta:6.3f} {sa:8.3f} {sd:8.3f} {lw:8.2f} {rw:8.2f} {tm:7.4f} {ps:7.3f}")
print()
print("raw sums per kernel:")
for k in tot:
    print(k, {c: f"{v:.4g}" for c, v in sorted(tot[k].items())})

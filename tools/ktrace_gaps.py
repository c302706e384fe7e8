#!/usr/bin/env python3
"""GPU busy vs idle along a rocprofv3 --kernel-trace CSV (one process, one stream):
the union of kernel intervals, the gaps between consecutive kernels (host work, syncs,
launch latency), and per window of the timeline the busy fraction and the kernel count.

usage: python tools/ktrace_gaps.py <kernel_trace.csv> [window_s]
"""
import collections
import csv
import re
import sys


def main():
    path = sys.argv[1]
    win = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    ev = []
    for r in csv.DictReader(open(path)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:48]))
    ev.sort()
    t0, t1 = ev[0][0], max(e[1] for e in ev)
    busy = 0
    gaps = []
    cur_s, cur_e = ev[0][0], ev[0][1]
    by_pair = collections.defaultdict(lambda: [0, 0])
    prev = ev[0][2]
    for s, e, name in ev[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, cur_e))
            if s - cur_e < 1e6:                          # start-up / teardown pauses apart
                bp = by_pair[(prev, name)]
                bp[0] += 1
                bp[1] += s - cur_e
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev = name
    busy += cur_e - cur_s
    span = t1 - t0
    print(f"kernels {len(ev)}  span {span / 1e9:.3f} s  busy {busy / 1e9:.3f} s ({busy / span:.1%})  "
          f"idle {(span - busy) / 1e9:.3f} s in {len(gaps)} gaps")
    for lo, hi in ((0, 5e3), (5e3, 2e4), (2e4, 1e5), (1e5, 1e6), (1e6, 1e12)):
        g = [x for x, _ in gaps if lo <= x < hi]
        print(f"  gaps {lo / 1e3:8.0f}-{hi / 1e3:<8.0f} us: {len(g):7d}  total {sum(g) / 1e9:.3f} s")
    print("gaps under 1 ms by (kernel before -> kernel after), largest total first:")
    for (a, b), (n, t) in sorted(by_pair.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"  {t / 1e6:9.1f} ms {n:7d}x  {a} -> {b}")
    nb = int(span / (win * 1e9)) + 1
    wb = [0] * nb
    wk = [0] * nb
    for s, e, _ in ev:
        b = int((s - t0) / (win * 1e9))
        wk[b] += 1
        wb[b] += e - s
    print(f"per {win:g} s window: kernels, kernel-time fraction")
    for b in range(nb):
        print(f"  {b * win:7.1f} s  {wk[b]:7d}  {min(1.0, wb[b] / (win * 1e9)):.2f}")


if __name__ == "__main__":
    main()

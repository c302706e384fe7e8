"""Per-shape A/B of whole-matrix SpMV times from two AMGD_MVLOG=1 logs (gzip), e.g. the
gather tables on / off (tools/gpurun_r06g.sh): summed ms per (rows, cols) shape of the
lane-kernel products with x, and the total.

  python tools/mvlog_ab.py gpurun_out/r06g/mv_t1.txt.gz gpurun_out/r06g/mv_t0.txt.gz
"""
import collections
import gzip
import re
import sys


def load(path):
    d = collections.defaultdict(list)
    tab = {}
    pending = None
    for line in gzip.open(path, "rt"):
        m = re.match(r"spmvtab rw (\d+) tr (\d+) tiles (\d+) direct (\d+)", line)
        if m:
            pending = tuple(int(v) for v in m.groups())
            continue
        m = re.match(r"spmv (\d+) x (\d+) nnz (\d+) (\S+) x(\d) ([\d.]+) ms", line)
        if not m:
            continue
        rn, cn, nnz, kind, hx, ms = m.groups()
        if kind == "lane" and hx == "1":
            d[(int(rn), int(cn))].append((int(nnz), float(ms)))
            if pending:
                tab[(int(rn), int(cn))] = pending
        pending = None
    return d, tab


def main():
    (a, ta), (b, _) = load(sys.argv[1]), load(sys.argv[2])
    t1 = t0 = 0.0
    print(f"{'rows':>8} {'cols':>8} {'n':>5} {'mean':>6} {'ms A':>8} {'ms B':>8}  A/B   table (rw, rows/tile, tiles, direct)")
    for key in sorted(set(a) | set(b), key=lambda k: -k[0]):
        x, y = a.get(key, []), b.get(key, [])
        s1, s0 = sum(v[1] for v in x), sum(v[1] for v in y)
        t1 += s1
        t0 += s0
        if s0 + s1 < 10:
            continue
        mean = (sum(v[0] for v in y) / len(y) / key[0]) if y else 0
        print(f"{key[0]:8d} {key[1]:8d} {len(x):5d} {mean:6.0f} {s1:8.1f} {s0:8.1f} {s1 / max(s0, 1e-9):5.2f}  "
              f"{ta.get(key, '')}")
    print(f"total ms: A {t1:.1f}  B {t0:.1f}")


if __name__ == "__main__":
    main()

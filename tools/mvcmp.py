"""Compare AMGD_MVLOG SpMV logs of several runs per matrix shape (rows, cols, nnz)."""
import collections
import sys


def load(fn):
    d = collections.defaultdict(lambda: [0, 0.0, ""])
    for l in open(fn):
        if not l.startswith("spmv "):
            continue
        t = l.split()
        key = (int(t[1]), int(t[3]), int(t[5]) // 1000000)
        d[key][0] += 1
        d[key][1] += float(t[8])
        d[key][2] = t[6]
    return d


runs = [(fn, load(fn)) for fn in sys.argv[1:]]
keys = sorted(set().union(*[r.keys() for _, r in runs]), key=lambda k: -max(r[k][1] for _, r in runs if k in r))
print("rows cols Mnnz meanrow | " + " | ".join(fn.split("/")[-1] for fn, _ in runs))
tot = [0.0] * len(runs)
for k in keys:
    cells = []
    for q, (_, r) in enumerate(runs):
        if k in r:
            cells.append(f"{r[k][2]:>6} {r[k][1] / r[k][0]:7.3f}ms x{r[k][0]}")
            tot[q] += r[k][1]
        else:
            cells.append("-")
    if max(r[k][1] for _, r in runs if k in r) > 50:
        print(k[0], k[1], k[2], f"{k[2] * 1e6 / max(k[0], 1):.0f}", "|", " | ".join(cells))
print("total ms", [round(t) for t in tot])

#!/usr/bin/env python3
"""Compare the interpolation-loop traces of the oracle and the GPU library
(tools/oracle_trace.py output): per level, per interpolation iteration, the
skeleton size, the count of coarse columns above gamma, the worst ratio, and the
constraint solve (rows, PCG iterations, final rho).  Prints a side-by-side table
up to the shorter trace and the first line that differs.

usage: python tools/trace_diff.py oracle.txt gpu.txt [out.txt]
"""
import re
import sys

PAT = [
    ("level", re.compile(r"Level (\d+), dim\(A\) = (\d+)")),
    ("skel", re.compile(r"^\s*(\d+) nzs, (\d+) cols > ([0-9.e+-]+), worst = ([0-9.e+-]+)")),
    ("cons", re.compile(r"constraint: (\d+) of (\d+) rows, pcg (\d+) its, rho ([0-9.e+-]+) stop ([0-9.e+-]+)"
                        r"(?:, sp_add off-row (\d+) past-end (\d+))?")),
]


def parse(path):
    ev = []
    for line in open(path):
        body = re.sub(r"^\[\s*[0-9.]+s\]\s?", "", line.rstrip("\n"))
        for kind, rx in PAT:
            m = rx.search(body)
            if m:
                g = m.groups()
                if kind == "cons":
                    key = ("cons",) + g[:5]            # off-row counts: oracle only
                    extra = g[5:]
                else:
                    key = (kind,) + g
                    extra = ()
                ev.append((key, extra, body.strip()))
                break
    return ev


def main():
    a, b = parse(sys.argv[1]), parse(sys.argv[2])
    if not any(e[0][0] == "cons" for e in a) or not any(e[0][0] == "cons" for e in b):
        # one trace predates the constraint lines: compare levels and skeleton lines only
        a = [e for e in a if e[0][0] != "cons"]
        b = [e for e in b if e[0][0] != "cons"]
    out = open(sys.argv[3], "w") if len(sys.argv) > 3 else sys.stdout
    n = min(len(a), len(b))
    first = None
    for i in range(n):
        same = a[i][0] == b[i][0]
        if not same and first is None:
            first = i
        mark = "  " if same else "!!"
        extra = f"   [oracle sp_add off-row {a[i][1][0]}, past-end {a[i][1][1]}]" if a[i][1] and a[i][1][0] else ""
        out.write(f"{mark} {a[i][2]}{extra}\n")
        if not same:
            out.write(f"!! gpu: {b[i][2]}\n")
    out.write(f"# {n} events compared (oracle {len(a)}, gpu {len(b)}); "
              + ("identical" if first is None else f"first difference at event {first}") + "\n")
    return 0 if first is None else 1


if __name__ == "__main__":
    sys.exit(main())

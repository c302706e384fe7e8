#!/usr/bin/env python3
"""Re-derive stored oracle digests from the REFERENCE itself (run here, on the CPU;
TEST INFRASTRUCTURE, never on the GPU box).

For every named case of tests/golden/digests.json, runs the case's generator through
oracle/_ref/libref_amg.so (the reference's own amg_setup, compiled from
/root/reference by `make -C oracle ref`) and compares the SHA-256 of every hierarchy
array with the stored digest (made by the oracle).  Equal digests pin the oracle at
that size with the reference's own output, not only with its fixtures.  The result
is appended to tests/golden/ref_digest_check.json (case -> identical / first
differing array, reference seconds).

usage: python tests/golden/ref_digest_check.py p27_20 [case ...]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_digests as md  # noqa: E402

OUT = os.path.join(HERE, "ref_digest_check.json")


def main():
    db = json.load(open(md.OUT))
    res = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for name in sys.argv[1:]:
        want = db["cases"][name]
        gen = want["gen"]
        import ctypes as C
        from omp_amg_amd import abi
        lib = abi.bind_setup(C.CDLL(md.REF_SO))
        Ai, Aj, Av = md.generate(gen)
        assert md.input_digest(Ai, Aj, Av) == want["input_sha256"], name
        t0 = time.time()
        h = abi.run_setup(lib, Ai, Aj, Av)
        secs = round(time.time() - t0, 1)
        got = md.hierarchy_digest(h)
        diff = sorted(k for k in set(got) | set(want["arrays"]) if got.get(k) != want["arrays"].get(k))
        res[name] = {"identical": not diff, "arrays": len(got), "differ": diff[:5],
                     "reference_secs": secs, "oracle_secs": want["secs"], "levels": h.nlevels}
        print(name, res[name], flush=True)
        with open(OUT, "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()

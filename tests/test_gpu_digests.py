"""Parity at sizes where the DEFAULT kernel routing engages, with no forcing switch.

tests/golden/digests.json (tests/golden/make_digests.py) holds, per case, the
generator of the input, its SHA-256, and a SHA-256 of every array of the expected
hierarchy -- from the reference itself (sem_e3_N7, 8 000 rows, order N = 7 as in
BASELINE configs[2]) or from the oracle, which tests/test_oracle_golden.py pins bit
for bit to the reference's own outputs.  Equal digests = bit-identical hierarchy
(C/F sets, ids, every CSR pattern and every double).

The GPU run also records which kernel routes ran (omp_amg_amd.route_stats), so each
case shows that the paths the small fixtures reach only by forcing -- incremental
coarsening and find_support sweeps, the pipelined long-row SpMV (k_spmv_pipe) with 4 / 16
rows per wavefront, wave-private windowed / k-sequential SpGEMM, the 512- / 1024-point
Q-factor tiers -- were the ones that produced the matching bits.
"""
import json
import os

import pytest

from conftest import GOLD
import omp_amg_amd as oa
from omp_amg_amd import abi

DIGESTS = os.path.join(GOLD, "digests.json")


def _db():
    return json.load(open(DIGESTS)) if os.path.exists(DIGESTS) else {"cases": {}, "excluded": {}}


def _mk():
    import sys
    sys.path.insert(0, GOLD)
    import make_digests
    return make_digests


# routes each case must take with the default routing (what its sizes guarantee; the
# 64-rows-per-wavefront SpMV needs a >= 2^22-row long-row matrix, which no digest here has
# -- test_gpu_matches_digest_rw64_forced covers its shape on p7_96 / p7_128).  "mv_long"
# (the grid-wide scan for outlier rows past max(4096, 16 x mean)) runs only where such a
# row exists; none of these cases has one (round 5: find_support's R / R' are checked
# once per call, the path is no longer launched for nothing), so the forced-threshold
# kernel tests (test_gpu_kernels.py, mv_long / fs_long fixtures) cover it.
EXPECT_ROUTES = {
    "p7_48": ("cs_inc", "fs_inc", "spmv_pipe", "mv_rw4", "sg_tiny", "sg_wwin", "sg_wwin_sym",
              "qf_reuse", "sg_symreuse", "spat_inc"),
    "p7_64": ("cs_inc", "fs_inc", "spmv_pipe", "mv_rw4", "sg_tiny", "sg_wwin", "sg_wwin_sym",
              "qf_reuse", "mv_pair", "fs_amx", "sg_symreuse", "spat_inc"),
    "p7_96": ("cs_inc", "fs_inc", "spmv_pipe", "mv_rw4", "mv_rw16", "sg_tiny", "sg_wwin",
              "sg_wwin_sym", "qf_reuse", "qf_t512", "qf_t1024", "mv_pair", "fs_amx", "sg_symreuse", "spat_inc"),
    "p7_128": ("cs_inc", "fs_inc", "spmv_pipe", "mv_rw4", "mv_rw16", "sg_tiny", "sg_wwin",
               "sg_wwin_sym", "qf_reuse", "qf_t512", "qf_t1024", "mv_pair", "fs_amx", "sg_symreuse", "spat_inc"),
    "aniso_20": ("fs_inc",),
    "aniso_32": ("fs_inc", "spmv_pipe"),
    "p27_20": ("fs_inc", "spmv_pipe", "sg_wwin_sym", "sg_symreuse", "spat_inc"),
    "sem_e3_N7": ("spmv_pipe", "sg_wwin_sym"),
    "sem_e4_N7": ("spmv_pipe", "sg_kseq", "sg_wwin_sym"),
    "sem_e5_N7": ("spmv_pipe", "sg_kseq"),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(_db()["cases"]))
def test_gpu_matches_digest_default_routing(case):
    mk = _mk()
    d = _db()["cases"][case]
    Ai, Aj, Av = mk.generate(d["gen"])
    assert mk.input_digest(Ai, Aj, Av) == d["input_sha256"], "input generator drifted"
    oa.route_stats(reset=True)
    h = abi.run_setup(oa.lib(), Ai, Aj, Av)
    routes = oa.route_stats(reset=True)
    got = mk.hierarchy_digest(h)
    exp = d["arrays"]
    bad = sorted(k for k in set(got) | set(exp) if got.get(k) != exp.get(k))
    assert not bad, f"{len(bad)} arrays differ from the {d['source']}: {bad[:12]} (summary {mk.summary(h)} " \
                    f"vs {d['summary']})"
    missing = [r for r in EXPECT_ROUTES.get(case, ()) if routes[r] == 0]
    assert not missing, f"default routes not taken: {missing} ({routes})"
    print(case, d["source"], d["summary"]["n"], routes)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["p7_64", "p7_96"])
def test_gpu_matches_digest_unfused_selection(case):
    """find_support's selection by its own pass over the bad columns (k_fs_select) instead
    of the maxima fused into the full sweeps' w = R' rs product (the default since round
    5): the same stored digest either way"""
    mk = _mk()
    d = _db()["cases"][case]
    Ai, Aj, Av = mk.generate(d["gen"])
    oa.fs_amx(0)
    oa.route_stats(reset=True)
    try:
        h = abi.run_setup(oa.lib(), Ai, Aj, Av)
    finally:
        oa.fs_amx(-1)
    assert oa.route_stats(reset=True)["fs_amx"] == 0
    got = mk.hierarchy_digest(h)
    exp = d["arrays"]
    bad = sorted(k for k in set(got) | set(exp) if got.get(k) != exp.get(k))
    assert not bad, f"{len(bad)} arrays differ from the {d['source']}: {bad[:12]}"


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["p7_64", "p27_20"])
def test_gpu_matches_digest_whole_constraint_pattern(case):
    """the constraint operator's pattern W_skel W_skel' formed whole in every interpolation
    iteration instead of grown from the previous iteration's (the default since round 6):
    the same stored digest either way"""
    mk = _mk()
    d = _db()["cases"][case]
    Ai, Aj, Av = mk.generate(d["gen"])
    oa.spat_inc(0)
    oa.route_stats(reset=True)
    try:
        h = abi.run_setup(oa.lib(), Ai, Aj, Av)
    finally:
        oa.spat_inc(-1)
    assert oa.route_stats(reset=True)["spat_inc"] == 0
    got = mk.hierarchy_digest(h)
    exp = d["arrays"]
    bad = sorted(k for k in set(got) | set(exp) if got.get(k) != exp.get(k))
    assert not bad, f"{len(bad)} arrays differ from the {d['source']}: {bad[:12]}"


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["p7_96", "p7_128"])
def test_gpu_matches_digest_rw64_forced(case):
    """the 64-rows-per-wavefront long-row SpMV (k_spmv_pipe<*,64,16>, by default only on
    >= 2^22-row long-row matrices, amgd_sparse.hip lane_rw) forced on every long-row
    product of the 0.9 M / 2.1 M-row digests: the whole hierarchy stays bit-identical"""
    mk = _mk()
    d = _db()["cases"][case]
    Ai, Aj, Av = mk.generate(d["gen"])
    oa.route_stats(reset=True)
    oa.spmv_rw(64)
    try:
        h = abi.run_setup(oa.lib(), Ai, Aj, Av)
    finally:
        oa.spmv_rw(-1)
    routes = oa.route_stats(reset=True)
    got = mk.hierarchy_digest(h)
    exp = d["arrays"]
    bad = sorted(k for k in set(got) | set(exp) if got.get(k) != exp.get(k))
    assert not bad, f"{len(bad)} arrays differ: {bad[:12]}"
    assert routes["mv_rw64"] > 0 and routes["mv_rw16"] == 0 and routes["mv_rw4"] == 0, routes
    print(case, routes)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["aniso_32", "p27_24"])
def test_gpu_matches_digest_long_paths_forced(case):
    """the outlier-row paths forced from 8 entries on (find_support's grid-wide expansion,
    the chunked long-column selection k_fsl_*, the exact long-row products) on digests
    whose orphan columns span many 2048-entry chunks: the stored digest"""
    mk = _mk()
    d = _db()["cases"][case]
    Ai, Aj, Av = mk.generate(d["gen"])
    oa.fs_long(8)
    oa.mv_long(8)
    try:
        h = abi.run_setup(oa.lib(), Ai, Aj, Av)
    finally:
        oa.fs_long(-1)
        oa.mv_long(-1)
    got = mk.hierarchy_digest(h)
    exp = d["arrays"]
    bad = sorted(k for k in set(got) | set(exp) if got.get(k) != exp.get(k))
    assert not bad, f"{len(bad)} arrays differ: {bad[:12]}"

"""interp_lmop (amg_setup.c:1589): the row-pull path (omp_amg_amd/csrc/amgd_lmop.hip)
against the general key/sort walk, bit for bit, on whole setups.

The fixtures (test_gpu_parity.py) already pin the default path to the reference;
here the two device paths are run on the same inputs and every double of the two
hierarchies must agree, and the counters must show the fast path was taken."""
import numpy as np
import pytest

import omp_amg_amd as oa
from omp_amg_amd import abi, parity, problems

pytestmark = pytest.mark.gpu


def _run(Ai, Aj, Av, mode):
    oa.lmop_mode(mode)
    oa.lmop_stats(reset=True)
    try:
        h = abi.run_setup(oa.lib(), Ai, Aj, Av)
    finally:
        oa.lmop_mode(0)
    return h, oa.lmop_stats(reset=True)


@pytest.mark.parametrize("gen", [
    ("p7_16", lambda: problems.poisson3d(16)),
    ("p7_20x12x9", lambda: problems.poisson3d(9, mx=20, my=12)),
    ("aniso_14", lambda: problems.poisson3d(14, eps=1e-3)),
    ("p27_10", lambda: problems.poisson3d(10, 27)),
    ("p2d9_40", lambda: problems.poisson2d(40, 9)),
    ("sem_e3_N3", lambda: problems.sem_laplacian(3, 3, 3, 3, seed=5, jitter=0.3)),
], ids=lambda g: g[0])
@pytest.mark.parametrize("small", [1, 0], ids=["small_rows_thread", "small_rows_wave"])
def test_lmop_fast_equals_general(gen, small):
    """row pull (S rows of <= 32 entries one thread each, or all on wavefronts) against
    the general walk"""
    Ai, Aj, Av = gen[1]()
    hg, sg = _run(Ai, Aj, Av, 1)
    oa.lmop_small(small)
    try:
        hf, sf = _run(Ai, Aj, Av, 0)
    finally:
        oa.lmop_small(-1)
    assert sg["fast"] == 0 and sg["general"] > 0
    assert sf["fast"] > 0, sf
    assert sf["misses"] == 0, sf
    bad = parity.compare(hg, hf, exact=True)
    assert not bad, bad


@pytest.mark.parametrize("wave", [-1, 1, 0], ids=["wave64", "wave", "thread"])
@pytest.mark.parametrize("mode", [0, 1], ids=["rowpull", "general"])
@pytest.mark.parametrize("gen", [
    ("aniso_14", lambda: problems.poisson3d(14, eps=1e-3)),
    ("aniso_16x10x8", lambda: problems.poisson3d(8, mx=16, my=10, eps=1e-3)),
    ("p7_16", lambda: problems.poisson3d(16)),
    ("sem_e3_N3", lambda: problems.sem_laplacian(3, 3, 3, 3, seed=5, jitter=0.3)),
], ids=lambda g: g[0])
def test_lmop_pruned_equals_full(gen, mode, wave):
    """the general walk with supports of >= 8 points pruned to same-component
    contributions of their factor graph (default: >= 4096 points) against no pruning:
    every double of the two hierarchies agrees.  In "general" mode every support takes
    the walk; in "rowpull" only the dirty ones (the orphan support of anisotropic levels)"""
    Ai, Aj, Av = gen[1]()
    oa.lmop_prune(0)
    oa.lmop_wave(wave)       # walks per wavefront from 64 points (default), always, never
    try:
        h_full, s_full = _run(Ai, Aj, Av, mode)
        oa.lmop_prune(8)
        h_pr, s_pr = _run(Ai, Aj, Av, mode)
    finally:
        oa.lmop_prune(-1)
        oa.lmop_wave(-1)
    assert s_full["pruned"] == 0
    if mode == 1 or gen[0].startswith("aniso"):
        assert s_pr["pruned"] > 0, s_pr
    bad = parity.compare(h_full, h_pr, exact=True)
    assert not bad, bad

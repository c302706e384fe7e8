"""CPU-only checks of the drop-in boundary: the HIP library loads without a
GPU and exports every function the public headers declare; host-side helpers."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = ["include/amg_setup.h", "include/crs.h", "include/omp_amg_amd.h"]


def declared_functions():
    names = set()
    for h in HEADERS:
        src = open(os.path.join(ROOT, h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", src):
            name = m.group(1)
            if name in ("if", "sizeof", "defined"):
                continue
            # only names in a declaration position: preceded by a type on the line
            line = src[src.rfind("\n", 0, m.start()) + 1:m.start()]
            if re.search(r"(void|int|double|char|u?int\d+_t|size_t|\*|struct\s+\w+\s*\*?)\s*$", line.strip() + " ") and \
                    not line.strip().startswith(("typedef", "#")):
                names.add(name)
    return names


def test_library_exports_every_declared_symbol():
    import omp_amg_amd as oa
    if not os.path.exists(oa.LIB_PATH):
        oa.build()
    lib = ctypes.CDLL(oa.LIB_PATH)   # loads without a GPU
    missing = [n for n in sorted(declared_functions()) if not hasattr(lib, n)]
    assert not missing, missing
    assert {"amg_setup", "amg_export", "free_data", "crs_setup", "crs_free",
            "amgd_setup_device"} <= declared_functions()


def test_only_api_symbols_exported():
    import omp_amg_amd as oa
    out = subprocess.run(["nm", "-D", "--defined-only", oa.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if l.strip()}
    internal = [s for s in syms if s.startswith("amgd_") and not s.startswith(("amgd_test_", "amgd_dev_"))
                and s not in declared_functions()]
    assert not internal, internal


def test_struct_layout_matches_reference():
    from omp_amg_amd import abi
    assert ctypes.sizeof(abi.CsrMat) == 5 * 8
    assert ctypes.sizeof(abi.AmgSetupData) == 2 * 8 + 6 * 8 + 8 + 8 + 2 * 8 + 3 * 8 + 3 * 8 + 2 * 8


def test_problem_generators_are_assembled():
    from omp_amg_amd import problems
    for Ai, Aj, Av in (problems.poisson3d(5), problems.poisson3d(4, 27), problems.poisson2d(6),
                       problems.sem_laplacian(2, 2, 2, 3)):
        key = Ai.astype(np.int64) * (int(Aj.max()) + 1) + Aj
        assert len(np.unique(key)) == len(key)
        assert np.all(Av != 0)
        d = {}
        for i, j, v in zip(Ai, Aj, Av):
            d[(int(i), int(j))] = v
        assert all(abs(d[(j, i)] - v) <= 1e-12 * abs(v) for (i, j), v in d.items())


def test_crs_setup_rejects_foreign_comm_without_gpu():
    """crs_setup with comm->np > 1 but no library communicator of those ranks returns
    NULL before touching the device (no hang waiting for peers, no abort)"""
    import omp_amg_amd as oa
    from omp_amg_amd import abi
    if not os.path.exists(oa.LIB_PATH):
        oa.build()
    lib = ctypes.CDLL(oa.LIB_PATH)
    A = np.array([2, -1, -1, 0, -1, 2, 0, -1, -1, 0, 2, -1, 0, -1, -1, 2], dtype=np.float64)
    h = abi.crs_setup(lib, 4, [1, 2, 3, 4], np.repeat(np.arange(4), 4), np.tile(np.arange(4), 4), A,
                      rank=1, np_=2, quiet=False)
    assert h is None

"""pytest configuration: the `gpu` marker and shared fixtures.

`-m "not gpu"` runs here (no GPU): oracle vs golden vectors, host logic, the
C-ABI library's exported symbols, multi-rank host logic over gloo.
`-m gpu` runs on an MI355X: parity of the HIP path (through the C ABI) against
the oracle / golden fixtures.
"""
import ctypes
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GOLD = os.path.join(ROOT, "tests", "golden")
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_amg.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def golden_cases():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "*.npz")))


@pytest.fixture(scope="session")
def oracle_lib():
    """CPU restatement (test infrastructure).  Built on demand from oracle/."""
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-s", "all"], check=True)
    from omp_amg_amd import abi
    return abi.bind_setup(ctypes.CDLL(ORACLE_SO))


@pytest.fixture(scope="session")
def ref_lib():
    """The reference compiled from /root/reference (present only where it was built)."""
    if not os.path.exists(REF_SO):
        if os.path.isdir("/root/reference"):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-s", "ref"], check=True)
        else:
            pytest.skip("reference build not available")
    from omp_amg_amd import abi
    return abi.bind_setup(ctypes.CDLL(REF_SO))

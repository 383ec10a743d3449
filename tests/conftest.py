"""Test configuration: `gpu` marker, import paths and library fixtures.

CPU tests (`-m "not gpu"`) cover the oracles (O1 message-level, O2 bitset),
known-answer tests, golden fixtures, host builders, the sharded protocol over
gloo, and that libgossip_hip.so loads and exports every gossip.h symbol.
GPU tests (`-m gpu`) are the parity tests of the HIP engine against O2/O1.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "gossip-glomers-distributed-systems_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

CPU_LIB = os.path.join(REPO, "oracle", "_build", "libgossip_cpu.so")
HIP_LIB = os.environ.get("GG_HIP_LIB") or os.path.join(PKG, "libgossip_hip.so")  # GG_HIP_LIB: A/B builds
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def cpu_lib():
    if not os.path.exists(CPU_LIB):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])
    return CPU_LIB


@pytest.fixture(scope="session")
def hip_lib():
    assert os.path.exists(HIP_LIB), "libgossip_hip.so missing: run make in the package dir"
    return HIP_LIB


@pytest.fixture(autouse=True)
def _no_orphan_ranks():
    """Rank processes a failed multi-process test left behind (one rank died
    in its rendezvous, the others wait in theirs) are killed when the test
    ends, so the run reports the failure instead of hanging at exit."""
    yield
    import multiprocessing
    for p in multiprocessing.active_children():
        p.kill()
        p.join(10)

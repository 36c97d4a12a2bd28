"""pytest configuration: markers, import paths, build-on-demand of the native
libraries (libnffacl for the product, liboracle for the checker)."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "nff-go_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _ensure_built():
    lib = PKG / "libnffacl.so"
    if not lib.exists():
        subprocess.run(["make", "-s", "-C", str(PKG), f"-j{min(8, os.cpu_count() or 1)}"], check=True)
    orc = ROOT / "oracle" / "liboracle.so"
    if not orc.exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)


_ensure_built()

GOLDEN = ROOT / "tests" / "golden"


@pytest.fixture(scope="session")
def golden():
    return GOLDEN


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()

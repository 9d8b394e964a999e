"""Shared fixtures.  `gpu` tests need a gfx950 device and the built HIP library;
everything else runs on the CPU (oracle, host logic, ABI exports)."""
import importlib.util
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG_DIR = ROOT / "orb_slam2-chinese-annotation_amd"
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X) and lib/liborb_amd.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_pkg():
    if "orb_amd" in sys.modules:
        return sys.modules["orb_amd"]
    spec = importlib.util.spec_from_file_location(
        "orb_amd", PKG_DIR / "__init__.py", submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["orb_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def orb():
    return load_pkg()


@pytest.fixture(scope="session")
def oracle():
    import oracle as o  # oracle/oracle.py
    o.lib()
    return o


@pytest.fixture(scope="session")
def gpu(orb):
    """The product library on a visible gfx950 device (fails loudly otherwise)."""
    if orb.device_count() <= 0:
        pytest.fail("gpu test but no HIP device is visible")
    return orb


REFERENCE = Path(os.environ.get("ORB_REFERENCE", "/root/reference"))

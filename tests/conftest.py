import importlib.util
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "adaptive-rgbd-localization-mappig_amd")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")


def load_pkg():
    """Import the package from its hyphenated directory as `arlm_amd`."""
    name = "arlm_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_synth():
    load_pkg_no_lib = None  # synth has no dependency on the HIP library
    name = "arlm_amd_synth"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, os.path.join(PKG_DIR, "synth.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


_SEQ_CACHE = {}


def sequence(n, w=640, h=480, intrinsics=None, seed=0x5EED0002, closed_loop=False, hard=False):
    key = (n, w, h, tuple(sorted((intrinsics or {}).items())), seed, closed_loop, hard)
    if key not in _SEQ_CACHE:
        _SEQ_CACHE[key] = load_synth().make_sequence(n, w, h, intrinsics=intrinsics, seed=seed,
                                                     closed_loop=closed_loop, hard=hard)
    return _SEQ_CACHE[key]


@pytest.fixture(scope="session")
def pkg():
    return load_pkg()


@pytest.fixture(scope="session")
def synth():
    return load_synth()


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False

"""CPU tests of the C-ABI library: it loads, exports every symbol include/odo.h
declares, its host-side glibc rand() restatement matches the real libc, and it
refuses to run without a gfx950 device (no CPU fallback)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import oracle_lib as O
from conftest import ROOT, gpu_available, load_pkg


def declared_functions():
    src = open(os.path.join(ROOT, "include", "odo.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(odo_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    pkg = load_pkg()
    lib = pkg.load()
    names = declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"libodo_hip.so does not export {n}"
        assert n in pkg._abi.SIGNATURES, f"python binding lacks {n}"


def test_header_compiles_as_c():
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write('#include "odo.h"\nint main(void){odo_config c; odo_default_config(&c,640,480,1);'
                           'return sizeof(orb_kp)==28 && sizeof(odo_dmatch)==16 ? 0 : 1;}\n')
        subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-c", c, "-I", os.path.join(ROOT, "include"),
                        "-o", os.path.join(d, "t.o")], check=True)


@pytest.mark.parametrize("seed", [1, 42, 0x5EED0000, 2**31 + 7])
def test_library_rng_matches_glibc(seed):
    pkg = load_pkg()
    ref = np.zeros(1000, np.int32)
    O.lib().oracle_libc_rand_stream(seed, 1000, O.ptr(ref))
    assert np.array_equal(pkg.rng_stream(seed, 1000), ref)


def test_pair_seed_is_splitmix64():
    pkg = load_pkg()
    assert pkg.pair_seed(0, 0) == 0xE220A8397B1DCDAF & 0xFFFFFFFF


def test_config_struct_size_checked():
    """odo_config carries its own size; a caller built against a
    different odo.h (a smaller or larger struct) fails in odo_create with a
    clear message instead of reading past its struct (checked before any
    device call, so this runs on CPU)."""
    pkg = load_pkg()
    lib = pkg.load()
    assert lib.odo_abi_version() == 5
    cfg = pkg.default_config(640, 480, 1)
    assert cfg.struct_size == C.sizeof(pkg._abi.Config)
    cfg.struct_size -= 8  # an older, shorter odo_config
    assert not lib.odo_create(C.byref(cfg), 0)
    assert b"struct_size" in lib.odo_last_error()


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU failure path")
def test_no_cpu_fallback():
    pkg = load_pkg()
    with pytest.raises(RuntimeError, match="no HIP device"):
        pkg.Odometry(pkg.default_config(640, 480, 1))

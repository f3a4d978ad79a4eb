"""The C++ mirror of the reference's hot-path classes (include/odo_frontend.hpp:
odo_hip::Extractor / Frame / Matcher / Ransac / PnPSolver / Kabsch, standing in
for Features/extractor.h, Core/frame.h, Features/matcher.h, Odometry/ransac.h,
Odometry/pnpsolver.h, Odometry/kabsch.h) driven by tests/cpp/frontend_parity.cpp
in the reference's Tracking::TrackFrame call pattern and checked against the
oracle inside that program (bit-exact features / matches / RANSAC, PnP pose
within 1e-4), then Matcher::ProjectionMatch of the last frame at its PnP pose
against the previous frame's landmarks (slots and isInFrustum projections
bit-exact). The binary is built by build() (tests/cpp/Makefile) and links
libodo_hip.so + liboracle.so through relative rpaths."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, sequence

CPP = os.path.join(ROOT, "tests", "cpp")
BIN = os.path.join(CPP, "build", "frontend_parity")


def _binary():
    if not os.path.exists(BIN):
        subprocess.run(["make", "-s", "-C", CPP], check=True)
    return BIN


def _write_frames(path, bgr, dep):
    with open(path, "wb") as f:
        f.write(np.ascontiguousarray(bgr).tobytes())
        f.write(np.ascontiguousarray(dep).tobytes())


def test_header_compiles_standalone(tmp_path):
    """odo_frontend.hpp is self-contained C++17 over odo.h (no OpenCV/Eigen)."""
    src = tmp_path / "t.cpp"
    src.write_text('#include "odo_frontend.hpp"\nint main() { odo_hip::Matcher m(0.9f); return (int)m.mfNNratio; }\n')
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter", "-fsyntax-only",
                    "-I", os.path.join(ROOT, "include"), str(src)], check=True)


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="checks the no-device path")
def test_fails_loudly_without_device(tmp_path):
    """No gfx950 device: the first GPU call throws odo_hip::Error (no CPU fallback)."""
    bgr, dep, _ = sequence(2, seed=0x5EED0031)
    p = tmp_path / "f.bin"
    _write_frames(p, bgr, dep)
    r = subprocess.run([_binary(), str(p), "640", "480", "2", "7"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 3, r.stderr
    assert "no CPU fallback" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["orb_slam2", "adaptive", "adaptive_orb"])
def test_frontend_parity(tmp_path, mode):
    bgr, dep, _ = sequence(5, seed=0x5EED0032)
    p = tmp_path / "f.bin"
    _write_frames(p, bgr, dep)
    args = [_binary(), str(p), "640", "480", "5", "0x1234"] + ([mode] if mode != "orb_slam2" else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=110)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "failures=0" in r.stdout
    stats = dict(kv.split("=") for kv in r.stdout.split()[2:])
    assert int(stats["matches"]) > 100 and int(stats["pnp_inliers"]) > 50
    assert int(stats["projection_matches"]) > 0

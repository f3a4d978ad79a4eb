"""TUM RGB-D input: associations.txt parsed as LoadImages
(Utils/utils.cpp:16-38) and frames read as main.cpp:93-95 (IMREAD_COLOR ->
BGR8, IMREAD_UNCHANGED -> depth16), on a small sequence written here."""
import os

import numpy as np
import pytest

from conftest import load_pkg  # noqa: F401  (package path set up by conftest)

Image = pytest.importorskip("PIL.Image")


def _tum():
    import importlib.util
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "adaptive-rgbd-localization-mappig_amd", "tum.py")
    spec = importlib.util.spec_from_file_location("arlm_tum", root)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_associations_and_frames(tmp_path):
    tum = _tum()
    rng = np.random.default_rng(0)
    (tmp_path / "rgb").mkdir()
    (tmp_path / "depth").mkdir()
    rgbs, deps, lines = [], [], []
    for k in range(3):
        rgb = rng.integers(0, 256, (12, 16, 3), dtype=np.uint8)
        dep = rng.integers(0, 65536, (12, 16), dtype=np.uint16)
        Image.fromarray(rgb, "RGB").save(tmp_path / "rgb" / f"{k}.png")
        Image.fromarray(dep).save(tmp_path / "depth" / f"{k}.png")
        rgbs.append(rgb)
        deps.append(dep)
        lines.append(f"{1305031102.175304 + k:.6f} rgb/{k}.png {1305031102.160407 + k:.6f} depth/{k}.png")
    # LoadImages skips empty lines only; the depth timestamp is read and dropped
    (tmp_path / "associations.txt").write_text(lines[0] + "\n\n" + "\n".join(lines[1:]) + "\n")
    ts, r, d = tum.load_associations(str(tmp_path / "associations.txt"))
    assert r == [f"rgb/{k}.png" for k in range(3)] and d == [f"depth/{k}.png" for k in range(3)]
    np.testing.assert_allclose(ts, [1305031102.175304 + k for k in range(3)])
    bgr, depth, ts2 = tum.load_sequence(str(tmp_path), 2, first=1)
    assert bgr.shape == (2, 12, 16, 3) and depth.shape == (2, 12, 16) and depth.dtype == np.uint16
    for i in range(2):
        assert np.array_equal(bgr[i], rgbs[1 + i][:, :, ::-1])  # IMREAD_COLOR is BGR
        assert np.array_equal(depth[i], deps[1 + i])
    np.testing.assert_allclose(ts2, ts[1:3])

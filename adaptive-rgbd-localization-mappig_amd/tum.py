"""TUM RGB-D sequence input (the harness accepts a real
`associations.txt` when one is present on the box).

load_associations restates LoadImages (Utils/utils.cpp:16-38): every
non-empty line is `t_rgb rgb_path t_depth depth_path`; the RGB timestamp is
the frame's timestamp and the depth timestamp is read and dropped. read_frames
restates main.cpp:93-95: `cv::imread(baseDir + rgb, IMREAD_COLOR)` (BGR8,
3 channels whatever the file holds) and `cv::imread(baseDir + depth,
IMREAD_UNCHANGED)` (the 16-bit depth PNG as stored, x5000 per metre). Decoding
is host I/O outside the timed region (§8(d) excludes decode); PIL decodes the
PNGs here (OpenCV is absent from the image).
"""
from __future__ import annotations

import os

import numpy as np


def load_associations(path: str):
    """(timestamps float64 [n], rgb paths, depth paths) in file order."""
    ts, rgb, dep = [], [], []
    with open(path) as f:
        for line in f:
            s = line.rstrip("\n")
            if not s:
                continue
            parts = s.split()
            # stringstream >> t >> sRGB >> t >> sD: missing fields stay empty
            ts.append(float(parts[0]) if parts else 0.0)
            rgb.append(parts[1] if len(parts) > 1 else "")
            dep.append(parts[3] if len(parts) > 3 else "")
    return np.asarray(ts, np.float64), rgb, dep


def imread_color(path: str) -> np.ndarray:
    """cv::imread(path, IMREAD_COLOR): H x W x 3 BGR u8."""
    from PIL import Image
    with Image.open(path) as im:
        a = np.asarray(im.convert("RGB"), np.uint8)
    return np.ascontiguousarray(a[:, :, ::-1])


def imread_unchanged_depth(path: str) -> np.ndarray:
    """cv::imread(path, IMREAD_UNCHANGED) of a TUM depth PNG: H x W u16."""
    from PIL import Image
    with Image.open(path) as im:
        if im.mode in ("I;16", "I;16B", "I;16L"):
            a = np.frombuffer(im.tobytes(), dtype="<u2" if im.mode != "I;16B" else ">u2").reshape(im.size[1], im.size[0])
        else:
            a = np.asarray(im)
    return np.ascontiguousarray(a.astype(np.uint16))


def read_frames(base_dir: str, rgb: list, dep: list, indices=None):
    """BGR8 [n, H, W, 3] and depth16 [n, H, W] of the listed frames."""
    idx = range(len(rgb)) if indices is None else indices
    b = [imread_color(os.path.join(base_dir, rgb[i])) for i in idx]
    d = [imread_unchanged_depth(os.path.join(base_dir, dep[i])) for i in idx]
    return np.stack(b), np.stack(d)


def load_sequence(base_dir: str, n: int, associations: str = "associations.txt", first: int = 0):
    """The first n frames (from `first`) of a TUM sequence directory."""
    ts, rgb, dep = load_associations(os.path.join(base_dir, associations))
    idx = list(range(first, min(first + n, len(rgb))))
    bgr, depth = read_frames(base_dir, rgb, dep, idx)
    return bgr, depth, ts[idx]

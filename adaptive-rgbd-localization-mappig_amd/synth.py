"""Deterministic synthetic RGB-D sequences (SURVEY.md §8d "Renderer").

TUM / ICL-NUIM data are not available offline, so benchmarks and parity tests
run on a ray-cast textured "room": an axis-aligned box with a few cuboids
inside, every surface carrying a procedural texture (a jittered brick mosaic
of random-grey tiles plus band-limited value noise, full uint8 range). Depth is the
camera-frame z stored as uint16 x 5000 (Utils/common.h:67 depthFactor 1/5000)
with ~3% dropped pixels and one hole blob. Consecutive frames follow a random
SE(3) walk with a bounded step.

Everything is integer-hash / float64 numpy, so the same seed gives the same
frames on any host.
"""
from __future__ import annotations

import dataclasses
import math
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

_M32 = np.uint64(0xFFFFFFFF)


def _hash(*keys: np.ndarray) -> np.ndarray:
    """Integer hash of int64 arrays -> float64 in [0,1)."""
    h = np.uint64(0x9E3779B9)
    for k in keys:
        k = np.asarray(k).astype(np.int64).astype(np.uint64) & _M32
        h = (h ^ k) * np.uint64(0x85EBCA6B) & _M32
        h = (h ^ (h >> np.uint64(13))) * np.uint64(0xC2B2AE35) & _M32
        h = h ^ (h >> np.uint64(16))
    return (h & np.uint64(0xFFFFFF)).astype(np.float64) / float(1 << 24)


def _value_noise(u, v, sid, seed, octaves=3, base=0.35):
    acc = np.zeros_like(u)
    amp, tot = 1.0, 0.0
    freq = 1.0 / base
    for o in range(octaves):
        x, y = u * freq, v * freq
        ix, iy = np.floor(x), np.floor(y)
        fx, fy = x - ix, y - iy
        fx = fx * fx * (3 - 2 * fx)
        fy = fy * fy * (3 - 2 * fy)
        ix = ix.astype(np.int64)
        iy = iy.astype(np.int64)
        k = sid * 7 + o + seed * 131
        a = _hash(ix, iy, k)
        b = _hash(ix + 1, iy, k)
        c = _hash(ix, iy + 1, k)
        d = _hash(ix + 1, iy + 1, k)
        acc += amp * ((a * (1 - fx) + b * fx) * (1 - fy) + (c * (1 - fx) + d * fx) * fy)
        tot += amp
        amp *= 0.5
        freq *= 2.0
    return acc / tot


def _texture(u, v, sid, seed):
    """Brick-like mosaic of random-grey tiles with jittered widths (sharp,
    distinctive corners for FAST/rBRIEF) blended with band-limited value noise."""
    tile = 0.08
    row = np.floor(v / tile).astype(np.int64)
    off = _hash(row, sid, 7) * tile
    tw = tile * (0.6 + 0.8 * _hash(row, sid, 3))
    tu = np.floor((u + off) / tw).astype(np.int64)
    mosaic = _hash(tu, row, sid + 1000 * seed)
    noise = _value_noise(u * 2, v * 2, sid, seed, octaves=4)
    return 0.5 * mosaic + 0.5 * noise


@dataclasses.dataclass
class Camera:
    w: int
    h: int
    fx: float
    fy: float
    cx: float
    cy: float


FR1 = dict(fx=517.3, fy=516.5, cx=318.6, cy=255.3)           # common.h:35-38
FR2 = dict(fx=520.9, fy=521.0, cx=325.1, cy=249.7)           # common.h:47-50
ICL = dict(fx=481.20, fy=-480.00, cx=319.50, cy=239.50)      # common.h:55-58


def _rot(ax, ay, az):
    cx_, sx_ = math.cos(ax), math.sin(ax)
    cy_, sy_ = math.cos(ay), math.sin(ay)
    cz_, sz_ = math.cos(az), math.sin(az)
    rx = np.array([[1, 0, 0], [0, cx_, -sx_], [0, sx_, cx_]])
    ry = np.array([[cy_, 0, sy_], [0, 1, 0], [-sy_, 0, cy_]])
    rz = np.array([[cz_, -sz_, 0], [sz_, cz_, 0], [0, 0, 1]])
    return rz @ ry @ rx


class Scene:
    """Desk-sized room [-1.7,1.7]x[-1.2,1.2]x[-1.0,3.0] with cuboid obstacles.

    hard=True (the "hard" workload): two extra cuboids move on their own
    periodic paths (dynamic outliers for RANSAC), the floor and ceiling carry an
    exactly periodic tile pattern (repeated texture: ambiguous descriptors),
    and the renderer adds image noise and depth noise."""

    def __init__(self, seed: int, hard: bool = False, period: int = 64):
        rng = np.random.default_rng(seed)
        self.seed = int(seed) & 0x7FFFFFFF
        self.hard, self.period = hard, period
        self.room_lo = np.array([-1.7, -1.2, -1.0])
        self.room_hi = np.array([1.7, 1.2, 3.0])
        boxes = []
        for _ in range(6):
            c = np.array([rng.uniform(-1.1, 1.1), rng.uniform(-0.7, 0.7), rng.uniform(1.0, 2.4)])
            s = np.array([rng.uniform(0.1, 0.35), rng.uniform(0.1, 0.4), rng.uniform(0.1, 0.35)])
            boxes.append((c - s, c + s))
        self.boxes = boxes
        # movers: (centre, half size, motion amplitude, phase), periodic in `period` frames
        self.movers = []
        if hard:
            for k in range(2):
                c = np.array([(-0.45 if k == 0 else 0.5), rng.uniform(-0.3, 0.3), rng.uniform(1.0, 1.5)])
                hs = np.array([0.36, 0.34, 0.22])
                amp = np.array([0.35, 0.15, 0.20]) * (1 if k == 0 else -1)
                self.movers.append((c, hs, amp, rng.uniform(0, 2 * math.pi)))

    def mover_boxes(self, frame: int):
        out = []
        for c, hs, amp, ph in self.movers:
            th = 2 * math.pi * (frame % self.period) / self.period * 3 + ph
            cc = c + amp * np.array([math.sin(th), math.cos(th), math.sin(2 * th)])
            out.append((cc - hs, cc + hs))
        return out

    def render(self, cam: Camera, Rwc: np.ndarray, twc: np.ndarray, frame_seed: int):
        """Return (bgr uint8 HxWx3, depth uint16 HxW) for camera pose (Rwc, twc)."""
        u, v = np.meshgrid(np.arange(cam.w, dtype=np.float64), np.arange(cam.h, dtype=np.float64))
        dc = np.stack([(u - cam.cx) / cam.fx, (v - cam.cy) / cam.fy, np.ones_like(u)], -1)
        dw = dc @ Rwc.T
        o = twc.astype(np.float64)
        with np.errstate(divide="ignore", invalid="ignore"):
            inv = 1.0 / dw
            # inside of the room: exit distance
            t1 = (self.room_lo - o) * inv
            t2 = (self.room_hi - o) * inv
            tfar = np.minimum(np.maximum(t1, t2)[..., 0], np.minimum(np.maximum(t1, t2)[..., 1], np.maximum(t1, t2)[..., 2]))
            best = tfar.copy()
            axis = np.argmin(np.maximum(t1, t2), -1)
            sid = axis * 2 + (np.take_along_axis(dw, axis[..., None], -1)[..., 0] > 0)
            for bi, (lo, hi) in enumerate(self.boxes + self.mover_boxes(frame_seed)):
                a1 = (lo - o) * inv
                a2 = (hi - o) * inv
                tmin3 = np.minimum(a1, a2)
                tn = tmin3.max(-1)
                tf = np.maximum(a1, a2).min(-1)
                hit = (tn <= tf) & (tn > 1e-6) & (tn < best)
                best = np.where(hit, tn, best)
                ax = np.argmax(tmin3, -1)
                sid = np.where(hit, 10 + bi * 3 + ax, sid)
        p = o + dw * best[..., None]
        # texture coordinates from the two axes tangent to the hit face
        face_axis = np.where(sid < 10, sid // 2, (sid - 10) % 3)
        ua = np.where(face_axis == 0, p[..., 1], p[..., 0])
        va = np.where(face_axis == 2, p[..., 1], p[..., 2])
        sidc = sid.astype(np.int64)
        g = _texture(ua, va, sidc, self.seed)
        r = _texture(ua + 0.37, va - 0.11, sidc + 50, self.seed)
        b = _texture(ua - 0.21, va + 0.53, sidc + 90, self.seed)
        col = np.stack([0.7 * b + 0.3 * g, g, 0.7 * r + 0.3 * g], -1)
        if self.hard:
            # floor and ceiling (faces of the y axis: sid 2, 3): an exactly
            # periodic 4 x 4 block of hashed tiles, repeated every 0.32 m
            rep = (sid == 2) | (sid == 3)
            tu = np.floor(ua / 0.08).astype(np.int64) & 3
            tv = np.floor(va / 0.08).astype(np.int64) & 3
            pat = _hash(tu, tv, sidc + 7) * 0.8 + 0.1 * (np.sin(ua * 40.0) > 0)
            col = np.where(rep[..., None], np.stack([pat, pat, pat], -1), col)
        rs = np.random.default_rng((self.seed * 1000003 + frame_seed) & 0xFFFFFFFF)
        if self.hard:
            col = col + rs.normal(0.0, 3.0 / 255.0, col.shape)  # sensor noise, sigma 3 grey levels
        bgr = np.clip(np.round(col * 255.0), 0, 255).astype(np.uint8)
        z = (p - o) @ Rwc[:, 2]
        if self.hard:
            z = z + rs.normal(0.0, 1.0, z.shape) * 1.425e-3 * z * z  # Kinect-like sigma_z = 1.425e-3 z^2
        d = np.round(z * 5000.0)
        d = np.where((z > 0.3) & (z < 10.0), d, 0).astype(np.uint16)
        drop = rs.random(d.shape) < 0.03
        d[drop] = 0
        hy, hx = rs.integers(0, cam.h), rs.integers(0, cam.w)
        rr = max(4, cam.w // 40)
        yy, xx = np.ogrid[: cam.h, : cam.w]
        d[(yy - hy) ** 2 + (xx - hx) ** 2 < rr * rr] = 0
        return np.ascontiguousarray(bgr), np.ascontiguousarray(d)


def _loop_pose(f: int, n: int, seed: int, speed: int = 1):
    """Closed periodic trajectory: frame n-1 -> frame 0 is an ordinary step
    (`speed` laps of the path per n frames: larger inter-frame motion)."""
    th = 2 * math.pi * f * speed / n
    ph = (seed % 997) / 997.0 * 2 * math.pi
    t = np.array([0.30 * math.sin(th + ph), 0.12 * math.sin(2 * th), -0.25 + 0.20 * math.cos(th)])
    R = _rot(0.05 + 0.10 * math.sin(th), -0.08 + 0.12 * math.cos(th + ph), 0.02 + 0.08 * math.sin(2 * th))
    return R, t


def make_sequence(n_frames: int, w: int = 640, h: int = 480, intrinsics=None, seed: int = 0x5EED0002,
                  max_step_m: float = 0.03, max_step_deg: float = 1.5, closed_loop: bool = False,
                  hard: bool = False):
    """Render n_frames consecutive frames. Returns (bgr [F,H,W,3] u8, depth [F,H,W] u16, poses [F,4,4] Twc).

    closed_loop: poses follow a periodic path so the sequence can be replayed
    back to back (bench steps) without a jump between its last and first frame.
    hard: the harder workload: image noise, depth noise
    sigma ~ z^2, two independently moving cuboids, repeated texture on the
    floor and ceiling, and twice the inter-frame motion.
    """
    intr = dict(FR1 if intrinsics is None else intrinsics)
    sx = w / 640.0
    cam = Camera(w, h, intr["fx"] * sx, intr["fy"] * sx, intr["cx"] * sx, intr["cy"] * sx)
    scene = Scene(seed, hard=hard, period=n_frames)
    rng = np.random.default_rng(seed ^ 0xABCDEF)
    R = _rot(0.05, -0.08, 0.02)
    t = np.array([0.1, 0.05, -0.3])
    bgr = np.empty((n_frames, h, w, 3), np.uint8)
    dep = np.empty((n_frames, h, w), np.uint16)
    poses = np.empty((n_frames, 4, 4))
    renders = []
    for f in range(n_frames):
        if closed_loop:
            R, t = _loop_pose(f, n_frames, seed, speed=2 if hard else 1)
        R_render = R
        if intr["fy"] < 0:  # ICL: negative fy flips the image rows
            R_render = R @ np.diag([1.0, -1.0, -1.0]) @ np.diag([1.0, -1.0, -1.0])
        renders.append((f, R_render, t))
        T = np.eye(4)
        T[:3, :3] = R
        T[:3, 3] = t
        poses[f] = T
        ang = np.deg2rad(max_step_deg) * (rng.random(3) * 2 - 1) / math.sqrt(3)
        R = R @ _rot(*ang)
        step = rng.random(3) * 2 - 1
        step *= max_step_m / max(1e-9, np.linalg.norm(step)) * rng.random()
        t = np.clip(t + step, [-0.8, -0.5, -0.6], [0.8, 0.5, 0.3])

    def render(job):
        f, Rr, tr = job
        bgr[f], dep[f] = scene.render(cam, Rr, tr, f)

    # frames are independent once the poses are drawn; numpy releases the GIL
    # in its array loops, so a thread pool renders them concurrently
    workers = max(1, min(16, os.cpu_count() or 1, n_frames))
    if workers > 1:
        with ThreadPoolExecutor(workers) as ex:
            list(ex.map(render, renders))
    else:
        for job in renders:
            render(job)
    return bgr, dep, poses


__all__ = ["make_sequence", "Scene", "Camera", "FR1", "FR2", "ICL"]

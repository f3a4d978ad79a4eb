"""Host-input path (odo_track_batch_host): the §8(d) unit starts from BGR8 +
depth16 in host memory, as Tracking::Track receives frames (main.cpp:93-102).

The upload of each batch runs on the copy stream into one of two device
staging buffers and overlaps the compute of earlier batches. The call returns
once the host buffers are consumed, so the caller refills them at once. These
tests queue batches back to back, refilling one pinned (HostFrames) or
pageable buffer right after each call, and require the results to be
identical to the device-resident path (odo_track_batch) on the same frames.
"""
import numpy as np
import pytest

from conftest import load_pkg, sequence

pytestmark = pytest.mark.gpu

B, NB, NF = 8, 5, 1000


def _cfg(pkg):
    return pkg.default_config(640, 480, B, nfeatures=NF, iterations=300, seed=0x5EED0101)


def _batches():
    bgr, dep, _ = sequence(16, seed=0x5EED0002, closed_loop=True)
    idx = [np.arange(k * B, (k + 1) * B) % 16 for k in range(NB)]
    return [(np.ascontiguousarray(bgr[i]), np.ascontiguousarray(dep[i])) for i in idx]


def _device_reference(pkg, batches):
    import torch
    odo = pkg.Odometry(_cfg(pkg))
    res = None
    for b, d in batches:
        tb = torch.from_numpy(b).to("cuda")
        td = torch.from_numpy(d.view(np.int16)).to("cuda")
        torch.cuda.synchronize()
        res = odo.track_batch(tb.data_ptr(), td.data_ptr(), B, want_results=True)
    frames = [odo.frame(i) for i in range(B)]
    pairs = [odo.pair(i)["matches"] for i in range(B)]
    latch = odo.latch
    odo.close()
    return res, frames, pairs, latch


def _check(odo, res, ref):
    rres, rframes, rpairs, rlatch = ref
    assert np.array_equal(res, rres), "pair results differ from the device-input path"
    for i in range(B):
        got = odo.frame(i)
        assert np.array_equal(got["kps"], rframes[i]["kps"]) and np.array_equal(got["desc"], rframes[i]["desc"])
        assert np.array_equal(odo.pair(i)["matches"], rpairs[i])
    assert odo.latch == rlatch


def test_pinned_host_batches_equal_device_path():
    pkg = load_pkg()
    batches = _batches()
    ref = _device_reference(pkg, batches)
    hf = pkg.HostFrames(B, 640, 480)
    odo = pkg.Odometry(_cfg(pkg))
    try:
        res = None
        for k, (b, d) in enumerate(batches):
            hf.bgr[:] = b  # refilled as soon as the previous call returned
            hf.depth[:] = d
            res = odo.track_batch_host(hf, want_results=(k == NB - 1))
        _check(odo, res, ref)
    finally:
        odo.close()
        hf.close()


def test_pageable_host_batches_equal_device_path():
    pkg = load_pkg()
    batches = _batches()
    ref = _device_reference(pkg, batches)
    bgr = np.empty_like(batches[0][0])
    dep = np.empty_like(batches[0][1])
    odo = pkg.Odometry(_cfg(pkg))
    try:
        res = None
        for k, (b, d) in enumerate(batches):
            bgr[:] = b
            dep[:] = d
            res = odo.track_batch_host(bgr, dep, want_results=(k == NB - 1))
        _check(odo, res, ref)
    finally:
        odo.close()


def test_partial_batches_from_pinned_buffer():
    """n < max_batch frames of a HostFrames buffer, alternating sizes (pair 0
    always links the previous call's last frame)."""
    pkg = load_pkg()
    bgr, dep, _ = sequence(16, seed=0x5EED0002, closed_loop=True)
    cuts = [0, 3, 8, 9, 14]
    import torch
    ref_odo = pkg.Odometry(_cfg(pkg))
    odo = pkg.Odometry(_cfg(pkg))
    hf = pkg.HostFrames(B, 640, 480)
    try:
        for a, b in zip(cuts[:-1], cuts[1:]):
            n = b - a
            tb = torch.from_numpy(np.ascontiguousarray(bgr[a:b])).to("cuda")
            td = torch.from_numpy(np.ascontiguousarray(dep[a:b]).view(np.int16)).to("cuda")
            torch.cuda.synchronize()
            r0 = ref_odo.track_batch(tb.data_ptr(), td.data_ptr(), n, want_results=True)
            hf.bgr[:n] = bgr[a:b]
            hf.depth[:n] = dep[a:b]
            r1 = odo.track_batch_host(hf, n=n, want_results=True)
            assert np.array_equal(r0, r1), f"batch [{a}, {b})"
    finally:
        odo.close()
        ref_odo.close()
        hf.close()


def test_sparse_depth_batches_equal_device_path():
    """odo_track_batch_host_sparse_depth: BGR uploaded, depth read in place
    from pinned memory (keypoint pixels only). The depth buffer must stay
    unchanged until the batch finishes, so each batch gets its own pinned
    buffer here; the BGR buffer is refilled right after each call."""
    pkg = load_pkg()
    batches = _batches()
    ref = _device_reference(pkg, batches)
    hfs = [pkg.HostFrames(B, 640, 480) for _ in batches]
    odo = pkg.Odometry(_cfg(pkg))
    try:
        res = None
        for k, (b, d) in enumerate(batches):
            hfs[k].bgr[:] = b
            hfs[k].depth[:] = d
            res = odo.track_batch_host_sparse_depth(hfs[k], want_results=(k == NB - 1))
        _check(odo, res, ref)
    finally:
        odo.close()
        for h in hfs:
            h.close()


def test_host_frames_are_checked():
    """an undersized or wrongly sized HostFrames never reaches the
    C-ABI (which trusts n * W * H bytes)."""
    pkg = load_pkg()
    odo = pkg.Odometry(_cfg(pkg))
    small = pkg.HostFrames(2, 640, 480)
    other = pkg.HostFrames(B, 320, 240)
    try:
        with pytest.raises(ValueError):
            odo.track_batch_host(small, n=3)
        with pytest.raises(ValueError):
            odo.track_batch_host_sparse_depth(small, n=3)
        with pytest.raises(ValueError):
            odo.track_batch_host(other)
        with pytest.raises(ValueError):
            odo.track_batch_host(np.zeros((2, 480, 640, 3), np.uint8), np.zeros((2, 240, 320), np.uint16))
    finally:
        odo.close()
        small.close()
        other.close()


def test_sparse_depth_buffer_is_held_until_read():
    """The depth frames of a sparse-depth batch are read in place: the view is
    read-only (a refill raises) until odo_host_depth_query / _wait release it."""
    pkg = load_pkg()
    b, d = _batches()[0]
    hf = pkg.HostFrames(B, 640, 480)
    odo = pkg.Odometry(_cfg(pkg))
    try:
        hf.bgr[:] = b
        hf.depth[:] = d
        odo.track_batch_host_sparse_depth(hf, want_results=False)
        with pytest.raises(ValueError):
            hf.depth[0, 0, 0] = 1
        hf.bgr[:] = 0  # the BGR frames were consumed when the call returned
        odo.depth_wait()
        assert not odo.depth_busy()
        hf.depth[:] = d
        odo.track_batch_host_sparse_depth(hf, want_results=False)
        odo.synchronize()
        assert hf.depth.flags.writeable
        assert odo.lib.odo_host_depth_query(odo.h) == 0
    finally:
        odo.close()
        hf.close()


def test_host_async_batches_equal_device_path():
    """odo_track_batch_host_async (the frames-mode from-host call): uploads of
    consecutive batches from one pinned buffer, refilled after each call, the
    records streamed into a pinned ring: identical to the device path."""
    pkg = load_pkg()
    batches = _batches()
    ref = _device_reference(pkg, batches)
    hf = pkg.HostFrames(B, 640, 480)
    ring = pkg.PinnedResults(NB, B)
    odo = pkg.Odometry(_cfg(pkg))
    try:
        for k, (b, d) in enumerate(batches):
            hf.bgr[:] = b
            hf.depth[:] = d
            odo.track_batch_host_async(hf, ring, k)
        odo.synchronize()
        _check(odo, ring.all[NB - 1].copy(), ref)
    finally:
        odo.close()
        ring.close()
        hf.close()

"""Frame sizes other than 640x480 (ORBextractor accepts any image): widths
that are not a multiple of 4 (k_gray's per-pixel path, unaligned pitches),
and small images whose upper pyramid levels are narrower than two 30-px FAST
cells (cell ROIs up to 65 px, orbextractor.cpp:688-711). The batched GPU path
against the oracle: keypoints, descriptors, geometry, matches and RANSAC
bit-exact, PnP pose within 1e-4."""
import numpy as np
import pytest

import oracle_lib as O
from conftest import load_pkg, sequence


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(320, 240), (330, 250), (354, 286), (642, 482)])
def test_gpu_frame_sizes(w, h):
    pkg = load_pkg()
    nf, iters, seed = 800, 200, 0x5EED0040
    bgr, dep, _ = sequence(3, w, h, seed=seed)
    cal = O.fr1_calib()
    fr = [O.extract_frame(bgr[i], dep[i], O.orb_params(nf), cal) for i in range(3)]
    cfg = pkg.default_config(w, h, 3, nfeatures=nf, iterations=iters)
    odo = pkg.Odometry(cfg)
    res = odo.track_batch_host(bgr, dep)
    for i in range(3):
        g = odo.frame(i)
        assert len(g["kps"]) == len(fr[i]["kps"]) > 50, f"{w}x{h} frame {i}: N"
        assert np.array_equal(g["kps"], fr[i]["kps"]), f"{w}x{h} frame {i}: keypoints"
        assert np.array_equal(g["desc"], fr[i]["desc"]), f"{w}x{h} frame {i}: descriptors"
        assert np.array_equal(g["kun"], fr[i]["kun"]) and np.array_equal(g["xyz"], fr[i]["xyz"])
    latch = float("nan")
    for p in range(1, 3):
        r, _, matches, latch = O.track_pair(fr[p - 1], fr[p], cal, O.ransac_params(iters),
                                            pkg.pair_seed(cfg.seed, p), latch)
        assert np.array_equal(odo.pair(p)["matches"], matches), f"{w}x{h} pair {p}: matches"
        assert (res[p]["n_matches"], res[p]["n_inliers"], res[p]["visited"], res[p]["n_queries"]) == \
            (r.n_matches, r.n_inliers, r.visited, r.n_queries), f"{w}x{h} pair {p}: counts"
        O.check_ransac_inliers(odo.pair(p), r, f"{w}x{h} pair {p}")
        assert np.array_equal(res[p]["T12"], np.array(r.T12, np.float32)), f"{w}x{h} pair {p}: T12"
        assert np.abs(res[p]["Tcw"] - np.array(r.Tcw, np.float32)).max() < 1e-4, f"{w}x{h} pair {p}: Tcw"
    odo.close()


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,inner", [(330, 250, "fast"), (642, 482, "fast"), (330, 250, "orb"), (642, 482, "orb"),
                                        (1280, 960, "orb")])
def test_gpu_adaptive_frame_sizes(w, h, inner):
    """Extractor(FAST | ORB, ORB, ADAPTIVE) at other sizes: the 3x3 grid's
    cells and edge bands follow the image (videogridadaptedfeaturedetector.cpp:
    62-71); with the cv::ORB inner detector every cell level's size follows
    the cell (odd widths, unaligned cell origins; 1280x960 cells of up to
    489 x 382 px, too large for the LDS cell pyramid, take its L2 variant)."""
    pkg = load_pkg()
    bgr, dep, _ = sequence(4, w, h, seed=0x5EED0041)
    det = pkg.DETECTOR_ADAPTIVE_ORB if inner == "orb" else pkg.DETECTOR_ADAPTIVE_FAST
    cfg = pkg.default_config(w, h, 4, nfeatures=1000, iterations=200, detector=det)
    odo = pkg.Odometry(cfg)
    cal = O.fr1_calib()
    ex = O.AdaptiveExtractor(inner=inner)
    ref = [ex.extract_frame(bgr[i], dep[i], cal) for i in range(4)]
    res = odo.track_batch_host(bgr, dep)
    for i in range(4):
        g = odo.frame(i)
        assert len(g["kps"]) == len(ref[i]["kps"]) > 20, f"{w}x{h} frame {i}: N"
        assert np.array_equal(g["kps"], ref[i]["kps"]) and np.array_equal(g["desc"], ref[i]["desc"]), \
            f"{w}x{h} frame {i}: keypoints / descriptors"
    latch = float("nan")
    for p in range(1, 4):
        r, _, _, latch = O.track_pair(ref[p - 1], ref[p], cal, O.ransac_params(200), pkg.pair_seed(cfg.seed, p), latch)
        assert np.array_equal(res[p]["T12"], np.array(r.T12, np.float32)), f"{w}x{h} pair {p}: T12"
        assert np.abs(res[p]["Tcw"] - np.array(r.Tcw, np.float32)).max() < 1e-4, f"{w}x{h} pair {p}: Tcw"
    odo.close()


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(640, 480), (330, 250), (642, 482), (517, 389)])
def test_gpu_blur_every_frame_and_level(w, h):
    """GaussianBlur 7x7 (orbextractor.cpp:795-796) of every pyramid level of
    every frame, byte for byte against the oracle's blur of the GPU's own
    pyramid (itself pinned by test_pyramid_and_blur_bit_exact): the
    row-strip kernel's interior, its overlapping last chunk and the
    reflect101 border ring at widths that are not multiples of 4 or 16."""
    pkg = load_pkg()
    n = 4
    bgr, dep, _ = sequence(n, w, h, seed=0x5EED0042)
    cfg = pkg.default_config(w, h, n, nfeatures=1000, iterations=50)
    odo = pkg.Odometry(cfg)
    odo.track_batch_host(bgr, dep)
    lw, lh = (O.C.c_int * 8)(), (O.C.c_int * 8)()
    O.lib().oracle_level_sizes(O.C.byref(O.orb_params(1000)), w, h, lw, lh, (O.C.c_float * 8)(), (O.C.c_int * 8)())
    total = sum(a * b for a, b in zip(lw, lh))
    for i in range(n):
        pyr = odo.debug_pyramid(i, total)
        blur = odo.debug_blur(i, total)
        assert pyr.size == blur.size == total
        off = 0
        for l in range(8):
            m = lw[l] * lh[l]
            rb = np.zeros(m, np.uint8)
            O.lib().oracle_blur(O.ptr(np.ascontiguousarray(pyr[off:off + m])), lw[l], lh[l], O.ptr(rb))
            bad = np.nonzero(blur[off:off + m] != rb)[0]
            assert bad.size == 0, f"{w}x{h} frame {i} level {l}: {bad.size} px differ, first (y, x) " \
                                  f"{divmod(int(bad[0]), lw[l])}"
            off += m
    odo.close()


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(640, 480), (330, 250), (642, 482), (517, 389), (1280, 960), (320, 240)])
def test_gpu_pyramid_forms_every_frame(w, h):
    """ComputePyramid (orbextractor.cpp:833-857) and the 7x7 GaussianBlur of
    every level (:795-796) through the three kernel forms, the one-launch
    k_pyramid with its blur (a workgroup per frame: every level, then each
    level's blur once it is complete), the same without the blur (k_blur_rows
    launch after it) and the k_gray + per-level k_resize chain, for every
    frame of a batch, byte for byte against the oracle's pyramid of the frame
    (cv::resize INTER_LINEAR restated) and the oracle's blur of it: widths
    that are not multiples of 4 (k_gray's per-pixel path), quads whose taps
    reach the row's last byte, 1280x960 (levels up to 320 quads wide), and
    320x240 (levels under 30 rows: the LDS-tiled blur)."""
    pkg = load_pkg()
    n = 5
    bgr, dep, _ = sequence(n, w, h, seed=0x5EED0043)
    lw, lh = (O.C.c_int * 8)(), (O.C.c_int * 8)()
    O.lib().oracle_level_sizes(O.C.byref(O.orb_params(1000)), w, h, lw, lh, (O.C.c_float * 8)(), (O.C.c_int * 8)())
    total = sum(a * b for a, b in zip(lw, lh))
    refs, blurs = [], []
    for i in range(n):
        ref = np.zeros(total, np.uint8)
        O.lib().oracle_pyramid(O.ptr(O.gray(bgr[i])), w, h, O.C.byref(O.orb_params(1000)), O.ptr(ref))
        refs.append(ref)
        rb, off = np.zeros(total, np.uint8), 0
        for l in range(8):
            m = lw[l] * lh[l]
            part = np.zeros(m, np.uint8)
            O.lib().oracle_blur(O.ptr(np.ascontiguousarray(ref[off:off + m])), lw[l], lh[l], O.ptr(part))
            rb[off:off + m] = part
            off += m
        blurs.append(rb)
    for form in (pkg.PYRAMID_FORM_FUSED, pkg.PYRAMID_FORM_FUSED_NOBLUR, pkg.PYRAMID_FORM_CHAIN):
        cfg = pkg.default_config(w, h, n, nfeatures=1000, iterations=50, forms={"pyramid": form})
        odo = pkg.Odometry(cfg)
        odo.track_batch_host(bgr, dep)
        for i in range(n):
            got = odo.debug_pyramid(i, total)
            bad = np.nonzero(got != refs[i])[0]
            assert bad.size == 0, f"{w}x{h} form {form} frame {i}: {bad.size} px differ, first at {bad[:4]}"
            got = odo.debug_blur(i, total)
            bad = np.nonzero(got != blurs[i])[0]
            assert bad.size == 0, f"{w}x{h} form {form} frame {i}: {bad.size} blurred px differ, first at {bad[:4]}"
        odo.close()

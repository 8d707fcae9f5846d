"""GPU ORB (mcs_orb_detect_host) vs its CPU restatement: the same keypoints (level, position,
order), responses, and bit-identical descriptors; BGR input through OpenCV's gray formula; and
the full GPU estimation chain ORB -> Hamming kNN-2 -> ratio -> RANSAC on a warped scene."""
import numpy as np
import pytest

from oracle import oracle
from multicamera_stitching_amd import rig

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("h,w,nf,nl", [(480, 640, 500, 8), (1080, 1920, 2000, 8),
                                       (300, 200, 300, 4), (240, 320, 100, 1)])
def test_orb_vs_oracle(h, w, nf, nl):
    from multicamera_stitching_amd import _capi
    img = rig.corner_texture(h, w, seed=h + w)
    got = _capi.orb_detect(img, nfeatures=nf, nlevels=nl)
    want = oracle.orb_detect(img, nfeatures=nf, nlevels=nl)
    assert len(got["xy"]) == len(want["xy"]) > 0
    assert np.array_equal(got["level"], want["level"])
    assert np.array_equal(got["xy"], want["xy"])
    assert np.array_equal(got["response"], want["response"].astype(np.float32))
    assert np.array_equal(got["desc"], want["desc"])
    ang = np.rad2deg(np.arctan2(want["cs_sn"][:, 1], want["cs_sn"][:, 0])) % 360
    assert np.allclose(got["angle"], ang, atol=1e-3)


@pytest.mark.parametrize("kind", ["noise", "blocks4", "blocks8"])
def test_orb_dense_candidates_vs_oracle(kind):
    """Many candidates per level: pixel noise puts more than kOrbSelMax (4096) on level 0 (the
    host ranks every level), blocky noise a few thousand (the device's bitonic ranking, with
    ties in response broken by position)."""
    from multicamera_stitching_amd import _capi
    rng = np.random.default_rng(7)
    if kind == "noise":
        img = rng.integers(0, 256, (480, 640), dtype=np.uint8)
    else:
        b = int(kind[-1])
        img = np.kron(rng.integers(0, 256, (480 // b, 640 // b)), np.ones((b, b))).astype(np.uint8)
    got = _capi.orb_detect(img, nfeatures=1500, nlevels=8)
    want = oracle.orb_detect(img, nfeatures=1500, nlevels=8)
    assert len(got["xy"]) == len(want["xy"]) > 0
    assert np.array_equal(got["level"], want["level"])
    assert np.array_equal(got["xy"], want["xy"])
    assert np.array_equal(got["response"], want["response"].astype(np.float32))
    assert np.array_equal(got["desc"], want["desc"])


def test_orb_bgr_input_uses_opencv_gray():
    from multicamera_stitching_amd import _capi
    rng = np.random.default_rng(3)
    bgr = rng.integers(0, 256, (200, 240, 3), dtype=np.uint8)
    bgr[50:150, 60:180] = [30, 200, 90]
    g = ((bgr[..., 0].astype(np.int32) * 1868 + bgr[..., 1].astype(np.int32) * 9617 +
          bgr[..., 2].astype(np.int32) * 4899 + 8192) >> 14).astype(np.uint8)
    a = _capi.orb_detect(bgr, nfeatures=200, nlevels=3)
    b = _capi.orb_detect(g, nfeatures=200, nlevels=3)
    assert np.array_equal(a["xy"], b["xy"]) and np.array_equal(a["desc"], b["desc"])


def test_gpu_estimation_chain_recovers_motion():
    from multicamera_stitching_amd import _capi
    from multicamera_stitching_amd.features import ratio_matches
    img = rig.corner_texture(720, 1280, seed=5)
    th = np.deg2rad(-5.0)
    Ht = np.array([[np.cos(th), -np.sin(th), -40.0], [np.sin(th), np.cos(th), 25.0],
                   [1e-5, 0, 1]])
    warped = oracle.warp_perspective(img, Ht, (1280, 720))
    a, b = _capi.orb_detect(img, 2000), _capi.orb_detect(warped, 2000)
    idx, dist = _capi.match_hamming_knn2(a["desc"], b["desc"])
    m = ratio_matches(idx, dist)
    src = np.float32([a["xy"][q] for (_, q) in m])
    dst = np.float32([b["xy"][t] for (t, _) in m])
    H, mask = _capi.ransac_homography(src, dst, 3.0)
    assert H is not None and mask.sum() > 100
    g = np.c_[np.random.default_rng(0).uniform(200, 600, (20, 2)), np.ones(20)]
    p, q = g @ H.T, g @ Ht.T
    assert np.abs(p[:, :2] / p[:, 2:] - q[:, :2] / q[:, 2:]).max() < 2.0


def test_dropin_calibrates_with_gpu_orb_backend(monkeypatch):
    """No OpenCV: Stitcher.calibrate_stitcher estimates each stage's homography with the GPU
    ORB -> Hamming -> ratio -> RANSAC path (the reference's detectAndDescribe/matchKeypoints
    roles), then stitches the captures."""
    from multicamera_stitching_amd import features
    from multicamera_stitching_amd.StitcherClass import Stitcher
    monkeypatch.setenv("MCS_FEATURES", "orb")
    assert features.backend() == "orb"
    world = rig.corner_texture(600, 1500, seed=7)
    w = 640
    cams = [np.ascontiguousarray(world[50:530, x:x + w]) for x in (0, 420, 840)]
    images = dict(zip(["CAM1", "CAM2", "CAM3"], cams))
    st = Stitcher(images)
    st.calibrate_stitcher(images, save=False)
    assert all(sb.cachedAH is not None for sb in st.stitchers)
    out = st.stitch(images)
    assert out.shape[0] >= 480 and out.shape[1] >= 1400
    # the mosaic reproduces the world strip (paste of camera 1 over exact warps of the others)
    y0 = st.stitchers[1].Bpts[0][1] if st.stitchers[1].Bpts else 0
    ref = world[50:530, :out.shape[1]].astype(np.int16)
    crop = out[y0:y0 + 480, :ref.shape[1]].astype(np.int16)
    if crop.ndim == 3:
        crop = crop[..., 0]
    err = np.abs(crop[:, 700:1300] - ref[:, 700:1300])
    assert np.median(err) <= 2


def test_orb_match_ransac_concurrent_threads_match_serial():
    """The per-frame entry points from several host threads at once (each thread has its own
    stream and device workspace in libmcs) give the serial results, call after call."""
    from concurrent.futures import ThreadPoolExecutor
    from multicamera_stitching_amd import _capi
    imgs = [rig.corner_texture(540, 960, seed=s) for s in range(4)]
    want = [_capi.orb_detect(im, 800) for im in imgs]
    want_m = [_capi.match_hamming_knn2(want[k]["desc"], want[k - 1]["desc"]) for k in (1, 2, 3)]
    with ThreadPoolExecutor(4) as ex:
        for _ in range(3):
            got = list(ex.map(lambda im: _capi.orb_detect(im, 800), imgs))
            for g, w in zip(got, want):
                assert np.array_equal(g["xy"], w["xy"]) and np.array_equal(g["desc"], w["desc"])
            got_m = list(ex.map(lambda k: _capi.match_hamming_knn2(got[k]["desc"],
                                                                   got[k - 1]["desc"]), (1, 2, 3)))
            for (gi, gd), (wi, wd) in zip(got_m, want_m):
                assert np.array_equal(gi, wi) and np.array_equal(gd, wd)

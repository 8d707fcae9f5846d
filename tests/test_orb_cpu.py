"""ORB restatement (oracle/orc_orb.c, spec csrc/mcs_orb_core.h): quotas, borders, ordering, and
that descriptors of the same scene point agree across a known warp so that the GPU matching +
RANSAC path recovers the homography (the per-frame estimation chain of SURVEY.md 8 C3)."""
import numpy as np

from oracle import oracle
from multicamera_stitching_amd import rig


def test_pattern_table_is_opencv_bit_pattern_31():
    pat = oracle.orb_pattern()
    assert pat.shape == (256, 4) and pat[0].tolist() == [8, -3, 9, 5]
    assert pat[1].tolist() == [4, 2, 7, -12] and np.abs(pat).max() <= 15


def test_quota_border_and_order():
    img = rig.corner_texture(480, 640, seed=1)
    r = oracle.orb_detect(img, nfeatures=500)
    n = len(r["xy"])
    assert 0 < n <= 500
    lv = r["level"]
    assert (np.diff(lv) >= 0).all()                       # levels in order
    for level in np.unique(lv):
        resp = r["response"][lv == level]
        assert (np.diff(resp) <= 0).all()                  # best first within a level
    scale = np.float32(1.2) ** lv.astype(np.float32)
    x = r["xy"][:, 0] / scale
    assert (x >= 31 - 1e-3).all()
    cs = r["cs_sn"]
    assert np.allclose((cs ** 2).sum(1), 1.0)


def test_warped_scene_matches_back():
    """Scene + a shifted/rotated copy: ORB + Hamming kNN-2 + ratio + RANSAC recover the motion."""
    from multicamera_stitching_amd.features import ratio_matches
    img = rig.corner_texture(480, 640, seed=2)
    th = np.deg2rad(7.0)
    Ht = np.array([[np.cos(th), -np.sin(th), 30.0], [np.sin(th), np.cos(th), -12.0], [0, 0, 1]])
    warped = oracle.warp_perspective(img, Ht, (640, 480))
    a, b = oracle.orb_detect(img, 1500), oracle.orb_detect(warped, 1500)
    idx, dist = oracle.hamming_knn2(a["desc"], b["desc"])
    m = ratio_matches(idx, dist)
    assert len(m) > 50
    src = np.float32([a["xy"][q] for (_, q) in m])
    dst = np.float32([b["xy"][t] for (t, _) in m])
    H, mask, best, _ = oracle.ransac_homography(src, dst, 3.0)
    assert H is not None and mask.sum() > 40
    g = np.c_[np.random.default_rng(0).uniform(100, 500, (20, 2)), np.ones(20)]
    p, q = g @ H.T, g @ Ht.T
    assert np.abs(p[:, :2] / p[:, 2:] - q[:, :2] / q[:, 2:]).max() < 2.0

"""GPU float-L2 kNN-2 (BFMatcher(NORM_L2).knnMatch(k=2) of the reference's SIFT
matching, StitcherClass.py:423-424) vs oracle/orc_match.c.  Integer-valued descriptors in
[0, 255] (what OpenCV's SIFT emits) take the exact int8-MFMA path: indices and float distances
identical to OpenCV's own (its float sums are exact for such data).  Arbitrary floats take the
f32-MFMA path: distances within 1e-4 relative of the double-precision truth, and the returned
neighbours are true nearest neighbours up to that tolerance."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _sift_like(rng, n, dim=128, base=None, noise=0):
    if base is None:
        return rng.integers(0, 256, (n, dim)).astype(np.float32)
    x = base[rng.integers(0, len(base), n)] + rng.integers(-noise, noise + 1, (n, dim))
    return np.clip(x, 0, 255).astype(np.float32)


@pytest.mark.parametrize("nq,nt,dim", [(1, 1, 128), (17, 2, 128), (300, 700, 128),
                                       (2000, 2500, 128), (70, 90, 64), (33, 41, 200),
                                       (5, 3, 1), (129, 1000, 256)])
def test_l2_exact_path_vs_oracle(nq, nt, dim):
    from multicamera_stitching_amd import _capi
    rng = np.random.default_rng(nq * 7 + nt)
    t = _sift_like(rng, nt, dim)
    q = _sift_like(rng, nq, dim, base=t, noise=6)      # near duplicates: small distances
    idx, dist, exact = _capi.match_l2_knn2(q, t)
    widx, wdist, wexact = oracle.l2_knn2(q, t)
    assert exact and wexact
    assert np.array_equal(idx, widx)
    assert np.array_equal(dist.view(np.uint32), wdist.view(np.uint32))


def test_l2_exact_ties_order_by_index():
    """Duplicate train descriptors: equal distances, OpenCV keeps the lower train index first."""
    from multicamera_stitching_amd import _capi
    rng = np.random.default_rng(1)
    t = _sift_like(rng, 40, 128)
    t[25] = t[7]
    t[31] = t[7]
    q = t[[7, 25, 3]].copy()
    idx, dist, exact = _capi.match_l2_knn2(q, t)
    assert exact
    assert idx[0].tolist() == [7, 25] and idx[1].tolist() == [7, 25]
    assert dist[0].tolist() == [0.0, 0.0]
    assert np.array_equal(idx, oracle.l2_knn2(q, t)[0])


def test_l2_float_path_tolerance():
    from multicamera_stitching_amd import _capi
    rng = np.random.default_rng(2)
    t = rng.standard_normal((600, 128)).astype(np.float32)
    q = (t[rng.integers(0, 600, 200)] + 0.05 * rng.standard_normal((200, 128))).astype(np.float32)
    idx, dist, exact = _capi.match_l2_knn2(q, t)
    assert not exact
    true = np.sqrt(((q[:, None, :].astype(np.float64) - t[None]) ** 2).sum(-1))
    srt = np.sort(true, axis=1)[:, :2]
    got_true = np.take_along_axis(true, idx.astype(np.int64), 1)
    assert np.allclose(got_true, srt, rtol=1e-4, atol=1e-4)        # true nearest two
    assert np.allclose(dist, got_true, rtol=1e-4, atol=1e-3)        # their distances


def test_l2_single_train_and_empty():
    from multicamera_stitching_amd import _capi
    rng = np.random.default_rng(3)
    q = _sift_like(rng, 4)
    idx, dist, _ = _capi.match_l2_knn2(q, q[:1])
    assert (idx[:, 1] == -1).all() and (dist[:, 1] == -1).all() and (idx[:, 0] == 0).all()
    idx, dist, _ = _capi.match_l2_knn2(q, np.zeros((0, 128), np.float32))
    assert (idx == -1).all()


def test_sift_style_calibration_matching_end_to_end():
    """features.match_keypoints with float descriptors (the reference's SIFT path) runs the GPU
    L2 matcher + ratio test: the homography of a shifted keypoint set is recovered."""
    from multicamera_stitching_amd import features
    rng = np.random.default_rng(4)
    n = 400
    desc = _sift_like(rng, n)
    kpsB = rng.uniform(0, 600, (n, 2)).astype(np.float32)
    kpsA = kpsB + np.float32([120.0, -7.0])
    perm = rng.permutation(n)
    featuresA, featuresB = desc[perm], desc.copy()
    kA = kpsA[perm]
    cv2 = features._cv2()
    if cv2 is None:   # no OpenCV here: check the matching half (the reference's RANSAC is cv2's)
        from multicamera_stitching_amd import _capi
        idx, dist, exact = _capi.match_l2_knn2(featuresA, featuresB)
        m = features.ratio_matches(idx, dist)
        assert exact and len(m) == n
        assert all(perm[q] == t for (t, q) in m)
        return
    H, matches, status = features.match_keypoints(None, kA, kpsB, featuresA, featuresB)
    assert H is not None and np.allclose(H[:2, 2], [-120.0, 7.0], atol=0.5)

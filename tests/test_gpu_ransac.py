"""GPU RANSAC homography (mcs_ransac_homography_host) vs its CPU restatement: the same best
hypothesis, the same inlier mask, the same refit H (FP64, identical operation order)."""
import numpy as np
import pytest

from oracle import oracle
from test_ransac_cpu import max_reproj_diff, synthetic

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,outliers,seed", [(600, 0.3, 0), (50, 0.5, 1), (5000, 0.2, 2),
                                              (8, 0.0, 3), (2000, 0.7, 4)])
def test_ransac_vs_oracle(n, outliers, seed):
    from multicamera_stitching_amd import _capi
    src, dst, Ht, out = synthetic(n=n, outliers=outliers, seed=seed)
    H, mask = _capi.ransac_homography(src, dst, 3.0, iters=2000, seed=seed)
    Hw, maskw, best, _ = oracle.ransac_homography(src, dst, 3.0, iters=2000, seed=seed)
    assert (H is None) == (Hw is None)
    assert np.array_equal(mask.reshape(-1), maskw)
    if H is not None:
        assert np.allclose(H, Hw, rtol=1e-12, atol=1e-12)
        if n >= 50:
            assert max_reproj_diff(H, Ht) < 2.0


def test_ransac_no_model():
    from multicamera_stitching_amd import _capi
    H, mask = _capi.ransac_homography(np.zeros((3, 2)), np.zeros((3, 2)), 3.0)
    assert H is None and mask.shape == (3, 1) and not mask.any()

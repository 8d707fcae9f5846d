"""GPU Hamming kNN-2 (mcs_match_hamming_knn2) vs the CPU restatement: exact indices and
distances, OpenCV's tie order, ragged sizes, device-pointer and host entry points."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _desc(rng, n):
    return rng.integers(0, 256, (n, 32), dtype=np.uint8)


@pytest.mark.parametrize("nq,nt", [(1, 2), (63, 3), (64, 300), (65, 257), (2000, 2000),
                                   (5000, 700), (10, 0), (10, 1), (129, 4096)])
def test_knn2_vs_oracle(nq, nt):
    from multicamera_stitching_amd import _capi
    rng = np.random.default_rng(nq * 31 + nt)
    q, t = _desc(rng, nq), _desc(rng, nt)
    idx, dist = _capi.match_hamming_knn2(q, t)
    widx, wdist = oracle.hamming_knn2(q, t)
    assert np.array_equal(idx, widx) and np.array_equal(dist, wdist)


def test_knn2_ties_take_lowest_train_index():
    """Duplicated train descriptors spread over several train chunks: equal distances must rank
    by train index across the chunk merge."""
    from multicamera_stitching_amd import _capi
    rng = np.random.default_rng(5)
    base = _desc(rng, 16)
    t = base[rng.integers(0, 16, 5000)]
    q = np.concatenate([base, base ^ np.uint8(1), _desc(rng, 100)])
    idx, dist = _capi.match_hamming_knn2(q, t)
    widx, wdist = oracle.hamming_knn2(q, t)
    assert np.array_equal(dist, wdist) and np.array_equal(idx, widx)


def test_knn2_device_pointers_on_stream():
    import torch
    from multicamera_stitching_amd import _capi
    rng = np.random.default_rng(9)
    q, t = _desc(rng, 777), _desc(rng, 1500)
    dq, dt = torch.from_numpy(q).cuda(), torch.from_numpy(t).cuda()
    di = torch.empty((777, 2), dtype=torch.int32, device="cuda")
    dd = torch.empty_like(di)
    s = torch.cuda.Stream()
    _capi.match_hamming_knn2_device(dq.data_ptr(), 777, dt.data_ptr(), 1500, di.data_ptr(),
                                    dd.data_ptr(), 0, s.cuda_stream)
    s.synchronize()
    widx, wdist = oracle.hamming_knn2(q, t)
    assert np.array_equal(di.cpu().numpy(), widx) and np.array_equal(dd.cpu().numpy(), wdist)

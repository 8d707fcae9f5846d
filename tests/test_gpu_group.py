"""The multi-GPU boundary (mcs_group_*, include/mcs.h) on one GPU: a one-rank RCCL group is
created from a fresh unique id and its gather delivers the rank's own mosaics into the
receive buffer (the root's device copy); argument errors are refused.  (More ranks need more
GPUs: the driver's 8-GPU bench gathers every rank's mosaics through it and verifies them.)"""
import pytest

pytestmark = pytest.mark.gpu


def test_single_rank_group_gather():
    import torch
    from multicamera_stitching_amd import _capi
    uid = _capi.Group.unique_id()
    assert len(uid) == _capi.MCS_GROUP_ID_BYTES
    g = _capi.Group(1, 0, uid, 0)
    try:
        src = torch.randint(0, 256, (3, 100, 301), dtype=torch.uint8, device="cuda:0")
        recv = torch.zeros((1, 3, 100, 301), dtype=torch.uint8, device="cuda:0")
        s = torch.cuda.current_stream().cuda_stream
        g.gather(src.data_ptr(), src.numel(), recv.data_ptr(), 0, s)
        torch.cuda.synchronize()
        assert torch.equal(recv[0], src)
        with pytest.raises(_capi.McsError):
            g.gather(src.data_ptr(), src.numel(), recv.data_ptr(), 1, s)   # root outside group
    finally:
        g.close()
    assert _capi.rccl_library()
    with pytest.raises(_capi.McsError):
        _capi.Group(2, 2, uid, 0)                                          # rank outside group

"""Config 3's per-capture chain geometry in libmcs (mcs_chain_stages, csrc/mcs_chain.cpp: the
geometry the rig job's wait_stitch builds its plan from) against its Python restatement
(estimate.chain_stages, plain FP64 floats in the same order): every stage descriptor field equal,
the homographies bit for bit, over rigs with random pair homographies, super mode on and off,
failed pairs and cameras of different sizes.  Host arithmetic only (no GPU)."""
import numpy as np
import pytest

from multicamera_stitching_amd import _capi, estimate, rig
from multicamera_stitching_amd.StitcherClass import _stage_desc


def _fields(d):
    return (list(d.H), d.calibrated, d.canvas_w, d.canvas_h, d.b_x, d.b_y, d.b_w, d.b_h, d.a_w,
            d.a_h, d.super_mode, d.x_lim0, d.x_lim1, d.y_lim0, d.y_lim1)


def _check(pair, shapes, super_mode):
    ok = [H is not None for H in pair]
    Hs = np.stack([np.asarray(H, np.float64).reshape(9) if H is not None else np.zeros(9)
                   for H in pair])
    got = _capi.chain_stages(Hs, ok, shapes, super_mode)
    want = [_stage_desc(sb) for sb in estimate.chain_stages(pair, shapes, super_mode)]
    assert len(got) == len(want)
    for g, w in zip(got, want):
        gf, wf = _fields(g), _fields(w)
        if not w.calibrated:
            assert g.calibrated == 0
            continue
        # (super-mode limits only count in super mode: the descriptor leaves them 0 otherwise)
        if not super_mode:
            gf, wf = gf[:11], wf[:11]
        assert np.array_equal(np.array(gf[0]).view(np.uint64), np.array(wf[0]).view(np.uint64))
        assert gf[1:] == wf[1:]


@pytest.mark.parametrize("super_mode", [False, True])
@pytest.mark.parametrize("seed", range(12))
def test_chain_stages_c_equals_python(seed, super_mode):
    n, w, h = 4 + seed % 3, 1920, 1080
    C = rig.camera_models(n, w, h, seed=seed, rot_deg=1.0 + seed % 4, persp=2e-5 * (seed % 3))
    rng = np.random.default_rng(seed)
    # estimation noise on the pair homographies (per-capture RANSAC + LM output)
    pair = [np.linalg.inv(C[k]) @ C[k + 1] @ (np.eye(3) + rng.normal(scale=1e-4, size=(3, 3)))
            for k in range(n - 1)]
    _check(pair, [(h, w, 3)] * n, super_mode)


def test_chain_stages_c_failed_pair_and_mixed_sizes():
    C = rig.camera_models(4, 640, 360, seed=3)
    pair = [np.linalg.inv(C[k]) @ C[k + 1] for k in range(3)]
    shapes = [(360, 640, 3), (360, 640, 3), (300, 500, 3), (360, 640, 3)]
    _check(pair, shapes, False)
    _check([pair[0], None, pair[2]], shapes, False)
    _check([None, pair[1], pair[2]], shapes, True)


def test_chain_stages_c_rejects_bad_input():
    with pytest.raises(_capi.McsError):
        _capi.chain_stages(np.zeros((1, 9)), [1], [(10, 0, 3), (10, 10, 3)])
    # a homography sending a corner to infinity (w = 0 at a corner)
    bad = np.array([[1.0, 0, 0], [0, 1.0, 0], [-1.0 / 10, 0, 1.0]]).reshape(1, 9)
    with pytest.raises(_capi.McsError):
        _capi.chain_stages(bad, [1], [(10, 10, 3), (10, 10, 3)])

"""GPU blended stitch modes (SURVEY.md 8 NS-1 multi-band, NS-2 feather) vs their CPU
restatement oracle/orc_blend.c.  No reference implementation exists (the reference pastes), so
the bar is our own specification: bit-exact (the north star allows 1 LSB for float blends; the
integer pyramids and IEEE-double blend reproduce the restatement exactly)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

MODES = {"feather": 1, "multiband": 2}


def _world_plan(n, w, h, ch, seed, interp=1, super_mode=False, **kw):
    from multicamera_stitching_amd import rig, _capi
    from multicamera_stitching_amd.StitcherClass import Stitcher, _stage_desc
    C = rig.camera_models(n, w, h, seed=seed, **kw)
    frames = rig.world_frames(C, w, h, ch, seed=seed)
    images = dict(zip(rig.labels(n), frames))
    st = Stitcher(images, super_mode=super_mode)
    st.calibrate_stitcher(images, save=False,
                          homographies=rig.homography_provider(C, lambda: st.stitchers))
    cams = [images[label] for label in st.img_labels]
    plan = _capi.Plan([_stage_desc(sb) for sb in st.stitchers], w, h, ch, interp)
    return plan, cams


def _diff(a, b):
    return int(np.abs(a.astype(np.int16) - b.astype(np.int16)).max()) if a.size else 0


@pytest.mark.parametrize("mode", ["feather", "multiband"])
@pytest.mark.parametrize("case", [
    dict(n=4, w=320, h=180, ch=3, seed=3),
    dict(n=3, w=200, h=120, ch=1, seed=4, rot_deg=4.0, persp=1e-4),
    dict(n=2, w=150, h=90, ch=4, seed=5, rot_deg=2.0),
    dict(n=3, w=160, h=100, ch=3, seed=6, interp=0),
    dict(n=3, w=180, h=100, ch=3, seed=7, super_mode=True, rot_deg=3.0),
    dict(n=2, w=40, h=20, ch=2, seed=8, overlap=0.5),
    dict(n=4, w=64, h=48, ch=3, seed=10, overlap=0.8),     # seams 13 px apart: 3-4 owners/tile
])
def test_blend_vs_oracle(mode, case):
    case = dict(case)
    interp = case.pop("interp", 1)
    plan, cams = _world_plan(interp=interp, **case)
    plan.set_blend(MODES[mode])
    got = plan.stitch_host(cams)
    want = oracle.blend_stitch(plan.describe(), cams, MODES[mode], interp)
    assert _diff(got.reshape(want.shape), want) == 0
    st = plan.stats()
    assert st["blend"] == MODES[mode] and st["blend_tiles"] > 0


def test_multiband_c2_full_size_batch():
    """Config 2 at full size (4 x 1920x1080, multi-band), a device batch of 3 captures."""
    import torch
    from multicamera_stitching_amd import rig
    plan, cams = _world_plan(4, 1920, 1080, 3, seed=0)
    plan.set_blend(MODES["multiband"])
    F = 3
    shots = [[np.roll(c, 7 * f, axis=0) for c in cams] for f in range(F)]
    dev = [torch.from_numpy(np.stack([shots[f][i] for f in range(F)])).cuda()
           for i in range(len(cams))]
    out = torch.zeros((F, plan.out_h, plan.out_w * 3), dtype=torch.uint8, device="cuda")
    plan.stitch_device([d.data_ptr() for d in dev], [d[0].numel() for d in dev],
                       out.data_ptr(), plan.out_w * 3, out[0].numel(), F, 0)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for f in (0, F - 1):
        want = oracle.blend_stitch(plan.describe(), shots[f], MODES["multiband"])
        assert _diff(got[f].reshape(want.shape), want) == 0


def test_blend_mode_switch_back_to_paste():
    plan, cams = _world_plan(3, 120, 80, 3, seed=9)
    paste = plan.stitch_host(cams)
    plan.set_blend(MODES["multiband"])
    mb = plan.stitch_host(cams)
    plan.set_blend(0)
    assert _diff(plan.stitch_host(cams), paste) == 0
    assert _diff(mb, paste) > 0


def test_multiband_more_than_four_owners_is_refused():
    """Five cameras 6 px apart put five owners into one 64 x 64 neighbourhood: the multi-band
    kernel holds four, so prepare fails loudly (MCS_E_UNSUPPORTED) instead of mis-blending."""
    from multicamera_stitching_amd import _capi
    plan, cams = _world_plan(5, 40, 30, 3, seed=11, overlap=0.85)
    plan.set_blend(MODES["multiband"])
    with pytest.raises(_capi.McsError) as e:
        plan.stitch_host(cams)
    assert e.value.code == _capi.MCS_E_UNSUPPORTED
    plan.set_blend(MODES["feather"])          # feather has no such limit
    want = oracle.blend_stitch(plan.describe(), cams, MODES["feather"])
    assert _diff(plan.stitch_host(cams).reshape(want.shape), want) == 0

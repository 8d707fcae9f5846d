"""GPU cylindrical panorama (8 cameras at 45 degree yaw steps, f = 1100)
vs its CPU restatement oracle/orc_blend.c orc_blend_stitch_cyl.  The reference has no
cylindrical path (it chains homographies); the specification is ours (include/mcs.h
mcs_plan_create_cylindrical), and the bar is bit-exact."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

MODES = {"seam": 3, "feather": 1, "multiband": 2}


def _rig(n, w, h, f, ch, seed, interp=1, **kw):
    from multicamera_stitching_amd import rig, _capi
    cams, frames, g = rig.cylinder_rig(n, w, h, f, ch, seed=seed, **kw)
    plan = _capi.Plan.cylindrical(cams, g["out_w"], g["out_h"], g["f_cyl"], g["u0"], g["v0"],
                                  ch, interp)
    return plan, cams, frames, g


def _want(cams, frames, g, mode, interp=1):
    return oracle.blend_stitch_cyl(cams, g["out_w"], g["out_h"], g["f_cyl"], g["u0"], g["v0"],
                                   frames, mode, interp)


def _diff(a, b):
    return int(np.abs(a.astype(np.int16) - b.astype(np.int16)).max()) if a.size else 0


@pytest.mark.parametrize("mode", ["seam", "feather", "multiband"])
@pytest.mark.parametrize("case", [
    dict(n=8, w=320, h=180, f=185.0, ch=3, seed=1),
    dict(n=8, w=320, h=180, f=185.0, ch=3, seed=2, jitter_deg=2.0),
    dict(n=6, w=200, h=150, f=120.0, ch=1, seed=3, jitter_deg=1.0),
    dict(n=5, w=160, h=120, f=90.0, ch=4, seed=4, interp=0, jitter_deg=1.0),
    dict(n=4, w=128, h=96, f=70.0, ch=2, seed=5),
    dict(n=3, w=96, h=64, f=60.0, ch=3, seed=6),            # gaps between cameras: uncovered
])
def test_cylinder_vs_oracle(mode, case, mb_path):
    if mode != "multiband" and mb_path == "bands":
        pytest.skip("one path")
    case = dict(case)
    interp = case.pop("interp", 1)
    plan, cams, frames, g = _rig(interp=interp, **case)
    plan.set_blend(MODES[mode])
    got = plan.stitch_host(frames)
    want = _want(cams, frames, g, MODES[mode], interp)
    assert _diff(got.reshape(want.shape), want) == 0


def test_cylinder_c4_full_size_batch(mb_path):
    """C4 at full size (8 x 1920x1080, f = 1100 -> 6912 x 1080 panorama, multi-band), a device
    batch of 2 captures checked against the restatement."""
    import torch
    plan, cams, frames, g = _rig(8, 1920, 1080, 1100.0, 3, seed=0, jitter_deg=0.5)
    assert (plan.out_w, plan.out_h) == (6912, 1080)
    F = 2
    shots = [[np.roll(c, 5 * f, axis=1) for c in frames] for f in range(F)]
    dev = [torch.from_numpy(np.stack([shots[f][i] for f in range(F)])).cuda()
           for i in range(len(frames))]
    out = torch.zeros((F, plan.out_h, plan.out_w * 3), dtype=torch.uint8, device="cuda")
    plan.stitch_device([d.data_ptr() for d in dev], [d[0].numel() for d in dev],
                       out.data_ptr(), plan.out_w * 3, out[0].numel(), F, 0)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for f in range(F):
        want = _want(cams, shots[f], g, MODES["multiband"])
        assert _diff(got[f].reshape(want.shape), want) == 0
    st = plan.stats()
    assert st["blend_tiles"] > 0 and st["tiles"] > 0


def test_cylinder_stream_pipeline():
    """The host streaming pipeline (mcs_stream_*) over a cylindrical plan."""
    from multicamera_stitching_amd import _capi
    plan, cams, frames, g = _rig(8, 320, 180, 185.0, 3, seed=7)
    want = _want(cams, frames, g, MODES["multiband"])
    sp = _capi.StreamPipeline(plan, 2, True)
    try:
        s0, s1 = sp.submit(frames), sp.submit(frames)
        assert _diff(sp.wait(s0).reshape(want.shape), want) == 0
        s2 = sp.submit(frames)
        for s in (s1, s2):
            assert _diff(sp.wait(s).reshape(want.shape), want) == 0
    finally:
        sp.close()

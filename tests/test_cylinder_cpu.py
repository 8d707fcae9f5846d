"""Cylindrical rig on the CPU: the oracle's geometry against the world
the synthetic rig was rendered from, the modes' relations, and the plan boundary's argument
checks (plan creation is host-only: no GPU needed)."""
import numpy as np
import pytest

from multicamera_stitching_amd import rig
from oracle import oracle


def _pano(cams, frames, g, mode, interp=1, want_owner=False):
    return oracle.blend_stitch_cyl(cams, g["out_w"], g["out_h"], g["f_cyl"], g["u0"], g["v0"],
                                   frames, mode, interp, want_owner=want_owner)


def test_rig_geometry_c4():
    cams, _, g = rig.cylinder_rig(8, 64, 36, 1100.0 * 64 / 1920, 3, seed=0)
    full = rig.cylinder_rig.__defaults__
    assert full[:3] == (8, 1920, 1080) and full[3] == 1100.0
    assert g["out_w"] == int(round(2 * np.pi * g["f_cyl"]))
    for k, c in enumerate(cams):   # camera k looks along yaw 2 pi k / 8
        fwd = c["R"].T @ np.array([0.0, 0.0, 1.0])
        assert np.allclose(fwd, [np.sin(np.pi * k / 4), 0, np.cos(np.pi * k / 4)])
        assert np.allclose(c["R"] @ c["R"].T, np.eye(3))


def test_seam_panorama_reproduces_the_world():
    """With equal gains the seam panorama is the world texture the cameras were rendered from,
    up to the two bilinear resamplings."""
    cams, frames, g = rig.cylinder_rig(8, 320, 180, 185.0, 3, seed=1, gain=0.0)
    out, own = _pano(cams, frames, g, oracle.BLEND_SEAM, want_owner=True)
    world = rig.texture(g["out_h"] + 96, g["out_w"] + 96, 3, seed=1)
    ref = world[48:48 + g["out_h"], 48:48 + g["out_w"]]
    m = own != 255
    assert m.mean() > 0.95
    d = np.abs(out.astype(int) - ref.astype(int))[m]
    assert d.mean() < 4.0 and np.percentile(d, 99) <= 16
    # the owner of the centre column of camera k's view is camera k
    for k in range(8):
        u = int(round(g["u0"] + g["f_cyl"] * 2 * np.pi * k / 8)) % g["out_w"]
        assert own[g["out_h"] // 2, u] == k


def test_modes_agree_away_from_seams():
    """Feather and multi-band equal the seam copy wherever one camera covers a whole
    neighbourhood (feather: exactly; multi-band: within rounding of the pyramid)."""
    cams, frames, g = rig.cylinder_rig(8, 320, 180, 185.0, 3, seed=2, jitter_deg=1.0)
    seam, own = _pano(cams, frames, g, oracle.BLEND_SEAM, want_owner=True)
    fea = _pano(cams, frames, g, oracle.BLEND_FEATHER)
    mb = _pano(cams, frames, g, oracle.BLEND_MULTIBAND)
    # camera 0's centre: the neighbours' 40.8 degree half-fields start ~4 degrees (~13 px) away
    u = int(round(g["u0"]))
    blk = (slice(60, 120), slice(u - 6, u + 6))
    assert (own[blk] == 0).all()
    assert np.array_equal(fea[blk], seam[blk])
    assert np.abs(mb[blk].astype(int) - seam[blk].astype(int)).max() <= 1
    # across a seam the blends differ from the hard copy (gains differ per camera)
    assert np.abs(mb.astype(int) - seam.astype(int)).max() > 2


def test_cylindrical_plan_boundary_checks():
    from multicamera_stitching_amd import _capi
    cams, _, g = rig.cylinder_rig(8, 64, 36, 37.0, 3, seed=0)
    plan = _capi.Plan.cylindrical(cams, g["out_w"], g["out_h"], g["f_cyl"], g["u0"], g["v0"], 3)
    assert (plan.out_w, plan.out_h, plan.channels) == (g["out_w"], g["out_h"], 3)
    assert plan.n_cams == 8 and plan.cam_shapes[3] == (36, 64)
    assert plan.stats()["blend"] == _capi.MCS_BLEND_MULTIBAND
    with pytest.raises(_capi.McsError) as e:
        plan.set_blend(_capi.MCS_BLEND_NONE)       # no paste order on a cylinder
    assert e.value.code == _capi.MCS_E_INVALID
    plan.set_blend(_capi.MCS_BLEND_SEAM)
    assert plan.stats()["blend"] == _capi.MCS_BLEND_SEAM
    bad = [dict(c) for c in cams]
    bad[2]["f"] = 0.0
    with pytest.raises(_capi.McsError):
        _capi.Plan.cylindrical(bad, g["out_w"], g["out_h"], g["f_cyl"], g["u0"], g["v0"], 3)
    with pytest.raises(_capi.McsError):
        _capi.Plan.cylindrical(cams * 2, g["out_w"], g["out_h"], g["f_cyl"], g["u0"], g["v0"], 3)
    with pytest.raises(_capi.McsError):
        _capi.Plan.cylindrical(cams, 0, g["out_h"], g["f_cyl"], g["u0"], g["v0"], 3)

"""GPU blended stitch modes (SURVEY.md 8 NS-1 multi-band, NS-2 feather) vs their CPU
restatement oracle/orc_blend.c.  No reference implementation exists (the reference pastes), so
the bar is our own specification: bit-exact (the north star allows 1 LSB for float blends; the
integer pyramids and IEEE-double blend reproduce the restatement exactly)."""
import numpy as np
import pytest

from conftest import check_mb_path
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
    dict(n=3, w=202, h=110, ch=3, seed=13),   # rows of 606 B: the band pass's unaligned windows
])
def test_blend_vs_oracle(mode, case, mb_path):
    if mode == "feather" and mb_path == "bands":
        pytest.skip("feather has one path")
    case = dict(case)
    interp = case.pop("interp", 1)
    plan, cams = _world_plan(interp=interp, **case)
    plan.set_blend(MODES[mode])
    got = plan.stitch_host(cams)
    want = oracle.blend_stitch(plan.describe(), cams, MODES[mode], interp)
    assert _diff(got.reshape(want.shape), want) == 0
    st = plan.stats()
    assert st["blend"] == MODES[mode] and st["blend_tiles"] > 0
    if mode == "multiband":
        # (the sweep: mosaics of >= 128 px a side with <= 3 channels)
        check_mb_path(st, mb_path, case["ch"] <= 3 and min(plan.out_w, plan.out_h) >= 128 and
                      st["mb_mixed_px"] > 0)


def test_multiband_c2_full_size_batch(mb_path):
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
    # band pass: both window forms ran in this launch -- most bands on the LDS ring, the bands
    # with reflected rows (top / bottom mosaic edge) on dword-aligned global windows
    st = plan.stats()
    check_mb_path(st, mb_path)
    if mb_path == "bands":
        assert 0 < st["mb_bands_lds"] < st["mb_bands"], st


def test_multiband_c2_full_launch_every_capture(mb_path):
    """The bench's own launch (BASELINE configs[1]: bench.py's rig, 64 captures of 4 x 1920x1080,
    256-B mosaic pitch) stitched three times: the three batches equal byte for byte on the device
    (an ordering race between the band pass's LDS-DMA refills and their readers showed as a few
    hundred wrong pixels that moved from run to run, round 4), and EVERY capture of the last
    equal to the restatement (StitcherClass.py:114-136 chain + orc_blend.c multi-band)."""
    import torch
    from multicamera_stitching_amd import rig, _capi
    from multicamera_stitching_amd.StitcherClass import _stage_desc
    st, images, _ = rig.calibrated_stitcher(4, 1920, 1080, 3, seed=0)
    cams = [images[label] for label in st.img_labels]
    plan = _capi.Plan([_stage_desc(sb) for sb in st.stitchers], 1920, 1080, 3, 1)
    plan.set_blend(MODES["multiband"])
    F = 64
    dev = []
    for c in cams:
        base = torch.from_numpy(c).cuda()
        dev.append(torch.stack([torch.roll(base, shifts=f, dims=0) for f in range(F)])
                   .contiguous())
    pitch = (plan.out_w * 3 + 255) // 256 * 256
    outs = [torch.zeros((F, plan.out_h, pitch), dtype=torch.uint8, device="cuda")
            for _ in range(3)]
    for out in outs:
        plan.stitch_device([d.data_ptr() for d in dev], [d[0].numel() for d in dev],
                           out.data_ptr(), pitch, out[0].numel(), F, 0)
    torch.cuda.synchronize()
    for out in outs[:-1]:
        assert torch.equal(out, outs[-1])
    got = outs[-1][:, :, :plan.out_w * 3].cpu().numpy()
    del outs, dev
    bad = []
    for f in range(F):
        want = oracle.blend_stitch(plan.describe(), [np.roll(c, f, axis=0) for c in cams],
                                   MODES["multiband"])
        d = _diff(got[f].reshape(want.shape), want)
        if d:
            bad.append((f, d))
    assert not bad, bad
    check_mb_path(plan.stats(), mb_path)


@pytest.mark.parametrize("shift, pad", [(1, 0), (3, 2)])
def test_multiband_c2_unaligned_frames(shift, pad, mb_path):
    """Config 2 at full size with camera frames that start off a 4-byte boundary (shift) and,
    for pad > 0, a frame stride that is not a multiple of 4: the launch takes the band pass's
    unaligned window form, whose descriptors must stay the frame-offset ones even though the
    plan's LDS-ring bands rewrote theirs (advisor finding, round 3) -- bit-exact vs the oracle."""
    import torch
    plan, cams = _world_plan(4, 1920, 1080, 3, seed=0)
    plan.set_blend(MODES["multiband"])
    F = 2
    shots = [[np.roll(c, 5 * f, axis=1) for c in cams] for f in range(F)]
    fb = cams[0].size
    stride = fb + pad
    dev = []
    for i in range(len(cams)):
        buf = torch.zeros(shift + F * stride, dtype=torch.uint8)
        for f in range(F):
            buf[shift + f * stride: shift + f * stride + fb] = torch.from_numpy(
                shots[f][i].reshape(-1))
        dev.append(buf.cuda())
    out = torch.zeros((F, plan.out_h, plan.out_w * 3), dtype=torch.uint8, device="cuda")
    plan.stitch_device([d.data_ptr() + shift for d in dev], [stride] * len(dev),
                       out.data_ptr(), plan.out_w * 3, out[0].numel(), F, 0)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for f in range(F):
        want = oracle.blend_stitch(plan.describe(), shots[f], MODES["multiband"])
        assert _diff(got[f].reshape(want.shape), want) == 0, f
    # the aligned launch of the same plan afterwards (band pass: still on the ring, its
    # descriptors intact)
    st = plan.stats()
    check_mb_path(st, mb_path)
    if mb_path == "bands":
        assert 0 < st["mb_bands_lds"] < st["mb_bands"], st
    want = oracle.blend_stitch(plan.describe(), cams, MODES["multiband"])
    assert _diff(plan.stitch_host(cams).reshape(want.shape), want) == 0


@pytest.mark.parametrize("F", [64, 70])
def test_multiband_batch_split_and_chunked(F, mb_path):
    """A multi-band device batch of F captures: F <= 64 takes the split launch (streaming tiles
    under mixed pixels first, the blend beside the rest), F > 64 the chunked launch (levels +
    blend per 64-capture chunk of the scratch after the streaming kernel) -- every capture equal
    to the restatement."""
    import torch
    plan, cams = _world_plan(3, 160, 140, 3, seed=12)   # (>= 128 px: the band pass)
    plan.set_blend(MODES["multiband"])
    shots = [[np.roll(c, 3 * f, axis=1) for c in cams] for f in range(F)]
    dev = [torch.from_numpy(np.stack([shots[f][i] for f in range(F)])).cuda()
           for i in range(len(cams))]
    pitch = (plan.out_w * 3 + 63) // 64 * 64
    out = torch.zeros((F, plan.out_h, pitch), dtype=torch.uint8, device="cuda")
    plan.stitch_device([d.data_ptr() for d in dev], [d[0].numel() for d in dev],
                       out.data_ptr(), pitch, out[0].numel(), F, 0)
    torch.cuda.synchronize()
    got = out[:, :, :plan.out_w * 3].cpu().numpy()
    assert plan.stats()["blend_tiles"] > 0
    for f in (0, 1, F // 2, F - 2, F - 1):
        want = oracle.blend_stitch(plan.describe(), shots[f], MODES["multiband"])
        assert _diff(got[f].reshape(want.shape), want) == 0, f


def test_blend_mode_switch_back_to_paste():
    plan, cams = _world_plan(3, 120, 80, 3, seed=9)
    paste = plan.stitch_host(cams)
    plan.set_blend(MODES["multiband"])
    mb = plan.stitch_host(cams)
    plan.set_blend(0)
    assert _diff(plan.stitch_host(cams), paste) == 0
    assert _diff(mb, paste) > 0


@pytest.mark.parametrize("n, w, step, owners", [
    (5, 40, 6, 5),      # five cameras 6 px apart: five owners in one 64 x 64 neighbourhood
    (6, 48, 5, 6),
    (8, 64, 5, 8),      # eight: the widest blend kernel
])
def test_multiband_dense_seams_vs_oracle(n, w, step, owners, mb_path):
    """Narrow-seam rigs put 5..8 owners into one neighbourhood: the <= 8-owner blend kernel
    (mcs_mb_blend_c*_s8) handles them, bit-exact vs the restatement (feather too)."""
    plan, cams = _world_plan(n, w, 30, 3, seed=11, step=step)
    for mode in ("multiband", "feather"):
        plan.set_blend(MODES[mode])
        want = oracle.blend_stitch(plan.describe(), cams, MODES[mode])
        assert _diff(plan.stitch_host(cams).reshape(want.shape), want) == 0, mode
        if mode == "multiband":
            assert owners - 3 <= plan.stats()["mb_owners"] <= owners and \
                plan.stats()["mb_owners"] > 4


@pytest.mark.parametrize("n, w, step", [(10, 64, 4), (12, 48, 3)])
def test_multiband_more_than_eight_owners_degrades_to_feather(n, w, step, mb_path):
    """Ten (twelve) cameras 4 (3) px apart put more than eight owners into 64 x 96
    neighbourhoods: more than the blend kernels hold, so those tiles take the feather rule on the
    GPU (orc_blend.c "dense seams"), the rest stay multi-band -- bit-exact vs the restatement,
    never an exception (never raise on expected failures)."""
    plan, cams = _world_plan(n, w, 30, 3, seed=11, step=step)
    plan.set_blend(MODES["multiband"])
    got = plan.stitch_host(cams)
    want = oracle.blend_stitch(plan.describe(), cams, MODES["multiband"])
    assert _diff(got.reshape(want.shape), want) == 0
    st = plan.stats()
    assert st["mb_degraded_tiles"] > 0 and st["mb_owners"] <= 8
    # the degraded tiles really are feathered (their pixels equal the feather mosaic's; the CPU
    # test test_blend_dense_cpu.py checks which tiles), the others are not
    plan.set_blend(MODES["feather"])
    fea = oracle.blend_stitch(plan.describe(), cams, MODES["feather"])
    assert _diff(plan.stitch_host(cams).reshape(fea.shape), fea) == 0
    same = (want == fea).all(axis=-1).mean()
    assert 0.2 < same < 1.0, same


def test_dropin_dense_rig_multiband_does_not_raise(monkeypatch):
    """The drop-in Stitcher on a 10-camera dense rig under MCS_BLEND=multiband: no exception, a
    logged warning, the mosaic bit-exact vs the oracle's degraded rule."""
    from multicamera_stitching_amd import rig, _capi
    from multicamera_stitching_amd.StitcherClass import Stitcher
    monkeypatch.setenv("MCS_BLEND", "multiband")
    C = rig.camera_models(10, 64, 30, seed=11, step=4)
    frames = rig.world_frames(C, 64, 30, 3, seed=11)
    images = dict(zip(rig.labels(10), frames))
    st = Stitcher(images)
    st.calibrate_stitcher(images, save=False,
                          homographies=rig.homography_provider(C, lambda: st.stitchers))
    logged = []
    monkeypatch.setattr(st, "debugger", lambda lvl, msg, log_type="info": logged.append(msg))
    got = st.stitch(images)
    plan = st.plan(channels=3)
    cams = [images[label] for label in st.img_labels]
    want = oracle.blend_stitch(plan.describe(), cams, MODES["multiband"])
    assert _diff(got.reshape(want.shape), want) == 0
    assert plan.stats()["mb_degraded_tiles"] > 0
    assert any("feather" in m for m in logged), logged


def test_plan_destroy_frees_multiband_tables(mb_path):
    """Creating, preparing and destroying multi-band plans (band pass, launch order, degraded
    list) in a loop leaves the device's free memory where it was (mcs_plan_destroy frees every
    prepared table)."""
    import gc
    import torch
    from multicamera_stitching_amd import _capi
    torch.cuda.init()

    def once():
        plan, cams = _world_plan(4, 320, 180, 3, seed=3)
        plan.set_blend(MODES["multiband"])
        plan.stitch_host(cams)
        assert plan.stats()["blend_tiles"] > 0
        plan.close()
    once()
    torch.cuda.synchronize()
    gc.collect()
    free0 = torch.cuda.mem_get_info()[0]
    for _ in range(12):
        once()
    gc.collect()
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    # (allocator granularity aside, a leak of the band tables is ~0.4 MB per plan)
    assert free0 - free1 < 2 * 1024 * 1024, (free0, free1)


@pytest.mark.parametrize("interp", [0, 1])
def test_c1_checker_feather_vs_oracle(interp, monkeypatch):
    """BASELINE configs[0]: 2 x 640x480 checkerboard, H = translation(400, 0), nearest-neighbour
    warp (and bilinear), linear feather blend -- through the drop-in Stitcher (MCS_BLEND=feather,
    MCS_INTERP) on the GPU, bit-exact vs orc_blend.c; the 240-px overlap is a weighted mix."""
    from multicamera_stitching_amd.StitcherClass import Stitcher
    monkeypatch.setenv("MCS_BLEND", "feather")
    monkeypatch.setenv("MCS_INTERP", "nearest" if interp == 0 else "linear")
    yy, xx = np.mgrid[0:480, 0:640]
    chk = np.where(((xx // 32) + (yy // 32)) % 2 == 0, 32, 224).astype(np.uint8)
    a = np.stack([chk, chk // 2 + 10, 255 - chk], -1)
    b = np.stack([255 - chk, chk, chk // 2 + 20], -1)
    images = {"CAM1": a, "CAM2": b}
    st = Stitcher(images)
    st.calibrate_stitcher(images, save=False, homographies=[[[1, 0, 400], [0, 1, 0], [0, 0, 1]]])
    got = st.stitch(images)
    assert got.shape == (480, 1040, 3)
    plan = st.plan(channels=3)
    assert plan.stats()["blend"] == MODES["feather"] and plan.stats()["blend_tiles"] > 0
    want = oracle.blend_stitch(plan.describe(), [a, b], MODES["feather"], interp)
    assert _diff(got, want) == 0
    # outside the overlap each camera alone; inside, every value between the two sources
    assert np.array_equal(got[:, :400], a[:, :400]) and np.array_equal(got[:, 640:], b[:, 240:])
    ov_a, ov_b, ov = a[:, 400:].astype(int), b[:, :240].astype(int), got[:, 400:640].astype(int)
    assert ((ov >= np.minimum(ov_a, ov_b)) & (ov <= np.maximum(ov_a, ov_b))).all()
    assert (ov != ov_a).any() and (ov != ov_b).any()

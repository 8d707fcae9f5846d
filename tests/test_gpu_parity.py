"""GPU parity: libmcs (HIP, gfx950) vs the reference's outputs and the CPU oracle.

Bar: bit-exact (max |diff| == 0) for the u8 mosaics -- bilinear and nearest alike, since the
kernel reproduces OpenCV's integer/fixed-point arithmetic.
"""
import numpy as np
import pytest

import goldens
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    from multicamera_stitching_amd import _capi
    n = _capi.device_count()
    assert n >= 1, "GPU tests need an MI355X (no HIP device visible)"


def _diff(a, b):
    assert a.shape == b.shape, (a.shape, b.shape)
    return int(np.abs(a.astype(np.int16) - b.astype(np.int16)).max()) if a.size else 0


@pytest.mark.parametrize("name", goldens.names())
def test_golden_via_capi(name):
    meta, calib, frames, out = goldens.load_full(name)
    cams = goldens.sorted_cams(meta, frames)
    ch = 1 if cams[0].ndim == 2 else cams[0].shape[2]
    plan = goldens.plan_for(meta, goldens.sorted_cams(meta, calib), channels=ch)
    got = plan.stitch_host(cams, [(c.shape[1], c.shape[0]) for c in cams])
    assert _diff(got.reshape(out.shape), out) == 0


@pytest.mark.parametrize("name", goldens.names())
def test_golden_via_dropin(name):
    """Calibrate our Stitcher with the fixture's homographies, stitch, compare to the reference."""
    from multicamera_stitching_amd.StitcherClass import Stitcher
    meta, calib, frames, out = goldens.load_full(name)
    st = Stitcher(dict(calib), super_mode=meta["super_mode"])
    assert [str(v) for v in st.img_labels] == meta["img_labels"]
    Hs = [s["H_in"] for s in meta["stages"]]
    st.calibrate_stitcher(dict(calib), save=False, homographies=Hs)
    got = st.stitch(dict(frames))
    assert _diff(got, out) == 0
    # the per-stage path (StitcherBase.stitch, used during feature calibration) agrees too
    cams = goldens.sorted_cams(meta, frames)
    img = cams[0]
    for i, sb in enumerate(st.stitchers):
        img = sb.stitch((img, cams[i + 1]))
    assert _diff(np.ascontiguousarray(img), out) == 0


def _rig_plan(n, w, h, ch, super_mode, seed, interp, **kw):
    from multicamera_stitching_amd import rig, _capi
    from multicamera_stitching_amd.StitcherClass import _stage_desc
    st, images, C = rig.calibrated_stitcher(n, w, h, ch, super_mode=super_mode, seed=seed, **kw)
    cams = [images[label] for label in st.img_labels]
    descs = [_stage_desc(sb) for sb in st.stitchers]
    plan = _capi.Plan(descs, w, h, ch, interp)
    stages = []
    for sb in st.stitchers:
        stages.append(dict(H=np.asarray(sb.cachedAH), canvas_w=sb.ABSize[0],
                           canvas_h=sb.ABSize[1], bx=sb.Bpts[0][0], by=sb.Bpts[0][1],
                           super_mode=super_mode, x_limits=sb.x_limits, y_limits=sb.y_limits))
    return plan, cams, stages


@pytest.mark.parametrize("interp", [oracle.INTER_LINEAR, oracle.INTER_NEAREST])
@pytest.mark.parametrize("super_mode", [False, True])
@pytest.mark.parametrize("ch", [3, 1])
def test_rig_vs_oracle_cascade(interp, super_mode, ch):
    plan, cams, stages = _rig_plan(4, 320, 180, ch, super_mode, seed=3, interp=interp,
                                   rot_deg=3.0, persp=5e-5)
    want = oracle.cascade_stitch(stages, cams, interp)
    got = plan.stitch_host(cams)
    assert _diff(got, want) == 0


def test_c2_full_size_vs_oracle():
    """North-star config 2 geometry at full size: 4 x 1920x1080 BGR, bilinear."""
    plan, cams, stages = _rig_plan(4, 1920, 1080, 3, False, seed=0,
                                   interp=oracle.INTER_LINEAR)
    want = oracle.cascade_stitch(stages, cams)
    got = plan.stitch_host(cams)
    assert got.shape[1] > 6000 and got.shape[0] >= 1080
    assert _diff(got, want) == 0


def test_c1_translation_nearest_equals_linear():
    """Config 1: 2 x 640x480 checkerboard, H = translation(400, 0): NN == bilinear == copy."""
    from multicamera_stitching_amd.StitcherClass import Stitcher
    yy, xx = np.mgrid[0:480, 0:640]
    chk = np.where(((xx // 32) + (yy // 32)) % 2 == 0, 32, 224).astype(np.uint8)
    a = np.stack([chk, chk // 2 + 10, 255 - chk], -1)
    b = np.stack([255 - chk, chk, chk // 2 + 20], -1)
    images = {"CAM1": a, "CAM2": b}
    H = [[[1, 0, 400], [0, 1, 0], [0, 0, 1]]]
    outs = {}
    for mode in ("linear", "nearest"):
        st = Stitcher(images)
        st.calibrate_stitcher(images, save=False, homographies=H)
        plan = st.plan(channels=3, interp=1 if mode == "linear" else 0)
        outs[mode] = plan.stitch_host([a, b])
    assert outs["linear"].shape == (480, 1040, 3)
    want = np.zeros((480, 1040, 3), np.uint8)
    want[:, 400:] = b
    want[:, :640] = a
    assert _diff(outs["linear"], want) == 0
    assert _diff(outs["nearest"], want) == 0


def test_device_batch_matches_host():
    """mcs_stitch_device over a batch of frames with a pitched output == per-frame host path."""
    import torch
    from multicamera_stitching_amd import rig
    plan, cams, _ = _rig_plan(4, 256, 144, 3, False, seed=5, interp=1, rot_deg=2.0)
    F = 3
    frames = [[rig.texture(c.shape[0], c.shape[1], 3, seed=100 * f + i)
               for i, c in enumerate(cams)] for f in range(F)]
    dev = [torch.from_numpy(np.stack([frames[f][i] for f in range(F)])).cuda()
           for i in range(len(cams))]
    pitch = (plan.out_w * 3 + 255) // 256 * 256
    out = torch.full((F, plan.out_h, pitch), 7, dtype=torch.uint8, device="cuda")
    strides = [d[0].numel() for d in dev]
    plan.stitch_device([d.data_ptr() for d in dev], strides, out.data_ptr(), pitch,
                       out[0].numel(), F, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for f in range(F):
        want = plan.stitch_host(frames[f])
        assert _diff(got[f, :, :plan.out_w * 3].reshape(plan.out_h, plan.out_w, 3), want) == 0
        assert (got[f, :, plan.out_w * 3:] == 7).all(), "kernel wrote past the row"


def test_footprint_counts():
    plan, cams, _ = _rig_plan(4, 320, 180, 3, False, seed=3, interp=1)
    fp = plan.footprint()
    assert fp[0] == 320 * 180          # camera 0 is pasted whole (no super crop)
    for i in range(1, 4):
        assert 0 < fp[i] <= 320 * 180


def _batch(plan, cams, F, seed, pad=None):
    """Device batch of F captures per camera; pad[i] extra bytes between frames of camera i."""
    import torch
    from multicamera_stitching_amd import rig
    frames = [[rig.texture(c.shape[0], c.shape[1], c.shape[2] if c.ndim == 3 else 1,
                           seed=seed + 100 * f + i) for i, c in enumerate(cams)]
              for f in range(F)]
    dev, strides = [], []
    for i, c in enumerate(cams):
        n = c.size + (pad[i] if pad else 0)
        buf = torch.zeros((F, n), dtype=torch.uint8)
        for f in range(F):
            buf[f, :c.size] = torch.from_numpy(np.ascontiguousarray(frames[f][i]).reshape(-1))
        dev.append(buf.cuda())
        strides.append(n)
    return frames, dev, strides


@pytest.mark.parametrize("force64", [False, True])
@pytest.mark.parametrize("pad", [None, [0, 64, 0, 4096]])
def test_batch_address_modes_and_mixed_strides(force64, pad):
    """32-bit-offset and 64-bit-address kernels; uniform and per-camera frame strides (the
    latter is split into per-frame launches) -- all equal to the per-frame host path."""
    import ctypes
    import torch
    from multicamera_stitching_amd import _capi
    L = _capi.load()
    plan, cams, _ = _rig_plan(4, 200, 120, 3, False, seed=7, interp=1, rot_deg=4.0, persp=1e-4)
    F = 3
    frames, dev, strides = _batch(plan, cams, F, seed=11, pad=pad)
    pitch = plan.out_w * 3 + 4
    out = torch.full((F, plan.out_h, pitch), 9, dtype=torch.uint8, device="cuda")
    L.mcs__force_off64(ctypes.c_int(1 if force64 else 0))
    try:
        plan.stitch_device([d.data_ptr() for d in dev], strides, out.data_ptr(), pitch,
                           out[0].numel(), F, 0)
        torch.cuda.synchronize()
    finally:
        L.mcs__force_off64(ctypes.c_int(0))
    got = out.cpu().numpy()
    for f in range(F):
        want = plan.stitch_host(frames[f])
        assert _diff(got[f, :, :plan.out_w * 3].reshape(plan.out_h, plan.out_w, 3), want) == 0
        assert (got[f, :, plan.out_w * 3:] == 9).all()


@pytest.mark.parametrize("ch", [1, 2, 4])
def test_channel_counts_vs_oracle(ch):
    plan, cams, stages = _rig_plan(3, 150, 90, ch, False, seed=9, interp=1, rot_deg=5.0,
                                   persp=2e-4)
    want = oracle.cascade_stitch(stages, cams, oracle.INTER_LINEAR)
    got = plan.stitch_host(cams)
    assert _diff(got.reshape(want.shape), want) == 0


@pytest.mark.parametrize("ch", [1, 3])
@pytest.mark.parametrize("w,h", [(37, 23), (101, 57)])
def test_frame_end_rows_stream_through_lds(ch, w, h):
    """Odd pitches: the footprint of a camera's last row reaches past the frame end, so its DMA
    row is fetched from earlier bytes (TileHdr::last_shift) -- every tile stays on the LDS path
    and the mosaic still equals the oracle, for single captures and dense batches."""
    import torch
    from multicamera_stitching_amd.StitcherClass import Stitcher
    from multicamera_stitching_amd import rig
    frames = rig.make_frames(3, w, h, ch, seed=21)
    images = dict(zip(rig.labels(3), frames))
    Hs = [[[0.99, 0.02, w * 0.6 + 0.37], [-0.01, 1.0, 1.6], [0, 0, 1]],
          [[1.0, -0.015, w * 1.2 + 0.61], [0.02, 0.98, -2.3], [1e-4, 0, 1]]]
    st = Stitcher(images)
    st.calibrate_stitcher(images, save=False, homographies=Hs)
    plan = st.plan(channels=ch, interp=1)
    cams = [images[label] for label in st.img_labels]
    stages = [dict(H=np.asarray(sb.cachedAH), canvas_w=sb.ABSize[0], canvas_h=sb.ABSize[1],
                   bx=sb.Bpts[0][0], by=sb.Bpts[0][1], super_mode=False,
                   x_limits=sb.x_limits, y_limits=sb.y_limits) for sb in st.stitchers]
    want = oracle.cascade_stitch(stages, cams, oracle.INTER_LINEAR)
    assert _diff(plan.stitch_host(cams).reshape(want.shape), want) == 0
    stats = plan.stats()
    assert stats["direct_tiles"] == 0 and stats["lds_tiles"] == stats["tiles"]
    F = 5
    batch, dev, strides = _batch(plan, cams, F, seed=31)
    out = torch.zeros((F, plan.out_h, plan.out_w * ch), dtype=torch.uint8, device="cuda")
    plan.stitch_device([d.data_ptr() for d in dev], strides, out.data_ptr(), plan.out_w * ch,
                       out[0].numel(), F, 0)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for f in range(F):
        want = oracle.cascade_stitch(stages, batch[f], oracle.INTER_LINEAR)
        assert _diff(got[f].reshape(want.shape), want) == 0



@pytest.mark.parametrize("ch", [1, 2, 3, 4])
@pytest.mark.parametrize("src,dst", [((53, 37), (72, 48)), ((144, 96), (72, 48)),
                                     ((40, 64), (64, 40)), ((1080, 1920), (1920, 1080)),
                                     ((7, 5), (3, 2)), ((31, 17), (31, 17)), ((2, 2), (9, 1))])
def test_resize_linear_device_vs_oracle(ch, src, dst):
    """mcs_resize_linear_device == cv2.resize(INTER_LINEAR) restatement: up, down, exact 2x
    (INTER_AREA path), transposed MediaPlayer frames, tiny, identity -- batch of 3 frames."""
    import torch
    from multicamera_stitching_amd import _capi
    (sw, sh), (dw, dh) = src, dst
    rng = np.random.default_rng(sw * 7 + dw + ch)
    F = 3
    frames = rng.integers(0, 256, (F, sh, sw, ch), dtype=np.uint8)
    d_src = torch.from_numpy(frames).cuda()
    d_dst = torch.full((F, dh, dw * ch + 8), 77, dtype=torch.uint8, device="cuda")
    _capi.resize_linear_device(d_src.data_ptr(), sw, sh, d_dst.data_ptr(), dw, dh, ch,
                               n_frames=F, dst_pitch=dw * ch + 8,
                               dst_frame_stride=d_dst[0].numel())
    torch.cuda.synchronize()
    got = d_dst.cpu().numpy()
    for f in range(F):
        want = oracle.resize_linear(frames[f], (dw, dh)).reshape(dh, dw * ch)
        assert _diff(got[f, :, :dw * ch], want) == 0
        assert (got[f, :, dw * ch:] == 77).all()


def test_dropin_off_size_frames_resized_on_gpu():
    """Stitcher.stitch with frames of another size (and MediaPlayer's transposed single-channel
    frames) == resize restatement + cascade, through one mcs_stitch_host_sized call."""
    from multicamera_stitching_amd import rig
    from multicamera_stitching_amd.StitcherClass import Stitcher
    w, h = 160, 96
    frames = rig.make_frames(3, w, h, 3, seed=41)
    images = dict(zip(rig.labels(3), frames))
    Hs = [[[0.99, 0.01, 121.3], [-0.01, 1.0, 2.6], [1e-5, 0, 1]],
          [[1.0, -0.02, 240.7], [0.01, 0.99, -1.4], [0, 1e-5, 1]]]
    st = Stitcher(images)
    st.calibrate_stitcher(images, save=False, homographies=Hs)
    stages = [dict(H=np.asarray(sb.cachedAH), canvas_w=sb.ABSize[0], canvas_h=sb.ABSize[1],
                   bx=sb.Bpts[0][0], by=sb.Bpts[0][1], super_mode=False,
                   x_limits=sb.x_limits, y_limits=sb.y_limits) for sb in st.stitchers]
    for shots in (rig.make_frames(3, 211, 130, 3, seed=42),
                  [np.ascontiguousarray(f.T) for f in rig.make_frames(3, w, h, 1, seed=43)]):
        got = st.stitch(dict(zip(rig.labels(3), shots)))
        cams = [oracle.resize_linear(c, (w, h)) for c in shots]
        want = oracle.cascade_stitch(stages, cams)
        assert _diff(got, want) == 0

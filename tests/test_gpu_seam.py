"""GPU graph-cut seams (mcs_plan_find_seams): device sampling of the seam
grid + device push-relabel max-flow (the host Dinic, MCS_SEAM_FLOW=host, is its checker), then
the seam-labelled owner rule inside the stitch kernels, against the CPU restatement
(oracle/orc_seam.c + orc_blend.c).  Bit-exact labels and panoramas."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _diff(a, b):
    return int(np.abs(a.astype(np.int16) - b.astype(np.int16)).max()) if a.size else 0


def _cyl(n, w, h, f, ch, seed, **kw):
    from multicamera_stitching_amd import rig, _capi
    cams, frames, g = rig.cylinder_rig(n, w, h, f, ch, seed=seed, **kw)
    plan = _capi.Plan.cylindrical(cams, g["out_w"], g["out_h"], g["f_cyl"], g["u0"], g["v0"],
                                  ch)
    ref = lambda fr, mode, k: oracle.blend_stitch_cyl(
        cams, g["out_w"], g["out_h"], g["f_cyl"], g["u0"], g["v0"], fr, mode, seam_k=k,
        want_seams=k is not None)
    return plan, frames, ref


@pytest.mark.parametrize("mode", [3, 2, 1])
@pytest.mark.parametrize("k", [0, 1, 2])
def test_cylinder_graphcut_vs_oracle(mode, k):
    plan, frames, ref = _cyl(8, 320, 180, 185.0, 3, seed=1, jitter_deg=1.0, gain=0.05)
    plan.set_blend(mode)
    plan.find_seams(frames, scale_log2=k)
    want, lab = ref(frames, mode, k)
    assert np.array_equal(plan.seam_labels(), lab)
    assert _diff(plan.stitch_host(frames).reshape(want.shape), want) == 0


def test_chain_plan_graphcut_vs_oracle():
    """Seams work on the reference's homography chains too."""
    from multicamera_stitching_amd import rig, _capi
    from multicamera_stitching_amd.StitcherClass import _stage_desc
    st, images, _ = rig.calibrated_stitcher(4, 320, 180, 3, seed=2, rot_deg=2.0, persp=5e-5)
    cams = [images[label] for label in st.img_labels]
    plan = _capi.Plan([_stage_desc(sb) for sb in st.stitchers], 320, 180, 3, 1)
    plan.set_blend(_capi.MCS_BLEND_MULTIBAND)
    plan.find_seams(cams, scale_log2=1)
    want, lab = oracle.blend_stitch(plan.describe(), cams, 2, seam_k=1, want_seams=True)
    assert np.array_equal(plan.seam_labels(), lab)
    assert _diff(plan.stitch_host(cams).reshape(want.shape), want) == 0
    plan.find_seams(method=_capi.MCS_SEAM_DISTANCE)          # back to distance seams
    assert plan.seam_labels() is None
    want = oracle.blend_stitch(plan.describe(), cams, 2)
    assert _diff(plan.stitch_host(cams).reshape(want.shape), want) == 0


def test_seams_found_once_then_reused_across_captures():
    """The seams are calibration state: later captures are stitched with them unchanged."""
    plan, frames, ref = _cyl(6, 200, 150, 120.0, 3, seed=4)
    plan.find_seams(frames, scale_log2=1)
    lab0 = plan.seam_labels().copy()
    moved = [np.roll(f, 9, axis=1) for f in frames]
    got = plan.stitch_host(moved)
    assert np.array_equal(plan.seam_labels(), lab0)
    # the oracle with the labels of the first capture: recompute them there, then stitch
    want0, lab = ref(frames, 2, 1)
    assert np.array_equal(lab, lab0)
    assert _diff(plan.stitch_host(frames).reshape(want0.shape), want0) == 0
    assert got.shape == want0.shape


def test_cylinder_c4_full_size_graphcut(mb_path):
    """C4 at full size (8 x 1920x1080 -> 6912 x 1080), graph-cut seams on the 1/4 grid,
    multi-band: labels and panorama bit-exact."""
    plan, frames, ref = _cyl(8, 1920, 1080, 1100.0, 3, seed=0, jitter_deg=0.5)
    plan.find_seams(frames, scale_log2=2)
    want, lab = ref(frames, 2, 2)
    assert np.array_equal(plan.seam_labels(), lab)
    assert _diff(plan.stitch_host(frames).reshape(want.shape), want) == 0


def _synthetic_seam_grid(gw, gh, n, seed, noise):
    """A cylinder-like grid: n cameras, each covering its column band plus overlaps, owner = the
    nearest band centre; samples = one world + per-camera noise (noise 0: flat costs)."""
    rng = np.random.default_rng(seed)
    cols = np.arange(gw)
    per = gw / n
    ov = max(2, int(per * 0.4))
    cov = np.zeros((gh, gw), np.uint16)
    dist = []
    for i in range(n):
        c = i * per + per / 2
        d = (cols - c + gw / 2) % gw - gw / 2
        cov[:, np.abs(d) <= per / 2 + ov] |= np.uint16(1 << i)
        dist.append(np.abs(d))
    lab = np.repeat(np.argmin(np.stack(dist), 0).astype(np.uint8)[None, :], gh, 0)
    world = rng.integers(0, 256, (gh, gw, 3), dtype=np.int32)
    smp = np.stack([np.clip(world + rng.integers(-noise, noise + 1, world.shape), 0, 255)
                    .astype(np.uint8) for _ in range(n)])
    return lab, cov, smp


@pytest.mark.parametrize("gw,gh,n,seed,noise", [(96, 40, 4, 0, 30), (160, 64, 6, 1, 60),
                                                 (64, 64, 3, 2, 0), (200, 90, 8, 3, 20)])
def test_device_maxflow_equals_host_dinic(gw, gh, n, seed, noise):
    """The device push-relabel cut (mcs_seam_graphcut_device) = the host Dinic's
    (mcs_seam_graphcut_host): the minimal minimum cut is unique."""
    from multicamera_stitching_amd import _capi
    lab, cov, smp = _synthetic_seam_grid(gw, gh, n, seed, noise)
    want = _capi.seam_graphcut_host(lab, cov, smp)
    got, st = _capi.seam_graphcut_device(lab, cov, smp, with_stats=True)
    assert st[0] > 0
    assert np.array_equal(got, want), (int((got != want).sum()), st)

"""Streaming pipeline (mcs_stream_*): captures submitted back to back through pinned staging,
copy/compute/copy streams and per-slot hipGraphs come out identical to one-at-a-time stitches,
in submission order, for the paste and the multi-band plans."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("blend,graphs,depth", [(0, True, 3), (0, False, 2), (2, True, 2),
                                               (1, True, 1)])
def test_stream_matches_single_stitches(blend, graphs, depth):
    from multicamera_stitching_amd import _capi, rig
    from multicamera_stitching_amd.StitcherClass import _stage_desc
    st, images, _ = rig.calibrated_stitcher(4, 200, 120, 3, seed=12, rot_deg=2.0)
    cams0 = [images[label] for label in st.img_labels]
    plan = _capi.Plan([_stage_desc(sb) for sb in st.stitchers], 200, 120, 3, 1)
    plan.set_blend(blend)
    F = 7
    shots = [[np.roll(c, 3 * f, axis=1) for c in cams0] for f in range(F)]
    want = [plan.stitch_host(s) for s in shots]
    pipe = _capi.StreamPipeline(plan, depth=depth, use_graphs=graphs)
    got, inflight = [], []
    for f in range(F):
        if len(inflight) == depth:
            got.append(pipe.wait(inflight.pop(0)))
        inflight.append(pipe.submit(shots[f]))
    while inflight:
        got.append(pipe.wait(inflight.pop(0)))
    pipe.close()
    assert len(got) == F
    for f in range(F):
        assert np.array_equal(got[f], want[f]), f


def test_stream_refuses_uncollected_slot():
    from multicamera_stitching_amd import _capi, rig
    from multicamera_stitching_amd.StitcherClass import _stage_desc
    st, images, _ = rig.calibrated_stitcher(2, 64, 48, 3, seed=13)
    cams = [images[label] for label in st.img_labels]
    plan = _capi.Plan([_stage_desc(sb) for sb in st.stitchers], 64, 48, 3, 1)
    pipe = _capi.StreamPipeline(plan, depth=1)
    s = pipe.submit(cams)
    with pytest.raises(_capi.McsError):
        pipe.submit(cams)
    assert np.array_equal(pipe.wait(s), plan.stitch_host(cams))
    pipe.close()

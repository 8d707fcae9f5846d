"""CPU checks against the fixtures produced by executing the reference's StitcherClass.py
(tests/golden/gen_golden.py).  No GPU: the C oracle renders, libmcs only builds plans."""
import json
import os
import pickle

import numpy as np
import pytest

import goldens
from oracle import oracle

NAMES = goldens.names()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_cascade_reproduces_reference(name):
    """The C cascade (paste/crop/chain restated) equals the reference's own stitch() output."""
    meta, frames, out = goldens.load(name)
    cams = goldens.sorted_cams(meta, frames)
    got = oracle.cascade_stitch(goldens.oracle_stages(meta), goldens.used_cams(meta, cams))
    assert got.shape == out.shape and np.array_equal(got, out)


@pytest.mark.parametrize("name", NAMES)
def test_plan_flattening_reproduces_reference(name):
    """libmcs' flattened geometry (nested paste rects, OpenCV-inverted matrices, block widths),
    rendered by the CPU flat gather, equals the reference cascade bit for bit."""
    meta, frames, out = goldens.load(name)
    cams = goldens.sorted_cams(meta, frames)
    plan = goldens.plan_for(meta, cams)
    assert plan.out_shape() == tuple(out.shape)
    got = oracle.flat_stitch(plan.describe(), cams)
    assert np.array_equal(got, out)


@pytest.mark.parametrize("name", NAMES)
def test_plan_inverse_is_opencv_closed_form(name):
    meta, frames, _ = goldens.load(name)
    cams = goldens.sorted_cams(meta, frames)
    fl = goldens.plan_for(meta, cams).describe()
    calibrated = [s for s in meta["stages"] if s["calibrated"]]
    for j, s in enumerate(calibrated):
        want = oracle.invert3x3(np.array(s["cachedAH"])).reshape(9)
        assert [float(v) for v in fl["minv"][j]] == [float(v) for v in want]


@pytest.mark.parametrize("name", NAMES)
def test_dropin_geometry_matches_reference(name):
    """Our StitcherBase.calibrate (with the fixture's homographies) yields exactly the reference's
    plan fields: patched cachedAH, inverses, ABSize, Bpts, Apts, super-mode limits, sizes."""
    from multicamera_stitching_amd.StitcherClass import Stitcher
    meta, frames, _ = goldens.load(name)
    st = Stitcher(dict(frames), super_mode=meta["super_mode"])
    assert [str(v) for v in st.img_labels] == meta["img_labels"]
    assert st.stitcher_labels == meta["stitcher_labels"]
    st.calibrate_stitcher(dict(frames), save=False,
                          homographies=[s["H_in"] for s in meta["stages"]])
    for sb, ref in zip(st.stitchers, meta["stages"]):
        assert sb.sid == ref["sid"]
        if not ref["calibrated"]:
            assert sb.cachedAH is None and sb.ABSize is None
            continue
        assert np.asarray(sb.cachedAH).tolist() == ref["cachedAH"]
        assert np.asarray(sb.cachedAINVH).tolist() == ref["cachedAINVH"]
        assert np.asarray(sb.cachedBH, np.float64).tolist() == ref["cachedBH"]
        assert [int(v) for v in sb.ABSize] == ref["ABSize"]
        assert [[int(a), int(b)] for a, b in sb.Bpts] == ref["Bpts"]
        assert [[int(a), int(b)] for a, b in sb.Apts] == ref["Apts"]
        assert [int(v) for v in sb.x_limits] == ref["x_limits"]
        assert [int(v) for v in sb.y_limits] == ref["y_limits"]
        assert list(sb.AimgSize) == ref["AimgSize"]
        assert list(sb.BimgSize) == ref["BimgSize"]


def test_reference_pickle_loads_into_dropin(tmp_path):
    """Stitcher_config.pkl written by the reference's save_stitcher (fixture) loads through our
    load_stitcher with identical geometry, and our re-saved pickle names module StitcherClass."""
    from multicamera_stitching_amd.StitcherClass import Stitcher
    meta, frames, _ = goldens.load("rig4_mild")
    pkl = os.path.join(goldens.GOLDEN, "rig4_mild_Stitcher_config.pkl")
    st = Stitcher(dict(frames)).load_stitcher(pkl)
    assert isinstance(st, Stitcher)
    for sb, ref in zip(st.stitchers, meta["stages"]):
        assert np.asarray(sb.cachedAH).tolist() == ref["cachedAH"]
        assert [int(v) for v in sb.ABSize] == ref["ABSize"]
    out = tmp_path / "again.pkl"
    st.save_stitcher(str(out))
    raw = out.read_bytes()
    assert b"StitcherClass" in raw and b"_mcs_cache" not in raw
    st2 = Stitcher(dict(frames)).load_stitcher(str(out))
    for a, b in zip(st.stitchers, st2.stitchers):
        assert np.array_equal(np.asarray(a.cachedAH), np.asarray(b.cachedAH))
        assert a.ABSize == b.ABSize


def test_fixture_manifest_is_consistent():
    for name in NAMES:
        meta, frames, out = goldens.load(name)
        assert sorted(frames) == sorted(meta["labels"])
        assert list(out.shape) == meta["out_shape"]
        assert json.dumps(meta)  # plain JSON only

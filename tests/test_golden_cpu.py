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
    meta, _, frames, out = goldens.load_full(name)
    cams = goldens.resized_for_oracle(meta, goldens.sorted_cams(meta, frames))
    got = oracle.cascade_stitch(goldens.oracle_stages(meta), goldens.used_cams(meta, cams))
    assert got.shape == out.shape and np.array_equal(got, out)


@pytest.mark.parametrize("name", NAMES)
def test_plan_flattening_reproduces_reference(name):
    """libmcs' flattened geometry (nested paste rects, OpenCV-inverted matrices, block widths),
    rendered by the CPU flat gather, equals the reference cascade bit for bit."""
    meta, calib, frames, out = goldens.load_full(name)
    cams = goldens.resized_for_oracle(meta, goldens.sorted_cams(meta, frames))
    ch = 1 if cams[0].ndim == 2 else cams[0].shape[2]
    plan = goldens.plan_for(meta, goldens.sorted_cams(meta, calib), channels=ch)
    assert plan.out_shape()[:2] == tuple(out.shape[:2])
    got = oracle.flat_stitch(plan.describe(), cams)
    assert np.array_equal(got.reshape(out.shape), out)


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


class _Hostile:
    """Pickles as a call of os.system (what a tampered Stitcher_config.pkl could hold)."""

    def __reduce__(self):
        return (os.system, ("echo pickle-ran-os.system >&2",))


@pytest.mark.parametrize("payload", ["os.system", "builtins.eval"])
def test_pickle_loader_refuses_foreign_globals(tmp_path, payload):
    """load_stitcher's unpickler allow-lists the globals a stitcher pickle holds: a pickle naming
    os.system (or eval) is refused before anything runs, while the reference-written
    rig4_mild_Stitcher_config.pkl (test above) still loads."""
    import pickle
    from multicamera_stitching_amd.StitcherClass import Stitcher
    meta, frames, _ = goldens.load("rig4_mild")
    bad = tmp_path / "Stitcher_config.pkl"
    obj = _Hostile() if payload == "os.system" else _Eval()
    bad.write_bytes(pickle.dumps({"stitchers": [obj]}, protocol=2))
    with pytest.raises(pickle.UnpicklingError, match=payload.split(".")[1]):
        Stitcher(dict(frames)).load_stitcher(str(bad))
    pkl = os.path.join(goldens.GOLDEN, "rig4_mild_Stitcher_config.pkl")
    assert isinstance(Stitcher(dict(frames)).load_stitcher(pkl), Stitcher)


class _Eval:
    def __reduce__(self):
        return (eval, ("1 + 1",))


def test_fixture_manifest_is_consistent():
    for name in NAMES:
        meta, frames, out = goldens.load(name)
        assert sorted(frames) == sorted(meta["labels"])
        assert list(out.shape) == meta["out_shape"]
        assert json.dumps(meta)  # plain JSON only


@pytest.mark.parametrize("name", [n for n in NAMES if n.startswith("resize_")])
def test_resize_branch_matches_reference_calls(name):
    """Which frames the drop-in resizes, and to what size, is what the reference's
    StitcherBase.stitch did (:226-233): every recorded cv2.resize that changes (h, w) is one of
    ours; the others (same size, e.g. a channel-only mismatch or the mosaic) are copies."""
    meta, _, frames, _ = goldens.load_full(name)
    cams = goldens.sorted_cams(meta, frames)
    hw = goldens.calibrated_hw(meta)
    ours = sorted((list(c.shape), [w[1], w[0]]) for c, w in zip(cams, hw)
                  if w is not None and tuple(c.shape[:2]) != w)
    ref = sorted((r["src"], r["dsize"]) for r in meta["resize_calls"]
                 if tuple(r["src"][:2]) != (r["dsize"][1], r["dsize"][0]))
    assert ours == ref and ref


def test_resize_known_answers():
    """cv2.resize(INTER_LINEAR) restatement: copy, 2x area mean, border taps, coefficient rounding."""
    a = np.array([[0, 100], [200, 50]], np.uint8)
    assert np.array_equal(oracle.resize_linear(a, (2, 2)), a)
    up = oracle.resize_linear(a, (4, 4))
    # row 0 / col 0 clamp to the first sample; (b0, b1) = (512, 1536) between samples
    assert up[0].tolist() == [0, 25, 75, 100] and up[:, 0].tolist() == [0, 50, 150, 200]
    q = (np.arange(16, dtype=np.uint8).reshape(4, 4) * 10)
    assert oracle.resize_linear(q, (2, 2)).tolist() == [[25, 45], [105, 125]]   # (sum + 2) >> 2
    two = np.array([[[1, 1], [2, 2]], [[3, 3], [4, 4]]], np.uint8)                 # sum 10: tie
    assert oracle.resize_linear(two, (1, 1)).reshape(-1).tolist() == [2, 2]       # half-to-even
    three = np.array([[[1] * 3, [2] * 3], [[3] * 3, [4] * 3]], np.uint8)
    assert oracle.resize_linear(three, (1, 1)).reshape(-1).tolist() == [3, 3, 3]  # (10+2)>>2
    ofs, coef = oracle.resize_axis(3, 7, True)
    assert ofs[0] == 0 and coef[0].tolist() == [2048, 0] and ofs[-1] == 2
    assert coef[-1].tolist() == [2048, 0]
    # separately rounded coefficient pairs can sum to 2049 (f * 2048 and (1 - f) * 2048 both
    # round up) -- the OpenCV 3.4 behaviour the restatement keeps
    sums = set()
    for s_, d_ in ((7, 3), (11, 5), (13, 9), (1920, 1080), (1080, 1920)):
        sums |= set(oracle.resize_axis(s_, d_, False)[1].sum(1).tolist())
    assert sums <= {2047, 2048, 2049}


def test_resize_matches_independent_float_restatement():
    """A second, numpy-only restatement of the same arithmetic agrees on random inputs."""
    rng = np.random.default_rng(3)

    def axis(ss, ds, is_x):
        d = np.arange(ds)
        f = ((d + 0.5) * (1.0 / (ds / ss)) - 0.5).astype(np.float32)
        s_ = np.floor(f).astype(np.int64)
        f = (f - s_.astype(np.float32)).astype(np.float32)
        if is_x:
            lo, hi = s_ < 0, s_ >= ss - 1
            f[lo | hi] = 0
            s_ = np.clip(s_, 0, ss - 1)
        c0 = np.rint((np.float32(1) - f) * np.float32(2048)).astype(np.int64)
        c1 = np.rint(f * np.float32(2048)).astype(np.int64)
        return s_, c0, c1

    for (sw, sh, dw, dh, cn) in ((17, 9, 31, 23, 3), (40, 30, 27, 11, 1), (9, 33, 9, 5, 4)):
        src = rng.integers(0, 256, (sh, sw, cn), dtype=np.uint8)
        sx, a0, a1 = axis(sw, dw, True)
        sy, b0, b1 = axis(sh, dh, False)
        S = src.astype(np.int64)
        x1 = np.minimum(sx + 1, sw - 1)
        one = (sx >= sw - 1)[:, None]

        def hrow(r):
            row = S[np.clip(r, 0, sh - 1)]
            v = row[:, sx] * a0[None, :, None] + row[:, x1] * a1[None, :, None]
            return np.where(one[None], row[:, sx] * 2048, v)

        D0, D1 = hrow(sy), hrow(sy + 1)
        want = ((((b0[:, None, None] * (D0 >> 4)) >> 16) + ((b1[:, None, None] * (D1 >> 4)) >> 16)
                 + 2) >> 2).astype(np.uint8)
        assert np.array_equal(oracle.resize_linear(src, (dw, dh)), want)

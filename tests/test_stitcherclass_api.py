"""Drop-in API behaviour of StitcherClass that needs no GPU: construction, label order, the
reference's fallback branches and return values (StitcherClass.py:114-136, 154-177, 211-256),
persistence, logging, and the PYTHONPATH entry point."""
import importlib
import logging
import os
import subprocess
import sys

import numpy as np
import pytest

from multicamera_stitching_amd import rig
from multicamera_stitching_amd.StitcherClass import Stitcher, StitcherBase

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def images(n=3, w=40, h=30, ch=3):
    return dict(zip(rig.labels(n), rig.make_frames(n, w, h, ch, seed=4)))


def test_labels_sorted_lexicographically_like_np_sort():
    st = Stitcher({"CAM2": 0, "CAM10": 0, "CAM1": 0})
    assert [str(v) for v in st.img_labels] == ["CAM1", "CAM10", "CAM2"]
    assert st.stitcher_labels == ["(CAM1&CAM10)", "((CAM1&CAM10)&CAM2)"]
    assert [s.sid for s in st.stitchers] == st.stitcher_labels
    assert all(isinstance(s, StitcherBase) for s in st.stitchers)


def test_super_mode_propagates():
    st = Stitcher(images(), super_mode=True)
    assert all(s.super_mode for s in st.stitchers)


def test_fewer_images_returns_last_label_image_object(caplog):
    imgs = images()
    st = Stitcher(imgs)
    partial = {"CAM1": imgs["CAM1"], "CAM3": imgs["CAM3"]}
    with caplog.at_level(logging.ERROR, logger="multicamera_stitching_amd"):
        got = st.stitch(partial)
    assert got is imgs["CAM3"]
    assert "inferior" in caplog.text


def test_uncalibrated_chain_returns_first_camera_object():
    imgs = images()
    st = Stitcher(imgs)
    assert st.stitch(imgs) is imgs["CAM1"]


def test_uncalibrated_stage_returns_b():
    sb = StitcherBase(sid="x")
    a, b = np.zeros((2, 2, 3), np.uint8), np.ones((2, 2, 3), np.uint8)
    assert sb.stitch((b, a)) is b


def test_single_camera_returns_it():
    img = np.zeros((4, 4, 3), np.uint8)
    st = Stitcher({"CAM1": img})
    assert st.stitchers == [] and st.stitch({"CAM1": img}) is img


def test_calibrate_without_feature_backend_logs_and_stays_uncalibrated(caplog):
    from multicamera_stitching_amd import features
    if features.available():
        pytest.skip("OpenCV contrib present")
    imgs = images()
    st = Stitcher(imgs)
    with caplog.at_level(logging.ERROR, logger="multicamera_stitching_amd"):
        st.calibrate_stitcher(imgs, save=False)
    assert all(s.cachedAH is None for s in st.stitchers)
    assert "feature" in caplog.text


def test_orb_fallback_is_logged_once(caplog, monkeypatch):
    """Without OpenCV contrib SIFT the drop-in calibrates with GPU ORB: logged once per process,
    at the reference's contrib guard (StitcherClass.py:87-93), never silently."""
    from multicamera_stitching_amd import StitcherClass as sc, features
    monkeypatch.setattr(features, "backend", lambda: "orb")
    monkeypatch.setattr(features, "available", lambda: True)
    monkeypatch.setattr(sc, "_orb_noted", False)
    monkeypatch.delenv("MCS_FEATURES", raising=False)
    # (no GPU here: the stages' feature matching is stubbed to "no homography")
    monkeypatch.setattr(StitcherBase, "calibrate",
                        lambda self, images, *a, **k: self.reset())
    imgs = images()
    with caplog.at_level(logging.WARNING, logger="multicamera_stitching_amd"):
        Stitcher(imgs).calibrate_stitcher(imgs, save=False)
        Stitcher(imgs).calibrate_stitcher(imgs, save=False)
    hits = [r for r in caplog.records if "instead of SIFT" in r.getMessage()]
    assert len(hits) == 1 and "not a contrib version" in hits[0].getMessage()


@pytest.mark.parametrize("code, raises", [(-2, False), (-3, False), (-5, True), (-1, True),
                                         (-4, True)])
def test_gpu_failure_fallback_only_for_runtime_errors(monkeypatch, caplog, code, raises):
    """A run-time failure of the GPU path (MCS_E_HIP / MCS_E_NOMEM) is logged and the fallback
    image returned, as the reference returns images on its expected failures; argument and
    programming errors (MCS_E_INVALID / MCS_E_SHAPE, round 3) and MCS_E_UNSUPPORTED from the call
    (API misuse, advisor finding round 5) raise.  The capacity limits are checked before the call
    (test_capacity_limits_take_the_fallback)."""
    from multicamera_stitching_amd import StitcherClass as sc, _capi
    imgs = images()
    st = Stitcher(imgs)
    st.calibrate_stitcher(imgs, save=False, homographies=[[[1, 0, 30], [0, 1, 2], [0, 0, 1]],
                                                          [[1, 0, 40], [0, 1, 0], [0, 0, 1]]])

    def boom(*a, **k):
        raise _capi.McsError(code, "injected")
    monkeypatch.setattr(sc, "_get_plan", boom)
    if raises:
        with pytest.raises(_capi.McsError):
            st.stitch(imgs)
    else:
        with caplog.at_level(logging.ERROR, logger="multicamera_stitching_amd"):
            out = st.stitch(imgs)
        assert isinstance(out, np.ndarray) and "GPU stitch failed" in caplog.text


def test_capacity_limits_take_the_fallback(monkeypatch, caplog):
    """Inputs the reference handles but the kernels do not -- a channel count outside 1-4 --
    give the logged fallback image, checked before any libmcs call (advisor finding, round 5)."""
    from multicamera_stitching_amd import StitcherClass as sc
    imgs = images()
    st = Stitcher(imgs)
    st.calibrate_stitcher(imgs, save=False, homographies=[[[1, 0, 30], [0, 1, 2], [0, 0, 1]],
                                                          [[1, 0, 40], [0, 1, 0], [0, 0, 1]]])
    called = []
    monkeypatch.setattr(sc, "_get_plan", lambda *a, **k: called.append(1))
    wide = {k: np.concatenate([v, v[:, :, :2]], axis=2) for k, v in imgs.items()}   # 5 channels
    with caplog.at_level(logging.ERROR, logger="multicamera_stitching_amd"):
        out = st.stitch(wide)
    assert isinstance(out, np.ndarray) and not called
    assert "unsupported (5 channels" in caplog.text
    assert sc._capacity_exceeded([np.zeros((4, 4, 3), np.uint8)] * 17).startswith("17 cameras")
    assert sc._capacity_exceeded([np.zeros((4, 4, 3), np.uint8)] * 3) is None


def test_failed_homography_resets_stage():
    imgs = images()
    st = Stitcher(imgs)
    st.calibrate_stitcher(imgs, save=False,
                          homographies=[[[1, 0, 20], [0, 1, 0], [0, 0, 1]], None])
    assert st.stitchers[0].cachedAH is not None
    assert st.stitchers[1].cachedAH is None and st.stitchers[1].BimgSize is None
    assert "Matches:0" in str(st.stitchers[1]) and "None" in str(st.stitchers[1])


def test_calibration_geometry_is_host_only_and_chains_shapes():
    imgs = images()
    st = Stitcher(imgs)
    st.calibrate_stitcher(imgs, save=False, homographies=[[[1, 0, 30], [0, 1, 2], [0, 0, 1]],
                                                          [[1, 0, 60], [0, 1, -3], [0, 0, 1]]])
    s0, s1 = st.stitchers
    assert s0.ABSize == (70, 32) and tuple(s1.BimgSize) == (32, 70, 3)
    assert s1.Bpts[0] == (0, 3)


def test_save_to_unwritable_path_logs(caplog, tmp_path):
    st = Stitcher(images())
    with caplog.at_level(logging.ERROR, logger="multicamera_stitching_amd"):
        st.save_stitcher(str(tmp_path / "no" / "such" / "dir" / "x.pkl"))
    assert "Problem saving" in caplog.text


def test_load_missing_file_returns_self(caplog):
    st = Stitcher(images())
    with caplog.at_level(logging.WARNING, logger="multicamera_stitching_amd"):
        assert st.load_stitcher("/nonexistent/Stitcher_config.pkl") is st
    assert "No Stitcher configuration file" in caplog.text


def test_save_load_roundtrip(tmp_path):
    imgs = images()
    st = Stitcher(imgs, super_mode=True)
    st.calibrate_stitcher(imgs, save=True, save_path=str(tmp_path / "c.pkl"),
                          homographies=[[[1, 0, 30], [0, 1, 2], [0, 0, 1]],
                                        [[0.99, 0.01, 55.5], [0, 1, 1], [1e-4, 0, 1]]])
    st2 = Stitcher(imgs).load_stitcher(str(tmp_path / "c.pkl"))
    for a, b in zip(st.stitchers, st2.stitchers):
        assert np.array_equal(np.asarray(a.cachedAH), np.asarray(b.cachedAH))
        assert isinstance(b.cachedAH, np.ndarray)      # params_to_array after load
        assert a.ABSize == b.ABSize and a.x_limits == b.x_limits and a.super_mode == b.super_mode
    # arrays are back to ndarrays on the saving side too (params_to_array after dump)
    assert isinstance(st.stitchers[0].cachedAH, np.ndarray)


def test_draw_descriptors_is_ignored_with_a_warning(caplog):
    sb = StitcherBase()
    img = np.zeros((3, 3, 3), np.uint8)
    with caplog.at_level(logging.WARNING, logger="multicamera_stitching_amd"):
        assert sb.draw_descriptors(img) is img


def test_geometry_helpers_truncate_toward_zero():
    from multicamera_stitching_amd.geometry import get_projection_point_dst
    M = np.array([[1.0, 0, -0.7], [0, 1, 2.9], [0, 0, 1]])
    assert get_projection_point_dst((0, 0, 1), M) == [0, 2]


def test_pythonpath_entry_point_and_pickle_module_name():
    """`from StitcherClass import Stitcher` with PostScripts/Stitcher on PYTHONPATH (the
    reference's launcher contract, MediaPlayer/visionsystem:8-9) resolves to this drop-in."""
    code = ("import StitcherClass, pickle; "
            "from multicamera_stitching_amd import StitcherClass as S; "
            "assert StitcherClass.Stitcher is S.Stitcher; "
            "assert S.Stitcher.__module__ == 'StitcherClass'; "
            "print('ok')")
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "PostScripts", "Stitcher"))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         cwd="/tmp")
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "ok"


def test_missing_library_fails_loudly(tmp_path):
    code = ("import multicamera_stitching_amd._capi as c; c.LIB_PATH = '/nonexistent/libmcs.so'; "
            "c._lib = None\ntry:\n    c.load()\nexcept ImportError as e:\n    print('raised', e)")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT)
    assert "raised" in out.stdout and "no CPU fallback" in out.stdout


def test_off_size_frames_log_the_reference_warnings(caplog):
    """Frames off their calibrated shape produce the reference's per-stage warnings
    (StitcherClass.py:226-233) and are sized for the GPU resize pre-pass."""
    from multicamera_stitching_amd.StitcherClass import _conform_cameras
    imgs = images()
    st = Stitcher(imgs)
    st.calibrate_stitcher(imgs, save=False, homographies=[[[1, 0, 30], [0, 1, 2], [0, 0, 1]],
                                                          [[1, 0, 60], [0, 1, -3], [0, 0, 1]]])
    shots = [np.zeros((30, 40, 3), np.uint8), np.zeros((25, 33, 3), np.uint8),
             np.zeros((30, 40, 3), np.uint8)]
    with caplog.at_level(logging.WARNING, logger="multicamera_stitching_amd"):
        cams, cam0_hw, sizes = _conform_cameras(st, st.stitchers, shots)
    assert cam0_hw == (30, 40) and sizes == [(40, 30), (33, 25), (40, 30)]
    assert "ImageA size should be (30, 40, 3), Image will be resized" in caplog.text
    assert caplog.text.count("Image will be resized") == 1
    with pytest.raises(ValueError):
        _conform_cameras(st, st.stitchers, [shots[0], shots[1][..., 0], shots[2]])

"""Drop-in replacement of the reference's ``StitcherClass`` module on MI355X.

Reference: PostScripts/Stitcher/StitcherClass.py (Stitcher :50-177, StitcherBase :180-529).
Callers (MediaPlayer/view.py:14,399-411; video_mapping_node.py:37,143-145,177,188) import
``from StitcherClass import Stitcher`` with PostScripts/Stitcher on PYTHONPATH; the module
PostScripts/Stitcher/StitcherClass.py of this repo re-exports this one, and importing this module
also registers it as ``StitcherClass`` so pickles written by either side name the same classes.

What changes: the per-frame pixel work.  ``Stitcher.stitch`` no longer runs N-1 cascaded
cv2.warpPerspective + paste (+ crop) steps on the CPU; the calibrated chain is compiled once into
an mcs plan (flattened nested-paste geometry, OpenCV-inverted matrices) and every call is one
gfx950 gather kernel through libmcs.so (include/mcs.h).  Results are bit-identical to the
reference chain (tests/test_gpu_parity.py).  There is no CPU fallback: without the HIP library
the import fails.

What stays: names, signatures, attribute names (so legacy ``Stitcher_config.pkl`` files load),
the fallback branches and their return values, logging through ``self.debugger``.
"""
from __future__ import annotations

import os
import pickle
import sys
import threading

import numpy as np

from . import _capi
from ._debugger import (DEBUG_LEVEL_0, DEBUG_LEVEL_1, DEBUG_LEVEL_2, DEBUG_LEVEL_3,  # noqa: F401
                        DEBUG_LEVEL_4, Debugger)
from .geometry import get_projection_point_dst, get_projection_point_src  # noqa: F401
from .geometry import stage_geometry

_capi.load()   # fail loudly at import when the HIP library is missing

INTERP = {"linear": _capi.MCS_INTER_LINEAR, "nearest": _capi.MCS_INTER_NEAREST}


def _env_device() -> int:
    try:
        return int(os.environ.get("MCS_DEVICE", "0"))
    except ValueError:
        return 0


def _env_interp() -> int:
    return INTERP.get(os.environ.get("MCS_INTERP", "linear").lower(), _capi.MCS_INTER_LINEAR)


BLEND = {"none": _capi.MCS_BLEND_NONE, "paste": _capi.MCS_BLEND_NONE,
         "feather": _capi.MCS_BLEND_FEATHER, "multiband": _capi.MCS_BLEND_MULTIBAND,
         "seam": _capi.MCS_BLEND_SEAM}


def _env_blend() -> int:
    """MCS_BLEND (extension, default "none" = the reference's overwrite paste, :240-241):
    "feather" / "multiband" blend the seams, "seam" = owner only."""
    return BLEND.get(os.environ.get("MCS_BLEND", "none").lower(), _capi.MCS_BLEND_NONE)


def is_cv3(or_better=False):
    """Reference helper (StitcherClass.py:30-39); False when OpenCV is absent."""
    major = get_opencv_major_version()
    if major is None:
        return False
    return major >= 3 if or_better else major == 3


def get_opencv_major_version(lib=None):
    if lib is None:
        try:
            import cv2 as lib   # noqa: F401  (optional: calibration features only)
        except ImportError:
            return None
    return int(lib.__version__.split(".")[0])


def _stage_desc(sb, b_shape_fallback=None) -> _capi.StageDesc:
    d = _capi.StageDesc()
    if sb.cachedAH is None:
        d.calibrated = 0
        return d
    H = np.asarray(sb.cachedAH, dtype=np.float64).reshape(9)
    d.H[:] = [float(v) for v in H]
    d.calibrated = 1
    d.canvas_w, d.canvas_h = int(sb.ABSize[0]), int(sb.ABSize[1])
    d.b_x, d.b_y = int(sb.Bpts[0][0]), int(sb.Bpts[0][1])
    d.b_w, d.b_h = int(sb.BimgSize[1]), int(sb.BimgSize[0])
    d.a_w, d.a_h = int(sb.AimgSize[1]), int(sb.AimgSize[0])
    d.super_mode = 1 if sb.super_mode else 0
    if sb.super_mode:
        d.x_lim0, d.x_lim1 = int(sb.x_limits[0]), int(sb.x_limits[1])
        d.y_lim0, d.y_lim1 = int(sb.y_limits[0]), int(sb.y_limits[1])
    return d


def _channels(img) -> int:
    return 1 if img.ndim == 2 else int(img.shape[2])


class _PlanCache(object):
    """One compiled plan per (geometry, channels, interp, device) key; not pickled."""

    def __init__(self):
        self.key = None
        self.plan = None
        self.lock = threading.Lock()

    def get(self, key, make):
        if key != self.key or self.plan is None:
            # drop the cache's reference only: a plan handed out by Stitcher.plan() (e.g. to a
            # live StreamPipeline, whose native stream and captured graphs use its tables) stays
            # alive until its last holder lets go (Plan.__del__ -> mcs_plan_destroy)
            self.plan = None
            self.plan = make()
            self.key = key
        return self.plan


def _plan_key(descs, cam0_shape, channels, interp, device):
    k = [tuple(cam0_shape[:2]), channels, interp, device]
    for d in descs:
        k.append((d.calibrated, tuple(d.H), d.canvas_w, d.canvas_h, d.b_x, d.b_y, d.b_w, d.b_h,
                  d.a_w, d.a_h, d.super_mode, d.x_lim0, d.x_lim1, d.y_lim0, d.y_lim1))
    return tuple(k)


class _Transient(object):
    """Mixin: keeps GPU state (plans, locks) out of pickles and deep copies."""

    _TRANSIENT = ("_mcs_cache",)

    def __getstate__(self):
        st = dict(self.__dict__)
        for k in self._TRANSIENT:
            st.pop(k, None)
        return st

    def __setstate__(self, state):
        self.__dict__.update(state)

    def _cache(self) -> _PlanCache:
        c = self.__dict__.get("_mcs_cache")
        if c is None:
            c = _PlanCache()
            self.__dict__["_mcs_cache"] = c
        return c


# =============================================================================================
class Stitcher(_Transient, Debugger):
    """Chained pairwise homography stitcher (reference StitcherClass.py:50-177)."""

    def __init__(self, images_dic, super_mode=False):
        # labels sorted like np.sort(dict.keys()) under Python 2 (lexicographic for str)
        self.img_labels = np.sort(list(images_dic.keys()))
        self.stitcher_labels = []
        for idx, _ in enumerate(self.img_labels[:-1]):
            left = self.img_labels[idx] if idx == 0 else self.stitcher_labels[-1]
            self.stitcher_labels.append("({}&{})".format(left, self.img_labels[idx + 1]))
        self.stitchers = [StitcherBase(sid=label, super_mode=super_mode)
                          for label in self.stitcher_labels]

    # ------------------------------------------------------------------ calibration (once)
    def calibrate_stitcher(self, images_dic, save=True, save_path="", homographies=None):
        """Calibrate every stage on one rig capture, then save (StitcherClass.py:77-112).

        homographies (extension, default None = feature matching like the reference): a list
        with one A->B 3x3 matrix (or None) per stage, or a callable
        ``f(stage_index, stitcher_base, imageB, imageA) -> H or None`` (imageB: the mosaic of
        the earlier stages, stitched as the reference does), for rigs whose homographies are
        known in advance (north-star config 2, synthetic rigs, tests).
        """
        if homographies is None and not _features_available():
            self.debugger(DEBUG_LEVEL_0, "No feature backend for calibration (OpenCV contrib "
                          "SIFT or the mcs feature kernels); pass homographies=",
                          log_type="err")
            return
        if homographies is None:
            _note_orb_fallback(self)
        img_result = None
        for idx, _ in enumerate(self.img_labels[:-1]):
            images = (images_dic[self.img_labels[idx]] if idx == 0 else img_result,
                      images_dic[self.img_labels[idx + 1]])
            H = None
            if homographies is not None:
                H = (homographies(idx, self.stitchers[idx], images[0], images[1])
                     if callable(homographies) else homographies[idx])
            self.stitchers[idx].calibrate(images=images, ratio=0.75, reprojThresh=3.0,
                                          xoffset=0, yoffset=0, homography=H,
                                          use_features=homographies is None)
            if homographies is None or (callable(homographies) and
                                        getattr(homographies, "needs_pixels", True)):
                # the next stage's B is the real mosaic so far: the reference's features, or a
                # callable that may estimate its H from imageB's pixels, see it (a callable that
                # declares needs_pixels = False gets B's shape only, like a list)
                img_result = self.stitchers[idx].stitch(images=images)
            else:
                # a list of matrices needs only the next stage's B shape: no pixels, no GPU work
                img_result = _shape_only(_stage_out_shape(self.stitchers[idx], images[0]))
        for stitcher in self.stitchers:
            self.debugger(DEBUG_LEVEL_0, "[STITCHER]: {}".format(stitcher),
                          log_type="err" if stitcher.status is None else "info")
        self._cache().key = None
        if save:
            self.save_stitcher(save_path)

    # ------------------------------------------------------------------ per-frame hot path
    def stitch(self, images_dic, draw_descriptors=False):
        """Panorama of one rig capture (StitcherClass.py:114-136), one GPU launch."""
        if len(images_dic) > len(self.img_labels):
            self.debugger(DEBUG_LEVEL_0, "[STITCHER] Images dictionary is bigger than list",
                          log_type="warn")
        elif len(images_dic) < len(self.img_labels):
            self.debugger(DEBUG_LEVEL_0, "[STITCHER] Images dictionary is inferior to labels list",
                          log_type="err")
            return images_dic[self.img_labels[-1]]
        if len(self.img_labels) < 2:
            return images_dic[self.img_labels[-1]]
        if draw_descriptors:
            _warn_draw(self)
        cams = [images_dic[label] for label in self.img_labels]
        if all(sb.cachedAH is None for sb in self.stitchers):
            return cams[0]   # every stage returns its B unchanged (:255-256)
        return _run_chain(self, self.stitchers, cams, images_dic[self.img_labels[-1]])

    # ------------------------------------------------------------------ persistence
    def save_stitcher(self, save_path):
        """Pickle the whole chain (StitcherClass.py:138-152); GPU state is not pickled."""
        try:
            with open(save_path, "wb") as output:
                for s in self.stitchers:
                    s.params_to_list()
                try:
                    pickle.dump(self, output, pickle.HIGHEST_PROTOCOL)
                finally:
                    for s in self.stitchers:
                        s.params_to_array()
            self.debugger(DEBUG_LEVEL_0, "[STITCHER]: Stitcher configuration saved")
        except IOError as e:
            self.debugger(DEBUG_LEVEL_0,
                          "[STITCHER]: Problem saving Stitcher configuration: {}".format(e),
                          log_type="err")

    def load_stitcher(self, load_path):
        """Return the unpickled chain, or self when the file is missing (:154-177).

        Reads pickles written by the reference (Python 2 or 3) and by this module.
        """
        loaded = self
        try:
            if os.path.isfile(load_path):
                with open(load_path, "rb") as f:
                    loaded = _StitcherUnpickler(f).load()
                for s in loaded.stitchers:
                    s.params_to_array()
                loaded.debugger(DEBUG_LEVEL_0, "[STITCHER]: Stitcher configuration loaded from file")
            else:
                self.debugger(DEBUG_LEVEL_0, "[STITCHER]: No Stitcher configuration file",
                              log_type="warn")
        except IOError as e:
            self.debugger(DEBUG_LEVEL_0,
                          "[STITCHER]: Problem saving Stitcher configuration: {}".format(e),
                          log_type="err")
        for stitcher in loaded.stitchers:
            loaded.debugger(DEBUG_LEVEL_0, "[STITCHER]: {}".format(stitcher),
                            log_type="err" if stitcher.status is None else "info")
        return loaded

    # ------------------------------------------------------------------ extensions
    def plan(self, channels=3, interp=None, device=None):
        """The compiled mcs plan of the current calibration (for device-resident pipelines)."""
        cam0 = self.stitchers[0].BimgSize if self.stitchers else None
        return _get_plan(self, self.stitchers, cam0, channels, interp, device)


# =============================================================================================
class StitcherBase(_Transient, Debugger):
    """One pairwise stage (reference StitcherClass.py:180-529)."""

    def __init__(self, sid=None, super_mode=False):
        self.sid = sid
        self.super_mode = super_mode
        self.cachedBH = None
        self.cachedBINVH = None
        self.Bpts = None
        self.BimgSize = None
        self.cachedAH = None
        self.cachedAINVH = None
        self.Apts = None
        self.AimgSize = None
        self.matches = None
        self.status = None
        self.ABSize = None
        self.x_limits = None
        self.y_limits = None

    def stitch(self, images, draw_descriptors=False):
        """Warp A onto B's plane and paste B over it (:211-256), on the GPU."""
        (imageB, imageA) = images
        if self.cachedAH is None:
            return imageB
        if draw_descriptors:
            _warn_draw(self)
        return _run_chain(self, [self], [imageB, imageA], imageB)

    def calibrate(self, images, ratio=0.75, reprojThresh=4.0, xoffset=10, yoffset=10,
                  homography=None, use_features=True):
        """Estimate the A->B homography and derive the stage geometry (:258-354).

        homography (extension): use this A->B matrix instead of feature matching.
        """
        self.reset()
        xoffset = abs(xoffset)
        yoffset = abs(yoffset)
        (imageB, imageA) = images
        self.BimgSize = imageB.shape
        self.AimgSize = imageA.shape

        if homography is not None:
            H = np.array(homography, dtype=np.float64, copy=True)
            self.matches, self.status = [], np.ones((0, 1), np.uint8)
        elif use_features:
            kpsA, featuresA = self.detectAndDescribe(imageA)
            kpsB, featuresB = self.detectAndDescribe(imageB)
            if kpsA is None or kpsB is None:
                return
            H, self.matches, self.status = self.matchKeypoints(
                kpsA=kpsA, kpsB=kpsB, featuresA=featuresA, featuresB=featuresB, ratio=ratio,
                reprojThresh=reprojThresh)
        else:
            H = None

        if H is None:
            self.reset()
            return
        g = stage_geometry(H, imageA.shape, imageB.shape, xoffset, yoffset)
        self.cachedAH = g["cachedAH"]
        self.cachedAINVH = g["cachedAINVH"]
        self.cachedBH = g["cachedBH"]
        self.cachedBINVH = g["cachedBINVH"]
        self.Apts = g["Apts"]
        self.Bpts = g["Bpts"]
        self.ABSize = g["ABSize"]
        self.x_limits = g["x_limits"]
        self.y_limits = g["y_limits"]
        self._cache().key = None

    def detectAndDescribe(self, image):
        """Keypoints + descriptors of one image (:356-403); OpenCV SIFT when available."""
        from . import features
        return features.detect_and_describe(self, image)

    def matchKeypoints(self, kpsA, kpsB, featuresA, featuresB, ratio=0.75, reprojThresh=4.0):
        """kNN-2 + Lowe ratio + RANSAC homography (:405-448)."""
        from . import features
        return features.match_keypoints(self, kpsA, kpsB, featuresA, featuresB, ratio,
                                        reprojThresh)

    def draw_descriptors(self, img_src):
        """Debug overlay (:450-483): OpenCV drawing, out of scope for the GPU path."""
        _warn_draw(self)
        return img_src

    def params_to_list(self):
        if self.cachedBH is not None: self.cachedBH = list(self.cachedBH)          # noqa: E701
        if self.cachedBINVH is not None: self.cachedBINVH = list(self.cachedBINVH)  # noqa: E701
        if self.cachedAH is not None: self.cachedAH = list(self.cachedAH)          # noqa: E701
        if self.cachedAINVH is not None: self.cachedAINVH = list(self.cachedAINVH)  # noqa: E701

    def params_to_array(self):
        if self.cachedBH is not None: self.cachedBH = np.asarray(self.cachedBH)          # noqa: E701
        if self.cachedBINVH is not None: self.cachedBINVH = np.asarray(self.cachedBINVH)  # noqa: E701
        if self.cachedAH is not None: self.cachedAH = np.asarray(self.cachedAH)          # noqa: E701
        if self.cachedAINVH is not None: self.cachedAINVH = np.asarray(self.cachedAINVH)  # noqa: E701

    def reset(self):
        for name in ("cachedBH", "cachedBINVH", "Bpts", "cachedAH", "cachedAINVH", "Apts",
                     "matches", "status", "ABSize", "x_limits", "y_limits", "AimgSize",
                     "BimgSize"):
            setattr(self, name, None)

    def __str__(self):
        return "Stitcher:{}| Matches:{}| StitcherSize:{}".format(
            self.sid, len(self.matches) if self.matches is not None else 0, self.ABSize)


# =============================================================================================
# GPU glue shared by Stitcher.stitch and StitcherBase.stitch
def _get_plan(owner, chain, cam0_shape, channels, interp=None, device=None):
    interp = _env_interp() if interp is None else interp
    device = _env_device() if device is None else device
    blend = _env_blend()
    descs = [_stage_desc(sb) for sb in chain]
    key = _plan_key(descs, cam0_shape, channels, interp, device) + (blend,)
    cache = owner._cache()

    def make():
        plan = _capi.Plan(descs, cam0_shape[1], cam0_shape[0], channels, interp, device)
        if blend != _capi.MCS_BLEND_NONE:
            plan.set_blend(blend)
        return plan
    return cache.get(key, make)


def _conform_cameras(owner, chain, cams):
    """The reference's shape checks (:226-233) for the chain's inputs.

    A frame whose shape differs from its calibrated one is logged as the reference logs it and is
    resized on the GPU to the calibrated (h, w) with cv2.resize(INTER_LINEAR) arithmetic, keeping
    its channel count (a same-size "resize" is a copy).  Returns the frames, the calibrated
    (h, w) of camera 0, and each frame's (w, h).
    """
    ch = {_channels(c) for c in cams}
    if len(ch) != 1:
        raise ValueError("cameras with different channel counts cannot be pasted together "
                         "(numpy broadcast error in the reference)")
    tail = tuple(cams[0].shape[2:])         # () for 2-D frames, (C,) for H x W x C
    cam0_hw = None
    b_shape = tuple(cams[0].shape)          # what imageB is at each stage
    for k, sb in enumerate(chain):
        if sb.cachedAH is None:
            continue                         # passthrough: returns B untouched (:255-256)
        if cam0_hw is None:
            cam0_hw = tuple(sb.BimgSize[:2])
        if b_shape != tuple(sb.BimgSize):
            owner.debugger(DEBUG_LEVEL_0, "[STITCHER][{}] ImageB size should be {}, Image will be "
                           "resized".format(sb.sid, sb.BimgSize), log_type="warn")
        a = cams[k + 1]
        if tuple(a.shape) != tuple(sb.AimgSize):
            owner.debugger(DEBUG_LEVEL_0, "[STITCHER][{}] ImageA size should be {}, Image will be "
                           "resized".format(sb.sid, sb.AimgSize), log_type="warn")
        b_shape = _stage_out_shape(sb, _shape_only(tuple(sb.BimgSize[:2]) + tail))
    sizes = [(int(c.shape[1]), int(c.shape[0])) for c in cams]
    return cams, cam0_hw, sizes


_orb_noted = False


def _note_orb_fallback(owner):
    """The reference calibrates with SIFT and refuses to run without OpenCV contrib
    (StitcherClass.py:87-93 logs "OpenCV is not a contrib version ..." and returns).  Where SIFT
    is absent the drop-in calibrates with the GPU ORB + Hamming + RANSAC path instead (SURVEY.md
    8 NS-3..5), whose homographies are not SIFT's: said once per process, at the reference's
    guard."""
    global _orb_noted
    from . import features
    if _orb_noted or features.backend() != "orb":
        return
    _orb_noted = True
    why = ("MCS_FEATURES=orb" if os.environ.get("MCS_FEATURES", "auto").lower() == "orb" else
           "OpenCV is not a contrib version (no xfeatures2d SIFT)")
    owner.debugger(DEBUG_LEVEL_0, "[STITCHER] {}: calibrating with GPU ORB features and "
                   "Hamming matching instead of SIFT; the homographies differ from the "
                   "reference's".format(why), log_type="warn")


# C-ABI statuses (include/mcs.h) _run_chain turns into a logged fallback image: run-time failures
# of the device.  The capacity limits -- inputs the reference handles but the kernels do not
# (more cameras than MCS_MAX_CAMS, a channel count outside 1-4) -- are checked before the call
# (_capacity_exceeded) and take the same logged fallback; every other status, MCS_E_UNSUPPORTED
# included (API misuse), raises.  (More than 8 cameras meeting in one multi-band neighbourhood is
# not an error: those tiles take the feather rule on the GPU.)
_RUNTIME_FAILURES = (_capi.MCS_E_HIP, _capi.MCS_E_NOMEM)


def _capacity_exceeded(cams):
    """Why the kernels cannot take these camera images (None when they can)."""
    if len(cams) > _capi.MCS_MAX_CAMS:
        return "{} cameras (at most {})".format(len(cams), _capi.MCS_MAX_CAMS)
    c = _channels(cams[0]) if cams else 1
    if not 1 <= c <= 4:
        return "{} channels (1-4)".format(c)
    return None


def _run_chain(owner, chain, cams, fallback):
    """One GPU stitch of the chain.  The reference never raises on an expected failure: it logs
    and returns a fallback image (:126-128 the last camera's image, :255-256 B).  A failure of
    the GPU path at run time (MCS_E_HIP, MCS_E_NOMEM: a device allocation or launch that fails) or
    an input the reference handles but these kernels do not (MCS_E_UNSUPPORTED: more cameras than
    MCS_MAX_CAMS, a channel count outside 1-4) is logged the same way and `fallback` is returned --
    the caller's thread (Qt GUI / worker) gets an image, never an exception, and the log says why.
    Argument and programming errors (MCS_E_INVALID, MCS_E_SHAPE) are raised: the reference has no
    catch for them either.  (There is no CPU stitch behind it: a missing libmcs.so fails at import.)"""
    cams, cam0_hw, sizes = _conform_cameras(owner, chain, cams)
    why = _capacity_exceeded(cams)
    if why is not None:
        owner.debugger(DEBUG_LEVEL_0, "[STITCHER] GPU stitch unsupported ({}); returning the "
                       "fallback image".format(why), log_type="err")
        return fallback
    cache = owner._cache()
    with cache.lock:
        try:
            plan = _get_plan(owner, chain, cam0_hw, _channels(cams[0]))
            out = plan.stitch_host(cams, sizes)
            if not getattr(plan, "_dense_logged", False):
                plan._dense_logged = True
                dense = plan.stats().get("mb_degraded_tiles", 0)
                if dense:
                    owner.debugger(DEBUG_LEVEL_0, "[STITCHER] multi-band: {} tiles have more than "
                                   "8 cameras meeting within 16 px; they take the feather "
                                   "blend".format(dense), log_type="warn")
            return out
        except _capi.McsError as e:
            if e.code not in _RUNTIME_FAILURES:
                raise
            cache.key = cache.plan = None     # rebuilt on the next call
            owner.debugger(DEBUG_LEVEL_0, "[STITCHER] GPU stitch failed ({}); returning the "
                           "fallback image".format(e), log_type="err")
            return fallback


def _stage_out_shape(sb, imageB):
    """Shape StitcherBase.stitch would return for this B (:237-256)."""
    if sb.cachedAH is None:
        return tuple(imageB.shape)
    W, H = int(sb.ABSize[0]), int(sb.ABSize[1])
    if sb.super_mode:
        x0, x1, _ = slice(int(sb.x_limits[0]), int(sb.x_limits[1])).indices(W)
        y0, y1, _ = slice(int(sb.y_limits[0]), int(sb.y_limits[1])).indices(H)
        W, H = max(0, x1 - x0), max(0, y1 - y0)
    return (H, W) + tuple(imageB.shape[2:])


def _shape_only(shape):
    return np.broadcast_to(np.zeros((), np.uint8), shape)


def _features_available() -> bool:
    from . import features
    return features.available()


_warned_draw = set()


def _warn_draw(obj):
    if id(type(obj)) not in _warned_draw:
        _warned_draw.add(id(type(obj)))
        obj.debugger(DEBUG_LEVEL_0, "[STITCHER] draw_descriptors is a CPU/OpenCV debug overlay "
                     "and is not drawn on the GPU path", log_type="warn")


class _StitcherUnpickler(pickle.Unpickler):
    """Maps the reference's module name onto this module (Python 2 and 3 pickles)."""

    def __init__(self, f):
        super().__init__(f, encoding="latin1")

    def find_class(self, module, name):
        """Only the globals a Stitcher_config.pkl holds (StitcherClass.py:138-177: the two
        classes, their Debugger base, numpy arrays / scalars / dtypes and the copy_reg
        reconstructor Python 2 writes for them); anything else -- os.system, eval, ... -- is
        refused, so loading a pickle never runs code it names."""
        if module in ("StitcherClass", __name__, "__main__") and name in ("Stitcher",
                                                                           "StitcherBase"):
            return globals()[name]
        if module == "extended_rospylogs" and name == "Debugger":
            return Debugger
        if (module, name) in _PICKLE_ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(
            "Stitcher_config.pkl names {}.{}, which a stitcher pickle never holds".format(module,
                                                                                      name))


# (module, name) pairs a legacy or re-saved stitcher pickle may name besides the classes above:
# numpy's array / scalar / dtype reconstructors (numpy 1.x "core" and 2.x "_core" paths) and the
# Python 2 copy_reg protocol-0/2 object reconstruction.
_PICKLE_ALLOWED = frozenset(
    [("numpy", "ndarray"), ("numpy", "dtype")] +
    [(m + ".multiarray", n) for m in ("numpy.core", "numpy._core")
     for n in ("_reconstruct", "scalar")] +
    [(m + ".numeric", "_frombuffer") for m in ("numpy.core", "numpy._core")] +
    [("copy_reg", "_reconstructor"), ("copyreg", "_reconstructor"),
     ("__builtin__", "object"), ("builtins", "object")])


# Pickles name the reference module so either side can read them.
Stitcher.__module__ = "StitcherClass"
StitcherBase.__module__ = "StitcherClass"
sys.modules.setdefault("StitcherClass", sys.modules[__name__])

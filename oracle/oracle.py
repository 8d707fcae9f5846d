"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper around the CPU restatements in mcs_oracle.c and
orc_resize.c.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module;
the product path (multicamera_stitching_amd) never does.  See mcs_oracle.c for what each
function restates (OpenCV 3.4 warpPerspective/remap/invert as called at
PostScripts/Stitcher/StitcherClass.py:239, and the reference's cascade at :114-136/:211-256).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle.so")
_lib = None

INTER_NEAREST = 0
INTER_LINEAR = 1


class OrcStage(ctypes.Structure):
    _fields_ = [
        ("H", ctypes.c_double * 9),
        ("canvas_w", ctypes.c_int),
        ("canvas_h", ctypes.c_int),
        ("bx", ctypes.c_int),
        ("by", ctypes.c_int),
        ("super_mode", ctypes.c_int),
        ("xl0", ctypes.c_int),
        ("xl1", ctypes.c_int),
        ("yl0", ctypes.c_int),
        ("yl1", ctypes.c_int),
    ]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def build_native(out_path: str, timeout: float = 180.0) -> str:
    """The same restatement built `-O3 -march=native` for the host running this (bench.py's CPU
    baseline: SURVEY.md 8d).  Returns out_path; raises on a failed build."""
    subprocess.run(["make", "-s", "-B", "-C", _HERE, "MARCH=native", "OUT=" + out_path],
                   check=True, timeout=timeout, capture_output=True)
    return out_path


class library:
    """Context manager: the oracle functions use the library at `path` (e.g. build_native's)
    inside the block, the portable liboracle.so again after it."""

    def __init__(self, path: str):
        self.path = path

    def __enter__(self):
        global _lib
        self.saved = _lib
        _lib = _load(self.path)
        return _lib

    def __exit__(self, *exc):
        global _lib
        _lib = self.saved
        return False


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        _lib = _load(_SO)
    return _lib


def _load(path: str):
    L = ctypes.CDLL(path)
    P = ctypes.c_void_p
    L.orc_invert3x3.argtypes = [P, P]
    L.orc_invert3x3.restype = ctypes.c_int
    L.orc_warp_perspective.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_long,
                                       ctypes.c_int, P, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_long, P, ctypes.c_int, ctypes.c_int]
    L.orc_cascade_out_size.argtypes = [P, ctypes.c_int, P, P]
    L.orc_cascade_stitch.argtypes = [P, ctypes.c_int, P, P, P, ctypes.c_int, ctypes.c_int, P]
    L.orc_flat_stitch.argtypes = [ctypes.c_int, P, P, P, P, P, P, P, P, ctypes.c_int,
                                  ctypes.c_int, P, ctypes.c_int, ctypes.c_int]
    L.orc_map_pixel.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                P, P]
    L.orc_bilinear_weights.argtypes = [ctypes.c_int, ctypes.c_int, P]
    L.orc_num_threads.restype = ctypes.c_int
    L.orc_set_num_threads.argtypes = [ctypes.c_int]
    L.orc_resize_linear.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_long,
                                    ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    L.orc_resize_linear.restype = ctypes.c_int
    L.orc_resize_axis.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P]
    L.orc_hamming_knn2.argtypes = [P, ctypes.c_int, P, ctypes.c_int, P, P]
    L.orc_hamming_knn2.restype = None
    L.orc_blend_stitch.argtypes = [ctypes.c_int, P, P, P, P, P, P, P, P, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, P, ctypes.c_int, ctypes.c_int,
                                   P, ctypes.c_int, P]
    L.orc_blend_stitch.restype = ctypes.c_int
    L.orc_blend_stitch_cyl.argtypes = [ctypes.c_int, P, P, P, P, ctypes.c_double,
                                       ctypes.c_double, ctypes.c_double, P, P, P,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, P,
                                       ctypes.c_int, ctypes.c_int, P, ctypes.c_int, P]
    L.orc_blend_stitch_cyl.restype = ctypes.c_int
    L.orc_ransac_homography.argtypes = [P, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                        ctypes.c_uint32, P, P, P]
    L.orc_ransac_homography.restype = ctypes.c_int
    L.orc_homography_refine.argtypes = [P, ctypes.c_int, P, P]
    L.orc_homography_refine.restype = None
    L.orc_orb_detect.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_float, ctypes.c_int, P, P, P, P, P, P]
    L.orc_orb_detect.restype = ctypes.c_int
    L.orc_seam_graphcut.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P,
                                    ctypes.c_int]
    L.orc_seam_graphcut.restype = ctypes.c_int
    L.orc_undistort.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P,
                                ctypes.c_int, P]
    L.orc_undistort.restype = ctypes.c_int
    L.orc_l2_knn2.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, P, P]
    L.orc_l2_knn2.restype = ctypes.c_int
    return L


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def set_threads(n: int):
    lib().orc_set_num_threads(int(n))


def num_threads() -> int:
    return int(lib().orc_num_threads())


def invert3x3(M) -> np.ndarray:
    m = np.ascontiguousarray(np.asarray(M, dtype=np.float64).reshape(9))
    out = np.zeros(9, np.float64)
    lib().orc_invert3x3(_p(m), _p(out))
    return out.reshape(3, 3)


def bilinear_weights(fx: int, fy: int) -> np.ndarray:
    w = np.zeros(4, np.int16)
    lib().orc_bilinear_weights(int(fx), int(fy), _p(w))
    return w


def map_pixel(Minv, interp: int, xb: int, x1: int, y: int):
    m = np.ascontiguousarray(np.asarray(Minv, dtype=np.float64).reshape(9))
    X = ctypes.c_int()
    Y = ctypes.c_int()
    lib().orc_map_pixel(_p(m), interp, xb, x1, y, ctypes.byref(X), ctypes.byref(Y))
    return X.value, Y.value


def warp_perspective(src: np.ndarray, M, dsize, interp: int = INTER_LINEAR,
                     inverse_map: bool = False) -> np.ndarray:
    """cv2.warpPerspective(src, M, dsize=(W, H), flags=interp, BORDER_CONSTANT, 0)."""
    src = np.ascontiguousarray(src, dtype=np.uint8)
    cn = 1 if src.ndim == 2 else src.shape[2]
    sh, sw = src.shape[:2]
    W, H = int(dsize[0]), int(dsize[1])
    dst = np.zeros((H, W, cn) if src.ndim == 3 else (H, W), np.uint8)
    m = np.ascontiguousarray(np.asarray(M, dtype=np.float64).reshape(9))
    lib().orc_warp_perspective(_p(src), sw, sh, sw * cn, cn, _p(dst), W, H, W * cn, _p(m),
                               interp, 1 if inverse_map else 0)
    return dst


def undistort(src: np.ndarray, K, dist=None) -> np.ndarray:
    """cv2.undistort(src, K, dist) (orc_undistort.c, OpenCV 3.4 semantics)."""
    src = np.ascontiguousarray(src, dtype=np.uint8)
    cn = 1 if src.ndim == 2 else src.shape[2]
    h, w = src.shape[:2]
    A = np.ascontiguousarray(np.asarray(K, np.float64).reshape(9))
    d = np.ascontiguousarray(np.zeros(0) if dist is None else
                             np.asarray(dist, np.float64).reshape(-1))
    dst = np.zeros_like(src)
    if lib().orc_undistort(_p(src), w, h, cn, _p(A), _p(d) if d.size else None, int(d.size),
                           _p(dst)) != 0:
        raise ValueError("orc_undistort: unsupported distortion vector")
    return dst


def resize_linear(src: np.ndarray, dsize) -> np.ndarray:
    """cv2.resize(src, dsize=(W, H), interpolation=cv2.INTER_LINEAR) (orc_resize.c)."""
    src = np.ascontiguousarray(src, dtype=np.uint8)
    cn = 1 if src.ndim == 2 else src.shape[2]
    sh, sw = src.shape[:2]
    W, H = int(dsize[0]), int(dsize[1])
    dst = np.zeros((H, W, cn) if src.ndim == 3 else (H, W), np.uint8)
    if lib().orc_resize_linear(_p(src), sw, sh, sw * cn, cn, _p(dst), W, H, W * cn) != 0:
        raise ValueError("orc_resize_linear failed")
    return dst


def resize_axis(ssize: int, dsize: int, is_x: bool):
    """OpenCV resize() per-axis source index and 11-bit coefficient pairs."""
    ofs = np.zeros(dsize, np.int32)
    coef = np.zeros(2 * dsize, np.int16)
    lib().orc_resize_axis(ssize, dsize, 1 if is_x else 0, _p(ofs), _p(coef))
    return ofs, coef.reshape(dsize, 2)


def hamming_knn2(query: np.ndarray, train: np.ndarray):
    """BFMatcher(NORM_HAMMING).knnMatch(query, train, k=2) on N x 32-byte descriptors
    (orc_match.c): (idx (nq, 2), dist (nq, 2)), -1 where no candidate."""
    q = np.ascontiguousarray(query, dtype=np.uint8).reshape(-1, 32)
    t = np.ascontiguousarray(train, dtype=np.uint8).reshape(-1, 32)
    idx = np.empty((q.shape[0], 2), np.int32)
    dist = np.empty((q.shape[0], 2), np.int32)
    lib().orc_hamming_knn2(_p(q), q.shape[0], _p(t), t.shape[0], _p(idx), _p(dist))
    return idx, dist


def l2_knn2(query, train):
    """BFMatcher(NORM_L2).knnMatch(k=2) of float descriptors (orc_match.c): (idx, dist, exact)."""
    q = np.ascontiguousarray(query, np.float32)
    t = np.ascontiguousarray(train, np.float32)
    dim = q.shape[1]
    idx = np.empty((q.shape[0], 2), np.int32)
    dist = np.empty((q.shape[0], 2), np.float32)
    ex = lib().orc_l2_knn2(_p(q), q.shape[0], _p(t), t.shape[0] if t.size else 0, dim, _p(idx),
                           _p(dist))
    return idx, dist, bool(ex)


def _stage_array(stages):
    arr = (OrcStage * len(stages))()
    for i, s in enumerate(stages):
        arr[i].H[:] = [float(v) for v in np.asarray(s["H"], np.float64).reshape(9)]
        arr[i].canvas_w, arr[i].canvas_h = int(s["canvas_w"]), int(s["canvas_h"])
        arr[i].bx, arr[i].by = int(s["bx"]), int(s["by"])
        arr[i].super_mode = 1 if s.get("super_mode") else 0
        xl = s.get("x_limits") or (0, 0)
        yl = s.get("y_limits") or (0, 0)
        arr[i].xl0, arr[i].xl1 = int(xl[0]), int(xl[1])
        arr[i].yl0, arr[i].yl1 = int(yl[0]), int(yl[1])
    return arr


def cascade_stitch(stages, cams, interp: int = INTER_LINEAR) -> np.ndarray:
    """Reference-structured cascade (per-stage full canvas warp + paste + crop).

    stages: list of dicts {H, canvas_w, canvas_h, bx, by, super_mode, x_limits, y_limits}
    cams: camera images in sorted-label order (len(stages)+1), all with the same channels.
    """
    n = len(stages)
    arr = _stage_array(stages)
    cams = [np.ascontiguousarray(c, dtype=np.uint8) for c in cams]
    cn = 1 if cams[0].ndim == 2 else cams[0].shape[2]
    ow = ctypes.c_int()
    oh = ctypes.c_int()
    L = lib()
    if L.orc_cascade_out_size(ctypes.byref(arr), n, ctypes.byref(ow), ctypes.byref(oh)) != 0:
        raise ValueError("no stages")
    out = np.zeros((oh.value, ow.value, cn) if cams[0].ndim == 3 else (oh.value, ow.value),
                   np.uint8)
    ptrs = (ctypes.c_void_p * len(cams))(*[c.ctypes.data for c in cams])
    cw = np.array([c.shape[1] for c in cams], np.int32)
    ch = np.array([c.shape[0] for c in cams], np.int32)
    rc = L.orc_cascade_stitch(ctypes.byref(arr), n, ptrs, _p(cw), _p(ch), cn, interp, _p(out))
    if rc != 0:
        raise ValueError("paste rectangle does not fit the canvas (numpy broadcast error)")
    return out


def flat_stitch(flat: dict, cams, interp: int = INTER_LINEAR) -> np.ndarray:
    """CPU flattened gather through the nested rects (see mcs_oracle.c orc_flat_stitch).

    flat: {n_stages, off_x[n+1], off_y[n+1], rect[n][4], minv[n][9], bw0[n], cam[n], out_w,
    out_h} as returned by libmcs' mcs_plan_describe; cams: all cameras in sorted-label order.
    """
    n = int(flat["n_stages"])
    offx = np.ascontiguousarray(flat["off_x"], np.int32)
    offy = np.ascontiguousarray(flat["off_y"], np.int32)
    rect = np.ascontiguousarray(flat["rect"], np.int32).reshape(-1)
    minv = np.ascontiguousarray(flat["minv"], np.float64).reshape(-1)
    bw0 = np.ascontiguousarray(flat["bw0"], np.int32)
    cams = [np.ascontiguousarray(c, dtype=np.uint8) for c in cams]
    # the C routine samples cams[s + 1] for stage s: reorder by the plan's camera map
    cams = [cams[0]] + [cams[int(c)] for c in flat.get("cam", range(1, n + 1))]
    cn = 1 if cams[0].ndim == 2 else cams[0].shape[2]
    ow, oh = int(flat["out_w"]), int(flat["out_h"])
    out = np.zeros((oh, ow, cn) if cams[0].ndim == 3 else (oh, ow), np.uint8)
    ptrs = (ctypes.c_void_p * len(cams))(*[c.ctypes.data for c in cams])
    cw = np.array([c.shape[1] for c in cams], np.int32)
    ch = np.array([c.shape[0] for c in cams], np.int32)
    lib().orc_flat_stitch(n, _p(offx), _p(offy), _p(rect), _p(minv), _p(bw0), ptrs, _p(cw),
                          _p(ch), cn, interp, _p(out), ow, oh)
    return out


BLEND_FEATHER = 1
BLEND_MULTIBAND = 2
BLEND_SEAM = 3


def _seam_buf(ow, oh, seam_k, seam_labels=None):
    """(k argument, label buffer): seam_labels (the 2^seam_k grid, e.g. a plan's graph-cut seams
    found once from another capture) are passed in as k + 256 (orc_blend.c)."""
    if seam_k is None or seam_k < 0:
        return -1, np.zeros(1, np.uint8)
    k = int(seam_k)
    shape = (((oh + (1 << k) - 1) >> k), ((ow + (1 << k) - 1) >> k))
    if seam_labels is not None:
        lab = np.ascontiguousarray(seam_labels, np.uint8).copy()
        if lab.shape != shape:
            raise ValueError(f"seam labels {lab.shape}, grid {shape}")
        return k + 256, lab
    return k, np.zeros(shape, np.uint8)


def blend_stitch(flat: dict, cams, mode: int, interp: int = INTER_LINEAR, want_owner=False,
                 seam_k=None, want_seams=False, seam_labels=None):
    """Blended mosaic of the plan's geometry (orc_blend.c: FEATHER = 1, MULTIBAND = 2,
    SEAM = 3).  flat: mcs_plan_describe dict; cams: all cameras in sorted-label order,
    calibrated sizes.  seam_k: graph-cut seams on the 2^k grid (orc_seam.c), None = distance."""
    n = int(flat["n_stages"])
    offx = np.ascontiguousarray(flat["off_x"], np.int32)
    offy = np.ascontiguousarray(flat["off_y"], np.int32)
    minv = np.ascontiguousarray(flat["minv"], np.float64).reshape(-1)
    bw0 = np.ascontiguousarray(flat["bw0"], np.int32)
    scam = np.ascontiguousarray(flat["cam"], np.int32)
    cams = [np.ascontiguousarray(c, dtype=np.uint8) for c in cams]
    cn = 1 if cams[0].ndim == 2 else cams[0].shape[2]
    ow, oh = int(flat["out_w"]), int(flat["out_h"])
    out = np.zeros((oh, ow, cn) if cams[0].ndim == 3 else (oh, ow), np.uint8)
    owner = np.zeros((oh, ow), np.uint8)
    ptrs = (ctypes.c_void_p * len(cams))(*[c.ctypes.data for c in cams])
    cw = np.array([c.shape[1] for c in cams], np.int32)
    ch = np.array([c.shape[0] for c in cams], np.int32)
    k, lab = _seam_buf(ow, oh, seam_k, seam_labels)
    rc = lib().orc_blend_stitch(n, _p(offx), _p(offy), _p(minv), _p(bw0), _p(scam), ptrs, _p(cw),
                                _p(ch), cn, interp, mode, _p(out), ow, oh, _p(owner), k, _p(lab))
    if rc != 0:
        raise ValueError("orc_blend_stitch failed")
    return _ret(out, owner, lab, want_owner, want_seams)


def _ret(out, owner, lab, want_owner, want_seams):
    r = (out,) + ((owner,) if want_owner else ()) + ((lab,) if want_seams else ())
    return r if len(r) > 1 else out


def blend_stitch_cyl(rig: list, out_w: int, out_h: int, f_cyl: float, u0: float, v0: float,
                     cams, mode: int, interp: int = INTER_LINEAR, want_owner=False, seam_k=None,
                     want_seams=False, seam_labels=None):
    """Cylindrical panorama (orc_blend.c orc_blend_stitch_cyl): rig = [dict(R, f, cx, cy)] per
    camera (as mcs_plan_create_cylindrical), cams = the frames; owner values = camera index."""
    n = len(rig)
    R = np.ascontiguousarray(np.concatenate([np.asarray(c["R"], np.float64).reshape(9)
                                             for c in rig]))
    f = np.array([c["f"] for c in rig], np.float64)
    cx = np.array([c["cx"] for c in rig], np.float64)
    cy = np.array([c["cy"] for c in rig], np.float64)
    cams = [np.ascontiguousarray(c, dtype=np.uint8) for c in cams]
    cn = 1 if cams[0].ndim == 2 else cams[0].shape[2]
    out = np.zeros((out_h, out_w, cn) if cams[0].ndim == 3 else (out_h, out_w), np.uint8)
    owner = np.zeros((out_h, out_w), np.uint8)
    ptrs = (ctypes.c_void_p * n)(*[c.ctypes.data for c in cams])
    cw = np.array([c.shape[1] for c in cams], np.int32)
    ch = np.array([c.shape[0] for c in cams], np.int32)
    k, lab = _seam_buf(out_w, out_h, seam_k, seam_labels)
    rc = lib().orc_blend_stitch_cyl(n, _p(R), _p(f), _p(cx), _p(cy), float(f_cyl), float(u0),
                                    float(v0), ptrs, _p(cw), _p(ch), cn, interp, mode, _p(out),
                                    int(out_w), int(out_h), _p(owner), k, _p(lab))
    if rc != 0:
        raise ValueError("orc_blend_stitch_cyl failed")
    return _ret(out, owner, lab, want_owner, want_seams)


def seam_graphcut(labels, cover, samples):
    """orc_seam.c on caller inputs (see _capi.seam_graphcut_host): returns the cut labels."""
    lab = np.ascontiguousarray(labels, np.uint8).copy()
    cov = np.ascontiguousarray(cover, np.uint16)
    smp = np.ascontiguousarray(samples, np.uint8)
    n, gh, gw = smp.shape[0], lab.shape[0], lab.shape[1]
    C = 1 if smp.ndim == 3 else smp.shape[3]
    if lib().orc_seam_graphcut(n, gw, gh, _p(lab), _p(cov), _p(smp), C) != 0:
        raise ValueError("orc_seam_graphcut failed")
    return lab


def ransac_homography(src, dst, thresh, iters=2000, seed=0):
    """RANSAC homography per csrc/mcs_ransac_core.h (orc_ransac.c): (H or None, mask, best_k,
    per-hypothesis scores).  src/dst: (n, 2) float32 (converted to double like the GPU path)."""
    src = np.asarray(src, np.float32).reshape(-1, 2)
    dst = np.asarray(dst, np.float32).reshape(-1, 2)
    pts = np.ascontiguousarray(np.concatenate([src, dst], axis=1).astype(np.float64))
    n = pts.shape[0]
    scores = np.zeros(iters, np.int32)
    mask = np.zeros(n, np.uint8)
    H = np.zeros(9, np.float64)
    best = lib().orc_ransac_homography(_p(pts), n, float(thresh), iters, seed & 0xffffffff,
                                       _p(scores), _p(mask), _p(H))
    return (None if best < 0 else H.reshape(3, 3)), mask, best, scores


def homography_refine(src, dst, mask, H):
    """findHomography's post-RANSAC refinement restated (orc_ransac.c orc_homography_refine):
    normalised DLT on the inliers + 10 LM iterations, starting from the 3x3 model H."""
    src = np.asarray(src, np.float32).reshape(-1, 2)
    dst = np.asarray(dst, np.float32).reshape(-1, 2)
    pts = np.ascontiguousarray(np.concatenate([src, dst], axis=1).astype(np.float64))
    m = np.ascontiguousarray(np.asarray(mask).reshape(-1), np.uint8)
    h = np.ascontiguousarray(np.asarray(H, np.float64).reshape(9)).copy()
    lib().orc_homography_refine(_p(pts), pts.shape[0], _p(m), _p(h))
    return h.reshape(3, 3)


def orb_pattern() -> np.ndarray:
    """The 256 x 4 rBRIEF pattern (OpenCV bit_pattern_31_) -- data, read from the generated
    header the GPU code compiles (csrc/mcs_orb_pattern.h, tools/gen_orb_pattern.py)."""
    import re
    hdr = os.path.join(os.path.dirname(_HERE), "multicamera_stitching_amd", "csrc",
                       "mcs_orb_pattern.h")
    body = open(hdr).read().split("kOrbPattern[256][4] = {", 1)[1]
    vals = [int(v) for v in re.findall(r"-?\d+", body.split("};", 1)[0])]
    pat = np.array(vals, np.int32).reshape(256, 4)
    assert pat[0].tolist() == [8, -3, 9, 5]
    return pat


def orb_detect(gray, nfeatures=2000, nlevels=8, scale_factor=1.2, threshold=20):
    """ORB per csrc/mcs_orb_core.h (orc_orb.c): dict of xy (n, 2) float32, response (n,)
    float64, level (n,), cs_sn (n, 2) orientation (cos, sin), desc (n, 32) uint8."""
    g = np.ascontiguousarray(gray, np.uint8)
    h, w = g.shape
    pat = np.ascontiguousarray(orb_pattern())
    xy = np.zeros((nfeatures, 2), np.float32)
    resp = np.zeros(nfeatures, np.float64)
    lvl = np.zeros(nfeatures, np.int32)
    cs = np.zeros((nfeatures, 2), np.float64)
    desc = np.zeros((nfeatures, 32), np.uint8)
    n = lib().orc_orb_detect(_p(g), w, h, nfeatures, nlevels, scale_factor, threshold, _p(pat),
                             _p(xy), _p(resp), _p(lvl), _p(cs), _p(desc))
    if n < 0:
        raise ValueError("orc_orb_detect failed")
    return dict(xy=xy[:n], response=resp[:n], level=lvl[:n], cs_sn=cs[:n], desc=desc[:n])

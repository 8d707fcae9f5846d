"""Drop-ins for the OpenCV calls either side of the stitch on the reference's per-frame path
(SURVEY.md section 8f-4): cv2.undistort before stitching (video_mapping_node.py:157-158,
MediaPlayer/view.py:380-381) and the extrinsic bird's-eye cv2.warpPerspective of the display path
(view.py:387-388, Calibration_Utils/Extrinsic.py:99).  Same signatures and results (bit-exact
with the OpenCV 3.4 arithmetic restated in oracle/); each distinct (matrix, coefficients, shape)
builds one plan, kept for the next frame, so the per-frame cost is the plan's remap on the GPU.
No CPU fallback: without libmcs.so these raise."""
from __future__ import annotations

import threading

import numpy as np

from . import _capi

_plans: dict = {}
_lock = threading.Lock()
_MAX_PLANS = 64


def _shape(src):
    src = np.ascontiguousarray(src, dtype=np.uint8)
    if src.ndim not in (2, 3) or (src.ndim == 3 and not 1 <= src.shape[2] <= 4):
        raise ValueError(f"u8 H x W (x 1..4) image expected, got {src.shape}")
    return src, src.shape[0], src.shape[1], (1 if src.ndim == 2 else src.shape[2])


def _cached(key, make):
    with _lock:
        plan = _plans.get(key)
        if plan is None:
            if len(_plans) >= _MAX_PLANS:
                _plans.pop(next(iter(_plans))).close()
            plan = _plans[key] = make()
        return plan


def undistort(src, cameraMatrix, distCoeffs=None, device: int = 0):
    """cv2.undistort(src, cameraMatrix, distCoeffs) (newCameraMatrix = cameraMatrix)."""
    src, h, w, c = _shape(src)
    K = np.asarray(cameraMatrix, np.float64).reshape(3, 3)
    d = np.zeros(0) if distCoeffs is None else np.asarray(distCoeffs, np.float64).reshape(-1)
    key = ("u", K.tobytes(), d.tobytes(), w, h, c, device)
    plan = _cached(key, lambda: _capi.Plan.undistort(K, d, w, h, c, device))
    return plan.stitch_host([src]).reshape(src.shape)


def warpPerspective(src, M, dsize, flags: int = 1, device: int = 0):
    """cv2.warpPerspective(src, M, dsize, flags=INTER_LINEAR (1) or INTER_NEAREST (0))."""
    src, h, w, c = _shape(src)
    M = np.asarray(M, np.float64).reshape(3, 3)
    W, H = int(dsize[0]), int(dsize[1])
    interp = _capi.MCS_INTER_NEAREST if flags == 0 else _capi.MCS_INTER_LINEAR
    if flags not in (0, 1):
        raise ValueError("flags: INTER_NEAREST (0) or INTER_LINEAR (1)")
    key = ("w", M.tobytes(), w, h, W, H, c, interp, device)
    plan = _cached(key, lambda: _capi.Plan.warp(M, w, h, W, H, c, interp, device))
    out = plan.stitch_host([src])
    return out.reshape((H, W) if src.ndim == 2 else (H, W, c))

"""Synthetic camera rigs for the bench and the tests.

A rig is a row of cameras looking at a plane.  Camera k maps its pixels to the world plane with
C_k = T(k*s, 0) . R(theta_k) . S(sigma_k) . P(p_k)  (s = (1 - overlap) * W), so the homography a
perfect matcher would return for stage k of the reference chain (A = camera k+1, B = mosaic of
cameras 0..k, StitcherClass.py:99-104) is
    H_k = T(o_k) . C_0^-1 . C_{k+1},
where o_k is where camera 0's origin sits in the stage-k mosaic: the sum over earlier stages of
their paste offset Bpts[0] minus their super-mode crop origin.  No feature matching is involved
(north-star config 2: "precomputed homographies").

Frames are procedural u8 textures (sum of sinusoids + 64 px checker + noise, clipped to
[1, 255] so that 0 always means "no camera here").
"""
from __future__ import annotations

import numpy as np


def _T(tx, ty):
    return np.array([[1.0, 0.0, tx], [0.0, 1.0, ty], [0.0, 0.0, 1.0]])


def _R(theta):
    c, s = np.cos(theta), np.sin(theta)
    return np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])


def _S(sigma):
    return np.diag([sigma, sigma, 1.0])


def _P(p1, p2):
    return np.array([[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [p1, p2, 1.0]])


def camera_models(n_cams, width, height, overlap=0.25, seed=0, rot_deg=0.5, scale_jitter=0.01,
                  persp=2e-6, step=None):
    """List of C_k (camera pixel -> world) for a left-to-right rig."""
    s = (1.0 - overlap) * width if step is None else step
    out = []
    for k in range(n_cams):
        rng = np.random.default_rng(1000 + seed * 97 + k)
        th = np.deg2rad(rng.uniform(-rot_deg, rot_deg))
        sg = 1.0 + rng.uniform(-scale_jitter, scale_jitter)
        p1, p2 = rng.uniform(-persp, persp, size=2)
        out.append(_T(k * s, 0.0) @ _R(th) @ _S(sg) @ _P(p1, p2))
    return out


def cam0_origin(prev_stages):
    """Position of camera 0's origin in the mosaic produced by `prev_stages` (StitcherBase list)."""
    ox, oy = 0, 0
    for sb in prev_stages:
        if sb.cachedAH is None:
            continue
        ox += int(sb.Bpts[0][0])
        oy += int(sb.Bpts[0][1])
        if sb.super_mode:
            ox -= int(sb.x_limits[0])
            oy -= int(sb.y_limits[0])
    return ox, oy


def stage_homography(C, k, prev_stages):
    """A->B homography of stage k (camera k+1 onto the stage-k mosaic), H[2][2] = 1."""
    ox, oy = cam0_origin(prev_stages)
    H = _T(ox, oy) @ np.linalg.inv(C[0]) @ C[k + 1]
    return H / H[2, 2]


def homography_provider(C, chain_getter):
    """Callable for Stitcher.calibrate_stitcher(homographies=...)."""
    def provide(idx, stitcher_base, imageB, imageA):
        chain = chain_getter()
        return stage_homography(C, idx, chain[:idx])
    provide.needs_pixels = False    # the rig's H follow from the camera models and the chain
    return provide


def texture(h, w, channels=3, seed=0):
    """Procedural u8 image in [1, 255]."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    base = np.zeros((h, w), np.float32)
    for _ in range(8):
        fx, fy = rng.uniform(0.002, 0.08, size=2)
        ph = rng.uniform(0, 2 * np.pi)
        base += np.sin(fx * xx + fy * yy + ph).astype(np.float32)
    base = 128.0 + 12.0 * base
    checker = (((xx // 64) + (yy // 64)) % 2).astype(np.float32) * 40.0 - 20.0
    base += checker
    chans = []
    for c in range(channels):
        noise = rng.uniform(-8, 8, size=(h, w)).astype(np.float32)
        tint = rng.uniform(-30, 30)
        chans.append(base + noise + tint)
    img = np.clip(np.stack(chans, axis=-1), 1, 255).astype(np.uint8)
    return img[..., 0] if channels == 1 else img


def make_frames(n_cams, width, height, channels=3, seed=0):
    return [texture(height, width, channels, seed=seed * 131 + k) for k in range(n_cams)]


def world_frames(C, width, height, channels=3, seed=0, world_fn=None):
    """Camera frames rendered from ONE shared world texture through the camera models C (so
    overlaps agree up to interpolation, as with a real rig); float bilinear, numpy.  world_fn(h,
    w, channels, seed) -> u8 image replaces the default procedural texture."""
    corners = np.array([[0, 0, 1], [width - 1, 0, 1], [0, height - 1, 1],
                        [width - 1, height - 1, 1]], np.float64).T
    pts = []
    for Ck in C:
        q = Ck @ corners
        pts.append(q[:2] / q[2])
    pts = np.concatenate(pts, axis=1)
    x0, y0 = np.floor(pts.min(axis=1)) - 2
    x1, y1 = np.ceil(pts.max(axis=1)) + 2
    make = world_fn or texture
    world = make(int(y1 - y0) + 1, int(x1 - x0) + 1, channels, seed=seed).astype(np.float64)
    if world.ndim == 2:
        world = world[..., None]
    v, u = np.mgrid[0:height, 0:width].astype(np.float64)
    frames = []
    for Ck in C:
        X = Ck[0, 0] * u + Ck[0, 1] * v + Ck[0, 2]
        Y = Ck[1, 0] * u + Ck[1, 1] * v + Ck[1, 2]
        W = Ck[2, 0] * u + Ck[2, 1] * v + Ck[2, 2]
        X = X / W - x0
        Y = Y / W - y0
        xi = np.clip(np.floor(X).astype(np.int64), 0, world.shape[1] - 2)
        yi = np.clip(np.floor(Y).astype(np.int64), 0, world.shape[0] - 2)
        fx = np.clip(X - xi, 0, 1)[..., None]
        fy = np.clip(Y - yi, 0, 1)[..., None]
        img = (world[yi, xi] * (1 - fx) * (1 - fy) + world[yi, xi + 1] * fx * (1 - fy) +
               world[yi + 1, xi] * (1 - fx) * fy + world[yi + 1, xi + 1] * fx * fy)
        img = np.clip(np.rint(img), 1, 255).astype(np.uint8)
        frames.append(img if channels > 1 else img[..., 0])
    return frames


def corner_texture(h, w, seed=0, n_rects=None):
    """Feature-rich u8 gray test image: random axis-aligned rectangles of random gray levels over
    a mid-gray background (corners for FAST/ORB), clipped to [1, 255]."""
    rng = np.random.default_rng(seed)
    img = np.full((h, w), 128, np.int32)
    for _ in range(n_rects or max(8, h * w // 900)):
        x0, y0 = rng.integers(0, w), rng.integers(0, h)
        rw, rh = rng.integers(4, max(5, w // 8)), rng.integers(4, max(5, h // 8))
        img[y0:y0 + rh, x0:x0 + rw] = rng.integers(0, 256)
    return np.clip(img, 1, 255).astype(np.uint8)


def corner_world(h, w, channels=3, seed=0):
    """World texture for estimation rigs (ORB needs corners): corner_texture with a small
    per-channel tint, clipped to [1, 255] (world_frames' world_fn)."""
    g = corner_texture(h, w, seed=seed).astype(np.int32)
    tint = np.array([0, 7, -9, 4][:channels], np.int32)
    return np.clip(g[..., None] + tint, 1, 255).astype(np.uint8)


def estimation_rig(n_cams=4, width=1920, height=1080, channels=3, seed=0):
    """(C, frames, truth) of a rig rendered from one shared corner world:
    truth[k] = the exact homography camera k+1 -> camera k (H[2][2] = 1)."""
    C = camera_models(n_cams, width, height, seed=seed)
    frames = world_frames(C, width, height, channels, seed=seed, world_fn=corner_world)
    truth = []
    for k in range(n_cams - 1):
        T = np.linalg.inv(C[k]) @ C[k + 1]
        truth.append(T / T[2, 2])
    return C, frames, truth


def labels(n_cams):
    return ["CAM{}".format(i + 1) for i in range(n_cams)]


def calibrated_stitcher(n_cams=4, width=1920, height=1080, channels=3, super_mode=False,
                        seed=0, **cam_kw):
    """(Stitcher, frames dict, C) for a synthetic rig, calibrated with exact homographies."""
    from .StitcherClass import Stitcher
    frames = make_frames(n_cams, width, height, channels, seed)
    images = dict(zip(labels(n_cams), frames))
    st = Stitcher(images, super_mode=super_mode)
    C = camera_models(n_cams, width, height, seed=seed, **cam_kw)
    st.calibrate_stitcher(images, save=False,
                          homographies=homography_provider(C, lambda: st.stitchers))
    return st, images, C


def _rot(axis, a):
    c, s = np.cos(a), np.sin(a)
    if axis == "x":
        return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])
    if axis == "y":
        return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def cylinder_rig(n_cams=8, width=1920, height=1080, f=1100.0, channels=3, seed=0,
                 jitter_deg=0.0, gain=0.06):
    """Rotation-only 360 degree rig (8 cameras at 45 degree yaw steps,
    f = 1100 px) and its frames rendered from ONE cylindrical world texture (float bilinear,
    numpy; per-camera gain in [1 - gain, 1 + gain] so that seams show).  Camera k looks along
    yaw 2 pi k / n (plus pitch/roll/yaw jitter); R maps rig rays to camera rays (x right,
    y down, z forward).  Returns (cams, frames, geometry) with cams as
    mcs_plan_create_cylindrical takes them and geometry = dict(out_w, out_h, f_cyl, u0, v0)
    (full circle at the cameras' focal length, panorama centre on camera 0)."""
    rng = np.random.default_rng(seed)
    f_cyl = float(f)
    out_w = int(round(2 * np.pi * f_cyl))
    out_h = int(height)
    u0, v0 = out_w / 2.0, (out_h - 1) / 2.0
    cams = []
    for k in range(n_cams):
        j = np.deg2rad(rng.uniform(-jitter_deg, jitter_deg, size=3)) if jitter_deg else (0, 0, 0)
        yaw = 2 * np.pi * k / n_cams + j[0]
        # camera -> rig: yaw about y, then pitch about x, then roll about z (camera frame)
        C = _rot("y", yaw) @ _rot("x", j[1]) @ _rot("z", j[2])
        cams.append(dict(R=np.ascontiguousarray(C.T), f=float(f), cx=(width - 1) / 2.0,
                         cy=(height - 1) / 2.0, w=int(width), h=int(height)))
    pad = 48
    world = texture(out_h + 2 * pad, out_w + 2 * pad, channels, seed=seed).astype(np.float64)
    if world.ndim == 2:
        world = world[..., None]
    v, u = np.mgrid[0:height, 0:width].astype(np.float64)
    frames = []
    for c in cams:
        rx, ry = (u - c["cx"]) / c["f"], (v - c["cy"]) / c["f"]
        Rt = c["R"].T   # camera -> rig
        dx = Rt[0, 0] * rx + Rt[0, 1] * ry + Rt[0, 2]
        dy = Rt[1, 0] * rx + Rt[1, 1] * ry + Rt[1, 2]
        dz = Rt[2, 0] * rx + Rt[2, 1] * ry + Rt[2, 2]
        th = np.arctan2(dx, dz)
        hh = dy / np.hypot(dx, dz)
        X = np.mod(th * f_cyl + u0, out_w) + pad
        Y = np.clip(hh * f_cyl + v0 + pad, 0, world.shape[0] - 1.001)
        xi = np.clip(np.floor(X).astype(np.int64), 0, world.shape[1] - 2)
        yi = np.floor(Y).astype(np.int64)
        fx = np.clip(X - xi, 0, 1)[..., None]
        fy = np.clip(Y - yi, 0, 1)[..., None]
        img = (world[yi, xi] * (1 - fx) * (1 - fy) + world[yi, xi + 1] * fx * (1 - fy) +
               world[yi + 1, xi] * (1 - fx) * fy + world[yi + 1, xi + 1] * fx * fy)
        img = img * rng.uniform(1 - gain, 1 + gain)
        img = np.clip(np.rint(img), 1, 255).astype(np.uint8)
        frames.append(img if channels > 1 else img[..., 0])
    return cams, frames, dict(out_w=out_w, out_h=out_h, f_cyl=f_cyl, u0=u0, v0=v0)

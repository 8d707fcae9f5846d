"""Per-capture homography estimation and stitch (SURVEY.md 8 C3 end to end, BASELINE configs[2]).

The reference estimates its homographies once, at calibration (Stitcher.calibrate_stitcher ->
StitcherBase.calibrate -> detectAndDescribe + matchKeypoints, PostScripts/Stitcher/
StitcherClass.py:77-112, :258-354, :356-448), and then warps every capture with them.  Config 3
re-estimates them for every capture; this module closes that loop on the GPU:

  1. ORB (nfeatures, 8 levels x 1.2, FAST 20) of every camera frame, read where it lies in device
     memory (mcs_orb_detect_device: the same frames are stitched afterwards, so nothing is
     uploaded twice);
  2. per adjacent pair (camera k+1 -> camera k): BF Hamming kNN-2 (mcs_match_hamming_knn2),
     Lowe's ratio 0.75 (strict, as :432), and findHomography's RANSAC + LM refinement
     (mcs_ransac_homography_host, 3.0 px);
     steps 1-2 run as one mcs_rig_job in libmcs (csrc/mcs_rig.cpp): the cameras' ORBs side by
     side on libmcs's worker threads (each with its own HIP stream), then the pairs, with no
     interpreter between the steps.  submit() returns at once, so a caller holding two captures
     in flight (slots 0 and 1) overlaps one capture's ORB with the previous one's pairs and
     stitch.  features() / pair_homography() are the same steps issued from Python (kept as the
     cross-check of the job: both give identical homographies);
  3. the chain geometry: stage k maps camera k+1 into the mosaic of cameras 0..k,
     H_k = T(o_k) . H_0 . H_1 ... H_k (pair homographies composed into camera 0's frame, o_k =
     camera 0's origin in that mosaic), and each stage's plan fields follow the arithmetic of
     StitcherBase.calibrate (:293-351) in one fixed FP64 order -- in libmcs (mcs_chain_stages,
     csrc/mcs_chain.cpp, which the rig job runs itself) and restated here (chain_stages);
  4. a plan for this capture (host flattening, microseconds) and mcs_stitch_direct: every output
     pixel mapped by the exact FP64 OpenCV map in the kernel itself, no prepared tables.

A pair whose estimate fails (too few matches or inliers, the reference's H = None) keeps the
previous capture's homography for that pair; with none yet, its stage stays uncalibrated and
passes B through, as the reference's reset() stage does (:253-256) -- and so do all the stages
after it: their pair homographies are relative to a camera that has no place in the mosaic.
(The reference would still try to match each later camera against the mosaic B of the cameras
before the gap, which for a linear rig's non-adjacent cameras has no overlap to match; a rig that
needs that case should calibrate once, StitcherClass's own path, rather than per capture.)

(The reference matches camera k+1 against the mosaic B_k; matching it against camera k and
composing gives the same homography up to estimation noise without re-stitching the mosaic
between stages -- each capture needs one stitch launch, not N - 1.)
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor
from types import SimpleNamespace

import numpy as np

from . import _capi


def _T(tx, ty):
    return np.array([[1.0, 0.0, tx], [0.0, 1.0, ty], [0.0, 0.0, 1.0]])


def ratio_filter(idx, dist, ratio: float = 0.75):
    """Query indices passing Lowe's test, m0.distance < ratio * m1.distance (strict, as
    StitcherClass.py:432), vectorised over the kNN-2 output."""
    ok = (idx[:, 1] >= 0) & (dist[:, 0].astype(np.float64) < dist[:, 1].astype(np.float64) * ratio)
    return np.nonzero(ok)[0]


def _proj(M, x, y):
    """M . (x, y, 1) / w truncated toward zero -- get_projection_point_dst (Utils.py:23-37) in one
    fixed FP64 order, ((m0 x + m1 y) + m2), as csrc/mcs_chain.cpp computes it."""
    p0 = (M[0][0] * x + M[0][1] * y) + M[0][2]
    p1 = (M[1][0] * x + M[1][1] * y) + M[1][2]
    p2 = (M[2][0] * x + M[2][1] * y) + M[2][2]
    return int(p0 / p2), int(p1 / p2)


def _mm(A, B):
    """A . B of 3 x 3 lists, ((a0 b0 + a1 b1) + a2 b2) per entry."""
    return [[(A[i][0] * B[0][j] + A[i][1] * B[1][j]) + A[i][2] * B[2][j] for j in range(3)]
            for i in range(3)]


def _stage_fields(H, a_shape, b_shape):
    """StitcherBase.calibrate's plan fields (StitcherClass.py:293-351, geometry.stage_geometry)
    of one stage, in the fixed FP64 order of _proj (H: a 3 x 3 list, patched in place)."""
    ha, wa = a_shape[0], a_shape[1]
    hb, wb = b_shape[0], b_shape[1]
    ca = [(0, 0), (wa, 0), (wa, ha), (0, ha)]
    a_proj = [_proj(H, x, y) for x, y in ca]
    both = a_proj + [(0, 0), (wb, 0), (wb, hb), (0, hb)]
    x_min = min(pt[0] for pt in both)
    y_min = min(pt[1] for pt in both)
    H[0][2] += float(-x_min)
    H[1][2] += float(-y_min)
    tx, ty = -x_min, -y_min
    Bpts = [(tx, ty), (tx + wb, ty), (tx + wb, hb + ty), (tx, hb + ty)]
    Apts = [_proj(H, x, y) for x, y in ca]
    xs = [pt[0] for pt in Apts + Bpts]
    ys = [pt[1] for pt in Apts + Bpts]
    ABSize = (abs(max(xs)), abs(max(ys)))
    x_limits = [max([v for v in xs if v < ABSize[0] * 0.5]),
                min([v for v in xs if v > ABSize[0] * 0.5])]
    y_limits = [max([v for v in ys if v < ABSize[1] * 0.5]),
                min([v for v in ys if v > ABSize[1] * 0.5])]
    return dict(cachedAH=np.array(H, np.float64), ABSize=ABSize, Bpts=Bpts, x_limits=x_limits,
                y_limits=y_limits)


def chain_stages(pair_H, cam_shapes, super_mode: bool = False):
    """Stage records (the StitcherBase fields the plan needs) of a left-to-right chain whose
    adjacent-pair homographies pair_H[k] map camera k+1 into camera k (None: uncalibrated).
    cam_shapes: (h, w[, C]) of every camera in sorted-label order.  The first None leaves its
    stage and every later one uncalibrated (pass-through): the later homographies are relative
    to cameras with no place in the mosaic (see the module docstring).

    The arithmetic is calibrate's (StitcherClass.py:293-351), restated in plain Python floats in
    one fixed FP64 order -- the order csrc/mcs_chain.cpp (mcs_chain_stages, the rig job's own
    geometry) follows, so the two agree bit for bit (tests/test_chain_cpu.py).  (numpy's 3 x 3
    matmul runs OpenBLAS FMA kernels whose rounding depends on the host CPU.)"""
    stages = []
    b_shape = tuple(cam_shapes[0])
    ox, oy = 0, 0               # camera 0's origin in the mosaic B_k
    P = [[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]]    # camera k+1 -> camera 0
    broken = False
    for k in range(len(cam_shapes) - 1):
        a_shape = tuple(cam_shapes[k + 1])
        rec = SimpleNamespace(cachedAH=None, super_mode=super_mode, AimgSize=a_shape,
                              BimgSize=b_shape)
        if pair_H[k] is None or broken:
            broken = True       # (the rest of the chain has no reference frame)
            stages.append(rec)
            continue
        Q = [[float(v) for v in row] for row in np.asarray(pair_H[k], np.float64)]
        P = _mm(P, Q)
        H = _mm([[1.0, 0.0, float(ox)], [0.0, 1.0, float(oy)], [0.0, 0.0, 1.0]], P)
        h22 = H[2][2]
        H = [[v / h22 for v in row] for row in H]
        g = _stage_fields(H, a_shape, b_shape)
        rec.cachedAH = g["cachedAH"]
        rec.ABSize, rec.Bpts = g["ABSize"], g["Bpts"]
        rec.x_limits, rec.y_limits = g["x_limits"], g["y_limits"]
        stages.append(rec)
        ox += int(g["Bpts"][0][0])
        oy += int(g["Bpts"][0][1])
        W, Hh = int(g["ABSize"][0]), int(g["ABSize"][1])
        if super_mode:
            x0, x1, _ = slice(int(g["x_limits"][0]), int(g["x_limits"][1])).indices(W)
            y0, y1, _ = slice(int(g["y_limits"][0]), int(g["y_limits"][1])).indices(Hh)
            ox -= x0
            oy -= y0
            W, Hh = max(0, x1 - x0), max(0, y1 - y0)
        b_shape = (Hh, W) + tuple(b_shape[2:])
    return stages


class CaptureEstimator:
    """ORB + Hamming kNN-2 + RANSAC homographies of every adjacent camera pair, per capture, and
    the stitch of that capture with them (see the module docstring)."""

    def __init__(self, n_cams: int, width: int, height: int, channels: int = 3,
                 nfeatures: int = 2000, nlevels: int = 8, scale_factor: float = 1.2,
                 fast_threshold: int = 20, ratio: float = 0.75, reproj_thresh: float = 3.0,
                 iters: int = 2000, seed: int = 0, super_mode: bool = False,
                 interp: int = _capi.MCS_INTER_LINEAR, device: int = 0, threads: int = None,
                 captures_per_job: int = 1):
        self.n_cams, self.w, self.h, self.c = n_cams, width, height, channels
        # rig jobs of several captures (mcs_rig_job_create_batch: one launch chain over all their
        # cameras; submit / collect_stitch then take that many captures at once)
        self.batch = captures_per_job
        self.orb = (nfeatures, nlevels, scale_factor, fast_threshold)
        self.ratio, self.thresh, self.iters, self.seed = ratio, reproj_thresh, iters, seed
        self.super_mode, self.interp, self.device = super_mode, interp, device
        self.pool = ThreadPoolExecutor(max_workers=threads or max(1, n_cams))
        # ORB of the NEXT capture runs on its own pool while this one's pairs are matched,
        # estimated and stitched (features_async: a two-stage software pipeline)
        self.fpool = ThreadPoolExecutor(max_workers=threads or max(1, n_cams))
        self.ahead = ThreadPoolExecutor(max_workers=1)
        self.last_H = [None] * (n_cams - 1)
        self.stats = {}
        self._jobs = []

    def close(self):
        for j in self._jobs:
            if j is not None:
                j.close()
        self._jobs = []
        self.ahead.shutdown()
        self.fpool.shutdown()
        self.pool.shutdown()

    def _job(self, slot):
        if slot >= len(self._jobs):
            self._jobs += [None] * (slot + 1 - len(self._jobs))
        if self._jobs[slot] is None:
            nf, nl, sf, ft = self.orb
            self._jobs[slot] = _capi.RigJob(self.n_cams, self.w, self.h, self.c, nf, nl, sf, ft,
                                            self.ratio, self.thresh, self.iters, self.seed,
                                            self.device, captures=self.batch)
        return self._jobs[slot]

    def submit(self, frame_ptrs, wait_event: int = 0, slot: int = 0):
        """Starts the estimation of one capture (device frame pointers) in rig-job `slot` (any
        small index: one job per capture in flight) and returns at once.  wait_event: a hipEvent_t (e.g. torch.cuda.Event.cuda_event)
        after which the frames are complete, or 0 when they already are.  The frames must stay
        untouched until collect(slot)."""
        self._job(slot).submit(frame_ptrs, wait_event)

    def collect(self, slot: int = 0):
        """Pair homographies of the capture submitted in `slot` (blocks until done); a failed
        pair keeps the previous capture's estimate."""
        out = self._jobs[slot].wait()
        per = []
        for res, st in (out if self.batch > 1 else [out]):
            pair_H = []
            for k, H in enumerate(res):
                if H is not None:
                    self.last_H[k] = H
                pair_H.append(self.last_H[k])
            self.stats = st
            per.append(pair_H)
        return per if self.batch > 1 else per[0]

    def collect_stitch(self, slot: int, out_ptr: int, out_pitch: int, out_capacity: int,
                       stream: int = 0):
        """collect(slot) and the stitch of that capture with its homographies, in libmcs
        (mcs_rig_job_wait_stitch: the chain geometry of mcs_chain_stages, a plan, the direct
        stitch on `stream`) -- no Python geometry or plan per capture.  Captures must be collected
        in submission order (a failed pair keeps the previous capture's estimate).  Returns the
        mosaic's (out_h, out_w); with captures_per_job > 1, out_ptr is a list of that many outputs
        and the result a list of shapes."""
        # one carry-over state: last_H (collect and collect_stitch both keep it); the C side
        # reads and updates it through these arrays (a failed pair keeps the previous estimate)
        if not hasattr(self, "_Hio"):
            self._Hio = np.zeros((self.n_cams - 1, 9), np.float64)
            self._okio = np.zeros(self.n_cams - 1, np.int32)
        for k, H in enumerate(self.last_H):
            if H is not None:
                self._Hio[k] = np.asarray(H, np.float64).reshape(9)
            self._okio[k] = 1 if H is not None else 0
        out = self._jobs[slot].wait_stitch(self._Hio, self._okio, out_ptr, out_pitch,
                                           out_capacity, stream, self.super_mode, self.interp)
        for k in range(self.n_cams - 1):
            self.last_H[k] = self._Hio[k].reshape(3, 3).copy() if self._okio[k] else None
        if self.batch > 1:
            self.stats = out[-1][1]
            return [shape for shape, _ in out]
        shape, st = out
        self.stats = st
        return shape

    def homographies(self):
        """The current pair homographies (after collect_stitch: the ones the last stitch used)."""
        return [None if H is None else np.asarray(H, np.float64).reshape(3, 3).copy()
                for H in self.last_H]

    def features(self, frame_ptrs, pool=None):
        """ORB of every camera frame (device pointers, dense h x w x C, producers finished)."""
        nf, nl, sf, ft = self.orb
        return list((pool or self.pool).map(
            lambda p: _capi.orb_detect_device(p, self.w, self.h, self.c, nf, nl, sf, ft,
                                              self.device), frame_ptrs))

    def features_async(self, frame_ptrs, ready=None):
        """Future of features(frame_ptrs) on the look-ahead pools: `ready()` (e.g. the upload
        event's synchronize) runs first on that thread.  The caller meanwhile runs
        estimate_from() / stitch() of the previous capture; the frames must stay untouched until
        the future is done."""
        def run():
            if ready is not None:
                ready()
            return self.features(frame_ptrs, self.fpool)
        return self.ahead.submit(run)

    def pair_homography(self, fa, fb):
        """Camera A -> camera B (A = query, as matchKeypoints' ptsA): H or None, matches,
        inliers."""
        idx, dist = _capi.match_hamming_knn2(fa["desc"], fb["desc"], self.device)
        q = ratio_filter(idx, dist, self.ratio)
        if len(q) <= 4:                       # matchKeypoints needs more than 4 (:437)
            return None, len(q), 0
        src = np.ascontiguousarray(fa["xy"][q], np.float32)
        dst = np.ascontiguousarray(fb["xy"][idx[q, 0]], np.float32)
        H, mask = _capi.ransac_homography(src, dst, self.thresh, self.iters, self.seed,
                                          device=self.device)
        n_in = int(mask.sum()) if mask is not None else 0
        return (H if n_in > 0 else None), len(q), n_in

    def estimate(self, frame_ptrs):
        """Pair homographies of one capture (camera k+1 -> camera k), through the rig job; a
        failed pair keeps the previous capture's estimate."""
        self.submit(frame_ptrs)
        return self.collect()

    def estimate_from(self, feats):
        """The pair step issued from Python, from the capture's features (features /
        features_async); same result as the rig job."""
        res = list(self.pool.map(lambda k: self.pair_homography(feats[k + 1], feats[k]),
                                 range(self.n_cams - 1)))
        pair_H = []
        for k, (H, n_m, n_in) in enumerate(res):
            if H is not None:
                self.last_H[k] = H
            pair_H.append(self.last_H[k])
        self.stats = {"keypoints": [len(f["xy"]) for f in feats],
                      "matches": [r[1] for r in res], "inliers": [r[2] for r in res]}
        return pair_H

    def plan(self, pair_H):
        """The plan of one capture's geometry (host only)."""
        from .StitcherClass import _stage_desc
        shapes = [(self.h, self.w, self.c)] * self.n_cams
        stages = chain_stages(pair_H, shapes, self.super_mode)
        return _capi.Plan([_stage_desc(sb) for sb in stages], self.w, self.h, self.c, self.interp,
                          device=self.device), stages

    def stitch(self, frame_ptrs, pair_H, out_ptr: int, out_pitch: int, out_capacity: int,
               stream: int = 0):
        """Stitch one capture with its homographies into out (rows out_pitch bytes apart,
        out_capacity bytes).  Returns the plan (its out_w / out_h give the mosaic's size)."""
        plan, _ = self.plan(pair_H)
        if plan.out_w * self.c > out_pitch or plan.out_h * out_pitch > out_capacity:
            plan.close()
            raise ValueError(f"mosaic {plan.out_w} x {plan.out_h} does not fit the output buffer")
        fs = self.w * self.h * self.c
        plan.stitch_direct(frame_ptrs, [fs] * self.n_cams, out_ptr, out_pitch,
                           out_pitch * plan.out_h, 1, stream)
        return plan

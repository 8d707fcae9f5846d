#!/usr/bin/env python3
"""C3 benchmark (BASELINE.json configs[2]): per rig capture, the homographies re-estimated on
the GPU -- ORB (nfeatures 2000, 8 levels x 1.2, FAST 20) on each of the 4 1920x1080 BGR camera
frames, BF Hamming kNN-2 + Lowe ratio 0.75 + RANSAC (3.0 px, 2000 hypotheses) for each adjacent
camera pair -- and the CPU restatement (oracle/, the checker) of the same chain beside it.

The frames are rendered from one shared world (rectangles of random grey levels, seed 0) through
the C2 rig's camera models, so overlaps agree and the true pair homographies are known; the
estimates are checked against them (max reprojection error over the pair's overlap).  Host
frames in, homographies out: the PCIe upload of each frame is inside the timed region.

One JSON line: rig estimations/s, ms per capture and per stage, matches / inliers, errors.

--stitch: the whole per-capture loop of config 3 (multicamera_stitching_amd/estimate.py): the
four frames uploaded once (pageable host -> device, timed), ORB on the device copies, matching +
RANSAC, the chain geometry and a fresh plan on the host, and the capture stitched with its own
homographies by mcs_stitch_direct; the line then reports captures/s and stitched MPix/s, and
checks one capture's mosaic against the CPU restatement of the same geometry.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def world(h, w, channels, seed):
    from multicamera_stitching_amd import rig
    return rig.corner_world(h, w, channels, seed)


def pair_error(H, Ht, w, h):
    """max |H p - Ht p| over a grid of the query camera's left quarter (the overlap)."""
    u, v = np.meshgrid(np.linspace(0, w * 0.2, 8), np.linspace(0, h - 1, 8))
    g = np.stack([u.ravel(), v.ravel(), np.ones(u.size)], axis=1)
    p, q = g @ H.T, g @ Ht.T
    return float(np.abs(p[:, :2] / p[:, 2:] - q[:, :2] / q[:, 2:]).max())


_POOL = None


def estimate_gpu(frames, args):
    """One capture: the cameras' ORB calls run concurrently (one host thread each: every thread
    has its own HIP stream and device workspace in libmcs, and ctypes releases the GIL), then the
    pairs' match + ratio + RANSAC, also one thread each."""
    global _POOL
    from concurrent.futures import ThreadPoolExecutor
    from multicamera_stitching_amd import _capi
    if _POOL is None:
        _POOL = ThreadPoolExecutor(max_workers=max(1, args.threads))
    t = {"orb": 0.0, "match_ransac": 0.0}
    t0 = time.perf_counter()
    feats = list(_POOL.map(lambda f: _capi.orb_detect(f, args.nfeatures, 8, 1.2, 20), frames))
    t1 = time.perf_counter()

    def pair(k):
        idx, dist = _capi.match_hamming_knn2(feats[k]["desc"], feats[k - 1]["desc"])
        # features.ratio_matches, vectorised: query order, strict d0 < 0.75 d1
        q = np.nonzero((idx[:, 1] >= 0) & (dist[:, 0].astype(np.float64) <
                                           dist[:, 1].astype(np.float64) * 0.75))[0]
        src = np.ascontiguousarray(feats[k]["xy"][q], np.float32)
        dst = np.ascontiguousarray(feats[k - 1]["xy"][idx[q, 0]], np.float32)
        H, mask = _capi.ransac_homography(src, dst, 3.0, 2000, 0)
        return H, len(q), int(mask.sum()), [len(f["xy"]) for f in feats]
    out = list(_POOL.map(pair, range(1, len(frames))))
    t["orb"] = t1 - t0
    t["match_ransac"] = time.perf_counter() - t1
    return out, t


def estimate_cpu(frames, args):
    from oracle import oracle
    from multicamera_stitching_amd.features import ratio_matches
    feats = []
    for f in frames:
        g = ((f[..., 0].astype(np.int32) * 1868 + f[..., 1].astype(np.int32) * 9617 +
              f[..., 2].astype(np.int32) * 4899 + 8192) >> 14).astype(np.uint8)
        feats.append(oracle.orb_detect(g, args.nfeatures, 8, 1.2, 20))
    out = []
    for k in range(1, len(frames)):
        idx, dist = oracle.hamming_knn2(feats[k]["desc"], feats[k - 1]["desc"])
        m = ratio_matches(idx, dist)
        src = np.float32([feats[k]["xy"][q] for (_, q) in m]).reshape(-1, 2)
        dst = np.float32([feats[k - 1]["xy"][tr] for (tr, _) in m]).reshape(-1, 2)
        H, mask, _, _ = oracle.ransac_homography(src, dst, 3.0, 2000, 0)
        out.append(H)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--threads", type=int, default=4,
                    help="host threads issuing the per-camera / per-pair calls (1: serial)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stitch", action="store_true",
                    help="estimate -> stitch per capture (estimate.py, mcs_stitch_direct)")
    ap.add_argument("--overlap", action="store_true",
                    help="with --pipelined: each capture's estimation in its own rig job "
                         "(mcs_rig_job), started once its upload is queued, so the ORBs of the "
                         "next captures run beside the pairs + stitch of this one")
    ap.add_argument("--pipelined", action="store_true",
                    help="with --stitch: upload capture f+1 (pinned host frames, own stream, two "
                         "device frame sets) while capture f is estimated and stitched")
    ap.add_argument("--depth", type=int, default=2,
                    help="with --pipelined: captures in flight (frame sets, rig jobs, outputs)")
    ap.add_argument("--python-stitch", action="store_true",
                    help="pipelined: the capture's chain geometry and plan built in Python "
                         "(estimate.chain_stages + Plan + stitch_direct) instead of inside the rig "
                         "job (mcs_rig_job_wait_stitch, the default with --overlap)")
    ap.add_argument("--resident", action="store_true",
                    help="with --pipelined: the frames stay in HBM (no per-capture upload): the "
                         "GPU-bound rate of estimate + stitch")
    ap.add_argument("--batch", type=int, default=1,
                    help="with --pipelined --overlap: captures per rig job "
                         "(mcs_rig_job_create_batch: one launch chain over all their cameras)")
    ap.add_argument("--stitch-streams", action="store_true",
                    help="pipelined: each slot's stitches on a stream of their own (default: one "
                         "stitch stream)")
    ap.add_argument("--pinned", action="store_true",
                    help="camera frames in pinned host buffers (default: pageable numpy arrays, "
                         "as the reference's capture loop holds them)")
    args = ap.parse_args()
    from multicamera_stitching_amd import rig
    W, Hh, N = 1920, 1080, 4
    C = rig.camera_models(N, W, Hh, seed=0)
    frames = rig.world_frames(C, W, Hh, 3, seed=0, world_fn=world)
    if args.pinned:
        import torch
        pinned = []
        for f in frames:
            t = torch.empty(f.shape, dtype=torch.uint8, pin_memory=True)
            t.numpy()[...] = f
            pinned.append(t)
        frames = [t.numpy() for t in pinned]
    truth = [np.linalg.inv(C[k - 1]) @ C[k] for k in range(1, N)]
    truth = [T / T[2, 2] for T in truth]
    if args.stitch:
        if args.pipelined:
            return pipelined_main(args, frames, truth, W, Hh, N)
        return stitch_main(args, frames, truth, W, Hh, N)
    for _ in range(args.warmup):
        estimate_gpu(frames, args)
    tot = {"orb": 0.0, "match_ransac": 0.0}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res, t = estimate_gpu(frames, args)
        for key in tot:
            tot[key] += t[key]
    elapsed = time.perf_counter() - t0
    captures = args.steps
    errs = [pair_error(h, T, W, Hh) if h is not None else None for (h, *_), T in zip(res, truth)]
    line = {
        "metric": "rig homography estimations/sec (C3: 4-cam 1080p, ORB + BF Hamming kNN-2 + "
                  "RANSAC per capture)",
        "value": round(captures / elapsed, 2), "unit": "captures/s", "n_gpus": 1,
        "steps": captures, "warmup": args.warmup,
        "ms_per_step": round(elapsed / captures * 1e3, 3), "higher_is_better": True,
        "dtype": "u8 / int popcount / f64", "data": "synthetic (shared-world rig, seed 0)",
        "config": {"workload": "BASELINE configs[2]: ORB nfeatures %d, 8 levels x 1.2, FAST 20; "
                               "Hamming kNN-2, ratio 0.75; RANSAC 3.0 px, 2000 hypotheses; 3 "
                               "adjacent pairs" % args.nfeatures,
                   "host_frames": "pinned" if args.pinned else "pageable",
                   "host_threads": args.threads},
        "stage_ms_per_capture": {k: round(v / args.steps * 1e3, 3) for k, v in tot.items()},
        "keypoints": res[0][3], "matches": [r[1] for r in res], "inliers": [r[2] for r in res],
        "max_reproj_err_px_vs_truth": errs,
    }
    if not args.no_cpu_baseline:
        from oracle import oracle
        tc = time.perf_counter()
        cpu = estimate_cpu(frames, args)
        dt = time.perf_counter() - tc
        diff = [pair_error(a, b, W, Hh) if a is not None and b is not None else None
                for a, b in zip([r[0] for r in res], cpu)]
        line["cpu_baseline"] = {"value": round(1.0 / dt, 3), "unit": "captures/s",
                                "cores": oracle.num_threads(), "kind": "port",
                                "sample": "1 capture through the C restatement (orc_orb.c, "
                                          "orc_match.c, orc_ransac.c), %.1f s" % dt}
        line["max_abs_H_reproj_diff_gpu_vs_cpu_px"] = diff
    print(json.dumps(line))


def stitch_main(args, frames, truth, W, Hh, N):
    """Config 3 end to end: per capture upload -> ORB -> match -> RANSAC -> geometry -> plan ->
    mcs_stitch_direct, frames and mosaic on the device."""
    import torch
    from multicamera_stitching_amd import estimate
    from oracle import oracle
    dev = torch.device("cuda", 0)
    d = [torch.empty(f.shape, dtype=torch.uint8, device=dev) for f in frames]
    pitch = 8192 * 3
    out = torch.empty((2048, pitch), dtype=torch.uint8, device=dev)
    est = estimate.CaptureEstimator(N, W, Hh, 3, nfeatures=args.nfeatures, threads=args.threads)
    ptrs = [t.data_ptr() for t in d]
    tot = {"upload": 0.0, "estimate": 0.0, "plan_stitch": 0.0}
    mpix = 0.0

    def capture(timed):
        nonlocal mpix
        t0 = time.perf_counter()
        for t, f in zip(d, frames):
            t.copy_(torch.from_numpy(f))
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        pair_H = est.estimate(ptrs)
        t2 = time.perf_counter()
        plan = est.stitch(ptrs, pair_H, out.data_ptr(), pitch, out.numel())
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        if timed:
            tot["upload"] += t1 - t0
            tot["estimate"] += t2 - t1
            tot["plan_stitch"] += t3 - t2
            mpix += plan.out_w * plan.out_h / 1e6
        return pair_H, plan
    for _ in range(args.warmup):
        capture(False)[1].close()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pair_H, plan = capture(True)
        plan.close()
    elapsed = time.perf_counter() - t0
    pair_H, plan = capture(False)
    ow, oh = plan.out_w, plan.out_h
    got = out[:oh, :ow * 3].cpu().numpy().reshape(oh, ow, 3)
    want = oracle.flat_stitch(plan.describe(), frames)
    plan.close()
    est.close()
    errs = [pair_error(h, T, W, Hh) if h is not None else None for h, T in zip(pair_H, truth)]
    print(json.dumps({
        "metric": "rig captures/sec estimated AND stitched with their own homographies (C3 end "
                  "to end: 4-cam 1080p, ORB + BF Hamming kNN-2 + RANSAC + stitch per capture)",
        "value": round(args.steps / elapsed, 2), "unit": "captures/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "stitched_mpix_per_s": round(mpix / elapsed, 1),
        "mosaic": [oh, ow, 3], "data": "synthetic (shared-world rig, seed 0)",
        "config": {"workload": "BASELINE configs[2] + per-capture stitch: ORB nfeatures %d, 8 "
                               "levels x 1.2, FAST 20; Hamming kNN-2, ratio 0.75; RANSAC 3.0 px, "
                               "2000 hypotheses + LM; chain geometry + plan on the host "
                               "(in Python); mcs_stitch_direct (paste)" % args.nfeatures,
                   "host_frames": "pageable, uploaded every capture",
                   "host_threads": args.threads},
        "stage_ms_per_capture": {k: round(v / args.steps * 1e3, 3) for k, v in tot.items()},
        "keypoints": est.stats.get("keypoints"), "matches": est.stats.get("matches"),
        "inliers": est.stats.get("inliers"), "max_reproj_err_px_vs_truth": errs,
        "max_abs_diff_vs_cpu_render": int(np.abs(got.astype(np.int16) -
                                                 want.astype(np.int16)).max()),
    }))


def pipelined_main(args, frames, truth, W, Hh, N):
    """Config 3 end to end, pipelined --depth captures deep: the cameras' frames of capture f+D-1
    go up (pinned host buffers, a dedicated stream, D device frame sets) while the captures before
    it are estimated (with --overlap: each in its own rig job, submitted as soon as its upload is
    queued, its ORB streams waiting on the upload event on the GPU) and stitched (its stitch on
    its own stream; a plan is released once its stitch has finished)."""
    import torch
    from multicamera_stitching_amd import estimate
    from oracle import oracle
    D = max(2, args.depth)
    B = max(1, args.batch)          # captures per rig job (and per frame set / output slot)
    if B > 1 and not (args.overlap and not args.python_stitch):
        raise SystemExit("--batch needs --overlap (rig jobs) and the in-library stitch")
    dev = torch.device("cuda", 0)
    host = []
    for f in frames:
        t = torch.empty(f.shape, dtype=torch.uint8, pin_memory=True)
        t.numpy()[...] = f
        host.append(t)
    # each frame set is one allocation (the capture's cameras side by side in HBM): the direct
    # stitch then addresses every camera with 32-bit offsets from one base (mcs_direct_*_o32; four
    # separate allocations can land more than 4 GiB apart and take the 64-bit form, ~1.5x slower)
    sets = [torch.empty((B * len(frames),) + tuple(frames[0].shape), dtype=torch.uint8,
                        device=dev) for _ in range(D)]
    d = [[ts[i] for i in range(B * len(frames))] for ts in sets]
    ptrs = [[t.data_ptr() for t in ds] for ds in d]
    host_b = host * B               # capture q of a set: cameras q N .. q N + N - 1
    pitch = 8192 * 3
    outs = [torch.empty((B, 2048, pitch), dtype=torch.uint8, device=dev) for _ in range(D)]
    out = [o[B - 1] for o in outs]  # (the set's last capture: the one the parity check reads)
    up = torch.cuda.Stream()
    # the stitches: one stream per slot with --stitch-streams (the captures' stitches are
    # independent: they overlap on the GPU), else one stream for all
    sts = [torch.cuda.Stream() for _ in range(D if args.stitch_streams else 1)]
    ev_up = [torch.cuda.Event() for _ in range(D)]
    ev_done = [torch.cuda.Event() for _ in range(D)]
    for e in ev_done:
        e.record(sts[0])
    est = estimate.CaptureEstimator(N, W, Hh, 3, nfeatures=args.nfeatures, threads=args.threads,
                                    captures_per_job=B)
    pending = [None] * D          # plan of the capture last stitched from frame set / output i
    lat = []

    def upload(slot):
        with torch.cuda.stream(up):
            up.wait_event(ev_done[slot])          # that set's previous stitch has read it
            if not args.resident:
                for t, h in zip(d[slot], host_b):
                    t.copy_(h, non_blocking=True)
            ev_up[slot].record(up)

    if args.resident:                             # the frames stay in HBM: uploaded once
        for ds in d:
            for t, h in zip(ds, host_b):
                t.copy_(h)
        torch.cuda.synchronize()

    def start(i, t_start):
        slot = i % D
        # (resident: the frames never change, so there is no upload to order after -- no event)
        if not args.resident:
            upload(slot)
        t_start[slot] = time.perf_counter()
        if args.overlap:
            est.submit(ptrs[slot], 0 if args.resident else ev_up[slot].cuda_event, slot)

    def run(n):
        n = max(1, n // B)          # rig jobs (B captures each)
        mpix = 0.0
        t_start = [0.0] * D
        lat.clear()
        for i in range(min(D - 1, n)):
            start(i, t_start)
        for i in range(n):
            slot = i % D
            if i + D - 1 < n:
                start(i + D - 1, t_start)
            if lib_stitch:
                # the capture's geometry, plan and stitch inside libmcs: one call per capture
                shapes = est.collect_stitch(
                    slot, [o.data_ptr() for o in outs[slot]] if B > 1 else out[slot].data_ptr(),
                    pitch, out[slot].numel(), sts[slot % len(sts)].cuda_stream)
                lat.append(time.perf_counter() - t_start[slot])
                ev_done[slot].record(sts[slot % len(sts)])
                mpix += sum(ow * oh for oh, ow in (shapes if B > 1 else [shapes])) / 1e6
                continue
            if args.overlap:
                pair_H = est.collect(slot)
            else:
                if not args.resident:
                    ev_up[slot].synchronize()         # this capture's frames are on the device
                pair_H = est.estimate(ptrs[slot])
            lat.append(time.perf_counter() - t_start[slot])
            if pending[slot] is not None:         # the set's previous plan: its stitch is done
                ev_done[slot].synchronize()
                pending[slot].close()
            plan = est.stitch(ptrs[slot], pair_H, out[slot].data_ptr(), pitch, out[slot].numel(),
                              stream=sts[slot % len(sts)].cuda_stream)
            ev_done[slot].record(sts[slot % len(sts)])
            pending[slot] = plan
            mpix += plan.out_w * plan.out_h / 1e6
        torch.cuda.synchronize()
        if lib_stitch:
            # (the plan of the last capture's geometry, for the check: chain_stages restates
            # mcs_chain_stages bit for bit)
            pair_H = est.homographies()
            plan, _ = est.plan(pair_H)
            pending.append(plan)
        return mpix, pair_H, plan, slot

    lib_stitch = args.overlap and not args.python_stitch
    run(args.warmup)
    t0 = time.perf_counter()
    mpix, pair_H, plan, slot = run(args.steps)
    elapsed = time.perf_counter() - t0
    captures = max(1, args.steps // B) * B
    # the host link's H2D ceiling for the same transfers (pinned frames -> device, back to back
    # on the upload stream): the uploaded form's bound
    link = None
    if not args.resident:
        with torch.cuda.stream(up):
            for _ in range(2):
                for t, h in zip(d[0][:len(host)], host):
                    t.copy_(h, non_blocking=True)
            torch.cuda.synchronize()
            tl = time.perf_counter()
            reps = 20
            for _ in range(reps):
                for t, h in zip(d[0][:len(host)], host):
                    t.copy_(h, non_blocking=True)
            torch.cuda.synchronize()
            link = reps * sum(h.numel() for h in host) / (time.perf_counter() - tl) / 1e9
    ow, oh = plan.out_w, plan.out_h
    got = out[slot][:oh, :ow * 3].cpu().numpy().reshape(oh, ow, 3)
    want = oracle.flat_stitch(plan.describe(), frames)
    for q in pending:
        if q is not None:
            q.close()
    est.close()
    errs = [pair_error(h, T, W, Hh) if h is not None else None for h, T in zip(pair_H, truth)]
    print(json.dumps({
        "metric": "rig captures/sec estimated AND stitched with their own homographies (C3 end "
                  "to end: 4-cam 1080p, ORB + BF Hamming kNN-2 + RANSAC + stitch per capture)",
        "value": round(args.steps / elapsed, 2), "unit": "captures/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "stitched_mpix_per_s": round(mpix / elapsed, 1),
        "mosaic": [oh, ow, 3], "data": "synthetic (shared-world rig, seed 0)",
        "config": {"workload": "BASELINE configs[2] + per-capture stitch: ORB nfeatures %d, 8 "
                               "levels x 1.2, FAST 20; Hamming kNN-2, ratio 0.75; RANSAC 3.0 px, "
                               "2000 hypotheses + LM; chain geometry + plan on the host "
                               "(%s); mcs_stitch_direct (paste)" % (
                                   args.nfeatures, "in libmcs: mcs_rig_job_wait_stitch"
                                   if lib_stitch else "in Python"),
                   "host_frames": "pinned, uploaded every capture on their own stream while the "
                                  "previous captures are estimated and stitched",
                   "pipeline_depth": D, "rig_jobs": bool(args.overlap),
                   "captures_per_rig_job": B, "stitch_streams": len(sts),
                   "host_threads": args.threads},
        "frames_resident_in_hbm": bool(args.resident),
        "h2d_gb_per_s": None if link is None else
        round(captures * sum(h.numel() for h in host) / elapsed / 1e9, 2),
        "h2d_link_ceiling_gb_per_s": None if link is None else round(link, 2),
        "frac_of_h2d_link": None if link is None else
        round(captures * sum(h.numel() for h in host) / elapsed / 1e9 / link, 3),
        "latency_ms_upload_to_homographies": round(float(np.mean(lat)) * 1e3, 3),
        "keypoints": est.stats.get("keypoints"), "matches": est.stats.get("matches"),
        "inliers": est.stats.get("inliers"), "max_reproj_err_px_vs_truth": errs,
        "max_abs_diff_vs_cpu_render": int(np.abs(got.astype(np.int16) - want).max()),
    }))


if __name__ == "__main__":
    main()

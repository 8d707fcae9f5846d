#!/usr/bin/env python3
"""Benchmark of the stitch hot path: stitched MPix/s on a synthetic 4 x 1920x1080 rig.

Workload (BASELINE.json configs[1]): 4 x 1920x1080 BGR cameras, precomputed homographies,
bilinear warp + 3-level multi-band blend (--blend multiband, the default); --blend none is the
reference's own per-stage semantics (warpPerspective + overwrite paste, StitcherClass.py:211-256)
and --blend feather the linear feather blend.  One "step" = one stitch launch over --frames rig
captures already resident in HBM (4 camera frames each), producing --frames mosaics: the
streaming gather kernel over every tile, then (blend modes) the blend kernel over the tiles the
blend changes.  Frame 0 is checked against the CPU restatement every run ("max_abs_diff").

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one process per GPU, each
stitching its own captures (rig frames are independent: weak scaling, no data-path collective);
barrier + synchronize around the timed region, time = max over ranks.

Extra fields: "roofline" (HBM-bound; algorithmic bytes = SURVEY.md 8d's B_frame -- every camera
frame read once + the mosaic written once -- per launch, over the launch's average duration
measured with HIP events on its stream; "touched" prices only the source pixels the mosaic reads;
both are lower bounds for the blend modes, whose seam tiles re-read their neighbourhoods),
"kernels" (the same launch without the blend pass, for the blend's share), and "cpu_baseline"
(the C restatement in oracle/, on the host cores, rank 0 only, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=64,
                    help="rig captures per launch (per GPU); SURVEY.md 8d: >= 64 per launch")
    ap.add_argument("--rig", choices=["chain", "cylinder"], default="chain",
                    help="chain: BASELINE configs[1] (homography chain, the reference's path); "
                         "cylinder: SURVEY.md 8 C4 (8 cameras at 45 degree yaw, f = 1100, "
                         "cylindrical 360 panorama)")
    ap.add_argument("--focal", type=float, default=1100.0, help="cylinder rig focal length (px)")
    ap.add_argument("--seam", choices=["graphcut", "distance"], default="graphcut",
                    help="cylinder rig seams: graph-cut (BASELINE configs[3], found once per plan "
                         "from capture 0 before the timed region, mcs_plan_find_seams on the 1/4 "
                         "grid) or the distance seam")
    ap.add_argument("--cams", type=int, default=None, help="default 4 (chain) / 8 (cylinder)")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--channels", type=int, default=3)
    ap.add_argument("--interp", choices=["linear", "nearest"], default="linear")
    ap.add_argument("--super-mode", action="store_true")
    ap.add_argument("--blend", choices=["multiband", "feather", "seam", "none"],
                    default="multiband",
                    help="multiband = BASELINE configs[1]; none = the reference's paste")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--gather", choices=["after", "timed", "none"], default="after",
                    help="N > 1: deliver every rank's F mosaics to rank 0 (RCCL point-to-point "
                         "over xGMI) after the timed region ('after', reported as 'gather'), "
                         "or additionally as part of every timed step ('timed')")
    ap.add_argument("--stub", action="store_true",
                    help="CPU rehearsal of the multi-rank orchestration (gloo, a stub step): "
                         "no GPU, no libmcs; tests/test_bench_dist.py")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-also", action="store_true",
                    help="skip the companion lines (C4 cylinder, C3 estimate + stitch, matcher, "
                         "C4 seams) that a 1-GPU run appends under 'also'")
    ap.add_argument("--no-paste-ref", action="store_true",
                    help="skip the paste-only reference launch (PMC passes: one plan's dispatches)")
    ap.add_argument("--pmc-json", default=None,
                    help="counter summary for roofline.traffic (default profiles/pmc_latest.json, "
                         "profiles/pmc_latest_cyl.json with --rig cylinder)")
    return ap.parse_args()


def spawn_ranks(args) -> int:
    """--gpus N > 1 without a torch.distributed launcher around us: start N rank processes (one
    per GPU) under torch.distributed.run as CHILDREN and return their exit code.  This parent
    never touches the GPU (nothing above imports torch.cuda)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def world_from_env(args):
    """(world, rank, local_rank).  Exits non-zero when the launcher's WORLD_SIZE disagrees with
    --gpus (a line must never report a GPU count it did not run)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per "
                         f"GPU (python bench.py --gpus N spawns them itself)")
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world, rank, local = world_from_env(args)
    if args.stub:
        return stub_main(args, world, rank)
    import torch
    import torch.distributed as dist

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from multicamera_stitching_amd import rig, shard, _capi
    from multicamera_stitching_amd.StitcherClass import _stage_desc

    interp = _capi.MCS_INTER_LINEAR if args.interp == "linear" else _capi.MCS_INTER_NEAREST
    cyl = args.rig == "cylinder"
    if args.cams is None:
        args.cams = 8 if cyl else 4
    if cyl and args.blend == "none":
        raise SystemExit("bench: a cylindrical rig has no paste order (use --blend seam)")
    st = geo = None
    if cyl:
        rig_cams, cams, geo = rig.cylinder_rig(args.cams, args.width, args.height, args.focal,
                                               args.channels, seed=0, jitter_deg=0.5)

        def make_plan():
            return _capi.Plan.cylindrical(rig_cams, geo["out_w"], geo["out_h"], geo["f_cyl"],
                                          geo["u0"], geo["v0"], args.channels, interp,
                                          device=torch.cuda.current_device())
    else:
        st, images, _ = rig.calibrated_stitcher(args.cams, args.width, args.height,
                                                args.channels, super_mode=args.super_mode,
                                                seed=0)
        cams = [images[label] for label in st.img_labels]
        descs = [_stage_desc(sb) for sb in st.stitchers]

        def make_plan():
            return _capi.Plan(descs, args.width, args.height, args.channels, interp,
                              device=torch.cuda.current_device())
    plan = make_plan()
    seam_k = None
    if cyl and args.seam == "graphcut":
        # calibration-time step (once per plan, outside the timed region): graph-cut seams on
        # the 2^2 grid from one capture; every timed capture then follows those seams
        seam_k = 2
        t_seam = time.perf_counter()
        plan.find_seams(cams, _capi.MCS_SEAM_GRAPHCUT, seam_k)
        seam_ms = (time.perf_counter() - t_seam) * 1e3
        seam_labels = plan.seam_labels()
    blend = {"none": _capi.MCS_BLEND_NONE, "feather": _capi.MCS_BLEND_FEATHER,
             "multiband": _capi.MCS_BLEND_MULTIBAND, "seam": _capi.MCS_BLEND_SEAM}[args.blend]
    plan.set_blend(blend)
    C = args.channels
    F = args.frames
    out_w, out_h = plan.out_w, plan.out_h

    # device-resident inputs: F captures per camera (frame f = camera texture rolled by f rows)
    d_cams = []
    for c in cams:
        base = torch.from_numpy(c).to(dev)
        d_cams.append(torch.stack([torch.roll(base, shifts=(rank * F + f) % c.shape[0], dims=0)
                                   for f in range(F)]).contiguous())
    pitch = (out_w * C + 255) // 256 * 256
    d_out = torch.empty((F, out_h, pitch), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    stream = torch.cuda.Stream()          # the kernel's own stream; events are recorded on it

    # one-time plan preparation (the exact OpenCV map -> per-tile LDS tables), outside the timing
    t_prep = time.perf_counter()
    plan.prepare(stream.cuda_stream)
    torch.cuda.synchronize()
    prep_ms = (time.perf_counter() - t_prep) * 1e3
    plan_stats = plan.stats()

    def stitch():
        plan.stitch_device([t.data_ptr() for t in d_cams], [t[0].numel() for t in d_cams],
                           d_out.data_ptr(), pitch, d_out[0].numel(), F, stream.cuda_stream)

    step = stitch
    if world > 1 and args.gather == "timed":
        # every step also delivers the F mosaics of every rank to rank 0 (mcs_group_gather)
        group = shard.mcs_group(dev.index)
        recv = (torch.empty((world,) + tuple(d_out.shape), dtype=torch.uint8, device=dev)
                if rank == 0 else None)

        def step():
            stitch()
            shard.gather_mosaics_group(group, d_out, recv, 0, stream.cuda_stream)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]

    # MCS_BENCH_MARKERS=1 (profiling runs only, never the driver's line): a tiny spin kernel on
    # the stream before the first and after the last timed launch, so tools/trace_stats.py can
    # select exactly the timed dispatches from a rocprofv3 kernel trace
    markers = os.environ.get("MCS_BENCH_MARKERS") == "1"

    def marker():
        if markers:
            with torch.cuda.stream(stream):
                torch.cuda._sleep(64)

    def record(i, what):
        if what == "start" and i == 0:
            marker()
        ev[i][0 if what == "start" else 1].record(stream)
        if what == "end" and i == args.steps - 1:
            marker()

    elapsed = shard.timed_loop(step, args.steps, args.warmup, torch.cuda.synchronize, record)
    launch_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    elapsed, launch_ms = shard.max_over_ranks([elapsed, launch_ms], device=dev)
    gather = None
    if world > 1 and args.gather != "none":
        try:
            gather = gather_all(d_out, args, shard, torch, dev)
        except Exception as e:   # (outside the timed region: the line still reports the run)
            gather = {"error": f"{type(e).__name__}: {e}"}

    mpix_per_launch = F * out_w * out_h / 1e6
    value = shard.job_rate(mpix_per_launch, args.steps, elapsed, world)
    frame0 = d_out[0, :, :out_w * C].reshape(out_h, out_w, C).cpu().numpy()

    # the same launch with the reference's paste (cylinder: the hard seam) and no blend pass:
    # the blend's share of the time
    paste_ms = None
    if blend not in (_capi.MCS_BLEND_NONE, _capi.MCS_BLEND_SEAM) and not args.no_paste_ref:
        ref = make_plan()
        if cyl:
            if seam_k is not None:
                ref.find_seams(cams, _capi.MCS_SEAM_GRAPHCUT, seam_k)
            ref.set_blend(_capi.MCS_BLEND_SEAM)
        ref.prepare(stream.cuda_stream)

        def step_ref():
            ref.stitch_device([t.data_ptr() for t in d_cams], [t[0].numel() for t in d_cams],
                              d_out.data_ptr(), pitch, d_out[0].numel(), F, stream.cuda_stream)
        for _ in range(args.warmup):
            step_ref()
        torch.cuda.synchronize()
        evr = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        marker()
        for i in range(args.steps):
            evr[i][0].record(stream)
            step_ref()
            evr[i][1].record(stream)
        marker()
        torch.cuda.synchronize()
        paste_ms = shard.max_over_ranks([float(np.mean([a.elapsed_time(b) for a, b in evr]))],
                                        device=dev)[0]
        ref.close()

    # algorithmic bytes per launch: B_frame = every camera frame read once + the
    # mosaic written once (the roofline's bytes); beside it the touched-pixel figure: only the
    # source pixels the mosaic reads with non-zero weight (counted on the device)
    bframe = out_w * out_h * C + sum(int(np.prod(c.shape)) for c in cams)
    bytes_per_launch = F * bframe
    achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
    fp = plan.footprint()
    touched_per_launch = F * (out_w * out_h * C + sum(fp) * C)
    traffic = None
    workload = (f"{args.cams}x{args.width}x{args.height}x{C}-{args.interp}-"
                f"super{int(args.super_mode)}-F{F}-{args.blend}")
    if cyl:
        workload = f"cyl-f{args.focal:g}-" + workload + ("-gc2" if seam_k is not None else "")
    traffic_src = None
    try:
        if args.pmc_json is None:
            args.pmc_json = os.path.join(ROOT, "profiles",
                                         "pmc_latest_cyl.json" if cyl else "pmc_latest.json")
        pm = json.load(open(args.pmc_json))
        # counters count only for the kernels they were taken on: same workload AND same build
        # of the embedded code objects (mcs_build_id), else traffic stays null
        if pm.get("workload") == workload and pm.get("build_id") == _capi.build_id():
            traffic = pm.get("hbm_bytes_per_launch")
            traffic_src = os.path.relpath(args.pmc_json, ROOT)
    except (OSError, ValueError):
        pass

    # parity on EVERY rank (outside the timed region): this rank's capture 0 (read back above,
    # before the paste-only launch reuses d_out) against the CPU restatement fed the same camera
    # frames; the line reports the max over ranks
    runner = oracle_runner(st, args, interp, plan, blend, (rig_cams, geo) if cyl else None,
                           seams=(seam_k, seam_labels) if seam_k is not None else None)
    host = host_cpus()
    shift = [(rank * F) % c.shape[0] for c in cams]
    max_abs = check_frame0(runner, [np.roll(c, s, axis=0) for c, s in zip(cams, shift)], frame0,
                           max(1, host["usable"] // world))
    max_abs = shard.max_abs_over_ranks(max_abs, device=dev)
    seams_equal = None
    if seam_k is not None and rank == 0:
        # the plan's cut of capture 0 against the restatement's (orc_seam.c) on the same frames
        from oracle import oracle
        _, want_lab = oracle.blend_stitch_cyl(rig_cams, geo["out_w"], geo["out_h"], geo["f_cyl"],
                                              geo["u0"], geo["v0"], cams, _capi.MCS_BLEND_SEAM,
                                              interp, seam_k=seam_k, want_seams=True)
        seams_equal = bool(np.array_equal(want_lab, seam_labels))

    result = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(runner, cams, args, out_w, out_h, host)
        result = {
            "metric": ("stitched MPix/sec (8-cam 360 cylindrical rig)" if cyl else
                       "stitched MPix/sec (4-cam 1080p rig)"),
            "value": round(value, 3),
            "unit": "MPix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": describe_workload(args, cyl),
                "blend": args.blend,
                "mosaic": [out_h, out_w, C],
                "frames_per_step": F,
                "super_mode": bool(args.super_mode),
                "parallelism": f"captures sharded over {world} GPU(s), no data-path collective",
            },
            "max_abs_diff": max_abs,
            "gather": gather,
            "plan": {"prepare_ms_once": round(prep_ms, 3), "tiles": plan_stats["tiles"],
                     "lds_tiles": plan_stats["lds_tiles"],
                     "direct_tiles": plan_stats["direct_tiles"],
                     "blend_tiles_32x64": plan_stats["blend_tiles"],
                     "mb_bands": plan_stats["mb_bands"],
                     "mb_mixed_px_per_capture": plan_stats["mb_mixed_px"],
                     "mb_r1_entries_per_capture": plan_stats["mb_r1_entries"],
                     "table_mb": round(plan_stats["table_bytes"] / 1e6, 2),
                     "seams": None if seam_k is None else {
                         "method": "graph-cut (mcs_plan_find_seams, device push-relabel)",
                         "grid_log2": seam_k, "ms_once": round(seam_ms, 2),
                         "labels_equal_restatement": seams_equal}},
            "kernels": {"launch_ms": round(launch_ms, 4),
                        "paste_only_launch_ms": None if paste_ms is None else round(paste_ms, 4)},
            "roofline": {
                "bound": "hbm",
                "kernel": "mcs_stream_c%d%s (one launch)" % (
                    C, {"multiband": " + mcs_mb_bands(_br)_c%d + mcs_mb_blend_c%d" % (C, C),
                        "feather": " + mcs_feather_c%d_i1" % C, "none": "",
                        "seam": ""}[args.blend]),
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "traffic_workload": workload,
                "build_id": _capi.build_id(),
                "bytes": "SURVEY.md 8d B_frame: every camera frame read once + the mosaic "
                         "written once, x frames per launch",
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "kernel_ms_per_launch": round(launch_ms, 4),
                # the same launch priced with the source pixels it reads with non-zero weight
                # only (a tighter lower bound on the bytes: frac_touched <= frac)
                "touched": {"algorithmic_bytes_per_launch": touched_per_launch,
                            "achieved": round(touched_per_launch / (launch_ms * 1e-3) / 1e9, 1),
                            "frac": round(touched_per_launch / (launch_ms * 1e-3) / 1e9 /
                                          HBM_PEAK_GBS, 4)},
                # which fraction is the honest one: a cylinder's cameras are read only where the
                # panorama's rows curve through them (B_frame counts every frame byte), a chain
                # rig's B_frame and touched bytes differ by the few frame pixels no stage reads
                "honest_frac": "touched" if cyl else "frac",
                # the HBM-bound streaming kernel alone (the paste-only launch: the same gather
                # over every tile without the blend passes), same algorithmic bytes
                "stream_kernel": None if paste_ms is None else {
                    "achieved": round(bytes_per_launch / (paste_ms * 1e-3) / 1e9, 1),
                    "frac": round(bytes_per_launch / (paste_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "frac_touched": round(touched_per_launch / (paste_ms * 1e-3) / 1e9 /
                                          HBM_PEAK_GBS, 4),
                    "ms_per_launch": round(paste_ms, 4)},
            },
            "cpu_baseline": cpu,
        }
        if world == 1 and not args.no_also and not cyl and args.blend == "multiband":
            result["also"] = companion_lines()
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


def _child_line(cmd, timeout, keep):
    """Runs one companion benchmark as a child process (its own GPU context) and keeps `keep`
    fields of its JSON line; an error string instead of failing the headline line."""
    import subprocess
    try:
        r = subprocess.run([sys.executable] + cmd, cwd=ROOT, capture_output=True, text=True,
                           timeout=timeout)
        line = json.loads(r.stdout.strip().splitlines()[-1])
        return {k: line.get(k) for k in keep if k in line}
    except Exception as e:   # noqa: BLE001 -- recorded, the headline line stands
        return {"error": f"{type(e).__name__}: {str(e)[:200]}"}


def companion_lines():
    """SURVEY.md 8 configs beside the headline C2 line, measured in the same driver run: C4 (8-cam
    cylinder, multi-band, bench.py --rig cylinder), C3 (per-capture estimation + stitch through
    the rig jobs, frames uploaded every capture, tools/estimate_bench.py), the Hamming matcher's
    pairs/s (tools/match_bench.py), the C4 graph-cut seams per plan (tools/seam_bench.py) and the
    C5 4K stream (host frames in, host mosaics out, tools/stream_bench.py)."""
    return {
        "c4_cylinder_multiband": _child_line(
            ["bench.py", "--rig", "cylinder", "--no-cpu-baseline", "--no-also"], 400,
            ("metric", "value", "unit", "ms_per_step", "max_abs_diff", "config", "roofline",
             "kernels")),
        "c3_estimate_and_stitch": _child_line(
            ["tools/estimate_bench.py", "--stitch", "--pipelined", "--overlap", "--depth", "4",
             "--steps", "300", "--warmup", "20", "--no-cpu-baseline"], 300,
            ("metric", "value", "unit", "ms_per_step", "stitched_mpix_per_s", "config",
             "latency_ms_upload_to_homographies", "h2d_gb_per_s", "h2d_link_ceiling_gb_per_s",
             "frac_of_h2d_link", "max_reproj_err_px_vs_truth", "max_abs_diff_vs_cpu_render")),
        "hamming_matcher": _child_line(["tools/match_bench.py"], 200,
                                       ("metric", "unit", "sizes", "ops_per_pair",
                                        "peak_lane_ops_per_s")),
        "c4_seams": _child_line(["tools/seam_bench.py", "--no-check"], 200,
                                ("metric", "ms_per_plan", "grid", "max_flow",
                                 "stats_pairs_push_relabel_globalrelabels_us")),
        "c5_stream_4k": _child_line(["tools/stream_bench.py", "--sizes", "3840x2160",
                                     "--frames", "200", "--summary"], 300,
                                    ("metric", "unit", "lines")),
    }


def gather_all(d_out, args, shard, torch, dev, reps: int = 3):
    """Deliver every rank's F finished mosaics (the whole output batch) to rank 0 through the
    libmcs RCCL group (mcs_group_gather: one grouped send/recv, each peer over its own xGMI
    link), outside the timed region; verified by a checksum of checksums.  Reported separately:
    best-of-`reps` time, max over ranks."""
    import torch.distributed as dist
    from multicamera_stitching_amd import _capi
    world, rank = dist.get_world_size(), dist.get_rank()
    group = shard.mcs_group(dev.index)
    recv = (torch.empty((world,) + tuple(d_out.shape), dtype=torch.uint8, device=dev)
            if rank == 0 else None)
    stream = torch.cuda.current_stream().cuda_stream
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        dist.barrier()
        t = time.perf_counter()
        shard.gather_mosaics_group(group, d_out, recv, 0, stream)
        torch.cuda.synchronize()
        dt = shard.max_over_ranks([time.perf_counter() - t], device=dev)[0]
        best = dt if best is None else min(best, dt)
    mine = torch.tensor([shard.checksum(d_out)], dtype=torch.int64, device=dev)
    sums = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(sums, mine)
    ok = True
    if rank == 0:
        ok = all(shard.checksum(recv[r]) == int(sums[r].item()) for r in range(world))
    flag = torch.tensor([1 if ok else 0], dtype=torch.int64, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    group.close()
    moved = (world - 1) * d_out.numel()
    return {"what": f"all {d_out.shape[0]} mosaics of every rank -> rank 0 "
                    f"(mcs_group_gather: RCCL grouped send/recv)",
            "rccl": _capi.rccl_library(),
            "bytes_into_rank0": moved, "ms": round(best * 1e3, 3),
            "GBps_into_rank0": round(moved / best / 1e9, 1), "verified": bool(flag.item()),
            "in_timed_region": args.gather == "timed"}


def stub_main(args, world, rank):
    """CPU rehearsal of the multi-rank bench orchestration (gloo): the same spawn, world check,
    timed region, max over ranks, job rate and verified gather as the GPU path, around a stub
    step (a small host copy standing in for one stitch launch)."""
    import torch
    import torch.distributed as dist
    from multicamera_stitching_amd import shard
    if world > 1:
        dist.init_process_group("gloo")
    dev = torch.device("cpu")
    F, out_h, out_w, C = 4, 32, 48, 3
    src = torch.arange(F * out_h * out_w * C, dtype=torch.int64).remainder(251).to(torch.uint8)
    d_out = torch.empty((F, out_h, out_w * C), dtype=torch.uint8)

    def step():
        d_out.view(-1).copy_(src.roll(rank + 1))
        time.sleep(0.002 * (rank + 1))          # ranks of different speed: max over ranks

    elapsed = shard.timed_loop(step, args.steps, args.warmup, lambda: None)
    mine = elapsed
    elapsed = shard.max_over_ranks([elapsed], device=dev)[0]
    # every rank checks its own output against an independent restatement (numpy), max over
    # ranks -- the same reduction as the GPU path's per-rank oracle check
    want = np.roll(src.numpy(), rank + 1)
    max_abs = int(np.abs(d_out.view(-1).numpy().astype(np.int16) - want.astype(np.int16)).max())
    max_abs = shard.max_abs_over_ranks(max_abs, device=dev)
    mpix = F * out_w * out_h / 1e6
    gather = None
    if world > 1 and args.gather != "none":
        got, ok = shard.gather_and_verify(d_out, dst=0, device=dev)
        gather = {"verified": ok, "ranks": None if got is None else len(got),
                  "bytes_into_rank0": (world - 1) * d_out.numel()}
    result = None
    if rank == 0:
        result = {"metric": "stub (orchestration rehearsal, no GPU)",
                  "value": round(shard.job_rate(mpix, args.steps, elapsed, world), 6),
                  "unit": "MPix/s", "n_gpus": world, "steps": args.steps,
                  "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
                  "rank0_seconds": mine, "max_seconds": elapsed,
                  "mpix_per_step_per_rank": mpix, "higher_is_better": True, "scaling": "weak",
                  "max_abs_diff": max_abs, "gather": gather, "config": {"workload": "stub"}}
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


def describe_workload(args, cyl):
    if cyl and args.seam == "graphcut" and args.blend in ("multiband", "feather", "seam"):
        what = {"multiband": "graph-cut seams (SURVEY.md 8 NS-6, once per plan) + 3-level "
                             "multi-band blend (NS-1)",
                "feather": "graph-cut seams + linear feather blend",
                "seam": "graph-cut seams, no blend"}[args.blend]
        return (f"C4 rig: {args.cams} x {args.width}x{args.height} BGR cameras at "
                f"{360.0 / args.cams:g} degree yaw steps, f = {args.focal:g}, cylindrical warp "
                f"({args.interp}) + {what}")
    what = {"multiband": "3-level multi-band blend (SURVEY.md 8 NS-1)",
            "feather": "linear feather blend (SURVEY.md 8 NS-2)",
            "seam": "distance seam, no blend",
            "none": "overwrite paste (the reference's StitcherClass semantics)"}[args.blend]
    if cyl:
        return (f"C4 rig: {args.cams} x {args.width}x{args.height} BGR cameras at "
                f"{360.0 / args.cams:g} degree yaw steps, f = {args.focal:g}, cylindrical warp "
                f"({args.interp}) + {what}")
    return (f"C2 rig: {args.cams} x {args.width}x{args.height} BGR cameras, precomputed "
            f"homographies, {args.interp} warpPerspective + {what}")


def host_cpus() -> dict:
    """The host's CPUs as this process sees them: nproc (every CPU of the machine), the affinity
    set, the cgroup quota, and `usable` = the cores this process may actually run on at once
    (the CPU baseline's thread count), plus the lscpu model name."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.lower().startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"nproc": nproc, "affinity": aff, "cgroup_quota_cpus": quota, "usable": usable,
            "model": model}


def oracle_runner(st, args, interp, plan, blend, cyl=None, seams=None):
    """The workload's CPU restatement (oracle/, test infrastructure) as run(cams) -> mosaic, plus
    the reference-structured cascade (paste only) and the flattened gather, for the baseline.
    Returns {"workload": (run, what), "cascade": ..., "flat": ...} (None where not defined).
    seams = (k, labels): graph-cut seams found once per plan (the labels are checked equal to the
    restatement's own cut of the same capture by the caller); every capture follows them."""
    from oracle import oracle
    out = {"cascade": None, "flat": None}
    if st is not None:
        stages = [dict(H=np.asarray(sb.cachedAH), canvas_w=sb.ABSize[0], canvas_h=sb.ABSize[1],
                       bx=sb.Bpts[0][0], by=sb.Bpts[0][1], super_mode=sb.super_mode,
                       x_limits=sb.x_limits, y_limits=sb.y_limits) for sb in st.stitchers]
        out["cascade"] = (lambda cams: oracle.cascade_stitch(stages, cams, interp),
                          "reference-structured cascade: per-stage warpPerspective into the full "
                          "stage canvas + overwrite paste + crop (StitcherClass.py:114-136,"
                          "211-256), mcs_oracle.c")
    if blend == 0:
        out["workload"] = out["cascade"]
        if st is not None:
            flat = plan.describe()
            out["flat"] = (lambda cams: oracle.flat_stitch(flat, cams, interp),
                           "flattened single-pass gather (mcs_oracle.c orc_flat_stitch)")
    elif cyl is not None:
        rig_cams, g = cyl
        sk, lab = seams if seams is not None else (None, None)
        out["workload"] = (
            lambda cams: oracle.blend_stitch_cyl(rig_cams, g["out_w"], g["out_h"], g["f_cyl"],
                                                 g["u0"], g["v0"], cams, blend, interp,
                                                 seam_k=sk, seam_labels=lab),
            {1: "feather", 2: "3-level multi-band", 3: "seam"}[blend] +
            " cylindrical panorama (orc_blend.c" +
            (", graph-cut seams of the plan, orc_seam.c)" if sk is not None else ")"))
    else:
        flat = plan.describe()
        out["workload"] = (lambda cams: oracle.blend_stitch(flat, cams, blend, interp),
                           {1: "feather", 2: "3-level multi-band", 3: "seam"}[blend] +
                           " blend (orc_blend.c)")
    return out


def check_frame0(runner, cams, frame0, threads) -> int:
    """max |GPU - CPU restatement| over one capture (the portable, test-pinned oracle build)."""
    from oracle import oracle
    oracle.set_threads(threads)
    want = runner["workload"][0](cams)
    return int(np.abs(want.astype(np.int16) - frame0.astype(np.int16)).max())


def _time_line(run, cams, threads, seconds, mpix, what, max_n=5000):
    from oracle import oracle
    oracle.set_threads(threads)
    n = 0
    t0 = time.perf_counter()
    while True:
        run(cams)
        n += 1
        dt = time.perf_counter() - t0
        if dt >= seconds or n >= max_n:
            break
    return {"what": what, "threads": threads, "value": round(n * mpix / dt, 3), "unit": "MPix/s",
            "captures": n, "seconds": round(dt, 2)}


def cpu_baseline(runner, cams, args, out_w, out_h, host):
    """The same workload on the GPU box's own host cores (oracle/, C restatement):
    built -O3 -march=native here (the portable build if that fails), a bounded sample per line:
    the workload at every usable core (the headline) and at 1 thread, the reference-structured
    cascade (paste) at every usable core and at 1 thread, and the flattened gather."""
    import tempfile
    from oracle import oracle
    mpix = out_w * out_h / 1e6
    build = "-O3 -march=native"
    path = None
    try:
        path = oracle.build_native(os.path.join(tempfile.mkdtemp(prefix="mcs_orc_"),
                                                "liboracle_native.so"))
    except Exception as e:   # (a missing compiler on the host: the portable build, said so)
        build = f"-O3 -march=x86-64-v2 (native build failed: {type(e).__name__})"
    n_all = host["usable"]
    sec = args.cpu_seconds
    lines = []
    ctx = oracle.library(path) if path else _null_ctx()
    with ctx:
        run, what = runner["workload"]
        native_exact = None
        if path:
            want = runner["workload"][0](cams)
            with oracle.library(os.path.join(os.path.dirname(oracle.__file__), "liboracle.so")):
                native_exact = bool(np.array_equal(want, run(cams)))
        head = _time_line(run, cams, n_all, sec, mpix, what)
        lines.append(head)
        lines.append(_time_line(run, cams, 1, sec / 2, mpix, what))
        if runner["cascade"] is not None and runner["cascade"] is not runner["workload"]:
            # (blend workloads: the reference-structured paste cascade beside them)
            lines.append(_time_line(runner["cascade"][0], cams, n_all, sec / 2, mpix,
                                    runner["cascade"][1]))
            lines.append(_time_line(runner["cascade"][0], cams, 1, sec / 2, mpix,
                                    runner["cascade"][1]))
        if runner["flat"] is not None:
            lines.append(_time_line(runner["flat"][0], cams, n_all, sec / 2, mpix,
                                    runner["flat"][1]))
    return {
        "value": head["value"],
        "unit": "MPix/s",
        "cores": n_all,
        "kind": "port",
        "sample": f"{head['captures']} captures of the same rig through the {what} C "
                  f"restatement, {head['seconds']} s, OpenMP {n_all} threads "
                  f"(every core this process may use), built {build}",
        "build": build,
        "native_equals_portable": native_exact,
        "host": host,
        "lines": lines,
    }


class _null_ctx:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


if __name__ == "__main__":
    main()

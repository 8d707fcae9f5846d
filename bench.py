#!/usr/bin/env python3
"""Benchmark of the stitch hot path: stitched MPix/s on a synthetic 4 x 1920x1080 rig.

Workload (BASELINE.json configs[1]): 4 x 1920x1080 BGR cameras, precomputed homographies,
bilinear warp + 3-level multi-band blend (--blend multiband, the default); --blend none is the
reference's own per-stage semantics (warpPerspective + overwrite paste, StitcherClass.py:211-256)
and --blend feather the linear feather blend.  One "step" = one stitch launch over --frames rig
captures already resident in HBM (4 camera frames each), producing --frames mosaics: the
streaming gather kernel over every tile, then (blend modes) the blend kernel over the tiles the
blend changes.  Captures 0, F/2 and F-1 of the last timed step are checked against the CPU
restatement on every rank ("max_abs_diff", max over ranks and captures).

Multi-GPU (python bench.py --gpus N, or python -m torch.distributed.run ... bench.py --gpus N):
one process per GPU; capture g goes to rank g mod N (weak scaling, no data-path collective);
barrier + synchronize around the timed region, time = max over ranks.  Every N (1 included) also
measures, in the same rank processes, BASELINE configs[3] (C4: 8-camera cylinder + graph-cut +
multi-band, the mosaics gathered to rank 0 through mcs_group_gather) and configs[4] (C5: each
rank streams its share of 4 x 3840x2160 host captures through its own mcs_stream pipeline; the
last mosaics gathered to rank 0), under "also".

Extra fields: "roofline" (HBM-bound; algorithmic bytes = SURVEY.md 8d's B_frame -- every camera
frame read once + the mosaic written once -- per launch, over the launch's average duration
measured with HIP events on its stream; "touched" prices only the source pixels the mosaic reads;
both are lower bounds for the blend modes, whose seam tiles re-read their neighbourhoods),
"kernels" (the same launch without the blend pass, for the blend's share), and "cpu_baseline"
(the C restatement in oracle/, on the host cores, rank 0 only, bounded sample).
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse(argv=None):
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
                         "over xGMI) after the timed region ('after': a verified one-shot gather "
                         "plus a second timed loop of stitch + gather steps, reported as "
                         "'gather'), or as part of every timed step of the line itself ('timed')")
    ap.add_argument("--stream-frames", type=int, default=120,
                    help="C5 line: host captures each rank streams in its timed region")
    ap.add_argument("--stub", action="store_true",
                    help="CPU rehearsal of the multi-rank orchestration (gloo, stub steps): "
                         "no GPU, no libmcs; tests/test_bench_dist.py")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-also", action="store_true",
                    help="skip the companion lines (C4 cylinder and C5 4K stream at this N; at "
                         "N = 1 also C3 estimate + stitch, matcher, C4 seams)")
    ap.add_argument("--no-paste-ref", action="store_true",
                    help="skip the paste-only reference launch (PMC passes: one plan's dispatches)")
    ap.add_argument("--pmc-json", default=None,
                    help="counter summary for roofline.traffic (default profiles/pmc_latest.json, "
                         "profiles/pmc_latest_cyl.json with --rig cylinder)")
    return ap.parse_args(argv)


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


class Ctx:
    """This rank's place in the job: world, rank, its torch device."""

    def __init__(self, world, rank, dev):
        self.world, self.rank, self.dev = world, rank, dev


# ---- orchestration shared by the GPU lines and the --stub rehearsal ------------------------------

def capture_index(f: int, ctx: Ctx) -> int:
    """Global index of this rank's local capture f (capture g -> rank g mod N, shard.shard_frames)."""
    return f * ctx.world + ctx.rank


def check_captures(F: int):
    """The captures of a launch every rank checks against the oracle: first, middle, last."""
    return sorted({0, F // 2, F - 1})


def timed_rate(step, steps, warmup, sync, units_per_step, ctx, record=None):
    """The contract's timed region for one line on every rank (shard.timed_loop: barrier +
    synchronize on both sides), the slowest rank's seconds and the whole-job rate."""
    from multicamera_stitching_amd import shard
    mine = shard.timed_loop(step, steps, warmup, sync, record)
    slowest = shard.max_over_ranks([mine], device=ctx.dev)[0]
    return {"seconds_rank": mine, "seconds_max": slowest,
            "value": shard.job_rate(units_per_step, steps, slowest, ctx.world),
            "ms_per_step": slowest / steps * 1e3}


def pipeline_loop(submit, collect, depth, frames, warmup, units_per_capture, ctx):
    """C5's timed region: a ring of `depth` captures in flight (submit() -> token, collect(token)
    the oldest when the ring is full), drained before and after the timed captures; the same
    barrier / max-over-ranks bracket as every other line."""
    ring = []

    def step():
        if len(ring) == depth:
            collect(ring.pop(0))
        ring.append(submit())

    def drain():
        while ring:
            collect(ring.pop(0))
    return timed_rate(step, frames, warmup, drain, units_per_capture, ctx)


# ---- the GPU lines -------------------------------------------------------------------------------

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
        # (a bounded collective timeout: a rank that fails inside a companion line must not
        # leave the others waiting forever)
        import datetime
        dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                timeout=datetime.timedelta(seconds=300))
    else:
        torch.cuda.set_device(0)
    ctx = Ctx(world, rank, torch.device("cuda", torch.cuda.current_device()))

    result = rig_line(args, ctx, cpu=world == 1 and not args.no_cpu_baseline)
    if not args.no_also and args.rig == "chain" and args.blend == "multiband":
        # BASELINE configs[3] and configs[4] at this N, in these same rank processes
        also = {"c4_cylinder_multiband": guarded(lambda: rig_line(c4_args(args), ctx, cpu=False),
                                                 ctx, "c4"),
                "c5_stream_4k": guarded(lambda: stream_line(args, ctx), ctx, "c5")}
        if rank == 0:
            if world == 1:
                also.update(companion_lines())
            result["also"] = also
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


class PeerFailed(RuntimeError):
    """Another rank's line failed (it said so at this collective)."""


def _flag_min(ctx, ok: bool) -> bool:
    """All ranks' agreement (MIN of a 0/1 flag): one collective."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=ctx.dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.item()))


def guarded(fn, ctx, name="line"):
    """A companion line: its result, or an error in its place (the headline line stands).

    Every rank runs it.  At N > 1 each collective inside the line is preceded by an agreement
    flag (shard.set_collective_guard): a rank whose line raises contributes 0 at the others' next
    collective point -- they stop with PeerFailed instead of waiting out the 300 s collective
    timeout -- and every rank's error message is gathered to rank 0, which reports them all
    ({"error": ..., "rank_errors": {rank: message}}).  Protocol: a failing rank makes exactly
    one flag call (in its handler); a healthy rank makes one per collective point plus one at the
    end unless a flag already told it of a failure -- so the calls always pair.  (A failure inside
    a collective itself is not covered: the timeout bounds that.)"""
    from multicamera_stitching_amd import shard
    if ctx.world == 1:
        try:
            return fn()
        except Exception as e:   # noqa: BLE001 -- recorded in the line
            return {"error": f"{type(e).__name__}: {str(e)[:300]}"}
    import torch.distributed as dist

    def check():
        if not _flag_min(ctx, True):
            raise PeerFailed(f"another rank's {name} line failed")
    prev = shard.set_collective_guard(check)
    res, err, flagged = None, None, False
    try:
        res = fn()
    except PeerFailed as e:
        err, flagged = f"{type(e).__name__}: {e}", True
    except Exception as e:   # noqa: BLE001 -- recorded in the line
        err = f"{type(e).__name__}: {str(e)[:300]}"
    finally:
        shard.set_collective_guard(prev)
    if not flagged and not _flag_min(ctx, err is None) and err is None:
        err = f"PeerFailed: another rank's {name} line failed"
    errs = [None] * ctx.world
    dist.all_gather_object(errs, err)
    if ctx.rank != 0:
        return None
    bad = {r: e for r, e in enumerate(errs) if e is not None}
    if not bad:
        return res
    first = min(bad, key=lambda r: (bad[r].startswith("PeerFailed"), r))
    return {"error": f"rank {first}: {bad[first]}", "rank_errors": bad}


def _inject_failure(ctx, line):
    """Test hook (tests/test_bench_dist.py): MCS_BENCH_INJECT_FAIL=rank:line makes that rank's
    line raise after its timed region, before its parity / gather collectives."""
    v = os.environ.get("MCS_BENCH_INJECT_FAIL", "")
    if v and v == f"{ctx.rank}:{line}":
        raise RuntimeError(f"injected failure on rank {ctx.rank} in line {line}")


def c4_args(args):
    """BASELINE configs[3]: 8 x 1920x1080 cylinder, graph-cut seams, 3-level multi-band."""
    a = copy.copy(args)
    a.rig, a.cams, a.blend, a.seam = "cylinder", None, "multiband", "graphcut"
    a.pmc_json = None
    return a


def rig_line(args, ctx, cpu):
    """One bench line over a rig plan (args.rig): the timed launches, the paste-only reference,
    roofline, parity of captures 0, F/2, F-1 on every rank, the gather to rank 0 at N > 1, and the
    CPU baseline (cpu=True, rank 0).  Returns the line on rank 0, None elsewhere."""
    import torch
    from multicamera_stitching_amd import rig, shard, _capi
    from multicamera_stitching_amd.StitcherClass import _stage_desc

    world, rank, dev = ctx.world, ctx.rank, ctx.dev
    interp = _capi.MCS_INTER_LINEAR if args.interp == "linear" else _capi.MCS_INTER_NEAREST
    cyl = args.rig == "cylinder"
    n_cams = args.cams if args.cams is not None else (8 if cyl else 4)
    if cyl and args.blend == "none":
        raise SystemExit("bench: a cylindrical rig has no paste order (use --blend seam)")
    st = geo = rig_cams = None
    if cyl:
        rig_cams, cams, geo = rig.cylinder_rig(n_cams, args.width, args.height, args.focal,
                                               args.channels, seed=0, jitter_deg=0.5)

        def make_plan():
            return _capi.Plan.cylindrical(rig_cams, geo["out_w"], geo["out_h"], geo["f_cyl"],
                                          geo["u0"], geo["v0"], args.channels, interp,
                                          device=dev.index)
    else:
        st, images, _ = rig.calibrated_stitcher(n_cams, args.width, args.height,
                                                args.channels, super_mode=args.super_mode,
                                                seed=0)
        cams = [images[label] for label in st.img_labels]
        descs = [_stage_desc(sb) for sb in st.stitchers]

        def make_plan():
            return _capi.Plan(descs, args.width, args.height, args.channels, interp,
                              device=dev.index)
    plan = make_plan()
    seam_k = seam_labels = None
    if cyl and args.seam == "graphcut":
        # calibration-time step (once per plan, outside the timed region): graph-cut seams on
        # the 2^2 grid from one capture (the rig's capture 0, the same on every rank); every
        # timed capture then follows those seams
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

    # device-resident inputs: F captures per camera; global capture g = the camera texture
    # rolled by g rows, this rank's local capture f is g = f * N + rank
    d_cams = []
    for c in cams:
        base = torch.from_numpy(c).to(dev)
        d_cams.append(torch.stack([torch.roll(base, shifts=capture_index(f, ctx) % c.shape[0],
                                              dims=0)
                                   for f in range(F)]).contiguous())
        del base
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
    group = recv = None
    if world > 1 and args.gather != "none":
        group = shard.mcs_group(dev.index)
        recv = (torch.empty((world,) + tuple(d_out.shape), dtype=torch.uint8, device=dev)
                if rank == 0 else None)
    if world > 1 and args.gather == "timed":
        # every step also delivers the F mosaics of every rank to rank 0 (mcs_group_gather)
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

    mpix_per_launch = F * out_w * out_h / 1e6
    timed = timed_rate(step, args.steps, args.warmup, torch.cuda.synchronize, mpix_per_launch,
                       ctx, record)
    _inject_failure(ctx, "c4" if cyl else "c2")
    launch_ms = shard.max_over_ranks([float(np.mean([a.elapsed_time(b) for a, b in ev]))],
                                     device=dev)[0]
    value = timed["value"]
    # the captures parity checks, read back before anything else reuses d_out
    checked = check_captures(F)
    got = {f: d_out[f, :, :out_w * C].reshape(out_h, out_w, C).cpu().numpy() for f in checked}
    gather = None
    if group is not None:
        try:
            gather = gather_all(d_out, args, stitch, group, recv, stream, ctx, mpix_per_launch)
        except Exception as e:   # (outside the timed region: the line still reports the run)
            gather = {"error": f"{type(e).__name__}: {e}"}
        group.close()
        del recv

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
    fp = plan.footprint()
    del d_cams, d_out
    plan.close()
    torch.cuda.empty_cache()

    # algorithmic bytes per launch: B_frame = every camera frame read once + the
    # mosaic written once (the roofline's bytes); beside it the touched-pixel figure: only the
    # source pixels the mosaic reads with non-zero weight (counted on the device)
    bframe = out_w * out_h * C + sum(int(np.prod(c.shape)) for c in cams)
    bytes_per_launch = F * bframe
    achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
    touched_per_launch = F * (out_w * out_h * C + sum(fp) * C)
    traffic = None
    workload = (f"{n_cams}x{args.width}x{args.height}x{C}-{args.interp}-"
                f"super{int(args.super_mode)}-F{F}-{args.blend}")
    if cyl:
        workload = f"cyl-f{args.focal:g}-" + workload + ("-gc2" if seam_k is not None else "")
    traffic_src = traffic_sized = None
    try:
        pmc_json = args.pmc_json
        if pmc_json is None:
            pmc_json = os.path.join(ROOT, "profiles",
                                    "pmc_latest_cyl.json" if cyl else "pmc_latest.json")
        pm = json.load(open(pmc_json))
        # counters count only for the kernels they were taken on: same workload AND same build
        # of the embedded code objects (mcs_build_id), else traffic stays null
        if pm.get("workload") == workload and pm.get("build_id") == _capi.build_id():
            traffic = pm.get("hbm_bytes_per_launch")
            traffic_sized = pm.get("hbm_bytes_sized_per_launch")
            traffic_src = os.path.relpath(pmc_json, ROOT)
    except (OSError, ValueError):
        pass

    # parity on EVERY rank (outside the timed region): this rank's captures 0, F/2 and F-1 of the
    # last timed step against the CPU restatement fed the same camera frames; the line reports
    # the max over captures and ranks
    runner = oracle_runner(st, args, interp, plan, blend, (rig_cams, geo) if cyl else None,
                           seams=(seam_k, seam_labels) if seam_k is not None else None)
    host = host_cpus()
    threads = max(1, host["usable"] // ctx.world)
    diffs = {}
    for f in checked:
        shift = [capture_index(f, ctx) % c.shape[0] for c in cams]
        diffs[f] = check_frame(runner, [np.roll(c, s, axis=0) for c, s in zip(cams, shift)],
                               got[f], threads)
    max_abs = shard.max_abs_over_ranks(max(diffs.values()), device=dev)
    seams_equal = None
    if seam_k is not None and rank == 0:
        # the plan's cut of capture 0 against the restatement's (orc_seam.c) on the same frames
        from oracle import oracle
        _, want_lab = oracle.blend_stitch_cyl(rig_cams, geo["out_w"], geo["out_h"], geo["f_cyl"],
                                              geo["u0"], geo["v0"], cams, _capi.MCS_BLEND_SEAM,
                                              interp, seam_k=seam_k, want_seams=True)
        seams_equal = bool(np.array_equal(want_lab, seam_labels))

    if rank != 0:
        return None
    cpu_line = cpu_baseline(runner, cams, args, out_w, out_h, host) if cpu else None
    result = {
        "metric": ("stitched MPix/sec (8-cam 360 cylindrical rig)" if cyl else
                   "stitched MPix/sec (4-cam 1080p rig)"),
        "value": round(value, 3),
        "unit": "MPix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(timed["ms_per_step"], 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": describe_workload(args, cyl, n_cams),
            "blend": args.blend,
            "mosaic": [out_h, out_w, C],
            "frames_per_step": F,
            "super_mode": bool(args.super_mode),
            "parallelism": (f"captures sharded over {world} GPU(s) (capture g -> rank g mod "
                            f"{world}), no data-path collective" +
                            ("; every step gathers all mosaics to rank 0"
                             if world > 1 and args.gather == "timed" else "")),
        },
        "max_abs_diff": max_abs,
        "checked_captures": {"per_rank": checked, "ranks": world,
                             "max_abs_diff_rank0": {str(f): d for f, d in diffs.items()}},
        "gather": gather,
        "plan": {"prepare_ms_once": round(prep_ms, 3), "tiles": plan_stats["tiles"],
                 "lds_tiles": plan_stats["lds_tiles"],
                 "direct_tiles": plan_stats["direct_tiles"],
                 "blend_tiles_32x64": plan_stats["blend_tiles"],
                 "mb_bands": plan_stats["mb_bands"],
                 "mb_bands_lds_ring": plan_stats["mb_bands_lds"],
                 "big_footprint_tiles": plan_stats["big_tiles"],
                 "mb_mixed_px_per_capture": plan_stats["mb_mixed_px"],
                 "mb_r1_entries_per_capture": plan_stats["mb_r1_entries"],
                 "table_mb": round(plan_stats["table_bytes"] / 1e6, 2),
                 # streaming reads per launch: what the footprint DMAs fetch (row spans in 16-B
                 # chunks) and the footprint boxes they are cut from, beside the touched source
                 "stream_dma_gb_per_launch": round(F * plan_stats["dma_bytes_per_capture"] / 1e9, 4),
                 "stream_box_gb_per_launch": round(F * plan_stats["box_bytes_per_capture"] / 1e9, 4),
                 "touched_source_gb_per_launch": round(F * sum(fp) * C / 1e9, 4),
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
            # the same counters' read side from the sized request counts (32 / 64 / 128 B)
            # instead of FETCH_SIZE x 2 (the guide's correction assumes 128-B requests)
            "traffic_sized": traffic_sized,
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
        "cpu_baseline": cpu_line,
    }
    return result


def gather_all(d_out, args, stitch, group, recv, stream, ctx, mpix_per_launch, reps: int = 3):
    """N > 1: deliver every rank's F finished mosaics (the whole output batch) to rank 0 through
    the libmcs RCCL group (mcs_group_gather: one grouped send/recv, each peer over its own xGMI
    link).  (1) A one-shot transfer, best of `reps`, max over ranks, verified by a checksum of
    checksums; (2) a second timed loop whose steps are stitch + gather (the rate of a job that
    lands every mosaic on rank 0), unless the line's own steps already gather (--gather timed)."""
    import torch
    import torch.distributed as dist
    from multicamera_stitching_amd import _capi, shard
    world, rank, dev = ctx.world, ctx.rank, ctx.dev
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        shard._guard()
        dist.barrier()
        t = time.perf_counter()
        shard.gather_mosaics_group(group, d_out, recv, 0, stream.cuda_stream)
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
    moved = (world - 1) * d_out.numel()
    res = {"what": f"all {d_out.shape[0]} mosaics of every rank -> rank 0 "
                   f"(mcs_group_gather: RCCL grouped send/recv)",
           "rccl": _capi.rccl_library(),
           "bytes_into_rank0": moved, "ms": round(best * 1e3, 3),
           "GBps_into_rank0": round(moved / best / 1e9, 1), "verified": bool(flag.item()),
           "in_timed_region": args.gather == "timed"}
    if args.gather == "after":
        def step():
            stitch()
            shard.gather_mosaics_group(group, d_out, recv, 0, stream.cuda_stream)
        steps = max(3, args.steps // 2)
        tg = timed_rate(step, steps, 1, torch.cuda.synchronize, mpix_per_launch, ctx)
        res["stitch_and_gather"] = {"value": round(tg["value"], 3), "unit": "MPix/s",
                                    "ms_per_step": round(tg["ms_per_step"], 4), "steps": steps,
                                    "what": "timed steps of stitch + gather of every rank's "
                                            "mosaics to rank 0 (barrier + max over ranks)"}
    return res


def stream_line(args, ctx, w: int = 3840, h: int = 2160, depth: int = 3):
    """BASELINE configs[4] (C5) at this N: every rank streams its share of 4 x 3840x2160 host
    captures (capture g -> rank g mod N) through its own mcs_stream pipeline (pinned slots,
    hipGraph-captured stitch, H2D / stitch / D2H on three streams, `depth` captures in flight),
    host frames in and host mosaics out, multi-band.  Timed: barrier + max over ranks, whole-job
    captures/s and MPix/s.  After the timed region: each rank's last mosaic against the CPU
    restatement (max over ranks) and every rank's last mosaic gathered to rank 0 through
    mcs_group_gather (checksum-verified)."""
    import torch
    from multicamera_stitching_amd import _capi, rig, shard
    from multicamera_stitching_amd.StitcherClass import _stage_desc
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from stream_bench import link_probe
    dev = ctx.dev
    st, images, _ = rig.calibrated_stitcher(4, w, h, 3, seed=0)
    cams = [images[label] for label in st.img_labels]
    plan = _capi.Plan([_stage_desc(sb) for sb in st.stitchers], w, h, 3, _capi.MCS_INTER_LINEAR,
                      device=dev.index)
    plan.set_blend(_capi.MCS_BLEND_MULTIBAND)
    mpix = plan.out_w * plan.out_h / 1e6
    # two frame sets of this rank alternate (captures rank and rank + N: the rig rolled by g rows)
    sets = [[np.ascontiguousarray(np.roll(c, g % h, axis=0)) for c in cams]
            for g in (capture_index(0, ctx), capture_index(1, ctx))]
    pipe = _capi.StreamPipeline(plan, depth=depth, use_graphs=True)
    outs = [np.empty(plan.out_shape(), np.uint8) for _ in range(depth)]
    n = [0]
    last = [None]
    # N > 1: the ranks of a node share its host memory, so every frame crosses host DRAM once --
    # the producer's frames live in the pipeline's pinned slots (written there once, as a camera
    # driver or decoder would write them: mcs_stream_input / submit(NULL)) and the mosaics are
    # read in the pinned output slots (wait without a copy), no memcpy in the timed loop.  At
    # N = 1 the caller-array path (the Stitcher-like API: copy in, copy out).
    zero_copy = ctx.world > 1
    slot_set = [j % 2 for j in range(depth)]
    if zero_copy:
        for j in range(depth):
            for v, c in zip(pipe.input_views(j), sets[slot_set[j]]):
                np.copyto(v, c)

    def submit():
        if zero_copy:
            slot = pipe.submit_inplace()
            return (slot, slot_set[slot])
        k = n[0] % 2
        n[0] += 1
        return (pipe.submit(sets[k]), k)

    def collect(tok):
        slot, k = tok
        if zero_copy:
            pipe.wait(slot, copy=False)
        else:
            pipe.wait(slot, outs[slot])
        last[0] = (slot, k)
    frames = args.stream_frames
    tr = pipeline_loop(submit, collect, depth, frames, 2 * depth, mpix, ctx)
    slot, k = last[0]
    mosaic = pipe.output_view(slot).copy() if zero_copy else outs[slot].copy()
    pipe.close()
    _inject_failure(ctx, "c5")
    host = copy_workers_all_ranks(ctx)
    in_b = sum(c.nbytes for c in cams)
    pcie = frames * (in_b + mosaic.nbytes) / tr["seconds_rank"] / 1e9
    link = link_probe(in_b, mosaic.nbytes, reps=10)
    frac_min = -shard.max_over_ranks([-pcie / link["bidir_gbs"]], device=dev)[0]
    # parity: this rank's last mosaic against the multi-band restatement of its frames
    from oracle import oracle
    oracle.set_threads(max(1, host_cpus()["usable"] // ctx.world))
    want = oracle.blend_stitch(plan.describe(), sets[k], oracle.BLEND_MULTIBAND)
    diff = int(np.abs(want.astype(np.int16) - mosaic.astype(np.int16)).max())
    max_abs = shard.max_abs_over_ranks(diff, device=dev)
    gather = None
    if ctx.world > 1:
        gather = gather_last_mosaics(mosaic, ctx)
    plan.close()
    if ctx.rank != 0:
        return None
    return {"metric": "streamed 4-cam 4K rig captures/s (C5: host frames in, host mosaics out, "
                      "mcs_stream_*)",
            "value": round(frames * ctx.world / tr["seconds_max"], 2), "unit": "captures/s",
            "mpix_per_s": round(tr["value"], 1), "n_gpus": ctx.world, "frames_per_rank": frames,
            "ms_per_capture_per_rank": round(tr["ms_per_step"], 4),
            "config": {"cams": f"4x{w}x{h}x3", "blend": "multiband", "depth": depth,
                       "graphs": True, "mosaic": list(plan.out_shape()),
                       "parallelism": f"captures sharded over {ctx.world} GPU(s), each rank its "
                                      f"own host link"},
            "pcie_gb_per_s_rank0": round(pcie, 2), "link_rank0": link,
            "frac_of_link_min_over_ranks": round(frac_min, 3),
            "host_frames": ("zero-copy: frames in the pinned input slots, mosaics read in the "
                            "pinned output slots (no host memcpy per capture)" if zero_copy else
                            "caller arrays: copied into / out of the pinned slots by the copy "
                            "pool"),
            "host": host, "max_abs_diff": max_abs, "gather": gather}


def copy_workers_all_ranks(ctx):
    """The host copy-pool helpers of every rank (mcs_stream_copy_workers: the node's CPU quota
    shared by LOCAL_WORLD_SIZE ranks) and the quota itself, as rank 0 reports them."""
    from multicamera_stitching_amd import _capi
    mine = _capi.stream_copy_workers()
    allw = [mine] * ctx.world
    if ctx.world > 1:
        import torch.distributed as dist
        from multicamera_stitching_amd import shard
        shard._guard()
        allw = [None] * ctx.world
        dist.all_gather_object(allw, mine)
    return {"copy_workers_per_rank": allw, "host_cpus": host_cpus(),
            "local_world_size": int(os.environ.get("LOCAL_WORLD_SIZE", "1"))}


def gather_last_mosaics(mosaic, ctx):
    """Every rank's last C5 mosaic (host) to rank 0 through mcs_group_gather (device buffers),
    verified by a checksum of checksums; outside the timed region."""
    import torch
    import torch.distributed as dist
    from multicamera_stitching_amd import shard
    dev = ctx.dev
    d = torch.from_numpy(mosaic).to(dev).reshape(-1)
    recv = torch.empty((ctx.world, d.numel()), dtype=torch.uint8, device=dev) \
        if ctx.rank == 0 else None
    group = shard.mcs_group(dev.index)
    torch.cuda.synchronize()
    t = time.perf_counter()
    shard.gather_mosaics_group(group, d, recv, 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    dt = shard.max_over_ranks([time.perf_counter() - t], device=dev)[0]
    mine = torch.tensor([shard.checksum(d)], dtype=torch.int64, device=dev)
    sums = [torch.zeros_like(mine) for _ in range(ctx.world)]
    dist.all_gather(sums, mine)
    ok = True
    if ctx.rank == 0:
        ok = all(shard.checksum(recv[r]) == int(sums[r].item()) for r in range(ctx.world))
    flag = torch.tensor([1 if ok else 0], dtype=torch.int64, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    group.close()
    return {"what": "every rank's last mosaic -> rank 0 (mcs_group_gather)",
            "bytes_into_rank0": (ctx.world - 1) * d.numel(), "ms": round(dt * 1e3, 3),
            "verified": bool(flag.item())}


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
    """The 1-GPU companion lines beside C2, C4 and C5 (which every N measures in-process): C3
    (per-capture estimation + stitch through the rig jobs, frames uploaded every capture,
    tools/estimate_bench.py), the Hamming matcher's pairs/s (tools/match_bench.py) and the C4
    graph-cut seams per plan (tools/seam_bench.py); C3 again with the frames resident in HBM
    (the GPU-bound rate of the same estimate + stitch chain)."""
    return {
        "c3_estimate_and_stitch": _child_line(
            ["tools/estimate_bench.py", "--stitch", "--pipelined", "--overlap", "--depth", "4",
             "--steps", "300", "--warmup", "20", "--no-cpu-baseline"], 300,
            ("metric", "value", "unit", "ms_per_step", "stitched_mpix_per_s", "config",
             "latency_ms_upload_to_homographies", "h2d_gb_per_s", "h2d_link_ceiling_gb_per_s",
             "frac_of_h2d_link", "max_reproj_err_px_vs_truth", "max_abs_diff_vs_cpu_render")),
        "c3_estimate_and_stitch_resident": _child_line(
            ["tools/estimate_bench.py", "--stitch", "--pipelined", "--overlap", "--resident",
             "--depth", "4", "--steps", "400", "--warmup", "20", "--no-cpu-baseline"], 300,
            ("metric", "value", "unit", "ms_per_step", "stitched_mpix_per_s",
             "frames_resident_in_hbm", "max_reproj_err_px_vs_truth",
             "max_abs_diff_vs_cpu_render")),
        "hamming_matcher": _child_line(["tools/match_bench.py"], 200,
                                       ("metric", "unit", "sizes", "ops_per_pair",
                                        "peak_lane_ops_per_s")),
        "c4_seams": _child_line(["tools/seam_bench.py", "--no-check"], 200,
                                ("metric", "ms_per_plan", "grid", "max_flow",
                                 "stats_pairs_push_relabel_globalrelabels_us")),
    }


# ---- the CPU rehearsal ---------------------------------------------------------------------------

def stub_main(args, world, rank):
    """CPU rehearsal of the multi-rank bench orchestration (gloo): the same spawn, world check,
    timed region (timed_rate / pipeline_loop), max over ranks, job rate, per-rank parity of
    several captures reduced by max, and verified gathers as the GPU path -- for the headline
    line and for the C4 and C5 lines every N emits -- around stub steps (small host copies
    standing in for the stitch launches)."""
    import torch
    import torch.distributed as dist
    from multicamera_stitching_amd import shard
    if world > 1:
        dist.init_process_group("gloo")
    ctx = Ctx(world, rank, torch.device("cpu"))

    def stub_rig_line(F, out_h, out_w, C, metric, with_gather, line_name="c2"):
        # capture g of the job = a known byte pattern rolled by g; rank r holds g = f * N + r
        base = torch.arange(out_h * out_w * C, dtype=torch.int64).remainder(251).to(torch.uint8)
        d_out = torch.empty((F, out_h * out_w * C), dtype=torch.uint8)

        def stitch():
            for f in range(F):
                d_out[f].copy_(base.roll(capture_index(f, ctx) + 1))
            time.sleep(0.002 * (rank + 1))      # ranks of different speed: max over ranks
        mpix = F * out_w * out_h / 1e6
        tr = timed_rate(stitch, args.steps, args.warmup, lambda: None, mpix, ctx)
        _inject_failure(ctx, line_name)
        # every rank checks captures 0, F/2, F-1 against an independent restatement (numpy)
        diffs = []
        for f in check_captures(F):
            want = np.roll(base.numpy(), capture_index(f, ctx) + 1)
            diffs.append(int(np.abs(d_out[f].numpy().astype(np.int16) -
                                    want.astype(np.int16)).max()))
        max_abs = shard.max_abs_over_ranks(max(diffs), device=ctx.dev)
        gather = None
        if world > 1 and args.gather != "none" and with_gather:
            got, ok = shard.gather_and_verify(d_out, dst=0, device=ctx.dev)
            gather = {"verified": ok, "ranks": None if got is None else len(got),
                      "bytes_into_rank0": (world - 1) * d_out.numel()}

            def step_g():
                stitch()
                shard.gather_mosaics(d_out, dst=0)
            tg = timed_rate(step_g, max(3, args.steps // 2), 1, lambda: None, mpix, ctx)
            gather["stitch_and_gather"] = {"value": round(tg["value"], 6),
                                           "ms_per_step": round(tg["ms_per_step"], 4)}
        if rank != 0:
            return None
        return {"metric": metric, "value": round(tr["value"], 6), "unit": "MPix/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(tr["ms_per_step"], 4), "rank0_seconds": tr["seconds_rank"],
                "max_seconds": tr["seconds_max"], "mpix_per_step_per_rank": mpix,
                "higher_is_better": True, "scaling": "weak", "max_abs_diff": max_abs,
                "checked_captures": {"per_rank": check_captures(F), "ranks": world},
                "gather": gather, "config": {"workload": "stub"}}

    def stub_stream_line(frames=12, depth=3):
        src = [np.full((8, 12, 3), (rank * 7 + k) % 251, np.uint8) for k in range(2)]
        outs = [np.empty_like(src[0]) for _ in range(depth)]
        n = [0]
        last = [None]

        def submit():
            k = n[0] % 2
            n[0] += 1
            return (n[0] % depth, k)

        def collect(tok):
            slot, k = tok
            np.copyto(outs[slot], src[k])
            time.sleep(0.001 * (rank + 1))
            last[0] = tok
        tr = pipeline_loop(submit, collect, depth, frames, depth, 1e-4, ctx)
        _inject_failure(ctx, "c5")
        slot, k = last[0]
        diff = int(np.abs(outs[slot].astype(np.int16) - src[k].astype(np.int16)).max())
        max_abs = shard.max_abs_over_ranks(diff, device=ctx.dev)
        gather = None
        if world > 1:
            got, ok = shard.gather_and_verify(torch.from_numpy(outs[slot].copy()), dst=0,
                                              device=ctx.dev)
            gather = {"verified": ok, "ranks": None if got is None else len(got)}
        workers = copy_workers_all_ranks(ctx)
        if rank != 0:
            return None
        return {"metric": "stub stream", "value": round(frames * world / tr["seconds_max"], 3),
                "unit": "captures/s", "n_gpus": world, "frames_per_rank": frames,
                "max_abs_diff": max_abs, "gather": gather, "host": workers}

    result = stub_rig_line(4, 32, 48, 3, "stub (orchestration rehearsal, no GPU)",
                           with_gather=True)
    also = None
    if not args.no_also:
        also = {"c4_cylinder_multiband": guarded(
                    lambda: stub_rig_line(4, 16, 96, 3, "stub C4", True, "c4"), ctx, "c4"),
                "c5_stream_4k": guarded(stub_stream_line, ctx, "c5")}
    if rank == 0:
        if also is not None:
            result["also"] = also
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


# ---- descriptions, CPU restatement, baseline -----------------------------------------------------

def describe_workload(args, cyl, n_cams):
    if cyl and args.seam == "graphcut" and args.blend in ("multiband", "feather", "seam"):
        what = {"multiband": "graph-cut seams (SURVEY.md 8 NS-6, once per plan) + 3-level "
                             "multi-band blend (NS-1)",
                "feather": "graph-cut seams + linear feather blend",
                "seam": "graph-cut seams, no blend"}[args.blend]
        return (f"C4 rig: {n_cams} x {args.width}x{args.height} BGR cameras at "
                f"{360.0 / n_cams:g} degree yaw steps, f = {args.focal:g}, cylindrical warp "
                f"({args.interp}) + {what}")
    what = {"multiband": "3-level multi-band blend (SURVEY.md 8 NS-1)",
            "feather": "linear feather blend (SURVEY.md 8 NS-2)",
            "seam": "distance seam, no blend",
            "none": "overwrite paste (the reference's StitcherClass semantics)"}[args.blend]
    if cyl:
        return (f"C4 rig: {n_cams} x {args.width}x{args.height} BGR cameras at "
                f"{360.0 / n_cams:g} degree yaw steps, f = {args.focal:g}, cylindrical warp "
                f"({args.interp}) + {what}")
    return (f"C2 rig: {n_cams} x {args.width}x{args.height} BGR cameras, precomputed "
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


def check_frame(runner, cams, frame, threads) -> int:
    """max |GPU - CPU restatement| over one capture (the portable, test-pinned oracle build)."""
    from oracle import oracle
    oracle.set_threads(threads)
    want = runner["workload"][0](cams)
    return int(np.abs(want.astype(np.int16) - frame.astype(np.int16)).max())


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

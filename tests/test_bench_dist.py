"""bench.py's own multi-rank orchestration on CPU (gloo, --stub): `python bench.py --gpus 2`
spawns its two ranks itself, reports n_gpus 2, the whole-job rate over the slowest rank's time,
and a checksum-verified gather of every rank's mosaics onto rank 0; a launcher world that
disagrees with --gpus is refused."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                          capture_output=True, text=True, timeout=240, env=e, cwd=ROOT)


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_gpus2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--stub", "--steps", "4", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    res = _line(r.stdout)
    assert res["n_gpus"] == 2
    assert res["steps"] == 4 and res["warmup"] == 1
    # value = every rank's units / the slowest rank's time
    want = 2 * res["mpix_per_step_per_rank"] * 4 / res["max_seconds"]
    assert abs(res["value"] - want) <= 1e-5 * want + 1e-6
    assert res["max_seconds"] >= res["rank0_seconds"]
    g = res["gather"]
    assert (g["verified"], g["ranks"], g["bytes_into_rank0"]) == (True, 2, 4 * 32 * 48 * 3)
    # the second timed loop: steps of stitch + gather to rank 0, max over ranks
    assert g["stitch_and_gather"]["value"] > 0
    # every rank checked captures 0, F/2, F-1 of its own output; the line carries the max over
    # ranks and captures, a number
    assert res["max_abs_diff"] == 0
    assert res["checked_captures"] == {"per_rank": [0, 2, 3], "ranks": 2}
    # the C4 and C5 lines every N emits, measured by the same two ranks
    c4, c5 = res["also"]["c4_cylinder_multiband"], res["also"]["c5_stream_4k"]
    assert c4["n_gpus"] == 2 and c4["max_abs_diff"] == 0 and c4["gather"]["verified"]
    assert c4["max_seconds"] >= c4["rank0_seconds"]
    assert abs(c4["value"] - 2 * c4["mpix_per_step_per_rank"] * 4 / c4["max_seconds"]) <= \
        1e-5 * c4["value"] + 1e-6
    assert c5["n_gpus"] == 2 and c5["max_abs_diff"] == 0
    assert c5["gather"] == {"verified": True, "ranks": 2}
    assert c5["value"] > 0


def test_bench_gpus1_stub_single_process():
    r = _run(["--stub", "--steps", "2", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    res = _line(r.stdout)
    assert res["n_gpus"] == 1 and res["gather"] is None
    assert res["also"]["c4_cylinder_multiband"]["gather"] is None
    assert res["also"]["c5_stream_4k"]["gather"] is None


def test_bench_refuses_world_mismatch():
    r = _run(["--gpus", "1", "--stub", "--steps", "1"], env={"WORLD_SIZE": "2"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in (r.stderr + r.stdout)

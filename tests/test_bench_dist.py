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


def test_bench_gpus4_rank_failure_reported_not_hung():
    """A companion line that fails on rank 1 (after its timed region, before its parity and
    gather collectives): the other ranks stop at their next collective point instead of waiting
    out the 300 s collective timeout, rank 0's JSON line carries rank 1's message in that line,
    and the headline line and the other companion line stand (bench.py guarded)."""
    r = _run(["--gpus", "4", "--stub", "--steps", "2", "--warmup", "1"],
             env={"MCS_BENCH_INJECT_FAIL": "1:c4"})
    assert r.returncode == 0, r.stderr[-2000:]
    res = _line(r.stdout)
    assert res["n_gpus"] == 4 and res["max_abs_diff"] == 0
    c4 = res["also"]["c4_cylinder_multiband"]
    assert c4["error"].startswith("rank 1: RuntimeError: injected failure on rank 1"), c4
    assert set(c4["rank_errors"]) == {"0", "1", "2", "3"} or set(c4["rank_errors"]) == {0, 1, 2, 3}
    c5 = res["also"]["c5_stream_4k"]
    assert "error" not in c5 and c5["n_gpus"] == 4 and c5["gather"]["verified"]


def test_bench_gpus4_copy_pool_shared_by_ranks():
    """The C5 line's host copy pool is sized per rank: the node's CPU quota divided among the
    LOCAL_WORLD_SIZE ranks (mcs_stream_copy_workers), so N ranks never start more copy threads
    than the node's CPUs (verdict round 5: 7 per rank x 8 ranks on a 16-CPU quota)."""
    r = _run(["--gpus", "4", "--stub", "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    host = _line(r.stdout)["also"]["c5_stream_4k"]["host"]
    assert host["local_world_size"] == 4
    usable = host["host_cpus"]["usable"]
    for w in host["copy_workers_per_rank"]:
        assert 0 <= w <= max(0, min(7, (usable // 4) // 2 - 1)), host
    assert sum(w + 1 for w in host["copy_workers_per_rank"]) <= max(usable, 4), host

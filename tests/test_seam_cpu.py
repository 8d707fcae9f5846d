"""Graph-cut seams on the CPU: the product's host max-flow (Dinic,
mcs_seam_graphcut_host) against the oracle's independent restatement (Edmonds-Karp with
capacity scaling, oracle/orc_seam.c) -- the labels agree because both return the minimal
minimum cut -- and the seam's purpose: it crosses the overlaps where the cameras agree."""
import numpy as np
import pytest

from multicamera_stitching_amd import _capi, rig
from oracle import oracle


def _random_case(rng, trial):
    n = int(rng.integers(2, 6))
    gh, gw = int(rng.integers(4, 50)), int(rng.integers(4, 70))
    C = int(rng.integers(1, 5))
    cov = np.zeros((gh, gw), np.uint16)
    starts = np.sort(rng.integers(0, gw, size=n))
    for c in range(n):
        x0 = int(starts[c]) - int(rng.integers(0, gw // 2 + 1))
        x1 = int(starts[c]) + int(rng.integers(3, gw // 2 + 4))
        y0, y1 = int(rng.integers(0, gh // 3 + 1)), gh - int(rng.integers(0, gh // 3 + 1))
        cov[max(y0, 0):y1, max(x0, 0):min(x1, gw)] |= 1 << c
    smp = rng.integers(0, 256, size=(n, gh, gw, C)).astype(np.uint8)
    if trial % 3 == 0:
        smp = (smp // 64 * 64).astype(np.uint8)       # many equal costs: ties in the cut
    lab = np.full((gh, gw), 255, np.uint8)
    for y in range(gh):
        for x in range(gw):
            cs = [c for c in range(n) if cov[y, x] >> c & 1]
            if cs:
                lab[y, x] = cs[int(rng.integers(0, len(cs)))] if trial % 2 else cs[0]
    return lab, cov, smp


@pytest.mark.parametrize("seed", range(6))
def test_host_graphcut_matches_oracle(seed):
    rng = np.random.default_rng(seed)
    for trial in range(12):
        lab, cov, smp = _random_case(rng, trial)
        got = _capi.seam_graphcut_host(lab, cov, smp)
        want = oracle.seam_graphcut(lab, cov, smp)
        assert np.array_equal(got, want), trial
        # only points in an overlap change, and only to a camera covering them
        changed = got != lab
        assert (cov[changed] & (1 << got[changed].astype(np.int64))).all()


def test_cut_follows_the_low_cost_valley():
    """Two cameras overlapping over 30 columns and disagreeing everywhere except along a
    two-pixel-wide zig-zag valley: the cut runs through the valley (between its columns)."""
    gh, gw = 40, 60
    cov = np.zeros((gh, gw), np.uint16)
    cov[:, :45] |= 1
    cov[:, 15:] |= 2
    lab = np.where(np.arange(gw)[None, :] < 30, 0, 1).repeat(gh, 0).astype(np.uint8)
    smp = np.zeros((2, gh, gw, 1), np.uint8)
    smp[1] = 200
    path = 20 + (np.arange(gh) // 10) % 2 * 3           # columns 20 / 23 alternating
    for y in range(gh):
        smp[1, y, path[y]:path[y] + 2, 0] = 0           # the cameras agree only in the valley
    got = _capi.seam_graphcut_host(lab, cov, smp)
    assert np.array_equal(got, oracle.seam_graphcut(lab, cov, smp))
    exact = 0
    for y in range(gh):
        steps = np.flatnonzero(np.diff(got[y].astype(int)))
        assert len(steps) == 1 and abs(int(steps[0]) - int(path[y])) <= 1   # one 0 -> 1 step
        exact += int(steps[0]) == int(path[y])      # inside the valley (the cut costs 1 there)
    assert exact >= gh - 4                          # corners may be cut at the valley's shifts


def test_graphcut_seam_does_not_cut_through_an_object():
    """Cylindrical rig, an object (a bright blob) seen only by camera 1 inside its overlap with
    camera 0, straddling the distance seam: the distance seam cuts the blob in half (a hard
    step along the seam), the graph-cut seam passes beside it where the cameras agree (the blob
    shows whole or not at all), and the colour step across the seams collapses."""
    cams, frames, g = rig.cylinder_rig(8, 320, 180, 185.0, 3, seed=3, gain=0.0)
    frames = [f.copy() for f in frames]
    frames[1][40:140, 60:130] = 250
    args = (cams, g["out_w"], g["out_h"], g["f_cyl"], g["u0"], g["v0"], frames,
            oracle.BLEND_SEAM)
    d_out, d_own = oracle.blend_stitch_cyl(*args, want_owner=True)
    c_out, c_own = oracle.blend_stitch_cyl(*args, want_owner=True, seam_k=1)

    def seam_step(out, own):
        o = out.astype(int)
        h = (own[:, 1:] != own[:, :-1]) & (own[:, 1:] != 255) & (own[:, :-1] != 255)
        v = (own[1:, :] != own[:-1, :]) & (own[1:, :] != 255) & (own[:-1, :] != 255)
        s = (np.abs(o[:, 1:] - o[:, :-1]).sum(axis=2)[h].sum() +
             np.abs(o[1:] - o[:-1]).sum(axis=2)[v].sum())
        return s / (h.sum() + v.sum()), np.abs(o[:, 1:] - o[:, :-1]).sum(axis=2)[h].max()
    d_mean, d_max = seam_step(d_out, d_own)
    c_mean, c_max = seam_step(c_out, c_own)
    assert d_max > 300 and c_max < 100          # the blob edge is on the distance seam only
    assert c_mean < 0.3 * d_mean
    blob = lambda out: int((out >= 245).all(axis=2).sum())
    whole = blob(oracle.blend_stitch_cyl([cams[1]], *args[1:6], [frames[1]], oracle.BLEND_SEAM))
    assert 0 < blob(d_out) < whole and blob(c_out) in (0, whole)

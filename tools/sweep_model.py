"""Plan-time model of the multi-band sweep (tools only): owner maps of the C2 / C4 bench rigs from
the C restatement, the spec's mixed pixels (another owner's level-2 mask within reach), and per
blend-tile row the mixed column spans -> strip statistics for window widths W0."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402
from multicamera_stitching_amd import rig, _capi  # noqa: E402
from multicamera_stitching_amd.StitcherClass import _stage_desc  # noqa: E402


def refl(i, n):
    i = np.abs(i)
    return np.where(i >= n, 2 * n - 2 - i, i)


def reduce(a):
    h, w = a.shape
    mh, mw = (h + 1) // 2, (w + 1) // 2
    wt = np.array([1, 4, 6, 4, 1])
    ys = refl(2 * np.arange(mh)[:, None] + np.arange(5)[None, :] - 2, h)
    t = np.einsum("k,ykx->yx", wt, a[ys])
    xs = refl(2 * np.arange(mw)[:, None] + np.arange(5)[None, :] - 2, w)
    return np.einsum("k,ykx->yx", wt, t.T[xs].transpose(1, 0, 2).transpose(0, 1, 2)).T \
        if False else np.einsum("k,xky->yx", wt, t.T[xs])


def exp_reach(mask_c, n_f_h, n_f_w):
    """fine positions whose expand taps touch a True coarse entry"""
    hc, wc = mask_c.shape
    y = np.arange(n_f_h)
    x = np.arange(n_f_w)
    ty = [refl(np.where(y % 2 == 0, y // 2 + d, (y - 1) // 2 + (d + 1) // 2 if False else 0), hc)
          for d in (-1, 0, 1)]
    # explicit taps
    tys = []
    for yy in y:
        tys.append([refl(np.array([yy // 2 - 1, yy // 2, yy // 2 + 1]), hc)] if yy % 2 == 0
                   else [refl(np.array([(yy - 1) // 2, (yy + 1) // 2]), hc)])
    txs = []
    for xx in x:
        txs.append(refl(np.array([xx // 2 - 1, xx // 2, xx // 2 + 1]), wc) if xx % 2 == 0
                   else refl(np.array([(xx - 1) // 2, (xx + 1) // 2]), wc))
    rows = np.zeros((n_f_h, wc), bool)
    for i, t in enumerate(tys):
        rows[i] = mask_c[t[0]].any(0)
    out = np.zeros((n_f_h, n_f_w), bool)
    for j, t in enumerate(txs):
        out[:, j] = rows[:, t].any(1)
    return out


def mixed_pixels(owner):
    H, W = owner.shape
    h1, w1 = (H + 1) // 2, (W + 1) // 2
    slots = [s for s in np.unique(owner) if s != 255]
    touch = {}
    for s in slots:
        m0 = (owner == s).astype(np.int64)
        m2 = reduce(reduce(m0))
        t1 = exp_reach(m2 > 0, h1, w1)
        touch[s] = exp_reach(t1, H, W)
    mixed = np.zeros((H, W), bool)
    for s in slots:
        other = np.zeros((H, W), bool)
        for q in slots:
            if q != s:
                other |= touch[q]
        mixed |= (owner == s) & other
    return mixed


def strips(mixed, W0, margin=14, th=64):
    H, W = mixed.shape
    rows = []
    for ty in range(0, H, th):
        m = mixed[ty:ty + th].any(0)
        cols = np.flatnonzero(m)
        segs = []
        if len(cols):
            s = cols[0]
            p = cols[0]
            for c in cols[1:]:
                if c > p + 32:
                    segs.append((s & ~3, (p + 4) & ~3))
                    s = c
                p = c
            segs.append((s & ~3, (p + 4) & ~3))
        rows.append(segs)
    runs = []   # [x0, x1, row0, row1]
    open_runs = []
    for r, segs in enumerate(rows):
        nxt = []
        for (a, b) in segs:
            best = None
            for run in open_runs:
                x0, x1 = min(run[0], a), max(run[1], b)
                if x1 - x0 + 2 * margin <= W0 and min(run[1], b) > max(run[0], a) - 64:
                    best = run
                    break
            if best is not None:
                open_runs.remove(best)
                best[0], best[1], best[3] = min(best[0], a), max(best[1], b), r
                nxt.append(best)
            else:
                run = [a, b, r, r]
                runs.append(run)
                nxt.append(run)
        open_runs = nxt
    return rows, runs


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "c2"
    if which == "c2":
        st, images, _ = rig.calibrated_stitcher(4, 1920, 1080, 3, super_mode=False, seed=0)
        cams = [images[l] for l in st.img_labels]
        plan = _capi.Plan([_stage_desc(sb) for sb in st.stitchers], 1920, 1080, 3, 1)
        flat = plan.describe()
        _, owner = oracle.blend_stitch(flat, cams, 2, 1, want_owner=True)
    else:
        rig_cams, cams, geo = rig.cylinder_rig(8, 1920, 1080, None, 3, seed=0, jitter_deg=0.5)
        _, owner = oracle.blend_stitch_cyl(rig_cams, geo["out_w"], geo["out_h"], geo["f_cyl"],
                                           geo["u0"], geo["v0"], cams, 2, 1, want_owner=True,
                                           seam_k=2)
    np.save(f"/tmp/owner_{which}.npy", owner)
    mixed = mixed_pixels(owner)
    print(which, owner.shape, "mixed px", int(mixed.sum()))
    for W0 in (128, 192, 256):
        rows, runs = strips(mixed, W0)
        nseg = sum(len(s) for s in rows)
        out_cols = sum((b - a) for s in rows for (a, b) in s)
        print(f"W0={W0}: segments {nseg}, runs {len(runs)}, rows/run "
              f"{np.mean([r[3] - r[2] + 1 for r in runs]):.1f}, widths "
              f"{sorted(set(r[1] - r[0] for r in runs))[:12]}, region px/row-sum {out_cols}")


if __name__ == "__main__":
    main()

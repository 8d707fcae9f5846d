"""CPU emulation of the multi-band sweep (tools only): prepare_sweep's strips (mcs_capi.cpp) and
mcs_sweep.hip's step schedule restated in numpy, checked against the C restatement -- a debugging
aid for the kernel's ring / lag logic.  python tools/sweep_emu.py [c0|c1|...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle  # noqa: E402
from tools.sweep_model import mixed_pixels  # noqa: E402

TW, TH, VALID, MARGIN, LEAD = 32, 64, 100, 16, 16
NG0, NG1, NG2, NB2, NR1 = 24, 10, 4, 4, 4
DBG = int(os.environ.get('MCS_SWEEP_DBG', '0'))


def rf(i, n):
    i = -i if i < 0 else i
    return 2 * n - 2 - i if i >= n else i


def rf_far(i, n):
    while i < 0 or i >= n:
        i = -i if i < 0 else i
        if i >= n:
            i = 2 * n - 2 - i
    return i


def taps(x, n):
    if x % 2 == 0:
        return [rf(x // 2 - 1, n), rf(x // 2, n), rf(x // 2 + 1, n)], [1, 6, 1]
    return [rf((x - 1) // 2, n), rf((x + 1) // 2, n)], [4, 4]


def build_strips(owner, mixed):
    H, W = owner.shape
    gyb = (H + TH - 1) // TH

    def owners_in(x0, x1, y0, y1):
        x0, x1, y0, y1 = max(x0, 0), min(x1, W), max(y0, 0), min(y1, H)
        v = np.unique(owner[y0:y1, x0:x1])
        return set(int(o) for o in v if o != 255)

    segs = []
    for ty in range(gyb):
        row = []
        for tx in range((W + TW - 1) // TW):
            m = mixed[ty * TH:ty * TH + TH, tx * TW:tx * TW + TW]
            if not m.any():
                continue
            lo = [None] * TH
            hi = [None] * TH
            for r in range(m.shape[0]):
                c = np.flatnonzero(m[r])
                if len(c):
                    lo[r], hi[r] = tx * TW + c[0], tx * TW + c[-1]
            mn = min(v for v in lo if v is not None)
            mx = max(v for v in hi if v is not None)
            g = dict(x0=mn & ~3, x1=min((mx + 4) & ~3, W), lo=lo, hi=hi)
            if row and g["x0"] <= row[-1]["x1"] + 32 and max(row[-1]["x1"], g["x1"]) - row[-1]["x0"] <= VALID:
                b = row[-1]
                b["x1"] = max(b["x1"], g["x1"])
                for r in range(TH):
                    if g["lo"][r] is not None:
                        b["lo"][r] = g["lo"][r] if b["lo"][r] is None else min(b["lo"][r], g["lo"][r])
                        b["hi"][r] = g["hi"][r] if b["hi"][r] is None else max(b["hi"][r], g["hi"][r])
            else:
                row.append(g)
        segs.append(row)
    runs, open_ = [], []
    for ty in range(gyb):
        nxt = []
        for gi, g in enumerate(segs[ty]):
            pick = None
            for r in list(open_):
                x0, x1 = min(r["x0"], g["x0"]), max(r["x1"], g["x1"])
                if x1 - x0 > VALID or max(r["x0"], g["x0"]) > min(r["x1"], g["x1"]) + 32:
                    continue
                ow = owners_in(x0 - 16, x1 + 16, r["ty0"] * TH - 16, min(ty * TH + TH, H) + 16)
                if len(ow) > 4:
                    continue
                open_.remove(r)
                r.update(x0=x0, x1=x1, ty1=ty, owners=ow)
                r["seg"].append(gi)
                pick = r
                break
            if pick is None:
                ow = owners_in(g["x0"] - 16, g["x1"] + 16, ty * TH - 16, min(ty * TH + TH, H) + 16)
                assert g["x1"] - g["x0"] <= VALID and len(ow) <= 4
                pick = dict(x0=g["x0"], x1=g["x1"], ty0=ty, ty1=ty, seg=[gi], owners=ow)
                runs.append(pick)
            nxt.append(pick)
        open_ = nxt
    w1 = (W + 1) // 2
    w2 = (w1 + 1) // 2
    strips = []
    for r in runs:
        st = dict(c0=r["x0"] - MARGIN - (((VALID - (r["x1"] - r["x0"])) // 2) & ~3),
                  ya=r["ty0"] * TH, yb=min(r["ty1"] * TH + TH, H), slots=sorted(r["owners"]))
        st["r0"] = st["ya"] - LEAD
        last = (st["yb"] - 1 - st["ya"] + 34) // 4
        st["nsteps"] = (last + 1 + 2) // 3 * 3
        reg = []
        e1 = []
        for y in range(st["ya"], st["yb"]):
            g = segs[y // TH][r["seg"][y // TH - r["ty0"]]]
            lo, hi = g["lo"][y % TH], g["hi"][y % TH]
            xa = xb = 0
            if lo is not None:
                xa, xb = lo & ~3, min((hi + 4) & ~3, W)
            reg.append((xa, xb))
            for x in range(xa, xb):
                e1 += taps(x, w1)[0]
        st["reg"] = reg
        st["e1lo"], st["e1hi"] = min(e1), max(e1)
        z = []
        for E in range(st["e1lo"], st["e1hi"] + 1):
            z += taps(E, w2)[0]
        st["z2lo"], st["z2hi"] = min(z), max(z)
        c1, c2 = st["c0"] // 2, st["c0"] // 4
        assert all(1 <= E - c1 <= 62 for E in range(st["e1lo"], st["e1hi"] + 1)), st
        assert all(2 <= Z - c2 <= 30 for Z in range(st["z2lo"], st["z2hi"] + 1)), st
        strips.append(st)
    return strips


def sweep(strips, owner, g0all, out):
    """g0all[slot]: the slot's replicate-border warp over the mosaic (H, W, CN) uint8"""
    H, W = owner.shape
    CN = out.shape[2]
    w1, h1 = (W + 1) // 2, (H + 1) // 2
    w2, h2 = (w1 + 1) // 2, (h1 + 1) // 2
    for st in strips:
        c0, c1, c2, r0 = st["c0"], st["c0"] // 2, st["c0"] // 4, st["r0"]
        ns = len(st["slots"])
        K0 = r0 // 4
        cols = [rf_far(c0 + l, W) for l in range(128)]
        g0r = np.zeros((NG0, 128, 4), np.int64) - 1
        g1r = np.zeros((ns, NG1, 64, 4), np.int64)
        g2r = np.zeros((ns, NG2, 32, 4), np.int64)
        b2r = np.zeros((NB2, 32, CN))
        r1r = np.zeros((NR1, 64, CN))
        A1 = np.zeros((ns, 3, 128, 4), np.int64)
        A2 = np.zeros((ns, 3, 64, 4), np.int64)
        for s in range(st["nsteps"]):
            k = K0 + s
            sm = s % 3
            # phase A: producer
            s1 = np.zeros((2, ns, 128, 4), np.int64)
            for t in range(4):
                lr = 4 * s + t
                y = rf_far(r0 + lr, H)
                for j, slot in enumerate(st["slots"]):
                    p = np.zeros((128, 4), np.int64)
                    p[:, :CN] = g0all[slot][y, cols, :CN]
                    p[:, 3] = owner[y, cols] == slot
                    a0, a1, a2 = (2 * sm + 2) % 3, (2 * sm) % 3, (2 * sm + 1) % 3
                    if t == 0:
                        s1[0, j] = A1[j, a0] + p
                        A1[j, a1] += 6 * p
                        A1[j, a2] = p
                    elif t == 1:
                        A1[j, a1] += 4 * p
                        A1[j, a2] += 4 * p
                    elif t == 2:
                        s1[1, j] = A1[j, a1] + p
                        A1[j, a2] += 6 * p
                        A1[j, a0] = p
                    else:
                        A1[j, a2] += 4 * p
                        A1[j, a0] += 4 * p
                    own = owner[y, cols] == slot
                    for l in np.flatnonzero(own):
                        g0r[lr % NG0, l, :CN] = p[l, :CN]
                        g0r[lr % NG0, l, 3] = j
                    if j == 0:
                        for l in np.flatnonzero(owner[y, cols] == 255):
                            g0r[lr % NG0, l] = [0, 0, 0, 255]
            # phase A: R0 of rows 4k-18 .. 4k-15
            for rr in range(4):
                yy = 4 * k - 18 + rr
                if not (st["ya"] <= yy < st["yb"]):
                    continue
                xa, xb = st["reg"][yy - st["ya"]]
                for x in range(xa, xb):
                    gv = g0r[(yy - r0) % NG0, x - c0]
                    jo = int(gv[3])
                    if jo == 255:
                        out[yy, x] = 0
                        continue
                    iy, wy = taps(yy, h1)
                    ix, wx = taps(x, w1)
                    for kk in range(CN):
                        e1 = 0
                        acc = 0.0
                        for uu in range(len(iy)):
                            for vv in range(len(ix)):
                                wt = wy[uu] * wx[vv]
                                e1 += wt * int(g1r[jo, iy[uu] % NG1, ix[vv] - c1, kk])
                                acc += float(wt) * r1r[iy[uu] % NR1, ix[vv] - st["e1lo"], kk]
                        l0 = 16384 * int(gv[kk]) - e1
                        r0v = l0 / 16384.0 + acc / 64.0
                        if DBG == 1:
                            r0v = float(gv[kk])
                        elif DBG == 2:
                            r0v = 128.0 + l0 / 64.0
                        elif DBG == 3:
                            r0v = acc / 64.0
                        elif DBG == 4:
                            r0v = e1 / 16384.0
                        vf = np.floor(r0v + 0.5)
                        out[yy, x, kk] = int(min(max(vf, 0), 255))
            # phase B: P2
            for h in range(2):
                i = 2 * k - 1 + h
                for j in range(ns):
                    g = np.zeros((64, 4), np.int64)
                    for e in range(64):
                        b = 2 * e
                        idx = [max(b - 2, 0), max(b - 1, 0), b, b + 1, min(b + 2, 127)]
                        g[e] = sum(w * s1[h, j, q] for w, q in zip([1, 4, 6, 4, 1], idx))
                    if i < h1:
                        g1r[j, i % NG1] = g
                    else:
                        g = g1r[j, rf(i, h1) % NG1].copy()
                    b0, b1, b2i = (sm + 2) % 3, sm % 3, (sm + 1) % 3
                    if h == 0:
                        A2[j, b0] += 4 * g
                        A2[j, b1] += 4 * g
                    else:
                        A2[j, b0] += g
                        if j == 0:
                            s2 = np.zeros((ns, 64, 4), np.int64)
                        s2[j] = A2[j, b0]
                        A2[j, b1] += 6 * g
                        A2[j, b2i] = g
            # phase B: B2 of row k - 2
            z = k - 2
            if 0 <= z < h2:
                for u in range(st["z2hi"] - st["z2lo"] + 1):
                    el = st["z2lo"] + u - c2
                    den = sum(int(g2r[j, z % NG2, el, 3]) for j in range(ns))
                    for kk in range(CN):
                        num = sum(float(g2r[j, z % NG2, el, 3]) * float(g2r[j, z % NG2, el, kk])
                                  for j in range(ns))
                        b2r[z % NB2, u, kk] = num / (den * 65536.0) if den else 0.0
            # phase C: P3
            z = k - 1
            if z < h2:
                for j in range(ns):
                    for e2 in range(32):
                        Z = c2 + e2
                        acc = np.zeros(4, np.int64)
                        for v, wv in enumerate([1, 4, 6, 4, 1]):
                            q = min(max(rf(2 * Z - 2 + v, w1) - c1, 0), 63)
                            acc += wv * s2[j, q]
                        g2r[j, z % NG2, e2] = acc
            # phase C: R1 rows 2k-6, 2k-5
            for rr in range(2):
                q = 2 * k - 6 + rr
                if not (0 <= q < h1):
                    continue
                for E in range(st["e1lo"], st["e1hi"] + 1):
                    iy, wy = taps(q, h2)
                    ix, wx = taps(E, w2)
                    for kk in range(CN):
                        num, den = 0.0, 0
                        for j in range(ns):
                            e2v = sum(wy[a] * wx[b] * int(g2r[j, iy[a] % NG2, ix[b] - c2, kk])
                                      for a in range(len(iy)) for b in range(len(ix)))
                            g1 = g1r[j, q % NG1, E - c1]
                            num += float(g1[3]) * float(16384 * int(g1[kk]) - e2v)
                            den += int(g1[3])
                        acc = 0.0
                        for a in range(len(iy)):
                            for b in range(len(ix)):
                                acc += float(wy[a] * wx[b]) * b2r[iy[a] % NB2, ix[b] - st["z2lo"], kk]
                        b1 = num / (den * 4194304.0) if den else 0.0
                        r1r[q % NR1, E - st["e1lo"], kk] = b1 + acc / 64.0


def main():
    from test_gpu_blend import _world_plan
    from tools.sweep_debug import CASES
    name = sys.argv[1] if len(sys.argv) > 1 else "c0"
    case = dict(CASES[name])
    interp = case.pop("interp", 1)
    plan, cams = _world_plan(interp=interp, **case)
    flat = plan.describe()
    want, owner = oracle.blend_stitch(flat, cams, 2, interp, want_owner=True)
    if want.ndim == 2:
        want = want[:, :, None]
    mixed = mixed_pixels(owner)
    strips = build_strips(owner, mixed)
    print(name, "strips", len(strips), [(s["c0"], s["ya"], s["yb"], s["slots"], s["nsteps"]) for s in strips])
    # replicate-border warps of every slot: oracle seam mode per slot is not exposed; use the
    # feather/seam oracle trick: blend_stitch SEAM gives the owner sample only.  Build g0 per slot
    # by a tiny restatement of sample_replicate through oracle.map_pixel.
    g0all = slot_warps(flat, cams, owner.shape, interp)
    out = want.copy()
    out[:] = 77
    sweep(strips, owner, g0all, out)
    reg = np.zeros(owner.shape, bool)
    for st in strips:
        for y in range(st["ya"], st["yb"]):
            xa, xb = st["reg"][y - st["ya"]]
            reg[y, xa:xb] = True
    np.savez_compressed(f"/tmp/emu_{name}_dbg{DBG}.npz", out=out, reg=reg)
    d = np.abs(out.astype(np.int16) - want.astype(np.int16)).max(2)
    d[~reg] = 0
    ys, xs = np.nonzero(d)
    print("region px", int(reg.sum()), "bad", len(ys), "max", int(d.max()))
    for y, x in list(zip(ys, xs))[:10]:
        print("  ", y, x, out[y, x], want[y, x], owner[y, x])


def slot_warps(flat, cams, shape, interp):
    """per slot: its replicate-border sample at every mosaic pixel (orc__stage_xy +
    orc__sample_replicate, the oracle's own slot arithmetic)"""
    import ctypes
    L = oracle.lib()
    L.orc__stage_xy.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.orc__sample_replicate.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    H, W = shape
    n = int(flat["n_stages"])
    offx = np.asarray(flat["off_x"], np.int64)
    offy = np.asarray(flat["off_y"], np.int64)
    minv = np.ascontiguousarray(flat["minv"], np.float64).reshape(-1)
    bw0 = np.asarray(flat["bw0"], np.int64)
    scam = [0] + [int(c) for c in flat["cam"]]
    cams = [np.ascontiguousarray(c) for c in cams]
    CN = 1 if cams[0].ndim == 2 else cams[0].shape[2]
    x32 = ctypes.c_int()
    y32 = ctypes.c_int()
    d = (ctypes.c_uint8 * 4)()
    res = {}
    for s in range(n + 1):
        c = cams[scam[s]]
        h, w = c.shape[:2]
        g = np.zeros((H, W, CN), np.uint8)
        M = minv[9 * (s - 1):9 * s].copy() if s else None
        for y in range(H):
            for x in range(W):
                if s == 0:
                    x32.value, y32.value = (x + offx[n]) * 32, (y + offy[n]) * 32
                else:
                    L.orc__stage_xy(M.ctypes.data, int(bw0[s - 1]), interp, int(x + offx[s - 1]),
                                    int(y + offy[s - 1]), ctypes.byref(x32), ctypes.byref(y32))
                L.orc__sample_replicate(c.ctypes.data, w, h, CN, x32.value, y32.value, d)
                g[y, x] = d[:CN]
        res[s] = g
    return res


if __name__ == "__main__":
    main()

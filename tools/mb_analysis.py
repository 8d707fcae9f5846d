import sys, numpy as np
sys.path.insert(0, "/root/repo")
from multicamera_stitching_amd import rig, _capi
from multicamera_stitching_amd.StitcherClass import _stage_desc
from oracle import oracle

st, images, _ = rig.calibrated_stitcher(4, 1920, 1080, 3, seed=0)
cams = [images[l] for l in st.img_labels]
plan = _capi.Plan([_stage_desc(sb) for sb in st.stitchers], 1920, 1080, 3, 1)
flat = plan.describe()
out, owner = oracle.blend_stitch(flat, cams, oracle.BLEND_MULTIBAND, want_owner=True)
H, W = owner.shape
print("mosaic", W, H)
S = int(owner[owner != 255].max()) + 1
w1, h1 = (W + 1) // 2, (H + 1) // 2
w2, h2 = (w1 + 1) // 2, (h1 + 1) // 2

def refl(i, n):
    i = np.abs(i)
    return np.where(i >= n, 2 * n - 2 - i, i)

k5 = np.array([1, 4, 6, 4, 1])
def reduce(a):
    h, w = a.shape
    mh, mw = (h + 1) // 2, (w + 1) // 2
    ys = refl(np.arange(mh)[:, None] * 2 + np.arange(-2, 3)[None], h)
    xs = refl(np.arange(mw)[:, None] * 2 + np.arange(-2, 3)[None], w)
    t = (a[ys] * k5[None, :, None]).sum(1)          # mh x w
    return (t[:, xs] * k5[None, None, :]).sum(2)
m1 = [reduce((owner == s).astype(np.int64)) for s in range(S)]
m2 = [reduce(m) for m in m1]
# mixed pixels: any other owner's m2 > 0 at a level-2 tap of a level-1 tap
def taps(n_fine, n):
    x = np.arange(n_fine)
    even = (x & 1) == 0
    t = np.stack([np.where(even, x // 2 - 1, (x - 1) // 2), np.where(even, x // 2, (x + 1) // 2),
                  np.where(even, x // 2 + 1, (x + 1) // 2)], 1)
    return refl(t, n)
ty1, tx1 = taps(H, h1), taps(W, w1)
ty2, tx2 = taps(h1, h2), taps(w1, w2)
# level-1 entries: set of level-2 taps -> "any m2_s > 0" per slot
reach2 = [np.zeros((h1, w1), bool) for s in range(S)]
for s in range(S):
    pos = m2[s] > 0
    r = np.zeros((h1, w1), bool)
    for a in range(3):
        for b in range(3):
            r |= pos[ty2[:, a]][:, tx2[:, b]]
    reach2[s] = r
reach0 = [np.zeros((H, W), bool) for s in range(S)]
for s in range(S):
    r = np.zeros((H, W), bool)
    for a in range(3):
        for b in range(3):
            r |= reach2[s][ty1[:, a]][:, tx1[:, b]]
    reach0[s] = r
mixed = np.zeros((H, W), bool)
for s in range(S):
    mixed |= reach0[s] & (owner != s) & (owner != 255)
print("mixed pixels", mixed.sum(), "of", H * W)
# needed R1 entries: level-1 taps of mixed pixels
needR1 = np.zeros((h1, w1), bool)
ys, xs = np.nonzero(mixed)
for a in range(3):
    for b in range(3):
        needR1[ty1[ys, a], tx1[xs, b]] = True
print("R1 entries", needR1.sum())
# per slot: g1_s needed at R1 entries where m1_s>0 (L1) or where s owns a mixed pixel tapping it;
# g2_s needed at level-2 taps of those (E(g2)) and at B2 entries (level-2 taps of R1 entries) with m2_s>0
tot0 = 0
for s in range(S):
    need1 = needR1 & (m1[s] > 0)
    ym, xm = np.nonzero(mixed & (owner == s))
    for a in range(3):
        for b in range(3):
            need1[ty1[ym, a], tx1[xm, b]] = True
    need2 = np.zeros((h2, w2), bool)
    yy, xx = np.nonzero(need1)
    for a in range(3):
        for b in range(3):
            need2[ty2[yy, a], tx2[xx, b]] = True
    yr, xr = np.nonzero(needR1)
    for a in range(3):
        for b in range(3):
            sel = m2[s][ty2[yr, a], tx2[xr, b]] > 0
            need2[ty2[yr[sel], a], tx2[xr[sel], b]] = True
    # g1 inputs of g2 entries: 5x5 level-1 around 2z
    g1in = need1.copy()
    zy, zx = np.nonzero(need2)
    for u in range(-2, 3):
        for v in range(-2, 3):
            g1in[refl(2 * zy + u, h1), refl(2 * zx + v, w1)] = True
    g0in = np.zeros((H, W), bool)
    qy, qx = np.nonzero(g1in)
    for u in range(-2, 3):
        for v in range(-2, 3):
            g0in[refl(2 * qy + u, H), refl(2 * qx + v, W)] = True
    # column/row extents per row-band of 64
    print(f"slot {s}: need g1 {need1.sum()} g2 {need2.sum()} g1in {g1in.sum()} g0in {g0in.sum()}")
    tot0 += g0in.sum()
print("minimal level-0 samples per capture (all slots):", tot0)
# current design: per listed tile, per owner in the 64x? neighbourhood, 89 x w0

/*
 * orc_blend.c -- TEST INFRASTRUCTURE ONLY (the parity checker), never the product path.
 *
 * CPU restatement of the blended stitch modes.  The reference
 * has no blending -- StitcherBase.stitch pastes B over the warped A (StitcherClass.py:239-241) --
 * so there is nothing to pin these against: the specification is ours, and this file is it.
 * The GPU path (multicamera_stitching_amd/csrc) must reproduce it bit for bit; every quantity
 * is an integer or an IEEE double computed in the order written here.
 *
 * Geometry: the plan's flattened chain (mcs_plan_describe).  Camera "slots": slot 0 = camera 0
 * (integer offset into the mosaic), slot j+1 = the camera warped by calibrated stage j.  For
 * output pixel p and slot s, the OpenCV stage map gives a position (x32, y32) in 1/32 px
 * (orc__stage_xy: the exact cascade arithmetic).
 *   covered_s(p) : 0 <= x32 <= 32 (w-1) and 0 <= y32 <= 32 (h-1)
 *   d_s(p)       : min(x32, y32, 32 (w-1) - x32, 32 (h-1) - y32)   (distance to the image edge)
 *   I_s(p)       : bilinear sample at (x32, y32) with the taps clamped into the image
 *                  (BORDER_REPLICATE, remapBilinear fixed point); equals the reference-style warp
 *                  wherever covered
 *   owner(p)     : the covering slot with the largest d, ties to the lower camera index; none
 *                  when no slot covers p (output 0, as the reference's border)
 * FEATHER (NS-2): out = (sum_s d_s I_s + D / 2) / D over covering slots, D = sum_s d_s
 *   (integer); D == 0 -> I_owner.
 * MULTIBAND (NS-1), 3 levels, Burt-Adelson with the owner map as the seam masks:
 *   reduce   g_{l+1}(y, x) = sum_ij w_i w_j g_l(refl(2y+i), refl(2x+j)), w = [1 4 6 4 1],
 *            in integers: g0 = I (u8), g1 = 256 G1, g2 = 65536 G2; masks m0 = [owner == s],
 *            m1 = reduce(m0), m2 = reduce(m1);
 *   expand   taps of output x at the coarser level: even x -> (x/2-1, x/2, x/2+1) x (1, 6, 1),
 *            odd x -> ((x-1)/2, (x+1)/2) x (4, 4); separable, /64 overall;
 *   Laplace  L0 = 16384 g0 - E(g1) (= 16384 (G0 - up G1)), L1 = 16384 g1 - E(g2), L2 = g2;
 *   blend    B0 = L0_owner / 16384, B1 = sum m1 L1 / (sum m1 * 4194304),
 *            B2 = sum m2 g2 / (sum m2 * 65536)   (double; 0 where the mask sum is 0);
 *   collapse R1 = B1 + up(B2), R0 = B0 + up(R1), up in double: acc += (uy * ux) * R over the
 *            taps in the order listed (rows outer), then acc / 64;
 *   out = clamp(floor(R0 + 0.5), 0, 255) where an owner exists, else 0.
 *   Dense seams: the mosaic is cut into 32 x 64 blend tiles (columns x rows); a tile whose
 *   neighbourhood (the tile grown by 16 px on every side, clipped to the mosaic) holds more than
 *   8 distinct owners takes the FEATHER rule below for its own pixels instead (the GPU's blend
 *   kernels hold at most 8 owners; the pyramids of every other tile are unaffected, they depend
 *   on the samples and the owner map only).
 * SEAM: out = I_owner (the seam without blending), 0 where no slot covers p.
 * Graph-cut seams (seam_k >= 0, orc_seam.c): the owner is the seam label's camera when it
 *   covers p (d >= 0), else the distance owner above.  seam_k >= 256: the labels of the
 *   2^(seam_k - 256) grid are the caller's (found once per plan, from one capture).
 * Cylindrical rigs (orc_blend_stitch_cyl, NS-6): slot s = camera s, positions from
 *   orc__cyl_xy over the panorama's per-column (sin t, cos t) and per-row h, t = (u - u0) / fc,
 *   h = (v - v0) / fc (libm sin/cos, once per column); the rest as above.
 *   refl = reflect-101 at each level's own size (BORDER_DEFAULT); sizes n_{l+1} = (n_l + 1) / 2.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_BLEND_FEATHER 1
#define ORC_BLEND_MULTIBAND 2
#define ORC_BLEND_SEAM 3

void orc__stage_xy(const double *M, int bw0, int interp, int X, int Y, int *x32, int *y32);
void orc__sample_replicate(const uint8_t *src, int sw, int sh, int cn, int x32, int y32,
                           uint8_t *d);
void orc__cyl_xy(const double *R, double f, double cx, double cy, double sn, double cs, double hv,
                 int interp, int *x32, int *y32);

static inline int refl(int i, int n)
{
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

/* Slot geometry: the homography chain of a plan, or a cylindrical rig. */
typedef struct {
    int kind;                      /* 0: homography chain, 1: cylinder */
    int n_stages;
    const int *off_x, *off_y, *bw0;
    const double *minv;
    const double *R, *f, *cx, *cy; /* cylinder: per camera */
    const double *tab;             /* cylinder: (sin, cos) per column, then h per row */
    int ow;
} geo_t;

static void slot_xy(const geo_t *g, int s, int interp, int x, int y, int *x32, int *y32)
{
    if (g->kind == 1) {
        orc__cyl_xy(g->R + 9 * s, g->f[s], g->cx[s], g->cy[s], g->tab[2 * x], g->tab[2 * x + 1],
                    g->tab[2 * g->ow + y], interp, x32, y32);
    } else if (s == 0) {
        *x32 = (x + g->off_x[g->n_stages]) * 32;
        *y32 = (y + g->off_y[g->n_stages]) * 32;
    } else {
        int j = s - 1;
        orc__stage_xy(g->minv + 9 * j, g->bw0[j], interp, x + g->off_x[j], y + g->off_y[j], x32,
                      y32);
    }
}

/* reduce: src (n_h x n_w x cn, int32) -> dst (m_h x m_w x cn) */
static void reduce_i32(const int32_t *src, int nw, int nh, int cn, int32_t *dst, int mw, int mh)
{
    static const int w[5] = {1, 4, 6, 4, 1};
#pragma omp parallel for schedule(static)
    for (int y = 0; y < mh; y++)
        for (int x = 0; x < mw; x++)
            for (int k = 0; k < cn; k++) {
                int64_t acc = 0;
                for (int i = 0; i < 5; i++) {
                    const int32_t *row = src + (long)refl(2 * y + i - 2, nh) * nw * cn;
                    for (int j = 0; j < 5; j++)
                        acc += (int64_t)(w[i] * w[j]) * row[(long)refl(2 * x + j - 2, nw) * cn + k];
                }
                dst[((long)y * mw + x) * cn + k] = (int32_t)acc;
            }
}

/* expand taps of fine index x into a coarse level of size n */
static inline int exp_taps(int x, int n, int *idx, int *wt)
{
    if ((x & 1) == 0) {
        idx[0] = refl(x / 2 - 1, n), wt[0] = 1;
        idx[1] = refl(x / 2, n), wt[1] = 6;
        idx[2] = refl(x / 2 + 1, n), wt[2] = 1;
        return 3;
    }
    idx[0] = refl((x - 1) / 2, n), wt[0] = 4;
    idx[1] = refl((x + 1) / 2, n), wt[1] = 4;
    return 2;
}

/* integer expand of a coarse int32 image evaluated at fine (y, x), channel k: sum u u g */
static inline int64_t expand_i(const int32_t *g, int gw, int gh, int cn, int y, int x, int k)
{
    int iy[3], wy[3], ix[3], wx[3];
    int ny = exp_taps(y, gh, iy, wy), nx = exp_taps(x, gw, ix, wx);
    int64_t acc = 0;
    for (int a = 0; a < ny; a++)
        for (int b = 0; b < nx; b++)
            acc += (int64_t)(wy[a] * wx[b]) * g[((long)iy[a] * gw + ix[b]) * cn + k];
    return acc;
}

static inline double expand_d(const double *r, int gw, int gh, int cn, int y, int x, int k)
{
    int iy[3], wy[3], ix[3], wx[3];
    int ny = exp_taps(y, gh, iy, wy), nx = exp_taps(x, gw, ix, wx);
    double acc = 0.0;
    for (int a = 0; a < ny; a++)
        for (int b = 0; b < nx; b++)
            acc += (double)(wy[a] * wx[b]) * r[((long)iy[a] * gw + ix[b]) * cn + k];
    return acc / 64.0;
}

int orc_seam_graphcut(int n_cams, int gw, int gh, uint8_t *lab, const uint16_t *cov,
                      const uint8_t *smp, int cn);

/* Graph-cut seam labels (orc_seam.c) on the 2^k seam grid: inputs from the slot geometry. */
static int seam_labels(const geo_t *geo, int S, const int *scam, const uint8_t *const *cams,
                       const int *cw, const int *ch, int cn, int interp, int ow, int oh, int k,
                       uint8_t *lab)
{
    const int gw = (ow + (1 << k) - 1) >> k, gh = (oh + (1 << k) - 1) >> k;
    const long np = (long)gw * gh;
    int n_cams = 0;
    for (int s = 0; s < S; s++)
        if (scam[s] + 1 > n_cams) n_cams = scam[s] + 1;
    uint16_t *cov = (uint16_t *)calloc((size_t)np, sizeof(uint16_t));
    uint8_t *smp = (uint8_t *)calloc((size_t)np * cn * n_cams, 1);
    if (!cov || !smp) { free(cov); free(smp); return -1; }
#pragma omp parallel for schedule(static)
    for (long q = 0; q < np; q++) {
        const int x = (int)(q % gw) << k, y = (int)(q / gw) << k;
        int best = -1, bestd = -1;
        for (int s = 0; s < S; s++) {
            const int c = scam[s], w = cw[c], h = ch[c];
            int x32, y32;
            slot_xy(geo, s, interp, x, y, &x32, &y32);
            if (!(x32 >= 0 && y32 >= 0 && x32 <= 32 * (w - 1) && y32 <= 32 * (h - 1))) continue;
            int d = x32;
            if (y32 < d) d = y32;
            if (32 * (w - 1) - x32 < d) d = 32 * (w - 1) - x32;
            if (32 * (h - 1) - y32 < d) d = 32 * (h - 1) - y32;
            if (d > bestd || (d == bestd && c < scam[best])) best = s, bestd = d;
            cov[q] |= (uint16_t)(1u << c);
            orc__sample_replicate(cams[c], w, h, cn, x32, y32, smp + ((long)c * np + q) * cn);
        }
        lab[q] = (uint8_t)(best < 0 ? 255 : scam[best]);
    }
    const int rc = orc_seam_graphcut(n_cams, gw, gh, lab, cov, smp, cn);
    free(cov);
    free(smp);
    return rc;
}

/* FEATHER at pixel p: (sum_s d_s I_s + D / 2) / D over the slots at positive distance. */
static void feather_px(int S, long npx, int cn, const uint8_t *owner, const int32_t *dist,
                       const uint8_t *g0, long p, uint8_t *d)
{
    if (owner[p] == 255) {
        memset(d, 0, (size_t)cn);
        return;
    }
    int64_t den = 0;
    for (int s = 0; s < S; s++)
        if (dist[(long)s * npx + p] > 0) den += dist[(long)s * npx + p];
    for (int k = 0; k < cn; k++) {
        if (den == 0) {
            d[k] = g0[((long)owner[p] * npx + p) * cn + k];
            continue;
        }
        int64_t num = 0;
        for (int s = 0; s < S; s++) {
            const int32_t ds = dist[(long)s * npx + p];
            if (ds > 0) num += (int64_t)ds * g0[((long)s * npx + p) * cn + k];
        }
        d[k] = (uint8_t)((num + den / 2) / den);
    }
}

/* Multi-band blend tiles (32 x 64) whose 16-px neighbourhood holds more than 8 owners: 1. */
#define ORC_MB_TILE_W 32
#define ORC_MB_TILE_H 64
#define ORC_MB_HALO 16
#define ORC_MB_MAX_OWNERS 8
static uint8_t *dense_tiles(const uint8_t *owner, int ow, int oh, int *gx_out)
{
    const int gx = (ow + ORC_MB_TILE_W - 1) / ORC_MB_TILE_W;
    const int gy = (oh + ORC_MB_TILE_H - 1) / ORC_MB_TILE_H;
    uint8_t *dense = (uint8_t *)calloc((size_t)gx * gy, 1);
    if (!dense) return NULL;
#pragma omp parallel for schedule(static)
    for (int t = 0; t < gx * gy; t++) {
        const int tx = t % gx, ty = t / gx;
        int x0 = tx * ORC_MB_TILE_W - ORC_MB_HALO, x1 = tx * ORC_MB_TILE_W + ORC_MB_TILE_W + ORC_MB_HALO;
        int y0 = ty * ORC_MB_TILE_H - ORC_MB_HALO, y1 = ty * ORC_MB_TILE_H + ORC_MB_TILE_H + ORC_MB_HALO;
        if (x0 < 0) x0 = 0;
        if (y0 < 0) y0 = 0;
        if (x1 > ow) x1 = ow;
        if (y1 > oh) y1 = oh;
        uint32_t m = 0;
        for (int y = y0; y < y1; y++)
            for (int x = x0; x < x1; x++) {
                const int o = owner[(long)y * ow + x];
                if (o != 255) m |= 1u << o;
            }
        dense[t] = __builtin_popcount(m) > ORC_MB_MAX_OWNERS;
    }
    *gx_out = gx;
    return dense;
}

static int blend_core(const geo_t *geo, int S, const int *scam, const uint8_t *const *cams,
                      const int *cw, const int *ch, int cn, int interp, int mode, uint8_t *out,
                      int ow, int oh, uint8_t *owner_out, int seam_k, uint8_t *seam_lab)
{
    const long npx = (long)ow * oh;
    /* seam_k >= 256: the labels of the 2^(seam_k - 256) grid are given in seam_lab (a plan's
     * seams are found once, from one capture, and then serve every capture) */
    const int given = seam_k >= 256;
    if (given) seam_k -= 256;
    const int gw = seam_k >= 0 ? (ow + (1 << seam_k) - 1) >> seam_k : 0;
    if (seam_k >= 0 && !given &&
        seam_labels(geo, S, scam, cams, cw, ch, cn, interp, ow, oh, seam_k, seam_lab) != 0)
        return -1;
    uint8_t *owner = (uint8_t *)malloc((size_t)npx);
    uint8_t *g0 = (uint8_t *)malloc((size_t)npx * cn * S);
    int32_t *dist = (int32_t *)malloc(sizeof(int32_t) * (size_t)npx * S);
    if (!owner || !g0 || !dist) { free(owner); free(g0); free(dist); return -1; }

#pragma omp parallel for schedule(static)
    for (long p = 0; p < npx; p++) {
        const int y = (int)(p / ow), x = (int)(p % ow);
        int best = -1, bestd = -1;
        for (int s = 0; s < S; s++) {
            const int c = scam[s], w = cw[c], h = ch[c];
            int x32, y32;
            slot_xy(geo, s, interp, x, y, &x32, &y32);
            orc__sample_replicate(cams[c], w, h, cn, x32, y32, g0 + ((long)s * npx + p) * cn);
            int d = -1;
            if (x32 >= 0 && y32 >= 0 && x32 <= 32 * (w - 1) && y32 <= 32 * (h - 1)) {
                d = x32;
                if (y32 < d) d = y32;
                if (32 * (w - 1) - x32 < d) d = 32 * (w - 1) - x32;
                if (32 * (h - 1) - y32 < d) d = 32 * (h - 1) - y32;
                if (d > bestd || (d == bestd && c < scam[best])) best = s, bestd = d;
            }
            dist[(long)s * npx + p] = d;
        }
        if (seam_k >= 0) {   /* the seam label's camera, when it covers the pixel */
            const int hc = seam_lab[(long)(y >> seam_k) * gw + (x >> seam_k)];
            for (int s = 0; s < S && hc != 255; s++)
                if (scam[s] == hc && dist[(long)s * npx + p] >= 0) best = s;
        }
        owner[p] = (uint8_t)(best < 0 ? 255 : best);
    }
    if (owner_out) memcpy(owner_out, owner, (size_t)npx);

    int rc = 0;
    if (mode == ORC_BLEND_SEAM) {
        for (long p = 0; p < npx; p++) {
            if (owner[p] == 255) memset(out + p * cn, 0, (size_t)cn);
            else memcpy(out + p * cn, g0 + ((long)owner[p] * npx + p) * cn, (size_t)cn);
        }
    } else if (mode == ORC_BLEND_FEATHER) {
#pragma omp parallel for schedule(static)
        for (long p = 0; p < npx; p++) feather_px(S, npx, cn, owner, dist, g0, p, out + p * cn);
    } else if (mode == ORC_BLEND_MULTIBAND) {
        const int w1 = (ow + 1) / 2, h1 = (oh + 1) / 2, w2 = (w1 + 1) / 2, h2 = (h1 + 1) / 2;
        const long n1 = (long)w1 * h1, n2 = (long)w2 * h2;
        int32_t *t0 = (int32_t *)malloc(sizeof(int32_t) * (size_t)npx * cn);
        int32_t *g1 = (int32_t *)malloc(sizeof(int32_t) * (size_t)n1 * cn * S);
        int32_t *g2 = (int32_t *)malloc(sizeof(int32_t) * (size_t)n2 * cn * S);
        int32_t *m0 = (int32_t *)malloc(sizeof(int32_t) * (size_t)npx);
        int32_t *m1 = (int32_t *)malloc(sizeof(int32_t) * (size_t)n1 * S);
        int32_t *m2 = (int32_t *)malloc(sizeof(int32_t) * (size_t)n2 * S);
        double *b2 = (double *)malloc(sizeof(double) * (size_t)n2 * cn);
        double *r1 = (double *)malloc(sizeof(double) * (size_t)n1 * cn);
        if (!t0 || !g1 || !g2 || !m0 || !m1 || !m2 || !b2 || !r1) {
            rc = -1;
            goto done;
        }
        for (int s = 0; s < S; s++) {
            for (long i = 0; i < npx * cn; i++) t0[i] = g0[(long)s * npx * cn + i];
            reduce_i32(t0, ow, oh, cn, g1 + (long)s * n1 * cn, w1, h1);
            reduce_i32(g1 + (long)s * n1 * cn, w1, h1, cn, g2 + (long)s * n2 * cn, w2, h2);
            for (long i = 0; i < npx; i++) m0[i] = owner[i] == s;
            reduce_i32(m0, ow, oh, 1, m1 + (long)s * n1, w1, h1);
            reduce_i32(m1 + (long)s * n1, w1, h1, 1, m2 + (long)s * n2, w2, h2);
        }
#pragma omp parallel for schedule(static)
        for (long q = 0; q < n2; q++)
            for (int k = 0; k < cn; k++) {
                int64_t num = 0, den = 0;
                for (int s = 0; s < S; s++) {
                    num += (int64_t)m2[(long)s * n2 + q] * g2[((long)s * n2 + q) * cn + k];
                    den += m2[(long)s * n2 + q];
                }
                b2[q * cn + k] = den ? (double)num / ((double)den * 65536.0) : 0.0;
            }
#pragma omp parallel for schedule(static)
        for (long q = 0; q < n1; q++) {
            const int y = (int)(q / w1), x = (int)(q % w1);
            for (int k = 0; k < cn; k++) {
                int64_t num = 0, den = 0;
                for (int s = 0; s < S; s++) {
                    const int64_t l1 = 16384 * (int64_t)g1[((long)s * n1 + q) * cn + k] -
                                       expand_i(g2 + (long)s * n2 * cn, w2, h2, cn, y, x, k);
                    num += (int64_t)m1[(long)s * n1 + q] * l1;
                    den += m1[(long)s * n1 + q];
                }
                const double b1 = den ? (double)num / ((double)den * 4194304.0) : 0.0;
                r1[q * cn + k] = b1 + expand_d(b2, w2, h2, cn, y, x, k);
            }
        }
        int gxd = 0;
        uint8_t *dense = dense_tiles(owner, ow, oh, &gxd);
        if (!dense) {
            rc = -1;
            goto done;
        }
#pragma omp parallel for schedule(static)
        for (long p = 0; p < npx; p++) {
            const int y = (int)(p / ow), x = (int)(p % ow);
            uint8_t *d = out + p * cn;
            const int s = owner[p];
            if (dense[(long)(y / ORC_MB_TILE_H) * gxd + x / ORC_MB_TILE_W]) {
                feather_px(S, npx, cn, owner, dist, g0, p, d);
                continue;
            }
            for (int k = 0; k < cn; k++) {
                if (s == 255) {
                    d[k] = 0;
                    continue;
                }
                const int64_t l0 = 16384 * (int64_t)g0[((long)s * npx + p) * cn + k] -
                                   expand_i(g1 + (long)s * n1 * cn, w1, h1, cn, y, x, k);
                const double r0 = (double)l0 / 16384.0 + expand_d(r1, w1, h1, cn, y, x, k);
                const double v = floor(r0 + 0.5);
                d[k] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
            }
        }
        free(dense);
    done:
        free(t0); free(g1); free(g2); free(m0); free(m1); free(m2); free(b2); free(r1);
    } else {
        rc = -1;
    }
    free(owner); free(g0); free(dist);
    return rc;
}

int orc_blend_stitch(int n_stages, const int *off_x, const int *off_y, const double *minv,
                     const int *bw0, const int *stage_cam, const uint8_t *const *cams,
                     const int *cw, const int *ch, int cn, int interp, int mode, uint8_t *out,
                     int ow, int oh, uint8_t *owner_out, int seam_k, uint8_t *seam_lab)
{
    if (n_stages < 0 || n_stages > 15 || ow <= 0 || oh <= 0) return -1;
    int scam[16];
    scam[0] = 0;
    for (int j = 0; j < n_stages; j++) scam[j + 1] = stage_cam[j];
    geo_t g;
    memset(&g, 0, sizeof(g));
    g.n_stages = n_stages;
    g.off_x = off_x;
    g.off_y = off_y;
    g.bw0 = bw0;
    g.minv = minv;
    return blend_core(&g, n_stages + 1, scam, cams, cw, ch, cn, interp, mode, out, ow, oh,
                      owner_out, seam_k, seam_lab);
}

/* Cylindrical rig (include/mcs.h mcs_plan_create_cylindrical): slot s = camera s; panorama
 * pixel (u, v) is the ray (sin t, h, cos t), t = (u - u0) / fc, h = (v - v0) / fc. */
int orc_blend_stitch_cyl(int n_cams, const double *R, const double *f, const double *cx,
                         const double *cy, double fc, double u0, double v0,
                         const uint8_t *const *cams, const int *cw, const int *ch, int cn,
                         int interp, int mode, uint8_t *out, int ow, int oh, uint8_t *owner_out,
                         int seam_k, uint8_t *seam_lab)
{
    if (n_cams < 1 || n_cams > 15 || ow <= 0 || oh <= 0) return -1;
    double *tab = (double *)malloc(sizeof(double) * (2 * (size_t)ow + (size_t)oh));
    if (!tab) return -1;
    for (int u = 0; u < ow; u++) {
        const double t = ((double)u - u0) / fc;
        tab[2 * u] = sin(t);
        tab[2 * u + 1] = cos(t);
    }
    for (int v = 0; v < oh; v++) tab[2 * ow + v] = ((double)v - v0) / fc;
    int scam[16];
    for (int c = 0; c < n_cams; c++) scam[c] = c;
    geo_t g;
    memset(&g, 0, sizeof(g));
    g.kind = 1;
    g.R = R;
    g.f = f;
    g.cx = cx;
    g.cy = cy;
    g.tab = tab;
    g.ow = ow;
    const int rc = blend_core(&g, n_cams, scam, cams, cw, ch, cn, interp, mode, out, ow, oh,
                              owner_out, seam_k, seam_lab);
    free(tab);
    return rc;
}

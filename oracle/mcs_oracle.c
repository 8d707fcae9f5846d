/*
 * mcs_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker), never the product path.
 *
 * CPU restatement of the pixel arithmetic on the reference's per-frame stitch path:
 *
 *   PostScripts/Stitcher/StitcherClass.py:211-256  StitcherBase.stitch
 *     :239      cv2.warpPerspective(src=imageA, M=cachedAH, dsize=ABSize)
 *     :240-241  dst[By:By+hB, Bx:Bx+wB] = imageB         (overwrite paste)
 *     :248-251  dst = dst[y0:y1, x0:x1]                   (super-mode crop)
 *   PostScripts/Stitcher/StitcherClass.py:114-136  Stitcher.stitch (stage chain)
 *
 * The warp arithmetic lives in OpenCV (third-party, NOT vendored in the reference and
 * not installed here; the reference's code requires OpenCV 2.4 or 3.x,
 * StitcherClass.py:30-47,376-396).  It is restated from OpenCV 3.4 sources:
 *   - cv::warpPerspective / WarpPerspectiveInvoker   (modules/imgproc/src/imgwarp.cpp)
 *       64-column x 16-row blocks; per row X0 = M0*xb + M1*y + M2 (xb = block start column);
 *       per pixel W = W0 + M6*x1, W = W ? 32/W : 0 (1/W for nearest),
 *       fX = clamp((X0 + M0*x1)*W, INT_MIN, INT_MAX), X = cvRound(fX) (round half even).
 *   - cv::remap -> remapBilinear<FixedPtCast<int,uchar,15>> / remapNearest, BORDER_CONSTANT 0.
 *   - initInterTab2D(INTER_LINEAR): 15-bit weights; entry (0,0) saturates to 32767 and the
 *       sum fix-up lands on w11 (=1).  Restated faithfully in bilinear_tab().
 *   - cv::invert(DECOMP_LU) for 3x3 CV_64F: closed-form cofactor inverse (lapack.cpp, n<=3).
 *
 * Parity status: orchestration/geometry pinned by fixtures produced by executing the
 * reference's own StitcherClass.py (tests/golden/gen_golden.py); the OpenCV arithmetic itself
 * is pinned only by known-answer tests derived from the OpenCV semantics above
 * ("parity unpinned" against a real cv2 -- none exists in this image or on the GPU box).
 *
 * Build: oracle/Makefile (gcc -O3 -fopenmp -ffp-contract=off).  No FMA contraction: OpenCV's
 * x86 SSE2/SSE4.1 baseline code has none.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <limits.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_INTER_NEAREST 0
#define ORC_INTER_LINEAR  1
#define INTER_BITS 5
#define INTER_TAB_SIZE (1 << INTER_BITS)
#define COEF_BITS 15
#define COEF_SCALE (1 << COEF_BITS)

/* ------------------------------------------------------------------------------------------ */
/* cv::invert, n == 3, CV_64F, DECOMP_LU: the closed form (lapack.cpp, "n <= 3" branch).      */
int orc_invert3x3(const double *m, double *out)
{
#define Md(i, j) m[(i) * 3 + (j)]
    double d = Md(0, 0) * (Md(1, 1) * Md(2, 2) - Md(1, 2) * Md(2, 1)) -
               Md(0, 1) * (Md(1, 0) * Md(2, 2) - Md(1, 2) * Md(2, 0)) +
               Md(0, 2) * (Md(1, 0) * Md(2, 1) - Md(1, 1) * Md(2, 0));
    double t[9];
    if (d == 0.) {
        for (int i = 0; i < 9; i++) out[i] = 0.;
        return 0;
    }
    d = 1. / d;
    t[0] = (Md(1, 1) * Md(2, 2) - Md(1, 2) * Md(2, 1)) * d;
    t[1] = (Md(0, 2) * Md(2, 1) - Md(0, 1) * Md(2, 2)) * d;
    t[2] = (Md(0, 1) * Md(1, 2) - Md(0, 2) * Md(1, 1)) * d;
    t[3] = (Md(1, 2) * Md(2, 0) - Md(1, 0) * Md(2, 2)) * d;
    t[4] = (Md(0, 0) * Md(2, 2) - Md(0, 2) * Md(2, 0)) * d;
    t[5] = (Md(0, 2) * Md(1, 0) - Md(0, 0) * Md(1, 2)) * d;
    t[6] = (Md(1, 0) * Md(2, 1) - Md(1, 1) * Md(2, 0)) * d;
    t[7] = (Md(0, 1) * Md(2, 0) - Md(0, 0) * Md(2, 1)) * d;
    t[8] = (Md(0, 0) * Md(1, 1) - Md(0, 1) * Md(1, 0)) * d;
#undef Md
    memcpy(out, t, sizeof(t));
    return 1;
}

/* ------------------------------------------------------------------------------------------ */
/* initInterTab2D(INTER_LINEAR, fixpt=true) restated, including the (0,0) saturation quirk.   */
static short g_bilin[INTER_TAB_SIZE * INTER_TAB_SIZE][4];
static int g_bilin_ready = 0;

/* Built once at load (a constructor): the fix-up below reads the next, not yet written entry,
 * so concurrent lazy builds from OpenMP threads would race on the shared scratch table. */
static void bilinear_tab_build(void) __attribute__((constructor));
static void bilinear_tab(void)
{
    if (!g_bilin_ready) bilinear_tab_build();
}

static void bilinear_tab_build(void)
{
    if (g_bilin_ready) return;
    /* flat table like OpenCV's BilinearTab_i: entry e occupies [4e, 4e+4) */
    static short flat[INTER_TAB_SIZE * INTER_TAB_SIZE * 4 + 8];
    memset(flat, 0, sizeof(flat));
    float tab1[INTER_TAB_SIZE][2];
    for (int i = 0; i < INTER_TAB_SIZE; i++) {
        float x = i * 1.f / INTER_TAB_SIZE;
        tab1[i][0] = 1.f - x;
        tab1[i][1] = x;
    }
    for (int i = 0; i < INTER_TAB_SIZE; i++)
        for (int j = 0; j < INTER_TAB_SIZE; j++) {
            short *itab = flat + (i * INTER_TAB_SIZE + j) * 4;
            int isum = 0;
            for (int k1 = 0; k1 < 2; k1++) {
                float vy = tab1[i][k1];
                for (int k2 = 0; k2 < 2; k2++) {
                    float v = vy * tab1[j][k2];
                    float s = v * COEF_SCALE;
                    int r = (int)lrintf(s);
                    if (r > SHRT_MAX) r = SHRT_MAX;
                    if (r < SHRT_MIN) r = SHRT_MIN;
                    itab[k1 * 2 + k2] = (short)r;
                    isum += r;
                }
            }
            if (isum != COEF_SCALE) {
                /* ksize2 = ksize/2 = 1: the fix-up scans k1,k2 in {1,2}; for ksize 2 this reads
                 * w11 and the (not yet written, zero) next entry, so it always lands on w11. */
                int diff = isum - COEF_SCALE;
                int Mk = 3, mk = 3;
                int cand[4] = {3, 4, 5, 6};
                for (int c = 0; c < 4; c++) {
                    int k = cand[c];
                    if (itab[k] < itab[mk]) mk = k;
                    else if (itab[k] > itab[Mk]) Mk = k;
                }
                if (diff < 0) itab[Mk] = (short)(itab[Mk] - diff);
                else itab[mk] = (short)(itab[mk] - diff);
            }
        }
    memcpy(g_bilin, flat, sizeof(g_bilin));
    g_bilin_ready = 1;
}

void orc_bilinear_weights(int fx, int fy, short *w4)
{
    bilinear_tab();
    memcpy(w4, g_bilin[fy * INTER_TAB_SIZE + fx], 4 * sizeof(short));
}

static inline int sat_i32_round(double v)
{
    /* std::max((double)INT_MIN, std::min((double)INT_MAX, v)) then cvRound (round half even) */
    double a = (double)INT_MAX, b = (double)INT_MIN;
    v = (v < a) ? v : a;    /* std::min(a, v) returns a unless v < a (NaN -> INT_MAX) */
    v = (b < v) ? v : b;    /* std::max(b, v) */
    return (int)lrint(v);
}

static inline short sat_i16(int v)
{
    return (short)(v < SHRT_MIN ? SHRT_MIN : (v > SHRT_MAX ? SHRT_MAX : v));
}

/* Map one canvas row segment [x, x+bw) of row y in block-structured OpenCV order.
 * Emits integer source coords (nearest) or (coord>>5, alpha) (bilinear). */
static void map_block_row(const double *M, int interp, int x, int y, int bw, short *xy,
                          unsigned short *alpha)
{
    double X0 = M[0] * x + M[1] * y + M[2];
    double Y0 = M[3] * x + M[4] * y + M[5];
    double W0 = M[6] * x + M[7] * y + M[8];
    for (int x1 = 0; x1 < bw; x1++) {
        double W = W0 + M[6] * x1;
        if (interp == ORC_INTER_NEAREST) {
            W = W ? 1. / W : 0;
            int X = sat_i32_round((X0 + M[0] * x1) * W);
            int Y = sat_i32_round((Y0 + M[3] * x1) * W);
            xy[x1 * 2] = sat_i16(X);
            xy[x1 * 2 + 1] = sat_i16(Y);
        } else {
            W = W ? INTER_TAB_SIZE / W : 0;
            int X = sat_i32_round((X0 + M[0] * x1) * W);
            int Y = sat_i32_round((Y0 + M[3] * x1) * W);
            xy[x1 * 2] = sat_i16(X >> INTER_BITS);
            xy[x1 * 2 + 1] = sat_i16(Y >> INTER_BITS);
            alpha[x1] = (unsigned short)((Y & (INTER_TAB_SIZE - 1)) * INTER_TAB_SIZE +
                                         (X & (INTER_TAB_SIZE - 1)));
        }
    }
}

/* remapNearest / remapBilinear for one pixel, BORDER_CONSTANT value 0. */
static inline void sample_px(const uint8_t *src, int sw, int sh, long sstep, int cn, int interp,
                             int sx, int sy, int alpha, uint8_t *d)
{
    if (interp == ORC_INTER_NEAREST) {
        if ((unsigned)sx < (unsigned)sw && (unsigned)sy < (unsigned)sh) {
            const uint8_t *S = src + (long)sy * sstep + (long)sx * cn;
            for (int k = 0; k < cn; k++) d[k] = S[k];
        } else {
            for (int k = 0; k < cn; k++) d[k] = 0;
        }
        return;
    }
    if (sx >= sw || sx + 1 < 0 || sy >= sh || sy + 1 < 0) {
        for (int k = 0; k < cn; k++) d[k] = 0;
        return;
    }
    const short *w = g_bilin[alpha];
    int x0ok = sx >= 0 && sx < sw, x1ok = sx + 1 >= 0 && sx + 1 < sw;
    int y0ok = sy >= 0 && sy < sh, y1ok = sy + 1 >= 0 && sy + 1 < sh;
    for (int k = 0; k < cn; k++) {
        int v0 = (x0ok && y0ok) ? src[(long)sy * sstep + (long)sx * cn + k] : 0;
        int v1 = (x1ok && y0ok) ? src[(long)sy * sstep + (long)(sx + 1) * cn + k] : 0;
        int v2 = (x0ok && y1ok) ? src[(long)(sy + 1) * sstep + (long)sx * cn + k] : 0;
        int v3 = (x1ok && y1ok) ? src[(long)(sy + 1) * sstep + (long)(sx + 1) * cn + k] : 0;
        int s = v0 * w[0] + v1 * w[1] + v2 * w[2] + v3 * w[3];
        int r = (s + (1 << (COEF_BITS - 1))) >> COEF_BITS;
        d[k] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
    }
}

/* remapBilinear of one pixel from a CV_16SC2 (sx, sy) + CV_16UC1 (alpha) map entry. */
void orc__remap_bilinear_px(const uint8_t *src, int sw, int sh, long sstep, int cn, int sx, int sy,
                            int alpha, uint8_t *d)
{
    bilinear_tab();
    sample_px(src, sw, sh, sstep, cn, ORC_INTER_LINEAR, sx, sy, alpha, d);
}

/* Block geometry of WarpPerspectiveInvoker (BLOCK_SZ = 32). */
static void block_geom(int dw, int dh, int *bw0_out)
{
    int bh0 = dh < 16 ? dh : 16;
    if (bh0 < 1) bh0 = 1;
    int bw0 = 1024 / bh0;
    if (bw0 > dw) bw0 = dw;
    if (bw0 < 1) bw0 = 1;
    *bw0_out = bw0;
}

/* cv::warpPerspective(src, M, dsize, flags=interp [| WARP_INVERSE_MAP], BORDER_CONSTANT, 0).
 * M is the matrix as passed by the caller; it is inverted unless inverse_map is set. */
int orc_warp_perspective(const uint8_t *src, int sw, int sh, long sstep, int cn, uint8_t *dst,
                         int dw, int dh, long dstep, const double *M_in, int interp,
                         int inverse_map)
{
    double M[9];
    if (inverse_map) memcpy(M, M_in, sizeof(M));
    else orc_invert3x3(M_in, M);
    bilinear_tab();
    int bw0;
    block_geom(dw, dh, &bw0);
#pragma omp parallel for schedule(static)
    for (int y = 0; y < dh; y++) {
        short xy[2 * 1024];
        unsigned short alpha[1024];
        uint8_t *D = dst + (long)y * dstep;
        for (int x = 0; x < dw; x += bw0) {
            int bw = dw - x < bw0 ? dw - x : bw0;
            map_block_row(M, interp, x, y, bw, xy, alpha);
            for (int x1 = 0; x1 < bw; x1++)
                sample_px(src, sw, sh, sstep, cn, interp, xy[2 * x1], xy[2 * x1 + 1],
                          interp == ORC_INTER_NEAREST ? 0 : alpha[x1], D + (long)(x + x1) * cn);
        }
    }
    return 0;
}

/* Python slice normalisation for a[start:stop] on an axis of length n (step 1). */
static void py_slice(long start, long stop, long n, long *s0, long *s1)
{
    if (start < 0) { start += n; if (start < 0) start = 0; }
    else if (start > n) start = n;
    if (stop < 0) { stop += n; if (stop < 0) stop = 0; }
    else if (stop > n) stop = n;
    if (stop < start) stop = start;
    *s0 = start;
    *s1 = stop;
}

/* One calibrated stage of the reference chain, restated from StitcherBase.stitch
 * (StitcherClass.py:223-253): warp A into a fresh (ABSize) canvas, overwrite-paste B at
 * Bpts[0], then (super mode) crop [y_limits[0]:y_limits[1], x_limits[0]:x_limits[1]].
 * Writes the (cropped) result into out (pitch ow*cn), returns its size via ow/oh.
 * Returns 0, or -1 if B does not fit (numpy would raise a broadcast error). */
typedef struct orc_stage {
    double H[9];                /* cachedAH, forward (as passed to cv2.warpPerspective) */
    int canvas_w, canvas_h;     /* ABSize */
    int bx, by;                 /* int(Bpts[0][0]), int(Bpts[0][1]) */
    int super_mode;
    int xl0, xl1, yl0, yl1;     /* x_limits, y_limits (used when super_mode) */
} orc_stage;

int orc_stage_stitch(const orc_stage *st, const uint8_t *A, int aw, int ah,
                     const uint8_t *B, int bw, int bh, int cn, int interp,
                     uint8_t *canvas /* canvas_w*canvas_h*cn scratch */,
                     uint8_t *out, int *ow, int *oh)
{
    int W = st->canvas_w, H = st->canvas_h;
    orc_warp_perspective(A, aw, ah, (long)aw * cn, cn, canvas, W, H, (long)W * cn, st->H, interp,
                         0);
    /* numpy: dst[By:By+hB, Bx:Bx+wB] = imageB (slice clipped, shapes must then match) */
    long ys0, ys1, xs0, xs1;
    py_slice(st->by, (long)st->by + bh, H, &ys0, &ys1);
    py_slice(st->bx, (long)st->bx + bw, W, &xs0, &xs1);
    if (ys1 - ys0 != bh || xs1 - xs0 != bw) return -1;
    for (long y = 0; y < bh; y++)
        memcpy(canvas + ((ys0 + y) * W + xs0) * cn, B + y * (long)bw * cn, (size_t)bw * cn);
    long cy0 = 0, cy1 = H, cx0 = 0, cx1 = W;
    if (st->super_mode) {
        py_slice(st->yl0, st->yl1, H, &cy0, &cy1);
        py_slice(st->xl0, st->xl1, W, &cx0, &cx1);
    }
    long w2 = cx1 - cx0, h2 = cy1 - cy0;
    for (long y = 0; y < h2; y++)
        memcpy(out + y * w2 * cn, canvas + ((cy0 + y) * W + cx0) * cn, (size_t)(w2 * cn));
    *ow = (int)w2;
    *oh = (int)h2;
    return 0;
}

/* Whole cascade (Stitcher.stitch, StitcherClass.py:130-136) for calibrated stages.
 * cams[0..n_stages]: camera images in sorted-label order, sizes cw/ch.  out must hold the
 * final mosaic (size queried with orc_cascade_out_size).  Returns 0 or -1. */
int orc_cascade_out_size(const orc_stage *st, int n_stages, int *ow, int *oh)
{
    if (n_stages <= 0) return -1;
    const orc_stage *s = &st[n_stages - 1];
    long cy0 = 0, cy1 = s->canvas_h, cx0 = 0, cx1 = s->canvas_w;
    if (s->super_mode) {
        py_slice(s->yl0, s->yl1, s->canvas_h, &cy0, &cy1);
        py_slice(s->xl0, s->xl1, s->canvas_w, &cx0, &cx1);
    }
    *ow = (int)(cx1 - cx0);
    *oh = (int)(cy1 - cy0);
    return 0;
}

int orc_cascade_stitch(const orc_stage *st, int n_stages, const uint8_t *const *cams,
                       const int *cw, const int *ch, int cn, int interp, uint8_t *out)
{
    long maxc = 0;
    for (int k = 0; k < n_stages; k++) {
        long c = (long)st[k].canvas_w * st[k].canvas_h * cn;
        if (c > maxc) maxc = c;
    }
    uint8_t *canvas = (uint8_t *)malloc((size_t)maxc);
    uint8_t *prev = (uint8_t *)malloc((size_t)maxc);
    uint8_t *cur = (uint8_t *)malloc((size_t)maxc);
    if (!canvas || !prev || !cur) { free(canvas); free(prev); free(cur); return -1; }
    const uint8_t *B = cams[0];
    int bw = cw[0], bh = ch[0], rc = 0;
    for (int k = 0; k < n_stages && rc == 0; k++) {
        int ow, oh;
        uint8_t *dst = (k == n_stages - 1) ? out : cur;
        rc = orc_stage_stitch(&st[k], cams[k + 1], cw[k + 1], ch[k + 1], B, bw, bh, cn, interp,
                              canvas, dst, &ow, &oh);
        if (k != n_stages - 1) {
            uint8_t *t = prev; prev = cur; cur = t;
            B = prev;
        }
        bw = ow;
        bh = oh;
    }
    free(canvas); free(prev); free(cur);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* Flattened single-pass gather on the CPU: the same mosaic rendered per output pixel through
 * the nested paste rectangles (SURVEY.md section 3 "Verified equivalence").  Used to check
 * the flattening itself independently of the GPU.  Per stage k the caller passes:
 *   off_x/off_y[k] : output coords -> stage-k canvas coords,
 *   rect[k]        : B rect of stage k in output coords (x0,y0,x1,y1),
 *   minv[k]        : OpenCV-inverted stage matrix, bw0[k]: block width of its canvas,
 *   off_x/off_y[n_stages] : output coords -> camera-0 coords.                               */
int orc_flat_stitch(int n_stages, const int *off_x, const int *off_y, const int *rect,
                    const double *minv, const int *bw0, const uint8_t *const *cams,
                    const int *cw, const int *ch, int cn, int interp, uint8_t *out, int ow,
                    int oh)
{
    bilinear_tab();
#pragma omp parallel for schedule(static)
    for (int y = 0; y < oh; y++) {
        for (int x = 0; x < ow; x++) {
            uint8_t *d = out + ((long)y * ow + x) * cn;
            int s = n_stages - 1;
            while (s >= 0 && x >= rect[4 * s] && y >= rect[4 * s + 1] && x < rect[4 * s + 2] &&
                   y < rect[4 * s + 3])
                s--;
            if (s < 0) {
                int X = x + off_x[n_stages], Y = y + off_y[n_stages];
                const uint8_t *S = cams[0] + ((long)Y * cw[0] + X) * cn;
                for (int k = 0; k < cn; k++) d[k] = S[k];
                continue;
            }
            int X = x + off_x[s], Y = y + off_y[s];
            int xb = (X / bw0[s]) * bw0[s];
            short xy[2];
            unsigned short al = 0;
            /* per-pixel evaluation with the block-start X0 of its OpenCV block */
            {
                const double *M = minv + 9 * s;
                double X0 = M[0] * xb + M[1] * Y + M[2];
                double Y0 = M[3] * xb + M[4] * Y + M[5];
                double W0 = M[6] * xb + M[7] * Y + M[8];
                int x1 = X - xb;
                double W = W0 + M[6] * x1;
                if (interp == ORC_INTER_NEAREST) {
                    W = W ? 1. / W : 0;
                    xy[0] = sat_i16(sat_i32_round((X0 + M[0] * x1) * W));
                    xy[1] = sat_i16(sat_i32_round((Y0 + M[3] * x1) * W));
                } else {
                    W = W ? INTER_TAB_SIZE / W : 0;
                    int Xi = sat_i32_round((X0 + M[0] * x1) * W);
                    int Yi = sat_i32_round((Y0 + M[3] * x1) * W);
                    xy[0] = sat_i16(Xi >> INTER_BITS);
                    xy[1] = sat_i16(Yi >> INTER_BITS);
                    al = (unsigned short)((Yi & 31) * 32 + (Xi & 31));
                }
            }
            int c = s + 1;
            sample_px(cams[c], cw[c], ch[c], (long)cw[c] * cn, cn, interp, xy[0], xy[1], al, d);
        }
    }
    return 0;
}

/* Stage map of one canvas pixel (X, Y) in 1/32-px fixed point, evaluated like the cascade:
 * block-start X0 of its OpenCV block, per-pixel W; integer coordinates x 32 for nearest.
 * Shared with orc_blend.c. */
void orc__stage_xy(const double *M, int bw0, int interp, int X, int Y, int *x32, int *y32)
{
    int xb = (X / bw0) * bw0;
    double X0 = M[0] * xb + M[1] * Y + M[2];
    double Y0 = M[3] * xb + M[4] * Y + M[5];
    double W0 = M[6] * xb + M[7] * Y + M[8];
    int x1 = X - xb;
    double W = W0 + M[6] * x1;
    if (interp == ORC_INTER_NEAREST) {
        W = W ? 1. / W : 0;
        *x32 = sat_i16(sat_i32_round((X0 + M[0] * x1) * W)) * 32;
        *y32 = sat_i16(sat_i32_round((Y0 + M[3] * x1) * W)) * 32;
    } else {
        W = W ? INTER_TAB_SIZE / W : 0;
        int Xi = sat_i32_round((X0 + M[0] * x1) * W);
        int Yi = sat_i32_round((Y0 + M[3] * x1) * W);
        *x32 = sat_i16(Xi >> INTER_BITS) * 32 + (Xi & 31);
        *y32 = sat_i16(Yi >> INTER_BITS) * 32 + (Yi & 31);
    }
}

/* Bilinear sample at (x32, y32) with BORDER_REPLICATE (taps clamped into the image), the
 * remapBilinear fixed-point arithmetic (weights of the initInterTab2D table). */
void orc__sample_replicate(const uint8_t *src, int sw, int sh, int cn, int x32, int y32,
                           uint8_t *d)
{
    bilinear_tab();
    int sx = x32 >> 5, sy = y32 >> 5;
    const short *w = g_bilin[(y32 & 31) * INTER_TAB_SIZE + (x32 & 31)];
    int xa = sx < 0 ? 0 : (sx >= sw ? sw - 1 : sx);
    int xb = sx + 1 < 0 ? 0 : (sx + 1 >= sw ? sw - 1 : sx + 1);
    int ya = sy < 0 ? 0 : (sy >= sh ? sh - 1 : sy);
    int yb = sy + 1 < 0 ? 0 : (sy + 1 >= sh ? sh - 1 : sy + 1);
    long st = (long)sw * cn;
    for (int k = 0; k < cn; k++) {
        int v0 = src[ya * st + (long)xa * cn + k], v1 = src[ya * st + (long)xb * cn + k];
        int v2 = src[yb * st + (long)xa * cn + k], v3 = src[yb * st + (long)xb * cn + k];
        int s = v0 * w[0] + v1 * w[1] + v2 * w[2] + v3 * w[3];
        int r = (s + (1 << (COEF_BITS - 1))) >> COEF_BITS;
        d[k] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
    }
}

/* Single-pixel coordinate probe (known-answer tests). */
void orc_map_pixel(const double *Minv, int interp, int xb, int x1, int y, int *X, int *Y)
{
    short xy[2 * 1024];
    unsigned short al[1024];
    map_block_row(Minv, interp, xb, y, x1 + 1, xy, al);
    if (interp == ORC_INTER_NEAREST) {
        *X = xy[2 * x1];
        *Y = xy[2 * x1 + 1];
    } else {
        *X = xy[2 * x1] * 32 + (al[x1] & 31);
        *Y = xy[2 * x1 + 1] * 32 + (al[x1] >> 5);
    }
}

int orc_num_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void orc_set_num_threads(int n)
{
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* Cylinder slot map (orc_blend.c, cylindrical plans): the rig ray
 * (sn, hv, cs) of a panorama column/row rotated into the camera by R (explicit summation order),
 * projected x = f dx / dz + cx; rays with dz <= 0 land far outside every frame.  Same fixed-point
 * conventions as orc__stage_xy. */
void orc__cyl_xy(const double *R, double f, double cx, double cy, double sn, double cs, double hv,
                 int interp, int *x32, int *y32)
{
    const double dx = (R[0] * sn + R[1] * hv) + R[2] * cs;
    const double dy = (R[3] * sn + R[4] * hv) + R[5] * cs;
    const double dz = (R[6] * sn + R[7] * hv) + R[8] * cs;
    int X, Y;
    if (!(dz > 0.0)) {
        X = Y = interp == ORC_INTER_NEAREST ? -(1 << 20) : -(1 << 25);
    } else {
        const double k = interp == ORC_INTER_NEAREST ? 1.0 : (double)INTER_TAB_SIZE;
        X = sat_i32_round(((f * dx) / dz + cx) * k);
        Y = sat_i32_round(((f * dy) / dz + cy) * k);
    }
    if (interp == ORC_INTER_NEAREST) {
        *x32 = sat_i16(X) * 32;
        *y32 = sat_i16(Y) * 32;
    } else {
        *x32 = sat_i16(X >> INTER_BITS) * 32 + (X & (INTER_TAB_SIZE - 1));
        *y32 = sat_i16(Y >> INTER_BITS) * 32 + (Y & (INTER_TAB_SIZE - 1));
    }
}

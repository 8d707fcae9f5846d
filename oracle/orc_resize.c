/*
 * orc_resize.c -- TEST INFRASTRUCTURE ONLY (the parity checker), never the product path.
 *
 * CPU restatement of the resize the reference applies before warping when a frame does not
 * have its calibrated shape:
 *
 *   PostScripts/Stitcher/StitcherClass.py:226-233  StitcherBase.stitch
 *     imageB = cv2.resize(imageB, (BimgSize[1], BimgSize[0]), interpolation=cv2.INTER_LINEAR)
 *     imageA = cv2.resize(imageA, (AimgSize[1], AimgSize[0]), interpolation=cv2.INTER_LINEAR)
 *
 * OpenCV is third-party (not vendored, version unpinned; the reference's code needs 2.4 or 3.x).
 * Restated from OpenCV 3.4 modules/imgproc/src/resize.cpp, generic (non-IPP, non-OpenCL) path
 * for CV_8U:
 *   - dsize == ssize: plain copy.
 *   - scale_x == scale_y == 2 exactly: INTER_LINEAR becomes INTER_AREA, whose fast 2x2 path is
 *     (a + b + c + d + 2) >> 2 per channel for 1/3/4 channels (ResizeAreaFastVec) and
 *     saturate_cast<uchar>(sum * 0.25f) (round half to even) otherwise (resizeAreaFast_).
 *   - otherwise fixed-point bilinear, INTER_RESIZE_COEF_BITS = 11:
 *       scale = (double)ssize / dsize;  f = (float)((d + 0.5) * scale - 0.5);  s = cvFloor(f);
 *       f -= s;  x: s < 0 -> (s, f) = (0, 0); s >= sw-1 -> (s, f) = (sw-1, 0)  (one tap, x ONE)
 *       coefficients saturate_cast<short>((1-f) * 2048), saturate_cast<short>(f * 2048)
 *       (rounded separately, so a pair may sum to 2047 or 2049); rows clipped to [0, sh-1]
 *       with their coefficients kept;
 *       horizontal: D = S[sx] * a0 + S[sx + cn] * a1 (int);
 *       vertical (VResizeLinear<uchar, int, short, FixedPtCast<int, uchar, 22>>):
 *       dst = (((b0 * (D0 >> 4)) >> 16) + ((b1 * (D1 >> 4)) >> 16) + 2) >> 2.
 * Parity against a real cv2 is unpinned (none in this image); pinned by known-answer tests.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define RESIZE_COEF_BITS 11
#define RESIZE_COEF_SCALE (1 << RESIZE_COEF_BITS)

static inline short sat_short_round(float v)
{
    /* saturate_cast<short>(float): cvRound (round half to even) then clamp */
    long r = lrintf(v);
    if (r > 32767) r = 32767;
    if (r < -32768) r = -32768;
    return (short)r;
}

/* Coefficient tables of one axis (OpenCV resize(): xofs/ialpha, yofs/ibeta before expansion). */
void orc_resize_axis(int ssize, int dsize, int is_x, int *ofs, short *coef)
{
    const double scale = 1. / ((double)dsize / ssize);
    for (int d = 0; d < dsize; d++) {
        float f = (float)((d + 0.5) * scale - 0.5);
        int s = (int)floorf(f);
        f -= (float)s;
        if (is_x) {
            if (s < 0) f = 0.f, s = 0;
            if (s >= ssize - 1) f = 0.f, s = ssize - 1;
        }
        ofs[d] = s;
        coef[2 * d] = sat_short_round((1.f - f) * RESIZE_COEF_SCALE);
        coef[2 * d + 1] = sat_short_round(f * RESIZE_COEF_SCALE);
    }
}

static inline int clip_row(int y, int h) { return y < 0 ? 0 : (y >= h ? h - 1 : y); }

int orc_resize_linear(const uint8_t *src, int sw, int sh, long sstep, int cn, uint8_t *dst,
                      int dw, int dh, long dstep)
{
    if (sw <= 0 || sh <= 0 || dw <= 0 || dh <= 0 || cn <= 0) return -1;
    if (sw == dw && sh == dh) {
        for (int y = 0; y < dh; y++) memcpy(dst + y * dstep, src + y * sstep, (size_t)dw * cn);
        return 0;
    }
    const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
    if (scale_x == 2. && scale_y == 2.) {
        for (int y = 0; y < dh; y++) {
            const uint8_t *s0 = src + (long)(2 * y) * sstep, *s1 = s0 + sstep;
            for (int x = 0; x < dw; x++)
                for (int k = 0; k < cn; k++) {
                    const int a = s0[2 * x * cn + k], b = s0[(2 * x + 1) * cn + k];
                    const int c = s1[2 * x * cn + k], d = s1[(2 * x + 1) * cn + k];
                    const int sum = a + b + c + d;
                    /* cn 1/3/4: ResizeAreaFastVec, (sum + 2) >> 2; otherwise the generic
                     * saturate_cast<uchar>(sum * 0.25f): round half to even */
                    dst[y * dstep + (long)x * cn + k] =
                        (uint8_t)(cn == 2 ? (int)lrintf((float)sum * 0.25f) : (sum + 2) >> 2);
                }
        }
        return 0;
    }
    int *xofs = (int *)malloc(sizeof(int) * dw), *yofs = (int *)malloc(sizeof(int) * dh);
    short *alpha = (short *)malloc(sizeof(short) * 2 * dw);
    short *beta = (short *)malloc(sizeof(short) * 2 * dh);
    int *rows = (int *)malloc(sizeof(int) * 2 * (size_t)dw * cn);
    if (!xofs || !yofs || !alpha || !beta || !rows) {
        free(xofs); free(yofs); free(alpha); free(beta); free(rows);
        return -1;
    }
    orc_resize_axis(sw, dw, 1, xofs, alpha);
    orc_resize_axis(sh, dh, 0, yofs, beta);
    for (int y = 0; y < dh; y++) {
        for (int r = 0; r < 2; r++) {
            const uint8_t *S = src + (long)clip_row(yofs[y] + r, sh) * sstep;
            int *D = rows + (size_t)r * dw * cn;
            for (int x = 0; x < dw; x++) {
                const int sx = xofs[x] * cn;
                const int a0 = alpha[2 * x], a1 = alpha[2 * x + 1];
                for (int k = 0; k < cn; k++)
                    D[x * cn + k] = xofs[x] >= sw - 1 ? S[sx + k] * RESIZE_COEF_SCALE
                                                      : S[sx + k] * a0 + S[sx + cn + k] * a1;
            }
        }
        const int b0 = beta[2 * y], b1 = beta[2 * y + 1];
        const int *D0 = rows, *D1 = rows + (size_t)dw * cn;
        uint8_t *out = dst + y * dstep;
        for (int i = 0; i < dw * cn; i++)
            out[i] = (uint8_t)((((b0 * (D0[i] >> 4)) >> 16) + ((b1 * (D1[i] >> 4)) >> 16) + 2) >> 2);
    }
    free(xofs); free(yofs); free(alpha); free(beta); free(rows);
    return 0;
}

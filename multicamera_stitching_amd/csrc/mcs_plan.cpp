// mcs_plan.cpp -- host side of libmcs: turns the reference's calibrated StitcherBase chain
// (PostScripts/Stitcher/StitcherClass.py:190-209, 258-351) into the flattened single-pass
// geometry the gather kernel consumes.
//
// Why a flattening is exact: StitcherBase.stitch (:239-251) warps A into a fresh canvas, pastes
// the previous mosaic B over it at an integer offset and optionally crops; the chain (:130-136)
// feeds each result in as the next B.  So every output pixel is either inside the innermost
// paste rectangle that contains it (-> recurse into that B, a pure integer translation) or it
// is the warped A of the first stage (outermost-first) whose rectangle does NOT contain it.
// Each pixel therefore needs one ownership walk and one sample from one camera, evaluated at
// the same canvas coordinates (so with the same OpenCV 64-column block start) as the cascade.
//
// Compiled with -ffp-contract=off: the inverse must be bit-identical to cv::invert.
#include "mcs_common.h"

#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <cmath>
#include <cstring>

namespace mcs {

static thread_local char g_err[512];

int fail(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

const char *last_error() { return g_err; }
void clear_error() { g_err[0] = 0; }

// cv::invert(src, dst, DECOMP_LU) for a 3x3 CV_64F matrix: OpenCV's n <= 3 closed form
// (modules/core/src/lapack.cpp, det3 + cofactors scaled by 1/d; d == 0 -> all zeros).
void invert3x3_cv(const double *m, double *out)
{
#define Md(i, j) m[(i) * 3 + (j)]
    double d = Md(0, 0) * (Md(1, 1) * Md(2, 2) - Md(1, 2) * Md(2, 1)) -
               Md(0, 1) * (Md(1, 0) * Md(2, 2) - Md(1, 2) * Md(2, 0)) +
               Md(0, 2) * (Md(1, 0) * Md(2, 1) - Md(1, 1) * Md(2, 0));
    if (d == 0.) {
        for (int i = 0; i < 9; i++) out[i] = 0.;
        return;
    }
    double t[9];
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
}

// Python slice normalisation a[start:stop] on an axis of length n (numpy basic slicing).
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

// WarpPerspectiveInvoker block geometry (BLOCK_SZ = 32): bh0 = min(16, H); bw0 = min(1024/bh0, W).
int block_width(int W, int H)
{
    int bh0 = H < 16 ? H : 16;
    if (bh0 < 1) bh0 = 1;
    int bw0 = 1024 / bh0;
    if (bw0 > W) bw0 = W;
    return bw0 < 1 ? 1 : bw0;
}

int build_flat(const mcs_stage_desc *stages, int n_stages, int cam0_w, int cam0_h, int channels,
               int interp, mcs_flat_desc *fd)
{
    if (n_stages < 1 || n_stages > MCS_MAX_STAGES)
        return fail(MCS_E_UNSUPPORTED, "n_stages=%d outside [1,%d]", n_stages, MCS_MAX_STAGES);
    if (channels < 1 || channels > 4)
        return fail(MCS_E_UNSUPPORTED, "channels=%d outside [1,4]", channels);
    if (interp != MCS_INTER_LINEAR && interp != MCS_INTER_NEAREST)
        return fail(MCS_E_INVALID, "interp=%d", interp);
    if (cam0_w < 1 || cam0_h < 1) return fail(MCS_E_SHAPE, "camera 0 size %dx%d", cam0_w, cam0_h);
    if ((long)cam0_w * cam0_h * channels < 8)
        return fail(MCS_E_UNSUPPORTED, "camera 0 frame of %ld bytes (< 8)",
                    (long)cam0_w * cam0_h * channels);

    memset(fd, 0, sizeof(*fd));
    fd->channels = channels;
    fd->interp = interp;
    fd->n_cams = n_stages + 1;
    fd->cam_w[0] = cam0_w;
    fd->cam_h[0] = cam0_h;

    // Forward walk: sizes and crop windows of every calibrated stage.
    struct Fw { int k; long cx0, cy0, ow, oh; };
    Fw fw[MCS_MAX_STAGES];
    int m = 0;
    long bw = cam0_w, bh = cam0_h;   // current B (previous output) size
    for (int k = 0; k < n_stages; k++) {
        const mcs_stage_desc &s = stages[k];
        fd->cam_w[k + 1] = s.a_w;
        fd->cam_h[k + 1] = s.a_h;
        if (!s.calibrated) continue;   // StitcherClass.py:255-256: returns B unchanged
        if (s.a_w < 1 || s.a_h < 1)
            return fail(MCS_E_SHAPE, "stage %d: A size %dx%d", k, s.a_w, s.a_h);
        if ((long)s.a_w * s.a_h * channels < 8)
            return fail(MCS_E_UNSUPPORTED, "stage %d: camera frame of %ld bytes (< 8)", k,
                        (long)s.a_w * s.a_h * channels);
        if (s.b_w != bw || s.b_h != bh)
            return fail(MCS_E_SHAPE,
                        "stage %d: calibrated B size %dx%d != chain size %ldx%ld (the reference "
                        "would cv2.resize the mosaic here)", k, s.b_w, s.b_h, bw, bh);
        if (s.canvas_w < 1 || s.canvas_h < 1)
            return fail(MCS_E_SHAPE, "stage %d: ABSize %dx%d", k, s.canvas_w, s.canvas_h);
        // numpy slice-assign dst[By:By+hB, Bx:Bx+wB] = B must not clip (else broadcast error)
        long ys0, ys1, xs0, xs1;
        py_slice(s.b_y, (long)s.b_y + bh, s.canvas_h, &ys0, &ys1);
        py_slice(s.b_x, (long)s.b_x + bw, s.canvas_w, &xs0, &xs1);
        if (ys1 - ys0 != bh || xs1 - xs0 != bw || ys0 != s.b_y || xs0 != s.b_x)
            return fail(MCS_E_SHAPE, "stage %d: B %ldx%ld at (%d,%d) does not fit canvas %dx%d",
                        k, bw, bh, s.b_x, s.b_y, s.canvas_w, s.canvas_h);
        long cx0 = 0, cx1 = s.canvas_w, cy0 = 0, cy1 = s.canvas_h;
        if (s.super_mode) {
            py_slice(s.y_lim0, s.y_lim1, s.canvas_h, &cy0, &cy1);
            py_slice(s.x_lim0, s.x_lim1, s.canvas_w, &cx0, &cx1);
        }
        fw[m].k = k;
        fw[m].cx0 = cx0;
        fw[m].cy0 = cy0;
        fw[m].ow = cx1 - cx0;
        fw[m].oh = cy1 - cy0;
        bw = fw[m].ow;
        bh = fw[m].oh;
        m++;
    }
    fd->n_stages = m;
    fd->out_w = (int)bw;
    fd->out_h = (int)bh;
    if (m == 0) {   // every stage passes through: the mosaic is camera 0
        fd->cam0_off_x = 0;
        fd->cam0_off_y = 0;
        return MCS_OK;
    }
    // Backward walk: output coords -> canvas coords of each calibrated stage.
    long ox = fw[m - 1].cx0, oy = fw[m - 1].cy0;
    for (int j = m - 1; j >= 0; j--) {
        const mcs_stage_desc &s = stages[fw[j].k];
        mcs_flat_stage &f = fd->st[j];
        invert3x3_cv(s.H, f.minv);
        f.off_x = (int)ox;
        f.off_y = (int)oy;
        f.bw0 = block_width(s.canvas_w, s.canvas_h);
        f.cam = fw[j].k + 1;
        long bwj = (j == 0) ? cam0_w : fw[j - 1].ow;
        long bhj = (j == 0) ? cam0_h : fw[j - 1].oh;
        f.rect[0] = (int)(s.b_x - ox);
        f.rect[1] = (int)(s.b_y - oy);
        f.rect[2] = (int)(s.b_x - ox + bwj);
        f.rect[3] = (int)(s.b_y - oy + bhj);
        // canvas_j = B + b  ->  B coords = canvas_j - b = out + off_j - b;
        // previous canvas = B coords + previous crop origin
        ox = ox - s.b_x + (j > 0 ? fw[j - 1].cx0 : 0);
        oy = oy - s.b_y + (j > 0 ? fw[j - 1].cy0 : 0);
    }
    fd->cam0_off_x = (int)ox;
    fd->cam0_off_y = (int)oy;
    return MCS_OK;
}

void fill_kparams(const mcs_flat_desc &fd, KParams *kp)
{
    memset(kp, 0, sizeof(*kp));
    kp->n_stages = fd.n_stages;
    kp->out_w = fd.out_w;
    kp->out_h = fd.out_h;
    kp->cam0_offx = fd.cam0_off_x;
    kp->cam0_offy = fd.cam0_off_y;
    kp->cam0_w = fd.cam_w[0];
    kp->cam0_h = fd.cam_h[0];
    for (int i = 0; i < fd.n_cams; i++) {
        kp->cam_w[i] = fd.cam_w[i];
        kp->cam_h[i] = fd.cam_h[i];
    }
    for (int j = 0; j < fd.n_stages; j++) {
        const mcs_flat_stage &s = fd.st[j];
        KStage &k = kp->st[j];
        memcpy(k.m, s.minv, sizeof(k.m));
        k.rx0 = s.rect[0];
        k.ry0 = s.rect[1];
        k.rx1 = s.rect[2];
        k.ry1 = s.rect[3];
        k.offx = s.off_x;
        k.offy = s.off_y;
        k.bw0 = s.bw0;
        k.bw_shift = -1;
        for (int b = 0; b < 31; b++)
            if ((1 << b) == s.bw0) k.bw_shift = b;
        k.cam = s.cam;
        k.src_w = fd.cam_w[s.cam];
        k.src_h = fd.cam_h[s.cam];
    }
}

// cv::undistort(src, K, dist) coordinate map (OpenCV 3.4 imgproc/src/undistort.cpp): stripes of
// min(max(1, 4096 / w), h) rows, each with the new camera matrix's cy shifted by the stripe's
// first row, initUndistortRectifyMap's scalar loop (iR = inv(A_r) by cv::invert DECOMP_LU; x, y,
// w accumulated along the row by repeated addition; the rational + tangential + thin-prism model,
// tilt identity) and its CV_16SC2 + CV_16UC1 packing.  tab[2 p] / tab[2 p + 1]: the map value of
// output pixel p as (short)(iu >> 5) * 32 + (iu & 31), i.e. the bilinear fixed point the stitch
// kernels sample with.  Returns false for distortion vectors the map does not cover.
bool undistort_map(const double *K, const double *dist, int n_dist, int w, int h, int32_t *tab)
{
    double k[14] = {0};
    if (!(n_dist == 0 || n_dist == 4 || n_dist == 5 || n_dist == 8 || n_dist == 12 ||
          n_dist == 14))
        return false;
    for (int i = 0; i < n_dist; i++) k[i] = dist[i];
    if (k[12] != 0.0 || k[13] != 0.0) return false;   // sensor tilt: not supported
    const double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3], k3 = k[4], k4 = k[5], k5 = k[6],
                 k6 = k[7], s1 = k[8], s2 = k[9], s3 = k[10], s4 = k[11];
    const double u0 = K[2], v0 = K[5], fx = K[0], fy = K[4];
    const int stripe0 = std::min(std::max(1, (1 << 12) / std::max(w, 1)), h);
    for (int y0 = 0; y0 < h; y0 += stripe0) {
        const int rows = std::min(stripe0, h - y0);
        double Ar[9];
        memcpy(Ar, K, sizeof(Ar));
        Ar[5] = v0 - y0;
        double ir[9];
        invert3x3_cv(Ar, ir);
        for (int i = 0; i < rows; i++) {
            int32_t *row = tab + 2 * (int64_t)(y0 + i) * w;
            double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
            for (int j = 0; j < w; j++, _x += ir[0], _y += ir[3], _w += ir[6]) {
                const double ww = 1. / _w, x = _x * ww, y = _y * ww;
                const double x2 = x * x, y2 = y * y;
                const double r2 = x2 + y2, _2xy = 2 * x * y;
                const double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) /
                                  (1 + ((k6 * r2 + k5) * r2 + k4) * r2);
                const double xd = x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2;
                const double yd = y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2;
                // tilt = identity: vecTilt = (1 xd + 0 yd + 0, 0 xd + 1 yd + 0, 1), invProj = 1
                const double tx = 1.0 * xd + 0.0 * yd + 0.0 * 1.0;
                const double ty = 0.0 * xd + 1.0 * yd + 0.0 * 1.0;
                const double u = fx * 1.0 * tx + u0, v = fy * 1.0 * ty + v0;
                const int iu = (int)lrint(u * 32), iv = (int)lrint(v * 32);
                row[2 * j] = (int32_t)(int16_t)(iu >> 5) * 32 + (iu & 31);
                row[2 * j + 1] = (int32_t)(int16_t)(iv >> 5) * 32 + (iv & 31);
            }
        }
    }
    return true;
}

}  // namespace mcs


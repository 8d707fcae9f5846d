// mcs_chain.cpp -- the chain geometry of one rig capture from its adjacent-pair homographies
// (SURVEY.md 8 C3 end to end): stage k maps camera k+1 into the mosaic of cameras 0..k,
// H_k = T(o_k) . H_0 . H_1 ... H_k (pair homographies composed into camera 0's frame, o_k =
// camera 0's origin in that mosaic), and each stage's plan fields follow
// StitcherBase.calibrate's arithmetic (PostScripts/Stitcher/StitcherClass.py:293-351,
// Utils.get_projection_point_dst Utils.py:23-37): corners projected and truncated toward zero,
// the translation patched into H[0][2] / H[1][2], ABSize from the re-projected corners, the
// super-mode limits.  The reference computes this once per calibration with numpy; config 3
// computes it for every capture, here, in FP64 in one fixed order (every 3-term dot product
// ((a0 b0 + a1 b1) + a2 b2), no contraction: the library builds with -ffp-contract=off), which
// estimate.chain_stages restates in plain Python floats -- the two agree bit for bit
// (tests/test_chain_cpu.py).  (numpy's 3x3 matmul goes through OpenBLAS, whose FMA kernels round
// differently and depend on the host CPU, so the per-capture path does not use it.)
#include <cmath>
#include <cstring>
#include <limits>

#include "mcs_common.h"

namespace {

struct Shape {
    int w, h;
};

// M . (x, y, 1) divided by its w, each coordinate truncated toward zero (int()), false when a
// coordinate is not finite or outside int range.
bool project(const double (&M)[9], int x, int y, int &px, int &py)
{
    const double X = (double)x, Y = (double)y;
    const double p0 = (M[0] * X + M[1] * Y) + M[2];
    const double p1 = (M[3] * X + M[4] * Y) + M[5];
    const double p2 = (M[6] * X + M[7] * Y) + M[8];
    const double u = p0 / p2, v = p1 / p2;
    const double lim = (double)std::numeric_limits<int>::max();
    if (!std::isfinite(u) || !std::isfinite(v) || std::fabs(u) >= lim || std::fabs(v) >= lim)
        return false;
    px = (int)u;   // truncation toward zero, as Python's int()
    py = (int)v;
    return true;
}

// Python slice(v, None).indices(n)[0] for step 1 (start / stop clamping).
int slice_index(int v, int n)
{
    if (v < 0) {
        v += n;
        return v < 0 ? 0 : v;
    }
    return v > n ? n : v;
}

// One calibrated stage from its A -> mosaic homography H (patched in place like cachedAH).
int stage_fields(double (&H)[9], Shape a, Shape b, int super_mode, mcs_stage_desc &d)
{
    const int ca[4][2] = {{0, 0}, {a.w, 0}, {a.w, a.h}, {0, a.h}};
    const int cb[4][2] = {{0, 0}, {b.w, 0}, {b.w, b.h}, {0, b.h}};
    int ax[4], ay[4];
    for (int i = 0; i < 4; i++)
        if (!project(H, ca[i][0], ca[i][1], ax[i], ay[i]))
            return mcs::fail(MCS_E_SHAPE, "chain geometry: a corner of camera A projects to "
                             "infinity or past int range");
    int x_min = ax[0], y_min = ay[0];
    for (int i = 0; i < 4; i++) {
        x_min = std::min(x_min, std::min(ax[i], cb[i][0]));
        y_min = std::min(y_min, std::min(ay[i], cb[i][1]));
    }
    H[2] = H[2] + (double)(-x_min);
    H[5] = H[5] + (double)(-y_min);
    const int tx = -x_min, ty = -y_min;
    const int bx[4] = {tx, tx + b.w, tx + b.w, tx}, by[4] = {ty, ty, b.h + ty, b.h + ty};
    for (int i = 0; i < 4; i++)
        if (!project(H, ca[i][0], ca[i][1], ax[i], ay[i]))
            return mcs::fail(MCS_E_SHAPE, "chain geometry: a corner of camera A projects to "
                             "infinity or past int range");
    int xmax = bx[0], ymax = by[0];
    for (int i = 0; i < 4; i++) {
        xmax = std::max(xmax, std::max(ax[i], bx[i]));
        ymax = std::max(ymax, std::max(ay[i], by[i]));
    }
    const int W = std::abs(xmax), Hh = std::abs(ymax);
    memcpy(d.H, H, sizeof(d.H));
    d.calibrated = 1;
    d.canvas_w = W;
    d.canvas_h = Hh;
    d.b_x = tx;
    d.b_y = ty;
    d.b_w = b.w;
    d.b_h = b.h;
    d.a_w = a.w;
    d.a_h = a.h;
    d.super_mode = super_mode ? 1 : 0;
    d.x_lim0 = d.x_lim1 = d.y_lim0 = d.y_lim1 = 0;
    if (super_mode) {
        // [max coordinate below half the size, min coordinate above it] over the 8 corners
        const double hw = W * 0.5, hh = Hh * 0.5;
        bool lo_x = false, hi_x = false, lo_y = false, hi_y = false;
        int xl0 = 0, xl1 = 0, yl0 = 0, yl1 = 0;
        for (int i = 0; i < 8; i++) {
            const int x = i < 4 ? ax[i] : bx[i - 4], y = i < 4 ? ay[i] : by[i - 4];
            if (x < hw && (!lo_x || x > xl0)) xl0 = x, lo_x = true;
            if (x > hw && (!hi_x || x < xl1)) xl1 = x, hi_x = true;
            if (y < hh && (!lo_y || y > yl0)) yl0 = y, lo_y = true;
            if (y > hh && (!hi_y || y < yl1)) yl1 = y, hi_y = true;
        }
        if (!(lo_x && hi_x && lo_y && hi_y))
            return mcs::fail(MCS_E_SHAPE, "chain geometry: no super-mode limit on one side "
                             "(the reference's max() / min() of an empty list)");
        d.x_lim0 = xl0, d.x_lim1 = xl1, d.y_lim0 = yl0, d.y_lim1 = yl1;
    }
    return MCS_OK;
}

}  // namespace

extern "C" int mcs_chain_stages(int n_cams, const int *cam_w, const int *cam_h,
                                const double *pair_H, const int *pair_ok, int super_mode,
                                mcs_stage_desc *out)
{
    mcs::clear_error();
    if (n_cams < 1 || n_cams > MCS_MAX_CAMS || !cam_w || !cam_h || !out ||
        (n_cams > 1 && (!pair_H || !pair_ok)))
        return mcs::fail(MCS_E_INVALID, "mcs_chain_stages: bad arguments");
    for (int i = 0; i < n_cams; i++)
        if (cam_w[i] <= 0 || cam_h[i] <= 0)
            return mcs::fail(MCS_E_INVALID, "mcs_chain_stages: camera %d size %d x %d", i,
                             cam_w[i], cam_h[i]);
    double P[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};   // camera k+1 -> camera 0
    int ox = 0, oy = 0;                           // camera 0's origin in the mosaic B_k
    Shape b{cam_w[0], cam_h[0]};
    bool broken = false;
    for (int k = 0; k + 1 < n_cams; k++) {
        mcs_stage_desc &d = out[k];
        memset(&d, 0, sizeof(d));
        const Shape a{cam_w[k + 1], cam_h[k + 1]};
        if (!pair_ok[k] || broken) {
            // (uncalibrated: B passes through; every later pair has no reference frame)
            broken = true;
            continue;
        }
        const double *Q = pair_H + 9 * k;
        double N[9];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)
                N[3 * i + j] = (P[3 * i] * Q[j] + P[3 * i + 1] * Q[3 + j]) + P[3 * i + 2] * Q[6 + j];
        memcpy(P, N, sizeof(P));
        const double T[9] = {1, 0, (double)ox, 0, 1, (double)oy, 0, 0, 1};
        double H[9];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)
                H[3 * i + j] = (T[3 * i] * P[j] + T[3 * i + 1] * P[3 + j]) + T[3 * i + 2] * P[6 + j];
        const double h22 = H[8];
        for (int i = 0; i < 9; i++) H[i] = H[i] / h22;
        const int rc = stage_fields(H, a, b, super_mode, d);
        if (rc) return rc;
        ox += d.b_x;
        oy += d.b_y;
        int W = d.canvas_w, Hh = d.canvas_h;
        if (super_mode) {
            const int x0 = slice_index(d.x_lim0, W), x1 = slice_index(d.x_lim1, W);
            const int y0 = slice_index(d.y_lim0, Hh), y1 = slice_index(d.y_lim1, Hh);
            ox -= x0;
            oy -= y0;
            W = std::max(0, x1 - x0);
            Hh = std::max(0, y1 - y0);
        }
        b = Shape{W, Hh};
    }
    return MCS_OK;
}

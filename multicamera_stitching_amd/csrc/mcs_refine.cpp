// mcs_refine.cpp -- what cv2.findHomography(src, dst, cv2.RANSAC, t) does after the RANSAC
// loop picked its model (the reference's call: PostScripts/Stitcher/StitcherClass.py:443-444;
// OpenCV 3.4 modules/calib3d/src/fundam.cpp, third-party, not vendored -- restated from its
// published source):
//
//   1. the correspondences are compressed to the RANSAC inliers;
//   2. HomographyEstimatorCallback::runKernel re-estimates the model on all of them: Hartley
//      normalisation (centroid, mean absolute deviation), the 9x9 LtL of the DLT rows (upper
//      triangle accumulated, then mirrored), its eigenvector of the smallest eigenvalue by
//      cv::eigen (the cyclic-max Jacobi of lapack.cpp, eigenvalues sorted descending),
//      denormalised (invHnorm * H0 * Hnorm2) and scaled by 1 / H[2][2];
//   3. cv::LMSolver (levmarq.cpp) refines h0..h7 for at most 10 iterations with
//      HomographyRefineCallback (residuals (proj - dst), analytic Jacobian, h8 taken as 1), each
//      step solving (JtJ + lambda diag(JtJ)) d = Jt r by DECOMP_EIG (Jacobi + back-substitution
//      dropping eigenvalues <= 2 eps sum(w)).
//
// Host FP64: an 8-parameter problem over the inliers (a few hundred to a few thousand points,
// microseconds) that runs once per estimated homography, after the GPU has scored every RANSAC
// hypothesis.  Restated independently in oracle/orc_ransac.c (orc_homography_refine).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <utility>
#include <vector>

#include "mcs_common.h"

namespace {

double cv_hypot(double a, double b)
{
    a = std::fabs(a);
    b = std::fabs(b);
    if (a > b) {
        b /= a;
        return a * std::sqrt(1 + b * b);
    }
    if (b > 0) {
        a /= b;
        return b * std::sqrt(1 + a * a);
    }
    return 0;
}

// cv::eigen of the symmetric N x N matrix A (its upper triangle; A is destroyed): eigenvalues
// W in descending order, eigenvectors as the rows of V.
template <int N>
void eigen_sym(double (&A)[N][N], double (&W)[N], double (&V)[N][N])
{
    int row_max[N], col_max[N];
    for (int i = 0; i < N; i++)
        for (int j = 0; j < N; j++) V[i][j] = i == j ? 1.0 : 0.0;
    // largest off-diagonal |a| right of the diagonal in row k / above it in column k
    auto scan_row = [&](int k) {
        int m = k + 1;
        double mv = std::fabs(A[k][m]);
        for (int i = k + 2; i < N; i++) {
            const double v = std::fabs(A[k][i]);
            if (mv < v) mv = v, m = i;
        }
        row_max[k] = m;
    };
    auto scan_col = [&](int k) {
        int m = 0;
        double mv = std::fabs(A[0][k]);
        for (int i = 1; i < k; i++) {
            const double v = std::fabs(A[i][k]);
            if (mv < v) mv = v, m = i;
        }
        col_max[k] = m;
    };
    for (int k = 0; k < N; k++) {
        W[k] = A[k][k];
        if (k < N - 1) scan_row(k);
        if (k > 0) scan_col(k);
    }
    for (int it = 0; it < N * N * 30; it++) {
        int k = 0;
        double mv = std::fabs(A[0][row_max[0]]);
        for (int i = 1; i < N - 1; i++) {
            const double v = std::fabs(A[i][row_max[i]]);
            if (mv < v) mv = v, k = i;
        }
        int l = row_max[k];
        for (int i = 1; i < N; i++) {
            const double v = std::fabs(A[col_max[i]][i]);
            if (mv < v) mv = v, k = col_max[i], l = i;
        }
        const double p = A[k][l];
        if (std::fabs(p) <= DBL_EPSILON) break;
        const double y = (W[l] - W[k]) * 0.5;
        double t = std::fabs(y) + cv_hypot(p, y);
        double s = cv_hypot(p, t);
        const double c = t / s;
        s = p / s;
        t = (p / t) * p;
        if (y < 0) s = -s, t = -t;
        A[k][l] = 0;
        W[k] -= t;
        W[l] += t;
        auto rot = [&](double &v0, double &v1) {
            const double a0 = v0, b0 = v1;
            v0 = a0 * c - b0 * s;
            v1 = a0 * s + b0 * c;
        };
        for (int i = 0; i < k; i++) rot(A[i][k], A[i][l]);
        for (int i = k + 1; i < l; i++) rot(A[k][i], A[i][l]);
        for (int i = l + 1; i < N; i++) rot(A[k][i], A[l][i]);
        for (int i = 0; i < N; i++) rot(V[k][i], V[l][i]);
        for (int idx : {k, l}) {
            if (idx < N - 1) scan_row(idx);
            if (idx > 0) scan_col(idx);
        }
    }
    for (int k = 0; k < N - 1; k++) {
        int m = k;
        for (int i = k + 1; i < N; i++)
            if (W[m] < W[i]) m = i;
        if (k != m) {
            std::swap(W[m], W[k]);
            for (int i = 0; i < N; i++) std::swap(V[m][i], V[k][i]);
        }
    }
}

// eigen -> back-substitution weights: 1/w for |w| above 2 eps sum(w), else 0 (SVBkSb)
template <int N>
void eig_inverse_weights(const double (&W)[N], double (&inv)[N])
{
    double thr = 0;
    for (int i = 0; i < N; i++) thr += W[i];
    thr *= DBL_EPSILON * 2;
    for (int i = 0; i < N; i++) inv[i] = std::fabs(W[i]) <= thr ? 0.0 : 1 / W[i];
}

// solve(A, b, x, DECOMP_EIG) for symmetric 8x8 A
void solve_eig8(const double (&A)[8][8], const double (&b)[8], double (&x)[8])
{
    double a[8][8], w[8], v[8][8], iw[8];
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) a[i][j] = A[i][j];
    eigen_sym<8>(a, w, v);
    eig_inverse_weights<8>(w, iw);
    for (int j = 0; j < 8; j++) x[j] = 0;
    for (int i = 0; i < 8; i++) {
        if (iw[i] == 0.0) continue;
        double s = 0;
        for (int j = 0; j < 8; j++) s += v[i][j] * b[j];
        s *= iw[i];
        for (int j = 0; j < 8; j++) x[j] = x[j] + s * v[i][j];
    }
}

// diagonal of invert(A, DECOMP_EIG) for symmetric 8x8 A
void inverse_diag_eig8(const double (&A)[8][8], double (&dg)[8])
{
    double a[8][8], w[8], v[8][8], iw[8];
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) a[i][j] = A[i][j];
    eigen_sym<8>(a, w, v);
    eig_inverse_weights<8>(w, iw);
    for (int j = 0; j < 8; j++) dg[j] = 0;
    for (int i = 0; i < 8; i++) {
        if (iw[i] == 0.0) continue;
        for (int j = 0; j < 8; j++) dg[j] = dg[j] + v[i][j] * (v[i][j] * iw[i]);
    }
}

struct Corr {
    const float *src, *dst;   // n x 2 each (Point2f, as findHomography converts them)
    int n;
};

// HomographyEstimatorCallback::runKernel; false when a coordinate spread is below DBL_EPSILON
bool dlt_normalised(const Corr &P, double *H)
{
    const int n = P.n;
    double cmx = 0, cmy = 0, cMx = 0, cMy = 0;
    for (int i = 0; i < n; i++) {
        cmx += P.dst[2 * i];
        cmy += P.dst[2 * i + 1];
        cMx += P.src[2 * i];
        cMy += P.src[2 * i + 1];
    }
    cmx /= n, cmy /= n, cMx /= n, cMy /= n;
    double smx = 0, smy = 0, sMx = 0, sMy = 0;
    for (int i = 0; i < n; i++) {
        smx += std::fabs(P.dst[2 * i] - cmx);
        smy += std::fabs(P.dst[2 * i + 1] - cmy);
        sMx += std::fabs(P.src[2 * i] - cMx);
        sMy += std::fabs(P.src[2 * i + 1] - cMy);
    }
    if (std::fabs(smx) < DBL_EPSILON || std::fabs(smy) < DBL_EPSILON ||
        std::fabs(sMx) < DBL_EPSILON || std::fabs(sMy) < DBL_EPSILON)
        return false;
    smx = n / smx, smy = n / smy, sMx = n / sMx, sMy = n / sMy;
    double L[9][9] = {};
    for (int i = 0; i < n; i++) {
        const double x = (P.dst[2 * i] - cmx) * smx, y = (P.dst[2 * i + 1] - cmy) * smy;
        const double X = (P.src[2 * i] - cMx) * sMx, Y = (P.src[2 * i + 1] - cMy) * sMy;
        const double Lx[9] = {X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x};
        const double Ly[9] = {0, 0, 0, X, Y, 1, -y * X, -y * Y, -y};
        for (int j = 0; j < 9; j++)
            for (int k = j; k < 9; k++) L[j][k] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
    }
    for (int j = 0; j < 9; j++)
        for (int k = 0; k < j; k++) L[j][k] = L[k][j];
    double W[9], V[9][9];
    eigen_sym<9>(L, W, V);
    const double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
    const double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
    double T[9], R[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++)
            T[3 * r + c] = invHnorm[3 * r] * V[8][c] + invHnorm[3 * r + 1] * V[8][3 + c] +
                           invHnorm[3 * r + 2] * V[8][6 + c];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++)
            R[3 * r + c] = T[3 * r] * Hnorm2[c] + T[3 * r + 1] * Hnorm2[3 + c] +
                           T[3 * r + 2] * Hnorm2[6 + c];
    const double scale = 1. / R[8];
    for (int i = 0; i < 9; i++) H[i] = R[i] * scale;
    return true;
}

// HomographyRefineCallback::compute: r (2n) and, when J != nullptr, J (2n x 8)
void residuals(const Corr &P, const double *h, double *r, double *J)
{
    for (int i = 0; i < P.n; i++) {
        const double Mx = P.src[2 * i], My = P.src[2 * i + 1];
        double ww = h[6] * Mx + h[7] * My + 1.;
        ww = std::fabs(ww) > DBL_EPSILON ? 1. / ww : 0;
        const double xi = (h[0] * Mx + h[1] * My + h[2]) * ww;
        const double yi = (h[3] * Mx + h[4] * My + h[5]) * ww;
        r[2 * i] = xi - P.dst[2 * i];
        r[2 * i + 1] = yi - P.dst[2 * i + 1];
        if (J) {
            double *a = J + 16 * i, *b = a + 8;
            a[0] = Mx * ww, a[1] = My * ww, a[2] = ww;
            a[3] = a[4] = a[5] = 0.;
            a[6] = -Mx * ww * xi, a[7] = -My * ww * xi;
            b[0] = b[1] = b[2] = 0.;
            b[3] = Mx * ww, b[4] = My * ww, b[5] = ww;
            b[6] = -Mx * ww * yi, b[7] = -My * ww * yi;
        }
    }
}

double sum_sq(const std::vector<double> &r)
{
    double s = 0;
    for (double v : r) s += v * v;
    return s;
}

// A = Jt J, v = Jt r (rows of J in order)
void normal_eq(const std::vector<double> &J, const std::vector<double> &r, int rows,
               double (&A)[8][8], double (&v)[8])
{
    for (int i = 0; i < 8; i++) {
        for (int j = 0; j < 8; j++) {
            double s = 0;
            for (int q = 0; q < rows; q++) s += J[8 * q + i] * J[8 * q + j];
            A[i][j] = s;
        }
        double s = 0;
        for (int q = 0; q < rows; q++) s += J[8 * q + i] * r[q];
        v[i] = s;
    }
}

// cv::LMSolver::run(h0..h7) with HomographyRefineCallback, at most max_iters iterations
void lm_refine(const Corr &P, double *h8, int max_iters)
{
    const int rows = 2 * P.n;
    std::vector<double> x(h8, h8 + 8), xd(8), r(rows), rd(rows), J((size_t)rows * 8);
    residuals(P, x.data(), r.data(), J.data());
    double S = sum_sq(r);
    double A[8][8], v[8], D[8];
    normal_eq(J, r, rows, A, v);
    for (int i = 0; i < 8; i++) D[i] = A[i][i];
    const double Rlo = 0.25, Rhi = 0.75;
    double lambda = 1, lc = 0.75;
    for (int iter = 0;;) {
        double Ap[8][8], d[8];
        for (int i = 0; i < 8; i++)
            for (int j = 0; j < 8; j++) Ap[i][j] = A[i][j];
        for (int i = 0; i < 8; i++) Ap[i][i] += lambda * D[i];
        solve_eig8(Ap, v, d);
        for (int i = 0; i < 8; i++) xd[i] = x[i] - d[i];
        residuals(P, xd.data(), rd.data(), nullptr);
        const double Sd = sum_sq(rd);
        double dS = 0;
        for (int i = 0; i < 8; i++) {
            double Ad = 0;
            for (int j = 0; j < 8; j++) Ad += A[i][j] * d[j];
            dS += d[i] * (-Ad + 2 * v[i]);
        }
        const double R = (S - Sd) / (std::fabs(dS) > DBL_EPSILON ? dS : 1);
        if (R > Rhi) {
            lambda *= 0.5;
            if (lambda < lc) lambda = 0;
        } else if (R < Rlo) {
            double t = 0;
            for (int i = 0; i < 8; i++) t += d[i] * v[i];
            double nu = (Sd - S) / (std::fabs(t) > DBL_EPSILON ? t : 1) + 2;
            nu = std::min(std::max(nu, 2.), 10.);
            if (lambda == 0) {
                double dg[8];
                inverse_diag_eig8(A, dg);
                double maxval = DBL_EPSILON;
                for (int i = 0; i < 8; i++) maxval = std::max(maxval, std::fabs(dg[i]));
                lambda = lc = 1. / maxval;
                nu *= 0.5;
            }
            lambda *= nu;
        }
        if (Sd < S) {
            S = Sd;
            std::swap(x, xd);
            residuals(P, x.data(), r.data(), J.data());
            normal_eq(J, r, rows, A, v);
        }
        iter++;
        double dmax = 0, rmax = 0;
        for (int i = 0; i < 8; i++) dmax = std::max(dmax, std::fabs(d[i]));
        for (double e : r) rmax = std::max(rmax, std::fabs(e));
        if (!(iter < max_iters && dmax >= FLT_EPSILON && rmax >= FLT_EPSILON)) break;
    }
    for (int i = 0; i < 8; i++) h8[i] = x[i];
}

}  // namespace

namespace mcs {

void homography_refine(const float *src_xy, const float *dst_xy, int n, const uint8_t *mask,
                       double *H)
{
    // findHomography refines only when RANSAC found a model and had more than 4 points
    if (n <= 4) return;
    std::vector<float> s, d;
    for (int i = 0; i < n; i++)
        if (mask[i]) {
            s.push_back(src_xy[2 * i]), s.push_back(src_xy[2 * i + 1]);
            d.push_back(dst_xy[2 * i]), d.push_back(dst_xy[2 * i + 1]);
        }
    const Corr P{s.data(), d.data(), (int)(s.size() / 2)};
    if (P.n == 0) return;
    double Hk[9];
    if (dlt_normalised(P, Hk))
        for (int i = 0; i < 9; i++) H[i] = Hk[i];
    lm_refine(P, H, 10);
}

}  // namespace mcs

extern "C" int mcs_homography_refine_host(const float *src_xy, const float *dst_xy, int n,
                                          const uint8_t *mask, double *H)
{
    mcs::clear_error();
    if (!src_xy || !dst_xy || !mask || !H || n < 0)
        return mcs::fail(MCS_E_INVALID, "NULL buffer / n=%d", n);
    mcs::homography_refine(src_xy, dst_xy, n, mask, H);
    return MCS_OK;
}

// mcs_features.cpp -- C ABI of the per-frame estimation path (include/mcs.h, "Matching"):
// brute-force Hamming kNN-2 on the GPU.
#include <algorithm>
#include <cstdio>
#include <mutex>

#include <vector>

#include "mcs_common.h"
#include "mcs_fparams.h"
#include "mcs_ransac_core.h"

namespace {

using mcs::DeviceGuard;
using mcs::rt::Api;

struct FeatureKernels {
    bool loaded = false;
    hipFunction_t knn2 = nullptr, knn2_finalize = nullptr;
    hipFunction_t ransac_score = nullptr, ransac_mask = nullptr;
};
FeatureKernels g_fk[mcs::kMaxDevices];
std::mutex g_fk_mu;

int feature_kernels(const Api *A, int device, const FeatureKernels **out)
{
    if (device < 0 || device >= mcs::kMaxDevices) return mcs::fail(MCS_E_INVALID, "device %d", device);
    std::lock_guard<std::mutex> lk(g_fk_mu);
    FeatureKernels &k = g_fk[device];
    if (!k.loaded) {
        int rc = mcs::module_function(A, device, mcs::kModFeatures, "mcs_hamming_knn2", &k.knn2);
        if (rc == MCS_OK)
            rc = mcs::module_function(A, device, mcs::kModFeatures, "mcs_hamming_knn2_finalize",
                                      &k.knn2_finalize);
        if (rc == MCS_OK)
            rc = mcs::module_function(A, device, mcs::kModFeatures, "mcs_ransac_score",
                                      &k.ransac_score);
        if (rc == MCS_OK)
            rc = mcs::module_function(A, device, mcs::kModFeatures, "mcs_ransac_mask",
                                      &k.ransac_mask);
        if (rc) return rc;
        k.loaded = true;
    }
    *out = &k;
    return MCS_OK;
}

int launch(const Api *A, hipFunction_t f, unsigned gx, unsigned gy, unsigned bx, void *args,
           size_t sz, hipStream_t s)
{
    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                   HIP_LAUNCH_PARAM_END};
    HIP_TRY(A->hipModuleLaunchKernel(f, gx, gy, 1, bx, 1, 1, 0, s, nullptr, cfg));
    return MCS_OK;
}

int knn2(const Api *A, const FeatureKernels *k, const uint8_t *q, int nq, const uint8_t *t, int nt,
         int32_t *idx2, int32_t *dist2, hipStream_t s)
{
    HIP_TRY(A->hipMemsetAsync(idx2, 0xff, (size_t)nq * 2 * sizeof(int32_t), s));
    mcs::KHammingArgs a;
    a.query = reinterpret_cast<const uint32_t *>(q);
    a.train = reinterpret_cast<const uint32_t *>(t);
    a.keys = reinterpret_cast<uint32_t *>(idx2);
    a.dist = dist2;
    a.nq = nq;
    a.nt = nt;
    a.pad_ = 0;
    // enough (query wave x train chunk) blocks to fill the chip, chunks of >= 256 descriptors
    const int qblocks = (nq + mcs::kKnnQueriesPerBlock - 1) / mcs::kKnnQueriesPerBlock;
    int chunks = (4096 + qblocks - 1) / qblocks;
    chunks = std::max(1, std::min(chunks, (nt + 255) / 256));
    a.per_chunk = (nt + chunks - 1) / chunks;
    chunks = nt > 0 ? (nt + a.per_chunk - 1) / a.per_chunk : 0;
    int rc = MCS_OK;
    if (chunks > 0)
        rc = launch(A, k->knn2, qblocks, chunks, mcs::kKnnQueriesPerBlock, &a, sizeof(a), s);
    if (rc == MCS_OK)
        rc = launch(A, k->knn2_finalize, (2 * nq + 255) / 256, 1, 256, &a, sizeof(a), s);
    return rc;
}

int check_sizes(int nq, int nt)
{
    if (nq < 0 || nt < 0 || nt >= mcs::kKnnMaxTrain || nq > (1 << 26))
        return mcs::fail(MCS_E_INVALID, "n_query=%d n_train=%d (train < %d)", nq, nt,
                         mcs::kKnnMaxTrain);
    return MCS_OK;
}

}  // namespace

extern "C" {

int mcs_match_hamming_knn2(const uint8_t *d_query, int n_query, const uint8_t *d_train,
                           int n_train, int32_t *d_idx2, int32_t *d_dist2, int device,
                           void *stream)
{
    mcs::clear_error();
    int rc = check_sizes(n_query, n_train);
    if (rc) return rc;
    if (n_query == 0) return MCS_OK;
    if (!d_query || (!d_train && n_train) || !d_idx2 || !d_dist2)
        return mcs::fail(MCS_E_INVALID, "NULL buffer");
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    DeviceGuard g(A, device);
    if (g.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", device, A->hipGetErrorString(g.err));
    const FeatureKernels *k = nullptr;
    rc = feature_kernels(A, device, &k);
    if (rc) return rc;
    return knn2(A, k, d_query, n_query, d_train, n_train, d_idx2, d_dist2, (hipStream_t)stream);
}

int mcs_match_hamming_knn2_host(const uint8_t *query, int n_query, const uint8_t *train,
                                int n_train, int32_t *idx2, int32_t *dist2, int device)
{
    mcs::clear_error();
    int rc = check_sizes(n_query, n_train);
    if (rc) return rc;
    if (n_query == 0) return MCS_OK;
    if (!query || (!train && n_train) || !idx2 || !dist2)
        return mcs::fail(MCS_E_INVALID, "NULL buffer");
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    DeviceGuard g(A, device);
    if (g.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", device, A->hipGetErrorString(g.err));
    const FeatureKernels *k = nullptr;
    rc = feature_kernels(A, device, &k);
    if (rc) return rc;
    const size_t qb = (size_t)n_query * mcs::kDescBytes, tb = (size_t)n_train * mcs::kDescBytes;
    const size_t ob = (size_t)n_query * 2 * sizeof(int32_t);
    uint8_t *buf = nullptr;
    HIP_TRY(A->hipMalloc((void **)&buf, qb + tb + 2 * ob + 64));
    uint8_t *dq = buf, *dt = buf + qb;
    int32_t *di = reinterpret_cast<int32_t *>(buf + ((qb + tb + 15) & ~(size_t)15));
    int32_t *dd = di + (size_t)n_query * 2;
    hipStream_t s = nullptr;
    hipError_t e = A->hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = A->hipMemcpyAsync(dq, query, qb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && tb) e = A->hipMemcpyAsync(dt, train, tb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) rc = knn2(A, k, dq, n_query, dt, n_train, di, dd, s);
    if (e == hipSuccess && rc == MCS_OK)
        e = A->hipMemcpyAsync(idx2, di, ob, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && rc == MCS_OK)
        e = A->hipMemcpyAsync(dist2, dd, ob, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && s) e = A->hipStreamSynchronize(s);
    if (s) (void)A->hipStreamDestroy(s);
    (void)A->hipFree(buf);
    if (e != hipSuccess) return mcs::fail(MCS_E_HIP, "knn2 host path: %s", A->hipGetErrorString(e));
    return rc;
}

int mcs_ransac_homography_host(const float *src_xy, const float *dst_xy, int n, double thresh,
                               int iters, uint32_t seed, double *H, uint8_t *mask,
                               int *n_inliers, int device)
{
    mcs::clear_error();
    if (!src_xy || !dst_xy || !H || !n_inliers) return mcs::fail(MCS_E_INVALID, "NULL buffer");
    if (n < 0 || iters <= 0 || iters > (1 << 20) || !(thresh >= 0.0))
        return mcs::fail(MCS_E_INVALID, "n=%d iters=%d thresh=%g", n, iters, thresh);
    *n_inliers = 0;
    for (int i = 0; i < 9; i++) H[i] = 0.0;
    if (mask)
        for (int i = 0; i < n; i++) mask[i] = 0;
    if (n < 4) return MCS_OK;   // no model (the reference needs > 4 matches to try)
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    DeviceGuard g(A, device);
    if (g.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", device, A->hipGetErrorString(g.err));
    const FeatureKernels *k = nullptr;
    int rc = feature_kernels(A, device, &k);
    if (rc) return rc;
    std::vector<double> pts((size_t)n * 4);
    for (int i = 0; i < n; i++) {
        pts[4 * i] = src_xy[2 * i], pts[4 * i + 1] = src_xy[2 * i + 1];
        pts[4 * i + 2] = dst_xy[2 * i], pts[4 * i + 3] = dst_xy[2 * i + 1];
    }
    const size_t pb = pts.size() * sizeof(double), hb = (size_t)iters * 8 * sizeof(double);
    const size_t sb = (size_t)iters * sizeof(int32_t);
    uint8_t *buf = nullptr;
    HIP_TRY(A->hipMalloc((void **)&buf, pb + hb + sb + (size_t)n + 64));
    mcs::KRansacArgs a;
    a.pts = reinterpret_cast<double *>(buf);
    a.hyps = reinterpret_cast<double *>(buf + pb);
    a.scores = reinterpret_cast<int32_t *>(buf + pb + hb);
    a.mask = buf + pb + hb + sb;
    a.t2 = thresh * thresh;
    a.n = n;
    a.iters = iters;
    a.best = 0;
    a.seed = seed;
    std::vector<int32_t> scores((size_t)iters);
    std::vector<uint8_t> m8((size_t)n);
    double hb8[8];
    hipStream_t s = nullptr;
    hipError_t e = A->hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = A->hipMemcpyAsync((void *)a.pts, pts.data(), pb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) rc = launch(A, k->ransac_score, iters, 1, mcs::kRansacBlock, &a, sizeof(a), s);
    if (e == hipSuccess && rc == MCS_OK)
        e = A->hipMemcpyAsync(scores.data(), a.scores, sb, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && rc == MCS_OK) e = A->hipStreamSynchronize(s);
    int best = -1, best_score = -1;
    if (e == hipSuccess && rc == MCS_OK) {
        for (int i = 0; i < iters; i++)
            if (scores[i] > best_score) best_score = scores[i], best = i;
        if (best_score >= 4) {
            a.best = best;
            rc = launch(A, k->ransac_mask, (n + 255) / 256, 1, 256, &a, sizeof(a), s);
            if (rc == MCS_OK)
                e = A->hipMemcpyAsync(m8.data(), a.mask, (size_t)n, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess && rc == MCS_OK)
                e = A->hipMemcpyAsync(hb8, a.hyps + (size_t)best * 8, sizeof(hb8),
                                      hipMemcpyDeviceToHost, s);
            if (e == hipSuccess && rc == MCS_OK) e = A->hipStreamSynchronize(s);
        }
    }
    if (s) (void)A->hipStreamDestroy(s);
    (void)A->hipFree(buf);
    if (e != hipSuccess) return mcs::fail(MCS_E_HIP, "ransac: %s", A->hipGetErrorString(e));
    if (rc) return rc;
    if (best_score < 4) return MCS_OK;
    // least-squares refit over the best hypothesis' inliers (8x8 normal equations, point order)
    double M[8][9] = {};
    for (int i = 0; i < n; i++) {
        if (!m8[i]) continue;
        double ru[9], rv[9];
        mcs::rs_rows(pts[4 * i], pts[4 * i + 1], pts[4 * i + 2], pts[4 * i + 3], ru, rv);
        for (const double *r : {ru, rv})
            for (int p = 0; p < 8; p++)
                for (int q = 0; q < 9; q++) M[p][q] = M[p][q] + r[p] * r[q];
    }
    double hr[8];
    const bool ok = mcs::rs_solve8(M, hr);
    for (int i = 0; i < 8; i++) H[i] = ok ? hr[i] : hb8[i];
    H[8] = 1.0;
    *n_inliers = best_score;
    if (mask)
        for (int i = 0; i < n; i++) mask[i] = m8[i];
    return MCS_OK;
}

}  // extern "C"

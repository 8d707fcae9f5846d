// mcs_features.cpp -- C ABI of the per-frame estimation path (include/mcs.h, "Matching"):
// brute-force Hamming kNN-2 on the GPU.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>

#include <vector>

#include "mcs_common.h"
#include "mcs_feat_int.h"
#include "mcs_fparams.h"
#include "mcs_orb_core.h"
#include "mcs_ransac_core.h"

namespace {

using mcs::DeviceGuard;
using mcs::rt::Api;
using mcs::feat::FeatureKernels;
using mcs::feat::feature_kernels;
using mcs::feat::launch;

FeatureKernels g_fk[mcs::kMaxDevices];
std::mutex g_fk_mu;

// Scratch buffer + stream of the synchronous per-frame entry points (ORB, Hamming kNN-2, RANSAC:
// called for every rig capture in the C3 estimation loop), one per thread and device: grown on
// demand, reused across calls, kept for the thread's lifetime (no per-call hipMalloc / stream
// creation; released with the process).  The entry points are synchronous, so a thread never has
// two calls in flight on its workspace.
struct Workspace {
    uint8_t *buf = nullptr;
    size_t cap = 0;
    hipStream_t s = nullptr;
    hipEvent_t ev = nullptr;   // blocking-sync event: ws_sync's wait point
};
thread_local Workspace tl_ws[mcs::kMaxDevices];

// Waits for the work queued on workspace stream `s`: hipStreamSynchronize, or with
// MCS_FEATURE_SYNC=block through an event created with hipEventBlockingSync (the thread sleeps
// instead of spinning; measured slower for the C3 loop on the 16-CPU box, so not the default).
hipError_t ws_sync(const Api *A, hipStream_t s)
{
    static const bool spin =
        !getenv("MCS_FEATURE_SYNC") || strcmp(getenv("MCS_FEATURE_SYNC"), "block");
    if (!spin)
        for (Workspace &w : tl_ws)
            if (w.s == s) {
                if (!w.ev) {
                    // hipEventBlockingSync | hipEventDisableTiming
                    hipError_t e = A->hipEventCreateWithFlags(&w.ev, 0x1u | 0x2u);
                    if (e != hipSuccess) return e;
                }
                hipError_t e = A->hipEventRecord(w.ev, s);
                return e == hipSuccess ? A->hipEventSynchronize(w.ev) : e;
            }
    return A->hipStreamSynchronize(s);
}

int workspace(const Api *A, int device, size_t bytes, uint8_t **buf, hipStream_t *s)
{
    if (device < 0 || device >= mcs::kMaxDevices)
        return mcs::fail(MCS_E_INVALID, "device %d", device);
    Workspace &w = tl_ws[device];
    if (!w.s) HIP_TRY(A->hipStreamCreateWithFlags(&w.s, hipStreamNonBlocking));
    if (w.cap < bytes) {
        if (w.buf) HIP_TRY(A->hipFree(w.buf));
        w.buf = nullptr;
        w.cap = 0;
        const size_t want = std::max(bytes, (size_t)1 << 20);
        HIP_TRY(A->hipMalloc((void **)&w.buf, want));
        w.cap = want;
    }
    *buf = w.buf;
    *s = w.s;
    return MCS_OK;
}

}  // namespace

int mcs::features_stream_wait(int device, void *event)
{
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    DeviceGuard g(A, device);
    if (g.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", device, A->hipGetErrorString(g.err));
    uint8_t *buf = nullptr;
    hipStream_t s = nullptr;
    int rc = workspace(A, device, 0, &buf, &s);
    if (rc) return rc;
    HIP_TRY(A->hipStreamWaitEvent(s, (hipEvent_t)event, 0));
    return MCS_OK;
}

int mcs::feat::feature_kernels(const Api *A, int device, const FeatureKernels **out)
{
    if (device < 0 || device >= mcs::kMaxDevices)
        return mcs::fail(MCS_E_INVALID, "device %d", device);
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
        const struct {
            const char *name;
            hipFunction_t *f;
        } orb[] = {{"mcs_orb_gray", &k.orb_gray},     {"mcs_orb_level", &k.orb_level},
                   {"mcs_orb_pyramid", &k.orb_pyramid},
                   {"mcs_orb_describe", &k.orb_describe},
                   {"mcs_orb_select", &k.orb_select},
                   {"mcs_l2_prep", &k.l2_prep},       {"mcs_l2_knn2_i8", &k.l2_i8},
                   {"mcs_l2_knn2_f32", &k.l2_f32},    {"mcs_l2_knn2_finalize", &k.l2_finalize},
                   {"mcs_rig_knn2", &k.rig_knn2},     {"mcs_rig_match", &k.rig_match},
                   {"mcs_rig_ransac", &k.rig_ransac}, {"mcs_rig_best", &k.rig_best},
                   {"mcs_rig_hyp", &k.rig_hyp},
                   {"mcs_seam_flow_init", &k.seam_init}, {"mcs_seam_flow_hinit", &k.seam_hinit},
                   {"mcs_seam_flow_relabel", &k.seam_relabel},
                   {"mcs_seam_flow_push", &k.seam_push},
                   {"mcs_seam_flow_active", &k.seam_active},
                   {"mcs_seam_flow_label", &k.seam_label},
                   {"mcs_seam_flow_relabel_lds", &k.seam_relabel_lds}};
        for (const auto &o : orb)
            if (rc == MCS_OK) rc = mcs::module_function(A, device, mcs::kModFeatures, o.name, o.f);
        if (rc) return rc;
        k.loaded = true;
    }
    *out = &k;
    return MCS_OK;
}

int mcs::feat::launch(const Api *A, hipFunction_t f, unsigned gx, unsigned gy, unsigned bx,
                      void *args, size_t sz, hipStream_t s, unsigned gz, unsigned lds)
{
    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                   HIP_LAUNCH_PARAM_END};
    HIP_TRY(A->hipModuleLaunchKernel(f, gx, gy, gz, bx, 1, 1, lds, s, nullptr, cfg));
    return MCS_OK;
}

namespace {

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
    // enough (query wave x train chunk) blocks to fill the chip twice over (16384 waves: 16 per
    // SIMD, the compare loop's LDS-read latency needs them; 4096 left waves waiting on it half
    // their cycles) with chunks of >= 64 descriptors (3 atomics per query and chunk)
    const int qblocks = (nq + mcs::kKnnQueriesPerBlock - 1) / mcs::kKnnQueriesPerBlock;
    int chunks = (mcs::kKnnTargetBlocks + qblocks - 1) / qblocks;
    chunks = std::max(1, std::min(chunks, (nt + 63) / 64));
    a.per_chunk = (nt + chunks - 1) / chunks;
    chunks = nt > 0 ? (nt + a.per_chunk - 1) / a.per_chunk : 0;
    int rc = MCS_OK;
    if (chunks > 0)
        rc = launch(A, k->knn2, qblocks, chunks, mcs::kKnnLanes, &a, sizeof(a), s);
    if (rc == MCS_OK)
        rc = launch(A, k->knn2_finalize, (2 * nq + 255) / 256, 1, 256, &a, sizeof(a), s);
    return rc;
}

// L2 kNN-2 on device buffers (float descriptors); scratch allocated here; synchronises.
int l2_knn2(const Api *A, const FeatureKernels *k, const float *dq, int nq, const float *dt, int nt,
            int dim, int32_t *idx2, float *dist2, int *exact, hipStream_t s)
{
    const int dimp = (dim + 63) / 64 * 64;
    const size_t n = (size_t)nq + nt;
    const size_t b8 = n * dimp, bi = n * 4, bk = (size_t)nq * 2 * 8;
    uint8_t *buf = nullptr;
    HIP_TRY(A->hipMalloc((void **)&buf, b8 + 5 * bi + bk + 256));
    int8_t *d8 = reinterpret_cast<int8_t *>(buf);
    uint8_t *p = buf + ((b8 + 15) & ~(size_t)15);
    int32_t *norm_i = reinterpret_cast<int32_t *>(p);
    int32_t *sum_i = norm_i + n;
    float *norm_f = reinterpret_cast<float *>(sum_i + n);
    uint32_t *flag = reinterpret_cast<uint32_t *>(norm_f + n);
    unsigned long long *keys =
        reinterpret_cast<unsigned long long *>(((uintptr_t)(flag + 4) + 15) & ~(uintptr_t)15);
    int rc = MCS_OK;
    hipError_t e = A->hipMemsetAsync(flag, 0, 4, s);
    if (e == hipSuccess) e = A->hipMemsetAsync(keys, 0xff, bk, s);
    for (int side = 0; side < 2 && e == hipSuccess && rc == MCS_OK; side++) {
        mcs::KL2PrepArgs pa;
        pa.desc = side ? dt : dq;
        pa.n = side ? nt : nq;
        const size_t o = side ? (size_t)nq : 0;
        pa.i8 = d8 + o * dimp;
        pa.norm_i = norm_i + o;
        pa.sum_i = sum_i + o;
        pa.norm_f = norm_f + o;
        pa.flag = flag;
        pa.dim = dim;
        pa.dimp = dimp;
        pa.pad_ = 0;
        if (pa.n > 0) rc = launch(A, k->l2_prep, (pa.n + 3) / 4, 1, 256, &pa, sizeof(pa), s);
    }
    mcs::KL2Args a;
    a.q8 = d8;
    a.t8 = d8 + (size_t)nq * dimp;
    a.qf = dq;
    a.tf = dt;
    a.qn = norm_i, a.tn = norm_i + nq, a.qs = sum_i, a.ts = sum_i + nq;
    a.qnf = norm_f, a.tnf = norm_f + nq;
    a.flag = flag;
    a.keys = keys;
    a.idx = idx2;
    a.dist = dist2;
    a.nq = nq, a.nt = nt, a.dim = dim, a.dimp = dimp, a.pad_ = 0;
    const int qblocks = (nq + mcs::kL2QueriesPerBlock - 1) / mcs::kL2QueriesPerBlock;
    int chunks = (2048 + qblocks - 1) / qblocks;
    chunks = std::max(1, std::min(chunks, (nt + 255) / 256));
    a.per_chunk = ((nt + chunks - 1) / chunks + 15) / 16 * 16;
    chunks = nt > 0 ? (nt + a.per_chunk - 1) / a.per_chunk : 0;
    if (e == hipSuccess && rc == MCS_OK && chunks > 0) {
        rc = launch(A, k->l2_i8, qblocks, chunks, 256, &a, sizeof(a), s);
        if (rc == MCS_OK) rc = launch(A, k->l2_f32, qblocks, chunks, 256, &a, sizeof(a), s);
    }
    if (e == hipSuccess && rc == MCS_OK)
        rc = launch(A, k->l2_finalize, (2 * nq + 255) / 256, 1, 256, &a, sizeof(a), s);
    uint32_t hflag = 0;
    if (e == hipSuccess && rc == MCS_OK)
        e = A->hipMemcpyAsync(&hflag, flag, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = ws_sync(A, s);
    (void)A->hipFree(buf);
    if (rc) return rc;
    if (e != hipSuccess) return mcs::fail(MCS_E_HIP, "l2 knn2: %s", A->hipGetErrorString(e));
    if (exact) *exact = hflag ? 0 : 1;
    return MCS_OK;
}

int check_l2(int nq, int nt, int dim)
{
    if (nq < 0 || nt < 0 || nq > (1 << 26) || nt > (1 << 30) || dim < 1 || dim > mcs::kL2MaxDim)
        return mcs::fail(MCS_E_INVALID, "n_query=%d n_train=%d dim=%d (1..%d)", nq, nt, dim,
                         mcs::kL2MaxDim);
    return MCS_OK;
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
    hipStream_t s = nullptr;
    rc = workspace(A, device, qb + tb + 2 * ob + 64, &buf, &s);
    if (rc) return rc;
    uint8_t *dq = buf, *dt = buf + qb;
    int32_t *di = reinterpret_cast<int32_t *>(buf + ((qb + tb + 15) & ~(size_t)15));
    int32_t *dd = di + (size_t)n_query * 2;
    hipError_t e = A->hipMemcpyAsync(dq, query, qb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && tb) e = A->hipMemcpyAsync(dt, train, tb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) rc = knn2(A, k, dq, n_query, dt, n_train, di, dd, s);
    if (e == hipSuccess && rc == MCS_OK)
        e = A->hipMemcpyAsync(idx2, di, ob, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && rc == MCS_OK)
        e = A->hipMemcpyAsync(dist2, dd, ob, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = ws_sync(A, s);
    if (e != hipSuccess) return mcs::fail(MCS_E_HIP, "knn2 host path: %s", A->hipGetErrorString(e));
    return rc;
}

int mcs_match_l2_knn2(const float *d_query, int n_query, const float *d_train, int n_train,
                      int dim, int32_t *d_idx2, float *d_dist2, int *exact, int device,
                      void *stream)
{
    mcs::clear_error();
    int rc = check_l2(n_query, n_train, dim);
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
    return l2_knn2(A, k, d_query, n_query, d_train, n_train, dim, d_idx2, d_dist2, exact,
                   (hipStream_t)stream);
}

int mcs_match_l2_knn2_host(const float *query, int n_query, const float *train, int n_train,
                           int dim, int32_t *idx2, float *dist2, int *exact, int device)
{
    mcs::clear_error();
    int rc = check_l2(n_query, n_train, dim);
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
    const size_t qb = (size_t)n_query * dim * 4, tb = (size_t)n_train * dim * 4;
    const size_t ob = (size_t)n_query * 2 * 4;
    uint8_t *buf = nullptr;
    HIP_TRY(A->hipMalloc((void **)&buf, qb + tb + 2 * ob + 64));
    float *dq = reinterpret_cast<float *>(buf);
    float *dt = reinterpret_cast<float *>(buf + qb);
    int32_t *di = reinterpret_cast<int32_t *>(buf + ((qb + tb + 15) & ~(size_t)15));
    float *dd = reinterpret_cast<float *>(di + (size_t)n_query * 2);
    hipStream_t s = nullptr;
    hipError_t e = A->hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = A->hipMemcpyAsync(dq, query, qb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && tb) e = A->hipMemcpyAsync(dt, train, tb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) rc = l2_knn2(A, k, dq, n_query, dt, n_train, dim, di, dd, exact, s);
    if (e == hipSuccess && rc == MCS_OK)
        e = A->hipMemcpyAsync(idx2, di, ob, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && rc == MCS_OK)
        e = A->hipMemcpyAsync(dist2, dd, ob, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && s) e = ws_sync(A, s);
    if (s) (void)A->hipStreamDestroy(s);
    (void)A->hipFree(buf);
    if (e != hipSuccess) return mcs::fail(MCS_E_HIP, "l2 host path: %s", A->hipGetErrorString(e));
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
    hipStream_t s = nullptr;
    rc = workspace(A, device, pb + hb + sb + (size_t)n + 64, &buf, &s);
    if (rc) return rc;
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
    hipError_t e = A->hipMemcpyAsync((void *)a.pts, pts.data(), pb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
        rc = launch(A, k->ransac_score, iters, 1, mcs::kRansacBlock, &a, sizeof(a), s);
    if (e == hipSuccess && rc == MCS_OK)
        e = A->hipMemcpyAsync(scores.data(), a.scores, sb, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && rc == MCS_OK) e = ws_sync(A, s);
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
            if (e == hipSuccess && rc == MCS_OK) e = ws_sync(A, s);
        }
    }
    if (e != hipSuccess) return mcs::fail(MCS_E_HIP, "ransac: %s", A->hipGetErrorString(e));
    if (rc) return rc;
    if (best_score < 4) return MCS_OK;
    // findHomography's refinement of the chosen model on its inliers (mcs_refine.cpp:
    // normalised DLT re-estimate + Levenberg-Marquardt, StitcherClass.py:443-444)
    for (int i = 0; i < 8; i++) H[i] = hb8[i];
    H[8] = 1.0;
    mcs::homography_refine(src_xy, dst_xy, n, m8.data(), H);
    *n_inliers = best_score;
    if (mask)
        for (int i = 0; i < n; i++) mask[i] = m8[i];
    return MCS_OK;
}

}  // extern "C"

// Source index of destination index d in OpenCV's resize(INTER_LINEAR) (mcs_orb_pyramid's
// pyr_axis, the same float arithmetic).
static int pyr_src(int d, double scale, int ssize, bool is_x)
{
    float f = (float)((d + 0.5) * scale - 0.5);
    int si = (int)std::floor(f);
    if (is_x) {
        if (si < 0) si = 0;
        if (si >= ssize - 1) si = ssize - 1;
    }
    return si;
}

// mcs_orb_pyramid's arguments: last-level tiles of 32 x 16 (8 x 8 for small levels), the LDS
// buffer size from every block's dependency regions (the kernel's top-down walk, on the host).
// Returns the block count, 0 when the fused launch does not apply (a >= 2x level step, or
// regions too large for LDS).
unsigned mcs::feat::pyramid_args(const OrbGeom &g, uint8_t *lvl, KOrbBuildArgs &a)
{
    const int *lw = g.lw, *lh = g.lh, nlevels = g.nlevels;
    const size_t *off = g.off;
    std::memset(&a, 0, sizeof(a));
    const int L = nlevels - 1;
    for (int l = 1; l <= L; l++) {
        if (2 * lw[l] <= lw[l - 1] || 2 * lh[l] <= lh[l - 1]) return 0;
        a.sx[l] = 1. / ((double)lw[l] / lw[l - 1]);
        a.sy[l] = 1. / ((double)lh[l] / lh[l - 1]);
    }
    for (int l = 0; l <= L; l++) {
        a.off[l] = (int64_t)off[l];
        a.w[l] = lw[l];
        a.h[l] = lh[l];
    }
    a.lvl = lvl;
    a.nlevels = nlevels;
    a.tw = lw[L] >= 256 ? 32 : 8;
    a.th = lw[L] >= 256 ? 16 : 8;
    a.gx = (lw[L] + a.tw - 1) / a.tw;
    const int gy = (lh[L] + a.th - 1) / a.th;
    int mw = 1, mh = 1;
    for (int t = 0; t < a.gx * gy; t++) {
        int x0 = (t % a.gx) * a.tw, y0 = (t / a.gx) * a.th;
        int x1 = std::min(x0 + a.tw, lw[L]), y1 = std::min(y0 + a.th, lh[L]);
        for (int l = L; l >= 2; l--) {
            const int sw = lw[l - 1], sh = lh[l - 1];
            const int nx0 = pyr_src(x0, a.sx[l], sw, true), sxl = pyr_src(x1 - 1, a.sx[l], sw, true);
            const int nx1 = sxl >= sw - 1 ? sw : sxl + 2;
            const int ny0 = std::min(std::max(pyr_src(y0, a.sy[l], sh, false), 0), sh - 1);
            const int ny1 = std::min(std::max(pyr_src(y1 - 1, a.sy[l], sh, false) + 1, 0), sh - 1) + 1;
            x0 = nx0, x1 = nx1, y0 = ny0, y1 = ny1;
            if (l - 1 >= 1 && l - 1 < L) mw = std::max(mw, x1 - x0), mh = std::max(mh, y1 - y0);
        }
    }
    a.lds_w = mw;
    a.lds_h = mh;
    if (2 * (size_t)mw * mh + 16 > 64 * 1024) return 0;   // (+16: mcs_orb_pyramid reads 8 bytes past a row)
    return (unsigned)(a.gx * gy);
}

int mcs::feat::orb_geom(int w, int h, int nfeatures, int nlevels, float scale_factor,
                        OrbGeom *g)
{
    g->nlevels = nlevels;
    for (int l = 0; l < nlevels; l++) {
        g->lscale[l] = (float)std::pow((double)scale_factor, (double)l);
        g->lw[l] = (int)std::lrint((float)w / g->lscale[l]);
        g->lh[l] = (int)std::lrint((float)h / g->lscale[l]);
        if (g->lw[l] < 1 || g->lh[l] < 1) return mcs::fail(MCS_E_INVALID, "level %d is empty", l);
        g->off[l + 1] = g->off[l] + (((size_t)g->lw[l] * g->lh[l] + 255) & ~(size_t)255);
    }
    const float factor = (float)(1.0 / scale_factor);
    float per = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; l++) {
        g->quota[l] = (int)std::lrint(per);
        sum += g->quota[l];
        per *= factor;
    }
    g->quota[nlevels - 1] = std::max(nfeatures - sum, 0);
    g->n_bound = 0;
    g->cap_total = 0;
    for (int l = 0; l < nlevels; l++) {
        g->n_bound += g->quota[l];
        g->cap[l] = std::max((size_t)4096, (size_t)g->lw[l] * g->lh[l] / 8);
        g->coff[l + 1] = g->coff[l] + g->cap[l];
        g->cap_total += g->cap[l];
    }
    return MCS_OK;
}

namespace {
// ORB of one image (host memory, or device memory when on_device); mcs_orb_detect_host /
// mcs_orb_detect_device below.
int orb_detect(const uint8_t *image, bool on_device, int w, int h, int channels, int nfeatures,
               int nlevels, float scale_factor, int fast_threshold, float *kp_xy,
               float *kp_response, float *kp_angle, int *kp_level, uint8_t *desc, int *n_out,
               int device)
{
    mcs::clear_error();
    if (!image || !kp_xy || !desc || !n_out) return mcs::fail(MCS_E_INVALID, "NULL buffer");
    // (w, h < 2^16: the device ranking packs a keypoint's position as y << 16 | x)
    if (w <= 0 || h <= 0 || w > 65535 || h > 65535 || (channels != 1 && channels != 3) ||
        nfeatures < 0 ||
        nlevels < 1 || nlevels > mcs::kOrbMaxLevels || !(scale_factor > 1.0f) ||
        fast_threshold < 0 || fast_threshold > 255)
        return mcs::fail(MCS_E_INVALID, "w=%d h=%d channels=%d nfeatures=%d nlevels=%d "
                         "scale=%g threshold=%d", w, h, channels, nfeatures, nlevels,
                         (double)scale_factor, fast_threshold);
    *n_out = 0;
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    DeviceGuard g(A, device);
    if (g.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", device, A->hipGetErrorString(g.err));
    const FeatureKernels *k = nullptr;
    int rc = feature_kernels(A, device, &k);
    if (rc) return rc;
    // level sizes and quotas, as OpenCV's ORB computes them (float arithmetic)
    mcs::feat::OrbGeom geo;
    rc = mcs::feat::orb_geom(w, h, nfeatures, nlevels, scale_factor, &geo);
    if (rc) return rc;
    const int *lw = geo.lw, *lh = geo.lh, *quota = geo.quota;
    const float *lscale = geo.lscale;
    const size_t *off = geo.off, *cap = geo.cap, *coff = geo.coff;
    const size_t pix = off[nlevels], cap_total = geo.cap_total;
    // one allocation: input, levels, blur (u16 pass + u8), scores, candidates, counts, keypoints,
    // descriptors, orientations
    const size_t in_bytes = (size_t)w * h * channels;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += (bytes + 255) & ~(size_t)255;
        return at;
    };
    const size_t o_in = take(in_bytes), o_lvl = take(pix), o_blur = take(pix);
    const size_t o_cand = take(cap_total * sizeof(mcs::OrbCand));
    const size_t o_cnt = take(mcs::kOrbMaxLevels * sizeof(int));
    const size_t o_kp = take((size_t)std::max(nfeatures, 1) * 3 * sizeof(int));
    const size_t o_desc = take((size_t)std::max(nfeatures, 1) * 32);
    const size_t o_or = take((size_t)std::max(nfeatures, 1) * 2 * sizeof(double));
    const size_t o_resp = take((size_t)std::max(nfeatures, 1) * sizeof(double));
    const size_t o_sel = take(2 * sizeof(int));
    const size_t o_end = o;   // [o_cnt, o_end): everything the device ranking path copies back
    uint8_t *buf = nullptr;
    hipStream_t s = nullptr;
    rc = workspace(A, device, o, &buf, &s);
    if (rc) return rc;
    std::vector<int> counts(nlevels);
    // host copy of the candidates: per thread, grown on demand, never cleared (only the
    // entries the counts cover are copied and read)
    static thread_local std::vector<mcs::OrbCand> cand;
    if (cand.size() < cap_total) cand.resize(cap_total);
    std::vector<int> kp;
    std::vector<double> orient, resp;
    uint8_t *lvl0 = buf + o_lvl;
    // the frame: uploaded into the workspace, or read where it lies on the device
    const uint8_t *in = on_device ? image : buf + o_in;
    hipError_t e = on_device ? hipSuccess
                             : A->hipMemcpyAsync(buf + o_in, image, in_bytes, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = A->hipMemsetAsync(buf + o_cnt, 0, mcs::kOrbMaxLevels * sizeof(int), s);
    if (e == hipSuccess) {
        if (channels == 3) {
            mcs::KGrayArgs ga;
            std::memset(&ga, 0, sizeof(ga));
            ga.bgr[0] = in;
            ga.gray = lvl0;
            ga.n = w * h;
            rc = launch(A, k->orb_gray, (w * h + 1023) / 1024, 1, 256, &ga, sizeof(ga), s);
        } else {
            e = A->hipMemcpyAsync(lvl0, in, in_bytes, hipMemcpyDeviceToDevice, s);
        }
    }
    // levels 1 .. nlevels-1: one launch (mcs_orb_pyramid) when every level is a < 2x
    // downscale of the one before (its blocks' dependency regions then tile every level), else
    // one resize launch per level
    mcs::KOrbBuildArgs ba;
    const unsigned pyr_blocks = e == hipSuccess && rc == MCS_OK && nlevels > 1
                                    ? mcs::feat::pyramid_args(geo, buf + o_lvl, ba)
                                    : 0u;
    if (pyr_blocks > 0) {
        size_t sz = sizeof(ba);
        void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &ba, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                       HIP_LAUNCH_PARAM_END};
        e = A->hipModuleLaunchKernel(k->orb_pyramid, pyr_blocks, 1, 1, 256, 1, 1,
                                     (unsigned)(2 * ba.lds_w * ba.lds_h + 16), s, nullptr, cfg);
    } else {
        for (int l = 1; l < nlevels && e == hipSuccess && rc == MCS_OK; l++)
            rc = mcs_resize_linear_device(buf + o_lvl + off[l - 1], lw[l - 1], lh[l - 1],
                                          lw[l - 1], 0, buf + o_lvl + off[l], lw[l], lh[l], lw[l],
                                          0, 1, 1, device, s);
    }
    if (e == hipSuccess && rc == MCS_OK) {
        // blur, FAST, NMS and Harris of every level: one launch (mcs_orb_level, kOrbTileW x kOrbTileH tiles)
        mcs::KOrbPyrArgs pa;
        std::memset(&pa, 0, sizeof(pa));
        pa.img = buf + o_lvl;
        pa.blur = buf + o_blur;
        pa.cand = reinterpret_cast<mcs::OrbCand *>(buf + o_cand);
        pa.ncand = reinterpret_cast<int *>(buf + o_cnt);
        pa.nlevels = nlevels;
        pa.threshold = fast_threshold;
        for (int l = 0; l < nlevels; l++) {
            pa.off[l] = (int64_t)off[l];
            pa.coff[l] = (int)coff[l];
            pa.w[l] = lw[l];
            pa.h[l] = lh[l];
            pa.cap[l] = (int)cap[l];
            pa.bstart[l + 1] = pa.bstart[l] + (lw[l] + mcs::kOrbTileW - 1) / mcs::kOrbTileW *
                                            ((lh[l] + mcs::kOrbTileH - 1) / mcs::kOrbTileH);
        }
        rc = launch(A, k->orb_level, (unsigned)pa.bstart[nlevels], 1, mcs::kOrbLevelThreads, &pa,
                    sizeof(pa), s);
    }
    // Device ranking (mcs_orb_select) and description, then ONE copy back of counts,
    // keypoints, descriptors, orientations and responses.  A level with more than kOrbSelMax
    // candidates sets the overflow flag instead; the host then ranks (below).
    static thread_local std::vector<uint8_t> blob;
    if (blob.size() < o_end - o_cnt) blob.resize(o_end - o_cnt);
    auto at = [&](size_t off) { return blob.data() + (off - o_cnt); };
    mcs::KOrbDescArgs da;
    std::memset(&da, 0, sizeof(da));
    for (int l = 0; l < mcs::kOrbMaxLevels; l++) {
        const int ll = l < nlevels ? l : 0;
        da.img[l] = buf + o_lvl + off[ll];
        da.blur[l] = buf + o_blur + off[ll];
        da.w[l] = lw[ll];
    }
    da.kp = reinterpret_cast<const int *>(buf + o_kp);
    da.desc = buf + o_desc;
    da.orient = reinterpret_cast<double *>(buf + o_or);
    const int n_bound = geo.n_bound;
    if (e == hipSuccess && rc == MCS_OK) {
        mcs::KOrbSelArgs sa;
        std::memset(&sa, 0, sizeof(sa));
        sa.cand = reinterpret_cast<const mcs::OrbCand *>(buf + o_cand);
        sa.ncand = reinterpret_cast<const int *>(buf + o_cnt);
        sa.kp = reinterpret_cast<int *>(buf + o_kp);
        sa.resp = reinterpret_cast<double *>(buf + o_resp);
        sa.sel = reinterpret_cast<int *>(buf + o_sel);
        for (int l = 0; l < nlevels; l++) {
            sa.coff[l] = (int)coff[l];
            sa.cap[l] = (int)cap[l];
            sa.quota[l] = quota[l];
        }
        sa.nlevels = nlevels;
        rc = launch(A, k->orb_select, (unsigned)nlevels, 1, mcs::kOrbSelThreads, &sa, sizeof(sa), s);
        da.sel = sa.sel;
        da.n = n_bound;
        if (rc == MCS_OK && n_bound > 0)
            rc = launch(A, k->orb_describe, (unsigned)n_bound, 1, 64, &da, sizeof(da), s);
    }
    if (e == hipSuccess && rc == MCS_OK)
        e = A->hipMemcpyAsync(blob.data(), buf + o_cnt, o_end - o_cnt, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && rc == MCS_OK) e = ws_sync(A, s);
    int n = 0;
    const int *sel = reinterpret_cast<const int *>(at(o_sel));
    const int *kpd = reinterpret_cast<const int *>(at(o_kp));
    const double *respd = reinterpret_cast<const double *>(at(o_resp));
    const double *ord = reinterpret_cast<const double *>(at(o_or));
    if (e == hipSuccess && rc == MCS_OK && !sel[1]) {
        n = sel[0];
        kp.assign(kpd, kpd + 3 * (size_t)n);
        resp.assign(respd, respd + n);
        orient.assign(ord, ord + 2 * (size_t)n);
        std::memcpy(desc, at(o_desc), (size_t)n * 32);
    } else if (e == hipSuccess && rc == MCS_OK) {
        // host ranking: only the candidates each level found come back
        std::memcpy(counts.data(), at(o_cnt), nlevels * sizeof(int));
        for (int l = 0; l < nlevels && e == hipSuccess; l++) {
            const int c = std::min(std::max(counts[l], 0), (int)cap[l]);
            if (c > 0)
                e = A->hipMemcpyAsync(cand.data() + coff[l],
                                      buf + o_cand + coff[l] * sizeof(mcs::OrbCand),
                                      (size_t)c * sizeof(mcs::OrbCand), hipMemcpyDeviceToHost, s);
        }
        if (e == hipSuccess) e = ws_sync(A, s);
        if (e == hipSuccess) {
            // per level: rank by response (desc), then y, then x; keep the level's quota (a
            // strict total order -- positions are unique -- so selecting the quota first and
            // sorting only it gives the full sort's prefix)
            for (int l = 0; l < nlevels; l++) {
                const int c = std::min(counts[l], (int)cap[l]);
                mcs::OrbCand *b = cand.data() + coff[l];
                auto rank = [](const mcs::OrbCand &p, const mcs::OrbCand &q) {
                    if (p.response != q.response) return p.response > q.response;
                    return p.y != q.y ? p.y < q.y : p.x < q.x;
                };
                const int keep = std::min(c, quota[l]);
                if (keep < c) std::nth_element(b, b + keep, b + c, rank);
                std::sort(b, b + keep, rank);
                for (int i = 0; i < keep; i++) {
                    kp.push_back(l);
                    kp.push_back(b[i].x);
                    kp.push_back(b[i].y);
                    resp.push_back(b[i].response);
                }
            }
            n = (int)kp.size() / 3;
            orient.resize(2 * (size_t)std::max(n, 1));
        }
        if (e == hipSuccess && n > 0) {
            e = A->hipMemcpyAsync(buf + o_kp, kp.data(), kp.size() * sizeof(int),
                                  hipMemcpyHostToDevice, s);
            da.sel = nullptr;
            da.n = n;
            if (e == hipSuccess) rc = launch(A, k->orb_describe, n, 1, 64, &da, sizeof(da), s);
            if (e == hipSuccess && rc == MCS_OK)
                e = A->hipMemcpyAsync(desc, buf + o_desc, (size_t)n * 32, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess && rc == MCS_OK)
                e = A->hipMemcpyAsync(orient.data(), buf + o_or, (size_t)n * 2 * sizeof(double),
                                      hipMemcpyDeviceToHost, s);
            if (e == hipSuccess && rc == MCS_OK) e = ws_sync(A, s);
        }
    }
    if (e == hipSuccess && rc != MCS_OK) e = ws_sync(A, s);   // drain on error
    if (e != hipSuccess) return mcs::fail(MCS_E_HIP, "orb: %s", A->hipGetErrorString(e));
    if (rc) return rc;
    for (int i = 0; i < n; i++) {
        const int l = kp[3 * i];
        kp_xy[2 * i] = (float)kp[3 * i + 1] * lscale[l];
        kp_xy[2 * i + 1] = (float)kp[3 * i + 2] * lscale[l];
        if (kp_level) kp_level[i] = l;
        if (kp_response) kp_response[i] = (float)resp[i];
        if (kp_angle) {
            double a = std::atan2(orient[2 * i + 1], orient[2 * i]) * (180.0 / M_PI);
            if (a < 0) a += 360.0;
            kp_angle[i] = (float)a;
        }
    }
    *n_out = n;
    return MCS_OK;
}
}  // namespace

extern "C" {

int mcs_orb_detect_host(const uint8_t *image, int w, int h, int channels, int nfeatures,
                        int nlevels, float scale_factor, int fast_threshold, float *kp_xy,
                        float *kp_response, float *kp_angle, int *kp_level, uint8_t *desc,
                        int *n_out, int device)
{
    return orb_detect(image, false, w, h, channels, nfeatures, nlevels, scale_factor,
                      fast_threshold, kp_xy, kp_response, kp_angle, kp_level, desc, n_out, device);
}

int mcs_orb_detect_device(const uint8_t *d_image, int w, int h, int channels, int nfeatures,
                          int nlevels, float scale_factor, int fast_threshold, float *kp_xy,
                          float *kp_response, float *kp_angle, int *kp_level, uint8_t *desc,
                          int *n_out, int device)
{
    return orb_detect(d_image, true, w, h, channels, nfeatures, nlevels, scale_factor,
                      fast_threshold, kp_xy, kp_response, kp_angle, kp_level, desc, n_out, device);
}

}  // extern "C"

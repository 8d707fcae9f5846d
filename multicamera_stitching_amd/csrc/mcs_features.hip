// mcs_features.hip -- gfx950 kernels of the per-frame homography estimation path
// (SURVEY.md section 8 NS-3..5): descriptor matching first.
//
// Brute-force Hamming kNN-2 (NS-4; BFMatcher(NORM_HAMMING).knnMatch(k=2), the reference's matcher
// at StitcherClass.py:405-448 with binary descriptors).  VALU popcount-bound: per (query, train)
// pair 8 v_xor_b32 + 8 v_bcnt_u32_b32 (accumulating) + 3 min/max for the running top-2, with
// no HBM traffic to speak of (train descriptors are wave-uniform: scalar loads, one per 32 B,
// shared by the 64 queries of a wave).
//
// Top-2 order = OpenCV's: a train descriptor enters only with a strictly smaller distance, so
// among equal distances the earlier train index wins.  Encoded as key = distance << 23 | index:
// the two smallest keys are exactly OpenCV's best and second.  The train set is split into
// chunks over grid.y; chunk results merge through two atomicMin per query:
//   old = atomicMin(best, k0); atomicMin(second, max(old, k0)); atomicMin(second, k1)
// (every key that is not the overall minimum is offered to `second` at least once, the minimum
// never is, so `second` ends as the second smallest key).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mcs_fparams.h"
#include "mcs_ransac_core.h"

namespace mcs {

constexpr uint32_t kKeyNone = 0xffffffffu;

__device__ __forceinline__ void top2(uint32_t &k0, uint32_t &k1, uint32_t k)
{
    k1 = min(k1, max(k0, k));
    k0 = min(k0, k);
}

__device__ __forceinline__ uint32_t hamming(const uint32_t (&q)[8], const uint32_t *__restrict__ t)
{
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) c += __popc(q[i] ^ t[i]);   // v_bcnt_u32_b32 accumulates
    return c;
}

}  // namespace mcs

// grid (ceil(nq / 64), chunks), block 64.  keys must hold 0xffffffff on entry (memset).
extern "C" __global__ __launch_bounds__(64) void mcs_hamming_knn2(const mcs::KHammingArgs a)
{
    using namespace mcs;
    const int q = blockIdx.x * kKnnQueriesPerBlock + threadIdx.x;
    uint32_t d[8];
    const uint4 *qs = reinterpret_cast<const uint4 *>(a.query + (int64_t)min(q, a.nq - 1) * 8);
    const uint4 v0 = qs[0], v1 = qs[1];
    d[0] = v0.x, d[1] = v0.y, d[2] = v0.z, d[3] = v0.w;
    d[4] = v1.x, d[5] = v1.y, d[6] = v1.z, d[7] = v1.w;
    const int j0 = blockIdx.y * a.per_chunk, j1 = min(a.nt, j0 + a.per_chunk);
    const uint32_t *__restrict__ train = a.train;
    uint32_t k0 = kKeyNone, k1 = kKeyNone;
    int j = j0;
    for (; j + 4 <= j1; j += 4) {
        uint32_t c[4];
#pragma unroll
        for (int u = 0; u < 4; u++) c[u] = hamming(d, train + (int64_t)(j + u) * 8);
#pragma unroll
        for (int u = 0; u < 4; u++) top2(k0, k1, (c[u] << kKnnKeyShift) | (uint32_t)(j + u));
    }
    for (; j < j1; j++) top2(k0, k1, (hamming(d, train + (int64_t)j * 8) << kKnnKeyShift) | j);
    if (q >= a.nq) return;
    const uint32_t old = atomicMin(&a.keys[2 * q], k0);
    atomicMin(&a.keys[2 * q + 1], max(old, k0));
    atomicMin(&a.keys[2 * q + 1], k1);
}

// keys -> (train index, distance) pairs; -1 where fewer than two train descriptors exist.
extern "C" __global__ __launch_bounds__(256) void mcs_hamming_knn2_finalize(
    const mcs::KHammingArgs a)
{
    using namespace mcs;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= 2 * a.nq) return;
    const uint32_t k = a.keys[i];
    const bool none = k == kKeyNone;
    a.keys[i] = none ? 0xffffffffu : (k & (kKnnMaxTrain - 1));
    a.dist[i] = none ? -1 : (int32_t)(k >> kKnnKeyShift);
}

// ---- RANSAC homography (NS-5) ------------------------------------------------------------------
// grid (iters), block kRansacBlock: thread 0 draws hypothesis k and solves its 4-point model,
// then the block counts its inliers over all n correspondences (FP64, mcs_ransac_core.h).
extern "C" __global__ __launch_bounds__(256) void mcs_ransac_score(const mcs::KRansacArgs a)
{
    using namespace mcs;
    __shared__ double h[8];
    __shared__ int valid;
    __shared__ int wsum[kRansacBlock / 64];
    const int k = blockIdx.x, tid = threadIdx.x;
    if (tid == 0) {
        int idx[4];
        double s[8], d[8], hh[8];
        bool ok = rs_subset(a.seed, (uint32_t)k, (uint32_t)a.n, idx);
        if (ok) {
            for (int m = 0; m < 4; m++) {
                s[2 * m] = a.pts[4 * idx[m]], s[2 * m + 1] = a.pts[4 * idx[m] + 1];
                d[2 * m] = a.pts[4 * idx[m] + 2], d[2 * m + 1] = a.pts[4 * idx[m] + 3];
            }
            ok = rs_model4(s, d, hh);
        }
        valid = ok;
        for (int j = 0; j < 8; j++) {
            h[j] = ok ? hh[j] : 0.0;
            a.hyps[(int64_t)k * 8 + j] = ok ? hh[j] : __builtin_nan("");
        }
    }
    __syncthreads();
    if (!valid) {
        if (tid == 0) a.scores[k] = -1;
        return;
    }
    int c = 0;
    for (int i = tid; i < a.n; i += kRansacBlock) {
        const double *p = a.pts + 4 * (int64_t)i;
        c += rs_inlier(h, p[0], p[1], p[2], p[3], a.t2) ? 1 : 0;
    }
    for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
    if ((tid & 63) == 0) wsum[tid >> 6] = c;
    __syncthreads();
    if (tid == 0) {
        int t = 0;
        for (int w = 0; w < kRansacBlock / 64; w++) t += wsum[w];
        a.scores[k] = t;
    }
}

// grid (ceil(n / 256)), block 256: inlier mask of hypothesis a.best.
extern "C" __global__ __launch_bounds__(256) void mcs_ransac_mask(const mcs::KRansacArgs a)
{
    using namespace mcs;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    const double *h = a.hyps + (int64_t)a.best * 8;
    const double *p = a.pts + 4 * (int64_t)i;
    a.mask[i] = rs_inlier(h, p[0], p[1], p[2], p[3], a.t2) ? 1 : 0;
}

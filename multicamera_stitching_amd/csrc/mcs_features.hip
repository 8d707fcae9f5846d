// mcs_features.hip -- gfx950 kernels of the per-frame homography estimation path
// (SURVEY.md section 8 NS-3..5): descriptor matching first.
//
// Brute-force Hamming kNN-2 (NS-4; BFMatcher(NORM_HAMMING).knnMatch(k=2), the reference's matcher
// at StitcherClass.py:405-448 with binary descriptors).  VALU popcount-bound: per (query, train)
// pair 8 v_xor_b32 + 8 v_bcnt_u32_b32 (accumulating) + 3 min/max for the running top-2, with
// no HBM traffic to speak of.  The wave's train chunk is staged in LDS, 64 descriptors per pass
// (one coalesced 32-byte load per lane), and every lane reads the same descriptor back
// (ds_read_b128 broadcast, no bank conflict): no per-descriptor scalar-load round trip in the
// compare loop (the round-2 form, wave-uniform s_load_dwordx8 per descriptor, was latency-bound:
// VALU active 0.18).
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
#include "mcs_orb_core.h"

namespace mcs {

constexpr uint32_t kKeyNone = 0xffffffffu;

__device__ __forceinline__ void top2(uint32_t &k0, uint32_t &k1, uint32_t k)
{
    k1 = min(k1, max(k0, k));
    k0 = min(k0, k);
}

// Hamming distance of query q to a train descriptor staged in LDS (two 16-byte broadcast reads;
// v_bcnt_u32_b32 accumulates).
__device__ __forceinline__ uint32_t hamming_lds(const uint32_t (&q)[8], const uint4 *t)
{
    const uint4 a = t[0], b = t[1];
    return __popc(q[0] ^ a.x) + __popc(q[1] ^ a.y) + __popc(q[2] ^ a.z) + __popc(q[3] ^ a.w) +
           __popc(q[4] ^ b.x) + __popc(q[5] ^ b.y) + __popc(q[6] ^ b.z) + __popc(q[7] ^ b.w);
}

}  // namespace mcs

namespace mcs {

// One block of the kNN-2: queries qblock * kKnnQueriesPerBlock + lane + 64 i (i < kKnnQueriesPerLane)
// against train chunk `chunk`, merged into keys (0xffffffff on entry) by atomicMin.  Each train
// descriptor staged in LDS is read back once per lane (two 16-byte broadcast reads) and compared
// with all of the lane's queries: the LDS return path (1 KiB per wave per read) is shared by more
// pairs.  nq > 0.
__device__ __forceinline__ void knn2_block(const uint32_t *query, const uint32_t *train,
                                           uint32_t *keys, int nq, int nt, int per_chunk,
                                           int qblock, int chunk)
{
    constexpr int QL = kKnnQueriesPerLane;
    uint32_t d[QL][8];
#pragma unroll
    for (int i = 0; i < QL; i++) {
        const int q = qblock * kKnnQueriesPerBlock + i * kKnnLanes + threadIdx.x;
        const uint4 *qs = reinterpret_cast<const uint4 *>(query + (int64_t)min(q, nq - 1) * 8);
        const uint4 v0 = qs[0], v1 = qs[1];
        d[i][0] = v0.x, d[i][1] = v0.y, d[i][2] = v0.z, d[i][3] = v0.w;
        d[i][4] = v1.x, d[i][5] = v1.y, d[i][6] = v1.z, d[i][7] = v1.w;
    }
    const int j0 = chunk * per_chunk, j1 = min(nt, j0 + per_chunk);
    const uint4 *__restrict__ train4 = reinterpret_cast<const uint4 *>(train);
    __shared__ uint4 tl[2 * kKnnLanes];
    uint32_t k0[QL], k1[QL];
#pragma unroll
    for (int i = 0; i < QL; i++) k0[i] = k1[i] = kKeyNone;
    for (int jt = j0; jt < j1; jt += kKnnLanes) {
        const int n = min(kKnnLanes, j1 - jt);
        if ((int)threadIdx.x < n) {
            const uint4 *src = train4 + (int64_t)(jt + threadIdx.x) * 2;
            const uint4 t0 = src[0], t1 = src[1];
            tl[2 * threadIdx.x] = t0;
            tl[2 * threadIdx.x + 1] = t1;
        }
        __syncthreads();
        int u = 0;
        for (; u + 4 <= n; u += 4) {
            uint32_t c[QL][4];
#pragma unroll
            for (int v = 0; v < 4; v++) {
                const uint4 a = tl[2 * (u + v)], b = tl[2 * (u + v) + 1];
#pragma unroll
                for (int i = 0; i < QL; i++)
                    c[i][v] = __popc(d[i][0] ^ a.x) + __popc(d[i][1] ^ a.y) +
                              __popc(d[i][2] ^ a.z) + __popc(d[i][3] ^ a.w) +
                              __popc(d[i][4] ^ b.x) + __popc(d[i][5] ^ b.y) +
                              __popc(d[i][6] ^ b.z) + __popc(d[i][7] ^ b.w);
            }
#pragma unroll
            for (int v = 0; v < 4; v++)
#pragma unroll
                for (int i = 0; i < QL; i++)
                    top2(k0[i], k1[i], (c[i][v] << kKnnKeyShift) | (uint32_t)(jt + u + v));
        }
        for (; u < n; u++)
#pragma unroll
            for (int i = 0; i < QL; i++)
                top2(k0[i], k1[i],
                     (hamming_lds(d[i], tl + 2 * u) << kKnnKeyShift) | (uint32_t)(jt + u));
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < QL; i++) {
        const int q = qblock * kKnnQueriesPerBlock + i * kKnnLanes + threadIdx.x;
        if (q >= nq) break;
        const uint32_t old = atomicMin(&keys[2 * q], k0[i]);
        atomicMin(&keys[2 * q + 1], max(old, k0[i]));
        atomicMin(&keys[2 * q + 1], k1[i]);
    }
}

}  // namespace mcs

// grid (ceil(nq / kKnnQueriesPerBlock), chunks), block 64.  keys must hold 0xffffffff on entry
// (memset).
extern "C" __global__ __launch_bounds__(64) void mcs_hamming_knn2(const mcs::KHammingArgs a)
{
    mcs::knn2_block(a.query, a.train, a.keys, a.nq, a.nt, a.per_chunk, blockIdx.x, blockIdx.y);
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

// ---- L2 kNN-2 --------------------------------------------------------------
// Prep: one wave per descriptor (block 256 = 4 descriptors).
extern "C" __global__ __launch_bounds__(256) void mcs_l2_prep(const mcs::KL2PrepArgs a)
{
    const int lane = threadIdx.x & 63, i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n) return;
    const float *d = a.desc + (int64_t)i * a.dim;
    int8_t *o = a.i8 + (int64_t)i * a.dimp;
    int ni = 0, si = 0;
    float nf = 0.f;
    bool ok = true;
    for (int e = lane; e < a.dimp; e += 64) {
        const float v = e < a.dim ? d[e] : 0.f;
        const bool iv = v >= 0.f && v <= 255.f && v == __builtin_rintf(v);
        ok = ok && iv;
        const int x = iv ? (int)v : 0;
        o[e] = (int8_t)(x - 128);
        ni += x * x;
        si += x - 128;
        nf = __builtin_fmaf(v, v, nf);
    }
    for (int off = 32; off > 0; off >>= 1) {
        ni += __shfl_xor(ni, off, 64);
        si += __shfl_xor(si, off, 64);
        nf += __shfl_xor(nf, off, 64);
    }
    const bool all = __all(ok);
    if (lane == 0) {
        a.norm_i[i] = ni;
        a.sum_i[i] = si;
        a.norm_f[i] = nf;
        if (!all) atomicOr(a.flag, 1u);
    }
}

namespace {

__device__ __forceinline__ void top2_u64(unsigned long long &k0, unsigned long long &k1,
                                         unsigned long long k)
{
    const unsigned long long lo = k < k0 ? k : k0, hi = k < k0 ? k0 : k;
    k0 = lo;
    k1 = hi < k1 ? hi : k1;
}

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m)
{
    const int lo = __shfl_xor((int)(uint32_t)v, m, 64), hi = __shfl_xor((int)(v >> 32), m, 64);
    return ((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo;
}

// Key of squared distance d2 (>= 0) to train j: float distance bits, then the index.
__device__ __forceinline__ unsigned long long l2_key(double d2, int j)
{
    const float f = (float)__builtin_sqrt(d2);
    return ((unsigned long long)__float_as_uint(f) << 32) | (uint32_t)j;
}

// Lanes 16g .. 16g+15 hold partial top-2 lists of the same 4 queries: merge them, then lane 16g
// merges into the global keys (3 atomics per query, as the Hamming matcher).
__device__ __forceinline__ void l2_publish(const mcs::KL2Args &a, int q0, int lane,
                                           unsigned long long (&k0)[4],
                                           unsigned long long (&k1)[4])
{
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) {
            const unsigned long long b0 = shfl_xor_u64(k0[r], m), b1 = shfl_xor_u64(k1[r], m);
            top2_u64(k0[r], k1[r], b0);
            top2_u64(k0[r], k1[r], b1);
        }
    if ((lane & 15) != 0) return;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int q = q0 + (lane >> 4) * 4 + r;
        if (q >= a.nq) continue;
        const unsigned long long old = atomicMin(&a.keys[2 * q], k0[r]);
        atomicMin(&a.keys[2 * q + 1], old > k0[r] ? old : k0[r]);
        atomicMin(&a.keys[2 * q + 1], k1[r]);
    }
}

typedef int l2_v4i __attribute__((ext_vector_type(4)));
typedef float l2_v4f __attribute__((ext_vector_type(4)));

}  // namespace

// Exact path: grid (query blocks, train chunks), block 256.  Wave w: queries q0 .. q0+15 as the
// MFMA A tile (lane l: query q0 + (l & 15), bytes 16 (l >> 4) .. +16 of each 64-byte k step),
// trains in tiles of 16 as B (same lane map); C[g*4 + r][l & 15] = (a - 128).(b - 128).
extern "C" __global__ __launch_bounds__(256) void mcs_l2_knn2_i8(const mcs::KL2Args a)
{
    using namespace mcs;
    if (*a.flag) return;
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int q0 = blockIdx.x * kL2QueriesPerBlock + (threadIdx.x >> 6) * 16;
    if (q0 >= a.nq) return;
    const int steps = a.dimp / 64;
    const int qa = min(q0 + (lane & 15), a.nq - 1);
    l2_v4i A[kL2MaxDim / 64];
#pragma unroll
    for (int s = 0; s < kL2MaxDim / 64; s++)
        A[s] = s < steps ? *reinterpret_cast<const l2_v4i *>(a.q8 + (int64_t)qa * a.dimp + s * 64 +
                                                          g * 16)
                         : l2_v4i{0, 0, 0, 0};
    int qn[4], qs[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int q = min(q0 + g * 4 + r, a.nq - 1);
        qn[r] = a.qn[q];
        qs[r] = a.qs[q];
    }
    unsigned long long k0[4], k1[4];
#pragma unroll
    for (int r = 0; r < 4; r++) k0[r] = k1[r] = kL2KeyNone;
    const int j0 = blockIdx.y * a.per_chunk, j1 = min(a.nt, j0 + a.per_chunk);
    const int bias = 16384 * a.dimp;
    for (int t0 = j0; t0 < j1; t0 += 16) {
        const int j = t0 + (lane & 15), jr = min(j, a.nt - 1);
        l2_v4i acc = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < kL2MaxDim / 64; s++) {
            if (s >= steps) break;
            const l2_v4i B =
                *reinterpret_cast<const l2_v4i *>(a.t8 + (int64_t)jr * a.dimp + s * 64 + g * 16);
            acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[s], B, acc, 0, 0, 0);
        }
        const int tn = a.tn[jr], ts = a.ts[jr];
        if (j < j1) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int dot = acc[r] + 128 * (qs[r] + ts) + bias;
                top2_u64(k0[r], k1[r], l2_key((double)(qn[r] + tn - 2 * dot), j));
            }
        }
    }
    l2_publish(a, q0, lane, k0, k1);
}

// f32 path: the same tiling with v_mfma_f32_16x16x4_f32; k chunks of 128, lane group g supplies
// elements 32 g + s of the chunk at step s (the same map for A and B).
extern "C" __global__ __launch_bounds__(256) void mcs_l2_knn2_f32(const mcs::KL2Args a)
{
    using namespace mcs;
    if (!*a.flag) return;
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int q0 = blockIdx.x * kL2QueriesPerBlock + (threadIdx.x >> 6) * 16;
    if (q0 >= a.nq) return;
    const int qa = min(q0 + (lane & 15), a.nq - 1);
    float qn[4];
#pragma unroll
    for (int r = 0; r < 4; r++) qn[r] = a.qnf[min(q0 + g * 4 + r, a.nq - 1)];
    unsigned long long k0[4], k1[4];
#pragma unroll
    for (int r = 0; r < 4; r++) k0[r] = k1[r] = kL2KeyNone;
    const int j0 = blockIdx.y * a.per_chunk, j1 = min(a.nt, j0 + a.per_chunk);
    const float *qrow = a.qf + (int64_t)qa * a.dim;
    for (int t0 = j0; t0 < j1; t0 += 16) {
        const int j = t0 + (lane & 15), jr = min(j, a.nt - 1);
        const float *trow = a.tf + (int64_t)jr * a.dim;
        l2_v4f acc = {0.f, 0.f, 0.f, 0.f};
        for (int c = 0; c < a.dim; c += 128) {
#pragma unroll
            for (int s = 0; s < 32; s++) {
                const int e = c + 32 * g + s;
                const float x = e < a.dim ? qrow[e] : 0.f, y = e < a.dim ? trow[e] : 0.f;
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, acc, 0, 0, 0);
            }
        }
        const float tn = a.tnf[jr];
        if (j < j1) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const float d2 = qn[r] + tn - 2.f * acc[r];
                top2_u64(k0[r], k1[r], l2_key(d2 > 0.f ? (double)d2 : 0.0, j));
            }
        }
    }
    l2_publish(a, q0, lane, k0, k1);
}

// keys -> (train index, distance); -1 / -1.0f where fewer than two train descriptors exist.
extern "C" __global__ __launch_bounds__(256) void mcs_l2_knn2_finalize(const mcs::KL2Args a)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= 2 * a.nq) return;
    const unsigned long long k = a.keys[i];
    const bool none = k == mcs::kL2KeyNone;
    a.idx[i] = none ? -1 : (int32_t)(uint32_t)k;
    a.dist[i] = none ? -1.f : __uint_as_float((uint32_t)(k >> 32));
}

// ---- RANSAC homography (NS-5) ------------------------------------------------------------------
namespace mcs {

// Hypothesis k of a RANSAC over n correspondences (block kRansacBlock): thread 0 draws the
// sample and solves its 4-point model, then the block counts its inliers (FP64,
// mcs_ransac_core.h).  hyps[8 k ..] = the model (NaN: rejected), scores[k] = inliers (-1).
__device__ __forceinline__ void ransac_block(const double *pts, double *hyps, int32_t *scores,
                                             int n, uint32_t seed, double t2, int k)
{
    __shared__ double h[8];
    __shared__ int valid;
    __shared__ int wsum[kRansacBlock / 64];
    const int tid = threadIdx.x;
    if (tid == 0) {
        int idx[4];
        double s[8], d[8], hh[8];
        bool ok = rs_subset(seed, (uint32_t)k, (uint32_t)n, idx);
        if (ok) {
            for (int m = 0; m < 4; m++) {
                s[2 * m] = pts[4 * idx[m]], s[2 * m + 1] = pts[4 * idx[m] + 1];
                d[2 * m] = pts[4 * idx[m] + 2], d[2 * m + 1] = pts[4 * idx[m] + 3];
            }
            ok = rs_model4(s, d, hh);
        }
        valid = ok;
        for (int j = 0; j < 8; j++) {
            h[j] = ok ? hh[j] : 0.0;
            hyps[(int64_t)k * 8 + j] = ok ? hh[j] : __builtin_nan("");
        }
    }
    __syncthreads();
    if (!valid) {
        if (tid == 0) scores[k] = -1;
        return;
    }
    int c = 0;
    for (int i = tid; i < n; i += kRansacBlock) {
        const double *p = pts + 4 * (int64_t)i;
        c += rs_inlier(h, p[0], p[1], p[2], p[3], t2) ? 1 : 0;
    }
    for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
    if ((tid & 63) == 0) wsum[tid >> 6] = c;
    __syncthreads();
    if (tid == 0) {
        int t = 0;
        for (int w = 0; w < kRansacBlock / 64; w++) t += wsum[w];
        scores[k] = t;
    }
}

}  // namespace mcs

// grid (iters), block kRansacBlock: hypothesis blockIdx.x.
extern "C" __global__ __launch_bounds__(256) void mcs_ransac_score(const mcs::KRansacArgs a)
{
    mcs::ransac_block(a.pts, a.hyps, a.scores, a.n, a.seed, a.t2, blockIdx.x);
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

// ---- ORB (NS-3) ----------------------------------------------------------------------------
// BGR -> gray with OpenCV's fixed point: (1868 B + 9617 G + 4899 R + 8192) >> 14.
// Four pixels per thread: three dword loads (12 bytes of BGR) and one dword store when the
// frame is 4-byte aligned (the gray level always is), bytes otherwise.
extern "C" __global__ __launch_bounds__(256) void mcs_orb_gray(const mcs::KGrayArgs a)
{
    const int q = blockIdx.x * 256 + threadIdx.x, i = 4 * q;
    const uint8_t *bgr = a.bgr[blockIdx.y];
    uint8_t *gray = a.gray + blockIdx.y * a.stride;
    if (i >= a.n) return;
    auto g = [](uint32_t b, uint32_t gg, uint32_t r) {
        return (1868u * b + 9617u * gg + 4899u * r + 8192u) >> 14;
    };
    if (i + 4 <= a.n && ((uintptr_t)bgr & 3) == 0) {
        const uint32_t *p = reinterpret_cast<const uint32_t *>(bgr) + 3 * (int64_t)q;
        const uint32_t w0 = __builtin_nontemporal_load(p), w1 = __builtin_nontemporal_load(p + 1),
                       w2 = __builtin_nontemporal_load(p + 2);
        const uint32_t v0 = g(w0 & 255, (w0 >> 8) & 255, (w0 >> 16) & 255);
        const uint32_t v1 = g(w0 >> 24, w1 & 255, (w1 >> 8) & 255);
        const uint32_t v2 = g((w1 >> 16) & 255, w1 >> 24, w2 & 255);
        const uint32_t v3 = g((w2 >> 8) & 255, (w2 >> 16) & 255, w2 >> 24);
        reinterpret_cast<uint32_t *>(gray)[q] = v0 | v1 << 8 | v2 << 16 | v3 << 24;
        return;
    }
    for (int j = i; j < min(i + 4, a.n); j++) {
        const uint8_t *p = bgr + 3 * (int64_t)j;
        gray[j] = (uint8_t)g(p[0], p[1], p[2]);
    }
}

__device__ __forceinline__ int orb_refl(int i, int n)
{
    return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i);
}

// One launch per frame over every pyramid level: per 64 x 16 tile of a level (block ->
// level by the prefix table bstart, tiles row-major), the level image with a 4-pixel halo
// (reflect-101 positions, for the blur) is staged in LDS once; from it
//   - the 7-tap Gaussian blur (horizontal pass in u16 into LDS, vertical pass with one
//     rounding, (s + 32768) >> 16: the descriptors' image),
//   - the FAST-9 scores of the tile and a one-pixel ring (score > threshold, else 0; 0 outside
//     the region where a keypoint's NMS can look): the bit-mask segment test on every position,
//     the score only on the (compacted) positions that pass it,
//   - the 3x3 non-maximum suppression of the tile's pixels (strict, inside the kOrbEdge
//     border), the survivors compacted in LDS so that the Harris sums (32-bit exact, 7x7 Sobel
//     on the staged image) run on full waves, and appended to the level's candidates (their
//     order is irrelevant: the level is ranked afterwards by response, y, x).
// Same values as the four per-pixel passes it replaces (blur_h, blur_v, fast, nms).
constexpr int kOrbTX = mcs::kOrbTileW, kOrbTY = mcs::kOrbTileH, kOrbHalo = 4;
constexpr int kOrbLX = kOrbTX + 2 * kOrbHalo, kOrbLY = kOrbTY + 2 * kOrbHalo;   // 72 x 24
constexpr int kOrbSX = kOrbTX + 2, kOrbSY = kOrbTY + 2;                         // score ring

extern "C" __global__ __launch_bounds__(mcs::kOrbLevelThreads) void mcs_orb_level(const mcs::KOrbPyrArgs p)
{
    __shared__ __attribute__((aligned(16))) uint8_t img[kOrbLY * kOrbLX];
    __shared__ __attribute__((aligned(16))) uint16_t hb[(kOrbTY + 6) * kOrbTX];
    __shared__ uint8_t sc[kOrbSY * kOrbSX];
    // the FAST lists (fc: pre-test survivors, fl: segment-test survivors), then -- once the scores
    // are in, a barrier later -- the NMS survivors sx over the same bytes: 36 KB of LDS per block
    // instead of 52 KB, 4 blocks per CU instead of 3
    __shared__ __attribute__((aligned(16))) uint16_t lists[2 * kOrbSY * kOrbSX];
    uint16_t *const fl = lists, *const fc = lists + kOrbSY * kOrbSX;
    uint16_t *const sx = lists;
    static_assert(kOrbTX * kOrbTY <= 2 * kOrbSY * kOrbSX && kOrbTX * kOrbTY <= 65536,
                  "ORB level: the NMS list fits the FAST lists' bytes, indices in 16 bits");
    __shared__ int ns, nf, nc;
    const int b = blockIdx.x, tid = threadIdx.x, cam = blockIdx.y;
    int l = 0;
    for (int k = 1; k < p.nlevels; k++) l += b >= p.bstart[k] ? 1 : 0;
    const int w = p.w[l], h = p.h[l];
    const int bx = (w + kOrbTX - 1) / kOrbTX, loc = b - p.bstart[l];
    const int y0 = (loc / bx) * kOrbTY, x0 = (loc % bx) * kOrbTX;
    const uint8_t *im = p.img + cam * p.stride + p.off[l];
    if (tid == 0) ns = 0, nf = 0, nc = 0;
    if (x0 >= kOrbHalo && y0 >= kOrbHalo && x0 + kOrbTX + kOrbHalo <= w &&
        y0 + kOrbTY + kOrbHalo <= h) {   // interior tile: no reflection
        // (dword loads: a staged row is 18 dwords; the level rows start at any byte, and gfx950
        // global loads take unaligned dwords)
        const uint8_t *src = im + (int64_t)(y0 - kOrbHalo) * w + (x0 - kOrbHalo);
        constexpr int DW = kOrbLX / 4;
        static_assert(kOrbLX % 4 == 0, "ORB tile rows: whole dwords");
        for (int i = tid; i < kOrbLY * DW; i += mcs::kOrbLevelThreads) {
            uint32_t v;
            __builtin_memcpy(&v, src + (int64_t)(i / DW) * w + 4 * (i % DW), 4);
            reinterpret_cast<uint32_t *>(img)[i] = v;
        }
    } else {
        for (int i = tid; i < kOrbLY * kOrbLX; i += mcs::kOrbLevelThreads) {
            const int yy = orb_refl(min(max(y0 - kOrbHalo + i / kOrbLX, -(h - 1)), 2 * h - 2), h);
            const int xx = orb_refl(min(max(x0 - kOrbHalo + i % kOrbLX, -(w - 1)), 2 * w - 2), w);
            img[i] = im[(int64_t)yy * w + xx];
        }
    }
    __syncthreads();
    // blur: horizontal over rows y0 - 3 .. y0 + kOrbTY + 2, then vertical; 4 columns per thread
    // (the horizontal pass reads its 10 bytes as 4 dwords + v_alignbyte and writes 4 u16 at once)
    typedef __attribute__((address_space(3))) const uint32_t lu32;
    typedef __attribute__((address_space(3))) const uint8_t lu8;
    typedef __attribute__((address_space(3))) uint2 lu2;
    constexpr int Q = kOrbTX / 4;
    for (int i = tid; i < (kOrbTY + 6) * Q; i += mcs::kOrbLevelThreads) {
        const int row = i / Q, c4 = 4 * (i - row * Q);
        const int a = (row + 1) * kOrbLX + c4 + 1;   // the first tap of the 4 outputs
        const lu32 *d = (const lu32 *)((lu8 *)img + (a & ~3));
        const uint32_t sh = (uint32_t)a & 3u, x0 = d[0], x1 = d[1], x2 = d[2], x3 = d[3];
        const uint32_t b[3] = {__builtin_amdgcn_alignbyte(x1, x0, sh),
                               __builtin_amdgcn_alignbyte(x2, x1, sh),
                               __builtin_amdgcn_alignbyte(x3, x2, sh)};
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint32_t v = 0;
#pragma unroll
            for (int t = 0; t < 7; t++)
                v += (uint32_t)mcs::kOrbBlur[t] * ((b[(j + t) >> 2] >> (8 * ((j + t) & 3))) & 255u);
            o[j] = v;
        }
        *(lu2 *)(hb + row * kOrbTX + c4) = make_uint2(o[0] | (o[1] << 16), o[2] | (o[3] << 16));
    }
    // FAST on the tile and a one-pixel ring (positions x0 - 1 .., y0 - 1 ..), in three compacted
    // stages so that every stage runs on full waves: the cardinal pre-test everywhere, the
    // segment test (= score > threshold) on its survivors, the score on the corners
    const int lo = mcs::kOrbEdge - 1;
    auto append = [&](int *count, uint16_t *list, int i) {   // (called by the active lanes)
        const unsigned long long act = __ballot(1);
        const int lane = __lane_id(), leader = __ffsll((long long)act) - 1;
        int base = 0;
        if (lane == leader) base = atomicAdd(count, __popcll(act));
        list[__shfl(base, leader) + __popcll(act & ((1ull << lane) - 1ull))] = (uint16_t)i;
    };
    auto at = [&](int i) { return img + (i / kOrbSX + kOrbHalo - 1) * kOrbLX + i % kOrbSX + kOrbHalo - 1; };
    for (int i = tid; i < kOrbSY * kOrbSX; i += mcs::kOrbLevelThreads) {
        const int yy = y0 - 1 + i / kOrbSX, xx = x0 - 1 + i % kOrbSX;
        sc[i] = 0;
        if (xx >= lo && yy >= lo && xx < w - lo && yy < h - lo &&
            mcs::orb_fast_pretest(at(i), kOrbLX, p.threshold))
            append(&nc, fc, i);
    }
    __syncthreads();
    for (int j = tid; j < nc; j += mcs::kOrbLevelThreads) {
        const int i = fc[j];
        if (mcs::orb_fast_test(at(i), kOrbLX, p.threshold)) append(&nf, fl, i);
    }
    __syncthreads();
    for (int j = tid; j < nf; j += mcs::kOrbLevelThreads) {
        const int i = fl[j];
        sc[i] = (uint8_t)mcs::orb_fast_score(at(i), kOrbLX);
    }
    uint8_t *blur = p.blur + cam * p.stride + p.off[l];
    for (int i = tid; i < kOrbTY * Q; i += mcs::kOrbLevelThreads) {
        const int row = i / Q, c4 = 4 * (i - row * Q);
        const int yy = y0 + row, xx = x0 + c4;
        if (yy >= h || xx >= w) continue;
        uint32_t sv[4] = {32768u, 32768u, 32768u, 32768u};
#pragma unroll
        for (int t = 0; t < 7; t++) {
            const uint2 v = *(const lu2 *)(hb + (row + t) * kOrbTX + c4);
            sv[0] += (uint32_t)mcs::kOrbBlur[t] * (v.x & 0xffffu);
            sv[1] += (uint32_t)mcs::kOrbBlur[t] * (v.x >> 16);
            sv[2] += (uint32_t)mcs::kOrbBlur[t] * (v.y & 0xffffu);
            sv[3] += (uint32_t)mcs::kOrbBlur[t] * (v.y >> 16);
        }
        uint8_t *o = blur + (int64_t)yy * w + xx;
        if (xx + 4 <= w) {   // (an unaligned dword store: level rows start at any byte)
            const uint32_t word = (sv[0] >> 16) | ((sv[1] >> 16) << 8) | ((sv[2] >> 16) << 16) |
                                  ((sv[3] >> 16) << 24);
            __builtin_memcpy(o, &word, 4);
        } else {
            for (int j = 0; j < w - xx; j++) o[j] = (uint8_t)(sv[j] >> 16);
        }
    }
    __syncthreads();
    // 3x3 NMS of the tile's pixels; survivors (packed y << 16 | x) compacted in LDS
    const int e = mcs::kOrbEdge;
    for (int i = tid; i < kOrbTY * kOrbTX; i += mcs::kOrbLevelThreads) {
        const int yy = y0 + i / kOrbTX, xx = x0 + i % kOrbTX;
        bool keep = xx >= e && yy >= e && xx < w - e && yy < h - e;
        if (keep) {
            const uint8_t *s = sc + (i / kOrbTX + 1) * kOrbSX + i % kOrbTX + 1;
            const int c = s[0];
            keep = c != 0;
#pragma unroll
            for (int dy = -1; dy <= 1; dy++)
#pragma unroll
                for (int dx = -1; dx <= 1; dx++)
                    if (dx || dy) keep = keep && c > s[dy * kOrbSX + dx];
        }
        if (keep) {
            const unsigned long long act = __ballot(1);
            const int lane = __lane_id(), leader = __ffsll((long long)act) - 1;
            int base = 0;
            if (lane == leader) base = atomicAdd(&ns, __popcll(act));
            sx[__shfl(base, leader) + __popcll(act & ((1ull << lane) - 1ull))] = (uint16_t)i;
        }
    }
    __syncthreads();
    const int n = ns;
    for (int j0 = 0; j0 < n; j0 += mcs::kOrbLevelThreads) {
        const int j = j0 + tid;
        if (j >= n) break;
        const int i = sx[j];
        const double r = mcs::orb_harris(
            img + (i / kOrbTX + kOrbHalo) * kOrbLX + i % kOrbTX + kOrbHalo, kOrbLX);
        const unsigned long long act = __ballot(1);
        const int lane = __lane_id(), leader = __ffsll((long long)act) - 1;
        int base = 0;
        if (lane == leader) base = atomicAdd(p.ncand + cam * mcs::kOrbMaxLevels + l, __popcll(act));
        const int q = __shfl(base, leader) + __popcll(act & ((1ull << lane) - 1ull));
        if (q < p.cap[l]) {
            mcs::OrbCand *cand = p.cand + cam * p.cstride + p.coff[l];
            cand[q].x = x0 + i % kOrbTX;
            cand[q].y = y0 + i / kOrbTX;
            cand[q].response = r;
        }
    }
}

// grid (nlevels), block kOrbSelThreads: the level's candidates ranked in LDS by a bitonic sort
// (response descending, then y, then x: the host ranking's total order; (y, x) packed as
// y << 16 | x), then its quota written at the level's offset (the kept counts of the levels
// before it).  More than kOrbSelMax candidates on any level: overflow, the host ranks instead.
extern "C" __global__ __launch_bounds__(1024) void mcs_orb_select(const mcs::KOrbSelArgs a)
{
    using namespace mcs;
    __shared__ double rs[kOrbSelMax];
    __shared__ uint32_t ks[kOrbSelMax];
    const int l = blockIdx.x, tid = threadIdx.x, cam = blockIdx.y;
    const int *ncand = a.ncand + cam * kOrbMaxLevels;
    int *kp = a.kp + 3 * cam * a.kstride, *sel = a.sel + 2 * cam;
    double *resp = a.resp + cam * a.kstride;
    auto kept = [&](int i) { return min(min(ncand[i], a.cap[i]), a.quota[i]); };
    int base = 0, total = 0;
    for (int i = 0; i < a.nlevels; i++) {
        if (i < l) base += kept(i);
        total += kept(i);
    }
    bool over = false;
    for (int i = 0; i < a.nlevels; i++) over = over || min(ncand[i], a.cap[i]) > kOrbSelMax;
    if (l == 0 && tid == 0) {
        sel[0] = total;
        sel[1] = over ? 1 : 0;
    }
    if (over) return;   // uniform
    const int c = min(ncand[l], a.cap[l]), q = kept(l);
    int n = 64;
    while (n < c) n <<= 1;
    const OrbCand *cd = a.cand + cam * a.cstride + a.coff[l];
    for (int i = tid; i < n; i += kOrbSelThreads) {
        const bool v = i < c;
        rs[i] = v ? cd[i].response : -__builtin_inf();
        ks[i] = v ? ((uint32_t)cd[i].y << 16) | (uint32_t)cd[i].x : 0xffffffffu;
    }
    __syncthreads();
    // (a stage of stride <= 64 pairs elements inside each wave's own 128-element segments: the
    // wave's LDS accesses stay in issue order, so only strides >= 128 need the block barrier)
    for (int size = 2; size <= n; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = tid; t < n / 2; t += kOrbSelThreads) {
                const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
                const double rl = rs[lo], rh = rs[hi];
                const uint32_t kl = ks[lo], kh = ks[hi];
                const bool hi_first = rh > rl || (rh == rl && kh < kl);
                if (hi_first == ((lo & size) == 0)) {
                    rs[lo] = rh, rs[hi] = rl;
                    ks[lo] = kh, ks[hi] = kl;
                }
            }
            if (stride >= 128 || (stride == 1 && size * 2 > 128) || size == n) {
                __syncthreads();
            } else {
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
            }
        }
    for (int i = tid; i < q; i += kOrbSelThreads) {
        const int o = base + i;
        kp[3 * o] = l;
        kp[3 * o + 1] = (int)(ks[i] & 0xffffu);
        kp[3 * o + 2] = (int)(ks[i] >> 16);
        resp[o] = rs[i];
    }
}

// The orientation disk (rows v = 0 .. kOrbHalfPatch, |u| <= kOrbUmax[v]) as a flat list of
// (v, u) entries, (v << 8) | (u & 255); an entry of row v >= 1 stands for the pixels (u, v) and
// (u, -v).  Dealt over the wave's 64 lanes (~6 entries each) instead of one row per lane.
struct OrbMomTab {
    int16_t e[512];
    int n;
};
constexpr OrbMomTab orb_mom_tab()
{
    OrbMomTab t{};
    int i = 0;
    for (int u = -mcs::kOrbHalfPatch; u <= mcs::kOrbHalfPatch; u++) t.e[i++] = (int16_t)(u & 255);
    for (int v = 1; v <= mcs::kOrbHalfPatch; v++)
        for (int u = -mcs::kOrbUmax[v]; u <= mcs::kOrbUmax[v]; u++)
            t.e[i++] = (int16_t)((v << 8) | (u & 255));
    t.n = i;
    return t;
}
__constant__ OrbMomTab kOrbMom = orb_mom_tab();
static_assert(orb_mom_tab().n <= 512, "ORB orientation disk entries");

// grid (n), block 64: one wave per keypoint -- orientation moments (the disk's entries dealt over
// the lanes, integer sums, wave reduction), then 4 rBRIEF pairs per lane packed into the 32
// descriptor bytes.
extern "C" __global__ __launch_bounds__(64) void mcs_orb_describe(const mcs::KOrbDescArgs a)
{
    using namespace mcs;
    const int k = blockIdx.x, lane = threadIdx.x, cam = blockIdx.y;
    const int *sel = a.sel ? a.sel + 2 * cam : nullptr;
    if (sel && (k >= sel[0] || sel[1])) return;   // past the device ranking's count
    const int *kp = a.kp + 3 * cam * a.kstride;
    const int lvl = kp[3 * k], x = kp[3 * k + 1], y = kp[3 * k + 2];
    const int w = a.w[lvl];
    const int64_t co = cam * a.stride;
    const uint8_t *p = a.img[lvl] + co + (int64_t)y * w + x;
    long long m10 = 0, m01 = 0;
    for (int i = lane; i < kOrbMom.n; i += 64) {
        const int e = kOrbMom.e[i], v = e >> 8, u = (int)(int8_t)(e & 255);
        if (v == 0) {
            m10 += u * (int)p[u];
        } else {
            const int q = p[u + v * w], r = p[u - v * w];
            m01 += (long long)(v * (q - r));
            m10 += (long long)(u * (q + r));
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        m10 += __shfl_down(m10, off, 64);
        m01 += __shfl_down(m01, off, 64);
    }
    m10 = __shfl(m10, 0, 64);
    m01 = __shfl(m01, 0, 64);
    const double fx = (double)m10, fy = (double)m01;
    const double r = sqrt(fx * fx + fy * fy);
    const double cs = r > 0.0 ? fx / r : 1.0, sn = r > 0.0 ? fy / r : 0.0;
    const uint8_t *b = a.blur[lvl] + co + (int64_t)y * w + x;
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const signed char *t = kOrbPattern[4 * lane + j];
        const int v1 = b[orb_rot_off(t[0], t[1], cs, sn, w)];
        const int v2 = b[orb_rot_off(t[2], t[3], cs, sn, w)];
        bits |= (uint32_t)(v1 < v2) << j;
    }
    const uint32_t hi = __shfl_down(bits, 1, 64);
    if ((lane & 1) == 0) a.desc[32 * ((int64_t)cam * a.kstride + k) + (lane >> 1)] = (uint8_t)(bits | (hi << 4));
    if (lane == 0) {
        a.orient[2 * ((int64_t)cam * a.kstride + k)] = cs;
        a.orient[2 * ((int64_t)cam * a.kstride + k) + 1] = sn;
    }
}

// ---- ORB pyramid in one launch ----------------------------------------------------------------
namespace mcs {

// OpenCV 3.4 resize(INTER_LINEAR) source index and 11-bit coefficients of destination index d
// (the float arithmetic of mcs_kernels.hip resize_axis / oracle/orc_resize.c).
__device__ __forceinline__ void pyr_axis(int d, double scale, int ssize, bool is_x, int &s,
                                         int &c0, int &c1)
{
    float f = (float)((d + 0.5) * scale - 0.5);
    int si = (int)floorf(f);
    f -= (float)si;
    if (is_x) {
        if (si < 0) f = 0.f, si = 0;
        if (si >= ssize - 1) f = 0.f, si = ssize - 1;
    }
    s = si;
    c0 = __float2int_rn((1.f - f) * 2048.f);
    c1 = __float2int_rn(f * 2048.f);
}

}  // namespace mcs

extern "C" __global__ __launch_bounds__(256) void mcs_orb_pyramid(const mcs::KOrbBuildArgs a)
{
    using namespace mcs;
    extern __shared__ uint8_t pyr_lds[];
    const int L = a.nlevels - 1, tid = threadIdx.x;
    const int t = blockIdx.x, tx = t % a.gx, ty = t / a.gx;
    uint8_t *const lvl = a.lvl + blockIdx.y * a.stride;
    // regions [x0, x1) x [y0, y1) of every level, top down (block-uniform)
    int x0[12], x1[12], y0[12], y1[12];
    x0[L] = tx * a.tw;
    y0[L] = ty * a.th;
    x1[L] = min(x0[L] + a.tw, a.w[L]);
    y1[L] = min(y0[L] + a.th, a.h[L]);
    for (int l = L; l >= 2; l--) {
        int s, c0, c1;
        const int sw = a.w[l - 1], sh = a.h[l - 1];
        pyr_axis(x0[l], a.sx[l], sw, true, s, c0, c1);
        x0[l - 1] = s;
        pyr_axis(x1[l] - 1, a.sx[l], sw, true, s, c0, c1);
        x1[l - 1] = s >= sw - 1 ? sw : s + 2;
        pyr_axis(y0[l], a.sy[l], sh, false, s, c0, c1);
        y0[l - 1] = min(max(s, 0), sh - 1);
        pyr_axis(y1[l] - 1, a.sy[l], sh, false, s, c0, c1);
        y1[l - 1] = min(max(s + 1, 0), sh - 1) + 1;
    }
    uint8_t *buf[2] = {pyr_lds, pyr_lds + a.lds_w * a.lds_h};
    typedef __attribute__((address_space(3))) const uint32_t lu32;
    typedef __attribute__((address_space(3))) uint8_t lu8;
    // 8 bytes of a source row from byte o: level 0 by an unaligned global dwordx2, the LDS regions
    // by three aligned dword reads + v_alignbyte (the LDS block has 16 bytes of slack past them)
    auto row8_global = [](const uint8_t *q, int o) {
        uint2 v;
        __builtin_memcpy(&v, q + o, 8);
        return v;
    };
    auto row8_lds = [](const uint8_t *q, int o) {
        const uint32_t a8 = (uint32_t)(uintptr_t)((const lu8 *)q) + (uint32_t)o;
        const lu32 *d = (const lu32 *)(uintptr_t)(a8 & ~3u);
        const uint32_t sh = a8 & 3u, x0 = d[0], x1 = d[1], x2 = d[2];
        return make_uint2(__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh));
    };
    // one level's region, 4 horizontally adjacent pixels per thread: their source columns lie
    // within 8 bytes of the first's (every level step is below 2x), so each source row is read once
    auto level = [&](int l, const uint8_t *src, int spitch, int sx0, int sy0, auto row8) {
        const int rw = x1[l] - x0[l], rh = y1[l] - y0[l];
        const int sw = a.w[l - 1], sh = a.h[l - 1];
        lu8 *dst = (lu8 *)buf[l & 1];
        uint8_t *out = lvl + a.off[l];
        const int gw = (rw + 3) >> 2;
        for (int i = tid; i < gw * rh; i += 256) {
            const int gy = i / gw, gx = i - gy * gw;
            const int y = y0[l] + gy, xs = x0[l] + 4 * gx, n = min(4, x1[l] - xs);
            int sy, b0, b1;
            pyr_axis(y, a.sy[l], sh, false, sy, b0, b1);
            const int r0 = min(max(sy, 0), sh - 1), r1 = min(max(sy + 1, 0), sh - 1);
            int sc[4], c0[4], c1[4];
#pragma unroll
            for (int j = 0; j < 4; j++) pyr_axis(min(xs + j, x1[l] - 1), a.sx[l], sw, true, sc[j], c0[j], c1[j]);
            const int o = sc[0] - sx0;
            const uint2 w0 = row8(src + (int64_t)(r0 - sy0) * spitch, o);
            const uint2 w1 = row8(src + (int64_t)(r1 - sy0) * spitch, o);
            auto byte_at = [](uint2 w, int k) {
                return (int)(((k < 4 ? w.x : w.y) >> (8 * (k & 3))) & 255u);
            };
            uint32_t word = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int k = sc[j] - sc[0];
                const bool one = sc[j] >= sw - 1;
                const int d0 = one ? byte_at(w0, k) * 2048 : byte_at(w0, k) * c0[j] + byte_at(w0, k + 1) * c1[j];
                const int d1 = one ? byte_at(w1, k) * 2048 : byte_at(w1, k) * c0[j] + byte_at(w1, k + 1) * c1[j];
                const uint32_t v = (uint32_t)((((b0 * (d0 >> 4)) >> 16) + ((b1 * (d1 >> 4)) >> 16) + 2) >> 2) & 255u;
                word |= v << (8 * j);
                if (l < L && j < n) dst[gy * rw + 4 * gx + j] = (uint8_t)v;
            }
            uint8_t *po = out + (int64_t)y * a.w[l] + xs;
            if (n == 4) __builtin_memcpy(po, &word, 4);   // (an unaligned dword store)
            else
                for (int j = 0; j < n; j++) po[j] = (uint8_t)(word >> (8 * j));
        }
        __syncthreads();
    };
    level(1, lvl + a.off[0], a.w[0], 0, 0, row8_global);
    for (int l = 2; l <= L; l++)
        level(l, buf[(l - 1) & 1], x1[l - 1] - x0[l - 1], x0[l - 1], y0[l - 1], row8_lds);
}

// ---- A rig capture on the device (mcs_rig.cpp; KRigArgs) ---------------------------------------
// grid (ceil(kstride / kKnnQueriesPerBlock), chunks, pairs), block 64: pair p's kNN-2, query camera p + 1 against
// train camera p, the keypoint counts read from the device (a camera whose ranking overflowed
// counts as empty: the host redoes that capture through the per-call path).
extern "C" __global__ __launch_bounds__(64) void mcs_rig_knn2(const mcs::KRigArgs a)
{
    using namespace mcs;
    const int p = blockIdx.z;
    const int nq = a.sel[2 * (p + 1) + 1] ? 0 : a.sel[2 * (p + 1)];
    const int nt = a.sel[2 * p + 1] ? 0 : a.sel[2 * p];
    if ((int)blockIdx.x * kKnnQueriesPerBlock >= nq || (int)blockIdx.y * a.per_chunk >= nt)
        return;   // block-uniform
    knn2_block(reinterpret_cast<const uint32_t *>(a.desc + (int64_t)32 * (p + 1) * a.kstride),
               reinterpret_cast<const uint32_t *>(a.desc + (int64_t)32 * p * a.kstride),
               a.keys + (int64_t)2 * p * a.kstride, nq, nt, a.per_chunk, blockIdx.x, blockIdx.y);
}

// grid (pairs), block 1024: pair p's kNN-2 keys -> Lowe's ratio (a second neighbour exists and
// (double)d0 < (double)d1 * ratio, strict) -> the passing queries' positions (query and its best
// train keypoint, level-0 pixels as the float (float)x * lscale[level]) compacted in query order
// into pts; info[4 p] = their count.
extern "C" __global__ __launch_bounds__(1024) void mcs_rig_match(const mcs::KRigArgs a)
{
    using namespace mcs;
    const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nq = a.sel[2 * (p + 1) + 1] ? 0 : a.sel[2 * (p + 1)];
    const int nt = a.sel[2 * p + 1] ? 0 : a.sel[2 * p];
    const uint32_t *keys = a.keys + (int64_t)2 * p * a.kstride;
    const int *kq = a.kp + (int64_t)3 * (p + 1) * a.kstride, *kt = a.kp + (int64_t)3 * p * a.kstride;
    double *pts = a.pts + (int64_t)4 * p * a.kstride;
    __shared__ int wcount[16];
    int base = 0;
    for (int q0 = 0; q0 < (nt > 0 ? nq : 0); q0 += 1024) {
        const int q = q0 + tid;
        bool pass = false;
        uint32_t k0 = kKeyNone;
        if (q < nq) {
            k0 = keys[2 * q];
            const uint32_t k1 = keys[2 * q + 1];
            pass = k1 != kKeyNone &&
                   (double)(k0 >> kKnnKeyShift) < (double)(k1 >> kKnnKeyShift) * a.ratio;
        }
        const unsigned long long bal = __ballot(pass);
        if (lane == 0) wcount[wave] = __popcll(bal);
        __syncthreads();
        int before = 0, total = 0;
        for (int w = 0; w < 16; w++) {
            before += w < wave ? wcount[w] : 0;
            total += wcount[w];
        }
        if (pass) {
            const int o = base + before + __popcll(bal & ((1ull << lane) - 1ull));
            const int t = (int)(k0 & (kKnnMaxTrain - 1));
            pts[4 * o] = (double)((float)kq[3 * q + 1] * a.lscale[kq[3 * q]]);
            pts[4 * o + 1] = (double)((float)kq[3 * q + 2] * a.lscale[kq[3 * q]]);
            pts[4 * o + 2] = (double)((float)kt[3 * t + 1] * a.lscale[kt[3 * t]]);
            pts[4 * o + 3] = (double)((float)kt[3 * t + 2] * a.lscale[kt[3 * t]]);
        }
        base += total;
        __syncthreads();
    }
    if (tid == 0) {
        a.info[4 * p] = base;
        a.info[4 * p + 3] = 0;
    }
}

// grid (iters, pairs), block kRansacBlock: pair p's hypotheses (none -- scores -1 -- with 4 or
// fewer matches: the reference needs more than 4 to call findHomography).
// The rig's RANSAC in two launches: mcs_rig_hyp solves the hypotheses, one per lane (grid
// (ceil(iters / 64), pairs), block 64: the 4-point solves of 64 hypotheses side by side instead
// of each on thread 0 of its own block while the other 255 wait), mcs_rig_ransac scores them,
// one block per hypothesis.  Same functions, same operands: the same models and scores as
// ransac_block.
extern "C" __global__ __launch_bounds__(64) void mcs_rig_hyp(const mcs::KRigArgs a)
{
    using namespace mcs;
    const int p = blockIdx.y, k = blockIdx.x * 64 + threadIdx.x, n = a.info[4 * p];
    if (k >= a.iters || n <= 4) return;
    const double *pts = a.pts + (int64_t)4 * p * a.kstride;
    double *hyps = a.hyps + (int64_t)8 * p * a.iters;
    int idx[4];
    double sp[8], dp[8], hh[8];
    bool ok = rs_subset(a.seed, (uint32_t)k, (uint32_t)n, idx);
    if (ok) {
        for (int m = 0; m < 4; m++) {
            sp[2 * m] = pts[4 * idx[m]], sp[2 * m + 1] = pts[4 * idx[m] + 1];
            dp[2 * m] = pts[4 * idx[m] + 2], dp[2 * m + 1] = pts[4 * idx[m] + 3];
        }
        ok = rs_model4(sp, dp, hh);
    }
    for (int j = 0; j < 8; j++) hyps[(int64_t)k * 8 + j] = ok ? hh[j] : __builtin_nan("");
    a.scores[(int64_t)p * a.iters + k] = ok ? 0 : -1;   // (validity, for mcs_rig_ransac)
}

// grid (iters, pairs), block kRansacBlock: the inliers of hypothesis blockIdx.x (mcs_rig_hyp's
// model; its score slot holds -1 for a rejected one, which keeps it).
extern "C" __global__ __launch_bounds__(256) void mcs_rig_ransac(const mcs::KRigArgs a)
{
    using namespace mcs;
    const int p = blockIdx.y, k = blockIdx.x, n = a.info[4 * p], tid = threadIdx.x;
    int32_t *scores = a.scores + (int64_t)p * a.iters;
    __shared__ int wsum[kRansacBlock / 64];
    if (n <= 4) {
        if (tid == 0) scores[k] = -1;
        return;
    }
    if (scores[k] < 0) return;   // (block-uniform: rejected by mcs_rig_hyp, score stays -1)
    const double *hk = a.hyps + (int64_t)8 * p * a.iters + (int64_t)8 * k;
    double h[8];
    for (int j = 0; j < 8; j++) h[j] = hk[j];
    const double *pts = a.pts + (int64_t)4 * p * a.kstride;
    int c = 0;
    for (int i = tid; i < n; i += kRansacBlock) {
        const double *q = pts + 4 * (int64_t)i;
        c += rs_inlier(h, q[0], q[1], q[2], q[3], a.t2) ? 1 : 0;
    }
    for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
    if ((tid & 63) == 0) wsum[tid >> 6] = c;
    __syncthreads();
    if (tid == 0) {
        int t = 0;
        for (int w = 0; w < kRansacBlock / 64; w++) t += wsum[w];
        scores[k] = t;
    }
}

// grid (pairs), block 1024: pair p's best hypothesis -- the first of the highest score, as the
// host scan -- into info[4 p + 1 ..] (index, score; -1, -1 without matches to score), its model
// into hbest and, when it has 4 or more inliers, its inlier mask.
extern "C" __global__ __launch_bounds__(1024) void mcs_rig_best(const mcs::KRigArgs a)
{
    using namespace mcs;
    const int p = blockIdx.x, tid = threadIdx.x, n = a.info[4 * p];
    const int32_t *scores = a.scores + (int64_t)p * a.iters;
    __shared__ int ws[16], wi[16];
    __shared__ int best_s, best_i;
    int bs = -1, bi = -1;
    if (n > 4)
        for (int i = tid; i < a.iters; i += 1024)
            if (scores[i] > bs) bs = scores[i], bi = i;   // ascending i: the first of the max
    for (int off = 32; off > 0; off >>= 1) {
        const int s2 = __shfl_down(bs, off, 64), i2 = __shfl_down(bi, off, 64);
        if (s2 > bs || (s2 == bs && i2 >= 0 && (bi < 0 || i2 < bi))) bs = s2, bi = i2;
    }
    if ((tid & 63) == 0) ws[tid >> 6] = bs, wi[tid >> 6] = bi;
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < 16; w++)
            if (ws[w] > bs || (ws[w] == bs && wi[w] >= 0 && (bi < 0 || wi[w] < bi)))
                bs = ws[w], bi = wi[w];
        best_s = bs;
        best_i = bi;
        a.info[4 * p + 1] = bi;
        a.info[4 * p + 2] = bs;
    }
    __syncthreads();
    bs = best_s;
    bi = best_i;
    if (bs < 4) return;
    const double *h = a.hyps + ((int64_t)p * a.iters + bi) * 8;
    if (tid < 8) a.hbest[8 * p + tid] = h[tid];
    const double *pts = a.pts + (int64_t)4 * p * a.kstride;
    uint8_t *mask = a.mask + (int64_t)p * a.kstride;
    for (int i = tid; i < n; i += 1024) {
        const double *q = pts + 4 * (int64_t)i;
        mask[i] = rs_inlier(h, q[0], q[1], q[2], q[3], a.t2) ? 1 : 0;
    }
}

// ---- Graph-cut seams: push-relabel on one camera pair's overlap graph (KSeamFlowArgs) ----------
// grid (ceil(bw / 16), ceil(bh / 16)), block 256: one thread per grid point of the pair's box.
namespace mcs {

__device__ __forceinline__ bool seam_box_point(const KSeamFlowArgs &a, int &X, int &Y, int64_t &q)
{
    X = a.x0 + (int)blockIdx.x * kSeamTile + (int)(threadIdx.x % kSeamTile);
    Y = a.y0 + (int)blockIdx.y * kSeamTile + (int)(threadIdx.x / kSeamTile);
    q = (int64_t)Y * a.gw + X;
    return X < a.x0 + a.bw && Y < a.y0 + a.bh;
}

__device__ __forceinline__ bool seam_in(const KSeamFlowArgs &a, int64_t q)
{
    const uint32_t c = a.cov[q], l = a.lab[q];
    return ((c >> a.a) & 1u) && ((c >> a.b) & 1u) && (l == (uint32_t)a.a || l == (uint32_t)a.b);
}

__device__ __forceinline__ int32_t seam_cost(const KSeamFlowArgs &a, int64_t q)
{
    const uint8_t *pa = a.smp + ((int64_t)a.a * a.np + q) * a.cn;
    const uint8_t *pb = a.smp + ((int64_t)a.b * a.np + q) * a.cn;
    int32_t s = 0;
    for (int k = 0; k < a.cn; k++) s += abs((int)pa[k] - (int)pb[k]);
    return s;
}

// neighbour d of (X, Y) inside the grid, -1 outside
__device__ __forceinline__ int64_t seam_nb(const KSeamFlowArgs &a, int X, int Y, int64_t q, int d)
{
    switch (d) {
    case 0: return X + 1 < a.gw ? q + 1 : -1;
    case 1: return X > 0 ? q - 1 : -1;
    case 2: return Y + 1 < a.gh ? q + a.gw : -1;
    default: return Y > 0 ? q - a.gw : -1;
    }
}

template <class T>
__device__ __forceinline__ T seam_ld(const T *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace mcs

// The pair's graph: node mask, arc capacities e(q) + e(r) + 1 (e = sum over channels of
// |I_a - I_b|), terminals from the neighbours outside the graph (next to a's region: the
// original source arc -> here an arc to the sink; next to b's region: the original sink arc ->
// here the source's arc, saturated at once: excess kSeamBig).
extern "C" __global__ __launch_bounds__(256) void mcs_seam_flow_init(const mcs::KSeamFlowArgs a)
{
    using namespace mcs;
    int X, Y;
    int64_t q;
    if (!seam_box_point(a, X, Y, q)) return;
    const bool in = seam_in(a, q);
    a.in[q] = in ? 1 : 0;
    a.h[q] = kSeamHInf;
    long long sk = 0, e0 = 0;
    const int32_t eq = in ? seam_cost(a, q) : 0;
#pragma unroll
    for (int d = 0; d < 4; d++) {
        const int64_t r = seam_nb(a, X, Y, q, d);
        int32_t c = 0;
        if (in && r >= 0) {
            if (seam_in(a, r)) {
                c = eq + seam_cost(a, r) + 1;
            } else {
                if (a.lab[r] == (uint8_t)a.a) sk = kSeamBig;
                if (a.lab[r] == (uint8_t)a.b) e0 = kSeamBig;
            }
        }
        a.cap[d * a.np + q] = c;
    }
    a.snk[q] = sk;
    a.ex[q] = e0;
}

// Global relabel, first step: height 1 next to the sink, kSeamHInf elsewhere.
extern "C" __global__ __launch_bounds__(256) void mcs_seam_flow_hinit(const mcs::KSeamFlowArgs a)
{
    using namespace mcs;
    int X, Y;
    int64_t q;
    if (!seam_box_point(a, X, Y, q)) return;
    a.h[q] = a.in[q] && a.snk[q] > 0 ? 1 : kSeamHInf;
}

// Global relabel: `iters` rounds of h(u) = 1 + min h(v) over residual arcs u -> v (atomicMin:
// heights only fall), flag[0] set on any change.  A launch without a change is the fixpoint:
// the exact residual distances to the sink.
extern "C" __global__ __launch_bounds__(256) void mcs_seam_flow_relabel(const mcs::KSeamFlowArgs a)
{
    using namespace mcs;
    int X, Y;
    int64_t q;
    const bool live = seam_box_point(a, X, Y, q) && a.in[q];
    bool changed = false;
    for (int it = 0; it < a.iters; it++) {
        if (live) {
            int32_t hm = kSeamHInf;
#pragma unroll
            for (int d = 0; d < 4; d++) {
                if (seam_ld(&a.cap[d * a.np + q]) <= 0) continue;
                const int64_t r = seam_nb(a, X, Y, q, d);
                hm = min(hm, seam_ld(&a.h[r]));
            }
            if (hm < kSeamHInf && hm + 1 < seam_ld(&a.h[q])) {
                atomicMin(&a.h[q], hm + 1);
                changed = true;
            }
        }
        __syncthreads();
    }
    if (changed) atomicOr(&a.flag[0], 1);
}

// Global relabel, tiled: the block's 16 x 16 heights and their one-point ring staged in LDS,
// `iters` relaxation rounds there (LDS latency per round instead of an L2 round trip; the ring
// is the value other blocks had at the launch's start), then every lowered height written back
// with atomicMin and flag[0] set.  Launched until a launch changes nothing: the same fixpoint
// (exact residual distances to the sink) as mcs_seam_flow_relabel.
extern "C" __global__ __launch_bounds__(256) void mcs_seam_flow_relabel_lds(
    const mcs::KSeamFlowArgs a)
{
    using namespace mcs;
    constexpr int T = kSeamTile, R = kSeamTile + 2;
    __shared__ int32_t hl[R * R];
    __shared__ uint8_t arc[T * T];   // bit d: residual arc toward neighbour d (bit 4: the sink)
    int X, Y;
    int64_t q;
    const bool live = seam_box_point(a, X, Y, q) && a.in[q];
    const int tx = (int)(threadIdx.x % T), ty = (int)(threadIdx.x / T);
    // stage the tile and its ring (points outside the box or the graph: kSeamHInf)
    for (int i = threadIdx.x; i < R * R; i += 256) {
        const int lx = i % R - 1, ly = i / R - 1;
        const int gx = a.x0 + (int)blockIdx.x * T + lx, gy = a.y0 + (int)blockIdx.y * T + ly;
        int32_t v = kSeamHInf;
        if (gx >= 0 && gy >= 0 && gx < a.gw && gy < a.gh) {
            const int64_t r = (int64_t)gy * a.gw + gx;
            v = seam_ld(&a.h[r]);
        }
        hl[i] = v;
    }
    uint32_t m = 0;
    if (live) {
#pragma unroll
        for (int d = 0; d < 4; d++) m |= seam_ld(&a.cap[d * a.np + q]) > 0 ? 1u << d : 0u;
        m |= a.snk[q] > 0 ? 16u : 0u;
    }
    arc[threadIdx.x] = (uint8_t)m;
    __syncthreads();
    const int c = (ty + 1) * R + tx + 1;
    const int32_t h0 = hl[c];
    for (int it = 0; it < a.iters; it++) {
        if (live) {
            int32_t hm = (m & 16u) ? 0 : kSeamHInf;
            if (m & 1u) hm = min(hm, hl[c + 1]);
            if (m & 2u) hm = min(hm, hl[c - 1]);
            if (m & 4u) hm = min(hm, hl[c + R]);
            if (m & 8u) hm = min(hm, hl[c - R]);
            if (hm < kSeamHInf && hm + 1 < hl[c]) hl[c] = hm + 1;
        }
        __syncthreads();
    }
    if (live && hl[c] < h0) {
        atomicMin(&a.h[q], hl[c]);
        atomicOr(&a.flag[0], 1);
    }
}

// Push-relabel rounds (Hong's lock-free rule).  A node's own height changes only here (by its
// own thread) and in the global relabel, so it stays in a register for the launch; each round
// issues all of its loads at once (excess, sink and arc residuals, the four neighbours'
// heights): one L2 round trip per round.
extern "C" __global__ __launch_bounds__(256) void mcs_seam_flow_push(const mcs::KSeamFlowArgs a)
{
    using namespace mcs;
    int X, Y;
    int64_t q;
    const bool live = seam_box_point(a, X, Y, q) && a.in[q];
    int64_t nb[4];
#pragma unroll
    for (int d = 0; d < 4; d++) {
        const int64_t r = live ? seam_nb(a, X, Y, q, d) : -1;
        nb[d] = r >= 0 ? r : q;
    }
    int32_t hu = live ? a.h[q] : kSeamHInf;
    for (int it = 0; it < a.iters; it++) {
        if (live && hu < kSeamHInf) {
            const long long e = seam_ld(&a.ex[q]);
            const long long sk = seam_ld(&a.snk[q]);
            int32_t c[4], hv[4];
#pragma unroll
            for (int d = 0; d < 4; d++) {
                c[d] = seam_ld(&a.cap[d * a.np + q]);
                hv[d] = seam_ld(&a.h[nb[d]]);
            }
            if (e > 0) {
                // the lowest residual target: the sink (height 0) or a neighbour
                int best = sk > 0 ? 4 : -1;
                int32_t hm = sk > 0 ? 0 : kSeamHInf;
#pragma unroll
                for (int d = 0; d < 4; d++)
                    if (c[d] > 0 && hv[d] < hm) hm = hv[d], best = d;
                if (best < 0 || hm >= a.hmax - 1) {
                    hu = kSeamHInf;                        // no way to the sink
                    atomicExch(&a.h[q], hu);
                } else if (hu > hm) {
                    if (best == 4) {
                        const long long dl = min(e, sk);
                        atomicAdd((unsigned long long *)&a.snk[q], (unsigned long long)(-dl));
                        atomicAdd((unsigned long long *)&a.ex[q], (unsigned long long)(-dl));
                    } else {
                        const long long dl = min(e, (long long)c[best]);
                        const int64_t rb = nb[best];
                        atomicSub(&a.cap[best * a.np + q], (int32_t)dl);
                        atomicAdd(&a.cap[(best ^ 1) * a.np + rb], (int32_t)dl);
                        atomicAdd((unsigned long long *)&a.ex[rb], (unsigned long long)dl);
                        atomicAdd((unsigned long long *)&a.ex[q], (unsigned long long)(-dl));
                    }
                } else {
                    hu = hm + 1;                           // relabel
                    atomicExch(&a.h[q], hu);
                }
            }
        }
        __syncthreads();
    }
}

// Nodes with excess that can still reach the sink (after a global relabel) -> flag[1].
extern "C" __global__ __launch_bounds__(256) void mcs_seam_flow_active(const mcs::KSeamFlowArgs a)
{
    using namespace mcs;
    int X, Y;
    int64_t q;
    const bool act = seam_box_point(a, X, Y, q) && a.in[q] && a.ex[q] > 0 && a.h[q] < kSeamHInf;
    const unsigned long long b = __ballot(act);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(&a.flag[1], (int)__popcll(b));
}

// The cut: nodes that reach the sink (the a side) keep camera a, the others take b.
extern "C" __global__ __launch_bounds__(256) void mcs_seam_flow_label(const mcs::KSeamFlowArgs a)
{
    using namespace mcs;
    int X, Y;
    int64_t q;
    if (!seam_box_point(a, X, Y, q) || !a.in[q]) return;
    a.lab[q] = (uint8_t)(a.h[q] < kSeamHInf ? a.a : a.b);
}

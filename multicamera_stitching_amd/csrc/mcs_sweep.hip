// mcs_sweep.hip -- the multi-band sweep: band pass and blend of the
// 3-level multi-band blend fused into one gfx950 kernel, bit-exact to oracle/orc_blend.c (the
// specification: integer Gaussian pyramids of every owner's replicate-border warp, integer masks,
// IEEE doubles in a fixed order for B2 / R1 / R0).
//
// The stitch kernels (mcs_kernels.hip) write every mosaic pixel from its owner camera except the
// pixels of the sweep's output regions; this kernel writes those.  A strip (MbStrip, built once
// per plan by mcs_capi.cpp prepare_sweep) is a 128-column window over a run of blend-tile rows
// around one seam region, with the <= 4 owners whose masks reach its region.  One workgroup per
// (strip, capture), 128 threads per owner, walks the window top to bottom, 4 level-0 rows per step
// in three phases separated by barriers:
//
//   A  producer: each thread (owner j, column l) samples its 4 rows (window descriptors from the
//      plan's table, the source rows by dword-aligned global loads issued a step ahead), adds them
//      into three rolling vertical 5-tap sums (registers) and writes the two finished level-1
//      columns sums to LDS (s1); the owner's sample of a pixel goes to the level-0 ring (g0).
//      The owner mask m0 = (owner == j) rides along as channel 3 of the packed u16 lanes, so the
//      masks m1 / m2 come out of the same reduces as the image levels.
//      consumer: R0 = L0_owner / 16384 + up(R1) / 64 for the output rows 18..15 above the
//      step's first level-0 row -> bytes to the mosaic.
//   B  producer: level-1 horizontal 5-tap of the two rows (thread = owner, level-1 column) into
//      the level-1 ring; their values feed the rolling vertical level-2 sums; a finished level-2
//      row's column sums to LDS (s2).  consumer: B2 = sum m2 g2 / (sum m2 * 65536), 2 rows up.
//   C  producer: level-2 horizontal 5-tap into the level-2 ring.  consumer: R1 = B1 + up(B2),
//      B1 = sum m1 (16384 g1 - up(g2)) / (sum m1 * 4194304), two level-1 rows.
//
// Rows and columns past a mosaic edge: level-0 samples at reflected positions (descriptors);
// level-1 / level-2 entries are always read at reflected coordinates (rows / columns past the
// bottom / right edge are never computed into the rings; past the top / left edge reflect-101
// commutes with the decimation), so every read is the specification's value.  Ring depths follow
// the step schedule: R0 of rows y reads R1 rows written one step earlier, R1 reads B2 rows of the
// same step's phase B, B2 reads level-2 rows of the previous step's phase C.
#include "mcs_dev.h"

#include "mcs_blend.h"

namespace mcs {

template <int CN, int JB>
struct SwLds {
    uint32_t g0[kSwNG0 + 1][kSwCols];        // owner sample (bytes 0..2) | local owner << 24
                                             // (row kSwNG0: the writes of non-owners)
    uint2 s1[2][JB][kSwCols];                // finished vertical level-1 sums (u16 lanes)
    uint2 g1[JB][kSwNG1][kSwCols / 2];       // level 1: x = (c0, c2), y = (c1, m)
    int4 s2[JB][kSwCols / 2];                // finished vertical level-2 sums (c0, c1, c2, m)
    int4 g2[JB][kSwNG2][kSwCols / 4];        // level 2
    double b2[kSwNB2][kSwMaxB2][CN];
    double r1[kSwNR1][kSwMaxR1][CN];
};

// Reflect-101 of i into [0, n) for -n < i < 2n - 1.
__device__ __forceinline__ int sw_refl(int i, int n)
{
    i = i < 0 ? -i : i;
    return i >= n ? 2 * n - 2 - i : i;
}

// Expand taps of fine coordinate x into a coarse level of size n (reflected), as exp_taps:
// returns the tap count (3 even, 2 odd).
__device__ __forceinline__ int sw_taps(int x, int n, int *idx, int *wt)
{
    if ((x & 1) == 0) {
        const int h = x >> 1;
        idx[0] = sw_refl(h - 1, n), wt[0] = 1;
        idx[1] = sw_refl(h, n), wt[1] = 6;
        idx[2] = sw_refl(h + 1, n), wt[2] = 1;
        return 3;
    }
    idx[0] = sw_refl((x - 1) >> 1, n), wt[0] = 4;
    idx[1] = sw_refl((x + 1) >> 1, n), wt[1] = 4;
    idx[2] = idx[1], wt[2] = 0;
    return 2;
}

// (a + e) + 4 (b + d) + 6 c for packed u16 lanes (no carry between lanes: every lane sum <= 65280)
__device__ __forceinline__ uint32_t sw_h5(uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                          uint32_t e)
{
    return mad6_u32(c, (a + e) + 4u * (b + d));
}

__device__ __forceinline__ int sw_ch(uint2 v, int k)
{
    return (int)((((k & 1) ? v.y : v.x) >> ((k & 2) ? 16 : 0)) & 0xffffu);
}

__device__ __forceinline__ int sw_i4(const int4 &v, int k)
{
    return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));
}

// Ring slot of row i for a ring of N rows (i > -N * 64).
template <int N>
__device__ __forceinline__ int sw_slot(int i)
{
    return (int)((unsigned)(i + 64 * N) % (unsigned)N);
}

// Plan slot of owner j (uniform j; no dynamic indexing of the register copy).
__device__ __forceinline__ int strip_slot(const MbStrip &S, int j)
{
    return j == 0 ? S.slot[0] : (j == 1 ? S.slot[1] : (j == 2 ? S.slot[2] : S.slot[3]));
}

template <int CN, int JB, bool AL>
__device__ __forceinline__ void mb_sweep(const KMbSweepArgs &a, SwLds<CN, JB> &L)
{
    typedef __attribute__((address_space(1))) const uint8_t gu8;
    struct __attribute__((packed)) U2 {
        uint32_t x, y;
    };
    struct U3 {
        uint32_t x, y, z;
    };
    typedef __attribute__((address_space(1))) const U2 gu2;
    typedef __attribute__((address_space(1))) const U3 gu3;
    typedef std::conditional_t<AL, uint3, uint2> Win;
    constexpr int T = kSwCols * JB;
    constexpr int C1 = kSwCols / 2;
    const KParams &P = a.P;
    int si, fl;
    if (!xcd_unit(a.n_strips, a.nf, si, fl)) return;   // (block-uniform, before any barrier)
    const MbStrip S = a.strips[si];
    const int tid = threadIdx.x;
    const int ns = S.ns, c0 = S.c0, c1 = c0 >> 1, c2 = c0 >> 2;
    const int W = P.out_w, H = P.out_h;
    const int w1 = (W + 1) / 2, h1 = (H + 1) / 2, w2 = (w1 + 1) / 2, h2 = (h1 + 1) / 2;
    const int f = a.f0 + fl;
    const int K0 = S.r0 >> 2;              // r0 = 4 K0 (K0 may be negative)
    const int nsteps = S.nsteps, nrows = 4 * nsteps + kSwDescPad;
    const int ya = S.ya, yb = S.yb;
    const int e1lo = S.e1lo, e1n = S.e1n, z2lo = S.z2lo, z2n = S.z2n;
    // ---- producer role: owner pj (wave-uniform), column pl
    const int pj = __builtin_amdgcn_readfirstlane(tid >> 7), pl = tid & (kSwCols - 1);
    const bool prod = pj < ns;
    int cam = 0, sw = 2, shh = 2;
    if (prod) slot_info(P, strip_slot(S, pj), cam, sw, shh);
    const uint32_t pitch = (uint32_t)(sw * CN);
    const gu8 *fb = (const gu8 *)(P.cams[cam] + (int64_t)f * P.cam_fstride[cam]);
    const uint64_t *dp = a.sdesc + ((int64_t)S.dsc + (int64_t)(prod ? pj : 0) * nrows) * kSwCols + pl;
    // descriptor ring: row r in slot r % 12, loaded 8 rows ahead; windows: row r in slot r % 6,
    // loaded 4 rows ahead.  A new load never targets the slot just read (loaded into the same
    // registers, the compiler scheduled the load above the old value's use and then copied the
    // registers at the loop's back edge, waiting for every load in flight).
    uint2 D[12];
    Win Wa[6], Wb[6];
    auto load_desc = [&](int row) -> uint2 {
        const uint64_t v = dp[(int64_t)row * kSwCols];
        return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
    };
    auto load_win = [&](uint2 d, Win &wa, Win &wb) {
        const uint32_t sh = AL ? (d.y >> 15) & 15u : (d.y >> 12) & 7u;
        const uint32_t o = (d.x & 0x7fffffffu) - sh, ob = o + ((d.x >> 31) ? pitch : 0u);
        if constexpr (AL) {
            const U3 ra = *(const gu3 *)(fb + o), rb = *(const gu3 *)(fb + ob);
            wa = make_uint3(ra.x, ra.y, ra.z);
            wb = make_uint3(rb.x, rb.y, rb.z);
        } else {
            const U2 ra = *(const gu2 *)(fb + o), rb = *(const gu2 *)(fb + ob);
            wa = make_uint2(ra.x, ra.y);
            wb = make_uint2(rb.x, rb.y);
        }
    };
    // (every wave runs the producer code -- a wave past the strip's owners samples owner 0's
    // rows into its own unused s1 slot and writes no level-0 ring entry: a conditional producer
    // block made the compiler copy the in-flight window registers at its join, draining the loads)
#pragma unroll
    for (int q = 0; q < 8; q++) D[q] = load_desc(q);
#pragma unroll
    for (int t = 0; t < 4; t++) load_win(D[t], Wa[t], Wb[t]);
    // one level-0 sample: (c0, c2) and (c1, m) as u16 lanes, and the level-0 ring word
    auto sample = [&](uint2 d, const Win &wa, const Win &wb, uint32_t &pl_, uint32_t &ph_,
                      uint32_t &g0w, bool &wr) {
        uint32_t wA, wB;
        mb_weights2(d.y, wA, wB);
        uint2 r0, r1;
        uint32_t dd = 0u;
        if constexpr (AL) {
            const uint32_t sh = (d.y >> 15) & 15u;
            r0 = mb_win_shift<CN>(wa, sh);
            r1 = mb_win_shift<CN>(wb, sh);
        } else {
            r0 = wa;
            r1 = wb;
            dd = (d.y >> 12) & 7u;
        }
        uint32_t t[3];
#pragma unroll
        for (int c = 0; c < 3; c++) t[c] = c < CN ? mb_tap2<CN>(r0, r1, wA, wB, c, dd) : 0u;
        const uint32_t own = d.y >> 31, none = (d.y >> 30) & 1u;
        // channel k of the sample = byte 2 of t[k]
        if constexpr (CN == 3) pl_ = __builtin_amdgcn_perm(t[2], t[0], 0x0c060c02u);
        else pl_ = (t[0] >> 16) & 0xffu;
        ph_ = (CN >= 2 ? (t[1] >> 16) & 0xffu : 0u) | (own << 16);
        const uint32_t px = ((t[0] >> 16) & 0xffu) | (CN >= 2 ? ((t[1] >> 8) & 0xff00u) : 0u) |
                            (CN >= 3 ? (t[2] & 0xff0000u) : 0u);
        g0w = own ? px | ((uint32_t)pj << 24) : 0xff000000u;
        wr = (own | (pj == 0 ? none : 0u)) != 0u;
    };
    uint32_t Al[3] = {0u, 0u, 0u}, Ah[3] = {0u, 0u, 0u};   // rolling level-1 sums
    int4 A2[3];                                               // rolling level-2 sums (phase B)
#pragma unroll
    for (int q = 0; q < 3; q++) A2[q] = make_int4(0, 0, 0, 0);
    // ---- phase B / C roles
    const int j2 = __builtin_amdgcn_readfirstlane(tid >> 6), e = tid & 63;   // level-1 producer
    const bool p2 = j2 < ns;
    const int j3 = tid >> 5, e2 = tid & 31;   // level-2 producer (two owners per wave)
    const bool p3 = j3 < ns;
    typedef __attribute__((address_space(1))) uint8_t g8;
    g8 *const outf = (g8 *)(P.out + (int64_t)f * P.out_fstride);
    // region entry (xa | xb << 16) of output row y, 0 outside [ya, yb)
    // (scalar loads through the constant address space: they count in lgkmcnt, so waiting for
    // them never drains the window loads in flight -- a vector load here made the compiler wait
    // vmcnt for it, behind every window load issued before it)
    typedef __attribute__((address_space(4))) const int ci32;
    const ci32 *rgn = (const ci32 *)a.region + S.reg - ya;
    auto load_reg = [&](int y) -> int { return rgn[min(max(y, ya), yb - 1)]; };
    int regn[4];
#pragma unroll
    for (int rr = 0; rr < 4; rr++) regn[rr] = load_reg(S.r0 - 18 + rr);   // step 0's rows

    for (int s3 = 0; s3 < nsteps; s3 += 3) {
        static_for<3>([&](auto SMc) {
            constexpr int sm = decltype(SMc)::value;
            const int s = s3 + sm, k = K0 + s;
            // ================= phase A: sample 4 rows; R0 of rows 4k - 18 .. 4k - 15
            {
                static_for<4>([&](auto TTc) {
                    constexpr int t = decltype(TTc)::value, q = 4 * sm + t, w = q % 6;
                    const int lr = 4 * s + t;                 // row index in the strip
                    uint32_t pl_, ph_, g0w;
                    bool wr;
                    sample(D[q], Wa[w], Wb[w], pl_, ph_, g0w, wr);
                    // (branch-free: rows past the ring take the entries nobody reads)
                    L.g0[(prod && wr) ? sw_slot<kSwNG0>(lr) : kSwNG0][pl] = g0w;
                    // loads: windows of row lr + 4, descriptor of row lr + 8
                    load_win(D[(q + 4) % 12], Wa[(q + 4) % 6], Wb[(q + 4) % 6]);
                    D[(q + 8) % 12] = load_desc(lr + 8);
                    // vertical 5-tap (level-1 row m of the strip: accumulator m % 3, rows
                    // 2s - 1 and 2s finish at t = 0 and t = 2)
                    constexpr int a0 = (2 * sm + 2) % 3, a1 = (2 * sm) % 3, a2 = (2 * sm + 1) % 3;
                    if constexpr (t == 0) {
                        L.s1[0][pj][pl] = make_uint2(Al[a0] + pl_, Ah[a0] + ph_);
                        Al[a1] += __umul24(pl_, 6u), Ah[a1] += __umul24(ph_, 6u);
                        Al[a2] = pl_, Ah[a2] = ph_;
                    } else if constexpr (t == 1) {
                        Al[a1] += 4u * pl_, Ah[a1] += 4u * ph_;
                        Al[a2] += 4u * pl_, Ah[a2] += 4u * ph_;
                    } else if constexpr (t == 2) {
                        L.s1[1][pj][pl] = make_uint2(Al[a1] + pl_, Ah[a1] + ph_);
                        Al[a2] += __umul24(pl_, 6u), Ah[a2] += __umul24(ph_, 6u);
                        Al[a0] = pl_, Ah[a0] = ph_;
                    } else {
                        Al[a2] += 4u * pl_, Ah[a2] += 4u * ph_;
                        Al[a0] += 4u * pl_, Ah[a0] += 4u * ph_;
                    }
                });
            }
            {
                // R0: rows y0r .. y0r + 3 (inside [ya, yb)), columns [xa, xb) of each row (the
                // region entries were loaded a step ahead; the next step's are issued here)
                const int y0r = 4 * k - 18;
                int xa_[4], nx_[4], tot = 0;
#pragma unroll
                for (int rr = 0; rr < 4; rr++) {
                    const int v = (y0r + rr >= ya && y0r + rr < yb) ? regn[rr] : 0;
                    xa_[rr] = v & 0xffff;
                    nx_[rr] = (v >> 16) - (v & 0xffff);
                    tot += nx_[rr];
                    regn[rr] = load_reg(y0r + 4 + rr);
                }
                for (int u = tid; u < tot; u += T) {
                    int rr = 0, x = u;
                    if (x >= nx_[0]) {
                        x -= nx_[0], rr = 1;
                        if (x >= nx_[1]) {
                            x -= nx_[1], rr = 2;
                            if (x >= nx_[2]) x -= nx_[2], rr = 3;
                        }
                    }
                    const int y = y0r + rr;
                    x += rr == 0 ? xa_[0] : (rr == 1 ? xa_[1] : (rr == 2 ? xa_[2] : xa_[3]));
                    const uint32_t gv = L.g0[sw_slot<kSwNG0>(y - S.r0)][x - c0];
                    const int jo = (int)(gv >> 24);
                    uint32_t outw = 0u;
                    if (jo != 255) {
                        int iy[3], wy[3], ix[3], wx[3];
                        const int ny = sw_taps(y, h1, iy, wy), nx = sw_taps(x, w1, ix, wx);
                        int e1[CN];
                        double acc[CN];
#pragma unroll
                        for (int kk = 0; kk < CN; kk++) e1[kk] = 0, acc[kk] = 0.0;
#pragma unroll
                        for (int uu = 0; uu < 3; uu++) {
                            if (uu == 2 && ny == 2) break;
                            const int sl1 = sw_slot<kSwNG1>(iy[uu]), sr = iy[uu] & (kSwNR1 - 1);
#pragma unroll
                            for (int vv = 0; vv < 3; vv++) {
                                if (vv == 2 && nx == 2) break;
                                const int wt = wy[uu] * wx[vv];
                                const uint2 g = L.g1[jo][sl1][ix[vv] - c1];
                                const double wd = (double)wt;
#pragma unroll
                                for (int kk = 0; kk < CN; kk++) {
                                    e1[kk] += wt * sw_ch(g, kk);
                                    acc[kk] += wd * L.r1[sr][ix[vv] - e1lo][kk];
                                }
                            }
                        }
#pragma unroll
                        for (int kk = 0; kk < CN; kk++) {
                            const int l0 = 16384 * (int)((gv >> (8 * kk)) & 0xffu) - e1[kk];
                            const double r0 = (double)l0 / 16384.0 + acc[kk] / 64.0;
                            const double vf = floor(r0 + 0.5);
                            outw |= (uint32_t)(vf < 0.0 ? 0.0 : (vf > 255.0 ? 255.0 : vf))
                                    << (8 * kk);
                        }
                    }
                    g8 *po = outf + (int64_t)y * P.out_pitch + (int64_t)x * CN;
#pragma unroll
                    for (int kk = 0; kk < CN; kk++) po[kk] = (uint8_t)(outw >> (8 * kk));
                }
            }
            __syncthreads();
            // ================= phase B: level-1 horizontal + vertical level-2; B2 of row k - 2
            if (p2) {
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int i = 2 * k - 1 + h;               // level-1 row
                    const uint2 *sr = L.s1[h][j2];
                    const int b = 2 * e;
                    const uint2 va = sr[max(b - 2, 0)], vb = sr[max(b - 1, 0)], vc = sr[b],
                                vd = sr[b + 1], ve = sr[min(b + 2, kSwCols - 1)];
                    uint2 g = make_uint2(sw_h5(va.x, vb.x, vc.x, vd.x, ve.x),
                                         sw_h5(va.y, vb.y, vc.y, vd.y, ve.y));
                    if (i < h1) L.g1[j2][sw_slot<kSwNG1>(i)][e] = g;
                    else g = L.g1[j2][sw_slot<kSwNG1>(sw_refl(i, h1))][e];
                    const int4 v = make_int4((int)(g.x & 0xffffu), (int)(g.y & 0xffffu),
                                             (int)(g.x >> 16), (int)(g.y >> 16));
                    // level-2 rows (strip-relative z - K0): odd level-1 row 2k - 1 feeds rows
                    // k - 1, k (4, 4); even row 2k finishes k - 1 (+1), feeds k (6), starts k + 1
                    constexpr int b0 = (sm + 2) % 3, b1 = sm % 3, b2i = (sm + 1) % 3;
                    auto add = [](int4 &x, const int4 &y, int m) {
                        x.x += m * y.x, x.y += m * y.y, x.z += m * y.z, x.w += m * y.w;
                    };
                    if (h == 0) {
                        add(A2[b0], v, 4);
                        add(A2[b1], v, 4);
                    } else {
                        add(A2[b0], v, 1);
                        L.s2[j2][e] = A2[b0];
                        add(A2[b1], v, 6);
                        A2[b2i] = v;
                    }
                }
            }
            {
                const int u = tid - 64 * JB, z = k - 2;
                if (u >= 0 && u < z2n && z >= 0 && z < h2) {
                    const int el = z2lo + u - c2;
                    double num[CN];
                    int den = 0;
#pragma unroll
                    for (int kk = 0; kk < CN; kk++) num[kk] = 0.0;
                    for (int j = 0; j < ns; j++) {
                        const int4 g = L.g2[j][z & (kSwNG2 - 1)][el];
                        const double m = (double)g.w;
#pragma unroll
                        for (int kk = 0; kk < CN; kk++) num[kk] += m * (double)sw_i4(g, kk);
                        den += g.w;
                    }
#pragma unroll
                    for (int kk = 0; kk < CN; kk++)
                        L.b2[z & (kSwNB2 - 1)][u][kk] =
                            den ? num[kk] / ((double)den * 65536.0) : 0.0;
                }
            }
            __syncthreads();
            // ================= phase C: level-2 horizontal (row k - 1); R1 of rows 2k - 6, 2k - 5
            if (p3) {
                const int z = k - 1;
                if (z < h2) {
                    const int Z = c2 + e2;
                    int4 acc = make_int4(0, 0, 0, 0);
#pragma unroll
                    for (int v = 0; v < 5; v++) {
                        const int wv = v == 2 ? 6 : ((v & 1) ? 4 : 1);
                        const int q = min(max(sw_refl(2 * Z - 2 + v, w1) - c1, 0), C1 - 1);
                        const int4 t = L.s2[j3][q];
                        acc.x += wv * t.x, acc.y += wv * t.y, acc.z += wv * t.z, acc.w += wv * t.w;
                    }
                    L.g2[j3][z & (kSwNG2 - 1)][e2] = acc;
                }
            }
            {
                const int u = tid - 32 * JB;
                if (u >= 0 && u < 2 * e1n) {
                    const int rr = u >= e1n ? 1 : 0;
                    const int q = 2 * k - 6 + rr, E = e1lo + u - rr * e1n;
                    if (q >= 0 && q < h1) {
                        int iy[3], wy[3], ix[3], wx[3];
                        const int ny = sw_taps(q, h2, iy, wy), nx = sw_taps(E, w2, ix, wx);
                        const int el = E - c1, sl1 = sw_slot<kSwNG1>(q);
                        double num[CN];
                        int den = 0;
#pragma unroll
                        for (int kk = 0; kk < CN; kk++) num[kk] = 0.0;
                        for (int j = 0; j < ns; j++) {
                            int e2v[CN];   // <= 64 * 65536 * 255 < 2^31
#pragma unroll
                            for (int kk = 0; kk < CN; kk++) e2v[kk] = 0;
#pragma unroll
                            for (int uu = 0; uu < 3; uu++) {
                                if (uu == 2 && ny == 2) break;
#pragma unroll
                                for (int vv = 0; vv < 3; vv++) {
                                    if (vv == 2 && nx == 2) break;
                                    const int wt = wy[uu] * wx[vv];
                                    const int4 g2 = L.g2[j][iy[uu] & (kSwNG2 - 1)][ix[vv] - c2];
#pragma unroll
                                    for (int kk = 0; kk < CN; kk++) e2v[kk] += wt * sw_i4(g2, kk);
                                }
                            }
                            const uint2 g1 = L.g1[j][sl1][el];
                            const int m1 = (int)(g1.y >> 16);
                            const double md = (double)m1;
#pragma unroll
                            for (int kk = 0; kk < CN; kk++)
                                num[kk] += md * (double)(16384 * sw_ch(g1, kk) - e2v[kk]);
                            den += m1;
                        }
                        double acc[CN];
#pragma unroll
                        for (int kk = 0; kk < CN; kk++) acc[kk] = 0.0;
#pragma unroll
                        for (int uu = 0; uu < 3; uu++) {
                            if (uu == 2 && ny == 2) break;
#pragma unroll
                            for (int vv = 0; vv < 3; vv++) {
                                if (vv == 2 && nx == 2) break;
                                const double wt = (double)(wy[uu] * wx[vv]);
#pragma unroll
                                for (int kk = 0; kk < CN; kk++)
                                    acc[kk] += wt * L.b2[iy[uu] & (kSwNB2 - 1)][ix[vv] - z2lo][kk];
                            }
                        }
#pragma unroll
                        for (int kk = 0; kk < CN; kk++) {
                            const double b1 = den ? num[kk] / ((double)den * 4194304.0) : 0.0;
                            L.r1[q & (kSwNR1 - 1)][E - e1lo][kk] = b1 + acc[kk] / 64.0;
                        }
                    }
                }
            }
            __syncthreads();
        });
    }
}

// Window descriptors of every strip (once per plan): grid (strips, kSwMaxOwners), block 256.  Per
// (owner j, strip row, column) mb_desc of the owner's replicate-border sample at the reflected
// mosaic position, bit 31 of .y = that position's owner is j, bit 30 (owner 0's rows only) = it
// has no owner.
template <int CN, int INTERP>
__device__ __forceinline__ void mb_sweep_desc(const KMbSweepArgs &a)
{
    const KParams &P = a.P;
    const MbStrip S = a.strips[blockIdx.x];
    const int j = blockIdx.y;
    if (j >= S.ns) return;
    const int slot = strip_slot(S, j);
    int cam, w, h;
    slot_info(P, slot, cam, w, h);
    const int nrows = 4 * S.nsteps + kSwDescPad;
    uint64_t *o = a.sdesc + ((int64_t)S.dsc + (int64_t)j * nrows) * kSwCols;
    for (int i = threadIdx.x; i < nrows * kSwCols; i += blockDim.x) {
        const int r = i / kSwCols, l = i % kSwCols;
        const int x = refl(S.c0 + l, P.out_w), y = refl(S.r0 + r, P.out_h);
        uint2 v = mb_desc<CN>(mb_src<INTERP>(P, slot, x, y), w, h);
        const int own = a.owner[(int64_t)y * P.out_w + x];
        if (own == slot) v.y |= 1u << 31;
        if (j == 0 && own == kBlendNone) v.y |= 1u << 30;
        o[i] = (uint64_t)v.x | ((uint64_t)v.y << 32);
    }
}

}  // namespace mcs

// Entry points: mcs_mb_sweep{_a}_c{CN}_j{JB} (grid 8 * ceil(strips * captures / 8), block
// 128 * JB; _a = dword-aligned window loads), mcs_mb_sweep_desc_c{CN}_i{INTERP} (grid (strips,
// kSwMaxOwners), block 256).
#define MCS_SWEEP_ENTRY(CN, JB, SFX, AL)                                                       \
    extern "C" __global__ __launch_bounds__(128 * JB) void mcs_mb_sweep##SFX##_c##CN##_j##JB(  \
        const mcs::KMbSweepArgs a)                                                             \
    {                                                                                          \
        __shared__ mcs::SwLds<CN, JB> lds;                                                     \
        mcs::mb_sweep<CN, JB, AL>(a, lds);                                                     \
    }
#define MCS_SWEEP_DESC_ENTRY(CN, IN)                                                           \
    extern "C" __global__ __launch_bounds__(256) void mcs_mb_sweep_desc_c##CN##_i##IN(         \
        const mcs::KMbSweepArgs a)                                                             \
    {                                                                                          \
        mcs::mb_sweep_desc<CN, IN>(a);                                                         \
    }
#define MCS_SWEEP_ENTRIES(CN)                                                                  \
    MCS_SWEEP_ENTRY(CN, 2, , false)                                                            \
    MCS_SWEEP_ENTRY(CN, 4, , false)                                                            \
    MCS_SWEEP_ENTRY(CN, 2, _a, true)                                                           \
    MCS_SWEEP_ENTRY(CN, 4, _a, true)                                                           \
    MCS_SWEEP_DESC_ENTRY(CN, 0)                                                                \
    MCS_SWEEP_DESC_ENTRY(CN, 1)
MCS_SWEEP_ENTRIES(1)
MCS_SWEEP_ENTRIES(2)
MCS_SWEEP_ENTRIES(3)

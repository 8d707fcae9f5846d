// mcs_seam.cpp -- graph-cut seam labels (include/mcs.h
// mcs_plan_find_seams).  Calibration time, once per plan (as OpenCV's seam finders run once on
// reduced images): the per-point inputs come from the plan's device kernels
// (mcs_seam_sample_*), then one minimum cut per camera pair on its 4-connected overlap graph --
// on the device by push-relabel (seam_graphcut_device, kernels mcs_seam_flow_* in
// mcs_features.hip), or here on the host with Dinic's algorithm (seam_graphcut: the C-ABI's
// mcs_seam_graphcut_host, and the cross-check of the device path).  Specification in
// oracle/orc_seam.c (restated there with a third max-flow algorithm); all return the source side
// of the minimal minimum cut, which every maximum flow shares.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <vector>

#include "mcs_common.h"
#include "mcs_feat_int.h"

namespace {

constexpr int64_t kBig = int64_t(1) << 40;

class Dinic {
public:
    explicit Dinic(int n) : head_(n, -1), level_(n), it_(n) {}

    void arc(int u, int v, int64_t c, int64_t rc)
    {
        to_.push_back(v), cap_.push_back(c), next_.push_back(head_[u]);
        head_[u] = (int)to_.size() - 1;
        to_.push_back(u), cap_.push_back(rc), next_.push_back(head_[v]);
        head_[v] = (int)to_.size() - 1;
    }

    // Maximum flow s -> t; afterwards reach[v] = v reachable from s in the residual graph.
    void run(int s, int t, std::vector<uint8_t> &reach)
    {
        while (levels(s, t)) {
            it_ = head_;
            blocking(s, t);
        }
        reach.assign(head_.size(), 0);
        std::vector<int> q{s};
        reach[s] = 1;
        for (size_t i = 0; i < q.size(); i++)
            for (int e = head_[q[i]]; e >= 0; e = next_[e])
                if (cap_[e] > 0 && !reach[to_[e]]) reach[to_[e]] = 1, q.push_back(to_[e]);
    }

private:
    bool levels(int s, int t)
    {
        std::fill(level_.begin(), level_.end(), -1);
        std::vector<int> q{s};
        level_[s] = 0;
        for (size_t i = 0; i < q.size(); i++)
            for (int e = head_[q[i]]; e >= 0; e = next_[e])
                if (cap_[e] > 0 && level_[to_[e]] < 0) {
                    level_[to_[e]] = level_[q[i]] + 1;
                    q.push_back(to_[e]);
                }
        return level_[t] >= 0;
    }

    // Blocking flow on the level graph, iterative (paths can be as long as the overlap).
    void blocking(int s, int t)
    {
        std::vector<int> path;
        int u = s;
        for (;;) {
            if (u == t) {
                int64_t b = kBig * 4;
                for (int e : path) b = std::min(b, cap_[e]);
                size_t first = path.size();
                for (size_t i = 0; i < path.size(); i++) {
                    cap_[path[i]] -= b;
                    cap_[path[i] ^ 1] += b;
                    if (cap_[path[i]] == 0 && first == path.size()) first = i;
                }
                u = to_[path[first] ^ 1];
                path.resize(first);
                continue;
            }
            int &e = it_[u];
            while (e >= 0 && !(cap_[e] > 0 && level_[to_[e]] == level_[u] + 1)) e = next_[e];
            if (e >= 0) {
                path.push_back(e);
                u = to_[e];
                continue;
            }
            if (u == s) return;
            level_[u] = -1;   // dead end: no longer on the level graph
            const int pe = path.back();
            path.pop_back();
            u = to_[pe ^ 1];
            it_[u] = next_[it_[u]];
        }
    }

    std::vector<int> head_, next_, to_, level_, it_;
    std::vector<int64_t> cap_;
};

}  // namespace

namespace mcs {

int seam_graphcut(int n_cams, int gw, int gh, uint8_t *lab, const uint16_t *cov,
                  const uint8_t *smp, int cn)
{
    const int64_t np = (int64_t)gw * gh;
    std::vector<int> id(np);
    std::vector<int32_t> e(np);
    std::vector<uint8_t> reach;
    for (int a = 0; a < n_cams; a++)
        for (int b = a + 1; b < n_cams; b++) {
            int n = 0;
            for (int64_t q = 0; q < np; q++) {
                const bool in = ((cov[q] >> a) & 1) && ((cov[q] >> b) & 1) &&
                                (lab[q] == a || lab[q] == b);
                id[q] = in ? n++ : -1;
                if (!in) continue;
                int32_t s = 0;
                for (int k = 0; k < cn; k++)
                    s += std::abs((int)smp[((int64_t)a * np + q) * cn + k] -
                                  (int)smp[((int64_t)b * np + q) * cn + k]);
                e[q] = s;
            }
            if (n == 0) continue;
            Dinic g(n + 2);
            const int S = n, T = n + 1;
            for (int64_t q = 0; q < np; q++) {
                if (id[q] < 0) continue;
                const int X = (int)(q % gw), Y = (int)(q / gw);
                if (X + 1 < gw && id[q + 1] >= 0) {
                    const int64_t w = (int64_t)e[q] + e[q + 1] + 1;
                    g.arc(id[q], id[q + 1], w, w);
                }
                if (Y + 1 < gh && id[q + gw] >= 0) {
                    const int64_t w = (int64_t)e[q] + e[q + gw] + 1;
                    g.arc(id[q], id[q + gw], w, w);
                }
                bool src = false, snk = false;
                const int64_t nb[4] = {X > 0 ? q - 1 : -1, X + 1 < gw ? q + 1 : -1,
                                       Y > 0 ? q - gw : -1, Y + 1 < gh ? q + gw : -1};
                for (int64_t r : nb) {
                    if (r < 0 || id[r] >= 0) continue;
                    src = src || lab[r] == a;
                    snk = snk || lab[r] == b;
                }
                if (src) g.arc(S, id[q], kBig, 0);
                if (snk) g.arc(id[q], T, kBig, 0);
            }
            g.run(S, T, reach);
            for (int64_t q = 0; q < np; q++)
                if (id[q] >= 0) lab[q] = (uint8_t)(reach[id[q]] ? a : b);
        }
    return MCS_OK;
}

}  // namespace mcs

namespace mcs {

int seam_graphcut_device(int device, hipStream_t s, int n_cams, int gw, int gh, uint8_t *d_lab,
                         const uint16_t *d_cov, const uint8_t *d_smp, int cn, const uint16_t *cov,
                         int64_t *stats)
{
    using rt::Api;
    const Api *A = rt::api();
    if (!A) return MCS_E_HIP;
    const feat::FeatureKernels *k = nullptr;
    int rc = feat::feature_kernels(A, device, &k);
    if (rc) return rc;
    const int64_t np = (int64_t)gw * gh;
    // each pair's box: the points both cameras cover
    const int NP = n_cams * n_cams;
    std::vector<int> bx0(NP, gw), by0(NP, gh), bx1(NP, -1), by1(NP, -1);
    for (int64_t q = 0; q < np; q++) {
        const uint32_t c = cov[q];
        if ((c & (c - 1)) == 0) continue;
        const int X = (int)(q % gw), Y = (int)(q / gw);
        for (int a = 0; a < n_cams; a++) {
            if (!((c >> a) & 1)) continue;
            for (int b = a + 1; b < n_cams; b++) {
                if (!((c >> b) & 1)) continue;
                const int i = a * n_cams + b;
                bx0[i] = std::min(bx0[i], X), bx1[i] = std::max(bx1[i], X);
                by0[i] = std::min(by0[i], Y), by1[i] = std::max(by1[i], Y);
            }
        }
    }
    int64_t st[5] = {0, 0, 0, 0, 0};
    const auto t0 = std::chrono::steady_clock::now();
    uint8_t *buf = nullptr;
    int32_t *hflag = nullptr;
    const size_t bytes = (size_t)np * (1 + 4 * 4 + 8 + 8 + 4) + 64;
    HIP_TRY(A->hipMalloc((void **)&buf, bytes));
    hipError_t e = A->hipHostMalloc((void **)&hflag, 2 * sizeof(int32_t), 0);
    mcs::KSeamFlowArgs fa;
    std::memset(&fa, 0, sizeof(fa));
    fa.lab = d_lab;
    fa.cov = d_cov;
    fa.smp = d_smp;
    fa.ex = reinterpret_cast<long long *>(buf);
    fa.snk = fa.ex + np;
    fa.cap = reinterpret_cast<int32_t *>(fa.snk + np);
    fa.h = fa.cap + 4 * np;
    fa.flag = fa.h + np;
    fa.in = reinterpret_cast<uint8_t *>(fa.flag + 16);
    fa.np = np;
    fa.gw = gw;
    fa.gh = gh;
    fa.cn = cn;
    // push-relabel rounds between global relabels / relaxation rounds per relabel launch;
    // a round bound far beyond any grid's need (a run-away loop fails loudly instead of hanging)
    // (tuned on C4 in round 3; the tuning scripts were pruned in round 4, the tuned form's record is
    // profiles/r04_final_seam_c4.json); global relabels run as
    // Bellman-Ford relaxation rounds in LDS tiles
    constexpr int kPushLaunches = 8, kPushIters = 16, kRelabelLdsIters = 32, kRelabelBatch = 8;
    constexpr int64_t kMaxRounds = 1 << 20;
    auto launch = [&](hipFunction_t f, unsigned gx, unsigned gy) {
        return feat::launch(A, f, gx, gy, 256, &fa, sizeof(fa), s);
    };
    auto read_flags = [&]() -> hipError_t {
        hipError_t r = A->hipMemcpyAsync(hflag, fa.flag, 2 * sizeof(int32_t),
                                         hipMemcpyDeviceToHost, s);
        return r == hipSuccess ? A->hipStreamSynchronize(s) : r;
    };
    for (int a = 0; a < n_cams && e == hipSuccess && rc == MCS_OK; a++)
        for (int b = a + 1; b < n_cams && e == hipSuccess && rc == MCS_OK; b++) {
            const int i = a * n_cams + b;
            if (bx1[i] < 0) continue;
            fa.a = a;
            fa.b = b;
            fa.x0 = bx0[i], fa.y0 = by0[i];
            fa.bw = bx1[i] - bx0[i] + 1, fa.bh = by1[i] - by0[i] + 1;
            fa.hmax = (int)std::min<int64_t>((int64_t)fa.bw * fa.bh + 2, kSeamHInf - 1);
            const unsigned gx = (unsigned)((fa.bw + kSeamTile - 1) / kSeamTile);
            const unsigned gy = (unsigned)((fa.bh + kSeamTile - 1) / kSeamTile);
            st[0]++;
            rc = launch(k->seam_init, gx, gy);
            for (int64_t round = 0; rc == MCS_OK && e == hipSuccess; round++) {
                if (round >= kMaxRounds) {
                    rc = mcs::fail(MCS_E_HIP, "seam max-flow: no convergence after %lld rounds",
                                   (long long)round);
                    break;
                }
                // global relabel: exact residual distances to the sink
                st[3]++;
                rc = launch(k->seam_hinit, gx, gy);
                // batches of relabel launches, the flag reset before each: the flag read after a
                // batch is its last launch's, zero only at the fixpoint
                fa.iters = kRelabelLdsIters;
                for (;;) {
                    for (int j = 0; j < kRelabelBatch && e == hipSuccess && rc == MCS_OK; j++) {
                        e = A->hipMemsetAsync(fa.flag, 0, 2 * sizeof(int32_t), s);
                        if (e == hipSuccess)
                            rc = launch(k->seam_relabel_lds, gx, gy);
                        st[2]++;
                    }
                    if (e == hipSuccess && rc == MCS_OK) e = read_flags();
                    if (e != hipSuccess || rc != MCS_OK || hflag[0] == 0) break;
                }
                if (e == hipSuccess && rc == MCS_OK) rc = launch(k->seam_active, gx, gy);
                if (e == hipSuccess && rc == MCS_OK) e = read_flags();
                if (e != hipSuccess || rc != MCS_OK || hflag[1] == 0) break;   // maximum preflow
                fa.iters = kPushIters;
                for (int j = 0; j < kPushLaunches && rc == MCS_OK; j++, st[1]++)
                    rc = launch(k->seam_push, gx, gy);
            }
            if (rc == MCS_OK && e == hipSuccess) rc = launch(k->seam_label, gx, gy);
        }
    if (e == hipSuccess && rc == MCS_OK) e = A->hipStreamSynchronize(s);
    (void)A->hipStreamSynchronize(s);
    if (hflag) (void)A->hipHostFree(hflag);
    (void)A->hipFree(buf);
    if (rc) return rc;
    if (e != hipSuccess) return mcs::fail(MCS_E_HIP, "seam max-flow: %s", A->hipGetErrorString(e));
    st[4] = std::chrono::duration_cast<std::chrono::microseconds>(
                std::chrono::steady_clock::now() - t0).count();
    if (stats)
        for (int j = 0; j < 5; j++) stats[j] = st[j];
    return MCS_OK;
}

}  // namespace mcs

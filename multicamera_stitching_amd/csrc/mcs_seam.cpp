// mcs_seam.cpp -- graph-cut seam labels (include/mcs.h
// mcs_plan_find_seams).  Calibration-time host work, once per plan (as OpenCV's seam finders run
// once on reduced images): the per-point inputs come from the plan's device kernels
// (mcs_seam_sample_*), the pairwise minimum cuts run here with Dinic's algorithm on the
// 4-connected overlap graph.  Specification in oracle/orc_seam.c (restated there with a
// different max-flow algorithm; both return the source side of the minimal minimum cut, which
// every maximum flow shares).
#include <algorithm>
#include <cstdint>
#include <vector>

#include "mcs_common.h"

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

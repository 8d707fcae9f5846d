/*
 * orc_seam.c -- TEST INFRASTRUCTURE ONLY (the parity checker), never the product path.
 *
 * CPU restatement of the graph-cut seam finder (include/mcs.h
 * mcs_plan_find_seams).  No reference implementation exists (the reference pastes; OpenCV's
 * GraphCutSeamFinder COST_COLOR is the model, third-party, not reproduced): the specification
 * is ours and is this comment.  The product (multicamera_stitching_amd/csrc/mcs_seam.cpp) uses a
 * different max-flow algorithm (Dinic); this file uses Edmonds-Karp with capacity scaling.  The
 * labels agree because the set of nodes reachable from the source in the residual graph is the
 * same for every maximum flow (integer capacities, exact arithmetic).
 *
 *   seam grid   q = (X, Y), 0 <= X < ceil(W / 2^k), 0 <= Y < ceil(H / 2^k); q sits on output
 *               pixel p = (X 2^k, Y 2^k);
 *   inputs      per camera c: cov_c(q) = c covers p (0 <= x32 <= 32 (w-1), 0 <= y32 <= 32 (h-1)),
 *               I_c(q) = the BORDER_REPLICATE bilinear sample at p (orc_blend.c); L(q) = the
 *               distance owner's camera at p (orc_blend.c owner rule), 255 when uncovered;
 *   pairs       for a < b (camera indices), in order, with the labels as left by earlier pairs:
 *               O = {q : cov_a(q), cov_b(q), L(q) in {a, b}}; skipped when empty;
 *   graph       nodes O; 4-neighbour edges inside O, both directions, capacity
 *               e(q) + e(r) + 1 with e(q) = sum over channels |I_a(q) - I_b(q)|;
 *               source -> q (capacity 2^40) when a 4-neighbour r of q in the grid is outside O
 *               with L(r) == a; q -> sink (2^40) when one is outside O with L(r) == b;
 *   cut         after a maximum flow, L(q) = a for the q reachable from the source in the
 *               residual graph, b for the rest of O.
 * The labels become per-pixel hints (orc_blend.c): output pixel (x, y) is owned by camera
 * L(x >> k, y >> k) when that camera covers it, else by the distance rule.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SEAM_BIG ((int64_t)1 << 40)

typedef struct {
    int n, m, cap_m;
    int *head, *next, *to;
    int64_t *cap;
} graph_t;

static int g_init(graph_t *g, int n, int max_arcs)
{
    g->n = n;
    g->m = 0;
    g->cap_m = max_arcs;
    g->head = (int *)malloc(sizeof(int) * (size_t)n);
    g->next = (int *)malloc(sizeof(int) * (size_t)max_arcs);
    g->to = (int *)malloc(sizeof(int) * (size_t)max_arcs);
    g->cap = (int64_t *)malloc(sizeof(int64_t) * (size_t)max_arcs);
    if (!g->head || !g->next || !g->to || !g->cap) return -1;
    for (int i = 0; i < n; i++) g->head[i] = -1;
    return 0;
}

static void g_free(graph_t *g)
{
    free(g->head); free(g->next); free(g->to); free(g->cap);
}

/* arc u -> v with capacity c and its reverse v -> u with capacity rc (index ^ 1) */
static void g_arc(graph_t *g, int u, int v, int64_t c, int64_t rc)
{
    int e = g->m;
    g->to[e] = v; g->cap[e] = c; g->next[e] = g->head[u]; g->head[u] = e;
    g->to[e + 1] = u; g->cap[e + 1] = rc; g->next[e + 1] = g->head[v]; g->head[v] = e + 1;
    g->m += 2;
}

/* Edmonds-Karp with capacity scaling; on return reach[v] = 1 for v reachable from s. */
static int maxflow_reach(graph_t *g, int s, int t, uint8_t *reach)
{
    int *prev = (int *)malloc(sizeof(int) * (size_t)g->n);
    int *queue = (int *)malloc(sizeof(int) * (size_t)g->n);
    if (!prev || !queue) { free(prev); free(queue); return -1; }
    int64_t delta = SEAM_BIG;
    while (delta >= 1) {
        for (;;) {
            for (int i = 0; i < g->n; i++) prev[i] = -2;
            int qh = 0, qt = 0;
            queue[qt++] = s;
            prev[s] = -1;
            while (qh < qt && prev[t] == -2) {
                const int u = queue[qh++];
                for (int e = g->head[u]; e >= 0; e = g->next[e])
                    if (g->cap[e] >= delta && prev[g->to[e]] == -2) {
                        prev[g->to[e]] = e;
                        queue[qt++] = g->to[e];
                    }
            }
            if (prev[t] == -2) break;
            int64_t b = SEAM_BIG * 4;
            for (int v = t; v != s; v = g->to[prev[v] ^ 1])
                if (g->cap[prev[v]] < b) b = g->cap[prev[v]];
            for (int v = t; v != s; v = g->to[prev[v] ^ 1]) {
                g->cap[prev[v]] -= b;
                g->cap[prev[v] ^ 1] += b;
            }
        }
        delta >>= 1;
    }
    memset(reach, 0, (size_t)g->n);
    int qh = 0, qt = 0;
    queue[qt++] = s;
    reach[s] = 1;
    while (qh < qt) {
        const int u = queue[qh++];
        for (int e = g->head[u]; e >= 0; e = g->next[e])
            if (g->cap[e] > 0 && !reach[g->to[e]]) {
                reach[g->to[e]] = 1;
                queue[qt++] = g->to[e];
            }
    }
    free(prev);
    free(queue);
    return 0;
}

/* Pairwise cuts over the seam grid.  lab: gw*gh camera labels (in/out), cov: per-point camera
 * mask, smp: samples [camera][point][cn]. */
int orc_seam_graphcut(int n_cams, int gw, int gh, uint8_t *lab, const uint16_t *cov,
                      const uint8_t *smp, int cn)
{
    const long np = (long)gw * gh;
    int *id = (int *)malloc(sizeof(int) * (size_t)np);
    int32_t *e = (int32_t *)malloc(sizeof(int32_t) * (size_t)np);
    uint8_t *reach = (uint8_t *)malloc((size_t)np + 2);
    if (!id || !e || !reach) { free(id); free(e); free(reach); return -1; }
    int rc = 0;
    for (int a = 0; a < n_cams && rc == 0; a++)
        for (int b = a + 1; b < n_cams && rc == 0; b++) {
            int n = 0;
            for (long q = 0; q < np; q++) {
                const int in = ((cov[q] >> a) & 1) && ((cov[q] >> b) & 1) &&
                               (lab[q] == a || lab[q] == b);
                id[q] = in ? n++ : -1;
                if (in) {
                    int32_t s = 0;
                    for (int k = 0; k < cn; k++) {
                        const int d = (int)smp[((long)a * np + q) * cn + k] -
                                      (int)smp[((long)b * np + q) * cn + k];
                        s += d < 0 ? -d : d;
                    }
                    e[q] = s;
                }
            }
            if (n == 0) continue;
            graph_t g;
            const int S = n, T = n + 1;
            if (g_init(&g, n + 2, 2 * (2 * n + 2 * n)) != 0) { g_free(&g); rc = -1; break; }
            for (long q = 0; q < np; q++) {
                if (id[q] < 0) continue;
                const int X = (int)(q % gw), Y = (int)(q / gw);
                if (X + 1 < gw && id[q + 1] >= 0) {
                    const int64_t w = (int64_t)e[q] + e[q + 1] + 1;
                    g_arc(&g, id[q], id[q + 1], w, w);
                }
                if (Y + 1 < gh && id[q + gw] >= 0) {
                    const int64_t w = (int64_t)e[q] + e[q + gw] + 1;
                    g_arc(&g, id[q], id[q + gw], w, w);
                }
                int src = 0, snk = 0;
                const long nb[4] = {X > 0 ? q - 1 : -1, X + 1 < gw ? q + 1 : -1,
                                    Y > 0 ? q - gw : -1, Y + 1 < gh ? q + gw : -1};
                for (int k = 0; k < 4; k++) {
                    if (nb[k] < 0 || id[nb[k]] >= 0) continue;
                    if (lab[nb[k]] == a) src = 1;
                    if (lab[nb[k]] == b) snk = 1;
                }
                if (src) g_arc(&g, S, id[q], SEAM_BIG, 0);
                if (snk) g_arc(&g, id[q], T, SEAM_BIG, 0);
            }
            if (maxflow_reach(&g, S, T, reach) != 0) rc = -1;
            else
                for (long q = 0; q < np; q++)
                    if (id[q] >= 0) lab[q] = (uint8_t)(reach[id[q]] ? a : b);
            g_free(&g);
        }
    free(id);
    free(e);
    free(reach);
    return rc;
}

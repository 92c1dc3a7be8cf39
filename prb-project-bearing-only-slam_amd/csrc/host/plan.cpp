#include "plan.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>

#include "../../../include/bos.h"

namespace bos {

namespace {

constexpr int kMfLeaf = 12;          // nested-dissection leaf size (nodes) for the multifrontal solver
// pose leaves of the Schur ordering: 10 keeps the leaf fronts (poses + their landmarks' rows) within
// one wavefront (m <= 64, so every landmark folds) at config 3; 6 / 8 / 12 measured slower
constexpr int kSchurLeaf = 10;
}  // namespace


namespace {

inline int node_size(int u, int NP) { return u < NP ? 3 : 2; }

struct Graph {
    int n = 0;
    std::vector<int64_t> ptr;
    std::vector<int32_t> adj;
};

// Node-level adjacency of H_nf (symmetric, no self loops, the fixed pose has no edges).
Graph build_graph(const ProblemIndex& pi) {
    Graph g;
    g.n = pi.NP + pi.NL;
    std::vector<int64_t> deg(g.n + 1, 0);
    auto each_edge = [&](auto&& f) {
        for (int k = 0; k < pi.Mb; ++k) {
            const int p = pi.b_pose[k];
            if (p == pi.fixed) continue;
            f(p, pi.NP + pi.b_lm[k]);
        }
        for (int k = 0; k < pi.Mo; ++k) {
            const int s = pi.o_src[k], d = pi.o_dst[k];
            if (s == d || s == pi.fixed || d == pi.fixed) continue;
            f(s, d);
        }
    };
    each_edge([&](int a, int b) { ++deg[a]; ++deg[b]; });
    g.ptr.assign(g.n + 1, 0);
    for (int u = 0; u < g.n; ++u) g.ptr[u + 1] = g.ptr[u] + deg[u];
    g.adj.resize(g.ptr[g.n]);
    std::vector<int64_t> fill(g.ptr.begin(), g.ptr.end() - 1);
    each_edge([&](int a, int b) { g.adj[fill[a]++] = b; g.adj[fill[b]++] = a; });
    // sort + unique each list, compact
    std::vector<int64_t> nptr(g.n + 1, 0);
    int64_t w = 0;
    for (int u = 0; u < g.n; ++u) {
        const int64_t b = g.ptr[u], e = g.ptr[u + 1];
        std::sort(g.adj.begin() + b, g.adj.begin() + e);
        nptr[u] = w;
        int32_t last = -1;
        for (int64_t i = b; i < e; ++i) {
            if (g.adj[i] == last) continue;
            last = g.adj[i];
            g.adj[w++] = last;
        }
    }
    nptr[g.n] = w;
    g.adj.resize(w);
    g.ptr.swap(nptr);
    return g;
}

struct SymbCost {
    int64_t nnz = 0;     // scalar entries of L (lower incl. diagonal)
    double flops = 0;    // ~ sum over columns of (scalar column count)^2
};

// Elimination tree + row structures (Liu / ereach) for the node ordering inv (position -> node).
// If rows_ptr/rows is given, stores the node-level row structures (positions, sorted).
SymbCost symbolic(const Graph& g, int NP, const std::vector<int32_t>& pos, const std::vector<int32_t>& inv,
                  std::vector<int64_t>* rows_ptr, std::vector<int32_t>* rows) {
    const int m = (int)inv.size();
    std::vector<int32_t> parent(m, -1), anc(m, -1);
    for (int i = 0; i < m; ++i) {
        const int u = inv[i];
        for (int64_t e = g.ptr[u]; e < g.ptr[u + 1]; ++e) {
            int r = pos[g.adj[e]];
            if (r < 0 || r >= i) continue;
            while (anc[r] != -1 && anc[r] != i) {
                const int t = anc[r];
                anc[r] = i;
                r = t;
            }
            if (anc[r] == -1) { anc[r] = i; parent[r] = i; }
        }
    }
    std::vector<int32_t> mark(m, -1);
    std::vector<int64_t> colcnt(m, 0);
    SymbCost c;
    if (rows_ptr) { rows_ptr->assign(m + 1, 0); rows->clear(); }
    std::vector<int32_t> row;
    for (int i = 0; i < m; ++i) {
        const int u = inv[i];
        const int su = node_size(u, NP);
        mark[i] = i;
        row.clear();
        int64_t rowW = 0;
        for (int64_t e = g.ptr[u]; e < g.ptr[u + 1]; ++e) {
            int j = pos[g.adj[e]];
            if (j < 0 || j >= i) continue;
            while (mark[j] != i) {
                mark[j] = i;
                row.push_back(j);
                rowW += node_size(inv[j], NP);
                colcnt[j] += su;
                j = parent[j];
            }
        }
        c.nnz += su * rowW + su * (su + 1) / 2;
        if (rows_ptr) {
            std::sort(row.begin(), row.end());
            rows->insert(rows->end(), row.begin(), row.end());
            (*rows_ptr)[i + 1] = (int64_t)rows->size();
        }
    }
    for (int j = 0; j < m; ++j) {
        const double s = node_size(inv[j], NP);
        const double cc = (double)colcnt[j] + s;
        c.flops += s * cc * cc;
    }
    return c;
}

// Separator balance of nested_dissection (percent of a part's nodes each side must keep): set per
// plan attempt by build_plan.
thread_local int t_nd_minpct = 40;
int nd_minpct() { return t_nd_minpct; }

// Nested dissection with BFS level-structure vertex separators (graph-based, no coordinates).
void nested_dissection(const Graph& g, const std::vector<char>& active, std::vector<int32_t>& order, int leaf,
                       std::vector<std::pair<int32_t, int32_t>>* blocks) {
    auto emit = [&](const std::vector<int32_t>& nodes) {
        if (nodes.empty()) return;
        const int32_t a = (int32_t)order.size();
        order.insert(order.end(), nodes.begin(), nodes.end());
        if (blocks) blocks->push_back({a, (int32_t)order.size()});
    };
    const int n = g.n;
    std::vector<int32_t> stamp(n, -1), level(n, -1);
    int next_stamp = 0;
    struct Job { std::vector<int32_t> nodes; bool emit; };
    std::vector<Job> stack;
    {
        Job root;
        for (int u = 0; u < n; ++u) if (active[u]) root.nodes.push_back(u);
        root.emit = false;
        stack.push_back(std::move(root));
    }
    std::vector<int32_t> queue;
    auto bfs = [&](int src, int st, std::vector<int32_t>& out, int& depth) {
        // BFS restricted to nodes with stamp == st; level[] valid for visited nodes
        out.clear();
        out.push_back(src);
        level[src] = 0;
        stamp[src] = st + 1;   // visited marker (st + 1), reset by the caller
        size_t h = 0;
        depth = 0;
        while (h < out.size()) {
            const int v = out[h++];
            depth = std::max(depth, (int)level[v]);
            for (int64_t e = g.ptr[v]; e < g.ptr[v + 1]; ++e) {
                const int w = g.adj[e];
                if (stamp[w] != st) continue;
                stamp[w] = st + 1;
                level[w] = level[v] + 1;
                out.push_back(w);
            }
        }
        for (int v : out) stamp[v] = st;
    };
    std::vector<int32_t> comp, tmp;
    while (!stack.empty()) {
        Job job = std::move(stack.back());
        stack.pop_back();
        if (job.emit || (int)job.nodes.size() <= leaf) {
            emit(job.nodes);
            continue;
        }
        const int st = next_stamp;
        next_stamp += 2;
        for (int v : job.nodes) stamp[v] = st;
        // connected components
        std::vector<std::vector<int32_t>> comps;
        for (int v : job.nodes) {
            if (stamp[v] != st) continue;
            int d;
            bfs(v, st, comp, d);
            for (int w : comp) stamp[w] = st + 1;   // retire this component
            comps.push_back(comp);
        }
        if (comps.size() > 1) {
            for (auto& c : comps) stack.push_back(Job{std::move(c), false});
            continue;
        }
        std::vector<int32_t>& C = comps[0];
        for (int v : C) stamp[v] = st;
        // pseudo-peripheral start node
        int start = C[0];
        for (int v : C)
            if (g.ptr[v + 1] - g.ptr[v] < g.ptr[start + 1] - g.ptr[start]) start = v;
        int depth = 0, best_depth = -1;
        for (int it = 0; it < 6; ++it) {
            bfs(start, st, tmp, depth);
            if (depth <= best_depth) break;
            best_depth = depth;
            int cand = tmp.back();
            for (int v : tmp)
                if (level[v] == depth && g.ptr[v + 1] - g.ptr[v] < g.ptr[cand + 1] - g.ptr[cand]) cand = v;
            start = cand;
        }
        bfs(start, st, tmp, depth);
        const int h = depth + 1;
        if (h <= 2) {   // no useful level separator
            emit(tmp);
            continue;
        }
        std::vector<int64_t> cnt(h, 0);
        for (int v : tmp) ++cnt[level[v]];
        std::vector<int64_t> cum(h, 0);
        for (int k = 0; k < h; ++k) cum[k] = cnt[k] + (k ? cum[k - 1] : 0);
        const int64_t tot = (int64_t)tmp.size();
        int bestk = -1;
        // balanced splits keep the assembly tree shallow (its depth is the solver's critical path):
        // each side must hold >= minpct % of the nodes (40: 17 levels at config 3 instead of 27
        // with 20, for 6 % more flops; build_plan tries other balances when a front does not fit)
        const int minpct = nd_minpct();
        for (int k = 1; k + 1 < h; ++k) {
            const int64_t below = cum[k - 1], above = tot - cum[k];
            if (below * 100 < tot * minpct || above * 100 < tot * minpct) continue;
            if (bestk < 0 || cnt[k] < cnt[bestk]) bestk = k;
        }
        if (bestk < 0) {
            bestk = 1;
            while (bestk + 1 < h - 1 && cum[bestk] * 2 < tot) ++bestk;
        }
        std::vector<int32_t> lower, upper, sep;
        for (int v : tmp) {
            const int lv = level[v];
            if (lv < bestk) lower.push_back(v);
            else if (lv > bestk) upper.push_back(v);
            else {
                bool up = false;
                for (int64_t e = g.ptr[v]; e < g.ptr[v + 1] && !up; ++e) {
                    const int w = g.adj[e];
                    up = stamp[w] == st && level[w] == bestk + 1;
                }
                (up ? sep : lower).push_back(v);
            }
        }
        stack.push_back(Job{std::move(sep), true});
        stack.push_back(Job{std::move(upper), false});
        stack.push_back(Job{std::move(lower), false});
    }
}

}  // namespace

// Pose graph of the Schur complement: odometry edges and every pair of poses observing a common
// landmark (the fill of eliminating that landmark). The fixed pose has no edges.
Graph build_schur_graph(const ProblemIndex& pi) {
    Graph g;
    g.n = pi.NP + pi.NL;   // landmark nodes stay isolated
    std::vector<std::vector<int32_t>> obs(pi.NL);
    for (int k = 0; k < pi.Mb; ++k)
        if (pi.b_pose[k] != pi.fixed) obs[pi.b_lm[k]].push_back(pi.b_pose[k]);
    std::vector<std::vector<int32_t>> adj(pi.NP);
    for (int l = 0; l < pi.NL; ++l) {
        std::vector<int32_t>& o = obs[l];
        std::sort(o.begin(), o.end());
        o.erase(std::unique(o.begin(), o.end()), o.end());
        for (size_t a = 0; a < o.size(); ++a)
            for (size_t b = a + 1; b < o.size(); ++b) { adj[o[a]].push_back(o[b]); adj[o[b]].push_back(o[a]); }
    }
    for (int k = 0; k < pi.Mo; ++k) {
        const int s = pi.o_src[k], d = pi.o_dst[k];
        if (s == d || s == pi.fixed || d == pi.fixed) continue;
        adj[s].push_back(d);
        adj[d].push_back(s);
    }
    g.ptr.assign(g.n + 1, 0);
    for (int u = 0; u < pi.NP; ++u) {
        std::sort(adj[u].begin(), adj[u].end());
        adj[u].erase(std::unique(adj[u].begin(), adj[u].end()), adj[u].end());
        g.ptr[u + 1] = g.ptr[u] + (int64_t)adj[u].size();
    }
    for (int u = pi.NP; u < g.n; ++u) g.ptr[u + 1] = g.ptr[u];
    g.adj.reserve(g.ptr[g.n]);
    for (int u = 0; u < pi.NP; ++u) g.adj.insert(g.adj.end(), adj[u].begin(), adj[u].end());
    return g;
}

int order_nodes(const ProblemIndex& pi, int mode, std::vector<int32_t>& node_pos,
                std::vector<std::pair<int32_t, int32_t>>* blocks, OrderingReport& rep, std::string& err) {
    const int NP = pi.NP, NL = pi.NL, n = NP + NL;
    const bool nd_only = mode == kFactorMultifrontal;
    const Graph g = build_graph(pi);
    if (mode == kFactorSchur) {
        // landmarks first, each its own supernode (ascending stix), then ND of the poses on S's graph
        std::vector<int32_t> order;
        order.reserve(n);
        for (int l = 0; l < NL; ++l) {
            order.push_back(NP + l);
            if (blocks) blocks->push_back({l, l + 1});
        }
        std::vector<char> active(n, 0);
        for (int u = 0; u < NP; ++u) active[u] = u != pi.fixed;
        std::vector<int32_t> ord_p;
        std::vector<std::pair<int32_t, int32_t>> pblocks;
        const int leaf = pi.schur_leaf > 0 ? pi.schur_leaf : kSchurLeaf;
        nested_dissection(build_schur_graph(pi), active, ord_p, leaf, &pblocks);
        if ((int)ord_p.size() != NP - 1) { err = "nested dissection of the pose graph lost nodes"; return BOS_ERR_INVALID; }
        order.insert(order.end(), ord_p.begin(), ord_p.end());
        if (blocks)
            for (const auto& b : pblocks) blocks->push_back({b.first + NL, b.second + NL});
        node_pos.assign(n, -1);
        for (size_t i = 0; i < order.size(); ++i) node_pos[order[i]] = (int32_t)i;
        const SymbCost c = symbolic(g, NP, node_pos, order, nullptr, nullptr);
        rep.flops_nd = c.flops;
        rep.nnz_nd = c.nnz;
        rep.chosen = "schur-landmarks-first";
        return BOS_OK;
    }
    // last pose observing each landmark (temporal key)
    std::vector<int32_t> last_obs(NL, -1);
    for (int k = 0; k < pi.Mb; ++k) last_obs[pi.b_lm[k]] = std::max(last_obs[pi.b_lm[k]], pi.b_pose[k]);
    auto order_to_pos = [&](const std::vector<int32_t>& order, std::vector<int32_t>& pos) {
        pos.assign(n, -1);
        for (size_t i = 0; i < order.size(); ++i) pos[order[i]] = (int32_t)i;
    };
    std::vector<int32_t> active_nodes;
    for (int u = 0; u < n; ++u) if (u != pi.fixed) active_nodes.push_back(u);

    // candidate 1: temporal — poses in file order, each landmark right after its last observer
    std::vector<int32_t> ord_t = active_nodes;
    auto tkey = [&](int u) -> int64_t {
        if (u < NP) return 2LL * u;
        return 2LL * std::max(0, (int)last_obs[u - NP]) + 1;
    };
    std::stable_sort(ord_t.begin(), ord_t.end(), [&](int a, int b) { return tkey(a) < tkey(b); });
    // candidate 2: landmarks first (the Schur-complement order), then poses in file order
    std::vector<int32_t> ord_s;
    for (int u = NP; u < n; ++u) ord_s.push_back(u);
    for (int u = 0; u < NP; ++u) if (u != pi.fixed) ord_s.push_back(u);
    // candidate 3: nested dissection
    std::vector<char> active(n, 1);
    if (pi.fixed >= 0) active[pi.fixed] = 0;
    std::vector<int32_t> ord_n;
    nested_dissection(g, active, ord_n, nd_only ? kMfLeaf : 64, nd_only ? blocks : nullptr);
    if (ord_n.size() != active_nodes.size()) { err = "nested dissection lost nodes"; return BOS_ERR_INVALID; }
    if (nd_only) {
        std::vector<int32_t> pos;
        order_to_pos(ord_n, pos);
        const SymbCost c = symbolic(g, NP, pos, ord_n, nullptr, nullptr);
        rep.flops_nd = c.flops;
        rep.nnz_nd = c.nnz;
        rep.chosen = "nested-dissection";
        node_pos = pos;
        return BOS_OK;
    }

    struct Cand { const char* name; std::vector<int32_t>* ord; SymbCost c; };
    Cand cands[3] = {{"temporal", &ord_t, {}}, {"landmarks-first", &ord_s, {}}, {"nested-dissection", &ord_n, {}}};
    int best = 0;
    std::vector<int32_t> pos;
    for (int c = 0; c < 3; ++c) {
        order_to_pos(*cands[c].ord, pos);
        cands[c].c = symbolic(g, NP, pos, *cands[c].ord, nullptr, nullptr);
        if (cands[c].c.flops < cands[best].c.flops) best = c;
    }
    rep.flops_temporal = cands[0].c.flops;
    rep.nnz_temporal = cands[0].c.nnz;
    rep.flops_nd = cands[2].c.flops;
    rep.nnz_nd = cands[2].c.nnz;
    rep.chosen = cands[best].name;
    order_to_pos(*cands[best].ord, node_pos);
    return BOS_OK;
}

int validate_plan(const ProblemIndex& pi, const Plan& P, std::string& err);
int build_layout(const ProblemIndex& pi, Plan& P, std::string& err);
int build_shard(const ProblemIndex& pi, Plan& P, int rank, int world, std::string& err);
int build_csr_src(const ProblemIndex& pi, Plan& P, const std::vector<int32_t>& inv, std::string& err);

int build_multifrontal(const Graph& g, int NP, Plan& P, const std::vector<int32_t>& inv,
                       const std::vector<std::pair<int32_t, int32_t>>& blocks, int n_fold_cand, std::string& err);

int build_plan_once(const ProblemIndex& pi, int rank, int world, int factor_mode, Plan& P, std::string& err) {
    const bool want_factor = factor_mode == kFactorScalar;
    const int NP = pi.NP, NL = pi.NL, n_nodes = NP + NL;
    if (NP <= 0) { err = "no poses"; return BOS_ERR_INVALID; }
    if (pi.fixed < 0 || pi.fixed >= NP) { err = "fixed pose stix out of range"; return BOS_ERR_INVALID; }
    if (world < 1 || rank < 0 || rank >= world) { err = "bad rank/world_size"; return BOS_ERR_INVALID; }
    for (int k = 0; k < pi.Mb; ++k)
        if (pi.b_pose[k] < 0 || pi.b_pose[k] >= NP || pi.b_lm[k] < 0 || pi.b_lm[k] >= NL) {
            err = "bearing " + std::to_string(k) + " references an unknown pose/landmark stix";
            return BOS_ERR_INVALID;
        }
    for (int k = 0; k < pi.Mo; ++k) {
        if (pi.o_src[k] < 0 || pi.o_src[k] >= NP || pi.o_dst[k] < 0 || pi.o_dst[k] >= NP) {
            err = "odometry edge " + std::to_string(k) + " references an unknown pose stix";
            return BOS_ERR_INVALID;
        }
    }
    P = Plan();
    P.NP = NP; P.NL = NL; P.Mb = pi.Mb; P.Mo = pi.Mo; P.fixed = pi.fixed;
    std::vector<std::pair<int32_t, int32_t>> blocks;
    const bool multifrontal = factor_mode == kFactorMultifrontal || factor_mode == kFactorSchur;
    int rc = order_nodes(pi, factor_mode, P.node_pos, &blocks, P.ordering, err);
    if (rc) return rc;
    const Graph g = build_graph(pi);
    const int m = n_nodes - 1;
    std::vector<int32_t> inv(m);
    for (int u = 0; u < n_nodes; ++u) if (P.node_pos[u] >= 0) inv[P.node_pos[u]] = u;

    // dof offsets in elimination order
    P.node_dof.assign(n_nodes, 0);
    int64_t dof = 0;
    for (int i = 0; i < m; ++i) { P.node_dof[inv[i]] = (int32_t)dof; dof += node_size(inv[i], NP); }
    P.n = dof;
    P.node_dof[pi.fixed] = (int32_t)dof;
    if (dof + 3 > INT32_MAX) { err = "system too large for 32-bit indices"; return BOS_ERR_UNSUPPORTED; }

    // lower neighbours (by position) of every node -> CSR rows of the lower triangle
    std::vector<int64_t> lptr(n_nodes + 1, 0);
    std::vector<int32_t> lnb;              // neighbour node ids, sorted by position
    lnb.reserve(g.adj.size() / 2 + 1);
    P.rowptr.assign(P.n + 1, 0);
    for (int i = 0; i < m; ++i) {
        const int u = inv[i];
        std::vector<int32_t> nb;
        for (int64_t e = g.ptr[u]; e < g.ptr[u + 1]; ++e)
            if (P.node_pos[g.adj[e]] < i) nb.push_back(g.adj[e]);
        std::sort(nb.begin(), nb.end(), [&](int a, int b) { return P.node_pos[a] < P.node_pos[b]; });
        lptr[u] = (int64_t)lnb.size();
        int32_t off = 0;
        for (int v : nb) { lnb.push_back(v); off += node_size(v, NP); }
        const int su = node_size(u, NP);
        const int64_t r0 = P.node_dof[u];
        for (int d = 0; d < su; ++d) P.rowptr[r0 + d + 1] = off + d + 1;   // row lengths for now
    }
    // per-node end pointers for lookups
    std::vector<int64_t> lend(n_nodes, 0);
    for (int i = 0; i < m; ++i) {
        const int u = inv[i];
        lend[u] = (i + 1 < m) ? lptr[inv[i + 1]] : (int64_t)lnb.size();
    }
    for (int64_t r = 0; r < P.n; ++r) P.rowptr[r + 1] += P.rowptr[r];
    if (P.rowptr[P.n] > INT32_MAX) { err = "H has too many entries for 32-bit indices"; return BOS_ERR_UNSUPPORTED; }
    P.colind.resize(P.rowptr[P.n]);
    for (int i = 0; i < m; ++i) {
        const int u = inv[i];
        const int su = node_size(u, NP);
        const int64_t r0 = P.node_dof[u];
        for (int d = 0; d < su; ++d) {
            int64_t w = P.rowptr[r0 + d];
            for (int64_t e = lptr[u]; e < lend[u]; ++e) {
                const int v = lnb[e];
                for (int c = 0; c < node_size(v, NP); ++c) P.colind[w++] = P.node_dof[v] + c;
            }
            for (int c = 0; c <= d; ++c) P.colind[w++] = (int32_t)(r0 + c);
        }
    }
    // symbolic Cholesky factor, scalar CSR (lower incl. diagonal)
    if (want_factor) {
        std::vector<int64_t> rptr;
        std::vector<int32_t> rows;
        symbolic(g, NP, P.node_pos, inv, &rptr, &rows);
        P.Lptr.assign(P.n + 1, 0);
        for (int i = 0; i < m; ++i) {
            const int u = inv[i];
            int64_t W = 0;
            for (int64_t e = rptr[i]; e < rptr[i + 1]; ++e) W += node_size(inv[rows[e]], NP);
            for (int d = 0; d < node_size(u, NP); ++d) P.Lptr[P.node_dof[u] + d + 1] = W + d + 1;
        }
        for (int64_t r = 0; r < P.n; ++r) P.Lptr[r + 1] += P.Lptr[r];
        if (P.Lptr[P.n] > INT32_MAX) { err = "Cholesky factor exceeds 32-bit indices"; return BOS_ERR_UNSUPPORTED; }
        P.Lind.resize(P.Lptr[P.n]);
        for (int i = 0; i < m; ++i) {
            const int u = inv[i];
            for (int d = 0; d < node_size(u, NP); ++d) {
                int64_t w = P.Lptr[P.node_dof[u] + d];
                for (int64_t e = rptr[i]; e < rptr[i + 1]; ++e) {
                    const int v = inv[rows[e]];
                    for (int c = 0; c < node_size(v, NP); ++c) P.Lind[w++] = P.node_dof[v] + c;
                }
                for (int c = 0; c <= d; ++c) P.Lind[w++] = P.node_dof[u] + c;
            }
        }
    }

    // one GPU: every node's lanes, in stix order
    P.shard = Shard();
    P.shard.lane_poses.resize(NP);
    std::iota(P.shard.lane_poses.begin(), P.shard.lane_poses.end(), 0);
    P.shard.own_pose_lanes = NP;
    P.shard.lane_lms.resize(NL);
    std::iota(P.shard.lane_lms.begin(), P.shard.lane_lms.end(), 0);
    if ((rc = build_layout(pi, P, err))) return rc;
    if ((rc = build_csr_src(pi, P, inv, err))) return rc;
    // Schur: the first NL blocks are the landmarks, candidates for folding into their parents
    const int n_fold_cand = factor_mode == kFactorSchur ? NL : 0;
    if (multifrontal && (rc = build_multifrontal(g, NP, P, inv, blocks, n_fold_cand, err))) return rc;
    if (multifrontal && (rc = build_shard(pi, P, rank, world, err))) return rc;
    if (world > 1) {
        if (!multifrontal) { err = "world_size > 1 needs a multifrontal solver (schur or supernodal)"; return BOS_ERR_UNSUPPORTED; }
        // this rank's lanes only: the layout, its stored-entry sources and the maps built from them
        // (the tree and every offset are the same on every rank)
        if ((rc = build_layout(pi, P, err)) || (rc = build_csr_src(pi, P, inv, err)) ||
            (rc = build_multifrontal(g, NP, P, inv, blocks, n_fold_cand, err)))
            return rc;
        if (P.shard.lane_poses.size() != P.blk.lane_pose.size()) { err = "shard: lane rebuild"; return BOS_ERR_INVALID; }
    }
    return validate_plan(pi, P, err);
}

// The Schur ordering's tree is cut at balanced separators (>= 40 % of a part on each side: few
// levels); some graphs then get a front the fast kernels do not take (m > 64 anywhere, or m > 48
// from level 2 up, where the dataflow launch starts), which costs far more than the balance buys.
// Such plans are rebuilt with other balances; the first plan without those fronts is kept (the
// first attempt's plan if none is).
void schur_front_report(Multifrontal& F) {
    F.max_m_upper = 0;
    F.fits = true;
    for (int l = 0; l < F.nlevels; ++l)
        for (int q = F.level_ptr[l]; q < F.level_ptr[l + 1]; ++q) {
            const int m = F.k[F.level[q]] + F.r[F.level[q]];
            if (l >= 2) F.max_m_upper = std::max(F.max_m_upper, m);
            if (m > kMfWaveMaxM || (l >= 2 && m > kMfFlowMaxM)) F.fits = false;
        }
}

int build_plan(const ProblemIndex& pi, int rank, int world, int factor_mode, Plan& P, std::string& err) {
    if (factor_mode != kFactorSchur) return build_plan_once(pi, rank, world, factor_mode, P, err);
    // The first attempt (40 %) decides success: a later, less balanced attempt has more fill, so an
    // error there (e.g. a 32-bit size limit) only means "does not fit" and the first plan is kept.
    const int tries[] = {40, 35, 45, 30, 20};
    Plan first;
    for (int i = 0; i < 5; ++i) {
        t_nd_minpct = tries[i];
        Plan attempt;
        std::string aerr;
        const int rc = build_plan_once(pi, rank, world, factor_mode, attempt, aerr);
        t_nd_minpct = 40;
        if (rc) {
            if (i == 0) { err = aerr; return rc; }
            continue;
        }
        schur_front_report(attempt.mf);
        attempt.mf.balance_pct = tries[i];
        if (attempt.mf.fits) { P = std::move(attempt); return BOS_OK; }
        if (i == 0) first = std::move(attempt);
    }
    P = std::move(first);   // no balance fits: the default plan (fronts the fast kernels do not take run
                            // on the general workgroup path)
    return BOS_OK;
}

// Wave-interleaved lane lists (LaneLists in plan.hpp) from per-lane item ranges.
void make_lane_lists(int lanes, const std::vector<int32_t>& lane_ptr, const std::vector<int32_t>& items, LaneLists& L,
                     bool even) {
    const int waves = (lanes + 63) / 64;
    L.w_base.assign(waves + 1, 0);
    L.w_len.assign(waves, 0);
    L.cnt.assign(lanes, 0);
    for (int g = 0; g < lanes; ++g) {
        L.cnt[g] = lane_ptr[g + 1] - lane_ptr[g];
        L.w_len[g / 64] = std::max(L.w_len[g / 64], L.cnt[g]);
    }
    if (even)   // the J+H kernel walks pose lists in pairs and stores the second item of the last pair
        for (int w = 0; w < waves; ++w) L.w_len[w] += L.w_len[w] & 1;
    // groups of consecutive waves with equal list lengths, each stored step-major
    L.w_stride.assign(waves, 64);
    int64_t base = 0;
    for (int w0 = 0; w0 < waves;) {
        int w1 = w0 + 1;
        while (w1 < waves && L.w_len[w1] == L.w_len[w0]) ++w1;
        for (int w = w0; w < w1; ++w) {
            L.w_base[w] = (int32_t)(base + 64 * (int64_t)(w - w0));
            L.w_stride[w] = 64 * (w1 - w0);
        }
        base += 64 * (int64_t)(w1 - w0) * L.w_len[w0];
        w0 = w1;
    }
    L.w_base[waves] = (int32_t)base;
    L.obs.assign(L.slots(), -1);
    for (int g = 0; g < lanes; ++g)
        for (int j = 0; j < L.cnt[g]; ++j) L.obs[L.slot(g, j)] = items[lane_ptr[g] + j];
}

inline int32_t lane_slot(const LaneLists& L, int g, int j) { return L.slot(g, j); }

bool duplicate_pairs(const ProblemIndex& pi) {
    std::vector<int64_t> key;
    key.reserve(std::max(pi.Mb, pi.Mo));
    for (int k = 0; k < pi.Mb; ++k) key.push_back((int64_t)pi.b_pose[k] * pi.NL + pi.b_lm[k]);
    std::sort(key.begin(), key.end());
    if (std::adjacent_find(key.begin(), key.end()) != key.end()) return true;
    key.clear();
    for (int k = 0; k < pi.Mo; ++k)
        if (pi.o_src[k] != pi.o_dst[k])
            key.push_back((int64_t)std::min(pi.o_src[k], pi.o_dst[k]) * pi.NP + std::max(pi.o_src[k], pi.o_dst[k]));
    std::sort(key.begin(), key.end());
    return std::adjacent_find(key.begin(), key.end()) != key.end();
}

// Block layout of H and the J+H work split (see BlockLayout in plan.hpp).
int build_layout(const ProblemIndex& pi, Plan& P, std::string& err) {
    const int NP = pi.NP, NL = pi.NL, Mb = pi.Mb, Mo = pi.Mo;
    BlockLayout& B = P.blk;
    B = BlockLayout();
    // bearings by (pose, landmark, index) and by (landmark, pose, index)
    std::vector<int32_t> pb_ptr(NP + 1, 0), lb_ptr(NL + 1, 0), pb_obs(Mb), lb_obs(Mb);
    for (int k = 0; k < Mb; ++k) { ++pb_ptr[pi.b_pose[k] + 1]; ++lb_ptr[pi.b_lm[k] + 1]; }
    for (int p = 0; p < NP; ++p) pb_ptr[p + 1] += pb_ptr[p];
    for (int l = 0; l < NL; ++l) lb_ptr[l + 1] += lb_ptr[l];
    {
        std::vector<int32_t> wp(pb_ptr.begin(), pb_ptr.end() - 1), wl(lb_ptr.begin(), lb_ptr.end() - 1);
        for (int k = 0; k < Mb; ++k) { pb_obs[wp[pi.b_pose[k]]++] = k; lb_obs[wl[pi.b_lm[k]]++] = k; }
    }
    for (int p = 0; p < NP; ++p)
        std::stable_sort(pb_obs.begin() + pb_ptr[p], pb_obs.begin() + pb_ptr[p + 1],
                         [&](int a, int b) { return pi.b_lm[a] < pi.b_lm[b]; });
    for (int l = 0; l < NL; ++l)
        std::stable_sort(lb_obs.begin() + lb_ptr[l], lb_obs.begin() + lb_ptr[l + 1],
                         [&](int a, int b) { return pi.b_pose[a] < pi.b_pose[b]; });
    // Odometry entries of each pose, sorted by (other pose, edge). An odometry self-loop has a zero
    // Jacobian in the reference (its source and destination triplets land on the same columns and
    // cancel exactly, solver_jacobians.cpp:126-146 with setFromTriplets summing duplicates), so it
    // adds nothing to H or b: it gets no entries (its constant chi^2 is added by the step's stats).
    // The pose-pose block of an unordered pair {p, q} is stored by the lower pose's lane: every edge
    // between the two, in either direction, adds -H_ss (symmetric) to it.
    B.po_ptr.assign(NP + 1, 0);
    for (int k = 0; k < Mo; ++k)
        if (pi.o_src[k] != pi.o_dst[k]) { ++B.po_ptr[pi.o_src[k] + 1]; ++B.po_ptr[pi.o_dst[k] + 1]; }
    for (int p = 0; p < NP; ++p) B.po_ptr[p + 1] += B.po_ptr[p];
    B.po_ent.resize(B.po_ptr[NP]);
    {
        std::vector<int32_t> w(B.po_ptr.begin(), B.po_ptr.end() - 1);
        for (int k = 0; k < Mo; ++k)
            if (pi.o_src[k] != pi.o_dst[k]) { B.po_ent[w[pi.o_src[k]]++] = 2 * k; B.po_ent[w[pi.o_dst[k]]++] = 2 * k + 1; }
    }
    auto other = [&](int32_t ent) { return (ent & 1) ? pi.o_src[ent >> 1] : pi.o_dst[ent >> 1]; };
    for (int p = 0; p < NP; ++p)
        std::sort(B.po_ent.begin() + B.po_ptr[p], B.po_ent.begin() + B.po_ptr[p + 1], [&](int32_t a, int32_t b) {
            if (other(a) != other(b)) return other(a) < other(b);
            return a < b;
        });
    B.po_blk.assign(B.po_ent.size(), -1);
    B.uo_ptr.assign(NP + 1, 0);
    for (int p = 0; p < NP; ++p) {
        for (int x = B.po_ptr[p]; x < B.po_ptr[p + 1]; ++x) {
            const int32_t e = B.po_ent[x];
            if (other(e) < p) continue;
            if (x > B.po_ptr[p] && other(B.po_ent[x - 1]) == other(e)) {
                B.has_dups = true;
                B.po_blk[x] = B.po_blk[x - 1];
                continue;
            }
            B.po_blk[x] = (int32_t)B.uo_dst.size();
            B.uo_dst.push_back(other(e));
        }
        B.uo_ptr[p + 1] = (int32_t)B.uo_dst.size();
    }
    // odometry chain poses: exactly the entries (edge p - 1 from its destination side, edge p from its
    // source side) of edges p - 1 = (p - 1, p) and p = (p, p + 1) (LinParams / kOdoChain)
    B.po_chain.assign(NP, 0);
    for (int p = 1; p + 1 < NP; ++p) {
        const int x0 = B.po_ptr[p];
        if (B.po_ptr[p + 1] - x0 != 2 || p >= Mo) continue;
        if (B.po_ent[x0] != (((p - 1) << 1) | 1) || B.po_ent[x0 + 1] != (p << 1)) continue;
        if (pi.o_src[p - 1] != p - 1 || pi.o_dst[p] != p + 1) continue;
        B.po_chain[p] = 1;
    }
    // lanes per pose and their bearing segments (lane 0 also takes the odometry entries; a run of
    // duplicate observations of one pair never straddles two lanes)
    B.lpp = plan_lanes_per_pose(pi, P.shard.world);
    if (B.lpp != 1 && B.lpp != 2 && B.lpp != 4) { err = "lanes per pose must be 1, 2 or 4"; return BOS_ERR_INVALID; }
    const int L = B.lpp;
    auto same_lm = [&](int i, int j) { return pi.b_lm[pb_obs[i]] == pi.b_lm[pb_obs[j]]; };
    for (int p = 0; p < NP; ++p)
        for (int i = pb_ptr[p] + 1; i < pb_ptr[p + 1]; ++i)
            if (same_lm(i, i - 1)) B.has_dups = true;
    // pose lane groups in the shard's order (every pose in stix order on one GPU). Without duplicate
    // pairs the items are dealt round robin (item i of a pose to lane i % L, LinParams: interleaved
    // groups accumulate in pose order, bit-identical to one lane per pose); with them each lane takes
    // a contiguous range pb_obs[cut[j], cut[j + 1]) (runs never straddle lanes; partial sums combined).
    // lane_item[g]: the pb_obs offsets of lane g's items, in lane order.
    B.lane_pose = P.shard.lane_poses;
    const int G = (int)B.lane_pose.size();
    B.interleaved = L > 1 && !B.has_dups;
    std::vector<int32_t> lane_ptr((size_t)G * L + 1, 0), pitems, lane_item;
    pitems.reserve(Mb);
    lane_item.reserve(Mb);
    for (int i = 0; i < G; ++i) {
        const int p = B.lane_pose[i];
        if (B.interleaved) {
            for (int j = 0; j < L; ++j) {
                const size_t g = (size_t)i * L + j;
                if (p >= 0)
                    for (int q = pb_ptr[p] + j; q < pb_ptr[p + 1]; q += L) {
                        pitems.push_back(pb_obs[q]);
                        lane_item.push_back(q);
                    }
                lane_ptr[g + 1] = (int32_t)pitems.size();
            }
            continue;
        }
        int cut[5] = {0, 0, 0, 0, 0};   // bearing range of each lane (as pb_obs offsets)
        if (p >= 0) {
            const int b0 = pb_ptr[p], b1 = pb_ptr[p + 1], nb = b1 - b0;
            const int no = B.po_ptr[p + 1] - B.po_ptr[p];
            const int share = (nb + no + L - 1) / L;
            const int q0 = std::min(nb, std::max(0, share - no));
            int prev = b0;
            for (int j = 0; j < L; ++j) {
                cut[j] = prev;
                if (j + 1 < L) {
                    int c = b0 + q0 + (int)((int64_t)(nb - q0) * j / std::max(1, L - 1));
                    c = std::max(c, prev);
                    while (c > b0 && c < b1 && same_lm(c, c - 1)) ++c;
                    prev = c;
                }
            }
            cut[L] = b1;
        }
        for (int j = 0; j < L; ++j) {
            const size_t g = (size_t)i * L + j;
            pitems.insert(pitems.end(), pb_obs.begin() + cut[j], pb_obs.begin() + cut[j + 1]);
            for (int q = cut[j]; q < cut[j + 1]; ++q) lane_item.push_back(q);
            lane_ptr[g + 1] = (int32_t)pitems.size();
        }
    }
    make_lane_lists(G * L, lane_ptr, pitems, B.pose_lanes, true);
    if (B.interleaved)
        for (int c : B.pose_lanes.cnt)
            if (c > 0x3fff) { err = "interleaved pose lanes: more than 16383 bearings per lane"; return BOS_ERR_UNSUPPORTED; }
    {   // landmark lanes in the shard's order; inside each window consecutive-pose lanes first, then
        // by degree (ties by the shard's order: deterministic)
        B.lm_lane_lm = P.shard.lane_lms;
        const int NLL = (int)B.lm_lane_lm.size();
        auto deg = [&](int l) { return lb_ptr[l + 1] - lb_ptr[l]; };
        auto run0 = [&](int l) -> int32_t {   // poses p0, p0 + 1, ... (sorted by pose above)
            if (deg(l) < 1) return -1;
            const int32_t p0 = pi.b_pose[lb_obs[lb_ptr[l]]];
            for (int i = lb_ptr[l] + 1; i < lb_ptr[l + 1]; ++i)
                if (pi.b_pose[lb_obs[i]] != p0 + (i - lb_ptr[l])) return -1;
            return p0;
        };
        for (int w0 = 0; w0 < NLL; w0 += kLmWindow)
            std::stable_sort(B.lm_lane_lm.begin() + w0, B.lm_lane_lm.begin() + std::min(NLL, w0 + kLmWindow),
                             [&](int a, int b) {
                                 const bool ra = run0(a) >= 0, rb = run0(b) >= 0;
                                 if (ra != rb) return ra;
                                 return deg(a) > deg(b);
                             });
        std::vector<int32_t> lptr(NLL + 1, 0), litems;
        B.lm_lane_run.assign(NLL, -1);
        for (int g = 0; g < NLL; ++g) {
            const int l = B.lm_lane_lm[g];
            litems.insert(litems.end(), lb_obs.begin() + lb_ptr[l], lb_obs.begin() + lb_ptr[l + 1]);
            lptr[g + 1] = (int32_t)litems.size();
            B.lm_lane_run[g] = run0(l);
        }
        make_lane_lists(NLL, lptr, litems, B.lm_lanes, false);
    }
    // pose-landmark blocks of the lane poses: the slot of the last bearing of each (pose, landmark) run
    std::vector<int32_t> group_of(NP, -1);
    for (int i = 0; i < G; ++i)
        if (B.lane_pose[i] >= 0) group_of[B.lane_pose[i]] = i;
    // (in pose order: an item is its run's last when the pose's next item observes another
    // landmark; a contiguous split never cuts a run, an interleaved one has none)
    B.ub_ptr.assign(NP + 1, 0);
    {
        std::vector<int32_t> item_slot(Mb, -1);   // pb_obs offset -> the slot holding it
        for (size_t g = 0; g < B.pose_lanes.cnt.size(); ++g)
            for (int j = 0; j < B.pose_lanes.cnt[g]; ++j) item_slot[lane_item[lane_ptr[g] + j]] = lane_slot(B.pose_lanes, (int)g, j);
        for (int p = 0; p < NP; ++p) {
            if (group_of[p] >= 0)
                for (int q = pb_ptr[p]; q < pb_ptr[p + 1]; ++q)
                    if (q + 1 == pb_ptr[p + 1] || !same_lm(q + 1, q)) {
                        if (item_slot[q] < 0) { err = "pose lane item without a slot"; return BOS_ERR_INVALID; }
                        B.ub_lm.push_back(pi.b_lm[pb_obs[q]]);
                        B.ub_slot.push_back(item_slot[q]);
                    }
            B.ub_ptr[p + 1] = (int32_t)B.ub_lm.size();
        }
    }
    B.off_ldiag = 6 * (int64_t)NP;
    B.off_pl = (B.off_ldiag + 3 * (int64_t)NL + 1) & ~(int64_t)1;   // even: 2-value vector stores stay aligned
    B.off_pp = B.off_pl + 6 * B.pose_lanes.slots();
    B.size = B.off_pp + 6 * (int64_t)B.nuo();
    if (B.size > INT32_MAX) { err = "block array exceeds 32-bit indices"; return BOS_ERR_UNSUPPORTED; }
    return BOS_OK;
}

// Block value feeding every stored entry (row >= col) of the lower triangle of P^T H_nf P.
int build_csr_src(const ProblemIndex& pi, Plan& P, const std::vector<int32_t>& inv, std::string& err) {
    const int NP = pi.NP;
    const BlockLayout& B = P.blk;
    std::vector<int32_t> dof_node(P.n), dof_loc(P.n);
    for (int u : inv)
        for (int d = 0; d < node_size(u, NP); ++d) { dof_node[P.node_dof[u] + d] = u; dof_loc[P.node_dof[u] + d] = d; }
    auto tri = [](int r, int c) { return r >= c ? r * (r + 1) / 2 + c : c * (c + 1) / 2 + r; };
    auto pl_slot = [&](int p, int l) -> int64_t {
        const auto b = B.ub_lm.begin() + B.ub_ptr[p], e = B.ub_lm.begin() + B.ub_ptr[p + 1];
        const auto it = std::lower_bound(b, e, l);
        return (it != e && *it == l) ? (int64_t)B.ub_slot[it - B.ub_lm.begin()] : -1;
    };
    auto pp_block = [&](int s, int d) -> int64_t {
        const auto b = B.uo_dst.begin() + B.uo_ptr[s], e = B.uo_dst.begin() + B.uo_ptr[s + 1];
        const auto it = std::lower_bound(b, e, d);
        return (it != e && *it == d) ? (int64_t)(it - B.uo_dst.begin()) : -1;
    };
    // which nodes' lanes this rank's J+H runs (all of them on one GPU); a block is computed by the
    // lane of its pose (pose-landmark), of its lower pose (pose-pose) or of its node (diagonal)
    std::vector<char> lane_node(pi.NP + pi.NL, 0);
    for (int32_t p : B.lane_pose) if (p >= 0) lane_node[p] = 1;
    for (int32_t l : B.lm_lane_lm) lane_node[NP + l] = 1;
    P.blk.csr_src.resize(P.nnzA());
    for (int64_t row = 0; row < P.n; ++row) {
        const int U = dof_node[row], a = dof_loc[row];
        for (int64_t e = P.rowptr[row]; e < P.rowptr[row + 1]; ++e) {
            const int V = dof_node[P.colind[e]], c = dof_loc[P.colind[e]];
            int64_t v = -1;
            int owner = U;   // the node whose lane computes the block
            if (U == V) {
                v = U < NP ? 6 * (int64_t)U + tri(a, c) : B.off_ldiag + 3 * (int64_t)(U - NP) + tri(a, c);
            } else if (U < NP && V >= NP) {
                const int64_t k = pl_slot(U, V - NP);
                if (k >= 0) v = B.off_pl + 6 * k + 2 * a + c;
            } else if (U >= NP && V < NP) {
                owner = V;
                const int64_t k = pl_slot(V, U - NP);
                if (k >= 0) v = B.off_pl + 6 * k + 2 * c + a;
            } else if (U < NP && V < NP) {
                owner = std::min(U, V);
                int64_t k = pp_block(U, V);
                if (k < 0) k = pp_block(V, U);
                if (k >= 0) v = B.off_pp + 6 * k + tri(a, c);
            }
            if (!lane_node[owner]) { P.blk.csr_src[e] = -2; continue; }   // another rank's
            if (v < 0) { err = "internal error: stored entry without a block"; return BOS_ERR_INVALID; }
            P.blk.csr_src[e] = (int32_t)v;
        }
    }
    return BOS_OK;
}

void observation_lanes(const Plan& P, int rank, int world, int64_t& pb0, int64_t& pb1, int64_t& lb0, int64_t& lb1,
                       std::vector<char>* lane_node) {
    const BlockLayout& B = P.blk;
    split_range(B.pose_blocks(), rank, world, pb0, pb1);
    split_range(B.lm_blocks(), rank, world, lb0, lb1);
    if (!lane_node) return;
    lane_node->assign((size_t)P.NP + P.NL, 0);
    const int64_t G = (int64_t)B.lane_pose.size() * B.lpp, NLL = (int64_t)B.lm_lane_lm.size();
    for (int64_t g = pb0 * kJhBlock; g < std::min(G, pb1 * kJhBlock); ++g)
        if (B.lane_pose[g / B.lpp] >= 0) (*lane_node)[B.lane_pose[g / B.lpp]] = 1;
    for (int64_t g = lb0 * kJhBlock; g < std::min(NLL, lb1 * kJhBlock); ++g) (*lane_node)[P.NP + B.lm_lane_lm[g]] = 1;
}

void owned_entries(const Plan& P, const std::vector<char>& lane_node, std::vector<uint8_t>& owned) {
    const BlockLayout& B = P.blk;
    // the pose whose lane writes each pose-landmark slot, and the lower pose of each pose-pose block
    std::vector<int32_t> slot_pose(B.pose_lanes.slots(), -1), pp_pose(B.nuo(), -1);
    for (int64_t g = 0; g < (int64_t)B.lane_pose.size() * B.lpp; ++g) {
        const int p = B.lane_pose[g / B.lpp];
        if (p < 0) continue;
        for (int j = 0; j < B.pose_lanes.w_len[g / 64]; ++j) slot_pose[B.pose_lanes.slot((int)g, j)] = p;
    }
    for (int p = 0; p < P.NP; ++p)
        for (int q = B.uo_ptr[p]; q < B.uo_ptr[p + 1]; ++q) pp_pose[q] = p;
    owned.assign(P.nnzA(), 0);
    for (int64_t e = 0; e < P.nnzA(); ++e) {
        const int64_t v = B.csr_src[e];
        if (v < 0) continue;
        int owner;
        if (v < B.off_ldiag) owner = (int)(v / 6);
        else if (v < B.off_pl) owner = P.NP + (int)((v - B.off_ldiag) / 3);
        else if (v < B.off_pp) owner = slot_pose[(v - B.off_pl) / 6];
        else owner = pp_pose[(v - B.off_pp) / 6];
        owned[e] = owner >= 0 && lane_node[owner] ? 1 : 0;
    }
}

int build_multifrontal(const Graph& g, int NP, Plan& P, const std::vector<int32_t>& inv,
                       const std::vector<std::pair<int32_t, int32_t>>& blocks, int n_fold_cand, std::string& err) {
    const int m = (int)inv.size();
    Multifrontal& F = P.mf;
    F = Multifrontal();
    // node-level row structures of L -> column structures (rows ascending)
    std::vector<int64_t> rptr;
    std::vector<int32_t> rows;
    symbolic(g, NP, P.node_pos, inv, &rptr, &rows);
    std::vector<int64_t> cptr(m + 1, 0);
    for (int32_t j : rows) ++cptr[j + 1];
    for (int i = 0; i < m; ++i) cptr[i + 1] += cptr[i];
    std::vector<int32_t> cols(rows.size());
    {
        std::vector<int64_t> w(cptr.begin(), cptr.end() - 1);
        for (int i = 0; i < m; ++i)
            for (int64_t e = rptr[i]; e < rptr[i + 1]; ++e) cols[w[rows[e]]++] = i;
    }
    const int ns = (int)blocks.size();
    std::vector<int32_t> blk(m, -1);
    for (int b = 0; b < ns; ++b)
        for (int q = blocks[b].first; q < blocks[b].second; ++q) {
            if (blk[q] != -1) { err = "multifrontal: overlapping supernodes"; return BOS_ERR_INVALID; }
            blk[q] = b;
        }
    for (int q = 0; q < m; ++q)
        if (blk[q] < 0) { err = "multifrontal: position not covered by a supernode"; return BOS_ERR_INVALID; }
    F.nsuper = ns;
    F.col0.resize(ns); F.k.resize(ns); F.r.resize(ns); F.parent.assign(ns, -1);
    F.findex_off.resize(ns + 1);
    std::vector<int32_t> stamp(m, -1), R;
    for (int s = 0; s < ns; ++s) {
        const int a = blocks[s].first, e = blocks[s].second;
        R.clear();
        for (int q = a; q < e; ++q)
            for (int64_t t = cptr[q]; t < cptr[q + 1]; ++t) {
                const int i = cols[t];
                if (i >= e && stamp[i] != s) { stamp[i] = s; R.push_back(i); }
            }
        std::sort(R.begin(), R.end());
        F.parent[s] = R.empty() ? -1 : blk[R[0]];
        F.col0[s] = P.node_dof[inv[a]];
        int k = 0;
        for (int q = a; q < e; ++q) k += node_size(inv[q], NP);
        F.k[s] = k;
        F.findex_off[s] = (int64_t)F.findex.size();
        for (int d = 0; d < k; ++d) F.findex.push_back(F.col0[s] + d);
        int r = 0;
        for (int q : R) {
            const int u = inv[q];
            for (int d = 0; d < node_size(u, NP); ++d) F.findex.push_back(P.node_dof[u] + d);
            r += node_size(u, NP);
        }
        F.r[s] = r;
    }
    F.findex_off[ns] = (int64_t)F.findex.size();
    auto front_pos = [&](int s, int32_t dof) -> int32_t {
        const int k = F.k[s];
        if (dof >= F.col0[s] && dof < F.col0[s] + k) return dof - F.col0[s];
        const int32_t* b = F.findex.data() + F.findex_off[s] + k;
        const int32_t* e = F.findex.data() + F.findex_off[s + 1];
        const int32_t* it = std::lower_bound(b, e, dof);
        if (it == e || *it != dof) return -1;
        return k + (int32_t)(it - b);
    };
    // children, relative maps, offsets, levels
    F.child_ptr.assign(ns + 1, 0);
    for (int s = 0; s < ns; ++s) if (F.parent[s] >= 0) ++F.child_ptr[F.parent[s] + 1];
    for (int s = 0; s < ns; ++s) F.child_ptr[s + 1] += F.child_ptr[s];
    F.child.resize(F.child_ptr[ns]);
    {
        std::vector<int32_t> w(F.child_ptr.begin(), F.child_ptr.end() - 1);
        for (int s = 0; s < ns; ++s) if (F.parent[s] >= 0) F.child[w[F.parent[s]]++] = s;
    }
    // folding (Schur ordering): a parent factored by one wavefront or one blocked workgroup
    // (m <= kMfBlkMaxM) takes all its landmark children (2-column leaves with m <= kMfWaveMaxM) into
    // its own front; children lists are ascending, so the landmark supernodes (ids < n_fold_cand)
    // come first
    F.fold_cnt.assign(ns, 0);
    std::vector<char> folded(ns, 0);
    for (int p = 0; p < ns && n_fold_cand > 0; ++p) {
        if (F.k[p] + F.r[p] > kMfBlkMaxM) continue;
        int nf = 0;
        bool ok = true;
        for (int ci = F.child_ptr[p]; ci < F.child_ptr[p + 1]; ++ci) {
            const int c = F.child[ci];
            if (c >= n_fold_cand) break;
            ok = ok && F.k[c] == 2 && F.k[c] + F.r[c] <= kMfWaveMaxM && F.r[c] <= 3 * kFoldChunk &&
                 F.child_ptr[c] == F.child_ptr[c + 1];
            ++nf;
        }
        if (!ok || nf == 0) continue;
        F.fold_cnt[p] = nf;
        for (int ci = F.child_ptr[p]; ci < F.child_ptr[p] + nf; ++ci) folded[F.child[ci]] = 1;
    }
    F.rmap_off.resize(ns + 1);
    F.L_off.resize(ns); F.U_off.resize(ns); F.u_off.resize(ns);
    std::vector<int32_t> lev(ns, 0);
    for (int s = 0; s < ns; ++s) {
        const int k = F.k[s], r = F.r[s], mm = k + r;
        F.max_m = std::max(F.max_m, mm);
        F.L_off[s] = F.L_size; F.L_size += (int64_t)mm * k;
        F.U_off[s] = F.U_size; F.U_size += (int64_t)r * (r + 1) / 2;
        F.u_off[s] = F.u_size; F.u_size += r;
        F.flops += (double)k * k * k / 3.0 + (double)k * k * r + (double)k * r * r;
        F.rmap_off[s] = (int64_t)F.rmap.size();
        const int p = F.parent[s];
        if (p >= 0) {
            if (p <= s) { err = "multifrontal: parent precedes child"; return BOS_ERR_INVALID; }
            for (int t = k; t < mm; ++t) {
                const int32_t fp = front_pos(p, F.findex[F.findex_off[s] + t]);
                if (fp < 0) { err = "multifrontal: update row missing from the parent front"; return BOS_ERR_INVALID; }
                F.rmap.push_back(fp);
            }
            if (!folded[s]) lev[p] = std::max(lev[p], lev[s] + 1);
        } else if (r != 0) {
            err = "multifrontal: root with update rows";
            return BOS_ERR_INVALID;
        }
    }
    F.rmap_off[ns] = (int64_t)F.rmap.size();
    F.nlevels = 0;
    for (int s = 0; s < ns; ++s) F.nlevels = std::max(F.nlevels, lev[s] + 1);
    F.level_ptr.assign(F.nlevels + 1, 0);
    for (int s = 0; s < ns; ++s) if (!folded[s]) ++F.level_ptr[lev[s] + 1];
    for (int l = 0; l < F.nlevels; ++l) F.level_ptr[l + 1] += F.level_ptr[l];
    F.level.resize(F.level_ptr[F.nlevels]);
    {
        std::vector<int32_t> w(F.level_ptr.begin(), F.level_ptr.end() - 1);
        for (int s = 0; s < ns; ++s) if (!folded[s]) F.level[w[lev[s]]++] = s;
    }
    F.fold_list.clear();
    for (int s = 0; s < ns; ++s) if (folded[s]) F.fold_list.push_back(s);
    // assembly map: every stored entry of H (row i >= col j) goes to the front of col j's supernode,
    // read from its block value
    std::vector<int32_t> sn_of_dof(P.n);
    for (int s = 0; s < ns; ++s)
        for (int d = 0; d < F.k[s]; ++d) sn_of_dof[F.col0[s] + d] = s;
    const int64_t nnz = P.nnzA();
    std::vector<int32_t> tgt(nnz), dst(nnz);
    F.amap_ptr.assign(ns + 1, 0);
    for (int64_t row = 0; row < P.n; ++row)
        for (int64_t e = P.rowptr[row]; e < P.rowptr[row + 1]; ++e) {
            const int32_t j = P.colind[e];
            const int s = sn_of_dof[j];
            const int32_t li = front_pos(s, (int32_t)row);
            if (li < 0) { err = "multifrontal: H entry outside its front"; return BOS_ERR_INVALID; }
            tgt[e] = s;
            const int fm = F.k[s] + F.r[s];
            dst[e] = fm <= kMfWaveMaxM ? (int32_t)mf_packed(li, j - F.col0[s], fm) : li + (j - F.col0[s]) * fm;
            ++F.amap_ptr[s + 1];
        }
    for (int s = 0; s < ns; ++s) F.amap_ptr[s + 1] += F.amap_ptr[s];
    F.amap_src.resize(nnz);
    F.amap_dst.resize(nnz);
    {
        std::vector<int32_t> w(F.amap_ptr.begin(), F.amap_ptr.end() - 1);
        for (int64_t e = 0; e < nnz; ++e) {
            const int32_t q = w[tgt[e]]++;
            F.amap_src[q] = P.blk.csr_src[e];
            F.amap_dst[q] = dst[e];
        }
    }
    // fold records, one per observing pose of a folded child c — a group of 3 consecutive rows
    // t, t + 1, t + 2 (the pose's x, y, theta dofs) at consecutive positions of the parent front —
    // (parents in id order, their folded children in child-list order): {src (t, 0), src (t, 1),
    // src (0, 0), src (1, 0), src (1, 1), col0[c], t | r[c] << 6 | (row t's position in the parent
    // front) << kFoldPosShift | (c's index in the chunk) << kFoldLmShift, L_off[c]}; src = block-array index of the front
    // entry (-1: structurally zero, -2: another rank's); the group's 6 entries (t + g, j) are the
    // pose-landmark block's values src (t, 0) + 2 g + j
    F.fold_cptr.assign(ns + 1, 0);
    F.fold_chunk.clear();
    F.fold_rec.clear();
    if (!F.fold_list.empty() && F.L_size > INT32_MAX) { err = "multifrontal: factor too large for folding"; return BOS_ERR_UNSUPPORTED; }
    int32_t nrows = 0;
    for (int p = 0; p < ns; ++p) {
        F.fold_cptr[p] = (int32_t)F.fold_chunk.size();
        int32_t chunk_rows = kFoldChunk, chunk_lms = 0;   // forces a new chunk at the parent's first child
        const int cap = fold_chunk_landmarks(F.k[p] + F.r[p]);
        for (int ci = F.child_ptr[p]; ci < F.child_ptr[p] + F.fold_cnt[p]; ++ci) {
            const int c = F.child[ci], rc = F.r[c], mc = 2 + rc, ng = rc / 3;
            if (rc % 3) { err = "multifrontal: folded landmark rows not whole poses"; return BOS_ERR_INVALID; }
            if (chunk_rows + ng > kFoldChunk || chunk_lms >= cap) {
                F.fold_chunk.push_back(nrows);
                chunk_rows = 0;
                chunk_lms = 0;
            }
            std::vector<int32_t> src((size_t)mc * 2, -1);   // (i, j) -> i + j * mc
            for (int q = F.amap_ptr[c]; q < F.amap_ptr[c + 1]; ++q) {
                int64_t d = F.amap_dst[q], j = 0;
                while (d >= mc - j) { d -= mc - j; ++j; }
                src[(j + d) + j * mc] = F.amap_src[q];
            }
            const int32_t* rm = F.rmap.data() + F.rmap_off[c];
            for (int t = 0; t < rc; t += 3) {
                const int32_t b0 = src[2 + t];
                for (int g = 0; g < 3; ++g) {
                    const bool pos_ok = rm[t + g] == rm[t] + g;
                    const bool src_ok = b0 >= 0 ? src[2 + t + g] == b0 + 2 * g && src[2 + t + g + mc] == b0 + 2 * g + 1
                                                : src[2 + t + g] == b0 && src[2 + t + g + mc] == b0;
                    if (!pos_ok || !src_ok) { err = "multifrontal: folded pose rows not one block"; return BOS_ERR_INVALID; }
                }
                const int32_t rec[kFoldRec] = {b0, src[2 + t + mc], src[0], src[1], src[1 + mc], F.col0[c],
                                               t | rc << 6 | rm[t] << kFoldPosShift | chunk_lms << kFoldLmShift,
                                               (int32_t)F.L_off[c]};
                F.fold_rec.insert(F.fold_rec.end(), rec, rec + kFoldRec);
            }
            chunk_rows += ng;
            ++chunk_lms;
            nrows += ng;
        }
    }
    F.fold_cptr[ns] = (int32_t)F.fold_chunk.size();
    F.fold_chunk.push_back(nrows);
    return BOS_OK;
}

bool mf_fold_reads_fp32(const Plan& P) {
    const Multifrontal& F = P.mf;
    const int ns = (int)F.k.size();
    if (ns == 0 || F.fold_rec.empty()) return false;
    const int64_t lo = P.blk.off_ldiag, pl = P.blk.off_pl, hi = P.blk.off_pp;
    if (hi > INT32_MAX) return false;
    std::vector<char> folded(ns, 0);
    for (int p = 0; p < ns; ++p)
        for (int ci = F.child_ptr[p]; ci < F.child_ptr[p] + F.fold_cnt[p]; ++ci) folded[F.child[ci]] = 1;
    for (int s = 0; s < ns; ++s) {
        if (folded[s]) continue;
        for (int q = F.amap_ptr[s]; q < F.amap_ptr[s + 1]; ++q)
            if (F.amap_src[q] >= lo && F.amap_src[q] < hi) return false;
    }
    const size_t nrec = F.fold_rec.size() / kFoldRec;
    for (size_t q = 0; q < nrec; ++q) {
        const int32_t* r = &F.fold_rec[kFoldRec * q];
        if (r[0] >= 0 || r[1] >= 0) {   // a group's block: 6 values from slot (r[0] - pl) / 6
            if (r[0] < pl || r[0] + 6 > hi || (r[0] - pl) % 6 || r[1] != r[0] + 1) return false;
        }
        for (int j = 2; j < 5; ++j)
            if (r[j] >= 0 && (r[j] < lo || r[j] >= pl)) return false;
    }
    return true;
}

// Proves, on the host, that the J+H kernel's writes (simulated here exactly as hip/kernels.hip
// issues them for this rank's lanes) write every value of the block array and every b entry at
// most once, that every value a front this rank factors reads (assembly map and fold records) is
// written exactly once by this rank, and that chi^2 counts every observation once (one GPU; the
// sharded count is checked across ranks by bos_plan_shard_selftest). O(slots + nnz).
int validate_plan(const ProblemIndex& pi, const Plan& P, std::string& err) {
    const int NP = pi.NP, NL = pi.NL;
    const BlockLayout& B = P.blk;
    const Shard& S = P.shard;
    const int L = B.lpp;
    const LaneLists& PL = B.pose_lanes;
    const LaneLists& LL = B.lm_lanes;
    std::vector<uint8_t> hit(B.size, 0), bhit(3 * (size_t)NP + 2 * (size_t)NL, 0);
    std::vector<int32_t> chi(pi.Mb + pi.Mo, 0);
    auto mark = [&](int64_t v0, int cnt) -> bool {
        if (v0 < 0 || v0 + cnt > B.size) return false;
        for (int i = 0; i < cnt; ++i) ++hit[v0 + i];
        return true;
    };
    std::vector<int32_t> slot_block(PL.slots(), -1);   // landmark whose block lives in the slot
    for (int p = 0; p < NP; ++p)
        for (int u = B.ub_ptr[p]; u < B.ub_ptr[p + 1]; ++u) slot_block[B.ub_slot[u]] = B.ub_lm[u];
    if ((int64_t)PL.cnt.size() != (int64_t)B.lane_pose.size() * L) { err = "pose lane count"; return BOS_ERR_INVALID; }
    for (size_t i = 0; i < B.lane_pose.size(); ++i) {
        const int p = B.lane_pose[i];
        if (p < 0) {
            for (int sub = 0; sub < L; ++sub)
                if (PL.cnt[i * L + sub]) { err = "padding lane with items"; return BOS_ERR_INVALID; }
            continue;
        }
        if (!mark(6 * (int64_t)p, 6)) { err = "pose diagonal out of range"; return BOS_ERR_INVALID; }
        for (int d = 0; d < 3; ++d) ++bhit[3 * (size_t)p + d];
        const bool counts = (int)i < S.own_pose_lanes || S.rank == 0;   // chi^2 of top lanes: rank 0
        for (int sub = 0; sub < L; ++sub) {
            const int g = (int)i * L + sub, n = PL.cnt[g];
            if (n > PL.w_len[g / 64]) { err = "lane longer than its wave"; return BOS_ERR_INVALID; }
            for (int j = 0; j < n; ++j) {
                const int32_t sl = lane_slot(PL, g, j), k = PL.obs[sl];
                if (k < 0 || pi.b_pose[k] != p) { err = "bearing slot of the wrong pose"; return BOS_ERR_INVALID; }
                if (counts) ++chi[k];
                if (j + 1 == n || pi.b_lm[PL.obs[lane_slot(PL, g, j + 1)]] != pi.b_lm[k]) {
                    if (slot_block[sl] != pi.b_lm[k] || !mark(B.off_pl + 6 * (int64_t)sl, 6)) {
                        err = "pose-landmark block misplaced";
                        return BOS_ERR_INVALID;
                    }
                }
            }
        }
        for (int x = B.po_ptr[p]; x < B.po_ptr[p + 1]; ++x) {
            const int32_t e = B.po_ent[x];
            const int k = e >> 1;
            if ((e & 1) ? pi.o_dst[k] != p : pi.o_src[k] != p) { err = "odometry entry of the wrong pose"; return BOS_ERR_INVALID; }
            if (!(e & 1) && counts) ++chi[pi.Mb + k];
            const int q = (e & 1) ? pi.o_src[k] : pi.o_dst[k];
            const int u = B.po_blk[x];
            if ((u >= 0) != (q > p)) { err = "pose-pose block on the wrong side"; return BOS_ERR_INVALID; }
            if (u >= 0 && (x + 1 == B.po_ptr[p + 1] || B.po_blk[x + 1] != u)) {
                if (u < B.uo_ptr[p] || u >= B.uo_ptr[p + 1] || B.uo_dst[u] != q ||
                    !mark(B.off_pp + 6 * (int64_t)u, 6)) {
                    err = "pose-pose block misplaced";
                    return BOS_ERR_INVALID;
                }
            }
        }
    }
    const int NLL = (int)B.lm_lane_lm.size();
    if ((int)LL.cnt.size() != NLL) { err = "landmark lane count"; return BOS_ERR_INVALID; }
    for (int g = 0; g < NLL; ++g) {
        const int l = B.lm_lane_lm[g];
        if (LL.cnt[g] > LL.w_len[g / 64]) { err = "lane longer than its wave"; return BOS_ERR_INVALID; }
        for (int j = 0; j < LL.cnt[g]; ++j) {
            const int32_t k = LL.obs[lane_slot(LL, g, j)];
            if (k < 0 || pi.b_lm[k] != l) { err = "bearing slot of the wrong landmark"; return BOS_ERR_INVALID; }
        }
        if (!mark(B.off_ldiag + 3 * (int64_t)l, 3)) { err = "landmark diagonal out of range"; return BOS_ERR_INVALID; }
        for (int d = 0; d < 2; ++d) ++bhit[3 * (size_t)NP + 2 * (size_t)l + d];
    }
    for (int64_t v = 0; v < B.size; ++v)
        if (hit[v] > 1) {
            err = "block value " + std::to_string(v) + " written " + std::to_string((int)hit[v]) + " times";
            return BOS_ERR_INVALID;
        }
    for (size_t v = 0; v < bhit.size(); ++v)
        if (bhit[v] > 1 || (S.world == 1 && bhit[v] != 1)) { err = "b entry coverage"; return BOS_ERR_INVALID; }
    if (S.world == 1)   // every observation's chi^2 counted once (self-loops: by the step's stats)
        for (size_t k = 0; k < chi.size(); ++k)
            if (chi[k] != ((k >= (size_t)pi.Mb && pi.o_src[k - pi.Mb] == pi.o_dst[k - pi.Mb]) ? 0 : 1)) {
                err = "chi^2 of observation " + std::to_string(k) + " counted " + std::to_string(chi[k]) + " times";
                return BOS_ERR_INVALID;
            }
    // every stored entry this rank computes reads a block value it writes; pose-pose blocks are
    // symmetric (off-diagonal values read twice), every other value at most once
    std::vector<uint8_t> refs(B.size, 0);
    for (int32_t v : B.csr_src) {
        if (v == -2) { if (S.world == 1) { err = "stored entry not computed"; return BOS_ERR_INVALID; } continue; }
        if (v < 0 || v >= B.size) { err = "stored entry reads outside the block array"; return BOS_ERR_INVALID; }
        if (++refs[v] > (v >= B.off_pp ? 2 : 1)) { err = "block value read by two stored entries"; return BOS_ERR_INVALID; }
        if (hit[v] != 1) { err = "block value read by the solver is never written"; return BOS_ERR_INVALID; }
    }
    // the fronts this rank factors (its own and the top) read only values it computes
    const Multifrontal& F = P.mf;
    for (int s = 0; s < F.nsuper; ++s) {
        if (S.sn_owner.empty() || (S.sn_owner[s] != S.rank && S.sn_owner[s] != -1)) continue;
        for (int q = F.amap_ptr[s]; q < F.amap_ptr[s + 1]; ++q)
            if (F.amap_src[q] < 0) { err = "a front of this rank reads H computed by another rank"; return BOS_ERR_INVALID; }
    }
    for (int p = 0; p < F.nsuper; ++p) {
        if (F.fold_cnt.empty() || S.sn_owner.empty() || (S.sn_owner[p] != S.rank && S.sn_owner[p] != -1)) continue;
        for (int ch = F.fold_cptr[p]; ch < F.fold_cptr[p + 1]; ++ch)
            for (int q = F.fold_chunk[ch]; q < F.fold_chunk[ch + 1]; ++q)
                for (int t = 0; t < 5; ++t)
                    if (F.fold_rec[(size_t)kFoldRec * q + t] == -2) {
                        err = "a folded landmark of this rank reads H computed by another rank";
                        return BOS_ERR_INVALID;
                    }
    }
    return BOS_OK;
}

}  // namespace bos

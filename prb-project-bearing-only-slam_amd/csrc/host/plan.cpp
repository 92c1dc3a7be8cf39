#include "plan.hpp"

#include <algorithm>
#include <cstdio>
#include <numeric>

#include "../../../include/bos.h"

namespace bos {

namespace {

constexpr int kWave = 64;             // wavefront width on CDNA4
constexpr int kMfLeaf = 12;
constexpr int kStageCap = 1024;       // largest CSR span (values) a task assembles in LDS
constexpr int kMaxTaskNodes = 48;     // nodes of one multi-node J+H task (hip/kernels.hpp kMaxTaskNodes)

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
        for (int k = 1; k + 1 < h; ++k) {
            const int64_t below = cum[k - 1], above = tot - cum[k];
            if (below * 5 < tot || above * 5 < tot) continue;
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

int order_nodes(const ProblemIndex& pi, bool nd_only, std::vector<int32_t>& node_pos,
                std::vector<std::pair<int32_t, int32_t>>* blocks, OrderingReport& rep, std::string& err) {
    const int NP = pi.NP, NL = pi.NL, n = NP + NL;
    const Graph g = build_graph(pi);
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

int build_multifrontal(const Graph& g, int NP, Plan& P, const std::vector<int32_t>& inv,
                       const std::vector<std::pair<int32_t, int32_t>>& blocks, std::string& err);

template <typename BlockOffset>
int build_tasks(const ProblemIndex& pi, Plan& P, int q_begin, int q_end, const std::vector<int32_t>& pb_ptr,
                const std::vector<int32_t>& pb, const std::vector<int32_t>& lb_ptr, const std::vector<int32_t>& lb,
                const std::vector<int32_t>& po_ptr, const std::vector<int32_t>& po, BlockOffset&& block_offset,
                std::string& err);

int build_plan(const ProblemIndex& pi, int rank, int world, int factor_mode, Plan& P, std::string& err) {
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
        if (pi.o_src[k] == pi.o_dst[k]) {
            err = "odometry edge " + std::to_string(k) + " is a self loop (not supported)";
            return BOS_ERR_UNSUPPORTED;
        }
    }
    P = Plan();
    P.NP = NP; P.NL = NL; P.Mb = pi.Mb; P.Mo = pi.Mo; P.fixed = pi.fixed;
    std::vector<std::pair<int32_t, int32_t>> blocks;
    int rc = order_nodes(pi, factor_mode == kFactorMultifrontal, P.node_pos, &blocks, P.ordering, err);
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

    // lower neighbours (by position) of every node, with their offsets inside the node's rows
    std::vector<int64_t> lptr(n_nodes + 1, 0);
    std::vector<int32_t> lnb;              // neighbour node ids, sorted by position
    std::vector<int32_t> loff;             // entry offset of that neighbour's block in each row
    lnb.reserve(g.adj.size() / 2 + 1);
    P.node_base.assign(n_nodes, -1);
    P.node_row0.assign(n_nodes, -1);
    P.rowptr.assign(P.n + 1, 0);
    for (int i = 0; i < m; ++i) {
        const int u = inv[i];
        std::vector<int32_t> nb;
        for (int64_t e = g.ptr[u]; e < g.ptr[u + 1]; ++e)
            if (P.node_pos[g.adj[e]] < i) nb.push_back(g.adj[e]);
        std::sort(nb.begin(), nb.end(), [&](int a, int b) { return P.node_pos[a] < P.node_pos[b]; });
        lptr[u] = (int64_t)lnb.size();
        int32_t off = 0;
        for (int v : nb) { lnb.push_back(v); loff.push_back(off); off += node_size(v, NP); }
        P.node_base[u] = off;
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
        P.node_row0[u] = P.rowptr[r0];
        for (int d = 0; d < su; ++d) {
            int64_t w = P.rowptr[r0 + d];
            for (int64_t e = lptr[u]; e < lend[u]; ++e) {
                const int v = lnb[e];
                for (int c = 0; c < node_size(v, NP); ++c) P.colind[w++] = P.node_dof[v] + c;
            }
            for (int c = 0; c <= d; ++c) P.colind[w++] = (int32_t)(r0 + c);
        }
    }
    auto block_offset = [&](int owner, int other) -> int32_t {
        // offset of other's block inside owner's rows (binary search by position)
        int64_t lo = lptr[owner], hi = lend[owner];
        const int key = P.node_pos[other];
        while (lo < hi) {
            const int64_t mid = (lo + hi) / 2;
            if (P.node_pos[lnb[mid]] < key) lo = mid + 1; else hi = mid;
        }
        return (lo < lend[owner] && lnb[lo] == other) ? loff[lo] : -1;
    };

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

    // incidence lists
    std::vector<int32_t> pb_ptr(NP + 1, 0), lb_ptr(NL + 1, 0), po_ptr(NP + 1, 0);
    for (int k = 0; k < pi.Mb; ++k) { ++pb_ptr[pi.b_pose[k] + 1]; ++lb_ptr[pi.b_lm[k] + 1]; }
    for (int k = 0; k < pi.Mo; ++k) { ++po_ptr[pi.o_src[k] + 1]; ++po_ptr[pi.o_dst[k] + 1]; }
    for (int i = 0; i < NP; ++i) { pb_ptr[i + 1] += pb_ptr[i]; po_ptr[i + 1] += po_ptr[i]; }
    for (int j = 0; j < NL; ++j) lb_ptr[j + 1] += lb_ptr[j];
    std::vector<int32_t> pb(pi.Mb), lb(pi.Mb), po(2 * (size_t)pi.Mo);
    {
        std::vector<int32_t> a(pb_ptr.begin(), pb_ptr.end() - 1), b(lb_ptr.begin(), lb_ptr.end() - 1),
            c(po_ptr.begin(), po_ptr.end() - 1);
        for (int k = 0; k < pi.Mb; ++k) { pb[a[pi.b_pose[k]]++] = k; lb[b[pi.b_lm[k]]++] = k; }
        for (int k = 0; k < pi.Mo; ++k) { po[c[pi.o_src[k]]++] = 2 * k; po[c[pi.o_dst[k]]++] = 2 * k + 1; }
    }

    // ownership: contiguous position ranges balanced by work (incident items)
    std::vector<int64_t> work(m);
    int64_t total = 0;
    for (int i = 0; i < m; ++i) {
        const int u = inv[i];
        work[i] = 1 + (u < NP ? (pb_ptr[u + 1] - pb_ptr[u]) + (po_ptr[u + 1] - po_ptr[u]) : (lb_ptr[u - NP + 1] - lb_ptr[u - NP]));
        total += work[i];
    }
    std::vector<int32_t> cut(world + 1, 0);
    {
        int64_t acc = 0;
        int r = 1;
        for (int i = 0; i < m && r < world; ++i) {
            acc += work[i];
            while (r < world && acc * world >= total * r) cut[r++] = i + 1;
        }
        while (r < world) cut[r++] = m;
        cut[world] = m;
    }
    P.rank_row_begin.assign(world + 1, 0);
    for (int r = 0; r <= world; ++r) P.rank_row_begin[r] = cut[r] < m ? P.node_dof[inv[cut[r]]] : (int32_t)P.n;
    P.row_begin = P.rank_row_begin[rank];
    P.row_end = P.rank_row_begin[rank + 1];
    P.val_begin = P.rowptr[P.row_begin];
    P.val_end = P.rowptr[P.row_end];

    // per-position node layout (the J+H kernel walks positions)
    P.pos_node.assign(m, 0); P.pos_row0.assign(m + 1, 0); P.pos_base.assign(m, 0); P.pos_dof.assign(m + 1, 0);
    for (int q = 0; q < m; ++q) {
        const int u = inv[q];
        P.pos_node[q] = u; P.pos_row0[q] = P.node_row0[u]; P.pos_base[q] = P.node_base[u]; P.pos_dof[q] = P.node_dof[u];
    }
    P.pos_row0[m] = (int32_t)P.nnzA();
    P.pos_dof[m] = (int32_t)P.n;
    rc = build_tasks(pi, P, cut[rank], cut[rank + 1], pb_ptr, pb, lb_ptr, lb, po_ptr, po, block_offset, err);
    if (rc) return rc;
    if (factor_mode == kFactorMultifrontal && (rc = build_multifrontal(g, NP, P, inv, blocks, err))) return rc;
    return validate_plan(pi, P, err);
}

// Node-range tasks of the J+H kernel (see RangeTasks in plan.hpp).
template <typename BlockOffset>
int build_tasks(const ProblemIndex& pi, Plan& P, int q_begin, int q_end, const std::vector<int32_t>& pb_ptr,
                const std::vector<int32_t>& pb, const std::vector<int32_t>& lb_ptr, const std::vector<int32_t>& lb,
                const std::vector<int32_t>& po_ptr, const std::vector<int32_t>& po, BlockOffset&& block_offset,
                std::string& err) {
    const int NP = pi.NP;
    RangeTasks& T = P.tasks;
    T = RangeTasks();
    const int m = (int)P.pos_node.size();
    T.cl_ptr.assign(m + 1, 0);
    std::vector<int32_t> stamp_b(pi.Mb, -1), stamp_o(pi.Mo, -1);
    auto pos_of = [&](int node) { return node == pi.fixed ? -1 : P.node_pos[node]; };
    auto count_entries = [&](int q, int tid) {   // new entries node at q would add to task tid
        const int u = P.pos_node[q];
        int c = 0;
        if (u < NP) {
            for (int32_t e = pb_ptr[u]; e < pb_ptr[u + 1]; ++e) c += stamp_b[pb[e]] != tid;
            for (int32_t e = po_ptr[u]; e < po_ptr[u + 1]; ++e) c += stamp_o[po[e] >> 1] != tid;
        } else {
            const int l = u - NP;
            for (int32_t e = lb_ptr[l]; e < lb_ptr[l + 1]; ++e) c += stamp_b[lb[e]] != tid;
        }
        return c;
    };
    auto mark = [&](int q, int tid) {
        const int u = P.pos_node[q];
        if (u < NP) {
            for (int32_t e = pb_ptr[u]; e < pb_ptr[u + 1]; ++e) stamp_b[pb[e]] = tid;
            for (int32_t e = po_ptr[u]; e < po_ptr[u + 1]; ++e) stamp_o[po[e] >> 1] = tid;
        } else {
            for (int32_t e = lb_ptr[u - NP]; e < lb_ptr[u - NP + 1]; ++e) stamp_b[lb[e]] = tid;
        }
    };
    // 1. cut the position range into tasks
    T.task_q.push_back(q_begin);
    int tid = 0;
    for (int q = q_begin; q < q_end;) {
        int entries = count_entries(q, tid);
        mark(q, tid);
        int q1 = q + 1;
        if (entries <= kWave && P.pos_row0[q1] - P.pos_row0[q] <= kStageCap) {
            while (q1 < q_end && q1 - q < kMaxTaskNodes) {
                const int add = count_entries(q1, tid);
                if (entries + add > kWave || P.pos_row0[q1 + 1] - P.pos_row0[q] > kStageCap) break;
                entries += add;
                mark(q1, tid);
                ++q1;
            }
        }
        T.task_q.push_back(q1);
        q = q1;
        ++tid;
    }
    // 2. entries, flags, contribution lists
    std::fill(stamp_b.begin(), stamp_b.end(), -1);
    std::fill(stamp_o.begin(), stamp_o.end(), -1);
    T.task_be.push_back(0);
    T.task_oe.push_back(0);
    std::vector<std::vector<uint16_t>> node_slots;
    for (int t = 0; t < (int)T.task_q.size() - 1; ++t) {
        const int q0 = T.task_q[t], q1 = T.task_q[t + 1];
        const int v0 = P.pos_row0[q0];
        const bool single = q1 - q0 == 1;
        const bool staged = P.pos_row0[q1] - v0 <= kStageCap;
        T.task_flags.push_back((uint8_t)((staged ? 1 : 0) | (single ? 2 : 0)));
        auto inside = [&](int node) { const int q = pos_of(node); return q >= q0 && q < q1; };
        auto owner_and_slot = [&](int a, int b, int& meta) {
            // the block (a, b) lives in the rows of the later of the two (the fixed pose has no rows)
            if (a == pi.fixed || b == pi.fixed) return;
            const bool b_owner = P.node_pos[b] > P.node_pos[a];
            const int own = b_owner ? b : a, oth = b_owner ? a : b;
            if (!inside(own)) return;
            const int32_t off = block_offset(own, oth);
            if (off < 0) { meta = -1; return; }
            meta |= 8 | (b_owner ? 16 : 0) | ((P.node_row0[own] + off - v0) << 8);
        };
        auto counts_here = [&](int a, int b) {
            // chi^2 of an observation is counted in the task of its owner (or of its non-fixed end)
            int own;
            if (a == pi.fixed) own = b;
            else if (b == pi.fixed) own = a;
            else own = P.node_pos[b] > P.node_pos[a] ? b : a;
            return inside(own);
        };
        const int be_first = (int)T.be_pose.size(), oe_first = (int)T.oe_edge.size();
        for (int q = q0; q < q1; ++q) {
            const int u = P.pos_node[q];
            if (u < NP) {
                for (int32_t e = pb_ptr[u]; e < pb_ptr[u + 1]; ++e) {
                    const int k = pb[e];
                    if (stamp_b[k] == t) continue;
                    stamp_b[k] = t;
                    const int p = pi.b_pose[k], l = NP + pi.b_lm[k];
                    int meta = (inside(p) ? 1 : 0) | (inside(l) ? 2 : 0) | (counts_here(p, l) ? 4 : 0);
                    owner_and_slot(p, l, meta);
                    if (meta < 0) { err = "internal error: bearing block missing"; return BOS_ERR_INVALID; }
                    T.be_pose.push_back(pi.b_pose[k]); T.be_lm.push_back(pi.b_lm[k]);
                    T.be_meta.push_back(meta); T.be_obs.push_back(k);
                }
                for (int32_t e = po_ptr[u]; e < po_ptr[u + 1]; ++e) {
                    const int k = po[e] >> 1;
                    if (stamp_o[k] == t) continue;
                    stamp_o[k] = t;
                    const int s = pi.o_src[k], d = pi.o_dst[k];
                    int meta = (inside(s) ? 1 : 0) | (inside(d) ? 2 : 0) | (counts_here(s, d) ? 4 : 0);
                    owner_and_slot(s, d, meta);
                    if (meta < 0) { err = "internal error: odometry block missing"; return BOS_ERR_INVALID; }
                    T.oe_edge.push_back(k); T.oe_meta.push_back(meta);
                }
            } else {
                for (int32_t e = lb_ptr[u - NP]; e < lb_ptr[u - NP + 1]; ++e) {
                    const int k = lb[e];
                    if (stamp_b[k] == t) continue;
                    stamp_b[k] = t;
                    const int p = pi.b_pose[k], l = NP + pi.b_lm[k];
                    int meta = (inside(p) ? 1 : 0) | (inside(l) ? 2 : 0) | (counts_here(p, l) ? 4 : 0);
                    owner_and_slot(p, l, meta);
                    if (meta < 0) { err = "internal error: bearing block missing"; return BOS_ERR_INVALID; }
                    T.be_pose.push_back(pi.b_pose[k]); T.be_lm.push_back(pi.b_lm[k]);
                    T.be_meta.push_back(meta); T.be_obs.push_back(k);
                }
            }
        }
        const int nb = (int)T.be_pose.size() - be_first, no = (int)T.oe_edge.size() - oe_first;
        T.max_entries = std::max(T.max_entries, nb + no);
        if (!single && nb + no > kWave) { err = "internal error: task too large"; return BOS_ERR_INVALID; }
        // contribution slots per node (entry order = fixed reduction order)
        for (int q = q0; q < q1; ++q) {
            const int u = P.pos_node[q];
            std::vector<uint16_t> sl;
            for (int i = 0; i < nb; ++i) {
                const int bi = be_first + i;
                if (u < NP ? (T.be_pose[bi] == u) : (T.be_lm[bi] == u - NP)) sl.push_back((uint16_t)(2 * i + (u < NP ? 0 : 1)));
            }
            for (int j = 0; j < no; ++j) {
                const int k = T.oe_edge[oe_first + j];
                if (u < NP && pi.o_src[k] == u) sl.push_back((uint16_t)(2 * (nb + j)));
                if (u < NP && pi.o_dst[k] == u) sl.push_back((uint16_t)(2 * (nb + j) + 1));
            }
            T.cl_ptr[q + 1] = (int32_t)sl.size();
            if (!single) T.cl.insert(T.cl.end(), sl.begin(), sl.end());
            else T.cl_ptr[q + 1] = 0;   // single-node tasks reduce every entry
        }
        T.task_be.push_back((int32_t)T.be_pose.size());
        T.task_oe.push_back((int32_t)T.oe_edge.size());
    }
    for (int q = 0; q < m; ++q) T.cl_ptr[q + 1] += T.cl_ptr[q];
    // 3. duplicate off-diagonal blocks: the first entry of a group writes, with the group's summed
    //    information; the others do not write
    T.be_woff.clear();
    T.oe_omoff.clear();
    {
        std::vector<std::pair<int64_t, int>> key;   // (absolute slot, entry)
        for (int t = 0; t < T.ntask(); ++t) {
            const int v0 = P.pos_row0[T.task_q[t]];
            for (int i = T.task_be[t]; i < T.task_be[t + 1]; ++i)
                if (T.be_meta[i] & 8) key.push_back({(int64_t)v0 + (T.be_meta[i] >> 8), i});
            for (int j = T.task_oe[t]; j < T.task_oe[t + 1]; ++j)
                if (T.oe_meta[j] & 8) key.push_back({(int64_t)v0 + (T.oe_meta[j] >> 8), -1 - j});
        }
        std::sort(key.begin(), key.end());
        for (size_t a = 0; a < key.size();) {
            size_t b = a + 1;
            while (b < key.size() && key[b].first == key[a].first) ++b;
            if (b - a > 1) {
                if (!T.has_dups) {
                    T.has_dups = true;
                    T.be_woff.assign(T.be_pose.size(), 0.0);
                    T.oe_omoff.assign(6 * T.oe_edge.size(), 0.0);
                    for (size_t i = 0; i < T.be_pose.size(); ++i) T.be_woff[i] = (T.be_meta[i] & 8) ? 1.0 : 0.0;
                }
                const bool bearing = key[a].second >= 0;
                for (size_t c = a; c < b; ++c)
                    if ((key[c].second >= 0) != bearing) { err = "bearing and odometry share a block"; return BOS_ERR_INVALID; }
                if (bearing) {
                    double wsum = 0;
                    for (size_t c = a; c < b; ++c) {
                        const int i = key[c].second;
                        wsum += pi.b_omega ? pi.b_omega[T.be_obs[i]] : 1.0;
                        if (c > a) { T.be_meta[i] &= ~8; T.be_woff[i] = 0.0; }
                    }
                    T.be_woff[key[a].second] = wsum;
                } else {
                    const int j0 = -1 - key[a].second;
                    const int s0 = pi.o_src[T.oe_edge[j0]];
                    double om[6] = {0, 0, 0, 0, 0, 0};
                    for (size_t c = a; c < b; ++c) {
                        const int j = -1 - key[c].second;
                        if (pi.o_src[T.oe_edge[j]] != s0) {
                            err = "odometry edges in both directions between the same poses (not supported)";
                            return BOS_ERR_UNSUPPORTED;
                        }
                        const double* M = pi.o_omega + 9 * (size_t)T.oe_edge[j];
                        const double u6[6] = {M[0], M[1], M[2], M[4], M[5], M[8]};
                        for (int z = 0; z < 6; ++z) om[z] += u6[z];
                        if (c > a) T.oe_meta[j] &= ~8;
                    }
                    for (int z = 0; z < 6; ++z) T.oe_omoff[6 * (size_t)j0 + z] = om[z];
                }
            }
            a = b;
        }
        if (T.has_dups) {   // entries of singleton blocks use their own information
            for (size_t j = 0; j < T.oe_edge.size(); ++j) {
                bool zero = true;
                for (int z = 0; z < 6; ++z) zero = zero && T.oe_omoff[6 * j + z] == 0.0;
                if (zero && (T.oe_meta[j] & 8)) {
                    const double* M = pi.o_omega + 9 * (size_t)T.oe_edge[j];
                    const double u6[6] = {M[0], M[1], M[2], M[4], M[5], M[8]};
                    for (int z = 0; z < 6; ++z) T.oe_omoff[6 * j + z] = u6[z];
                }
            }
        }
    }
    return BOS_OK;
}

int build_multifrontal(const Graph& g, int NP, Plan& P, const std::vector<int32_t>& inv,
                       const std::vector<std::pair<int32_t, int32_t>>& blocks, std::string& err) {
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
    F.rmap_off.resize(ns + 1);
    F.L_off.resize(ns); F.U_off.resize(ns); F.u_off.resize(ns);
    std::vector<int32_t> lev(ns, 0);
    for (int s = 0; s < ns; ++s) {
        const int k = F.k[s], r = F.r[s], mm = k + r;
        F.max_m = std::max(F.max_m, mm);
        F.L_off[s] = F.L_size; F.L_size += (int64_t)mm * k;
        F.U_off[s] = F.U_size; F.U_size += (int64_t)r * r;
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
            lev[p] = std::max(lev[p], lev[s] + 1);
        } else if (r != 0) {
            err = "multifrontal: root with update rows";
            return BOS_ERR_INVALID;
        }
    }
    F.rmap_off[ns] = (int64_t)F.rmap.size();
    F.nlevels = 0;
    for (int s = 0; s < ns; ++s) F.nlevels = std::max(F.nlevels, lev[s] + 1);
    F.level_ptr.assign(F.nlevels + 1, 0);
    for (int s = 0; s < ns; ++s) ++F.level_ptr[lev[s] + 1];
    for (int l = 0; l < F.nlevels; ++l) F.level_ptr[l + 1] += F.level_ptr[l];
    F.level.resize(ns);
    {
        std::vector<int32_t> w(F.level_ptr.begin(), F.level_ptr.end() - 1);
        for (int s = 0; s < ns; ++s) F.level[w[lev[s]]++] = s;
    }
    // assembly map: every stored entry of H (row i >= col j) goes to the front of col j's supernode
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
            dst[e] = li + (j - F.col0[s]) * (F.k[s] + F.r[s]);
            ++F.amap_ptr[s + 1];
        }
    for (int s = 0; s < ns; ++s) F.amap_ptr[s + 1] += F.amap_ptr[s];
    F.amap_src.resize(nnz);
    F.amap_dst.resize(nnz);
    {
        std::vector<int32_t> w(F.amap_ptr.begin(), F.amap_ptr.end() - 1);
        for (int64_t e = 0; e < nnz; ++e) {
            const int32_t q = w[tgt[e]]++;
            F.amap_src[q] = (int32_t)e;
            F.amap_dst[q] = dst[e];
        }
    }
    return BOS_OK;
}

// Proves, on the host, that every address the J+H kernel writes (hip/kernels.hip diag_pos /
// off_pos) lies inside the intended CSR row at the intended column, so a kernel launch can
// never write out of bounds. O(items).
int validate_plan(const ProblemIndex& pi, const Plan& P, std::string& err) {
    const int NP = pi.NP;
    const int64_t nnz = P.nnzA();
    const RangeTasks& T = P.tasks;
    auto check_entry = [&](int owner, int r, int64_t pos, int32_t want_col) -> bool {
        const int64_t row = (int64_t)P.node_dof[owner] + r;
        if (row < 0 || row >= P.n) return false;
        if (pos < P.rowptr[row] || pos >= P.rowptr[row + 1] || pos >= nnz) return false;
        return P.colind[pos] == want_col;
    };
    auto pos_off = [](int64_t slot, int base, int r, int c) { return slot + (int64_t)r * base + r * (r + 1) / 2 + c; };
    auto pos_diag = [](int64_t row0, int base, int r, int c) { return row0 + (int64_t)r * base + r * (r + 1) / 2 + base + c; };
    std::vector<uint8_t> hit(nnz, 0);
    std::vector<int32_t> bcount(P.n, 0);
    std::vector<int32_t> chi(pi.Mb + pi.Mo, 0);
    for (int t = 0; t < T.ntask(); ++t) {
        const int q0 = T.task_q[t], q1 = T.task_q[t + 1];
        if (q1 <= q0) { err = "empty task"; return BOS_ERR_INVALID; }
        const int64_t v0 = P.pos_row0[q0];
        for (int q = q0; q < q1; ++q) {
            const int u = P.pos_node[q];
            const int su = node_size(u, NP);
            for (int r = 0; r < su; ++r) {
                ++bcount[P.node_dof[u] + r];
                for (int c = 0; c <= r; ++c) {
                    const int64_t pd = pos_diag(P.node_row0[u], P.node_base[u], r, c);
                    if (!check_entry(u, r, pd, P.node_dof[u] + c)) { err = "diagonal block misplaced"; return BOS_ERR_INVALID; }
                    ++hit[pd];
                }
            }
        }
        auto check_off = [&](int a, int b, int meta) -> bool {
            if (!(meta & 8)) return true;
            const int own = (meta & 16) ? b : a, oth = (meta & 16) ? a : b;
            const int qo = P.node_pos[own];
            if (qo < q0 || qo >= q1) return false;
            const int64_t slot = v0 + (meta >> 8);
            for (int r = 0; r < node_size(own, NP); ++r)
                for (int c = 0; c < node_size(oth, NP); ++c) {
                    const int64_t p = pos_off(slot, P.node_base[own], r, c);
                    if (!check_entry(own, r, p, P.node_dof[oth] + c)) return false;
                    ++hit[p];
                }
            return true;
        };
        for (int i = T.task_be[t]; i < T.task_be[t + 1]; ++i) {
            if (!check_off(T.be_pose[i], NP + T.be_lm[i], T.be_meta[i])) { err = "bearing block misplaced"; return BOS_ERR_INVALID; }
            if (T.be_meta[i] & 4) ++chi[T.be_obs[i]];
        }
        for (int j = T.task_oe[t]; j < T.task_oe[t + 1]; ++j) {
            const int k = T.oe_edge[j];
            if (!check_off(pi.o_src[k], pi.o_dst[k], T.oe_meta[j])) { err = "odometry block misplaced"; return BOS_ERR_INVALID; }
            if (T.oe_meta[j] & 4) ++chi[pi.Mb + k];
        }
        if (!(T.task_flags[t] & 2) && T.task_be[t + 1] - T.task_be[t] + T.task_oe[t + 1] - T.task_oe[t] > 64) {
            err = "multi-node task exceeds one wavefront";
            return BOS_ERR_INVALID;
        }
    }
    for (int64_t e = 0; e < nnz; ++e) {
        const bool owned = e >= P.val_begin && e < P.val_end;
        if (hit[e] != (owned ? 1 : 0)) {
            err = "CSR entry " + std::to_string(e) + " written " + std::to_string((int)hit[e]) + " times";
            return BOS_ERR_INVALID;
        }
    }
    for (int64_t i = 0; i < P.n; ++i)
        if (bcount[i] != ((i >= P.row_begin && i < P.row_end) ? 1 : 0)) { err = "b entry coverage"; return BOS_ERR_INVALID; }
    if (P.rank_row_begin.size() == 2)   // single shard: every observation's chi^2 counted once
        for (size_t k = 0; k < chi.size(); ++k)
            if (chi[k] != 1) { err = "chi^2 of observation " + std::to_string(k) + " counted " + std::to_string(chi[k]) + " times"; return BOS_ERR_INVALID; }
    return BOS_OK;
}

}  // namespace bos

// Multi-GPU sharding of the multifrontal solve (plan.hpp Shard).
//
// The reference solves the whole normal system on one CPU thread (slam/solver.cpp:75-85); the J+H
// build is one pass over independent observations (:28-69). Here the sparse Cholesky's assembly
// tree is cut into subtrees, one or more per rank, below a replicated top. Rank r then
//   * builds the part of H and b its fronts read: the J+H lanes of its own nodes and of the top
//     nodes (no part of H crosses ranks),
//   * factors its subtrees, exchanges the subtree roots' update matrices / u-vectors (exchange 1),
//     factors and solves the top (every rank, same arithmetic), solves its subtrees backward,
//   * exchanges the solution of the boundary nodes (exchange 2) and applies the box-plus to its
//     own, the top and the boundary nodes — exactly the nodes its next J+H reads.
// Every value is computed by the same operations in the same order as on one GPU, so a sharded
// iteration reproduces the single-GPU one bit for bit.
#include <algorithm>
#include <numeric>

#include "../../../include/bos.h"
#include "plan.hpp"

namespace bos {

// Ownership (cut of the assembly tree), lane sets, exchange tables. Needs P.mf (the tree) and
// P.node_dof / P.n.
int build_shard(const ProblemIndex& pi, Plan& P, int rank, int world, std::string& err) {
    const int NP = pi.NP, NL = pi.NL, nn = NP + NL;
    const Multifrontal& F = P.mf;
    Shard& S = P.shard;
    S = Shard();
    S.rank = rank;
    S.world = world;
    const int ns = F.nsuper;
    std::vector<char> folded(ns, 0);
    for (int s : F.fold_list) folded[s] = 1;
    // work of a subtree: its dofs (each front's own columns and its folded landmarks')
    std::vector<double> work(ns, 0.0), sub(ns, 0.0);
    for (int s = 0; s < ns; ++s) {
        work[s] = F.k[s];
        for (int ci = F.child_ptr[s]; ci < F.child_ptr[s] + F.fold_cnt[s]; ++ci) work[s] += F.k[F.child[ci]];
    }
    for (int s = 0; s < ns; ++s) {   // children precede parents
        if (folded[s]) continue;
        sub[s] += work[s];
        if (F.parent[s] >= 0) sub[F.parent[s]] += sub[s];
    }
    auto kids = [&](int s, std::vector<int>& out) {
        out.clear();
        for (int ci = F.child_ptr[s] + F.fold_cnt[s]; ci < F.child_ptr[s + 1]; ++ci) out.push_back(F.child[ci]);
    };
    std::vector<int> open, top, tmp;
    for (int s = 0; s < ns; ++s)
        if (!folded[s] && F.parent[s] < 0) open.push_back(s);
    std::vector<int> bin_of;   // LPT assignment of `open`
    auto assign = [&]() {
        std::vector<int> ord(open.size());
        std::iota(ord.begin(), ord.end(), 0);
        std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return sub[open[a]] > sub[open[b]]; });
        std::vector<double> load(world, 0.0);
        bin_of.assign(open.size(), 0);
        for (int i : ord) {
            const int b = (int)(std::min_element(load.begin(), load.end()) - load.begin());
            bin_of[i] = b;
            load[b] += sub[open[i]];
        }
        double tot = 0.0;
        for (double l : load) tot += l;
        return *std::max_element(load.begin(), load.end()) / std::max(tot / world, 1e-300);
    };
    if (world > 1) {
        // split the heaviest open subtree (its root joins the top) until the ranks' loads are within
        // 5 % of each other, or nothing is left to split
        for (;;) {
            const double imb = assign();
            if (imb <= 1.05 || (int)open.size() >= 32 * world) break;
            int best = -1;
            for (size_t i = 0; i < open.size(); ++i) {
                kids(open[i], tmp);
                if (!tmp.empty() && (best < 0 || sub[open[i]] > sub[open[best]])) best = (int)i;
            }
            if (best < 0) break;
            const int s = open[best];
            open.erase(open.begin() + best);
            top.push_back(s);
            kids(s, tmp);
            open.insert(open.end(), tmp.begin(), tmp.end());
        }
    } else {
        bin_of.assign(open.size(), 0);
    }
    S.sn_owner.assign(ns, -1);
    {
        std::vector<int> stack;
        for (size_t i = 0; i < open.size(); ++i) {
            stack.assign(1, open[i]);
            while (!stack.empty()) {
                const int s = stack.back();
                stack.pop_back();
                S.sn_owner[s] = (int8_t)bin_of[i];
                kids(s, tmp);
                stack.insert(stack.end(), tmp.begin(), tmp.end());
            }
        }
    }
    for (int s = 0; s < ns; ++s)   // folded landmarks belong to their parent's owner
        if (folded[s]) S.sn_owner[s] = S.sn_owner[F.parent[s]];
    for (int s = 0; s < ns; ++s) {
        if (folded[s]) continue;
        if (S.sn_owner[s] < 0) ++S.n_top_fronts;
        else if (S.sn_owner[s] == rank) ++S.n_own_fronts;
    }
    // node ownership through the supernode holding the node's first dof
    std::vector<int32_t> sn_of_dof(P.n, -1);
    for (int s = 0; s < ns; ++s)
        for (int d = 0; d < F.k[s]; ++d) sn_of_dof[F.col0[s] + d] = s;
    S.node_owner.assign(nn, -2);
    for (int u = 0; u < nn; ++u) {
        if (u == pi.fixed) continue;
        const int32_t s = sn_of_dof[P.node_dof[u]];
        if (s < 0) { err = "shard: node without a supernode"; return BOS_ERR_INVALID; }
        S.node_owner[u] = S.sn_owner[s];
    }
    // J+H lanes: own poses, padded to a whole J+H block (chi^2 partials of own lanes and of top
    // lanes fall in different blocks), then the top poses and the fixed pose
    const int lpp = plan_lanes_per_pose(pi, world);   // as build_layout
    const int poses_per_block = kJhBlock / lpp;
    for (int p = 0; p < NP; ++p)
        if (S.node_owner[p] == rank) S.lane_poses.push_back(p);
    if (world > 1)
        while (S.lane_poses.size() % poses_per_block) S.lane_poses.push_back(-1);
    S.own_pose_lanes = (int)S.lane_poses.size();
    if (world > 1 && ((int64_t)S.own_pose_lanes * lpp) % kJhBlock) {   // ranks != 0 count whole own blocks
        err = "shard: own pose lanes not a whole number of J+H blocks";
        return BOS_ERR_INVALID;
    }
    for (int p = 0; p < NP; ++p)
        if (S.node_owner[p] < 0) S.lane_poses.push_back(p);
    for (int l = 0; l < NL; ++l)
        if (S.node_owner[NP + l] == rank) S.lane_lms.push_back(l);
    for (int l = 0; l < NL; ++l)
        if (S.node_owner[NP + l] == -1) S.lane_lms.push_back(l);
    // exchange 1: subtree roots that have a parent (a top front), grouped by owner
    S.root_ptr.assign(world + 1, 0);
    std::vector<std::vector<int32_t>> rroots(world);
    for (size_t i = 0; i < open.size(); ++i)
        if (F.parent[open[i]] >= 0) rroots[bin_of[i]].push_back(open[i]);
    int64_t ex1 = 0;
    for (int q = 0; q < world; ++q) {
        std::sort(rroots[q].begin(), rroots[q].end());
        int64_t c = 0;
        for (int s : rroots[q]) c += (int64_t)F.r[s] * (F.r[s] + 1) / 2 + F.r[s];
        ex1 = std::max(ex1, c);
        S.roots.insert(S.roots.end(), rroots[q].begin(), rroots[q].end());
        S.root_ptr[q + 1] = (int32_t)S.roots.size();
    }
    S.ex1_count = kExHeader + ex1;
    // boundary: subtree nodes read by a top lane (a top pose, a top landmark or the fixed pose):
    // odometry neighbours, observed landmarks, observing poses (with the Schur ordering a top
    // landmark is observed by top poses only; nested dissection of the whole graph can put a
    // landmark in a separator above its poses)
    std::vector<char> bnd(nn, 0);
    auto touch = [&](int u) {
        if (S.node_owner[u] >= 0) bnd[u] = 1;
    };
    for (int k = 0; k < pi.Mb; ++k) {
        if (S.node_owner[pi.b_pose[k]] < 0) touch(NP + pi.b_lm[k]);
        if (S.node_owner[NP + pi.b_lm[k]] < 0) touch(pi.b_pose[k]);
    }
    for (int k = 0; k < pi.Mo; ++k) {
        const int a = pi.o_src[k], b = pi.o_dst[k];
        if (S.node_owner[a] < 0) touch(b);
        if (S.node_owner[b] < 0) touch(a);
    }
    S.bnd_ptr.assign(world + 1, 0);
    int64_t ex2 = 0;
    for (int q = 0; q < world; ++q) {
        int64_t c = 0;
        for (int u = 0; u < nn; ++u)
            if (bnd[u] && S.node_owner[u] == q) {
                const int sz = u < NP ? 3 : 2;
                for (int d = 0; d < sz; ++d) S.bnd_dof.push_back(P.node_dof[u] + d);
                c += sz;
            }
        S.bnd_ptr[q + 1] = (int32_t)S.bnd_dof.size();
        ex2 = std::max(ex2, c);
    }
    S.ex2_count = kExHeader + ex2;
    // box-plus node set
    for (int u = 0; u < nn; ++u)
        if (S.node_owner[u] == rank || S.node_owner[u] == -1) S.upd_nodes.push_back(u);
    S.n_upd_local = (int)S.upd_nodes.size();
    for (int u = 0; u < nn; ++u)
        if (bnd[u] && S.node_owner[u] >= 0 && S.node_owner[u] != rank) S.upd_nodes.push_back(u);
    return BOS_OK;
}

void exchange1_segments(const Plan& P, std::vector<ExchangeSeg>& pack, std::vector<ExchangeSeg>& unpack) {
    const Shard& S = P.shard;
    const Multifrontal& F = P.mf;
    pack.clear();
    unpack.clear();
    for (int q = 0; q < S.world; ++q) {
        int64_t off = kExHeader;
        for (int i = S.root_ptr[q]; i < S.root_ptr[q + 1]; ++i) {
            const int s = S.roots[i], r = F.r[s];
            const int64_t nu = (int64_t)r * (r + 1) / 2;
            if (q == S.rank) {
                pack.push_back({F.U_off[s], off, nu, 0, 2});
                pack.push_back({F.u_off[s], off + nu, r, 1, 2});
            } else {
                unpack.push_back({(int64_t)q * S.ex1_count + off, F.U_off[s], nu, 3, 0});
                unpack.push_back({(int64_t)q * S.ex1_count + off + nu, F.u_off[s], r, 3, 1});
            }
            off += nu + r;
        }
    }
}

}  // namespace bos

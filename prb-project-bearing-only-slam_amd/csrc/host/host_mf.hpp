// The multifrontal algorithm of hip/multifrontal.hip on the host: the test hooks
// (bos_plan_mf_selftest, bos_plan_shard_selftest) and the CPU baseline of bench.py
// (host/cpu_baseline.cpp) run it; no GPU solve path does. Fronts are processed level by level with
// the plan's maps, the fronts of one level in parallel when a pool is given (they are independent:
// a front reads only its children's update matrices / u-vectors, which are finished by then).
#pragma once

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "plan.hpp"

namespace bos {

// Fixed set of worker threads running parallel_for(n, f): f(i) for i in [0, n), the caller's
// thread taking part; returns when every i is done.
class Pool {
  public:
    explicit Pool(int threads) {
        for (int t = 1; t < threads; ++t) th_.emplace_back([this] { work(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (std::thread& t : th_) t.join();
    }
    int size() const { return (int)th_.size() + 1; }
    template <typename F> void parallel_for(int64_t n, F&& f) {
        if (n <= 0) return;
        if (th_.empty() || n == 1) {
            for (int64_t i = 0; i < n; ++i) f(i);
            return;
        }
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = [&f](int64_t i) { f(i); };
            n_ = n;
            next_ = 0;
            busy_ = (int)th_.size();
            ++gen_;
        }
        cv_.notify_all();
        drain();
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [&] { return busy_ == 0; });
        job_ = nullptr;
    }

  private:
    void drain() {
        for (;;) {
            const int64_t i = next_.fetch_add(1);
            if (i >= n_) break;
            job_(i);
        }
    }
    void work() {
        int seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            drain();
            {
                std::lock_guard<std::mutex> g(m_);
                if (--busy_ == 0) done_.notify_all();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    std::function<void(int64_t)> job_;
    std::atomic<int64_t> next_{0};
    int64_t n_ = 0;
    int gen_ = 0, busy_ = 0;
    bool stop_ = false;
};

struct HostMf {
    const Plan& P;
    const Multifrontal& F;
    std::vector<double> hval, L, U, u, x;
    std::vector<std::vector<double>> fwv;
    Pool* pool = nullptr;

    HostMf(const Plan& plan, Pool* p = nullptr)
        : P(plan), F(plan.mf), hval(plan.blk.size, 0.0), L(plan.mf.L_size), U(plan.mf.U_size), u(plan.mf.u_size),
          x(plan.n, 0.0), fwv(plan.mf.nsuper), pool(p) {}
    // the block array holds what this plan's J+H writes: vals (stored entries of H_nf, one-rank
    // order) through its csr_src
    HostMf(const Plan& plan, const double* vals, const double* rhs) : HostMf(plan) {
        for (int64_t e = 0; e < P.nnzA(); ++e)
            if (P.blk.csr_src[e] >= 0) hval[P.blk.csr_src[e]] = vals[e];
        std::copy(rhs, rhs + P.n, x.begin());
    }

    template <typename Sel, typename Body> void each_level(bool top_down, Sel sel, Body body) {
        std::vector<int32_t> fr;
        for (int i = 0; i < F.nlevels; ++i) {
            const int lv = top_down ? F.nlevels - 1 - i : i;
            fr.clear();
            for (int q = F.level_ptr[lv]; q < F.level_ptr[lv + 1]; ++q)
                if (sel(F.level[q])) fr.push_back(F.level[q]);
            if (pool) pool->parallel_for((int64_t)fr.size(), [&](int64_t j) { body(fr[j]); });
            else
                for (int s : fr) body(s);
        }
    }

    // folded landmark children (Schur ordering): the fold records (one per observing pose: rows t,
    // t + 1, t + 2), as fold_children reads them; their u entries accumulate per parent in fwv
    void fold(int s, std::vector<double>& W, int m) {
        fwv[s].assign(m, 0.0);
        for (int ch = F.fold_cptr[s]; ch < F.fold_cptr[s + 1]; ++ch) {
            const int q0 = F.fold_chunk[ch], nq = F.fold_chunk[ch + 1] - q0;
            std::vector<double> l0(3 * nq), l1(3 * nq);
            std::vector<int> pos(3 * nq), cl(3 * nq);
            for (int q = 0; q < nq; ++q) {
                const int32_t* rec = F.fold_rec.data() + (size_t)kFoldRec * (q0 + q);
                auto v = [&](int32_t src) { return src >= 0 ? hval[src] : 0.0; };
                const int col0 = rec[5], t = rec[6] & 63, rc = (rec[6] >> 6) & 63;
                const double l00 = std::sqrt(std::max(v(rec[2]), 1e-300)), l10 = v(rec[3]) / l00;
                const double l11 = std::sqrt(std::max(v(rec[4]) - l10 * l10, 1e-300));
                const double y0 = x[col0] / l00, y1 = (x[col0 + 1] - l10 * y0) / l11;
                double* Lc = L.data() + rec[7];
                const int mc = 2 + rc;
                for (int g = 0; g < 3; ++g) {
                    const int i = 3 * q + g;
                    l0[i] = v(rec[0] >= 0 ? rec[0] + 2 * g : rec[0]) / l00;
                    l1[i] = (v(rec[0] >= 0 ? rec[0] + 2 * g + 1 : rec[0]) - l0[i] * l10) / l11;
                    Lc[2 + t + g] = l0[i];
                    Lc[mc + 2 + t + g] = l1[i];
                    pos[i] = ((rec[6] >> kFoldPosShift) & kFoldPosMask) + g;
                    cl[i] = rec[7];   // the landmark (its L offset)
                    fwv[s][pos[i]] -= l0[i] * y0 + l1[i] * y1;
                }
                if (t == 0) { Lc[0] = l00; Lc[1] = l10; Lc[mc + 1] = l11; }
            }
            for (int q = 0; q < nq; ++q) {   // the landmarks' forward results, after every row used them
                const int32_t* rec = F.fold_rec.data() + (size_t)kFoldRec * (q0 + q);
                if ((rec[6] & 63) == 0) {
                    const int col0 = rec[5];
                    const double* Lc = L.data() + rec[7];
                    const double y0 = x[col0] / Lc[0];
                    x[col0 + 1] = (x[col0 + 1] - Lc[1] * y0) / Lc[2 + ((rec[6] >> 6) & 63) + 1];
                    x[col0] = y0;
                }
            }
            for (int j = 0; j < 3 * nq; ++j)   // W W^T within each landmark
                for (int i = j; i < 3 * nq && cl[i] == cl[j]; ++i)
                    W[pos[i] + (size_t)pos[j] * m] -= l0[i] * l0[j] + l1[i] * l1[j];
        }
    }

    void factor_front(int s) {
        const int k = F.k[s], r = F.r[s], m = k + r;
        std::vector<double> W((size_t)m * m, 0.0);
        for (int a = F.amap_ptr[s]; a < F.amap_ptr[s + 1]; ++a) {
            int64_t d = F.amap_dst[a];
            if (m <= kMfWaveMaxM) {   // packed lower column-major -> (i, j)
                int64_t j = 0;
                while (d >= m - j) { d -= m - j; ++j; }
                d = (j + d) + j * m;
            }
            W[d] = hval[F.amap_src[a]];
        }
        fold(s, W, m);
        for (int ci = F.child_ptr[s] + F.fold_cnt[s]; ci < F.child_ptr[s + 1]; ++ci) {
            const int c = F.child[ci], rc2 = F.r[c];
            const int32_t* map = F.rmap.data() + F.rmap_off[c];
            for (int j = 0; j < rc2; ++j)
                for (int i = j; i < rc2; ++i) W[map[i] + (size_t)map[j] * m] += U[F.U_off[c] + mf_packed(i, j, rc2)];
        }
        for (int j = 0; j < k; ++j) {
            const double d = std::sqrt(std::max(W[j + (size_t)j * m], 1e-300));
            W[j + (size_t)j * m] = d;
            for (int i = j + 1; i < m; ++i) W[i + (size_t)j * m] /= d;
            for (int l = j + 1; l < m; ++l) {
                const double f = W[l + (size_t)j * m];
                double* col = W.data() + (size_t)l * m;
                const double* cj = W.data() + (size_t)j * m;
                for (int i = l; i < m; ++i) col[i] -= cj[i] * f;
            }
        }
        for (int j = 0; j < k; ++j)
            for (int i = 0; i < m; ++i) L[F.L_off[s] + i + (size_t)j * m] = W[i + (size_t)j * m];
        for (int j = 0; j < r; ++j)
            for (int i = j; i < r; ++i) U[F.U_off[s] + mf_packed(i, j, r)] = W[(k + i) + (size_t)(k + j) * m];
    }

    void forward_front(int s) {
        const int k = F.k[s], r = F.r[s], m = k + r;
        std::vector<double> w(m, 0.0);
        for (int i = 0; i < k; ++i) w[i] = x[F.col0[s] + i];
        for (size_t i = 0; i < fwv[s].size(); ++i) w[i] += fwv[s][i];
        for (int ci = F.child_ptr[s] + F.fold_cnt[s]; ci < F.child_ptr[s + 1]; ++ci) {
            const int c = F.child[ci];
            for (int t = 0; t < F.r[c]; ++t) w[F.rmap[F.rmap_off[c] + t]] += u[F.u_off[c] + t];
        }
        const double* Ls = L.data() + F.L_off[s];
        for (int j = 0; j < k; ++j) {
            w[j] /= Ls[j + (size_t)j * m];
            for (int i = j + 1; i < m; ++i) w[i] -= Ls[i + (size_t)j * m] * w[j];
        }
        for (int i = 0; i < k; ++i) x[F.col0[s] + i] = w[i];
        for (int t = 0; t < r; ++t) u[F.u_off[s] + t] = w[k + t];
    }

    void backward_front(int s) {
        const int k = F.k[s], m = k + F.r[s];
        const double* Ls = L.data() + F.L_off[s];
        const int32_t* fi = F.findex.data() + F.findex_off[s];
        for (int j = k - 1; j >= 0; --j) {
            double acc = x[F.col0[s] + j];
            for (int i = j + 1; i < m; ++i) acc -= Ls[i + (size_t)j * m] * x[fi[i]];
            x[F.col0[s] + j] = acc / Ls[j + (size_t)j * m];
        }
    }

    template <typename Pred> void factor(Pred sel) { each_level(false, sel, [&](int s) { factor_front(s); }); }
    template <typename Pred> void forward(Pred sel) { each_level(false, sel, [&](int s) { forward_front(s); }); }
    // top-down over the selected fronts, then their folded landmarks
    template <typename Pred> void backward(Pred sel) {
        each_level(true, sel, [&](int s) { backward_front(s); });
        std::vector<int32_t> folds;
        for (int s : F.fold_list)
            if (sel(F.parent[s])) folds.push_back(s);
        if (pool) pool->parallel_for((int64_t)folds.size(), [&](int64_t j) { backward_front(folds[j]); });
        else
            for (int s : folds) backward_front(s);
    }
};

}  // namespace bos

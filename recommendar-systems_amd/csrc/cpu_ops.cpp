// cpu_ops.cpp — the CPU kernels behind torch.ops.rsx.* ("each with CPU and
// HIP kernels"), so that the reference's CPU configuration (BASELINE C1: "CPU PyTorch
// reference path (plumbing, no GPU)") runs through the same operator boundary as the GPU
// one.  Host memory, plain pointers; the torch CPU dispatch key calls these (rsx/torch_ops.py),
// the CUDA key calls the HIP kernels — a CPU tensor never reaches a GPU kernel and a GPU
// tensor never reaches these.  Rows are split over std::thread workers (RSX_CPU_THREADS,
// default: the hardware threads, at most 64); every output row is written by one worker in a
// fixed order, so results do not depend on the thread count.
//
//   rsx_cpu_spmm               torch.sparse.mm(A, x)                (lightgcn.py:121-122)
//   rsx_cpu_propagate_mean     LightGCN.forward's layer mean       (lightgcn.py:117-130)
//   rsx_cpu_layergcn_forward   LayerGCN.forward                    (layergcn.py:127-140)
//   rsx_cpu_layergcn_backward  its autograd backward (cosine gates: RSX_EPI_LAYERGCN_BWD's formulas)
//   rsx_cpu_bpr                BPR + regulariser, loss and gradients (loss.py:33-61,
//                              lightgcn.py:132-156, layergcn.py:142-177, smore.py:366-378)
//   rsx_cpu_fullsort_topk      scores, train mask -1e10, top-k      (trainer.py:509-528)
//   rsx_cpu_adam               torch.optim.Adam's update            (trainer.py:93-99, 238)
//   rsx_cpu_gcn_step           one whole training batch of LightGCN / LayerGCN (the C1 path)
#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include <unistd.h>

#include "rsx.h"

namespace {

int n_threads() {
    static const int n = [] {
        const char* v = getenv("RSX_CPU_THREADS");
        int t = v && *v ? atoi(v) : (int)std::thread::hardware_concurrency();
        return std::max(1, std::min(t, 64));
    }();
    return n;
}

// A persistent pool: n_threads() - 1 workers parked on a condition variable, the caller
// runs piece 0.  One job at a time (calls are serialised by `busy`); a call from inside a
// job, or while another thread's job runs, runs inline.
class Pool {
  public:
    static Pool& get() {
        // never destroyed (no join at process exit); a forked child gets its own pool (the
        // parent's workers do not exist in it)
        static Pool* p = nullptr;
        static pid_t owner = 0;
        if (!p || owner != getpid()) {
            p = new Pool(n_threads());
            owner = getpid();
        }
        return *p;
    }
    // fn(i) for i in [0, t), t <= size()
    void run(int t, const std::function<void(int)>& fn) {
        bool expect = false;
        if (t <= 1 || !busy_.compare_exchange_strong(expect, true)) {
            for (int i = 0; i < t; ++i) fn(i);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &fn;
            pieces_ = t;
            left_.store(t - 1);
            ++gen_;
        }
        cv_.notify_all();
        fn(0);
        while (left_.load(std::memory_order_acquire) != 0) std::this_thread::yield();
        job_ = nullptr;
        busy_.store(false);
    }
    int size() const { return (int)ws_.size() + 1; }

  private:
    explicit Pool(int n) {
        for (int i = 1; i < n; ++i) ws_.emplace_back([this, i] { loop(i); });
        for (auto& w : ws_) w.detach();
    }
    void loop(int id) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* job;
            int pieces;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                job = job_;
                pieces = pieces_;
            }
            if (id < pieces) {
                (*job)(id);
                left_.fetch_sub(1, std::memory_order_acq_rel);
            }
        }
    }
    std::vector<std::thread> ws_;
    std::mutex mu_;
    std::condition_variable cv_;
    const std::function<void(int)>* job_ = nullptr;
    int pieces_ = 0;
    uint64_t gen_ = 0;
    std::atomic<int> left_{0};
    std::atomic<bool> busy_{false};
};

// fn(r0, r1) over [0, n) in contiguous pieces, one per worker (small n: inline)
template <class F>
void parallel_rows(int64_t n, int64_t min_rows, F fn) {
    Pool& pool = Pool::get();
    const int t = (int)std::min<int64_t>(pool.size(), std::max<int64_t>(1, n / std::max<int64_t>(min_rows, 1)));
    if (t <= 1) {
        fn((int64_t)0, n);
        return;
    }
    pool.run(t, [&](int i) { fn(n * i / t, n * (i + 1) / t); });
}

// y = A x, rows [r0, r1): the neighbours summed in column order (torch's CSR order)
void spmm_rows(const int64_t* rp, const int32_t* col, const float* val, const float* x, int d, float* y, int64_t r0,
               int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
        float* yr = y + r * d;
        std::fill(yr, yr + d, 0.f);
        for (int64_t j = rp[r]; j < rp[r + 1]; ++j) {
            const float a = val[j];
            const float* xr = x + (int64_t)col[j] * d;
            for (int c = 0; c < d; ++c) yr[c] += a * xr[c];
        }
    }
}

void spmm(const int64_t* rp, const int32_t* col, const float* val, int64_t n, const float* x, int d, float* y) {
    parallel_rows(n, 256, [&](int64_t a, int64_t b) { spmm_rows(rp, col, val, x, d, y, a, b); });
}

// <a, b> in eight interleaved partial sums (vector lanes), then a fixed tree: a fixed
// order, so a result does not depend on the thread that computes it
inline float dotf(const float* a, const float* b, int d) {
    if (d % 8) {
        float s = 0.f;
        for (int c = 0; c < d; ++c) s += a[c] * b[c];
        return s;
    }
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < d; c += 8)
        for (int k = 0; k < 8; ++k) acc[k] += a[c + k] * b[c + k];
    return ((acc[0] + acc[4]) + (acc[2] + acc[6])) + ((acc[1] + acc[5]) + (acc[3] + acc[7]));
}

// y = A_r x: row r's neighbours in column order
inline void spmm_row(const int64_t* rp, const int32_t* col, const float* val, const float* x, int d, int64_t r,
                     float* __restrict__ yr) {
    std::fill(yr, yr + d, 0.f);
    for (int64_t j = rp[r]; j < rp[r + 1]; ++j) {
        const float a = val[j];
        const float* __restrict__ xr = x + (int64_t)col[j] * d;
        for (int c = 0; c < d; ++c) yr[c] += a * xr[c];
    }
}

void fill_par(float* y, size_t n, float v) {
    parallel_rows((int64_t)n, 1 << 16, [&](int64_t a, int64_t b) { std::fill(y + a, y + b, v); });
}

// F.cosine_similarity(z, e) with eps 1e-8 and its row norms
struct Cos {
    float c, rz, re;
};
inline Cos cosine(const float* z, const float* e, int d) {
    const float rz = std::sqrt(dotf(z, z, d)), re = std::sqrt(dotf(e, e, d));
    return {dotf(z, e, d) / (std::max(rz, 1e-8f) * std::max(re, 1e-8f)), rz, re};
}

// the gate's backward for one row (dE: the gradient reaching E = c z):
//   dz = c dE + <dE,z> (e/(nz ne) - c z/|z|^2),  dego += <dE,z> (z/(nz ne) - c e/|e|^2)
inline void gate_bwd_row(const float* de, const float* z, const float* e, float c, float rz, float re, int d,
                         float* __restrict__ dz, float* __restrict__ dego) {
    const float nz = std::max(rz, 1e-8f), ne = std::max(re, 1e-8f);
    const float gz = dotf(de, z, d);
    const float inv = 1.f / (nz * ne);
    const float kz = rz > 1e-8f ? c / (nz * nz) : 0.f;
    const float ke = re > 1e-8f ? c / (ne * ne) : 0.f;
    for (int j = 0; j < d; ++j) {
        dz[j] = c * de[j] + gz * inv * e[j] - gz * kz * z[j];
        dego[j] += gz * inv * z[j] - gz * ke * e[j];
    }
}

}  // namespace

extern "C" {

int rsx_cpu_spmm(const int64_t* rowptr, const int32_t* col, const float* val, int64_t n_rows, const float* x,
                 int32_t d, float* y) {
    if (!rowptr || n_rows < 0 || d <= 0 || (n_rows > 0 && (!y || (rowptr[n_rows] > 0 && (!col || !val || !x)))))
        return RSX_ERR_ARG;
    spmm(rowptr, col, val, n_rows, x, d, y);
    return RSX_OK;
}

int rsx_cpu_propagate_mean(const int64_t* rowptr, const int32_t* col, const float* val, int64_t n, const float* x,
                           int32_t d, int32_t n_layers, float* out) {
    if (!rowptr || !x || !out || n < 0 || d <= 0 || n_layers < 0) return RSX_ERR_ARG;
    const size_t nd = (size_t)n * d;
    std::vector<float> a(nd), b(nd);
    std::copy(x, x + nd, out);  // the running sum E^0 + E^1 + ... (torch.stack + mean: sum, then / (K+1))
    const float* cur = x;
    for (int k = 1; k <= n_layers; ++k) {
        float* y = (k & 1) ? a.data() : b.data();
        spmm(rowptr, col, val, n, cur, d, y);
        parallel_rows(n, 1024, [&](int64_t r0, int64_t r1) {
            for (size_t i = (size_t)r0 * d; i < (size_t)r1 * d; ++i) out[i] += y[i];
        });
        cur = y;
    }
    const float inv = (float)(n_layers + 1);
    parallel_rows(n, 1024, [&](int64_t r0, int64_t r1) {
        for (size_t i = (size_t)r0 * d; i < (size_t)r1 * d; ++i) out[i] /= inv;
    });
    return RSX_OK;
}

// E^k = c_k * z_k, z_k = A E^{k-1}, c_k = cos(z_k, E^0) (F.cosine_similarity, eps 1e-8:
// <z/max(|z|,eps), e/max(|e|,eps)>); out = sum_{k=1..K} E^k.  zs [K][n][d] / cs [K][n]
// (optional) keep every z_k and c_k for the backward.
int rsx_cpu_layergcn_forward(const int64_t* rowptr, const int32_t* col, const float* val, int64_t n, const float* x,
                             int32_t d, int32_t n_layers, float* out, float* zs, float* cs) {
    if (!rowptr || !x || !out || n < 0 || d <= 0 || n_layers < 1) return RSX_ERR_ARG;
    const size_t nd = (size_t)n * d;
    std::vector<float> z(nd), e(nd);
    std::fill(out, out + nd, 0.f);
    const float* cur = x;
    for (int k = 1; k <= n_layers; ++k) {
        float* zk = zs ? zs + (size_t)(k - 1) * nd : z.data();
        spmm(rowptr, col, val, n, cur, d, zk);
        parallel_rows(n, 256, [&](int64_t r0, int64_t r1) {
            for (int64_t r = r0; r < r1; ++r) {
                const float* zr = zk + r * d;
                const float* er = x + r * d;
                const float nz = std::max(std::sqrt(dotf(zr, zr, d)), 1e-8f);
                const float ne = std::max(std::sqrt(dotf(er, er, d)), 1e-8f);
                const float c = dotf(zr, er, d) / (nz * ne);
                if (cs) cs[(size_t)(k - 1) * n + r] = c;
                for (int j = 0; j < d; ++j) {
                    const float v = c * zr[j];
                    e[r * d + j] = v;
                    out[r * d + j] += v;
                }
            }
        });
        cur = e.data();
    }
    return RSX_OK;
}

// dx = d/dx <G, LayerGCN.forward(x)> with the saved z_k, c_k (rsx_cpu_layergcn_forward).
// The gate backward per row (dE the gradient reaching E^k = G + A dZ^{k+1}):
//   dZ^k  = c dE + <dE,z> (e/(nz ne) - c z/|z|^2)
//   d ego += <dE,z> (z/(nz ne) - c e/|e|^2)        (norms eps-clamped; a clamped norm is a constant)
// and dx = A dZ^1 + sum_k d ego_k (A symmetric: the adjacency is its own transpose).
int rsx_cpu_layergcn_backward(const int64_t* rowptr, const int32_t* col, const float* val, int64_t n,
                              const float* x, int32_t d, int32_t n_layers, const float* G, const float* zs,
                              const float* cs, float* dx) {
    if (!rowptr || !x || !G || !zs || !cs || !dx || n < 0 || d <= 0 || n_layers < 1) return RSX_ERR_ARG;
    const size_t nd = (size_t)n * d;
    std::vector<float> dz(nd), ad(nd), dego(nd, 0.f);
    for (int k = n_layers; k >= 1; --k) {
        const float* zk = zs + (size_t)(k - 1) * nd;
        const float* ck = cs + (size_t)(k - 1) * n;
        if (k < n_layers) spmm(rowptr, col, val, n, dz.data(), d, ad.data());  // A dZ^{k+1}
        const bool first = k == n_layers;
        parallel_rows(n, 256, [&](int64_t r0, int64_t r1) {
            std::vector<float> de(d);
            for (int64_t r = r0; r < r1; ++r) {
                const float* z = zk + r * d;
                const float* e = x + r * d;
                for (int j = 0; j < d; ++j) de[j] = (first ? 0.f : ad[r * d + j]) + G[r * d + j];
                const float c = ck[r];
                const float rz = std::sqrt(dotf(z, z, d)), re = std::sqrt(dotf(e, e, d));
                const float nz = std::max(rz, 1e-8f), ne = std::max(re, 1e-8f);
                const float gz = dotf(de.data(), z, d);
                const float inv = 1.f / (nz * ne);
                const float kz = rz > 1e-8f ? c / (nz * nz) : 0.f;
                const float ke = re > 1e-8f ? c / (ne * ne) : 0.f;
                for (int j = 0; j < d; ++j) {
                    dz[r * d + j] = c * de[j] + gz * inv * e[j] - gz * kz * z[j];
                    dego[r * d + j] += gz * inv * z[j] - gz * ke * e[j];
                }
            }
        });
    }
    spmm(rowptr, col, val, n, dz.data(), d, dx);  // A dZ^1
    parallel_rows(n, 1024, [&](int64_t r0, int64_t r1) {
        for (size_t i = (size_t)r0 * d; i < (size_t)r1 * d; ++i) dx[i] += dego[i];
    });
    return RSX_OK;
}

// The fused BPR loss of include/rsx.h rsx_bpr (same variants, same formulas; gradients are
// ADDED into g_final / g_ego, rows of the batch only), computed in the triplet order.
int rsx_cpu_bpr(int32_t variant, const float* fin, const float* ego, int64_t n_users, int64_t n_items, int32_t d,
                const int64_t* trip, int64_t B, float reg, float batch_cfg, float* g_fin, float* g_ego,
                float* loss_out) {
    if (!fin || !trip || !loss_out || B <= 0 || d <= 0 || variant < 0 || variant > 2) return RSX_ERR_ARG;
    if (variant != RSX_BPR_SMORE && !ego) return RSX_ERR_ARG;
    const int64_t N = n_users + n_items;
    for (int64_t b = 0; b < B; ++b)
        if (trip[b] < 0 || trip[b] >= n_users || trip[B + b] < 0 || trip[B + b] >= n_items || trip[2 * B + b] < 0 ||
            trip[2 * B + b] >= n_items)
            return RSX_ERR_ARG;
    (void)N;
    std::vector<float> coef(B);
    double t_loss = 0.0, q[3] = {0.0, 0.0, 0.0};
    const float* regsrc = variant == RSX_BPR_SMORE ? fin : ego;
    for (int64_t b = 0; b < B; ++b) {
        const int64_t rows[3] = {trip[b], n_users + trip[B + b], n_users + trip[2 * B + b]};
        const float* u = fin + rows[0] * d;
        const float sp = dotf(u, fin + rows[1] * d, d), sn = dotf(u, fin + rows[2] * d, d);
        const float delta = sp - sn;
        float term, c;
        if (variant == RSX_BPR_LIGHTGCN) {  // -log(1e-10 + sigmoid(delta)), mean over the batch
            const float sg = 1.f / (1.f + std::exp(-delta));
            term = -std::log(1e-10f + sg);
            c = -(sg * (1.f - sg)) / (1e-10f + sg) / (float)B;
        } else {  // -logsigmoid(delta) (stable): summed (LayerGCN) or mean (SMORE)
            term = delta >= 0.f ? std::log1p(std::exp(-delta)) : -delta + std::log1p(std::exp(delta));
            c = -1.f / (1.f + std::exp(delta));
            if (variant == RSX_BPR_SMORE) c /= (float)B;
        }
        coef[b] = c;
        t_loss += term;
        for (int k = 0; k < 3; ++k) {
            const float* e = regsrc + rows[k] * d;
            q[k] += (double)dotf(e, e, d);
        }
    }
    double loss;
    float ks[3];
    if (variant == RSX_BPR_LIGHTGCN) {
        double nrm[3];
        for (int k = 0; k < 3; ++k) nrm[k] = std::sqrt(q[k]);
        loss = t_loss / (double)B + (double)reg * (nrm[0] + nrm[1] + nrm[2]) / (double)B;
        for (int k = 0; k < 3; ++k) ks[k] = nrm[k] > 0 ? (float)((double)reg / ((double)B * nrm[k])) : 0.f;
    } else if (variant == RSX_BPR_LAYERGCN) {
        loss = t_loss + (double)reg * 0.5 * (q[0] + q[1] + q[2]);
        ks[0] = ks[1] = ks[2] = reg;
    } else {
        loss = t_loss / (double)B + (double)reg * 0.5 * (q[0] + q[1] + q[2]) / (double)batch_cfg;
        ks[0] = ks[1] = ks[2] = (float)((double)reg / (double)batch_cfg);
    }
    loss_out[0] = (float)loss;
    for (int64_t b = 0; b < B; ++b) {
        const int64_t rows[3] = {trip[b], n_users + trip[B + b], n_users + trip[2 * B + b]};
        const float* u = fin + rows[0] * d;
        const float* p = fin + rows[1] * d;
        const float* ng = fin + rows[2] * d;
        const float c = coef[b];
        if (g_fin) {
            for (int j = 0; j < d; ++j) {
                g_fin[rows[0] * d + j] += c * (p[j] - ng[j]);
                g_fin[rows[1] * d + j] += c * u[j];
                g_fin[rows[2] * d + j] -= c * u[j];
            }
        }
        float* gr = variant == RSX_BPR_SMORE ? g_fin : g_ego;
        if (gr) {
            for (int k = 0; k < 3; ++k) {
                const float* e = regsrc + rows[k] * d;
                for (int j = 0; j < d; ++j) gr[rows[k] * d + j] += ks[k] * e[j];
            }
        }
    }
    return RSX_OK;
}

// scores = user_emb[users[b]] . item_emb^T (dot in column order), items of the user's train
// mask row = -1e10, the top k in (score desc, item asc) order
int rsx_cpu_fullsort_topk(const float* user_emb, const int64_t* users, int64_t n_batch, const float* item_emb,
                          int64_t n_items, int32_t d, const int64_t* mask_rowptr, const int32_t* mask_col, int32_t k,
                          float* scores_out, int64_t* idx_out) {
    if (!user_emb || !item_emb || !scores_out || !idx_out || n_batch < 0 || n_items <= 0 || d <= 0 || k < 1 ||
        k > n_items || (mask_rowptr && !mask_col))
        return RSX_ERR_ARG;
    parallel_rows(n_batch, 16, [&](int64_t b0, int64_t b1) {
        std::vector<float> s(n_items);
        std::vector<int64_t> ord(n_items);
        for (int64_t b = b0; b < b1; ++b) {
            const int64_t u = users ? users[b] : b;
            const float* ur = user_emb + u * d;
            for (int64_t i = 0; i < n_items; ++i) s[i] = dotf(ur, item_emb + i * d, d);
            if (mask_rowptr)
                for (int64_t j = mask_rowptr[u]; j < mask_rowptr[u + 1]; ++j) s[mask_col[j]] = -1e10f;
            for (int64_t i = 0; i < n_items; ++i) ord[i] = i;
            auto better = [&](int64_t x, int64_t y) { return s[x] > s[y] || (s[x] == s[y] && x < y); };
            std::partial_sort(ord.begin(), ord.begin() + k, ord.end(), better);
            for (int j = 0; j < k; ++j) {
                scores_out[b * k + j] = s[ord[j]];
                idx_out[b * k + j] = ord[j];
            }
        }
    });
    return RSX_OK;
}

// torch.optim.Adam (single tensor, amsgrad off): g += wd p; m = lerp(m, g, 1 - b1);
// v = b2 v + (1 - b2) g^2; p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps); the bias
// corrections in double, as the GPU ADAM epilogue.  `step` is the already incremented count.
int rsx_cpu_adam(float* p, const float* g, float* m, float* v, int64_t n, int64_t step, float lr, float beta1,
                 float beta2, float eps, float weight_decay) {
    if (!p || !g || !m || !v || n < 0 || step < 1) return RSX_ERR_ARG;
    const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
    const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
    const float step_size = (float)((double)lr / bc1);
    const float bc2_sqrt = (float)std::sqrt(bc2);
    parallel_rows(n, 1 << 16, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            float gi = g[i];
            if (weight_decay != 0.f) gi += weight_decay * p[i];
            m[i] += (1.f - beta1) * (gi - m[i]);
            v[i] = v[i] * beta2 + (1.f - beta2) * gi * gi;
            const float denom = std::sqrt(v[i]) / bc2_sqrt + eps;
            p[i] -= step_size * (m[i] / denom);
        }
    });
    return RSX_OK;
}

// ---------------------------------------------------------------------------
// One training batch of the CPU configuration in one call (BASELINE C1): propagation
// (the last layer on the batch rows only: the loss reads no other row), the BPR loss and
// its gradient on compact batch rows, the backward propagation, Adam.  The same
// arithmetic as the torch.ops.rsx sequence (propagate + bpr_loss + autograd + adam_) but
// without its recomputed forward, full-table gradient fills and per-op dispatch.
//   LightGCN (lightgcn.py:117-156): f = mean_k A^k p; loss = mean -log(1e-10 + sigmoid)
//     + reg (|U0| + |P0| + |N0|) / B on the ego rows; dp = (1/(K+1)) H_K + R with
//     H_0 = G, H_k = G + A H_{k-1} (A symmetric).
//   LayerGCN (layergcn.py:127-177): E^k = cos(A E^{k-1}, E^0) A E^{k-1}, out = sum_{k>=1} E^k;
//     loss = sum softplus(-delta) + reg/2 sum |ego rows|^2; the gate backward of
//     rsx_cpu_layergcn_backward layer by layer.
// Workspace: rsx_cpu_gcn_step_ws_floats(kind, n, d, K, B) floats.
// ---------------------------------------------------------------------------
size_t rsx_cpu_gcn_step_ws_floats(int32_t kind, int64_t n, int32_t d, int32_t n_layers, int64_t batch) {
    const size_t nd = (size_t)n * d, bd = (size_t)3 * batch * d;
    const size_t K = (size_t)std::max(n_layers, 1);
    if (kind == 0) return 3 * nd + 3 * bd + 3 * (size_t)batch;
    return (K - 1) * (nd + (size_t)n) + 4 * nd + 5 * bd + 3 * (size_t)batch * 3;
}

int rsx_cpu_gcn_step(int32_t kind, const int64_t* rowptr, const int32_t* col, const float* val, int64_t n_users,
                     int64_t n_items, int32_t d, int32_t n_layers, const int64_t* trip, int64_t B, float reg, float* p,
                     float* m, float* v, int64_t step, float lr, float beta1, float beta2, float eps,
                     float weight_decay, float* ws, size_t ws_floats, float* loss_out) {
    const int64_t n = n_users + n_items;
    if ((kind != 0 && kind != 1) || !rowptr || !col || !val || !trip || !p || !m || !v || !ws || !loss_out ||
        n <= 0 || d <= 0 || n_layers < 1 || B <= 0 || step < 1)
        return RSX_ERR_ARG;
    if (ws_floats < rsx_cpu_gcn_step_ws_floats(kind, n, d, n_layers, B)) return RSX_ERR_WORKSPACE;
    for (int64_t b = 0; b < B; ++b)
        if (trip[b] < 0 || trip[b] >= n_users || trip[B + b] < 0 || trip[B + b] >= n_items || trip[2 * B + b] < 0 ||
            trip[2 * B + b] >= n_items)
            return RSX_ERR_ARG;
    const int K = n_layers;
    const int64_t R = 3 * B;  // compact batch rows [users; positives; negatives]
    const size_t nd = (size_t)n * d;
    std::vector<int64_t> rows(R);
    for (int64_t b = 0; b < B; ++b) {
        rows[b] = trip[b];
        rows[B + b] = n_users + trip[B + b];
        rows[2 * B + b] = n_users + trip[2 * B + b];
    }
    auto row_of = [&](int64_t j) { return rows[j]; };
    float* w = ws;
    auto take = [&](size_t k) {
        float* q = w;
        w += k;
        return q;
    };
    // ---- BPR on compact rows fc [R, d] -> loss, coefficients, compact gradients gc
    auto bpr = [&](const float* fc, float* gc, int variant, float* ks_out) {
        double t_loss = 0.0, q[3] = {0.0, 0.0, 0.0};
        std::vector<float> coef(B);
        for (int64_t b = 0; b < B; ++b) {
            const float* u = fc + b * d;
            const float sp = dotf(u, fc + (B + b) * d, d), sn = dotf(u, fc + (2 * B + b) * d, d);
            const float delta = sp - sn;
            float term, c;
            if (variant == RSX_BPR_LIGHTGCN) {
                const float sg = 1.f / (1.f + std::exp(-delta));
                term = -std::log(1e-10f + sg);
                c = -(sg * (1.f - sg)) / (1e-10f + sg) / (float)B;
            } else {
                term = delta >= 0.f ? std::log1p(std::exp(-delta)) : -delta + std::log1p(std::exp(delta));
                c = -1.f / (1.f + std::exp(delta));
            }
            coef[b] = c;
            t_loss += term;
            for (int k = 0; k < 3; ++k) {
                const float* e = p + row_of(k * B + b) * d;
                q[k] += (double)dotf(e, e, d);
            }
        }
        double loss;
        if (variant == RSX_BPR_LIGHTGCN) {
            double nrm[3];
            for (int k = 0; k < 3; ++k) nrm[k] = std::sqrt(q[k]);
            loss = t_loss / (double)B + (double)reg * (nrm[0] + nrm[1] + nrm[2]) / (double)B;
            for (int k = 0; k < 3; ++k) ks_out[k] = nrm[k] > 0 ? (float)((double)reg / ((double)B * nrm[k])) : 0.f;
        } else {
            loss = t_loss + (double)reg * 0.5 * (q[0] + q[1] + q[2]);
            ks_out[0] = ks_out[1] = ks_out[2] = reg;
        }
        loss_out[0] = (float)loss;
        parallel_rows(B, 256, [&](int64_t b0, int64_t b1) {
            for (int64_t b = b0; b < b1; ++b) {
                const float* u = fc + b * d;
                const float* pp = fc + (B + b) * d;
                const float* ng = fc + (2 * B + b) * d;
                const float c = coef[b];
                for (int j = 0; j < d; ++j) {
                    gc[b * d + j] = c * (pp[j] - ng[j]);
                    gc[(B + b) * d + j] = c * u[j];
                    gc[(2 * B + b) * d + j] = -c * u[j];
                }
            }
        });
    };
    auto adam = [&](const float* g) {
        rsx_cpu_adam(p, g, m, v, (int64_t)nd, step, lr, beta1, beta2, eps, weight_decay);
    };
    float ks[3];
    if (kind == 0) {  // ---------------------------------------------------- LightGCN
        float* a = take(nd);
        float* b2 = take(nd);
        float* G = take(nd);
        float* fc = take((size_t)R * d);
        float* gc = take((size_t)R * d);
        float* sc = take((size_t)R * d);
        // forward: the running sum on the batch rows, layer K on those rows only
        parallel_rows(R, 64, [&](int64_t j0, int64_t j1) {
            for (int64_t j = j0; j < j1; ++j) std::copy(p + row_of(j) * d, p + row_of(j) * d + d, sc + j * d);
        });
        const float* cur = p;
        for (int k = 1; k <= K; ++k) {
            if (k < K) {
                float* y = (k & 1) ? a : b2;
                spmm(rowptr, col, val, n, cur, d, y);
                parallel_rows(R, 64, [&](int64_t j0, int64_t j1) {
                    for (int64_t j = j0; j < j1; ++j)
                        for (int c = 0; c < d; ++c) sc[j * d + c] += y[row_of(j) * d + c];
                });
                cur = y;
            } else {
                parallel_rows(R, 64, [&](int64_t j0, int64_t j1) {
                    std::vector<float> t(d);
                    for (int64_t j = j0; j < j1; ++j) {
                        spmm_row(rowptr, col, val, cur, d, row_of(j), t.data());
                        for (int c = 0; c < d; ++c) fc[j * d + c] = (sc[j * d + c] + t[c]) * (1.f / (float)(K + 1));
                    }
                });
            }
        }
        bpr(fc, gc, RSX_BPR_LIGHTGCN, ks);
        fill_par(G, nd, 0.f);
        for (int64_t j = 0; j < R; ++j)  // G: the batch rows' gradients, added in occurrence order
            for (int c = 0; c < d; ++c) G[row_of(j) * d + c] += gc[j * d + c];
        // Horner: H_k = G + A H_{k-1}
        const float* h = G;
        float* out = nullptr;
        for (int k = 1; k <= K; ++k) {
            float* y = (k & 1) ? a : b2;
            parallel_rows(n, 256, [&](int64_t r0, int64_t r1) {
                for (int64_t r = r0; r < r1; ++r) {
                    spmm_row(rowptr, col, val, h, d, r, y + r * d);
                    for (int c = 0; c < d; ++c) y[r * d + c] += G[r * d + c];
                }
            });
            h = y;
            out = y;
        }
        const float inv = 1.f / (float)(K + 1);
        parallel_rows(n, 1024, [&](int64_t r0, int64_t r1) {
            for (size_t i = (size_t)r0 * d; i < (size_t)r1 * d; ++i) out[i] *= inv;
        });
        for (int64_t j = 0; j < R; ++j) {  // the regulariser on the ego rows
            const float kk = ks[j / B];
            const float* e = p + row_of(j) * d;
            for (int c = 0; c < d; ++c) out[row_of(j) * d + c] += kk * e[c];
        }
        adam(out);
        return RSX_OK;
    }
    // ----------------------------------------------------------------------- LayerGCN
    float* zs = take((size_t)(K - 1) * nd);  // z_k = A E^{k-1}, k < K (full)
    float* cs = take((size_t)(K - 1) * n);   // c_k, k < K
    float* E = take(nd);                     // E^{K-1} (the last full layer)
    float* dA = take(nd);
    float* dB = take(nd);
    float* dego = take(nd);
    float* zc = take((size_t)R * d);  // z_K on the batch rows
    float* oc = take((size_t)R * d);  // out on the batch rows
    float* gc = take((size_t)R * d);
    float* dzc = take((size_t)R * d);
    float* degc = take((size_t)R * d);
    float* cK = take((size_t)3 * R);  // c, |z|, |e| of layer K on the batch rows
    std::fill(oc, oc + (size_t)R * d, 0.f);
    const float* cur = p;
    for (int k = 1; k < K; ++k) {  // full layers, E^k kept in E (the next layer's input)
        float* z = zs + (size_t)(k - 1) * nd;
        float* ck = cs + (size_t)(k - 1) * n;
        spmm(rowptr, col, val, n, cur, d, z);
        parallel_rows(n, 256, [&](int64_t r0, int64_t r1) {
            for (int64_t r = r0; r < r1; ++r) {
                const Cos g = cosine(z + r * d, p + r * d, d);
                ck[r] = g.c;
                for (int c = 0; c < d; ++c) E[r * d + c] = g.c * z[r * d + c];
            }
        });
        parallel_rows(R, 64, [&](int64_t j0, int64_t j1) {
            for (int64_t j = j0; j < j1; ++j)
                for (int c = 0; c < d; ++c) oc[j * d + c] += E[row_of(j) * d + c];
        });
        cur = E;
    }
    parallel_rows(R, 64, [&](int64_t j0, int64_t j1) {  // layer K on the batch rows
        for (int64_t j = j0; j < j1; ++j) {
            float* z = zc + j * d;
            spmm_row(rowptr, col, val, cur, d, row_of(j), z);
            const Cos g = cosine(z, p + row_of(j) * d, d);
            cK[3 * j] = g.c;
            cK[3 * j + 1] = g.rz;
            cK[3 * j + 2] = g.re;
            for (int c = 0; c < d; ++c) oc[j * d + c] += g.c * z[c];
        }
    });
    bpr(oc, gc, RSX_BPR_LAYERGCN, ks);
    // layer K's gate backward per occurrence (dE^K = G), scattered in occurrence order
    parallel_rows(R, 64, [&](int64_t j0, int64_t j1) {
        for (int64_t j = j0; j < j1; ++j) {
            std::fill(degc + j * d, degc + j * d + d, 0.f);
            gate_bwd_row(gc + j * d, zc + j * d, p + row_of(j) * d, cK[3 * j], cK[3 * j + 1], cK[3 * j + 2], d,
                         dzc + j * d, degc + j * d);
        }
    });
    fill_par(dego, nd, 0.f);
    fill_par(dA, nd, 0.f);
    for (int64_t j = 0; j < R; ++j)
        for (int c = 0; c < d; ++c) {
            dA[row_of(j) * d + c] += dzc[j * d + c];
            dego[row_of(j) * d + c] += degc[j * d + c];
        }
    float* dz = dA;  // dZ^{k+1}
    float* de = dB;
    for (int k = K - 1; k >= 1; --k) {  // dE^k = A dZ^{k+1} + G, then the full gate backward
        spmm(rowptr, col, val, n, dz, d, de);
        for (int64_t j = 0; j < R; ++j)
            for (int c = 0; c < d; ++c) de[row_of(j) * d + c] += gc[j * d + c];
        const float* z = zs + (size_t)(k - 1) * nd;
        const float* ck = cs + (size_t)(k - 1) * n;
        parallel_rows(n, 256, [&](int64_t r0, int64_t r1) {
            std::vector<float> t(d);
            for (int64_t r = r0; r < r1; ++r) {
                const float* zr = z + r * d;
                const float* er = p + r * d;
                const float rz = std::sqrt(dotf(zr, zr, d)), re = std::sqrt(dotf(er, er, d));
                std::copy(de + r * d, de + r * d + d, t.data());
                gate_bwd_row(t.data(), zr, er, ck[r], rz, re, d, de + r * d, dego + r * d);
            }
        });
        std::swap(dz, de);
    }
    spmm(rowptr, col, val, n, dz, d, de);  // dE^0 = A dZ^1 + the cosine terms + the regulariser
    parallel_rows(n, 1024, [&](int64_t r0, int64_t r1) {
        for (size_t i = (size_t)r0 * d; i < (size_t)r1 * d; ++i) de[i] += dego[i];
    });
    for (int64_t j = 0; j < R; ++j) {
        const float* e = p + row_of(j) * d;
        for (int c = 0; c < d; ++c) de[row_of(j) * d + c] += reg * e[c];
    }
    adam(de);
    return RSX_OK;
}

}  // extern "C"

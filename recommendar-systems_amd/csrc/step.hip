// step.hip — device triplet sampler and the fused LightGCN step / forward (gfx950).
//
// Sampler: replaces TrainDataLoader's per-epoch shuffle + Python rejection
// sampling of negatives (reference src/utils/dataloader.py:226-275,307-309,
// src/utils/dataset.py:98-101) in throughput mode.  The epoch order is a keyed
// Feistel bijection of [0, n_inter) (cycle walking), so a batch needs no stored
// permutation; negatives are drawn uniformly from the training-item list and
// redrawn while they hit the user's sorted training history.
//
// LightGCN step: the reference batch (src/models/lightgcn.py:117-156, autograd
// backward, src/common/trainer.py:238 Adam) as 2K+2 launches (+1 per layer when
// the graph has hub rows split over several work items):
//   forward   E^k = A E^{k-1}, running sum S, last layer writes F = S/(K+1) and
//             zeroes the gradient scratch G, R;
//   loss      BPR fwd+bwd: G += dL/dF (batch rows), R += d reg / d E^0;
//   backward  H_k = A H_{k-1} (H_0 = G), S = sum H; the last layer
//             applies Adam to E^0 with g = S/(K+1) + R in its epilogue.
// With batch-row tags (rsx_lgcn_step.row_tag, K = 2..4) the step stores the
// layers instead of a running sum, computes the last forward layer on the batch
// rows only and runs the backward as the reference autograd's recursion on
// G' = G/(K+1) (lgcn_step_stored_layers below): about 110 MB less traffic per
// sports-shaped step.
#include "rsx_common.hpp"

namespace rsx {

int spmm_dispatch(const rsx_csr& a, const float* x, int d, const rsx_epilogue& e, float* slab, hipStream_t s);
int spmm_dispatch_tagging(const rsx_csr& a, const float* x, int d, const rsx_epilogue& e, float* slab,
                          hipStream_t s, const TagJob& tj);
int rowwise_dispatch(int64_t n, int d, const rsx_epilogue& e, hipStream_t s);
int bpr_call(int32_t variant, const float* fin, const float* ego, int64_t n_users, int64_t n_items, int32_t d,
             const int64_t* trip, int64_t batch, float reg, float batch_cfg, float* g_fin, float* g_ego,
             float* loss_out, double* loss_acc, void* ws, size_t ws_bytes, hipStream_t s, float g_div = 1.f,
             int32_t* halt = nullptr, int32_t tag = 0);

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t feistel(uint64_t x, int hb, uint64_t key) {
    const uint64_t mask = (1ull << hb) - 1;
    uint64_t L = x >> hb, R = x & mask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint64_t F = mix64(R ^ (key + (uint64_t)r * 0x632be59bd9b4e019ull)) & mask;
        const uint64_t nl = R;
        R = L ^ F;
        L = nl;
    }
    return (L << hb) | R;
}

__device__ __forceinline__ uint64_t permute(uint64_t i, uint64_t n, int hb, uint64_t key) {
    uint64_t x = i;
    do {
        x = feistel(x, hb, key);
    } while (x >= n);
    return x;
}

__device__ __forceinline__ bool in_sorted(const int32_t* a, int64_t lo, int64_t hi, int32_t v) {
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int32_t x = a[mid];
        if (x == v) return true;
        if (x < v) lo = mid + 1; else hi = mid;
    }
    return false;
}

// Triplet for epoch position pos = start + t.  Output layout: batch-major, batch
// j = t / bm holding [3][Bj] contiguous at out + 3*bm*j (Bj = min(bm, count - j*bm));
// with bm >= count this is the plain [3][count] layout.  With n_slices > 0 the batches
// are the n_slices balanced slices [floor(j count / S), floor((j+1) count / S)) instead
// (sizes differ by at most one), slice j stored [3][Bj] at out + 3*floor(j count / S).
__global__ __launch_bounds__(256) void sample_kernel(rsx_sampler_args s, int hb, int64_t count, int64_t bm,
                                                     int64_t* out, int64_t n_slices) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= count) return;
    const uint64_t key = mix64(s.seed ^ mix64((uint64_t)s.epoch + 0x1234567ull));
    const int64_t pos = s.start + t;
    const int64_t e = (int64_t)permute((uint64_t)pos, (uint64_t)s.n_inter, hb, key);
    const int32_t u = s.inter_u[e];
    const int32_t p = s.inter_i[e];
    const int64_t lo = s.hist_rowptr[u], hi = s.hist_rowptr[u + 1];
    uint64_t st = mix64(key ^ mix64((uint64_t)pos * 0x9e3779b97f4a7c15ull + 17));
    int32_t n = 0;
    for (int attempt = 0; attempt < 1024; ++attempt) {
        st = mix64(st + (uint64_t)attempt);
        n = s.all_items[st % (uint64_t)s.n_all_items];
        if (!in_sorted(s.hist_col, lo, hi, n)) break;
    }
    int64_t b, bj;
    int64_t* o;
    if (n_slices > 0) {
        const int64_t j = ((t + 1) * n_slices - 1) / count;  // the slice holding t
        const int64_t a = j * count / n_slices, e_ = (j + 1) * count / n_slices;
        b = t - a;
        bj = e_ - a;
        o = out + 3 * a;
    } else {
        const int64_t jb = t / bm;
        b = t - jb * bm;
        bj = (count - jb * bm) < bm ? (count - jb * bm) : bm;
        o = out + 3 * bm * jb;
    }
    o[b] = u;
    o[bj + b] = p;
    o[2 * bj + b] = n;
}

int sample_call(const rsx_sampler_args& s, int64_t batch, int64_t* out, hipStream_t st, int64_t bm = 0,
                int64_t n_slices = 0) {
    if (!s.inter_u || !s.inter_i || !s.hist_rowptr || !s.all_items || s.n_inter <= 0 || s.n_all_items <= 0 ||
        !out || batch <= 0 || s.start < 0 || s.start >= s.n_inter)
        return RSX_ERR_ARG;
    const int64_t count = (s.n_inter - s.start) < batch ? (s.n_inter - s.start) : batch;
    if (bm <= 0) bm = count;
    int bits = 2;
    while ((1ll << bits) < s.n_inter) ++bits;
    if (bits & 1) ++bits;
    hipLaunchKernelGGL(sample_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, s, bits / 2, count,
                       bm, out, n_slices);
    return last_rc();
}

// row_tag[u] = row_tag[n_users + i] = row_tag[n_users + j] = tag for every triplet
__global__ __launch_bounds__(256) void tag_rows_kernel(const int64_t* __restrict__ trip, int64_t batch,
                                                       int64_t n_users, int32_t* __restrict__ row_tag, int32_t tag,
                                                       const int32_t* __restrict__ tag_dev) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= 3 * batch) return;
    const int64_t id = trip[t];
    row_tag[t < batch ? id : n_users + id] = tag_dev ? *tag_dev : tag;
}

int bpr_fused_call(const float* fin, const float* ego, int64_t n_users, int64_t n_items, int32_t d,
                   const int64_t* trip, int64_t batch, float reg, float g_div, float* g_fin, int32_t* reg_cnt,
                   float* loss_out, double* loss_acc, void* ws, size_t ws_bytes, hipStream_t s, int32_t* halt = nullptr,
                   int32_t tag = 0);

int tag_rows(const int64_t* trip, int64_t batch, int64_t n_users, int32_t* row_tag, int32_t tag, hipStream_t s,
             const int32_t* tag_dev) {
    if (batch <= 0) return 0;
    hipLaunchKernelGGL(tag_rows_kernel, dim3((unsigned)((3 * batch + 255) / 256)), dim3(256), 0, s, trip, batch,
                       n_users, row_tag, tag, tag_dev);
    return last_rc();
}

static rsx_epilogue epi0(int kind) {
    rsx_epilogue e = {};
    e.kind = kind;
    e.alpha = 1.f;
    e.beta = 1.f;
    return e;
}

// forward: returns rc; writes final = mean_{k=0..K} A^k p; zeroes z0/z1 rows in the last pass.
static int lgcn_forward(const rsx_csr& A, int d, int K, const float* p, float* s, float* h0, float* h1, float* fin,
                        float* slab, float* z0, float* z1, hipStream_t st, const int32_t* row_tag = nullptr,
                        int32_t tag = 0) {
    const float beta = 1.f / (float)(K + 1);
    int rc;
    if (K == 0) {
        rsx_epilogue e = epi0(RSX_EPI_FINAL);
        e.s_in = p;
        e.f = fin;
        e.zero0 = z0;
        e.zero1 = z1;
        return rowwise_dispatch(A.n_rows, d, e, st);
    }
    const float* x = p;
    float* bufs[2] = {h0, h1};
    for (int k = 1; k <= K; ++k) {
        rsx_epilogue e;
        if (k == K) {
            e = epi0(RSX_EPI_FINAL);
            e.s_in = (k == 1) ? p : s;
            e.f = fin;
            e.beta = beta;
            e.zero0 = z0;
            e.zero1 = z1;
            if (row_tag) {  // only the tagged (batch) rows of the final table are needed
                e.row_tag = row_tag;
                e.tag = tag;
                e.tag_flags = RSX_TAG_ROWS;
            }
        } else {
            e = epi0(RSX_EPI_LAYERSUM);
            e.y = bufs[(k - 1) & 1];
            e.s_in = (k == 1) ? p : s;
            e.s_out = s;
        }
        if ((rc = spmm_dispatch(A, x, d, e, slab, st))) return rc;
        x = bufs[(k - 1) & 1];
    }
    return 0;
}

// The batch-tagged LightGCN step for K = 2, 3, 4 (4: the reference's default depth,
// src/configs/model/LightGCN.yaml:3): the forward keeps E^1..E^{K-1} in h0 / h1 / s
// (no running sum: s is free in this form) and computes the last layer and the mean on
// the batch rows only; BPR writes G' = dL/dfinal / (K+1) (each layer's share of the mean,
// MeanBackward); the backward is Horner on G', the reference autograd's own
// recursion  dE^{k-1} = G' + A dE^k  (A symmetric), so no layer sum is stored
// either: layer 1 gathers only the batch rows of G' (the rest are zero) and every
// layer adds G' on the batch rows only.  The last layer applies Adam with
// g = (G' + A dE^1) + R and clears G', R on the batch rows for the next step.
static int lgcn_step_stored_layers(const rsx_lgcn_step& st, int64_t batch, int32_t tag, hipStream_t s) {
    const rsx_csr& A = *st.adj;
    const int d = st.d, K = st.n_layers;
    int rc;
    float* layers[3] = {st.h0, st.h1, st.s};  // E^1, E^2, E^3
    float* bufs[2] = {st.h0, st.h1};         // the backward's ping-pong
    // forward: E^k = A E^{k-1} stored (k < K), then F = mean on the tagged rows
    const float* x = st.p;
    for (int k = 1; k < K; ++k) {
        rsx_epilogue e = epi0(RSX_EPI_STORE);
        e.y = layers[k - 1];
        TagJob tj;  // layer 1 also tags the batch rows (nothing reads the tags before the last layer)
        if (k == 1) {
            tj.trip = st.triplets;
            tj.batch = batch;
            tj.n_users = st.n_users;
            tj.row_tag = st.row_tag;
            tj.tag = tag;
        }
        if ((rc = spmm_dispatch_tagging(A, x, d, e, st.slab, s, tj))) return rc;
        x = layers[k - 1];
    }
    {
        rsx_epilogue e = epi0(RSX_EPI_FINAL);  // ((((E0 + E1) + E2) + E3) + A E^{K-1}) / (K+1)
        e.beta = 1.f / (float)(K + 1);
        e.f = st.final_emb;
        e.s_in = st.p;                        // E^0
        e.r_add = st.h0;                      // E^1
        e.aux = K >= 3 ? st.h1 : nullptr;     // E^2
        e.e0 = K == 4 ? st.s : nullptr;       // E^3
        e.row_tag = st.row_tag;
        e.tag = tag;
        e.tag_flags = RSX_TAG_ROWS;
        if ((rc = spmm_dispatch(A, x, d, e, st.slab, s))) return rc;
    }
    if (st.reg_cnt) {  // one launch; the regulariser gradient as occurrence counts for the Adam layer
        if ((rc = bpr_fused_call(st.final_emb, st.p, st.n_users, st.n_items, d, st.triplets, batch, st.reg,
                                 (float)(K + 1), st.g, st.reg_cnt, st.loss_out, st.loss_acc, st.ws, st.ws_bytes, s,
                                 st.halt, tag)))
            return rc;
    } else if ((rc = bpr_call(RSX_BPR_LIGHTGCN, st.final_emb, st.p, st.n_users, st.n_items, d, st.triplets, batch,
                              st.reg, (float)batch, st.g, st.r, st.loss_out, st.loss_acc, st.ws, st.ws_bytes, s,
                              (float)(K + 1), st.halt, tag))) {
        return rc;
    }
    // backward: H = G' + A H, H_0 = G'
    x = st.g;
    for (int k = 1; k < K; ++k) {
        rsx_epilogue e = epi0(RSX_EPI_ADD);
        e.y = bufs[(k - 1) & 1];
        e.s_in = st.g;
        e.row_tag = st.row_tag;
        e.tag = tag;
        e.tag_flags = RSX_TAG_SPARSE_S | (k == 1 ? RSX_TAG_SPARSE_X : 0);
        if ((rc = spmm_dispatch(A, x, d, e, st.slab, s))) return rc;
        x = bufs[(k - 1) & 1];
    }
    rsx_epilogue e = epi0(RSX_EPI_ADAM);
    e.s_in = st.g;
    e.r_add = st.r;
    e.p = st.p;
    e.m = st.m;
    e.v = st.v;
    e.adam = st.adam;
    e.zero0 = st.g;  // nothing reads G' or R after this layer (K >= 2)
    e.zero1 = st.r;
    if (st.reg_cnt) {
        e.r_add = nullptr;
        e.zero1 = nullptr;
        e.reg_cnt = st.reg_cnt;
        e.reg_k = reinterpret_cast<const float*>(st.reg_cnt + 3 * (st.n_users + st.n_items) + 1);
    }
    e.row_tag = st.row_tag;
    e.tag = tag;
    e.tag_flags = RSX_TAG_SPARSE_S | RSX_TAG_SPARSE_R | RSX_TAG_ZERO;
    e.halt = st.halt;  // set by the BPR above on a NaN loss
    return spmm_dispatch(A, x, d, e, st.slab, s);
}

}  // namespace rsx

extern "C" {

int rsx_sample_triplets(const int32_t* inter_u, const int32_t* inter_i, int64_t n_inter, const int64_t* hist_rowptr,
                        const int32_t* hist_col, const int32_t* all_items, int64_t n_all_items, uint64_t seed,
                        int64_t epoch, int64_t start, int64_t batch, int64_t* out, rsx_stream_t stream) {
    rsx_sampler_args s;
    s.inter_u = inter_u;
    s.inter_i = inter_i;
    s.n_inter = n_inter;
    s.hist_rowptr = hist_rowptr;
    s.hist_col = hist_col;
    s.all_items = all_items;
    s.n_all_items = n_all_items;
    s.seed = seed;
    s.epoch = epoch;
    s.start = start;
    return rsx::sample_call(s, batch, out, rsx::as_stream(stream));
}

int rsx_sample_epoch(const int32_t* inter_u, const int32_t* inter_i, int64_t n_inter, const int64_t* hist_rowptr,
                     const int32_t* hist_col, const int32_t* all_items, int64_t n_all_items, uint64_t seed,
                     int64_t epoch, int64_t batch, int64_t* out, rsx_stream_t stream) {
    rsx_sampler_args s;
    s.inter_u = inter_u;
    s.inter_i = inter_i;
    s.n_inter = n_inter;
    s.hist_rowptr = hist_rowptr;
    s.hist_col = hist_col;
    s.all_items = all_items;
    s.n_all_items = n_all_items;
    s.seed = seed;
    s.epoch = epoch;
    s.start = 0;
    if (batch <= 0) return RSX_ERR_ARG;
    return rsx::sample_call(s, n_inter, out, rsx::as_stream(stream), batch);
}

int rsx_sample_epoch_slices(const int32_t* inter_u, const int32_t* inter_i, int64_t n_inter,
                            const int64_t* hist_rowptr, const int32_t* hist_col, const int32_t* all_items,
                            int64_t n_all_items, uint64_t seed, int64_t epoch, int64_t n_slices, int64_t* out,
                            rsx_stream_t stream) {
    rsx_sampler_args s;
    s.inter_u = inter_u;
    s.inter_i = inter_i;
    s.n_inter = n_inter;
    s.hist_rowptr = hist_rowptr;
    s.hist_col = hist_col;
    s.all_items = all_items;
    s.n_all_items = n_all_items;
    s.seed = seed;
    s.epoch = epoch;
    s.start = 0;
    if (n_slices <= 0 || n_slices > n_inter) return RSX_ERR_ARG;  // every slice holds >= 1 triplet
    return rsx::sample_call(s, n_inter, out, rsx::as_stream(stream), n_inter, n_slices);
}

int rsx_layergcn_step(const rsx_layergcn_step_args* st, rsx_stream_t stream) {
    using namespace rsx;
    if (!st || !st->adj || !st->p || !st->m || !st->v || !st->out || !st->g || !st->r || !st->acc || !st->h0 ||
        !st->h1 || !st->zs || !st->cs || !st->triplets || st->batch <= 0 || st->n_layers < 1)
        return RSX_ERR_ARG;
    const rsx_csr& A = *st->adj;
    const int d = st->d, K = st->n_layers;
    const int64_t n = st->n_users + st->n_items;
    if (A.n_rows != n) return RSX_ERR_ARG;
    for (int k = 0; k < K; ++k)
        if (!st->zs[k] || !st->cs[k]) return RSX_ERR_ARG;
    hipStream_t s = as_stream(stream);
    float* h[2] = {st->h0, st->h1};
    int rc;
    // forward: E^k = cos-gated A E^{k-1}; out = sum_k E^k; the last layer zeroes g, r
    const float* x = st->p;
    for (int k = 1; k <= K; ++k) {
        rsx_epilogue e = epi0(RSX_EPI_LAYERGCN);
        e.e0 = st->p;
        e.y = h[(k - 1) & 1];
        e.s_out = st->out;
        e.s_in = k > 1 ? st->out : nullptr;
        e.aux = st->zs[k - 1];
        e.aux_w = st->cs[k - 1];
        if (k == K) {
            e.zero0 = st->g;
            e.zero1 = st->r;
        }
        if ((rc = spmm_dispatch(A, x, d, e, st->slab, s))) return rc;
        x = h[(k - 1) & 1];
    }
    if ((rc = bpr_call(RSX_BPR_LAYERGCN, st->out, st->p, st->n_users, st->n_items, d, st->triplets, st->batch,
                       st->reg, (float)st->batch, st->g, st->r, st->loss_out, st->loss_acc, st->ws, st->ws_bytes, s)))
        return rc;
    // dE^K = g -> dZ^K (rowwise), the ego-cosine terms into acc
    {
        rsx_epilogue e = epi0(RSX_EPI_LAYERGCN_BWD);
        e.r_add = st->g;
        e.aux = st->zs[K - 1];
        e.aux_w = st->cs[K - 1];
        e.e0 = st->p;
        e.y = h[0];
        e.s_out = st->acc;
        if ((rc = rowwise_dispatch(n, d, e, s))) return rc;
    }
    const float* hz = h[0];
    for (int k = K - 1; k >= 1; --k) {
        rsx_epilogue e = epi0(RSX_EPI_LAYERGCN_BWD);
        e.r_add = st->g;
        e.aux = st->zs[k - 1];
        e.aux_w = st->cs[k - 1];
        e.e0 = st->p;
        e.y = h[(K - k) & 1];
        e.s_in = st->acc;
        e.s_out = st->acc;
        if ((rc = spmm_dispatch(A, hz, d, e, st->slab, s))) return rc;
        hz = h[(K - k) & 1];
    }
    // dE^0 = A dZ^1 + cosine terms + reg -> Adam
    rsx_epilogue e = epi0(RSX_EPI_ADAM);
    e.s_in = st->acc;
    e.r_add = st->r;
    e.p = st->p;
    e.m = st->m;
    e.v = st->v;
    e.adam = st->adam;
    return spmm_dispatch(A, hz, d, e, st->slab, s);
}

int rsx_lightgcn_forward(const rsx_csr* adj, int32_t d, int32_t n_layers, const float* p, float* s, float* h0,
                         float* h1, float* final_emb, float* slab, rsx_stream_t stream) {
    if (!adj || !p || !final_emb || n_layers < 0) return RSX_ERR_ARG;
    if (n_layers >= 2 && (!s || !h0 || !h1)) return RSX_ERR_ARG;
    return rsx::lgcn_forward(*adj, d, n_layers, p, s, h0, h1, final_emb, slab, nullptr, nullptr,
                             rsx::as_stream(stream));
}

int rsx_lightgcn_step(const rsx_lgcn_step* st, rsx_stream_t stream) {
    using namespace rsx;
    if (!st || !st->adj || !st->p || !st->m || !st->v || !st->final_emb || !st->g || !st->r || !st->triplets)
        return RSX_ERR_ARG;
    const rsx_csr& A = *st->adj;
    const int d = st->d, K = st->n_layers;
    if (K < 0 || A.n_rows != st->n_users + st->n_items) return RSX_ERR_ARG;
    if (K >= 2 && (!st->s || !st->h0 || !st->h1)) return RSX_ERR_ARG;
    hipStream_t s = as_stream(stream);
    int rc;
    int64_t batch = st->batch;
    if (st->sample) {
        const rsx_sampler_args& sa = *st->sample;
        if ((rc = sample_call(sa, st->batch, st->triplets, s))) return rc;
        batch = (sa.n_inter - sa.start) < st->batch ? (sa.n_inter - sa.start) : st->batch;
    }
    // batch-row tags (K >= 2): last forward layer on the batch rows only, sparse G in
    // the first backward layer, G / R cleared on the batch rows by the Adam layer
    const bool tags = st->row_tag && K >= 2;
    const int32_t tag = (int32_t)st->tag;
    if (tags) {
        if (st->tag <= 0 || st->tag > INT32_MAX) return RSX_ERR_ARG;
        if (K <= 4) return lgcn_step_stored_layers(*st, batch, tag, s);  // tags written by its layer 1
        if ((rc = tag_rows(st->triplets, batch, st->n_users, st->row_tag, tag, s, nullptr))) return rc;
    }
    // forward (dense path: the last layer zeroes g and r)
    if ((rc = lgcn_forward(A, d, K, st->p, st->s, st->h0, st->h1, st->final_emb, st->slab, tags ? nullptr : st->g,
                           tags ? nullptr : st->r, s, tags ? st->row_tag : nullptr, tag)))
        return rc;
    // BPR loss + gradients
    if ((rc = bpr_call(RSX_BPR_LIGHTGCN, st->final_emb, st->p, st->n_users, st->n_items, d, st->triplets, batch,
                       st->reg, (float)batch, st->g, st->r, st->loss_out, st->loss_acc, st->ws, st->ws_bytes, s, 1.f,
                       st->halt, (int32_t)st->tag)))
        return rc;
    // backward (Horner) with Adam fused into the last layer
    const float beta = 1.f / (float)(K + 1);
    if (K == 0) {
        rsx_epilogue e = epi0(RSX_EPI_ADAM);
        e.s_in = st->g;
        e.r_add = st->r;
        e.p = st->p;
        e.m = st->m;
        e.v = st->v;
        e.adam = st->adam;
        e.halt = st->halt;
        return rowwise_dispatch(A.n_rows, d, e, s);
    }
    const float* x = st->g;
    float* bufs[2] = {st->h0, st->h1};
    for (int k = 1; k <= K; ++k) {
        rsx_epilogue e;
        if (k == K) {
            e = epi0(RSX_EPI_ADAM);
            e.s_in = (k == 1) ? st->g : st->s;
            e.beta = beta;
            e.r_add = st->r;
            e.p = st->p;
            e.m = st->m;
            e.v = st->v;
            e.adam = st->adam;
            e.halt = st->halt;  // set by the BPR above on a NaN loss
            if (tags) {  // K >= 2: nothing reads G or R after this layer
                e.row_tag = st->row_tag;
                e.tag = tag;
                e.tag_flags = RSX_TAG_SPARSE_R | RSX_TAG_ZERO;
                e.zero0 = st->g;
                e.zero1 = st->r;
            }
        } else {
            e = epi0(RSX_EPI_LAYERSUM);
            e.y = bufs[(k - 1) & 1];
            e.s_in = (k == 1) ? st->g : st->s;
            e.s_out = st->s;
            if (tags && k == 1) {  // X = G and s_in = G: zero off the batch rows
                e.row_tag = st->row_tag;
                e.tag = tag;
                e.tag_flags = RSX_TAG_SPARSE_X | RSX_TAG_SPARSE_S;
            }
        }
        if ((rc = spmm_dispatch(A, x, d, e, st->slab, s))) return rc;
        x = bufs[(k - 1) & 1];
    }
    return 0;
}

}  // extern "C"

// dp.hip — data-parallel LightGCN step over RCCL (gfx950, one process per GPU).
//
// The reference trains one batch of B triplets per step on one device
// (src/common/trainer.py:186-238, src/models/lightgcn.py:117-156).  Here every rank
// holds the WHOLE graph and a bit-identical replica of the tables, and each step trains
// the global batch of W * B triplets (rank r draws its own B): the reference objective
// at batch W * B — mean BPR over the global batch + reg * (|U|_F + |P|_F + |N|_F) / W B
// with the Frobenius norms over the global batch's rows.
//
// What crosses the ranks is small.  The propagation is linear, so the gradient of the
// embedding table is the backward operator applied to G' = dL/dfinal / (K+1), and G' is
// nonzero on the batch rows only: rank r's share G'_r lives on its own <= 3B rows.  So a
// step exchanges (1) every rank's triplets (3B int64, gathered while the forward runs)
// and (2) every rank's G'_r at its own occurrence rows plus four f64 loss totals
// (3B d floats): an all-gather of ~1.6 MB per rank at sports shape, against 13.8 MB for
// an all-reduce of the dense gradient.  Every rank then merges the blocks into the same
// G' (a deterministic rank-ordered sum per row, below), counts every triplet's rows for
// the regulariser, and runs the same backward and Adam: the replicas stay bit-identical
// with no parameter exchange.  Per step: 2 all-gathers; ~2 x 2.2 % of the C2 step's
// kernels extra (pack, gather, index, merge).
//
// Merge.  Rank r's block row j is G'_r at the row x of occurrence j (duplicate
// occurrences in one rank carry identical rows: gathered from the same table row).
// pos[r][x] = (stamp << 32) | j for SOME occurrence j of x in rank r (a benign race of
// equal candidates); the occurrence that won pos[r][x], in the lowest rank holding x, is
// x's leader, and the leader writes G'[x] = sum over ranks r' in rank order of
// block[r'][pos[r'][x]].  Every rank evaluates the same sums in the same order.  The
// stamp is the step's tag, so pos is never cleared.
#include "rsx_common.hpp"

namespace rsx {

int spmm_dispatch(const rsx_csr& a, const float* x, int d, const rsx_epilogue& e, float* slab, hipStream_t s);
int spmm_dispatch_tagging(const rsx_csr& a, const float* x, int d, const rsx_epilogue& e, float* slab,
                          hipStream_t s, const TagJob& tj);
int bpr_fused_args(const float* fin, const float* ego, int64_t n_users, int64_t n_items, int32_t d,
                   const int64_t* trip, int64_t batch, float reg, float g_div, float* g_fin, int32_t* reg_cnt,
                   float* loss_out, double* loss_acc, void* ws, size_t ws_bytes, hipStream_t s, int32_t* halt,
                   int32_t tag, const int64_t* dp_slots, int64_t dp_slot_len, int32_t dp_world, double* dp_tot);
int comm_rank(rsx_comm_t c);
int comm_world(rsx_comm_t c);
hipStream_t comm_stream(rsx_comm_t c, hipStream_t s);
hipEvent_t comm_event(rsx_comm_t c);
hipEvent_t collective(rsx_comm_t c, int op, void* buf, int64_t count, int dtype, hipStream_t s, int* rc);

namespace {

constexpr int kHdr = 8;  // block header: four f64 loss totals

// slot = [B, users[cap], positives[cap], negatives[cap]] (tail zero)
// (step: the Adam counter the step increments first, or NULL)
__global__ __launch_bounds__(256) void dp_pack(const int64_t* __restrict__ trip, int64_t B, int64_t cap,
                                               int64_t* __restrict__ slot, int64_t* __restrict__ step) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i > 3 * cap) return;
    if (i == 0) {
        slot[0] = B;
        if (step) step[0] += 1;
        return;
    }
    const int64_t j = i - 1, k = j / cap, t = j - k * cap;
    slot[i] = t < B ? trip[k * B + t] : 0;
}

// occurrence i = (r, j = kind cap + t) of the gathered slots -> its table row (or -1)
__device__ __forceinline__ int64_t occ_row(const int64_t* slots, int64_t L, int64_t cap, int64_t n_users, int64_t i,
                                           int64_t* r_out, int64_t* j_out) {
    const int64_t r = i / (3 * cap), j = i - r * 3 * cap;
    const int64_t* slot = slots + r * L;
    const int64_t t = j % cap;
    *r_out = r;
    *j_out = j;
    if (t >= slot[0]) return -1;
    const int64_t id = slot[1 + j];
    return j < cap ? id : n_users + id;
}

// Union tags, global occurrence counts (the regulariser's), and pos[r][x] for every
// occurrence of every rank (runs on the comm stream once the triplets are gathered).
__global__ __launch_bounds__(256) void dp_index(const int64_t* __restrict__ slots, int32_t W, int64_t cap,
                                                int64_t n_users, int64_t N, int64_t* __restrict__ pos,
                                                int32_t* __restrict__ row_tag, int32_t* __restrict__ reg_cnt,
                                                const int32_t* __restrict__ tag_dev) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)W * 3 * cap) return;
    int64_t r, j;
    const int64_t x = occ_row(slots, 3 * cap + 1, cap, n_users, i, &r, &j);
    if (x < 0) return;
    const int32_t stamp = *tag_dev;
    pos[r * N + x] = ((int64_t)stamp << 32) | j;
    row_tag[x] = stamp;
    atomicAdd(reg_cnt + 3 * x + j / cap, 1);
}

// One lane group (D/4 lanes, a float4 each) per occurrence: the leaders write the
// rank-ordered sums.  Block 0 also finishes the global loss (bpr_fused's formula on the
// summed totals) and the regulariser's three scales.
template <int D>
__global__ __launch_bounds__(256) void dp_merge(const int64_t* __restrict__ slots, int32_t W, int64_t cap,
                                                int64_t n_users, int64_t N, const int64_t* __restrict__ pos,
                                                const float* __restrict__ blocks, int64_t stride,
                                                float* __restrict__ g, const int32_t* __restrict__ tag_dev,
                                                int32_t* __restrict__ reg_cnt, float reg, float* loss_out,
                                                double* loss_acc, int32_t* halt) {
    constexpr int G = D / 4, GPB = 256 / G;
    const int32_t stamp = *tag_dev;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        double tl = 0.0, qu = 0.0, qp = 0.0, qn = 0.0;
        int64_t bg = 0;
        for (int r = 0; r < W; ++r) {
            const double* h = reinterpret_cast<const double*>(blocks + (int64_t)r * stride + 3 * cap * D);
            tl += h[0];
            qu += h[1];
            qp += h[2];
            qn += h[3];
            bg += slots[(int64_t)r * (3 * cap + 1)];
        }
        const double B = (double)bg;
        const double nu = sqrt(qu), np = sqrt(qp), nn = sqrt(qn);
        const double loss = tl / B + (double)reg * (nu + np + nn) / B;
        float* k = reinterpret_cast<float*>(reg_cnt + 3 * N + 1);
        k[0] = nu > 0 ? (float)((double)reg / (B * nu)) : 0.f;
        k[1] = np > 0 ? (float)((double)reg / (B * np)) : 0.f;
        k[2] = nn > 0 ? (float)((double)reg / (B * nn)) : 0.f;
        if (loss_out) loss_out[0] = (float)loss;
        if (loss_acc) loss_acc[0] += loss;
        if (halt && loss != loss && halt[0] == 0) {
            halt[1] = stamp;
            halt[0] = 1;
        }
    }
    const int li = threadIdx.x % G;
    const int64_t i = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
    if (i >= (int64_t)W * 3 * cap) return;
    int64_t r, j;
    const int64_t x = occ_row(slots, 3 * cap + 1, cap, n_users, i, &r, &j);
    if (x < 0) return;
    if (pos[r * N + x] != (((int64_t)stamp << 32) | j)) return;  // not this rank's representative of x
    for (int64_t q = 0; q < r; ++q)
        if ((int32_t)(pos[q * N + x] >> 32) == stamp) return;  // a lower rank holds x: its leader sums
    float4 acc = f4(0.f);
    for (int64_t q = r; q < W; ++q) {
        const int64_t pq = pos[q * N + x];
        if ((int32_t)(pq >> 32) != stamp) continue;
        acc = add4(acc, ld4(blocks + q * stride + (pq & 0xffffffffll) * D + li * 4));
    }
    st4(g + x * D + li * 4, acc);
}

// block[own] rows = G'_own at this rank's occurrences
__global__ __launch_bounds__(256) void dp_gather(const int64_t* __restrict__ trip, int64_t B, int64_t cap,
                                                 int64_t n_users, int d, const float* __restrict__ g,
                                                 float* __restrict__ blk) {
    const int q = d / 4;
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= 3 * B * q) return;
    const int64_t o = e / q;
    const int c = (int)(e - o * q) * 4;
    const int64_t k = o / B, t = o - k * B;
    const int64_t id = trip[k * B + t];
    const int64_t x = k == 0 ? id : n_users + id;
    st4(blk + (k * cap + t) * d + c, ld4(g + x * d + c));
}

rsx_epilogue epi(int kind) {
    rsx_epilogue e = {};
    e.kind = kind;
    e.alpha = 1.f;
    e.beta = 1.f;
    return e;
}

#define DP_TRY(x)              \
    do {                       \
        const int rc_ = (x);   \
        if (rc_) return rc_;   \
    } while (0)

int dp_step(const rsx_dp_lgcn_step& st, hipStream_t s) {
    const rsx_csr& A = *st.adj;
    const int d = st.d, K = st.n_layers;
    const int64_t nu = st.n_users, N = st.n_users + st.n_items, cap = st.cap, B = st.batch;
    const int32_t W = comm_world(st.comm), rank = comm_rank(st.comm);
    const int64_t L = 3 * cap + 1, stride = 3 * cap * d + kHdr;
    int rc = 0;
    // (1) this rank's triplets into its slot; every rank's gathered while the forward runs,
    // then indexed (union tags, counts, pos) on the comm stream
    hipLaunchKernelGGL(dp_pack, dim3((unsigned)((L + 255) / 256)), dim3(256), 0, s, st.triplets, B, cap,
                       st.slots + rank * L, st.inc_step ? const_cast<int64_t*>(st.adam.step_dev) : nullptr);
    DP_TRY(last_rc());
    if (!collective(st.comm, RSX_COLL_ALLGATHER, st.slots, L, RSX_COLL_I64, s, &rc)) return rc;
    hipStream_t cs = comm_stream(st.comm, s);
    const int64_t n_occ = (int64_t)W * 3 * cap;
    hipLaunchKernelGGL(dp_index, dim3((unsigned)((n_occ + 255) / 256)), dim3(256), 0, cs, st.slots, W, cap, nu, N,
                       st.pos, st.row_tag, st.reg_cnt, st.tag_dev);
    DP_TRY(last_rc());
    hipEvent_t j_idx = nullptr;
    if (cs != s) {
        j_idx = comm_event(st.comm);
        DP_TRY(hip_rc(hipEventRecord(j_idx, cs)));
    }
    // (2) forward: E^1..E^{K-1} stored (layer 1 also tags this rank's batch rows in own_tag),
    // the last layer and the mean on those rows only (lgcn_step_stored_layers' forward)
    float* layers[3] = {st.h0, st.h1, st.s};
    const float* x = st.p;
    for (int k = 1; k < K; ++k) {
        rsx_epilogue e = epi(RSX_EPI_STORE);
        e.y = layers[k - 1];
        TagJob tj;
        if (k == 1) {
            tj.trip = st.triplets;
            tj.batch = B;
            tj.n_users = nu;
            tj.row_tag = st.own_tag;
            tj.tag_dev = st.tag_dev;
        }
        DP_TRY(spmm_dispatch_tagging(A, x, d, e, st.slab, s, tj));
        x = layers[k - 1];
    }
    {
        rsx_epilogue e = epi(RSX_EPI_FINAL);
        e.beta = 1.f / (float)(K + 1);
        e.f = st.final_emb;
        e.s_in = st.p;
        e.r_add = st.h0;
        e.aux = K >= 3 ? st.h1 : nullptr;
        e.e0 = K == 4 ? st.s : nullptr;
        e.row_tag = st.own_tag;
        e.tag_dev = st.tag_dev;
        e.tag_flags = RSX_TAG_ROWS;
        DP_TRY(spmm_dispatch(A, x, d, e, st.slab, s));
    }
    // (3) this rank's BPR share over the global batch: G'_own (table), its totals into its block
    if (j_idx) DP_TRY(hip_rc(hipStreamWaitEvent(s, j_idx, 0)));  // the slots (global batch size)
    float* own_blk = st.blocks + rank * stride;
    DP_TRY(bpr_fused_args(st.final_emb, st.p, nu, st.n_items, d, st.triplets, B, st.reg, (float)(K + 1), st.g,
                          st.reg_cnt, nullptr, nullptr, st.ws, st.ws_bytes, s, nullptr, 0, st.slots, L, W,
                          reinterpret_cast<double*>(own_blk + 3 * cap * d)));
    {
        const int64_t n = 3 * B * (d / 4);
        hipLaunchKernelGGL(dp_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, st.triplets, B, cap, nu, d,
                           st.g, own_blk);
        DP_TRY(last_rc());
    }
    // (4) every rank's block, merged into the same G' on every rank
    hipEvent_t jb = collective(st.comm, RSX_COLL_ALLGATHER, st.blocks, stride, RSX_COLL_F32, s, &rc);
    if (!jb) return rc;
    DP_TRY(hip_rc(hipStreamWaitEvent(s, jb, 0)));
    {
        const int G = d / 4, gpb = 256 / G;
        const dim3 grid((unsigned)((n_occ + gpb - 1) / gpb));
#define DP_MERGE(DD)                                                                                                \
    hipLaunchKernelGGL((dp_merge<DD>), grid, dim3(256), 0, s, st.slots, W, cap, nu, N, st.pos, st.blocks, stride, \
                       st.g, st.tag_dev, st.reg_cnt, st.reg, st.loss_out, st.loss_acc, st.halt)
        switch (d) {
            case 32: DP_MERGE(32); break;
            case 64: DP_MERGE(64); break;
            case 128: DP_MERGE(128); break;
            case 256: DP_MERGE(256); break;
            default: return RSX_ERR_UNSUPPORTED;
        }
#undef DP_MERGE
        DP_TRY(last_rc());
    }
    // (5) backward on the union rows: H = G' + A H from H = G', Adam on g = H^K + R with the
    // global counts and scales, G' and the counts cleared on the union rows
    x = st.g;
    float* bufs[2] = {st.h0, st.h1};
    for (int k = 1; k < K; ++k) {
        rsx_epilogue e = epi(RSX_EPI_ADD);
        e.y = bufs[(k - 1) & 1];
        e.s_in = st.g;
        e.row_tag = st.row_tag;
        e.tag_dev = st.tag_dev;
        e.tag_flags = RSX_TAG_SPARSE_S | (k == 1 ? RSX_TAG_SPARSE_X : 0);
        DP_TRY(spmm_dispatch(A, x, d, e, st.slab, s));
        x = bufs[(k - 1) & 1];
    }
    rsx_epilogue e = epi(RSX_EPI_ADAM);
    e.s_in = st.g;
    e.p = st.p;
    e.m = st.m;
    e.v = st.v;
    e.adam = st.adam;
    e.zero0 = st.g;
    e.reg_cnt = st.reg_cnt;
    e.reg_k = reinterpret_cast<const float*>(st.reg_cnt + 3 * N + 1);
    e.row_tag = st.row_tag;
    e.tag_dev = st.tag_dev;
    e.tag_flags = RSX_TAG_SPARSE_S | RSX_TAG_SPARSE_R | RSX_TAG_ZERO;
    e.halt = st.halt;
    return spmm_dispatch(A, x, d, e, st.slab, s);
}

bool dp_valid(const rsx_dp_lgcn_step* st) {
    if (!st || !st->adj || !st->comm || !st->p || !st->m || !st->v || !st->h0 || !st->h1 || !st->final_emb ||
        !st->g || !st->triplets || !st->row_tag || !st->own_tag || !st->tag_dev || !st->reg_cnt || !st->slots ||
        !st->blocks || !st->pos || !st->ws)
        return false;
    if (st->n_layers < 2 || st->n_layers > 4 || (st->n_layers == 4 && !st->s)) return false;
    if (st->batch <= 0 || st->batch > st->cap || st->n_users < 0 || st->n_items <= 0) return false;
    if (st->adj->n_rows != st->n_users + st->n_items || st->adj->n_cols != st->adj->n_rows) return false;
    if (st->adj->n_long > 0 && !st->slab) return false;
    if (3 * st->cap > 0x7fffffffll) return false;  // occurrence index in pos's low word
    if (st->inc_step && (!st->adam.step_dev || (const void*)st->adam.step_dev != (const void*)st->tag_dev))
        return false;  // the incremented counter is the tag every later launch reads
    return true;
}

}  // namespace
}  // namespace rsx

extern "C" {

int rsx_dp_lightgcn_step(const rsx_dp_lgcn_step* st, rsx_stream_t stream) {
    if (!rsx::dp_valid(st)) return RSX_ERR_ARG;
    if (st->d != 32 && st->d != 64 && st->d != 128 && st->d != 256) return RSX_ERR_UNSUPPORTED;
    return rsx::dp_step(*st, rsx::as_stream(stream));
}

size_t rsx_dp_block_floats(int64_t cap, int32_t d) { return (size_t)(3 * cap * d + rsx::kHdr); }

}  // extern "C"

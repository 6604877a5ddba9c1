// dp.hip — data-parallel LightGCN step over RCCL (gfx950, one process per GPU).
//
// The reference trains one batch of B triplets per step on one device
// (src/common/trainer.py:186-238, src/models/lightgcn.py:117-156).  Here every rank
// holds the WHOLE graph and a bit-identical replica of the tables, and each step trains
// the global batch of W * B triplets (rank r draws its own B): the reference objective
// at batch W * B — mean BPR over the global batch + reg * (|U|_F + |P|_F + |N|_F) / W B
// with the Frobenius norms over the global batch's rows.
//
// Only the triplets cross the ranks.  The propagation is replicated (every rank runs it
// on the whole graph: on these graphs its cost is per step, not per triplet), so every
// rank can evaluate the loss of EVERY rank's triplets itself once it knows them: a step
// all-gathers the ranks' triplets (3B int64 per rank, 48 KB at B = 2048, on the comm
// stream while the forward runs) and nothing else.  Round 4 all-gathered every rank's
// dL/dfinal rows instead (1.6 MB per rank, on the critical path between the loss and the
// backward); that exchange is gone.  Every rank then runs the same kernels on the same
// inputs: the last forward layer on the union of the ranks' batch rows, the BPR loss of
// the global batch, its gradient G' = dL/dfinal / (K+1), the backward and Adam — so the
// replicas stay bit-identical with no parameter exchange, provided every kernel is
// deterministic.  The SpMMs and the loss reductions are (fixed orders); G' is a sum of
// per-occurrence terms over rows that repeat in the batch, so it is accumulated in
// 64-bit fixed point (integer adds commute: the order of the atomics cannot change a
// bit), at a power-of-two scale from a bound on the batch's rows, then rounded to f32
// once.  A row with one occurrence gets exactly the f32 term the single-GPU step adds.
//
// Per step on the comm stream (hidden behind the forward): the triplet all-gather, the
// union tags and global regulariser counts (dp_index), and the W 3 B occurrences bucketed
// by row (dp_alloc: each union row's first claimer reserves a run of its count;
// dp_scatter: each occurrence takes a place in its row's run), which lets the gradient
// pass add each run of equal rows in registers and issue one atomic per run instead of
// one per occurrence (hot items occur hundreds of times in a global batch).  Where a run
// lands and its order are not fixed, and need not be: the sums are integer (below).  Two
// small launches instead of a radix sort's five (merge-sort passes for these sizes,
// ~43 us at W = 1 and ~47 at W = 8 on the comm stream: the loss waited on them).
#include <cmath>

#include "rsx_common.hpp"

namespace rsx {

int spmm_dispatch(const rsx_csr& a, const float* x, int d, const rsx_epilogue& e, float* slab, hipStream_t s);
int comm_rank(rsx_comm_t c);
int comm_world(rsx_comm_t c);
int comm_sim_world(rsx_comm_t c);
hipStream_t comm_stream(rsx_comm_t c, hipStream_t s);
hipEvent_t comm_event(rsx_comm_t c);
hipEvent_t collective(rsx_comm_t c, int op, void* buf, int64_t count, int dtype, hipStream_t s, int* rc);

namespace {

constexpr int kBlk = 256;

// The step's workspace (rsx_dp_lgcn_step.work), carved in this order, 256-B aligned.
struct Work {
    unsigned long long* acc;  // [N][d] fixed-point G' accumulators (zero between steps)
    int32_t* start;           // [N] a union row's run start + 1 (0: unclaimed; cleared by dp_bpr_round)
    int32_t* cursor;          // [N] places taken in the row's run (cleared by dp_bpr_round)
    int32_t* keys;            // [W 3 cap] the row of each run place
    int32_t* occ;             // [W 3 cap] the occurrence at each run place
    float* coef;              // [W][cap] per-triplet dL/d(s+ - s-)
    double* part;             // [n_blk_a][5] loss, |U|^2, |P|^2, |N|^2, max |f| partials
    int32_t* meta;            // [4]: done counter, fixed-point exponent, run places taken
    size_t total;
};

size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

Work carve(void* base, int64_t N, int d, int64_t cap, int W) {
    Work w = {};
    const int64_t n_occ = (int64_t)W * 3 * cap, n_trip = (int64_t)W * cap;
    const int64_t n_blk = (n_trip + 3) / 4 + 1;  // phase A: >= 4 triplets per block (d <= 256)
    char* p = static_cast<char*>(base);
    size_t o = 0;
    auto take = [&](size_t bytes) {
        void* q = p ? p + o : nullptr;
        o += al(bytes);
        return q;
    };
    w.acc = static_cast<unsigned long long*>(take((size_t)N * d * 8));
    w.start = static_cast<int32_t*>(take((size_t)N * 4));
    w.cursor = static_cast<int32_t*>(take((size_t)N * 4));
    w.keys = static_cast<int32_t*>(take((size_t)n_occ * 4));
    w.occ = static_cast<int32_t*>(take((size_t)n_occ * 4));
    w.coef = static_cast<float*>(take((size_t)n_trip * 4));
    w.part = static_cast<double*>(take((size_t)n_blk * 5 * 8));
    w.meta = static_cast<int32_t*>(take(16));
    w.total = o;
    return w;
}

// slot = [B, users[cap], positives[cap], negatives[cap]] (tail zero)
// (step: the Adam counter the step increments first, or NULL)
// (meta[2], the run places the previous step took, is zeroed here: the step's first
// launch, ahead of the comm stream's fork)
__global__ __launch_bounds__(kBlk) void dp_pack(const int64_t* __restrict__ trip, int64_t B, int64_t cap,
                                                int64_t* __restrict__ slot, int64_t* __restrict__ step,
                                                int32_t* __restrict__ meta) {
    const int64_t i = (int64_t)blockIdx.x * kBlk + threadIdx.x;
    if (i > 3 * cap) return;
    if (i == 0) {
        slot[0] = B;
        if (step) step[0] += 1;
        meta[2] = 0;
        return;
    }
    const int64_t j = i - 1, k = j / cap, t = j - k * cap;
    slot[i] = t < B ? trip[k * B + t] : 0;
}

// one real rank (the slot is the gathered buffer): dp_pack and dp_index in one launch --
// each occurrence is packed and indexed by the thread that reads it (the same tags and
// integer counts).  The tag is the Adam counter, which this step increments: here every
// thread tags with the counter + inc, and dp_alloc, the next launch, does the increment
// (a thread of this launch may read the counter before or after another one writes it)
__global__ __launch_bounds__(kBlk) void dp_pack_index(const int64_t* __restrict__ trip, int64_t B, int64_t cap,
                                                      int64_t n_users, int64_t* __restrict__ slot, int32_t inc,
                                                      int32_t* __restrict__ meta, int32_t* __restrict__ row_tag,
                                                      int32_t* __restrict__ reg_cnt,
                                                      const int32_t* __restrict__ tag_dev) {
    const int64_t i = (int64_t)blockIdx.x * kBlk + threadIdx.x;
    if (i > 3 * cap) return;
    if (i == 0) {
        slot[0] = B;
        meta[2] = 0;
        return;
    }
    const int64_t j = i - 1, k = j / cap, t = j - k * cap;
    if (t >= B) {
        slot[i] = 0;
        return;
    }
    const int64_t id = trip[k * B + t];
    slot[i] = id;
    const int64_t x = k == 0 ? id : n_users + id;
    row_tag[x] = *tag_dev + inc;
    atomicAdd(reg_cnt + 3 * x + k, 1);
}

// occurrence i = (r, j = kind cap + t) of the gathered slots -> its table row (or -1)
__device__ __forceinline__ int64_t occ_row(const int64_t* slots, int64_t cap, int64_t n_users, int64_t i) {
    const int64_t L = 3 * cap + 1;
    const int64_t r = i / (3 * cap), j = i - r * 3 * cap;
    const int64_t* slot = slots + r * L;
    if (j % cap >= slot[0]) return -1;
    const int64_t id = slot[1 + j];
    return j < cap ? id : n_users + id;
}

// (comm stream, once the triplets are gathered) union tags and global occurrence counts
// (the regulariser's, and the runs' lengths)
__global__ __launch_bounds__(kBlk) void dp_index(const int64_t* __restrict__ slots, int32_t W, int64_t cap,
                                                 int64_t n_users, int32_t* __restrict__ row_tag,
                                                 int32_t* __restrict__ reg_cnt, const int32_t* __restrict__ tag_dev) {
    const int64_t i = (int64_t)blockIdx.x * kBlk + threadIdx.x;
    if (i >= (int64_t)W * 3 * cap) return;
    const int64_t x = occ_row(slots, cap, n_users, i);
    if (x < 0) return;
    row_tag[x] = *tag_dev;
    atomicAdd(reg_cnt + 3 * x + (i % (3 * cap)) / cap, 1);
}

// (comm stream) each union row's run: its first claimer reserves count places.  The
// claims of a wave are summed first (a scan over its lanes) and reserved with one atomic
// per wave: one counter taking an atomic per union row serialised at its L2 channel
// (12 us at W = 1, 16 at W = 8)
__global__ __launch_bounds__(kBlk) void dp_alloc(const int64_t* __restrict__ slots, int32_t W, int64_t cap,
                                                 int64_t n_users, const int32_t* __restrict__ reg_cnt,
                                                 int32_t* __restrict__ start, int32_t* __restrict__ meta,
                                                 int64_t* __restrict__ step) {
    const int64_t i = (int64_t)blockIdx.x * kBlk + threadIdx.x;
    const int lane = threadIdx.x % kWave;
    if (step && i == 0) step[0] += 1;  // the Adam counter, after dp_pack_index (one real rank)
    int64_t x = -1;
    int32_t n = 0;
    if (i < (int64_t)W * 3 * cap) {
        x = occ_row(slots, cap, n_users, i);
        if (x >= 0 && atomicCAS(start + x, 0, -1) == 0)
            n = reg_cnt[3 * x] + reg_cnt[3 * x + 1] + reg_cnt[3 * x + 2];
        else
            x = -1;
    }
    int32_t inc = n;  // inclusive scan of the wave's claims (every lane of the wave is here)
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const int32_t v = __shfl_up(inc, o, kWave);
        if (lane >= o) inc += v;
    }
    int32_t base = 0;
    if (lane == kWave - 1 && inc > 0) base = atomicAdd(meta + 2, inc);
    base = __shfl(base, kWave - 1, kWave);
    if (x >= 0) start[x] = base + (inc - n) + 1;
}

// (comm stream) every occurrence takes a place in its row's run
__global__ __launch_bounds__(kBlk) void dp_scatter(const int64_t* __restrict__ slots, int32_t W, int64_t cap,
                                                   int64_t n_users, const int32_t* __restrict__ start,
                                                   int32_t* __restrict__ cursor, int32_t* __restrict__ keys,
                                                   int32_t* __restrict__ occ) {
    const int64_t i = (int64_t)blockIdx.x * kBlk + threadIdx.x;
    if (i >= (int64_t)W * 3 * cap) return;
    const int64_t x = occ_row(slots, cap, n_users, i);
    if (x < 0) return;
    const int32_t p = start[x] - 1 + atomicAdd(cursor + x, 1);
    keys[p] = (int32_t)x;
    occ[p] = (int32_t)i;
}

// Phase A: every triplet of every rank — s+ - s- from the final rows, the BPR term and its
// coefficient (bpr_fused's formulas at the global batch size), the regulariser's squared
// norms on the ego rows and max |f| (the fixed-point scale's bound); per-block f64
// partials, reduced by the last block in a fixed order into the loss, the regulariser's
// three scales (reg_cnt's tail, as the single-GPU BPR leaves them) and the exponent.
// A lane group takes TPG triplets (4 on a large global batch) and issues all their row
// gathers before the first use (the kernel is a chain of dependent loads at ~1 wave a SIMD:
// the ids, then the rows), which also cuts the blocks, so the last block's partial loads
// are one round, issued together; a small batch keeps one triplet a group (more waves).
template <int D, int TPG>
__global__ __launch_bounds__(kBlk) void dp_bpr_coef(const int64_t* __restrict__ slots, int32_t W, int64_t cap,
                                                    int64_t n_users, int64_t N, const float* __restrict__ fin,
                                                    const float* __restrict__ ego, float g_div, float reg,
                                                    float* __restrict__ coef, double* __restrict__ part,
                                                    int32_t* __restrict__ meta, int32_t* __restrict__ reg_cnt,
                                                    float* loss_out, double* loss_acc, int32_t* halt,
                                                    const int32_t* __restrict__ tag_dev,
                                                    const int32_t* __restrict__ start, int32_t* __restrict__ cursor,
                                                    int32_t* __restrict__ keys, int32_t* __restrict__ occ) {
    constexpr int G = D / 4, GPB = kBlk / G;
    const int li = threadIdx.x % G;
    const int64_t L = 3 * cap + 1, n_trip = (int64_t)W * cap;
    const int64_t b0 = ((int64_t)blockIdx.x * GPB + threadIdx.x / G) * TPG;  // triplet slots r cap + t
    int64_t bg = 0;
    for (int r = 0; r < W; ++r) bg += slots[(int64_t)r * L];
    int64_t ru[TPG], rp[TPG], rn[TPG];
#pragma unroll
    for (int k = 0; k < TPG; ++k) {
        ru[k] = -1;
        const int64_t b = b0 + k;
        if (b < n_trip) {
            const int64_t r = b / cap, t = b - r * cap;
            const int64_t* slot = slots + r * L;
            if (t < slot[0]) {
                ru[k] = slot[1 + t];
                rp[k] = n_users + slot[1 + cap + t];
                rn[k] = n_users + slot[1 + 2 * cap + t];
            }
        }
    }
    float4 fu[TPG], fp[TPG], fn[TPG], eu[TPG], ep[TPG], en[TPG];
#pragma unroll
    for (int k = 0; k < TPG; ++k) {
        if (ru[k] >= 0) {
            fu[k] = ld4(fin + ru[k] * D + li * 4);
            fp[k] = ld4(fin + rp[k] * D + li * 4);
            fn[k] = ld4(fin + rn[k] * D + li * 4);
            eu[k] = ld4(ego + ru[k] * D + li * 4);
            ep[k] = ld4(ego + rp[k] * D + li * 4);
            en[k] = ld4(ego + rn[k] * D + li * 4);
        } else {
            fu[k] = fp[k] = fn[k] = eu[k] = ep[k] = en[k] = f4(0.f);
        }
    }
    if (keys && li < 3) {  // one real rank: dp_scatter's places, taken here (lanes 0..2: u, p, n)
#pragma unroll
        for (int k = 0; k < TPG; ++k) {
            if (ru[k] < 0) continue;
            const int64_t b = b0 + k, r = b / cap, t = b - r * cap;
            const int64_t x = li == 0 ? ru[k] : li == 1 ? rp[k] : rn[k];
            const int32_t q = start[x] - 1 + atomicAdd(cursor + x, 1);
            keys[q] = (int32_t)x;
            occ[q] = (int32_t)(r * 3 * cap + li * cap + t);
        }
    }
    double t_loss = 0.0, t_u = 0.0, t_p = 0.0, t_n = 0.0;
    float t_max = 0.f;
#pragma unroll
    for (int k = 0; k < TPG; ++k) {
        const int64_t b = b0 + k;
        if (b >= n_trip) break;  // (group-uniform)
        if (ru[k] < 0) {
            if (li == 0) coef[b] = 0.f;
            continue;
        }
        const float sp = group_sum<G>(dot4(fu[k], fp[k])), sn = group_sum<G>(dot4(fu[k], fn[k]));
        const float delta = sp - sn;
        const float sg = 1.f / (1.f + expf(-delta));
        const float term = -logf(1e-10f + sg);
        const float c = -(sg * (1.f - sg)) / (1e-10f + sg) / (float)bg;
        if (li == 0) {
            coef[b] = c;
            t_loss += (double)term;
        }
        t_u += (double)dot4(eu[k], eu[k]);
        t_p += (double)dot4(ep[k], ep[k]);
        t_n += (double)dot4(en[k], en[k]);
        const float m0 = fmaxf(fmaxf(fabsf(fu[k].x), fabsf(fu[k].y)), fmaxf(fabsf(fu[k].z), fabsf(fu[k].w)));
        const float m1 = fmaxf(fmaxf(fabsf(fp[k].x), fabsf(fp[k].y)), fmaxf(fabsf(fp[k].z), fabsf(fp[k].w)));
        const float m2 = fmaxf(fmaxf(fabsf(fn[k].x), fabsf(fn[k].y)), fmaxf(fabsf(fn[k].z), fabsf(fn[k].w)));
        float m = fmaxf(m0, fmaxf(m1, m2));
        if (m != m) m = __builtin_huge_valf();  // NaN rows: the scale's clamp below
        t_max = fmaxf(t_max, m);
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        t_loss += __shfl_xor(t_loss, o, kWave);
        t_u += __shfl_xor(t_u, o, kWave);
        t_p += __shfl_xor(t_p, o, kWave);
        t_n += __shfl_xor(t_n, o, kWave);
        t_max = fmaxf(t_max, __shfl_xor(t_max, o, kWave));
    }
    constexpr int NW = kBlk / kWave;
    __shared__ double red[NW][5];
    const int wv = threadIdx.x / kWave;
    if (threadIdx.x % kWave == 0) {
        red[wv][0] = t_loss;
        red[wv][1] = t_u;
        red[wv][2] = t_p;
        red[wv][3] = t_n;
        red[wv][4] = (double)t_max;
    }
    __syncthreads();
    __shared__ int last;
    if (threadIdx.x < 5) {
        double v = 0.0;
        for (int w = 0; w < NW; ++w) v = threadIdx.x == 4 ? fmax(v, red[w][4]) : v + red[w][threadIdx.x];
        __hip_atomic_store(part + (int64_t)blockIdx.x * 5 + threadIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the partials are stored and read sc1 (agent-scope atomics: write-through, L1 bypassed),
    // so the hand-off needs no L2 write-back fence per block (MI355X_MICROARCH.md, valid
    // forms: sc1 stores drained by vmcnt(0) before the counter add, sc1 loads by the last)
    if (threadIdx.x < 5) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the storing lanes (one wave)
    __syncthreads();
    if (threadIdx.x == 0) {
        const int prev = __hip_atomic_fetch_add(meta, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == (int)gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    // the last block: a fixed-order reduction of the per-block partials (every rank the same):
    // thread t sums blocks t, t + kBlk, ... in that order (kU of them loaded at once), then a
    // fixed shuffle tree per wave and the waves in order
    constexpr int kU = 4;
    double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    const int nb = (int)gridDim.x;
    for (int k0 = threadIdx.x; k0 < nb; k0 += kU * kBlk) {
        double v[kU][5];
#pragma unroll
        for (int j = 0; j < kU; ++j) {
            const int k = k0 + j * kBlk;
            const double* q = part + (int64_t)(k < nb ? k : 0) * 5;
#pragma unroll
            for (int c = 0; c < 5; ++c) v[j][c] = __hip_atomic_load(q + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int j = 0; j < kU; ++j) {
            if (k0 + j * kBlk >= nb) break;
#pragma unroll
            for (int c = 0; c < 4; ++c) s[c] += v[j][c];
            s[4] = fmax(s[4], v[j][4]);
        }
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
#pragma unroll
        for (int c = 0; c < 4; ++c) s[c] += __shfl_xor(s[c], o, kWave);
        s[4] = fmax(s[4], __shfl_xor(s[4], o, kWave));
    }
    __shared__ double tr[NW][5];
    if (threadIdx.x % kWave == 0) {
#pragma unroll
        for (int c = 0; c < 5; ++c) tr[wv][c] = s[c];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double r[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
        for (int w = 0; w < NW; ++w) {
            for (int c = 0; c < 4; ++c) r[c] += tr[w][c];
            r[4] = fmax(r[4], tr[w][4]);
        }
        const double B = (double)bg;
        const double nu = sqrt(r[1]), np = sqrt(r[2]), nn = sqrt(r[3]);
        const double loss = r[0] / B + (double)reg * (nu + np + nn) / B;
        float* k = reinterpret_cast<float*>(reg_cnt + 3 * N + 1);
        k[0] = nu > 0 ? (float)((double)reg / (B * nu)) : 0.f;
        k[1] = np > 0 ? (float)((double)reg / (B * np)) : 0.f;
        k[2] = nn > 0 ? (float)((double)reg / (B * nn)) : 0.f;
        if (loss_out) loss_out[0] = (float)loss;
        if (loss_acc) loss_acc[0] += loss;
        if (halt && loss != loss && halt[0] == 0) {
            halt[1] = *tag_dev;
            halt[0] = 1;
        }
        // |G'(x)| <= (3 B occurrences) * (2 max|f| / B) / g_div: the fixed-point scale 2^e keeps
        // every accumulated row below 2^61 (NaN / inf rows: e = 0, the halt flag stops Adam)
        const double bound = 6.0 * r[4] / (double)g_div;
        int e = 0;
        if (bound > 0.0 && bound < 1e300) e = 61 - (int)ceil(log2(bound));
        else if (bound == 0.0) e = 61;
        meta[1] = e < 0 ? 0 : (e > 900 ? 900 : e);
        meta[0] = 0;  // re-armed for the next launch (stream order)
    }
}

// Phase B: G' in fixed point.  Lane group c takes run places [c CH, (c+1) CH) (CH = 16 on a
// large global batch, 4 on a small one: four times the waves where there are few):
// each occurrence's term (bpr_fused's f32 arithmetic: coef (f_p - f_n) / g_div for a user,
// +-coef f_u / g_div for an item) scaled by 2^e and rounded to int64, the terms of a run
// segment summed in registers.  A run that lies wholly in the chunk (most rows occur once
// or a few times) is finished here: its sum scaled back and rounded to f32 once, stored
// as G' -- no atomics; only a run crossing a chunk boundary adds its segments into the
// int64 accumulators (integer adds commute: any order gives the same bits), which
// dp_bpr_round then finishes.  The chunk's bookkeeping (place -> occurrence -> triplet ->
// the rows to gather, the coefficient, the run's first place and length: dependent
// loads) is resolved by the group's lanes for all its places at once (lane q holds place
// q's) and broadcast by shuffles, and every gather of the chunk is issued before the first
// store or atomic (gfx9 counts loads, stores and atomics in one vmcnt: a load issued
// after them would wait for them).  (The per-run atomics of the previous form, one per
// run and column, cost ~50 us at W = 8.)
template <int D, int CH>
__global__ __launch_bounds__(kBlk) void dp_bpr_grad(const int64_t* __restrict__ slots, int64_t cap, int64_t n_users,
                                                    int64_t N, int64_t n_occ, const int32_t* __restrict__ key,
                                                    const int32_t* __restrict__ val,
                                                    const int32_t* __restrict__ start,
                                                    const int32_t* __restrict__ cursor, const float* __restrict__ fin,
                                                    const float* __restrict__ coef, float g_div, float g_inv,
                                                    const int32_t* __restrict__ meta,
                                                    unsigned long long* __restrict__ acc, float* __restrict__ gout) {
    constexpr int G = D / 4, GPB = kBlk / G;
    constexpr int KP = (CH + G - 1) / G;  // places whose bookkeeping one lane holds
    const int li = threadIdx.x % G;
    const int gl0 = (threadIdx.x % kWave) - li;  // the group's first lane in the wave
    const int64_t c0 = ((int64_t)blockIdx.x * GPB + threadIdx.x / G) * CH;
    const int64_t n_pl = meta[2] < n_occ ? meta[2] : n_occ;  // the run places taken this step
    if (c0 >= n_pl) return;  // group-uniform
    const double S = ldexp(1.0, meta[1]), inv = ldexp(1.0, -meta[1]);
    const int64_t L = 3 * cap + 1;
    // bookkeeping of place c0 + q, q = li + G k: its row (N: none), the rows it gathers
    // (b = -1 when only one), its signed coefficient, its run's first place and length
    int32_t xq[KP], sq[KP], nq[KP];
    int64_t aq[KP], bq[KP];
    float cq[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) {
        const int q = li + G * k;
        const int64_t i = c0 + q;
        xq[k] = (int32_t)N;
        sq[k] = nq[k] = 0;
        aq[k] = bq[k] = -1;
        cq[k] = 0.f;
        if (q < CH && i < n_pl) {
            const int32_t x = key[i];
            const int64_t o = val[i];
            const int64_t r = o / (3 * cap), j = o - r * 3 * cap, kind = j / cap, t = j - kind * cap;
            const int64_t* slot = slots + r * L;
            const float c = coef[r * cap + t];
            xq[k] = x;
            sq[k] = start[x] - 1;
            nq[k] = cursor[x];
            if (kind == 0) {
                aq[k] = n_users + slot[1 + cap + t];
                bq[k] = n_users + slot[1 + 2 * cap + t];
                cq[k] = c;
            } else {
                aq[k] = slot[1 + t];
                cq[k] = kind == 1 ? c : -c;
            }
        }
    }
    int32_t xs[CH], ss[CH], ns[CH];
    float cs[CH];
    bool two[CH];
    float4 va[CH], vb[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
        const int src = gl0 + u % G, k = u / G;
        xs[u] = __shfl(xq[k], src, kWave);
        ss[u] = __shfl(sq[k], src, kWave);
        ns[u] = __shfl(nq[k], src, kWave);
        cs[u] = __shfl(cq[k], src, kWave);
        const int64_t ra = __shfl(aq[k], src, kWave), rb = __shfl(bq[k], src, kWave);
        two[u] = rb >= 0;
        va[u] = ra >= 0 ? ld4(fin + ra * D + li * 4) : f4(0.f);
        vb[u] = rb >= 0 ? ld4(fin + rb * D + li * 4) : f4(0.f);
    }
    long long a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    int32_t cur = -1, seg0 = 0, segn = 0, cur_s = 0, cur_n = 0;
    auto flush = [&]() __attribute__((always_inline)) {
        if (cur < 0) return;
        if (seg0 == cur_s && segn == cur_n) {  // the whole run: G' here, rounded once
            float4 v;
            v.x = (float)((double)a0 * inv);
            v.y = (float)((double)a1 * inv);
            v.z = (float)((double)a2 * inv);
            v.w = (float)((double)a3 * inv);
            st4(gout + (int64_t)cur * D + li * 4, v);
        } else {
            unsigned long long* q = acc + (int64_t)cur * D + li * 4;
            atomicAdd(q + 0, (unsigned long long)a0);
            atomicAdd(q + 1, (unsigned long long)a1);
            atomicAdd(q + 2, (unsigned long long)a2);
            atomicAdd(q + 3, (unsigned long long)a3);
        }
    };
#pragma unroll
    for (int u = 0; u < CH; ++u) {
        const int32_t x = xs[u];
        if (x >= N) break;  // past the places taken (group-uniform)
        if (x != cur) {
            flush();
            cur = x;
            seg0 = (int32_t)(c0 + u);
            segn = 0;
            cur_s = ss[u];
            cur_n = ns[u];
            a0 = a1 = a2 = a3 = 0;
        }
        ++segn;
        const float c = cs[u];
        float4 g;
        if (two[u]) {
            g = make_float4(c * (va[u].x - vb[u].x), c * (va[u].y - vb[u].y), c * (va[u].z - vb[u].z),
                            c * (va[u].w - vb[u].w));
        } else {
            g = make_float4(c * va[u].x, c * va[u].y, c * va[u].z, c * va[u].w);
        }
        if (g_inv != 0.f) {  // g_div a power of two: x * 2^-k is x / 2^k rounded the same way
            g.x *= g_inv;
            g.y *= g_inv;
            g.z *= g_inv;
            g.w *= g_inv;
        } else if (g_div != 1.f) {
            g.x /= g_div;
            g.y /= g_div;
            g.z /= g_div;
            g.w /= g_div;
        }
        a0 += llrint((double)g.x * S);
        a1 += llrint((double)g.y * S);
        a2 += llrint((double)g.z * S);
        a3 += llrint((double)g.w * S);
    }
    flush();
}

// Phase C: every union row once (the first place of its run): a run that crossed a chunk
// boundary gets G'[x] = its accumulator / 2^e rounded to f32 and the accumulator cleared;
// every run's start and cursor are cleared for the next step.
template <int D>
__global__ __launch_bounds__(kBlk) void dp_bpr_round(int64_t n_occ, int32_t chunk, const int32_t* __restrict__ key,
                                                     int32_t* __restrict__ start, int32_t* __restrict__ cursor,
                                                     const int32_t* __restrict__ meta,
                                                     unsigned long long* __restrict__ acc, float* __restrict__ g) {
    constexpr int G = D / 4, GPB = kBlk / G;
    const int li = threadIdx.x % G;
    const int64_t i = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
    const int64_t n_pl = meta[2] < n_occ ? meta[2] : n_occ;
    if (i >= n_pl) return;
    const int32_t x = key[i];
    if (start[x] - 1 != i) return;  // (a first place clears start[x] below: the others then see 0)
    const int32_t n = cursor[x];
    if (i / chunk != (i + n - 1) / chunk) {  // finished by dp_bpr_grad otherwise
        const double inv = ldexp(1.0, -meta[1]);
        unsigned long long* q = acc + (int64_t)x * D + li * 4;
        float4 v;
        v.x = (float)((double)(long long)q[0] * inv);
        v.y = (float)((double)(long long)q[1] * inv);
        v.z = (float)((double)(long long)q[2] * inv);
        v.w = (float)((double)(long long)q[3] * inv);
        q[0] = 0ull;
        q[1] = 0ull;
        q[2] = 0ull;
        q[3] = 0ull;
        st4(g + (int64_t)x * D + li * 4, v);
    }
    if (li == 0) {
        start[x] = 0;
        cursor[x] = 0;
    }
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

template <int D>
int dp_loss_kernels(const rsx_dp_lgcn_step& st, const Work& w, int32_t W, bool places, hipStream_t s) {
    constexpr int GPB = kBlk / (D / 4);
    const int64_t nu = st.n_users, N = st.n_users + st.n_items, cap = st.cap;
    const int64_t n_trip = (int64_t)W * cap, n_occ = (int64_t)W * 3 * cap;
    const float g_div = (float)(st.n_layers + 1);
    int g_exp = 0;
    const float g_inv = std::frexp(g_div, &g_exp) == 0.5f ? std::ldexp(1.f, 1 - g_exp) : 0.f;  // 1 / g_div if 2^k
    // a smaller global batch takes narrower groups: the passes are chains of dependent
    // loads, and there the waves, not the issue, are few.  Measured latency-injected at
    // B = 2048 (profiles/r05/dp/groups/): W = 1, 2 best at 1 triplet / 4 run places a
    // group, W = 4 at 2 / 8 (0.2040 against 0.2114 ms a step wide), W = 8 at 4 / 16.
    // (RSX_DP_GROUPS: 0 by the batch, 1 narrow, 2 wide, 3 middle -- for the tests of each
    // form; RSX_DP_TPG / RSX_DP_CH: 1, 2, 4 triplets / 4, 8, 16 run places, for timing)
    static const int groups = env_knob("RSX_DP_GROUPS", 0, 0, 3);
    static const int tpg_knob = env_knob("RSX_DP_TPG", 0, 0, 4), ch_knob = env_knob("RSX_DP_CH", 0, 0, 16);
    const int form = groups ? groups : n_trip >= 16384 ? 2 : n_trip >= 8192 ? 3 : 1;
    int tpg = form == 2 ? 4 : form == 3 ? 2 : 1, ch = form == 2 ? 16 : form == 3 ? 8 : 4;
    if (tpg_knob == 1 || tpg_knob == 2 || tpg_knob == 4) tpg = tpg_knob;
    if (ch_knob == 4 || ch_knob == 8 || ch_knob == 16) ch = ch_knob;
    const int nb_a = (int)((n_trip + GPB * tpg - 1) / (GPB * tpg));
#define DP_COEF(T)                                                                                                   \
    hipLaunchKernelGGL((dp_bpr_coef<D, T>), dim3(nb_a), dim3(kBlk), 0, s, st.slots, W, cap, nu, N, st.final_emb, st.p, \
                       g_div, st.reg, w.coef, w.part, w.meta, st.reg_cnt, st.loss_out, st.loss_acc, st.halt, st.tag_dev, \
                       w.start, w.cursor, places ? w.keys : nullptr, w.occ)
    if (tpg == 4) DP_COEF(4);
    else if (tpg == 2) DP_COEF(2);
    else DP_COEF(1);
#undef DP_COEF
    DP_TRY(last_rc());
    const dim3 gg((unsigned)(((n_occ + ch - 1) / ch + GPB - 1) / GPB));
#define DP_GRAD(C)                                                                                                   \
    hipLaunchKernelGGL((dp_bpr_grad<D, C>), gg, dim3(kBlk), 0, s, st.slots, cap, nu, N, n_occ, w.keys, w.occ, w.start, \
                       w.cursor, st.final_emb, w.coef, g_div, g_inv, w.meta, w.acc, st.g)
    if (ch == 16) DP_GRAD(16);
    else if (ch == 8) DP_GRAD(8);
    else DP_GRAD(4);
#undef DP_GRAD
    DP_TRY(last_rc());
    hipLaunchKernelGGL((dp_bpr_round<D>), dim3((unsigned)((n_occ + GPB - 1) / GPB)), dim3(kBlk), 0, s, n_occ, ch,
                       w.keys, w.start, w.cursor, w.meta, w.acc, st.g);
    return last_rc();
}

int dp_step(const rsx_dp_lgcn_step& st, hipStream_t s) {
    const rsx_csr& A = *st.adj;
    const int d = st.d, K = st.n_layers;
    const int64_t nu = st.n_users, N = st.n_users + st.n_items, cap = st.cap, B = st.batch;
    // over a latency-injected communicator (rsx_comm_init_sim) the one rank times rank 0 of a
    // W-rank job: slots hold W ranks (the caller fills the other ranks' triplets), so the
    // index, sort, loss and backward see the job's global batch; the stand-in all-gather is
    // given its whole W-slot buffer (the sim's byte count is the buffer's) and moves (W-1)/W
    // of it, as one rank of the job does
    const int32_t sim_w = comm_sim_world(st.comm);
    const int32_t W = sim_w > 0 ? sim_w : comm_world(st.comm), rank = comm_rank(st.comm);
    const int64_t L = 3 * cap + 1, n_occ = (int64_t)W * 3 * cap;
    const int64_t ag = sim_w > 0 ? W : 1;  // all-gather count multiplier (sim: the whole buffer)
    Work w = carve(st.work, N, d, cap, W);
    if (w.total > st.work_bytes) return RSX_ERR_WORKSPACE;
    int rc = 0;
    // (1) on the comm stream, while the forward runs: this rank's triplets into its slot,
    // every rank's gathered, then indexed (union tags, global counts) and bucketed by row.
    // The forward's first launch depends on nothing of this step (in a replayed graph a
    // dependency across queues costs ~10 us: the slot pack used to sit ahead of it on the
    // compute stream)
    hipStream_t cs = comm_stream(st.comm, s);
    // one real rank: the branch has nothing worth three cross-queue operations to overlap
    // with (the fork and the two joins idle the compute queue ~20 us, §6.1), so it runs in
    // line on the compute stream, the all-gather of one slot is the slot itself, the pack
    // indexes what it packs (dp_pack_index), and the loss pass takes the run places
    // (dp_bpr_coef; RSX_DP_SOLO=0 keeps the forked branch, for timing)
    static const int solo_knob = env_knob("RSX_DP_SOLO", 1, 0, 1);
    const bool solo = solo_knob && sim_w <= 0 && W == 1;
    if (solo) cs = s;
    // (RSX_DP_PLACES_IN_LOSS=1: the loss pass takes the run places at W > 1 too, for timing)
    static const int places_knob = env_knob("RSX_DP_PLACES_IN_LOSS", 0, 0, 1);
    const bool places = solo || places_knob;
    hipEvent_t fork = nullptr;
    if (cs != s) {
        fork = comm_event(st.comm);
        DP_TRY(hip_rc(hipEventRecord(fork, s)));
    }
    // (2) forward: E^1..E^{K-1} stored -- issued first, so that the GPU starts them while the
    // host issues the comm branch (its RCCL call among them): a forward issued after the
    // branch started ~6 us after the previous step's last kernel at one rank
    float* layers[3] = {st.h0, st.h1, st.s};
    const float* x = st.p;
    for (int k = 1; k < K; ++k) {
        rsx_epilogue e = epi(RSX_EPI_STORE);
        e.y = layers[k - 1];
        DP_TRY(spmm_dispatch(A, x, d, e, st.slab, s));
        x = layers[k - 1];
    }
    if (fork) DP_TRY(hip_rc(hipStreamWaitEvent(cs, fork, 0)));
    int64_t* const step_dev = st.inc_step ? const_cast<int64_t*>(st.adam.step_dev) : nullptr;
    const dim3 go((unsigned)((n_occ + kBlk - 1) / kBlk));
    if (solo) {
        hipLaunchKernelGGL(dp_pack_index, dim3((unsigned)((L + kBlk - 1) / kBlk)), dim3(kBlk), 0, s, st.triplets, B,
                           cap, nu, st.slots, step_dev ? 1 : 0, w.meta, st.row_tag, st.reg_cnt, st.tag_dev);
        DP_TRY(last_rc());
    } else {
        hipLaunchKernelGGL(dp_pack, dim3((unsigned)((L + kBlk - 1) / kBlk)), dim3(kBlk), 0, cs, st.triplets, B, cap,
                           st.slots + rank * L, step_dev, w.meta);
        DP_TRY(last_rc());
        if (!collective(st.comm, RSX_COLL_ALLGATHER, st.slots, L * ag, RSX_COLL_I64, cs, &rc)) return rc;
        hipLaunchKernelGGL(dp_index, go, dim3(kBlk), 0, cs, st.slots, W, cap, nu, st.row_tag, st.reg_cnt, st.tag_dev);
        DP_TRY(last_rc());
    }
    hipEvent_t j_idx = nullptr, j_sort = nullptr;
    if (cs != s) {
        j_idx = comm_event(st.comm);
        DP_TRY(hip_rc(hipEventRecord(j_idx, cs)));
    }
    hipLaunchKernelGGL(dp_alloc, go, dim3(kBlk), 0, cs, st.slots, W, cap, nu, st.reg_cnt, w.start, w.meta,
                       solo ? step_dev : nullptr);
    DP_TRY(last_rc());
    if (!places) {  // (one real rank: dp_bpr_coef takes the places)
        hipLaunchKernelGGL(dp_scatter, go, dim3(kBlk), 0, cs, st.slots, W, cap, nu, w.start, w.cursor, w.keys,
                           w.occ);
        DP_TRY(last_rc());
    }
    if (cs != s) {
        j_sort = comm_event(st.comm);
        DP_TRY(hip_rc(hipEventRecord(j_sort, cs)));
    }
    // (2) (issued above) then the last layer and the mean on the union rows only
    if (j_idx) DP_TRY(hip_rc(hipStreamWaitEvent(s, j_idx, 0)));  // the union tags
    {
        rsx_epilogue e = epi(RSX_EPI_FINAL);
        e.beta = 1.f / (float)(K + 1);
        e.f = st.final_emb;
        e.s_in = st.p;
        e.r_add = st.h0;
        e.aux = K >= 3 ? st.h1 : nullptr;
        e.e0 = K == 4 ? st.s : nullptr;
        e.row_tag = st.row_tag;
        e.tag_dev = st.tag_dev;
        e.tag_flags = RSX_TAG_ROWS;
        DP_TRY(spmm_dispatch(A, x, d, e, st.slab, s));
    }
    // (3) the global batch's loss and G' = dL/dfinal / (K+1) on every rank
    if (j_sort) DP_TRY(hip_rc(hipStreamWaitEvent(s, j_sort, 0)));
    switch (d) {
        case 32: DP_TRY(dp_loss_kernels<32>(st, w, W, places, s)); break;
        case 64: DP_TRY(dp_loss_kernels<64>(st, w, W, places, s)); break;
        case 128: DP_TRY(dp_loss_kernels<128>(st, w, W, places, s)); break;
        case 256: DP_TRY(dp_loss_kernels<256>(st, w, W, places, s)); break;
        default: return RSX_ERR_UNSUPPORTED;
    }
    // (4) backward on the union rows: H = G' + A H from H = G', Adam on g = H^K + R with the
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
        !st->g || !st->triplets || !st->row_tag || !st->tag_dev || !st->reg_cnt || !st->slots || !st->work)
        return false;
    if (st->n_layers < 2 || st->n_layers > 4 || (st->n_layers == 4 && !st->s)) return false;
    if (st->batch <= 0 || st->batch > st->cap || st->n_users < 0 || st->n_items <= 0) return false;
    if (st->adj->n_rows != st->n_users + st->n_items || st->adj->n_cols != st->adj->n_rows) return false;
    if (st->adj->n_long > 0 && !st->slab) return false;
    if (st->n_users + st->n_items >= 0x7fffffffll) return false;  // int32 sort keys
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
    const int32_t sim_w = rsx::comm_sim_world(st->comm);
    const int64_t W = sim_w > 0 ? sim_w : rsx::comm_world(st->comm);
    if (W * 3 * st->cap >= 0x7fffffffll) return RSX_ERR_ARG;  // int32 occurrence ids
    return rsx::dp_step(*st, rsx::as_stream(stream));
}

size_t rsx_dp_work_bytes(int64_t n_rows, int32_t d, int64_t cap, int32_t world) {
    if (n_rows <= 0 || d <= 0 || cap <= 0 || world < 1) return 0;
    return rsx::carve(nullptr, n_rows, d, cap, world).total;
}

}  // extern "C"

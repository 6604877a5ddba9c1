// bpr.hip — fused BPR triplet loss forward + backward (gfx950).
//
// Replaces, per model variant, the gather / dot / logsigmoid / regulariser ops
// and their autograd backward:
//   LightGCN  src/models/lightgcn.py:132-156 + src/common/loss.py:33-51
//   LayerGCN  src/models/layergcn.py:142-177 + src/common/loss.py:58-61
//   SMORE     src/models/smore.py:366-378 (BPR part; InfoNCE is separate)
//
// Two launches: (A) one lane group per triplet computes s+, s-, the per-triplet
// loss term and dL/d(s+ - s-), plus per-block partial sums of the regulariser's
// squared norms (deterministic, f64); (B) every block re-reduces those partials
// in a fixed order (the LightGCN regulariser needs the global Frobenius norms
// before any gradient row is known) and scatters gradient rows with f32
// atomics.  Lane li of a group owns columns {li + c*G}, so each atomic
// wave-instruction adds G contiguous floats of a row.
#include "rsx_common.hpp"

namespace rsx {

constexpr int kBprBlock = 256;

struct BprArgs {
    int variant;
    int rows;        // RSX_BPR_SMORE_ROWS: every g_fin row is written by one triplet (stored, not added)
    const float* fin;
    const float* ego;
    int64_t n_users, n_items;
    const int64_t* trip;
    int64_t batch;
    float reg, batch_cfg;
    float g_div;     // LightGCN: dL/dfinal is divided by this (K+1: the mean's backward), 1 = none
    float* g_fin;
    float* g_ego;
    float* loss_out;
    double* loss_acc;
    float* coef;     // [batch]
    double* part;    // [n_blocks][4]
    int32_t* reg_cnt;  // bpr_fused: [n_rows][3] occurrence counts + [4] tail (done counter, ku, kp, kn)
    int64_t n_rows;
    int32_t* halt;     // bpr_fused (optional): [2] set to {1, tag} by the first NaN loss
    int32_t tag;
    // bpr_fused, data-parallel form (dp_tot != NULL): the loss is the mean over the GLOBAL
    // batch, B_glob = the sum of every rank's count in the gathered triplet slots
    // (dp_slots[r * dp_slot_len], r < dp_world); no occurrence counts are written (the
    // merge counts every rank's triplets) and the last block stores this rank's four f64
    // totals (loss terms, |U|^2, |P|^2, |N|^2) at dp_tot instead of finishing the loss
    const int64_t* dp_slots;
    int64_t dp_slot_len;
    int32_t dp_world;
    double* dp_tot;
};

__device__ __forceinline__ float softplus_neg(float x) {
    // -logsigmoid(x) = log(1 + exp(-x)), computed stably
    return x >= 0.f ? log1pf(expf(-x)) : -x + log1pf(expf(x));
}
__device__ __forceinline__ float sigmoidf(float x) { return 1.f / (1.f + expf(-x)); }

template <int D>
__global__ __launch_bounds__(kBprBlock) void bpr_fwd(BprArgs a) {
    constexpr int G = D / 4;
    constexpr int GPB = kBprBlock / G;
    constexpr int NC = D / G;  // columns per lane (=4)
    const int li = threadIdx.x % G;
    const int64_t b = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
    double t_loss = 0.0, t_u = 0.0, t_p = 0.0, t_n = 0.0;
    if (b < a.batch) {
        const int64_t u = a.trip[b];
        const int64_t p = a.trip[a.batch + b] + a.n_users;
        const int64_t n = a.trip[2 * a.batch + b] + a.n_users;
        float fu[NC], fp[NC], fn[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            fu[c] = a.fin[u * D + li + c * G];
            fp[c] = a.fin[p * D + li + c * G];
            fn[c] = a.fin[n * D + li + c * G];
        }
        float sp = 0.f, sn = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            sp += fu[c] * fp[c];
            sn += fu[c] * fn[c];
        }
        sp = group_sum<G>(sp);
        sn = group_sum<G>(sn);
        const float delta = sp - sn;
        float term, coef;
        if (a.variant == RSX_BPR_LIGHTGCN) {
            // -log(1e-10 + sigmoid(delta)), mean over the batch
            const float sg = sigmoidf(delta);
            term = -logf(1e-10f + sg);
            coef = -(sg * (1.f - sg)) / (1e-10f + sg) / (float)a.batch;
        } else if (a.variant == RSX_BPR_LAYERGCN) {
            term = softplus_neg(delta);          // sum over the batch
            coef = -sigmoidf(-delta);
        } else {
            term = softplus_neg(delta);          // mean over the batch
            coef = -sigmoidf(-delta) / (float)a.batch;
        }
        // compact rows: bpr_bwd STORES each triplet's three gradient rows, which is only
        // race-free (and complete) for the layout (b, b, B + b). Any other triplets poison
        // the loss with NaN, so the NaN halt stops the step instead of leaving racing or
        // unwritten rows in g_final
        if (a.rows && (u != b || a.trip[a.batch + b] != b || a.trip[2 * a.batch + b] != a.batch + b))
            term = __builtin_nanf("");
        // squared norms for the regulariser
        float qu = 0.f, qp = 0.f, qn = 0.f;
        if (a.variant == RSX_BPR_SMORE) {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                qu += fu[c] * fu[c];
                qp += fp[c] * fp[c];
                qn += fn[c] * fn[c];
            }
        } else {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const float eu = a.ego[u * D + li + c * G];
                const float ep = a.ego[p * D + li + c * G];
                const float en = a.ego[n * D + li + c * G];
                qu += eu * eu;
                qp += ep * ep;
                qn += en * en;
            }
        }
        t_u = (double)qu;  // per-lane partials; summed across the block below
        t_p = (double)qp;
        t_n = (double)qn;
        if (li == 0) {
            a.coef[b] = coef;
            t_loss = (double)term;
        }
    }
    // block reduction (fixed order: wave shuffles, then waves in order)
    __shared__ double red[kBprBlock / kWave][4];
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        t_loss += __shfl_xor(t_loss, o, kWave);
        t_u += __shfl_xor(t_u, o, kWave);
        t_p += __shfl_xor(t_p, o, kWave);
        t_n += __shfl_xor(t_n, o, kWave);
    }
    const int wv = threadIdx.x / kWave;
    if ((threadIdx.x % kWave) == 0) {
        red[wv][0] = t_loss;
        red[wv][1] = t_u;
        red[wv][2] = t_p;
        red[wv][3] = t_n;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        double s = 0.0;
        for (int w = 0; w < kBprBlock / kWave; ++w) s += red[w][threadIdx.x];
        a.part[(int64_t)blockIdx.x * 4 + threadIdx.x] = s;
    }
}

template <int D>
__global__ __launch_bounds__(kBprBlock) void bpr_bwd(BprArgs a, int n_part) {
    constexpr int G = D / 4;
    constexpr int GPB = kBprBlock / G;
    constexpr int NC = D / G;
    // every block reduces the per-block partials in the same fixed order
    // (thread t sums partials t, t+256, ...; then a fixed-shape tree)
    __shared__ double red[4][kBprBlock];
    __shared__ double tot[4];
    {
        double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
        for (int k = threadIdx.x; k < n_part; k += kBprBlock) {
            const double4 v = reinterpret_cast<const double4*>(a.part)[k];
            s0 += v.x;
            s1 += v.y;
            s2 += v.z;
            s3 += v.w;
        }
        red[0][threadIdx.x] = s0;
        red[1][threadIdx.x] = s1;
        red[2][threadIdx.x] = s2;
        red[3][threadIdx.x] = s3;
        __syncthreads();
        for (int w = kBprBlock / 2; w > 0; w >>= 1) {
            if (threadIdx.x < w) {
#pragma unroll
                for (int c = 0; c < 4; ++c) red[c][threadIdx.x] += red[c][threadIdx.x + w];
            }
            __syncthreads();
        }
        if (threadIdx.x < 4) tot[threadIdx.x] = red[threadIdx.x][0];
        __syncthreads();
    }
    const double B = (double)a.batch;
    double loss;
    float ku, kp, kn;  // regulariser gradient scale per row kind
    if (a.variant == RSX_BPR_LIGHTGCN) {
        const double nu = sqrt(tot[1]), np = sqrt(tot[2]), nn = sqrt(tot[3]);
        loss = tot[0] / B + (double)a.reg * (nu + np + nn) / B;
        ku = nu > 0 ? (float)((double)a.reg / (B * nu)) : 0.f;
        kp = np > 0 ? (float)((double)a.reg / (B * np)) : 0.f;
        kn = nn > 0 ? (float)((double)a.reg / (B * nn)) : 0.f;
    } else if (a.variant == RSX_BPR_LAYERGCN) {
        loss = tot[0] + (double)a.reg * 0.5 * (tot[1] + tot[2] + tot[3]);
        ku = kp = kn = a.reg;
    } else {
        loss = tot[0] / B + (double)a.reg * 0.5 * (tot[1] + tot[2] + tot[3]) / (double)a.batch_cfg;
        ku = kp = kn = (float)((double)a.reg / (double)a.batch_cfg);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (a.loss_out) a.loss_out[0] = (float)loss;
        if (a.loss_acc) a.loss_acc[0] += loss;
        if (a.halt && loss != loss && a.halt[0] == 0) {  // the first NaN batch: later Adam layers skip
            a.halt[1] = a.tag;
            a.halt[0] = 1;
        }
    }
    const int li = threadIdx.x % G;
    const int64_t b = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
    if (b >= a.batch) return;
    const int64_t u = a.trip[b];
    const int64_t p = a.trip[a.batch + b] + a.n_users;
    const int64_t n = a.trip[2 * a.batch + b] + a.n_users;
    const float coef = a.coef[b];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int col = li + c * G;
        const float fu = a.fin[u * D + col], fp = a.fin[p * D + col], fn = a.fin[n * D + col];
        float gu = coef * (fp - fn), gp = coef * fu, gn = -coef * fu;
        if (a.g_div != 1.f) {  // gradient of each layer's share of the mean (MeanBackward: grad / n)
            gu /= a.g_div;
            gp /= a.g_div;
            gn /= a.g_div;
        }
        if (a.variant == RSX_BPR_SMORE) {
            gu += ku * fu;
            gp += kp * fp;
            gn += kn * fn;
        } else if (a.g_ego) {
            atomicAdd(a.g_ego + u * D + col, ku * a.ego[u * D + col]);
            atomicAdd(a.g_ego + p * D + col, kp * a.ego[p * D + col]);
            atomicAdd(a.g_ego + n * D + col, kn * a.ego[n * D + col]);
        }
        if (a.rows) {
            a.g_fin[u * D + col] = gu;
            a.g_fin[p * D + col] = gp;
            a.g_fin[n * D + col] = gn;
            continue;
        }
        atomicAdd(a.g_fin + u * D + col, gu);
        atomicAdd(a.g_fin + p * D + col, gp);
        atomicAdd(a.g_fin + n * D + col, gn);
    }
}

// LightGCN BPR in ONE launch (the batch-tagged step): per triplet the loss term and
// dL/dfinal rows are scattered at once (divided by g_div); the regulariser's
// gradient, which needs the batch's global Frobenius norms, is left to the
// consumer as occurrence counts per row (as user, positive, negative) and three
// scales ku, kp, kn: R[row] = (c_u ku + c_p kp + c_n kn) ego[row] (the reference
// sums c equal terms per row).  Every block stores its f64 partials (sc1); the last
// block to arrive at one counter reduces them (sc1 loads) in bpr_bwd's fixed order,
// writes the loss and the scales and re-arms the counter.
template <int D>
__global__ __launch_bounds__(kBprBlock) void bpr_fused(BprArgs a) {
    constexpr int G = D / 4;
    constexpr int GPB = kBprBlock / G;
    constexpr int NC = D / G;
    const int li = threadIdx.x % G;
    const int64_t b = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
    double t_loss = 0.0, t_u = 0.0, t_p = 0.0, t_n = 0.0;
    int64_t bdiv = a.batch;  // the mean's batch: this launch's, or the global batch (dp)
    if (a.dp_tot) {
        bdiv = 0;
        for (int r = 0; r < a.dp_world; ++r) bdiv += a.dp_slots[(int64_t)r * a.dp_slot_len];
    }
    if (b < a.batch) {
        const int64_t u = a.trip[b];
        const int64_t p = a.trip[a.batch + b] + a.n_users;
        const int64_t n = a.trip[2 * a.batch + b] + a.n_users;
        float fu[NC], fp[NC], fn[NC], eu[NC], ep[NC], en[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            fu[c] = a.fin[u * D + li + c * G];
            fp[c] = a.fin[p * D + li + c * G];
            fn[c] = a.fin[n * D + li + c * G];
            eu[c] = a.ego[u * D + li + c * G];
            ep[c] = a.ego[p * D + li + c * G];
            en[c] = a.ego[n * D + li + c * G];
        }
        float sp = 0.f, sn = 0.f, qu = 0.f, qp = 0.f, qn = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            sp += fu[c] * fp[c];
            sn += fu[c] * fn[c];
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            qu += eu[c] * eu[c];
            qp += ep[c] * ep[c];
            qn += en[c] * en[c];
        }
        sp = group_sum<G>(sp);
        sn = group_sum<G>(sn);
        const float delta = sp - sn;
        const float sg = 1.f / (1.f + expf(-delta));
        const float term = -logf(1e-10f + sg);
        const float coef = -(sg * (1.f - sg)) / (1e-10f + sg) / (float)bdiv;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int col = li + c * G;
            float gu = coef * (fp[c] - fn[c]), gp = coef * fu[c], gn = -coef * fu[c];
            if (a.g_div != 1.f) {
                gu /= a.g_div;
                gp /= a.g_div;
                gn /= a.g_div;
            }
            atomicAdd(a.g_fin + u * D + col, gu);
            atomicAdd(a.g_fin + p * D + col, gp);
            atomicAdd(a.g_fin + n * D + col, gn);
        }
        if (li == 0) {
            if (!a.dp_tot) {
                atomicAdd(a.reg_cnt + 3 * u + 0, 1);
                atomicAdd(a.reg_cnt + 3 * p + 1, 1);
                atomicAdd(a.reg_cnt + 3 * n + 2, 1);
            }
            t_loss = (double)term;
        }
        t_u = (double)qu;
        t_p = (double)qp;
        t_n = (double)qn;
    }
    __shared__ double red[kBprBlock / kWave][4];
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        t_loss += __shfl_xor(t_loss, o, kWave);
        t_u += __shfl_xor(t_u, o, kWave);
        t_p += __shfl_xor(t_p, o, kWave);
        t_n += __shfl_xor(t_n, o, kWave);
    }
    const int wv = threadIdx.x / kWave;
    if ((threadIdx.x % kWave) == 0) {
        red[wv][0] = t_loss;
        red[wv][1] = t_u;
        red[wv][2] = t_p;
        red[wv][3] = t_n;
    }
    __syncthreads();
    __shared__ int last;
    if (threadIdx.x < 4) {
        double v = 0.0;
        for (int w = 0; w < kBprBlock / kWave; ++w) v += red[w][threadIdx.x];
        __hip_atomic_store(a.part + (int64_t)blockIdx.x * 4 + threadIdx.x, v, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    // the partials are stored and read sc1 (agent-scope atomics: write-through, L1 bypassed),
    // so the hand-off needs no per-block L2 write-back fence (MI355X_MICROARCH.md, valid
    // forms: sc1 stores drained by vmcnt(0) before the counter add, sc1 loads by the last)
    if (threadIdx.x < 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the storing lanes (one wave)
    __syncthreads();
    int* done = a.reg_cnt + 3 * a.n_rows;
    if (threadIdx.x == 0) {
        const int prev = __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == (int)gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    // the last block: bpr_bwd's fixed-order reduction of the per-block partials
    __shared__ double tr[4][kBprBlock];
    {
        double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
        for (int k = threadIdx.x; k < (int)gridDim.x; k += kBprBlock) {
            const double* q = a.part + (int64_t)k * 4;
            s0 += __hip_atomic_load(q + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s1 += __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s2 += __hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s3 += __hip_atomic_load(q + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        tr[0][threadIdx.x] = s0;
        tr[1][threadIdx.x] = s1;
        tr[2][threadIdx.x] = s2;
        tr[3][threadIdx.x] = s3;
        __syncthreads();
        for (int w = kBprBlock / 2; w > 0; w >>= 1) {
            if (threadIdx.x < w) {
#pragma unroll
                for (int c = 0; c < 4; ++c) tr[c][threadIdx.x] += tr[c][threadIdx.x + w];
            }
            __syncthreads();
        }
    }
    if (a.dp_tot) {  // this rank's totals for the merge (csrc/dp.hip), which finishes the loss
        if (threadIdx.x < 4) a.dp_tot[threadIdx.x] = tr[threadIdx.x][0];
        __syncthreads();
        if (threadIdx.x == 0) *done = 0;
        return;
    }
    if (threadIdx.x == 0) {
        const double B = (double)a.batch;
        const double nu = sqrt(tr[1][0]), np = sqrt(tr[2][0]), nn = sqrt(tr[3][0]);
        const double loss = tr[0][0] / B + (double)a.reg * (nu + np + nn) / B;
        float* k = reinterpret_cast<float*>(done + 1);
        k[0] = nu > 0 ? (float)((double)a.reg / (B * nu)) : 0.f;
        k[1] = np > 0 ? (float)((double)a.reg / (B * np)) : 0.f;
        k[2] = nn > 0 ? (float)((double)a.reg / (B * nn)) : 0.f;
        if (a.loss_out) a.loss_out[0] = (float)loss;
        if (a.loss_acc) a.loss_acc[0] += loss;
        if (a.halt && loss != loss && a.halt[0] == 0) {
            a.halt[1] = a.tag;
            a.halt[0] = 1;
        }
        *done = 0;  // re-armed for the next launch (stream order)
    }
}

int bpr_fused_call(const float* fin, const float* ego, int64_t n_users, int64_t n_items, int32_t d,
                   const int64_t* trip, int64_t batch, float reg, float g_div, float* g_fin, int32_t* reg_cnt,
                   float* loss_out, double* loss_acc, void* ws, size_t ws_bytes, hipStream_t s,
                   int32_t* halt = nullptr, int32_t tag = 0);

template <int D>
static int launch_bpr(const BprArgs& a, hipStream_t s) {
    constexpr int GPB = kBprBlock / (D / 4);
    const int nb = (int)((a.batch + GPB - 1) / GPB);
    hipLaunchKernelGGL((bpr_fwd<D>), dim3(nb), dim3(kBprBlock), 0, s, a);
    hipLaunchKernelGGL((bpr_bwd<D>), dim3(nb), dim3(kBprBlock), 0, s, a, nb);
    return last_rc();
}

int bpr_dispatch(const BprArgs& a, int d, hipStream_t s) {
    switch (d) {
        case 32: return launch_bpr<32>(a, s);
        case 64: return launch_bpr<64>(a, s);
        case 128: return launch_bpr<128>(a, s);
        case 256: return launch_bpr<256>(a, s);
        default: return RSX_ERR_UNSUPPORTED;
    }
}

size_t bpr_ws(int64_t batch) {
    const int64_t nb = (batch + 3) / 4 + 1;  // worst case G = 64 lanes (d = 256): 4 triplets per block
    size_t bytes = (size_t)batch * sizeof(float);
    bytes = (bytes + 255) & ~(size_t)255;
    return bytes + (size_t)nb * 4 * sizeof(double) + 256;
}

int bpr_call(int32_t variant, const float* fin, const float* ego, int64_t n_users, int64_t n_items, int32_t d,
             const int64_t* trip, int64_t batch, float reg, float batch_cfg, float* g_fin, float* g_ego,
             float* loss_out, double* loss_acc, void* ws, size_t ws_bytes, hipStream_t s, float g_div,
             int32_t* halt, int32_t tag) {
    if (!fin || !trip || !g_fin || batch <= 0 || !ws) return RSX_ERR_ARG;
    if (variant < 0 || variant > 3) return RSX_ERR_ARG;
    const int rows = variant == RSX_BPR_SMORE_ROWS;  // SMORE's arithmetic, rows stored
    if (rows && (n_users != batch || n_items != 2 * batch)) return RSX_ERR_ARG;
    if (rows) variant = RSX_BPR_SMORE;
    if (variant != RSX_BPR_SMORE && !ego) return RSX_ERR_ARG;
    if (ws_bytes < bpr_ws(batch)) return RSX_ERR_WORKSPACE;
    BprArgs a = {};
    a.variant = variant;
    a.rows = rows;
    a.fin = fin;
    a.ego = ego;
    a.n_users = n_users;
    a.n_items = n_items;
    a.trip = trip;
    a.batch = batch;
    a.reg = reg;
    a.batch_cfg = batch_cfg;
    a.g_div = variant == RSX_BPR_LIGHTGCN ? g_div : 1.f;
    a.g_fin = g_fin;
    a.g_ego = g_ego;
    a.loss_out = loss_out;
    a.loss_acc = loss_acc;
    char* w = static_cast<char*>(ws);
    a.coef = reinterpret_cast<float*>(w);
    size_t off = ((size_t)batch * sizeof(float) + 255) & ~(size_t)255;
    a.part = reinterpret_cast<double*>(w + off);
    a.halt = halt;
    a.tag = tag;
    return bpr_dispatch(a, d, s);
}

int bpr_fused_args(const float* fin, const float* ego, int64_t n_users, int64_t n_items, int32_t d,
                   const int64_t* trip, int64_t batch, float reg, float g_div, float* g_fin, int32_t* reg_cnt,
                   float* loss_out, double* loss_acc, void* ws, size_t ws_bytes, hipStream_t s, int32_t* halt,
                   int32_t tag, const int64_t* dp_slots, int64_t dp_slot_len, int32_t dp_world, double* dp_tot) {
    if (!fin || !ego || !trip || !g_fin || !reg_cnt || batch <= 0 || !ws) return RSX_ERR_ARG;
    if (ws_bytes < bpr_ws(batch)) return RSX_ERR_WORKSPACE;
    BprArgs a = {};
    a.variant = RSX_BPR_LIGHTGCN;
    a.fin = fin;
    a.ego = ego;
    a.n_users = n_users;
    a.n_items = n_items;
    a.trip = trip;
    a.batch = batch;
    a.reg = reg;
    a.batch_cfg = (float)batch;
    a.g_div = g_div;
    a.g_fin = g_fin;
    a.loss_out = loss_out;
    a.loss_acc = loss_acc;
    char* w = static_cast<char*>(ws);
    a.coef = reinterpret_cast<float*>(w);
    a.part = reinterpret_cast<double*>(w + (((size_t)batch * sizeof(float) + 255) & ~(size_t)255));
    a.reg_cnt = reg_cnt;
    a.n_rows = n_users + n_items;
    a.halt = halt;
    a.tag = tag;
    a.dp_slots = dp_slots;
    a.dp_slot_len = dp_slot_len;
    a.dp_world = dp_world;
    a.dp_tot = dp_tot;
    switch (d) {
        case 32: hipLaunchKernelGGL((bpr_fused<32>), dim3((unsigned)((batch + 31) / 32)), dim3(kBprBlock), 0, s, a); break;
        case 64: hipLaunchKernelGGL((bpr_fused<64>), dim3((unsigned)((batch + 15) / 16)), dim3(kBprBlock), 0, s, a); break;
        case 128: hipLaunchKernelGGL((bpr_fused<128>), dim3((unsigned)((batch + 7) / 8)), dim3(kBprBlock), 0, s, a); break;
        case 256: hipLaunchKernelGGL((bpr_fused<256>), dim3((unsigned)((batch + 3) / 4)), dim3(kBprBlock), 0, s, a); break;
        default: return RSX_ERR_UNSUPPORTED;
    }
    return last_rc();
}

int bpr_fused_call(const float* fin, const float* ego, int64_t n_users, int64_t n_items, int32_t d,
                   const int64_t* trip, int64_t batch, float reg, float g_div, float* g_fin, int32_t* reg_cnt,
                   float* loss_out, double* loss_acc, void* ws, size_t ws_bytes, hipStream_t s, int32_t* halt,
                   int32_t tag) {
    return bpr_fused_args(fin, ego, n_users, n_items, d, trip, batch, reg, g_div, g_fin, reg_cnt, loss_out, loss_acc,
                          ws, ws_bytes, s, halt, tag, nullptr, 0, 0, nullptr);
}

}  // namespace rsx

extern "C" {

size_t rsx_bpr_ws_bytes(int64_t batch) { return rsx::bpr_ws(batch); }

int rsx_bpr(int32_t variant, const float* final_emb, const float* ego_emb, int64_t n_users, int64_t n_items,
            int32_t d, const int64_t* triplets, int64_t batch, float reg, float batch_cfg, float* g_final,
            float* g_ego, float* loss_out, double* loss_acc, void* ws, size_t ws_bytes, rsx_stream_t stream) {
    return rsx::bpr_call(variant, final_emb, ego_emb, n_users, n_items, d, triplets, batch, reg, batch_cfg,
                         g_final, g_ego, loss_out, loss_acc, ws, ws_bytes, rsx::as_stream(stream), 1.f, nullptr, 0);
}

}  // extern "C"

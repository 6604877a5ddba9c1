// metrics.hip — the evaluation tail of the reference on the device:
// TopKEvaluator.evaluate + utils/metrics.py (src/utils/topk_evaluator.py:58-102,
// src/utils/metrics.py:12-118) for recall, recall2, precision, ndcg and map.
//
// Kernel 1, one thread per evaluation user: hit[r] = topk[u][r] in the user's
// held-out items (binary search in a sorted per-user CSR, replacing the
// reference's Python `i in m` loop), then the per-user metric values at each
// cutoff with the reference's float64 arithmetic in its order (cumulative sums
// over ranks 1..k; the gain table 1/log2(r+1) comes from the caller, computed by
// numpy exactly as the reference does).  Values are written [n_users][M].
// Kernel 2: every column summed over users SEQUENTIALLY in user order — numpy's
// mean(axis=0) over a C-contiguous [n, k] array adds rows in order — so the sums,
// and after the caller's division and round(., 4) the metric dict, are
// bit-identical to the reference's (metrics_sum_lds: one lane per column, all
// chains in one wave from LDS tiles; metrics_sum: one wave per column, m > 64).
#include "rsx_common.hpp"

namespace rsx {

constexpr int kMetricCols = 5;  // recall, precision, ndcg, map, cumhit (recall2 numerator)

constexpr int kUserBlock = 64;  // one wave per block: 35,598 users spread over all CUs (557 blocks, not 139)
__global__ __launch_bounds__(kUserBlock) void metrics_user(const int64_t* __restrict__ topk, int64_t n, int kmax,
                                                     const int64_t* __restrict__ erp,
                                                     const int32_t* __restrict__ ecol,
                                                     const int32_t* __restrict__ cut, int n_cut,
                                                     const double* __restrict__ gain, double* __restrict__ vals) {
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= n) return;
    const int64_t b = erp[u], e = erp[u + 1];
    const int64_t pos = e - b;
    const int cap = (int)(pos < kmax ? pos : kmax);
    double cum = 0.0, dcg = 0.0, ap = 0.0, idcg_full = 0.0;
    double idcg_cap = 0.0;
    int c = 0;
    double* out = vals + u * (int64_t)(kMetricCols * n_cut);
    // hits first (k <= 64): 8 binary searches in lockstep, so a thread has 8
    // independent loads in flight per probe instead of one dependent chain per rank
    uint64_t hits = 0;
    if (kmax <= 64) {
        const int rounds = pos > 0 ? 64 - __builtin_clzll((unsigned long long)pos) : 0;
        for (int r0 = 0; r0 < kmax; r0 += 8) {
            int64_t it[8], lo[8], hi[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                it[j] = r0 + j < kmax ? topk[u * kmax + r0 + j] : -1;
                lo[j] = b;
                hi[j] = e;
            }
            for (int q = 0; q < rounds; ++q) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (lo[j] < hi[j]) {
                        const int64_t mid = (lo[j] + hi[j]) >> 1;
                        if ((int64_t)ecol[mid] < it[j]) lo[j] = mid + 1; else hi[j] = mid;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (r0 + j < kmax && lo[j] < e && (int64_t)ecol[lo[j]] == it[j]) hits |= 1ull << (r0 + j);
        }
    }
    for (int r = 0; r < kmax; ++r) {
        bool hit;
        if (kmax <= 64) {
            hit = (hits >> r) & 1ull;
        } else {
            const int64_t it = topk[u * kmax + r];
            int64_t lo = b, hi = e;
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if ((int64_t)ecol[mid] < it) lo = mid + 1; else hi = mid;
            }
            hit = lo < e && (int64_t)ecol[lo] == it;
        }
        const double rank = (double)(r + 1);
        if (hit) cum += 1.0;
        dcg += hit ? gain[r] : 0.0;                  // cumsum(where(hit, gain, 0))
        ap += (cum / rank) * (hit ? 1.0 : 0.0);      // cumsum(prec * hit)
        idcg_full += gain[r];                        // cumsum(gain)
        if (r == cap - 1) idcg_cap = idcg_full;      // ideal_full[min(k, cap) - 1]
        while (c < n_cut && cut[c] == r + 1) {
            const double idcg = (r + 1 <= cap) ? idcg_full : idcg_cap;
            const double denom = (double)((r + 1) < cap ? (r + 1) : cap);
            out[0 * n_cut + c] = cum / (double)pos;  // recall
            out[1 * n_cut + c] = cum / rank;         // precision
            out[2 * n_cut + c] = dcg / idcg;         // ndcg
            out[3 * n_cut + c] = ap / denom;         // map
            out[4 * n_cut + c] = cum;                // recall2 numerator
            ++c;
        }
    }
}

template <int T>
__device__ __forceinline__ double lane_d(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, T);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), T);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
template <int T>
__device__ __forceinline__ double add_from(double s, double x) {
    if constexpr (T == 64) {
        return s;
    } else {
        return add_from<T + 1>(s + lane_d<T>(x), x);
    }
}
// s + x[lane 0] + x[lane 1] + ... + x[lane 63], in that order (constant-lane reads)
__device__ __forceinline__ double add_lanes(double s, double x) { return add_from<0>(s, x); }

// One wavefront per column: the 64 lanes load 64 users' values at a time (the next
// chunk is loaded before this one is added), then every lane adds them in user
// order from registers (shuffles): the serial chain is adds only, no load latency.
__global__ __launch_bounds__(64) void metrics_sum(const double* __restrict__ vals, int64_t n, int m,
                                                  double* __restrict__ out) {
    const int j = blockIdx.x, lane = threadIdx.x;
    double s = 0.0;
    double cur = lane < n ? vals[(int64_t)lane * m + j] : 0.0;
    for (int64_t base = 0; base < n; base += 64) {
        const int64_t nx = base + 64 + lane;
        const double nxt = nx < n ? vals[nx * m + j] : 0.0;
        // lanes past the end hold 0.0: adding +0.0 leaves s unchanged bit for bit
        // (s is never -0.0 here: it starts at +0.0 and the values are >= 0)
        s = add_lanes(s, cur);
        cur = nxt;
    }
    if (lane == 0) out[j] = s;
}

// All columns at once, one lane per column (m <= 64): every add of a column's
// serial chain is one v_add_f64 of wave 0 on operands already in LDS, so the m
// chains advance together and the cost is one dependent add per user, not m.
// Waves 1-3 stream the next tile of [users][m] values (contiguous in `vals`) into
// the other LDS buffer meanwhile.  Same order, same bits as metrics_sum.
constexpr int kSumTileD = 8192;  // doubles per LDS tile (64 KB; two tiles)
constexpr int kSumThreads = 256;
constexpr int kSumLoaders = kSumThreads - kWave;                    // waves 1..3
constexpr int kSumPer = (kSumTileD + kSumLoaders - 1) / kSumLoaders;  // loads per loader thread, all in flight
constexpr int kSumB = 32;                                            // users per register batch of the chain
__global__ __launch_bounds__(kSumThreads) void metrics_sum_lds(const double* __restrict__ vals, int64_t n, int m,
                                                               double* __restrict__ out) {
    __shared__ double buf[2][kSumTileD];
    const int upt = (kSumTileD / m) & ~(kSumB - 1);  // users per tile, a multiple of the batch
    const int64_t nt = (n + upt - 1) / upt;
    const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
    auto load = [&](int64_t t, double* dst) {  // loader waves: every load issued before any LDS write
        const int64_t u0 = t * upt;
        const int64_t cnt = ((n - u0) < upt ? (n - u0) : upt) * (int64_t)m;
        const double* src = vals + u0 * m;
        const int i0 = tid - kWave;
        double r[kSumPer];
#pragma unroll
        for (int q = 0; q < kSumPer; ++q) {
            const int64_t i = i0 + (int64_t)q * kSumLoaders;
            r[q] = i < cnt ? src[i] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < kSumPer; ++q) {
            const int64_t i = i0 + (int64_t)q * kSumLoaders;
            if (i < cnt) dst[i] = r[q];
        }
    };
    if (nt > 0 && wave > 0) load(0, buf[0]);
    __syncthreads();
    double s = 0.0;
    for (int64_t t = 0; t < nt; ++t) {
        if (wave > 0 && t + 1 < nt) load(t + 1, buf[(t + 1) & 1]);
        if (wave == 0 && lane < m) {
            // the column's serial chain: batches of 32 values read from LDS into
            // registers at once, then 32 dependent adds (one per user, in order)
            const double* b = buf[t & 1] + lane;
            const int64_t u0 = t * upt;
            const int cnt = (int)((n - u0) < upt ? (n - u0) : upt);
            int u = 0;
            for (; u + kSumB <= cnt; u += kSumB) {
                double x[kSumB];
#pragma unroll
                for (int q = 0; q < kSumB; ++q) x[q] = b[(u + q) * m];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 0; q < kSumB; ++q) s += x[q];
            }
            for (; u < cnt; ++u) s += b[u * m];
        }
        __syncthreads();
    }
    if (wave == 0 && lane < m) out[lane] = s;
}

// Fast form: the same column sums in a fixed PARALLEL order, deterministic but not
// numpy's: pass 1, block b of kParBlocks(n) and thread t add users b*256+t,
// b*256+t + 256*nblk, ... (ppt = ceil(n / (256*nblk)) of them), then a 64-lane
// butterfly and the block's 4 wave sums in order -> partial[b][col]; pass 2, one
// wave per column adds partial[lane], partial[lane+64], ... then a butterfly.
// Summation-tree depth h = ppt + 6 + 4 + ceil(nblk/64) + 6 (sum_par_depth), so
// |fast - sequential| <= (gamma_h + gamma_{n-1}) * sum|x| (all values are >= 0):
// the caller rounds to 4 decimals and re-runs the sequential kernels only when a
// mean lies within that bound of a rounding boundary (rsx/evaluator.py).
constexpr int kParCols = 8;
constexpr int kParThreads = 256;
constexpr int kParMaxBlocks = 1024;

__host__ __device__ inline int64_t par_blocks(int64_t n) {
    const int64_t b = (n + kParThreads - 1) / kParThreads;
    return b < 1 ? 1 : (b > kParMaxBlocks ? kParMaxBlocks : b);
}

__device__ __forceinline__ double wave_sum(double x) {  // butterfly: every lane ends with the same bits
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) x += __shfl_xor(x, o, kWave);
    return x;
}

__global__ __launch_bounds__(kParThreads) void metrics_sum_par1(const double* __restrict__ vals, int64_t n, int m,
                                                                double* __restrict__ partial) {
    const int64_t nblk = gridDim.x;
    const int c0 = blockIdx.y * kParCols;
    const int nc = (m - c0) < kParCols ? (m - c0) : kParCols;
    double s[kParCols];
#pragma unroll
    for (int j = 0; j < kParCols; ++j) s[j] = 0.0;
    for (int64_t u = (int64_t)blockIdx.x * kParThreads + threadIdx.x; u < n; u += nblk * kParThreads) {
        const double* r = vals + u * m + c0;
#pragma unroll
        for (int j = 0; j < kParCols; ++j)
            if (j < nc) s[j] += r[j];
    }
#pragma unroll
    for (int j = 0; j < kParCols; ++j) s[j] = wave_sum(s[j]);
    __shared__ double part[kParThreads / kWave][kParCols];
    const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    if (lane == 0)
#pragma unroll
        for (int j = 0; j < kParCols; ++j) part[wave][j] = s[j];
    __syncthreads();
    if ((int)threadIdx.x < nc) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < kParThreads / kWave; ++w) t += part[w][threadIdx.x];
        partial[(int64_t)blockIdx.x * m + c0 + threadIdx.x] = t;
    }
}

__global__ __launch_bounds__(kWave) void metrics_sum_par2(const double* __restrict__ partial, int64_t nblk, int m,
                                                          double* __restrict__ out) {
    const int c = blockIdx.x, lane = threadIdx.x;
    double t = 0.0;
    for (int64_t b = lane; b < nblk; b += kWave) t += partial[b * m + c];
    t = wave_sum(t);
    if (lane == 0) out[c] = t;
}

static int topk_metrics_impl(const int64_t* topk_idx, int64_t n_users, int32_t k_max, const int64_t* eval_rowptr,
                             const int32_t* eval_col, const int32_t* cutoffs, int32_t n_cut, const double* gain,
                             double* out_sums, void* ws, size_t ws_bytes, hipStream_t s, bool fast);

}  // namespace rsx

using namespace rsx;

extern "C" size_t rsx_topk_metrics_ws_bytes(int64_t n_users, int32_t n_cut) {
    // per-user values, then the fast form's per-block partials
    const size_t m = kMetricCols * (size_t)(n_cut > 0 ? n_cut : 0);
    return ((size_t)(n_users > 0 ? n_users : 0) + (size_t)par_blocks(n_users)) * m * sizeof(double);
}

static int rsx::topk_metrics_impl(const int64_t* topk_idx, int64_t n_users, int32_t k_max,
                                  const int64_t* eval_rowptr, const int32_t* eval_col, const int32_t* cutoffs,
                                  int32_t n_cut, const double* gain, double* out_sums, void* ws, size_t ws_bytes,
                                  hipStream_t s, bool fast) {
    if (n_users < 0 || k_max <= 0 || n_cut <= 0 || !cutoffs || !gain || !out_sums) return RSX_ERR_ARG;
    if (n_users > 0 && (!topk_idx || !eval_rowptr || !eval_col)) return RSX_ERR_ARG;
    if (ws_bytes < rsx_topk_metrics_ws_bytes(n_users, n_cut) || (n_users > 0 && !ws)) return RSX_ERR_WORKSPACE;
    const int m = kMetricCols * n_cut;
    if (n_users == 0) return hip_rc(hipMemsetAsync(out_sums, 0, (size_t)m * sizeof(double), s));
    double* vals = static_cast<double*>(ws);
    if (n_users > 0)
        hipLaunchKernelGGL(metrics_user, dim3((unsigned)((n_users + kUserBlock - 1) / kUserBlock)), dim3(kUserBlock), 0, s,
                           topk_idx, n_users,
                           (int)k_max, eval_rowptr, eval_col, cutoffs, (int)n_cut, gain, vals);
    if (fast) {
        const int64_t nblk = par_blocks(n_users);
        double* partial = vals + (size_t)(n_users > 0 ? n_users : 0) * m;
        hipLaunchKernelGGL(metrics_sum_par1, dim3((unsigned)nblk, (unsigned)((m + kParCols - 1) / kParCols)),
                           dim3(kParThreads), 0, s, vals, n_users, m, partial);
        hipLaunchKernelGGL(metrics_sum_par2, dim3((unsigned)m), dim3(kWave), 0, s, partial, nblk, m, out_sums);
    } else if (m <= kWave)
        hipLaunchKernelGGL(metrics_sum_lds, dim3(1), dim3(kSumThreads), 0, s, vals, n_users, m, out_sums);
    else
        hipLaunchKernelGGL(metrics_sum, dim3((unsigned)m), dim3(64), 0, s, vals, n_users, m, out_sums);
    return last_rc();
}

extern "C" int rsx_topk_metrics(const int64_t* topk_idx, int64_t n_users, int32_t k_max, const int64_t* eval_rowptr,
                                const int32_t* eval_col, const int32_t* cutoffs, int32_t n_cut, const double* gain,
                                double* out_sums, void* ws, size_t ws_bytes, rsx_stream_t stream) {
    return topk_metrics_impl(topk_idx, n_users, k_max, eval_rowptr, eval_col, cutoffs, n_cut, gain, out_sums, ws,
                             ws_bytes, as_stream(stream), false);
}

extern "C" int rsx_topk_metrics_fast(const int64_t* topk_idx, int64_t n_users, int32_t k_max,
                                     const int64_t* eval_rowptr, const int32_t* eval_col, const int32_t* cutoffs,
                                     int32_t n_cut, const double* gain, double* out_sums, void* ws, size_t ws_bytes,
                                     rsx_stream_t stream) {
    return topk_metrics_impl(topk_idx, n_users, k_max, eval_rowptr, eval_col, cutoffs, n_cut, gain, out_sums, ws,
                             ws_bytes, as_stream(stream), true);
}

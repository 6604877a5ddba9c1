// knn.hip — SMORE's item-item kNN graph builder (gfx950): build_sim +
// build_knn_normalized_graph(sparse, 'sym') of reference src/utils/utils.py:134-181
// (called at src/models/smore.py:58-61, 69-71), without materialising the n x n
// similarity matrix (2.1 GB at Amazon-clothing).
//
// 1. knn_norm: x / ||x|| per row (context.div(torch.norm(context, p=2, dim=-1))).
// 2. knn_topk: S = Xn Xn^T on f32 MFMA (16x16x4: exact f32 products, f32 sums) in
//    block tiles of 128 own rows x 256 other rows, K streamed through LDS in chunks
//    of 32 features (double-buffered, next chunk's float4s in registers while this
//    one is multiplied).  After a panel's K loop every lane holds 64 scores of one
//    own row (other columns 16t + 4g + r of the panel) and inserts the ones above
//    its list's k-th value into a register-resident sorted list of KMAX (value,
//    index) pairs — the four lanes of a row each keep the top of their quarter of
//    the columns, and the row's four lists are merged at the end: the exact top-k
//    in (value desc, index asc) order.  Self-similarity is included, as in the
//    reference (its diagonal is ~1).
// 3. knn_symnorm: deg_r = sum of row r's kept values (in rank order, f32, the
//    reference's scatter_add over the row-major edge list), d = deg^-1/2 (inf -> 0),
//    w = (d_r * v) * d_c.
#include <cmath>

#include "rsx_common.hpp"

namespace rsx {
namespace knn {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kOwn = 128;      // own rows per block (8 waves x 16)
constexpr int kPanel = 256;    // other rows per panel (16 tiles of 16)
constexpr int kChunk = 32;     // features per LDS chunk
constexpr int kLdo = kChunk + 4;  // padded LDS row stride (conflict-free operand reads)
constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kLoadRows = kOwn + kPanel;
constexpr int kPer = kLoadRows * kChunk / 4 / kThreads;  // float4s per thread per chunk
static_assert(kLoadRows * kChunk / 4 % kThreads == 0, "chunk split");

__global__ __launch_bounds__(256) void knn_norm(const float* __restrict__ x, int64_t n, int32_t f,
                                                float* __restrict__ xn) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= n) return;
    const float* xr = x + row * f;
    float ss = 0.f;
    for (int j = lane; j < f; j += 64) ss += xr[j] * xr[j];
    ss = group_sum<64>(ss);
    const float den = sqrtf(ss);
    for (int j = lane; j < f; j += 64) xn[row * f + j] = xr[j] / den;
}

// a (value, index) pair ranks above another: larger value, or equal value and smaller index
__device__ __forceinline__ bool better(float v, int32_t i, float w, int32_t j) { return v > w || (v == w && i < j); }

template <int KMAX>
__device__ __forceinline__ void insert(float (&vals)[KMAX], int32_t (&ids)[KMAX], float v, int32_t i) {
    // bubble the pair down a sorted list (static indices: the list stays in registers)
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        const bool b = better(v, i, vals[j], ids[j]);
        const float tv = vals[j];
        const int32_t ti = ids[j];
        vals[j] = b ? v : tv;
        ids[j] = b ? i : ti;
        v = b ? tv : v;
        i = b ? ti : i;
    }
}

template <int KMAX>
__global__ __launch_bounds__(kThreads) void knn_topk(const float* __restrict__ xn, int64_t n, int32_t f, int32_t k,
                                                     float* __restrict__ out_v, int64_t* __restrict__ out_i) {
    __shared__ __attribute__((aligned(16))) float sm[2][kLoadRows * kLdo];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
    const int64_t b0 = (int64_t)blockIdx.x * kOwn;
    float vals[KMAX];
    int32_t ids[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        vals[j] = -INFINITY;
        ids[j] = INT32_MAX;
    }
    const int nchunk = (f + kChunk - 1) / kChunk;
    float4 pre[kPer];
    // chunk loader: rows [0, kOwn) = own rows b0.., rows [kOwn, kLoadRows) = panel rows p0..
    auto fetch = [&](int64_t p0, int ch) {
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int e = threadIdx.x + kThreads * q;
            const int r = e / (kChunk / 4), c4 = e - r * (kChunk / 4);
            const int64_t row = r < kOwn ? b0 + r : p0 + (r - kOwn);
            const int col = ch * kChunk + 4 * c4;
            float4 v = f4(0.f);
            if (row < n) {
                const float* src = xn + row * f + col;
                if (col + 4 <= f && (f & 3) == 0) {
                    v = ld4(src);
                } else {
                    v.x = col < f ? src[0] : 0.f;
                    v.y = col + 1 < f ? src[1] : 0.f;
                    v.z = col + 2 < f ? src[2] : 0.f;
                    v.w = col + 3 < f ? src[3] : 0.f;
                }
            }
            pre[q] = v;
        }
    };
    auto stash = [&](int buf) {
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int e = threadIdx.x + kThreads * q;
            const int r = e / (kChunk / 4), c4 = e - r * (kChunk / 4);
            *reinterpret_cast<float4*>(&sm[buf][r * kLdo + 4 * c4]) = pre[q];
        }
    };
    const int64_t npanel = (n + kPanel - 1) / kPanel;
    fetch(0, 0);
    for (int64_t pi = 0; pi < npanel; ++pi) {
        const int64_t p0 = pi * kPanel;
        floatx4 acc[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
        for (int ch = 0; ch < nchunk; ++ch) {
            const int buf = ch & 1;
            __syncthreads();  // readers of this buffer (two chunks ago) are done
            stash(buf);
            __syncthreads();
            // the next chunk (or the next panel's first) is in flight during the MFMAs
            if (ch + 1 < nchunk) fetch(p0, ch + 1);
            else if (pi + 1 < npanel) fetch(p0 + kPanel, 0);
            const float* own = &sm[buf][(16 * w + c) * kLdo + g];
            const float* oth = &sm[buf][(kOwn + c) * kLdo + g];
#pragma unroll 2
            for (int s = 0; s < kChunk / 4; ++s) {
                const float bv = own[4 * s];  // B[k = g][own c]
#pragma unroll
                for (int t = 0; t < 16; ++t)  // A[other 16t + c][k = g]
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(oth[16 * t * kLdo + 4 * s], bv, acc[t], 0, 0, 0);
            }
        }
        // lane (c, g): acc[t][r] = S[own 16w + c][other p0 + 16t + 4g + r]
        const bool own_ok = b0 + 16 * w + c < n;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t m = p0 + 16 * t + 4 * g + r;
                const float v = acc[t][r];
                if (own_ok && m < n && better(v, (int32_t)m, vals[KMAX - 1], ids[KMAX - 1]))
                    insert<KMAX>(vals, ids, v, (int32_t)m);
            }
        }
    }
    // merge the four lanes' lists of each row through LDS (k entries each: the top k of
    // the union needs no more), waves 0-3 then 4-7; lane g = 0 writes the row
    float* mv = &sm[0][0];
    int32_t* mi = reinterpret_cast<int32_t*>(&sm[0][0] + 4 * 64 * 32);
    static_assert(2 * 4 * 64 * 32 <= 2 * kLoadRows * kLdo, "merge lists fit the chunk buffers");
    const int64_t row = b0 + 16 * w + c;
    for (int round = 0; round < 2; ++round) {
        __syncthreads();
        const bool mine = (w >> 2) == round;
        const int lr = (w & 3) * 16 + c;  // row slot within the round
        if (mine) {
#pragma unroll
            for (int j = 0; j < KMAX; ++j)
                if (j < k) {
                    mv[(lr * 4 + g) * 32 + j] = vals[j];
                    mi[(lr * 4 + g) * 32 + j] = ids[j];
                }
        }
        __syncthreads();
        if (!mine || g != 0 || row >= n) continue;
        const int rb = lr * 4 * 32;
        int h[4] = {0, 0, 0, 0};
        for (int j = 0; j < k; ++j) {
            int best = -1;
            float bv = -INFINITY;
            int32_t bi = INT32_MAX;
            for (int q = 0; q < 4; ++q) {
                if (h[q] >= k) continue;
                const float v = mv[rb + q * 32 + h[q]];
                const int32_t i = mi[rb + q * 32 + h[q]];
                if (best < 0 || better(v, i, bv, bi)) {
                    best = q;
                    bv = v;
                    bi = i;
                }
            }
            ++h[best];
            out_v[row * k + j] = bv;
            out_i[row * k + j] = bi;
        }
    }
}

// w = (d_r v) d_c with d = (sum of the row's kept values)^-1/2, inf -> 0
__global__ __launch_bounds__(256) void knn_symnorm(const float* __restrict__ v, const int64_t* __restrict__ idx,
                                                   int64_t n, int32_t k, float* __restrict__ dis,
                                                   float* __restrict__ w, int phase) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (phase == 0) {
        if (t >= n) return;
        float deg = 0.f;
        for (int j = 0; j < k; ++j) deg += v[t * k + j];  // index_add over row-major edges: rank order
        const float d = 1.f / sqrtf(deg);
        dis[t] = isinf(d) ? 0.f : d;
        return;
    }
    if (t >= n * k) return;
    const int64_t r = t / k;
    w[t] = (dis[r] * v[t]) * dis[idx[t]];
}

}  // namespace knn
}  // namespace rsx

using namespace rsx;

extern "C" {

size_t rsx_knn_ws_bytes(int64_t n, int32_t f) { return (size_t)(n > 0 ? n : 0) * (size_t)(f > 0 ? f : 0) * 4 + (size_t)(n > 0 ? n : 1) * 4; }

int rsx_knn_graph(const float* feat, int64_t n, int32_t f, int32_t k, float* vals, int64_t* idx, float* weights,
                  void* ws, size_t ws_bytes, rsx_stream_t stream) {
    if (!feat || n < 0 || f <= 0 || k <= 0 || !vals || !idx || !weights) return RSX_ERR_ARG;
    if (k > n) return RSX_ERR_ARG;
    if (k > 32) return RSX_ERR_UNSUPPORTED;
    if (n == 0) return RSX_OK;
    if (n >= INT32_MAX) return RSX_ERR_ARG;
    if (!ws || ws_bytes < rsx_knn_ws_bytes(n, f)) return RSX_ERR_WORKSPACE;
    hipStream_t s = as_stream(stream);
    float* xn = static_cast<float*>(ws);
    float* dis = xn + n * (int64_t)f;
    hipLaunchKernelGGL(knn::knn_norm, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, feat, n, f, xn);
    const dim3 grid((unsigned)((n + knn::kOwn - 1) / knn::kOwn));
    if (k <= 16) hipLaunchKernelGGL(knn::knn_topk<16>, grid, dim3(knn::kThreads), 0, s, xn, n, f, k, vals, idx);
    else if (k <= 24) hipLaunchKernelGGL(knn::knn_topk<24>, grid, dim3(knn::kThreads), 0, s, xn, n, f, k, vals, idx);
    else hipLaunchKernelGGL(knn::knn_topk<32>, grid, dim3(knn::kThreads), 0, s, xn, n, f, k, vals, idx);
    hipLaunchKernelGGL(knn::knn_symnorm, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, vals, idx, n, k, dis,
                       weights, 0);
    hipLaunchKernelGGL(knn::knn_symnorm, dim3((unsigned)((n * k + 255) / 256)), dim3(256), 0, s, vals, idx, n, k, dis,
                       weights, 1);
    return last_rc();
}

}  // extern "C"

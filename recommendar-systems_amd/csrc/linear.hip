// linear.hip — weight gradients with a long reduction:  dW = g^T x  with g [n, out],
// x [n, in], n >> out.  Two users in SMORE:
//   * the Linear(d, d) layers (reference src/models/smore.py:106-120: query_v / query_t
//     MLPs, gate_* and gate_*_prefer) applied to all 26k user+item rows: a 64 x 64
//     output with a 26k-long reduction;
//   * the modality projections image_trs / text_trs (:256-259) in the spectral
//     backward: d W_v = d img^T V, a 64 x 4096 output over the 7k items.
// A library GEMM sees a tiny output and runs the long reduction on a few
// workgroups.  Here the reduction is split: block (tile, s) computes one 32 x 32
// output tile over row range s with its 4 waves taking interleaved 16-row chunks
// (fp32 MFMA, exact f32 fma chains, next chunk prefetched), adds the 4 wave tiles
// in LDS in wave order and writes the tile of partial s; a second pass adds the
// partials in a fixed order.  Deterministic: the result depends only on the shapes.
#include "rsx_common.hpp"

namespace rsx {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kWgChunk = 16;        // rows per wave step: 8 MFMAs of 2 rows
constexpr int kWgMinRows = 64;      // rows per block at least (one chunk per wave)
constexpr int kWgTargetBlocks = 512;

struct WgPlan {
    int64_t rows;  // rows per block (multiple of 64)
    int splits;    // S
};

// S ~ kWgTargetBlocks / tiles, at most half the input bytes in partials, at least
// kWgMinRows rows per block.
static WgPlan wg_plan(int64_t n, int out_dim, int in_dim) {
    const int64_t tiles = (int64_t)(out_dim / 32) * (in_dim / 32);
    int64_t s = (kWgTargetBlocks + tiles - 1) / tiles;
    const int64_t cap = ((int64_t)n * (out_dim + in_dim) / 2) / ((int64_t)out_dim * in_dim);
    if (s > cap) s = cap;
    const int64_t smax = (n + kWgMinRows - 1) / kWgMinRows;
    if (s > smax) s = smax;
    if (s < 1) s = 1;
    int64_t rows = (n + s - 1) / s;
    rows = (rows + kWgMinRows - 1) / kWgMinRows * kWgMinRows;
    if (rows < kWgMinRows) rows = kWgMinRows;
    s = n > 0 ? (n + rows - 1) / rows : 1;
    return {rows, (int)s};
}

// lane l of a 16-row chunk at row c0: A = g[c0 + 2q + h][o0 + j], B = x[...][i0 + j]
// for the q-th MFMA (k index h = l >> 5 on both sides), zero past r1
__device__ __forceinline__ void wg_load(const float* __restrict__ g, const float* __restrict__ x, int64_t c0,
                                        int64_t r1, int out_dim, int in_dim, int o0, int i0, int j, int h,
                                        float (&av)[8], float (&bv)[8]) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int64_t row = c0 + 2 * q + h;
        const bool ok = row < r1;
        av[q] = ok ? g[row * out_dim + o0 + j] : 0.f;
        bv[q] = ok ? x[row * in_dim + i0 + j] : 0.f;
    }
}

__global__ __launch_bounds__(256) void wgrad_partial(const float* __restrict__ g, const float* __restrict__ x,
                                                     int64_t n, int out_dim, int in_dim, int64_t rows,
                                                     float* __restrict__ part) {
    __shared__ float red[4][32 * 33];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 31, h = lane >> 5;
    const int ti = in_dim / 32, tiles = (out_dim / 32) * ti;
    const int tile = blockIdx.x % tiles;
    const int64_t s = blockIdx.x / tiles;
    const int o0 = (tile / ti) * 32, i0 = (tile % ti) * 32;
    const int64_t r0 = s * rows;
    const int64_t r1 = min(n, r0 + rows);
    const int64_t nch = (r1 - r0 + kWgChunk - 1) / kWgChunk;
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    float av[8], bv[8];
    int64_t c = wave;  // wave-uniform: the MFMAs need the whole wave
    if (c < nch) wg_load(g, x, r0 + c * kWgChunk, r1, out_dim, in_dim, o0, i0, j, h, av, bv);
    for (; c < nch; c += 4) {
        float an[8], bn[8];
        const bool more = c + 4 < nch;
        if (more) wg_load(g, x, r0 + (c + 4) * kWgChunk, r1, out_dim, in_dim, o0, i0, j, h, an, bn);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], bv[q], acc, 0, 0, 0);
        if (more) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                av[q] = an[q];
                bv[q] = bn[q];
            }
        }
    }
    // C layout: lane holds column i0 + j, rows o0 + (r&3) + 8(r>>2) + 4h
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wave][((r & 3) + 8 * (r >> 2) + 4 * h) * 33 + j] = acc[r];
    __syncthreads();
    float* dst = part + s * (int64_t)out_dim * in_dim;
#pragma unroll
    for (int e = threadIdx.x; e < 1024; e += 256) {
        const int o = e >> 5, i = e & 31;
        const float v = ((red[0][o * 33 + i] + red[1][o * 33 + i]) + red[2][o * 33 + i]) + red[3][o * 33 + i];
        dst[(int64_t)(o0 + o) * in_dim + i0 + i] = v;
    }
}

// element e = blockIdx.x*64 + lane; wave w adds partials [w*S/4, (w+1)*S/4) in
// order, 8 loads in flight; the quarters are added in wave order
__global__ __launch_bounds__(256) void wgrad_reduce(const float* __restrict__ part, int S, int64_t sz,
                                                    float* __restrict__ dw) {
    __shared__ float q[4][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t e = (int64_t)blockIdx.x * 64 + lane;
    const int b = (int)((int64_t)S * wave / 4), en = (int)((int64_t)S * (wave + 1) / 4);
    float acc = 0.f;
    if (e < sz) {
        int p = b;
        for (; p + 8 <= en; p += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(p + u) * sz + e];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += v[u];
        }
        for (; p < en; ++p) acc += part[(int64_t)p * sz + e];
    }
    q[wave][lane] = acc;
    __syncthreads();
    if (wave == 0 && e < sz) dw[e] = ((q[0][lane] + q[1][lane]) + q[2][lane]) + q[3][lane];
}

}  // namespace rsx

using namespace rsx;

extern "C" size_t rsx_linear_wgrad_ws_bytes(int64_t n, int32_t out_dim, int32_t in_dim) {
    if (n <= 0 || out_dim <= 0 || in_dim <= 0 || (out_dim % 32) || (in_dim % 32)) return 0;
    const WgPlan p = wg_plan(n, out_dim, in_dim);
    return (size_t)p.splits * (size_t)out_dim * (size_t)in_dim * sizeof(float);
}

extern "C" int rsx_linear_wgrad(const float* g, const float* x, int64_t n, int32_t out_dim, int32_t in_dim, float* dw,
                                void* ws, size_t ws_bytes, rsx_stream_t stream) {
    if (n < 0 || out_dim <= 0 || in_dim <= 0 || !dw) return RSX_ERR_ARG;
    if ((out_dim % 32) || (in_dim % 32)) return RSX_ERR_UNSUPPORTED;
    if (n > 0 && (!g || !x)) return RSX_ERR_ARG;
    hipStream_t s = as_stream(stream);
    const int64_t sz = (int64_t)out_dim * in_dim;
    if (n == 0) {
        hipLaunchKernelGGL(wgrad_reduce, dim3((unsigned)((sz + 63) / 64)), dim3(256), 0, s, (const float*)nullptr, 0,
                           sz, dw);
        return last_rc();
    }
    if (ws_bytes < rsx_linear_wgrad_ws_bytes(n, out_dim, in_dim) || !ws) return RSX_ERR_WORKSPACE;
    const WgPlan p = wg_plan(n, out_dim, in_dim);
    const int64_t tiles = (int64_t)(out_dim / 32) * (in_dim / 32);
    float* part = static_cast<float*>(ws);
    hipLaunchKernelGGL(wgrad_partial, dim3((unsigned)(tiles * p.splits)), dim3(256), 0, s, g, x, n, (int)out_dim,
                       (int)in_dim, p.rows, part);
    hipLaunchKernelGGL(wgrad_reduce, dim3((unsigned)((sz + 63) / 64)), dim3(256), 0, s, (const float*)part, p.splits,
                       sz, dw);
    return last_rc();
}

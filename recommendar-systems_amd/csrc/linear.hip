// linear.hip — weight gradient of the small nn.Linear(d, d) layers of SMORE
// (reference src/models/smore.py:106-120: query_v / query_t MLPs, gate_* and
// gate_*_prefer), applied to all 26k user+item rows:  dW = g^T x  with
// g [n, out], x [n, in], n >> out, in.  A library GEMM sees a 64x64 output with a
// 26k-long reduction and runs it on a couple of workgroups; here the rows are
// split over many blocks (fp32 MFMA, exact f32 fma chains), each block writes its
// [out][in] partial, and a second pass adds the partials in block order, so the
// result is deterministic.
#include "rsx_common.hpp"

namespace rsx {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kWgRows = 512;  // rows per block

// Block b: rows [b*kWgRows, +kWgRows); its 4 waves take the 32x32 output tiles
// t = wave, wave+4, ...; an MFMA consumes 2 rows: lane l supplies g[row][o0 + (l&31)]
// (A, row index k = l>>5) and x[row][i0 + (l&31)] (B), both coalesced row reads.
__global__ __launch_bounds__(256) void wgrad_partial(const float* __restrict__ g, const float* __restrict__ x,
                                                     int64_t n, int out_dim, int in_dim, float* __restrict__ part) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 31, h = lane >> 5;
    const int64_t r0 = (int64_t)blockIdx.x * kWgRows;
    const int64_t r1 = min(n, r0 + kWgRows);
    const int to = out_dim / 32, ti = in_dim / 32;
    float* dst = part + (int64_t)blockIdx.x * out_dim * in_dim;
    for (int t = wave; t < to * ti; t += 4) {
        const int o0 = (t / ti) * 32, i0 = (t % ti) * 32;
        floatx16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
        int64_t base = r0;  // wave-uniform: MFMAs need the whole wave
        // 8 MFMAs (16 rows) per step, loads first
        for (; base + 16 <= r1; base += 16) {
            float av[8], bv[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int64_t row = base + 2 * q + h;
                av[q] = g[row * out_dim + o0 + j];
                bv[q] = x[row * in_dim + i0 + j];
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], bv[q], acc, 0, 0, 0);
        }
        for (; base < r1; base += 2) {
            const int64_t row = base + h;
            const bool ok = row < r1;
            const float av = ok ? g[row * out_dim + o0 + j] : 0.f;
            const float bv = ok ? x[row * in_dim + i0 + j] : 0.f;
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
        }
        // C layout: lane holds column i0 + j, rows o0 + (r&3) + 8(r>>2) + 4h
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int o = o0 + (r & 3) + 8 * (r >> 2) + 4 * h;
            dst[o * in_dim + i0 + j] = acc[r];
        }
    }
}

__global__ void wgrad_reduce(const float* __restrict__ part, int nblk, int64_t sz, float* __restrict__ dw) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= sz) return;
    float s = 0.f;
    for (int b = 0; b < nblk; ++b) s += part[(int64_t)b * sz + e];
    dw[e] = s;
}

}  // namespace rsx

using namespace rsx;

extern "C" size_t rsx_linear_wgrad_ws_bytes(int64_t n, int32_t out_dim, int32_t in_dim) {
    const int64_t nblk = (n + kWgRows - 1) / kWgRows;
    return (size_t)(nblk > 0 ? nblk : 1) * (size_t)out_dim * (size_t)in_dim * sizeof(float);
}

extern "C" int rsx_linear_wgrad(const float* g, const float* x, int64_t n, int32_t out_dim, int32_t in_dim, float* dw,
                                void* ws, size_t ws_bytes, rsx_stream_t stream) {
    if (n < 0 || out_dim <= 0 || in_dim <= 0 || !dw) return RSX_ERR_ARG;
    if ((out_dim % 32) || (in_dim % 32)) return RSX_ERR_UNSUPPORTED;
    if (n > 0 && (!g || !x)) return RSX_ERR_ARG;
    if (ws_bytes < rsx_linear_wgrad_ws_bytes(n, out_dim, in_dim) || !ws) return RSX_ERR_WORKSPACE;
    hipStream_t s = as_stream(stream);
    const int nblk = (int)((n + kWgRows - 1) / kWgRows);
    const int64_t sz = (int64_t)out_dim * in_dim;
    float* part = static_cast<float*>(ws);
    if (nblk > 0)
        hipLaunchKernelGGL(wgrad_partial, dim3((unsigned)nblk), dim3(256), 0, s, g, x, n, (int)out_dim, (int)in_dim,
                           part);
    hipLaunchKernelGGL(wgrad_reduce, dim3((unsigned)((sz + 255) / 256)), dim3(256), 0, s, part, nblk, sz, dw);
    return last_rc();
}

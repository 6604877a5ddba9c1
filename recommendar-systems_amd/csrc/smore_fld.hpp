// smore_fld.hpp — the row-field toolkit of the SMORE per-row kernels (smore_fuse.hip)
// and of the fused item-side pass (smore.hip): a 16-row tile of [rows x D] held in a
// wave as the transposed accumulator layout of v_mfma_f32_16x16x4f32 (lane
// l = n + 16 g holds row n, features 16 t + 4 g + r in register 4 t + r; see the
// header of smore_fuse.hip), Linear products on it, LDS weight staging, the
// activations and the dropout mask.
#pragma once
#include <cmath>

#include "rsx_common.hpp"

namespace rsx {
namespace sf {

typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int D>
struct Fld {
    floatx4 f[D / 16];
};

template <int D>
__device__ __forceinline__ Fld<D> fzero() {
    Fld<D> x;
#pragma unroll
    for (int t = 0; t < D / 16; ++t) x.f[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    return x;
}

// row `row` of X [.., D] (row < 0: zeros); this lane's features 16t + 4g .. +3
template <int D>
__device__ __forceinline__ Fld<D> fload(const float* X, int64_t row, int g) {
    Fld<D> x;
#pragma unroll
    for (int t = 0; t < D / 16; ++t) {
        if (row >= 0) {
            const float4 v = ld4(X + row * D + 16 * t + 4 * g);
            x.f[t] = floatx4{v.x, v.y, v.z, v.w};
        } else {
            x.f[t] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
    }
    return x;
}

template <int D>
__device__ __forceinline__ void fstore(float* Y, int64_t row, int g, const Fld<D>& x) {
    if (row < 0 || !Y) return;
#pragma unroll
    for (int t = 0; t < D / 16; ++t) st4(Y + row * D + 16 * t + 4 * g, make_float4(x.f[t][0], x.f[t][1], x.f[t][2], x.f[t][3]));
}

// a per-feature vector (bias) in the field layout
template <int D>
__device__ __forceinline__ Fld<D> fvec(const float* b, int g) {
    return b ? fload<D>(b, 0, g) : fzero<D>();
}

template <int D, class F>
__device__ __forceinline__ Fld<D> fmap(const Fld<D>& a, F fn) {
    Fld<D> z;
#pragma unroll
    for (int t = 0; t < D / 16; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) z.f[t][r] = fn(a.f[t][r]);
    return z;
}
template <int D, class F>
__device__ __forceinline__ Fld<D> fmap2(const Fld<D>& a, const Fld<D>& b, F fn) {
    Fld<D> z;
#pragma unroll
    for (int t = 0; t < D / 16; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) z.f[t][r] = fn(a.f[t][r], b.f[t][r]);
    return z;
}
template <int D, class F>
__device__ __forceinline__ Fld<D> fmap3(const Fld<D>& a, const Fld<D>& b, const Fld<D>& c, F fn) {
    Fld<D> z;
#pragma unroll
    for (int t = 0; t < D / 16; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) z.f[t][r] = fn(a.f[t][r], b.f[t][r], c.f[t][r]);
    return z;
}

// sum / max over a row's D features (every lane of the row gets it)
template <int D>
__device__ __forceinline__ float rsum(const Fld<D>& x) {
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < D / 16; ++t) s += (x.f[t][0] + x.f[t][1]) + (x.f[t][2] + x.f[t][3]);
    s += __shfl_xor(s, 16, kWave);
    s += __shfl_xor(s, 32, kWave);
    return s;
}
template <int D>
__device__ __forceinline__ float rmax(const Fld<D>& x) {
    float s = -INFINITY;
#pragma unroll
    for (int t = 0; t < D / 16; ++t) s = fmaxf(fmaxf(s, fmaxf(x.f[t][0], x.f[t][1])), fmaxf(x.f[t][2], x.f[t][3]));
    s = fmaxf(s, __shfl_xor(s, 16, kWave));
    s = fmaxf(s, __shfl_xor(s, 32, kWave));
    return s;
}

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// z[n][o] = sum_k W[o][k] x[n][k]  (+ b[o]),  W [D][D] row-major (nn.Linear weight)
// with row stride LD (the padded LDS copy: LD = D + 4, conflict-free float4 reads).
// K outer, output tiles inner: consecutive MFMAs go to different accumulators (the
// 16x16x4 form's dependent latency is 40 cycles against a 32-cycle issue).
template <int D, int LD>
__device__ __forceinline__ Fld<D> mv(const float* __restrict__ W, const float* b, const Fld<D>& x, int lane) {
    constexpr int T = D / 16;
    const int c = lane & 15, g = lane >> 4;
    Fld<D> z = fvec<D>(b, g);
    const float* wr = W + c * LD + 4 * g;
#pragma unroll
    for (int t = 0; t < T; ++t) {
        float4 w[T];
#pragma unroll
        for (int to = 0; to < T; ++to) w[to] = ld4(wr + 16 * to * LD + 16 * t);
#pragma unroll
        for (int to = 0; to < T; ++to) z.f[to] = mfma4(w[to].x, x.f[t][0], z.f[to]);
#pragma unroll
        for (int to = 0; to < T; ++to) z.f[to] = mfma4(w[to].y, x.f[t][1], z.f[to]);
#pragma unroll
        for (int to = 0; to < T; ++to) z.f[to] = mfma4(w[to].z, x.f[t][2], z.f[to]);
#pragma unroll
        for (int to = 0; to < T; ++to) z.f[to] = mfma4(w[to].w, x.f[t][3], z.f[to]);
    }
    return z;
}

// mv / mvt with a bounded register footprint: the weight operands of step t+1 are
// loaded while step t's MFMAs run, and a scheduling barrier keeps the compiler from
// hoisting every step's loads to the top (which needs D*D/16 registers at d = 128 and
// makes two waves a SIMD spill).  Same products, same accumulation order.
template <int D, int LD>
__device__ __forceinline__ Fld<D> mv_p(const float* __restrict__ W, const float* b, const Fld<D>& x, int lane) {
    constexpr int T = D / 16;
    const int c = lane & 15, g = lane >> 4;
    Fld<D> z = fvec<D>(b, g);
    const float* wr = W + c * LD + 4 * g;
    float4 w[2][T];
#pragma unroll
    for (int to = 0; to < T; ++to) w[0][to] = ld4(wr + 16 * to * LD);
#pragma unroll
    for (int t = 0; t < T; ++t) {
        if (t + 1 < T) {
#pragma unroll
            for (int to = 0; to < T; ++to) w[(t + 1) & 1][to] = ld4(wr + 16 * to * LD + 16 * (t + 1));
        }
        const float4* wc = w[t & 1];
#pragma unroll
        for (int to = 0; to < T; ++to) z.f[to] = mfma4(wc[to].x, x.f[t][0], z.f[to]);
#pragma unroll
        for (int to = 0; to < T; ++to) z.f[to] = mfma4(wc[to].y, x.f[t][1], z.f[to]);
#pragma unroll
        for (int to = 0; to < T; ++to) z.f[to] = mfma4(wc[to].z, x.f[t][2], z.f[to]);
#pragma unroll
        for (int to = 0; to < T; ++to) z.f[to] = mfma4(wc[to].w, x.f[t][3], z.f[to]);
        __builtin_amdgcn_sched_barrier(0);
    }
    return z;
}

template <int D, int LD>
__device__ __forceinline__ Fld<D> mvt_p(const float* __restrict__ W, const Fld<D>& x, int lane) {
    constexpr int T = D / 16;
    const int c = lane & 15, g = lane >> 4;
    Fld<D> z = fzero<D>();
    float wv[2][T];
    auto load = [&](int t, int r, float(&dst)[T]) __attribute__((always_inline)) {
        const float* wr = W + (16 * t + 4 * g + r) * LD + c;
#pragma unroll
        for (int tk = 0; tk < T; ++tk) dst[tk] = wr[16 * tk];
    };
    load(0, 0, wv[0]);
#pragma unroll
    for (int t = 0; t < T; ++t) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int q = t * 4 + r;
            if (q + 1 < 4 * T) load((q + 1) >> 2, (q + 1) & 3, wv[(q + 1) & 1]);
#pragma unroll
            for (int tk = 0; tk < T; ++tk) z.f[tk] = mfma4(wv[q & 1][tk], x.f[t][r], z.f[tk]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    return z;
}

// z[n][k] = sum_o W[o][k] x[n][o]  (the input gradient of a Linear)
template <int D, int LD>
__device__ __forceinline__ Fld<D> mvt(const float* __restrict__ W, const Fld<D>& x, int lane) {
    constexpr int T = D / 16;
    const int c = lane & 15, g = lane >> 4;
    Fld<D> z = fzero<D>();
#pragma unroll
    for (int t = 0; t < T; ++t) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float* wr = W + (16 * t + 4 * g + r) * LD + c;
#pragma unroll
            for (int tk = 0; tk < T; ++tk) z.f[tk] = mfma4(wr[16 * tk], x.f[t][r], z.f[tk]);
        }
    }
    return z;
}

// A block's copy of one [D][D] weight in LDS, rows padded to D + 4 floats: every
// wave of the block reads it (a 16-row tile each) instead of streaming it from L2
// per MFMA step.  All threads of the block call it, in the same order.
template <int D>
constexpr int kLd = D + 4;

// Staged by LDS-DMA (global_load_lds, 4 B a lane: a wave-instruction moves 64 consecutive
// floats of one row, so the padded rows stay intact): every piece of the block's share is
// in flight at once and no VGPR holds it -- a register-staged loop here waited out one
// L2 round trip per float4 (the store needs the load), 16 of them per thread at d = 128.
template <int D>
__device__ __forceinline__ const float* stage_w(float* __restrict__ lds, const float* __restrict__ W) {
    static_assert(D % 64 == 0, "stage_w: rows of whole 64-float pieces");
    __syncthreads();  // the previous weight's readers are done
    constexpr int PR = D / 64;        // pieces per row
    const int lane = threadIdx.x & 63;
    const int nw = blockDim.x >> 6;
    for (int pc = threadIdx.x >> 6; pc < D * PR; pc += nw) {  // wave-uniform
        const int row = pc / PR, c0 = (pc - row * PR) * 64;
        __builtin_amdgcn_global_load_lds(W + (int64_t)row * D + c0 + lane, lds + row * kLd<D> + c0, 4, 0, 0);
    }
    __syncthreads();  // (waits for the DMA: vmcnt(0) before the barrier)
    return lds;
}

// S^T tile: s[r] = <Y row (4g + r), X row c> over D (two accumulators, summed at the end)
template <int D>
__device__ __forceinline__ floatx4 tile_dot(const Fld<D>& Y, const Fld<D>& X) {
    constexpr int T = D / 16;
    floatx4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
            s0 = mfma4(Y.f[t][r], X.f[t][r], s0);
            s1 = mfma4(Y.f[t][r + 1], X.f[t][r + 1], s1);
        }
    return s0 + s1;
}

struct Sigm {
    __device__ float operator()(float x) const { return 1.f / (1.f + expf(-x)); }
};
struct Tanh {
    __device__ float operator()(float x) const { return tanhf(x); }
};
constexpr Sigm sigm{};
constexpr Tanh tanh_{};

template <int D>
__device__ __forceinline__ Fld<D> softmax_row(const Fld<D>& q) {
    const float mx = rmax<D>(q);
    const Fld<D> e = fmap<D>(q, [&](float v) { return expf(v - mx); });
    const float s = rsum<D>(e);
    return fmap<D>(e, [&](float v) { return v / s; });
}

// dropout keep-scale of element (row, feature) of preference gate `gate`: 0 or 1/(1-p)
__device__ __forceinline__ uint32_t mix32(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return (uint32_t)x;
}
template <int D>
__device__ __forceinline__ Fld<D> drop_scale(uint64_t seed, int gate, int64_t row, int g, float p, float scale) {
    Fld<D> m;
    const uint32_t thr = (uint32_t)fminf(p * 4294967296.f, 4294967295.f);
#pragma unroll
    for (int t = 0; t < D / 16; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint64_t key = seed * 0x9E3779B97F4A7C15ULL + ((uint64_t)gate << 58) + (uint64_t)row * D +
                                 (uint64_t)(16 * t + 4 * g + r);
            m.f[t][r] = mix32(key) >= thr ? scale : 0.f;
        }
    return m;
}

}  // namespace sf
}  // namespace rsx

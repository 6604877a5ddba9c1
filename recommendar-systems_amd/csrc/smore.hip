// smore.hip — SMORE's modality projection + spectral denoise / cross-modal fusion
// as one fused pass (reference src/models/smore.py:209-237 spectrum_convolution and
// :256-259 image_trs / text_trs), and the fused backward of the spectral part.
//
// Forward, per block of 32 items (4 wavefronts):
//   1. img = V W_v^T + b_v, txt = T W_t^T + b_t on fp32 MFMA (v_mfma_f32_32x32x2f32,
//      exact f32): the K dimension (feature width, 4096 raw image / 384 text at
//      Amazon-baby) is split over the 4 waves, partial tiles summed in LDS in wave
//      order (deterministic), bias first.
//   2. rfft(norm='ortho') of both rows as direct real DFTs against an LDS twiddle
//      table (d <= 128: d*(d/2+1) MACs per row, far below the projection), the
//      per-bin complex weights (already unit-normalised by the caller, as
//      reference :221-229), the cross-modal product Ft*Fi*wf, and three irfft's.
//   img / txt are written out as well (saved for the backward).
// Backward (spectral part): dY = irfft^T(dconv); dF = dY * conj(w) (+ the product
// rule for the fusion term); d img / d txt = rfft^T(dF); per-block partial sums of
// dw in the parameter layout [3][d/2+1][2].  The projection gradients
// (dW = d img^T V, dV = d img W, db) are plain GEMMs / reductions left to the
// caller (rocBLAS via torch).
#include "rsx_common.hpp"

namespace rsx {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct SpecFwdArgs {
    const float* X[2];  // V [n, K0], T [n, K1]
    int32_t K[2];
    const float* W[2];  // [d, K]
    const float* b[2];  // [d]
    const float* w[3];  // unit complex weights [(d/2+1)][2]: image, text, fusion
    int64_t n;
    float* xo[2];       // img, txt [n, d]
    float* conv[3];     // conv_v, conv_t, conv_f [n, d]
};

// MFMA projection of 32 rows (row0..) of X [n, K] by W [D, K] into xs[32][D+1]
// (+ bias).  Wave w owns the k-slice [w*per, (w+1)*per) in steps of 8; lane l
// feeds item row l&31 and, within a step of 8, k = 4*(l>>5) + q for the q-th of 4
// MFMAs (the same permutation on the A and B side).
template <int D>
__device__ __forceinline__ void project32(const float* __restrict__ X, int K, const float* __restrict__ W,
                                          const float* __restrict__ bias, int64_t row0, int64_t n,
                                          float (*xs)[D + 1]) {
    constexpr int NT = D / 32;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 31, h = lane >> 5;
    floatx16 acc[NT];
#pragma unroll
    for (int c = 0; c < NT; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
    const int steps = (K + 7) / 8;
    const int per = (steps + 3) / 4;
    const int kb = wave * per * 8, ke = min(K, (wave + 1) * per * 8);
    const int64_t row = row0 + j;
    const float* xr = X + (row < n ? row : 0) * (int64_t)K;
    for (int k = kb; k < ke; k += 8) {
        const int kk = k + 4 * h;
        const bool ok = kk < ke;  // K % 4 == 0: the whole float4 is in range
        const float4 a = (ok && row < n) ? ld4(xr + kk) : f4(0.f);
#pragma unroll
        for (int c = 0; c < NT; ++c) {
            const float4 bb = ok ? ld4(W + (int64_t)(c * 32 + j) * K + kk) : f4(0.f);
            acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bb.x, acc[c], 0, 0, 0);
            acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bb.y, acc[c], 0, 0, 0);
            acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, bb.z, acc[c], 0, 0, 0);
            acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bb.w, acc[c], 0, 0, 0);
        }
    }
    // C layout: lane holds column (feature) c*32 + j, rows (items) (r&3) + 8(r>>2) + 4h
    for (int w2 = 0; w2 < 4; ++w2) {
        if (wave == w2) {
#pragma unroll
            for (int c = 0; c < NT; ++c)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int i = (r & 3) + 8 * (r >> 2) + 4 * h, f = c * 32 + j;
                    const float base = w2 == 0 ? bias[f] : xs[i][f];
                    xs[i][f] = base + acc[c][r];
                }
        }
        __syncthreads();
    }
}

template <int D>
__device__ __forceinline__ void twiddles(float* twc, float* tws) {
    for (int t = threadIdx.x; t < D; t += blockDim.x) {
        double s, c;
        sincospi(2.0 * (double)t / (double)D, &s, &c);
        twc[t] = (float)c;
        tws[t] = (float)s;
    }
}

// rfft bin k of a length-D real row (norm='ortho'): (re, im)
template <int D>
__device__ __forceinline__ float2 dft_bin(const float* x, int k, const float* twc, const float* tws) {
    float re = 0.f, im = 0.f;
#pragma unroll 8
    for (int t = 0; t < D; ++t) {
        const int e = (k * t) & (D - 1);
        re = fmaf(x[t], twc[e], re);
        im = fmaf(-x[t], tws[e], im);
    }
    const float s = rsqrtf((float)D);
    return make_float2(re * s, im * s);
}

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {  // a * conj(b)
    return make_float2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}

template <int D>
__global__ __launch_bounds__(256) void smore_spec_fwd(SpecFwdArgs a) {
    constexpr int NB = D / 2 + 1;
    __shared__ float xs[2][32][D + 1];
    __shared__ float ys[32][3][2][NB];
    __shared__ float twc[D], tws[D];
    const int64_t row0 = (int64_t)blockIdx.x * 32;
    twiddles<D>(twc, tws);
    project32<D>(a.X[0], a.K[0], a.W[0], a.b[0], row0, a.n, xs[0]);
    project32<D>(a.X[1], a.K[1], a.W[1], a.b[1], row0, a.n, xs[1]);
    const int r = threadIdx.x >> 3, sub = threadIdx.x & 7;
    const int64_t row = row0 + r;
    // spectra and filtered spectra for bins k = sub + 8i
    for (int k = sub; k < NB; k += 8) {
        const float2 fi = dft_bin<D>(xs[0][r], k, twc, tws);
        const float2 ft = dft_bin<D>(xs[1][r], k, twc, tws);
        const float2 wv = make_float2(a.w[0][2 * k], a.w[0][2 * k + 1]);
        const float2 wt = make_float2(a.w[1][2 * k], a.w[1][2 * k + 1]);
        const float2 wf = make_float2(a.w[2][2 * k], a.w[2][2 * k + 1]);
        const float2 yv = cmul(fi, wv), yt = cmul(ft, wt), yf = cmul(cmul(ft, fi), wf);
        ys[r][0][0][k] = yv.x;
        ys[r][0][1][k] = yv.y;
        ys[r][1][0][k] = yt.x;
        ys[r][1][1][k] = yt.y;
        ys[r][2][0][k] = yf.x;
        ys[r][2][1][k] = yf.y;
    }
    __syncthreads();
    if (row >= a.n) return;
    const float s = rsqrtf((float)D);
    for (int t = sub; t < D; t += 8) {
        a.xo[0][row * D + t] = xs[0][r][t];
        a.xo[1][row * D + t] = xs[1][r][t];
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            // irfft(norm='ortho'): bins 0 and D/2 once (their imaginary parts ignored), others twice
            float acc = ys[r][m][0][0] + ((t & 1) ? -ys[r][m][0][D / 2] : ys[r][m][0][D / 2]);
            float mid = 0.f;
            for (int k = 1; k < D / 2; ++k) {
                const int e = (k * t) & (D - 1);
                mid = fmaf(ys[r][m][0][k], twc[e], mid);
                mid = fmaf(-ys[r][m][1][k], tws[e], mid);
            }
            acc = fmaf(2.f, mid, acc);
            a.conv[m][row * D + t] = acc * s;
        }
    }
}

struct SpecBwdArgs {
    const float* xo[2];  // img, txt [n, d]
    const float* w[3];
    const float* g[3];   // d conv_v / conv_t / conv_f [n, d] (NULL = 0)
    int64_t n;
    float* gx[2];        // d img, d txt [n, d]
    float* gw;           // [gridDim.x][3][d/2+1][2] per-block partials
};

template <int D>
__global__ __launch_bounds__(256) void smore_spec_bwd(SpecBwdArgs a) {
    constexpr int NB = D / 2 + 1;
    __shared__ float xs[2][32][D + 1];
    __shared__ float gs[3][32][D + 1];
    __shared__ float df[32][2][2][NB];  // d spectrum of img / txt
    __shared__ float dws[4][3][2][NB];  // per-wave d weight (8 rows each)
    __shared__ float twc[D], tws[D];
    const int64_t row0 = (int64_t)blockIdx.x * 32;
    twiddles<D>(twc, tws);
    for (int e = threadIdx.x; e < 32 * D; e += 256) {
        const int r = e / D, t = e % D;
        const int64_t row = row0 + r;
        const bool ok = row < a.n;
#pragma unroll
        for (int m = 0; m < 2; ++m) xs[m][r][t] = ok ? a.xo[m][row * D + t] : 0.f;
#pragma unroll
        for (int m = 0; m < 3; ++m) gs[m][r][t] = (ok && a.g[m]) ? a.g[m][row * D + t] : 0.f;
    }
    __syncthreads();
    const int r = threadIdx.x >> 3, sub = threadIdx.x & 7;
    const float s = rsqrtf((float)D);
    // uniform trip count over the wave (the d-weight sums below shuffle across rows)
    for (int i = 0; i < (NB + 7) / 8; ++i) {
        const int kr = sub + 8 * i;
        const bool kv = kr < NB;
        const int k = kv ? kr : 0;
        const float2 fi = dft_bin<D>(xs[0][r], k, twc, tws);
        const float2 ft = dft_bin<D>(xs[1][r], k, twc, tws);
        // dY = irfft^T(g): d/dRe = a_k cos/sqrt(D), d/dIm = -a_k sin/sqrt(D)
        const float ak = (k == 0 || k == D / 2) ? 1.f : 2.f;
        float2 dy[3];
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            float re = 0.f, im = 0.f;
            for (int t = 0; t < D; ++t) {
                const int e = (k * t) & (D - 1);
                re = fmaf(gs[m][r][t], twc[e], re);
                im = fmaf(-gs[m][r][t], tws[e], im);
            }
            dy[m] = make_float2(re * ak * s, im * ak * s);
        }
        const float2 wv = make_float2(a.w[0][2 * k], a.w[0][2 * k + 1]);
        const float2 wt = make_float2(a.w[1][2 * k], a.w[1][2 * k + 1]);
        const float2 wf = make_float2(a.w[2][2 * k], a.w[2][2 * k + 1]);
        const float2 p = cmul(ft, fi);
        const float2 dp = cmulc(dy[2], wf);
        float2 dfi = cmulc(dy[0], wv), dft = cmulc(dy[1], wt);
        const float2 a1 = cmulc(dp, ft), a2 = cmulc(dp, fi);
        dfi = make_float2(dfi.x + a1.x, dfi.y + a1.y);
        dft = make_float2(dft.x + a2.x, dft.y + a2.y);
        const float2 dwv = cmulc(dy[0], fi), dwt = cmulc(dy[1], ft), dwf = cmulc(dy[2], p);
        if (kv) {
            df[r][0][0][k] = dfi.x;
            df[r][0][1][k] = dfi.y;
            df[r][1][0][k] = dft.x;
            df[r][1][1][k] = dft.y;
        }
        // sum the 8 rows of this wave that share bin k (lanes sub, sub+8, ..., sub+56)
        float c6[6] = {dwv.x, dwv.y, dwt.x, dwt.y, dwf.x, dwf.y};
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            float v = c6[q];
            v += __shfl_xor(v, 8, kWave);
            v += __shfl_xor(v, 16, kWave);
            v += __shfl_xor(v, 32, kWave);
            c6[q] = v;
        }
        if (kv && (threadIdx.x & 63) < 8) {
            const int w = threadIdx.x >> 6;
#pragma unroll
            for (int q = 0; q < 6; ++q) dws[w][q >> 1][q & 1][k] = c6[q];
        }
    }
    __syncthreads();
    // per-block d weight partial, waves summed in order (deterministic)
    for (int e = threadIdx.x; e < 3 * NB * 2; e += 256) {
        const int m = e / (2 * NB), k = (e / 2) % NB, c = e & 1;
        const float acc = ((dws[0][m][c][k] + dws[1][m][c][k]) + dws[2][m][c][k]) + dws[3][m][c][k];
        a.gw[((int64_t)blockIdx.x * 3 + m) * NB * 2 + k * 2 + c] = acc;
    }
    const int64_t row = row0 + r;
    if (row >= a.n) return;
    // d x[t] = sum_k (dF_re cos - dF_im sin) / sqrt(D)
    for (int t = sub; t < D; t += 8) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            float acc = 0.f;
            for (int k = 0; k < NB; ++k) {
                const int e = (k * t) & (D - 1);
                acc = fmaf(df[r][m][0][k], twc[e], acc);
                acc = fmaf(-df[r][m][1][k], tws[e], acc);
            }
            a.gx[m][row * D + t] = acc * s;
        }
    }
}

}  // namespace rsx

using namespace rsx;

extern "C" int rsx_smore_spectral_fwd(const float* V, int32_t dv, const float* Wv, const float* bv, const float* T,
                                      int32_t dt, const float* Wt, const float* bt, const float* wv, const float* wt,
                                      const float* wf, int64_t n_items, int32_t d, float* img, float* txt,
                                      float* conv_v, float* conv_t, float* conv_f, rsx_stream_t stream) {
    if (n_items < 0 || dv <= 0 || dt <= 0 || (dv & 3) || (dt & 3)) return RSX_ERR_ARG;
    if (!V || !Wv || !bv || !T || !Wt || !bt || !wv || !wt || !wf || !img || !txt || !conv_v || !conv_t || !conv_f)
        return RSX_ERR_ARG;
    if (n_items == 0) return RSX_OK;
    SpecFwdArgs a;
    a.X[0] = V;
    a.X[1] = T;
    a.K[0] = dv;
    a.K[1] = dt;
    a.W[0] = Wv;
    a.W[1] = Wt;
    a.b[0] = bv;
    a.b[1] = bt;
    a.w[0] = wv;
    a.w[1] = wt;
    a.w[2] = wf;
    a.n = n_items;
    a.xo[0] = img;
    a.xo[1] = txt;
    a.conv[0] = conv_v;
    a.conv[1] = conv_t;
    a.conv[2] = conv_f;
    const dim3 g((unsigned)((n_items + 31) / 32));
    hipStream_t s = as_stream(stream);
    switch (d) {
        case 64: hipLaunchKernelGGL(smore_spec_fwd<64>, g, dim3(256), 0, s, a); break;
        case 128: hipLaunchKernelGGL(smore_spec_fwd<128>, g, dim3(256), 0, s, a); break;
        default: return RSX_ERR_UNSUPPORTED;
    }
    return last_rc();
}

extern "C" size_t rsx_smore_spectral_bwd_partials(int64_t n_items, int32_t d) {
    return (size_t)((n_items + 31) / 32) * 3 * (size_t)(d / 2 + 1) * 2;
}

extern "C" int rsx_smore_spectral_bwd(const float* img, const float* txt, const float* wv, const float* wt,
                                      const float* wf, const float* g_v, const float* g_t, const float* g_f,
                                      int64_t n_items, int32_t d, float* g_img, float* g_txt, float* g_w_partial,
                                      rsx_stream_t stream) {
    if (n_items < 0 || !img || !txt || !wv || !wt || !wf || !g_img || !g_txt || !g_w_partial) return RSX_ERR_ARG;
    if (n_items == 0) return RSX_OK;
    SpecBwdArgs a;
    a.xo[0] = img;
    a.xo[1] = txt;
    a.w[0] = wv;
    a.w[1] = wt;
    a.w[2] = wf;
    a.g[0] = g_v;
    a.g[1] = g_t;
    a.g[2] = g_f;
    a.n = n_items;
    a.gx[0] = g_img;
    a.gx[1] = g_txt;
    a.gw = g_w_partial;
    const dim3 g((unsigned)((n_items + 31) / 32));
    hipStream_t s = as_stream(stream);
    switch (d) {
        case 64: hipLaunchKernelGGL(smore_spec_bwd<64>, g, dim3(256), 0, s, a); break;
        case 128: hipLaunchKernelGGL(smore_spec_bwd<128>, g, dim3(256), 0, s, a); break;
        default: return RSX_ERR_UNSUPPORTED;
    }
    return last_rc();
}

// smore.hip — SMORE's modality projection + spectral denoise / cross-modal fusion
// (reference src/models/smore.py:209-237 spectrum_convolution and :256-259
// image_trs / text_trs) and the backward of the spectral part, all on fp32 MFMA
// (exact f32 products, f32 sums: the same arithmetic as an fmaf chain).
//
// 1. smore_proj: img = V W_v^T, txt = T W_t^T (v_mfma_f32_32x32x2f32), an LDS-staged
//    GEMM; the feature width K (4096 raw image / 384 text at Amazon-baby, 768 CLIP at
//    clothing) is split over blocks where it is long, the splits (and the bias) are
//    added in order by smore_spec_fwd as it loads the rows.
// 2. smore_spec_fwd: a length-d real DFT is a d x (d+2) real matrix, so
//    rfft(norm='ortho') of 16 items is a [(d+2) x d] x [d x 16] product on
//    v_mfma_f32_16x16x4f32: the rows (Re, Im of bin b at 2b, 2b+1) come from an LDS
//    twiddle table with 1/sqrt(d) folded in, the items are the MFMA's columns.  The
//    accumulator of one MFMA holds (Re, Im) pairs of whole bins per lane, so the
//    per-bin complex weights (unit-normalised by the caller, reference :221-229)
//    and the cross-modal product Ft*Fi*wf are register ops, and those registers
//    feed the three irfft products directly as B operands (the k index of an MFMA
//    may be permuted freely as long as A uses the same permutation): no LDS
//    transposes.  One wave = 16 items, no block-level synchronisation.
// 3. smore_spec_bwd_freq / _feat: dY = irfft^T(d conv) (the same matrices transposed), the
//    complex product rules against the spectra the forward saved, d w per block
//    (lane-group reductions, waves added in order: deterministic), d img / d txt
//    = rfft^T(dF).  The projection gradients
//    (dW = d img^T V on the split-K kernel, dV = d img W, db) are left to the caller.
#include <cstdlib>
#include <type_traits>

#include "rsx_common.hpp"
#include "smore_fld.hpp"

namespace rsx {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// projection
// ---------------------------------------------------------------------------
// out_m = X_m W_m^T (bias added by smore_spec_fwd) as an LDS-staged GEMM: a block
// owns 64 items x all d features of one modality and one K range (split s of S_m:
// the 4096-wide raw image features are split so that the grid fills the chip);
// K is streamed in 32-wide chunks, float4 global loads two chunks ahead, LDS
// double-buffered.  Waves: item tile (w & 1) x feature tiles {w >> 1, + 2, ...}.
constexpr int kPjItems = 64, kPjK = 32, kPjPad = 36;

__device__ __forceinline__ float f4_at(const float4& v, int i) {  // i: a compile-time constant after unrolling
    return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}

struct SpecProjArgs {
    const float* X[2];  // V [n, K0], T [n, K1]
    int32_t K[2];
    const float* W[2];  // [d, K]
    int64_t n;
    int32_t S[2];       // K splits per modality
    int32_t tiles;      // item tiles (ceil(n / 64))
    float* out[2][8];   // split s of modality m: [n, d] (s = 0: img / txt themselves)
};

// LDS floats of one projection block: X and W chunks, double-buffered
template <int D>
constexpr int kPjLds = 2 * kPjItems * kPjPad + 2 * D * kPjPad;

// Block `bid`'s share of the projection (all 256 threads); returns its item tile.
// lds: kPjLds<D> floats.  DS > D (smore_proj_half): the block computes output features
// [fh D, fh D + D) of rows DS wide, from W's rows fh D .. fh D + D - 1.
template <int D, int DS = D>
__device__ __forceinline__ int proj_block(const SpecProjArgs& a, int bid, float* __restrict__ lds, int fh = 0) {
    constexpr int FT = D / 32;            // feature tiles
    constexpr int TPW = 2 * FT / 4;       // tiles per wave (FT/2: 1 for d=64, 2 for d=128)
    constexpr int NX = kPjItems * kPjK / 4, NW = D * kPjK / 4;  // float4s per chunk
    constexpr int PER = (NX + NW) / 256;
    static_assert((NX + NW) % 256 == 0, "chunk split");
    float (*xs)[kPjItems * kPjPad] = reinterpret_cast<float (*)[kPjItems * kPjPad]>(lds);
    float (*ws)[D * kPjPad] = reinterpret_cast<float (*)[D * kPjPad]>(lds + 2 * kPjItems * kPjPad);
    // blocks: modality 0 splits, then modality 1 splits, each over the item tiles
    const int nb0 = a.tiles * a.S[0];
    const int m = bid < nb0 ? 0 : 1;
    if (m) bid -= nb0;
    const int S = a.S[m];
    const int tile = bid % a.tiles, sp = bid / a.tiles;
    const float* __restrict__ X = a.X[m];
    const int K = a.K[m];
    const float* __restrict__ W = a.W[m] + (int64_t)fh * D * K;
    const int nch_all = (K + kPjK - 1) / kPjK;
    const int per = (nch_all + S - 1) / S;
    const int c_beg = sp * per, c_end = min(nch_all, c_beg + per);
    const int nch = max(0, c_end - c_beg);
    const int64_t i0 = (int64_t)tile * kPjItems;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 31, h = lane >> 5;
    const int it = wave & 1;              // item tile of this wave
    floatx16 acc[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[q][e] = 0.f;
    float4 st[2][PER];
    auto gload = [&](int c, float4(&v)[PER]) __attribute__((always_inline)) {
        const int k0 = (c_beg + c) * kPjK;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int e = threadIdx.x + 256 * q;
            float4 t = f4(0.f);
            if (e < NX) {
                const int r = e / (kPjK / 4), kk = k0 + (e % (kPjK / 4)) * 4;
                const int64_t row = i0 + r;
                if (row < a.n && kk < K) t = ld4(X + row * K + kk);
            } else {
                const int e2 = e - NX;
                const int r = e2 / (kPjK / 4), kk = k0 + (e2 % (kPjK / 4)) * 4;
                if (kk < K) t = ld4(W + (int64_t)r * K + kk);
            }
            v[q] = t;
        }
    };
    auto sstore = [&](int b, const float4(&v)[PER]) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int e = threadIdx.x + 256 * q;
            if (e < NX)
                *reinterpret_cast<float4*>(&xs[b][(e / (kPjK / 4)) * kPjPad + (e % (kPjK / 4)) * 4]) = v[q];
            else
                *reinterpret_cast<float4*>(&ws[b][((e - NX) / (kPjK / 4)) * kPjPad + ((e - NX) % (kPjK / 4)) * 4]) =
                    v[q];
        }
    };
    if (nch > 0) {
        gload(0, st[0]);
        if (nch > 1) gload(1, st[1]);
        sstore(0, st[0]);
    }
    __syncthreads();
    auto step = [&](int c, auto bc) __attribute__((always_inline)) {
        constexpr int B = decltype(bc)::value;
        if (c + 2 < nch) gload(c + 2, st[B]);
        // the chunk's K order permuted (A and B alike): MFMA step u, lane half h takes
        // k = 16 h + u, so a lane's 16 operands of a chunk are contiguous in its LDS row
        // (four 16-B reads per operand instead of sixteen 4-B reads; rows padded to 36
        // floats: 16 lanes' 16-B reads hit distinct banks)
        float4 av[4], bv[TPW][4];
        const float* xb = xs[B] + (it * 32 + j) * kPjPad + 16 * h;
#pragma unroll
        for (int r = 0; r < 4; ++r) av[r] = *reinterpret_cast<const float4*>(xb + 4 * r);
#pragma unroll
        for (int q = 0; q < TPW; ++q) {
            const float* wb = ws[B] + (((wave >> 1) + 2 * q) * 32 + j) * kPjPad + 16 * h;
#pragma unroll
            for (int r = 0; r < 4; ++r) bv[q][r] = *reinterpret_cast<const float4*>(wb + 4 * r);
        }
#pragma unroll
        for (int u = 0; u < kPjK / 2; ++u) {
            const float a_u = f4_at(av[u >> 2], u & 3);
#pragma unroll
            for (int q = 0; q < TPW; ++q)
                acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a_u, f4_at(bv[q][u >> 2], u & 3), acc[q], 0, 0, 0);
        }
        if (c + 1 < nch) sstore(B ^ 1, st[B ^ 1]);
        __syncthreads();
    };
    for (int c = 0; c < nch; c += 2) {  // block-uniform
        step(c, std::integral_constant<int, 0>{});
        if (c + 1 < nch) step(c + 1, std::integral_constant<int, 1>{});
    }
    // C layout: lane holds column (feature) ft*32 + j, rows (items) it*32 + (e&3) + 8(e>>2) + 4h
    float* out = a.out[m][sp] + fh * D;
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int f = ((wave >> 1) + 2 * q) * 32 + j;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int64_t row = i0 + it * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
            if (row < a.n) out[row * DS + f] = acc[q][e];
        }
    }
    return tile;
}

template <int D>
__global__ __launch_bounds__(256) void smore_proj(SpecProjArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[kPjLds<D>];
    proj_block<D>(a, blockIdx.x, lds);
}

// smore_proj at d = 128 as two blocks per (item tile, K split), one per half of the output
// features: the d = 64 block's LDS footprint (37 KB instead of 55 KB: four blocks a CU, not
// two), so twice the waves hide the K-chunk loads.  The two halves of a pair are blocks
// b and b + 8 (the same XCD under the round-robin deal): the X chunks come from its L2 for
// the second.  Same products in the same K order: the results are smore_proj<128>'s bits.
// Grid: 16 * ceil(nb / 8) for nb = tiles * (S0 + S1); blocks past nb exit.
template <int D>
__global__ __launch_bounds__(256) void smore_proj_half(SpecProjArgs a, int nb) {
    __shared__ __attribute__((aligned(16))) float lds[kPjLds<D / 2>];
    const int b = blockIdx.x;
    const int bid = (b & 7) | ((b >> 4) << 3);
    if (bid >= nb) return;
    proj_block<D / 2, D>(a, bid, lds, (b >> 3) & 1);
}

// ---------------------------------------------------------------------------
// spectral part on 16x16x4 MFMAs
// ---------------------------------------------------------------------------
template <int D>
struct Spec {
    static constexpr int NB = D / 2 + 1;          // rfft bins
    static constexpr int MR = 2 * NB;             // real rows (Re, Im per bin)
    static constexpr int MT = (MR + 15) / 16;     // 16-row tiles of the spectrum
    static constexpr int SI = D / 4;              // MFMA steps over the d features
    static constexpr int OT = D / 16;             // 16-row tiles of the d features
};

__device__ __forceinline__ int opaque(int x) {
    asm volatile("" : "+v"(x));
    return x;
}
// The coefficient reads of one MFMA step group must not be hoisted into earlier groups
// (a fully unrolled loop otherwise loads every group up front: hundreds of live
// registers, spills).  tie() "rewrites" the previous group's coefficients after the
// MFMAs that read them, and the next group's table offset passes through opaque()
// after it: volatile asm keeps that order, so the next reads cannot pass those MFMAs
// (and still overlap their execution).
template <int N>
__device__ __forceinline__ void tie(float4 (&c)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(c[i].x), "+v"(c[i].y), "+v"(c[i].z), "+v"(c[i].w));
}

__device__ __forceinline__ floatx4 mfma16(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float f4c(const float4& v, int i) {  // i: a compile-time constant after unrolling
    return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {  // a * conj(b)
    return make_float2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}

// tw[e] = cos(2 pi e / D) / sqrt(D), tw[D + e] = -sin(2 pi e / D) / sqrt(D)  (norm='ortho')
template <int D>
__device__ __forceinline__ void twiddles(float* tw) {
    const double r = 1.0 / sqrt((double)D);
    for (int t = threadIdx.x; t < D; t += blockDim.x) {
        double s, c;
        sincospi(2.0 * (double)t / (double)D, &s, &c);
        tw[t] = (float)(c * r);
        tw[D + t] = (float)(-s * r);
    }
}

// rfft matrix: row j (Re of bin j/2 for even j, Im for odd j), feature f
template <int D>
__device__ __forceinline__ float fwd_coef(int j, int f, const float* tw) {
    const float v = tw[(((j >> 1) * f) & (D - 1)) + (j & 1) * D];
    return j < Spec<D>::MR ? v : 0.f;
}

// irfft matrix: output feature t, spectrum row j; bins 0 and D/2 once (their
// imaginary parts drop out: sin 0 = sin(pi t) = 0), the others twice
template <int D>
__device__ __forceinline__ float inv_coef(int t, int j, const float* tw) {
    const int b = j >> 1;
    const float v = tw[((b * t) & (D - 1)) + (j & 1) * D];
    const float c = (b == 0 || b == D / 2) ? 1.f : 2.f;
    return j < Spec<D>::MR ? c * v : 0.f;
}

// ---------------------------------------------------------------------------
// coefficient tables: the DFT matrices as MFMA A operands in LDS, in the order the
// MFMA steps read them (one conflict-free ds_read_b128 per lane = four steps' operands,
// at a constant offset: no index arithmetic, no twiddle-table bank conflicts).  The
// spectrum's last 16-row tile holds 2 real rows (Re / Im of bin D/2: MR = D + 2 =
// 16 (MT - 1) + 2), so its operands are stored compactly and the other lanes read 0.
// ---------------------------------------------------------------------------
template <int D>
struct Tab {
    static constexpr int MT = Spec<D>::MT, Q = D / 16;       // Q: step groups (SI / 4) = feature tiles (OT)
    static constexpr int kMain = (MT - 1) * Q * 64;          // float4s of the full tiles
    static constexpr int kFloats = 4 * (kMain + 8 * Q);      // + the compact last tile
};

// k-step layout (rfft over the features / the irfft's transpose): entry (t, q), lane
// (n, g), component r = coef(spectrum row j = 16 t + n, feature f = g SI + 4 q + r)
template <int D, class F>
__device__ __forceinline__ void tab_ks(float4* __restrict__ tab, F coef) {
    using T = Tab<D>;
    constexpr int SI = Spec<D>::SI;
    for (int e = threadIdx.x; e < T::kMain; e += blockDim.x) {
        const int lane = e & 63, tq = e >> 6, t = tq / T::Q, q = tq % T::Q;
        const int j = 16 * t + (lane & 15), f0 = (lane >> 4) * SI + 4 * q;
        tab[e] = make_float4(coef(j, f0), coef(j, f0 + 1), coef(j, f0 + 2), coef(j, f0 + 3));
    }
    for (int e = threadIdx.x; e < 8 * T::Q; e += blockDim.x) {
        const int n = e & 1, g = (e >> 1) & 3, q = e >> 3;
        const int j = 16 * (T::MT - 1) + n, f0 = g * SI + 4 * q;
        tab[T::kMain + e] = make_float4(coef(j, f0), coef(j, f0 + 1), coef(j, f0 + 2), coef(j, f0 + 3));
    }
}
template <int D>
__device__ __forceinline__ float4 ks_at(const float4* __restrict__ tab, int base, int t, int q, int lane) {
    using T = Tab<D>;
    if (t < T::MT - 1) return tab[base + (t * T::Q + q) * 64];
    const float4 v = tab[T::kMain + (q * 4 + (lane >> 4)) * 2 + (lane & 1)];
    return (lane & 15) < 2 ? v : f4(0.f);
}

// output-tile layout (rfft^T onto the features / the irfft): entry (tau, t), lane
// (n, g), component i = coef(spectrum row j = 16 t + 4 g + i, output o = 16 tau + n)
template <int D, class F>
__device__ __forceinline__ void tab_ot(float4* __restrict__ tab, F coef) {
    using T = Tab<D>;
    for (int e = threadIdx.x; e < T::kMain; e += blockDim.x) {
        const int lane = e & 63, tt = e >> 6, tau = tt / (T::MT - 1), t = tt % (T::MT - 1);
        const int j0 = 16 * t + 4 * (lane >> 4), o = 16 * tau + (lane & 15);
        tab[e] = make_float4(coef(j0, o), coef(j0 + 1, o), coef(j0 + 2, o), coef(j0 + 3, o));
    }
    float2* last = reinterpret_cast<float2*>(tab + T::kMain);
    for (int e = threadIdx.x; e < 16 * T::Q; e += blockDim.x) {
        const int j0 = 16 * (T::MT - 1), o = 16 * (e >> 4) + (e & 15);
        last[e] = make_float2(coef(j0, o), coef(j0 + 1, o));
    }
}
template <int D>
__device__ __forceinline__ float4 ot_at(const float4* __restrict__ tab, int base, int tau, int t, int lane) {
    using T = Tab<D>;
    if (t < T::MT - 1) return tab[base + (tau * (T::MT - 1) + t) * 64];
    const float2 v = reinterpret_cast<const float2*>(tab + T::kMain)[tau * 16 + (lane & 15)];
    return (lane >> 4) == 0 ? make_float4(v.x, v.y, 0.f, 0.f) : f4(0.f);
}

// B operand of 16 item rows: lane (g = l>>4, n = l&15) holds x[item][g*SI + s] for
// step s (contiguous: float4 loads)
template <int D>
__device__ __forceinline__ void load_rows(const float* __restrict__ x, int64_t item, bool ok, int g,
                                          float (&v)[Spec<D>::SI]) {
    constexpr int SI = Spec<D>::SI;
    const float* p = x + (ok ? item : 0) * D + g * SI;
#pragma unroll
    for (int q = 0; q < SI / 4; ++q) {
        const float4 t = (ok && x) ? ld4(p + 4 * q) : f4(0.f);
        v[4 * q] = t.x;
        v[4 * q + 1] = t.y;
        v[4 * q + 2] = t.z;
        v[4 * q + 3] = t.w;
    }
}

// acc[t] += sum_s A_t(s) x[s] over the SI steps (k-step table): the rfft of 16 items
// (fwd table; two signals) or irfft^T of a gradient (inv table; one signal).  F[t]
// (t < MT): lane (g, n) holds rows 16t + 4g + i, i.e. the (Re, Im) of bins 8t + 2g and
// 8t + 2g + 1 of item n
template <int D, int NS, int T0 = 0, int NT = Spec<D>::MT>
__device__ __forceinline__ void ks_product(const float4* __restrict__ tab, const float (*x[NS])[Spec<D>::SI],
                                           floatx4 (*acc[NS])[NT], int lane) {
    constexpr int Q = Tab<D>::Q;  // (tiles T0 .. T0 + NT - 1 of the spectrum only)
#pragma unroll
    for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int t = 0; t < NT; ++t) (*acc[k])[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    float4 c[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) c[t] = f4(0.f);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        tie(c);
        const int base = opaque(lane);
#pragma unroll
        for (int t = 0; t < NT; ++t) c[t] = ks_at<D>(tab, base, T0 + t, q, lane);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int k = 0; k < NS; ++k) (*acc[k])[t] = mfma16(f4c(c[t], r), (*x[k])[4 * q + r], (*acc[k])[t]);
    }
}

// ks_product for one signal read straight from its rows [n, D] (the B operand of step
// 4q + r is x[g SI + 4q + r]: one float4 per step group, the next group's in flight)
// instead of a register copy of the whole row slice: SI - 8 fewer live registers
template <int D, int T0, int NT>
__device__ __forceinline__ void ks_product_rows(const float4* __restrict__ tab, const float* __restrict__ x,
                                                int64_t item, bool ok, int g, floatx4 (&acc)[NT], int lane) {
    constexpr int Q = Tab<D>::Q, SI = Spec<D>::SI;
    const float* p = x + (ok ? item : 0) * D + g * SI;
    const bool ld = ok && x;
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    float4 c[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) c[t] = f4(0.f);
    float4 xv = ld ? ld4(p) : f4(0.f);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        tie(c);
        const int base = opaque(lane);
#pragma unroll
        for (int t = 0; t < NT; ++t) c[t] = ks_at<D>(tab, base, T0 + t, q, lane);
        const float4 xn = (ld && q + 1 < Q) ? ld4(p + 4 * (q + 1)) : f4(0.f);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = mfma16(f4c(c[t], r), f4c(xv, r), acc[t]);
        xv = xn;
    }
}

__device__ __forceinline__ float2 pair(const floatx4& v, int p) { return make_float2(v[2 * p], v[2 * p + 1]); }
__device__ __forceinline__ void set_pair(floatx4& v, int p, float2 x) {
    v[2 * p] = x.x;
    v[2 * p + 1] = x.y;
}

struct SpecFwdArgs {
    float* x[2];        // img, txt [n, d]: projection split 0 in, the final projection out
    const float* part[2][8];  // projection splits 1.. (S[m] - 1 of them)
    int32_t S[2];
    const float* b[2];  // biases [d]
    const float* w[3];  // unit complex weights [(d/2+1)][2]: image, text, fusion
    int64_t n;
    float* conv[3];     // conv_v, conv_t, conv_f [n, d]
    float* spec;        // saved spectra [n][2][16 MT] (Fi, Ft) for the backward
};

// saved spectrum of item `item`, signal `sig`, rows 16t + 4g .. 16t + 4g + 3
template <int D>
__device__ __forceinline__ int64_t spec_off(int64_t item, int sig, int t, int g) {
    return (item * 2 + sig) * (16 * Spec<D>::MT) + 16 * t + 4 * g;
}

// the projection rows of modality m for the 16 items (B layout, see load_rows):
// split 0 + split 1 + ... + bias, in that order; written back as img / txt
template <int D>
__device__ __forceinline__ void proj_rows(const SpecFwdArgs& a, int m, int64_t item, bool iv, int g,
                                          float (&v)[Spec<D>::SI]) {
    constexpr int SI = Spec<D>::SI;
    load_rows<D>(a.x[m], item, iv, g, v);
    for (int s = 1; s < a.S[m]; ++s) {
        float p[SI];
        load_rows<D>(a.part[m][s], item, iv, g, p);
#pragma unroll
        for (int k = 0; k < SI; ++k) v[k] += p[k];
    }
    const float* bias = a.b[m] + g * SI;
#pragma unroll
    for (int q = 0; q < SI / 4; ++q) {
        const float4 bb = ld4(bias + 4 * q);
        v[4 * q] += bb.x;
        v[4 * q + 1] += bb.y;
        v[4 * q + 2] += bb.z;
        v[4 * q + 3] += bb.w;
    }
    if (iv) {
        float* o = a.x[m] + item * D + g * SI;
#pragma unroll
        for (int q = 0; q < SI / 4; ++q) st4(o + 4 * q, make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]));
    }
}

// LDS of the spectral part (floats): one coefficient table, the twiddles (2 D), the
// three unit complex weight vectors (3 NB float2s)
template <int D>
constexpr int kSpecLds = Tab<D>::kFloats + 2 * D + 6 * Spec<D>::NB;

template <int D>
__device__ __forceinline__ void spec_setup(const SpecFwdArgs& a, float* __restrict__ lds) {
    constexpr int NB = Spec<D>::NB;
    float* tw = lds + Tab<D>::kFloats;
    twiddles<D>(tw);
    float2* ws = reinterpret_cast<float2*>(tw + 2 * D);
    for (int e = threadIdx.x; e < 3 * NB; e += blockDim.x)
        ws[e] = make_float2(a.w[e / NB][2 * (e % NB)], a.w[e / NB][2 * (e % NB) + 1]);
    __syncthreads();
    tab_ks<D>(reinterpret_cast<float4*>(lds), [&](int j, int f) { return fwd_coef<D>(j, f, tw); });
    __syncthreads();
}

// The spectral part of one 64-item tile (4 waves x 16 items; all 256 threads, block-
// uniform: it rebuilds the LDS table between the rfft and the irfft; spec_setup before)
template <int D>
__device__ __forceinline__ void spec_tile(const SpecFwdArgs& a, int64_t tile, float* __restrict__ lds) {
    using S = Spec<D>;
    constexpr int SI = S::SI, MT = S::MT, NB = S::NB, OT = S::OT;
    const float4* tab = reinterpret_cast<const float4*>(lds);
    const float* tw = lds + Tab<D>::kFloats;
    const float2(*ws)[NB] = reinterpret_cast<const float2(*)[NB]>(tw + 2 * D);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, n16 = lane & 15, g = lane >> 4;
    const int64_t item = (tile * 4 + wave) * 16 + n16;
    const bool iv = item < a.n;  // a wave past the end runs on zeros (MFMAs need the whole wave)
    floatx4 fi[MT], ft[MT], yf[MT];
    {
        float xi[SI], xt[SI];
        proj_rows<D>(a, 0, item, iv, g, xi);
        proj_rows<D>(a, 1, item, iv, g, xt);
        const float (*xs[2])[SI] = {&xi, &xt};
        floatx4 (*accs[2])[MT] = {&fi, &ft};
        ks_product<D, 2>(tab, xs, accs, lane);
    }
    __syncthreads();  // every wave is done with the rfft table
    tab_ot<D>(reinterpret_cast<float4*>(lds), [&](int j, int o) { return inv_coef<D>(o, j, tw); });
    if (iv) {
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            st4(a.spec + spec_off<D>(item, 0, t, g), make_float4(fi[t][0], fi[t][1], fi[t][2], fi[t][3]));
            st4(a.spec + spec_off<D>(item, 1, t, g), make_float4(ft[t][0], ft[t][1], ft[t][2], ft[t][3]));
        }
    }
    // filtered spectra: Yv = Fi wv, Yt = Ft wt, Yf = (Ft Fi) wf  (in place for v, t)
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int b = 8 * t + 2 * g + p;
            const bool bv = b < NB;
            const int bb = bv ? b : 0;
            const float2 Fi = pair(fi[t], p), Ft = pair(ft[t], p);
            const float2 z = make_float2(0.f, 0.f);
            set_pair(fi[t], p, bv ? cmul(Fi, ws[0][bb]) : z);
            set_pair(ft[t], p, bv ? cmul(Ft, ws[1][bb]) : z);
            set_pair(yf[t], p, bv ? cmul(cmul(Ft, Fi), ws[2][bb]) : z);
        }
    __syncthreads();  // the irfft table is complete
    // conv_m = irfft(Y_m): output tile tau, step (t, i) <-> spectrum row 16t + 4g + i
#pragma unroll
    for (int tau = 0; tau < OT; ++tau) {
        floatx4 cv{0.f, 0.f, 0.f, 0.f}, ct = cv, cf = cv;
        float4 c[1] = {f4(0.f)};
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            tie(c);
            c[0] = ot_at<D>(tab, opaque(lane), tau, t, lane);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                cv = mfma16(f4c(c[0], i), fi[t][i], cv);
                ct = mfma16(f4c(c[0], i), ft[t][i], ct);
                cf = mfma16(f4c(c[0], i), yf[t][i], cf);
            }
        }
        if (iv) {  // lane (g, n) holds features 16 tau + 4g + r of item n
            const int64_t o = item * D + 16 * tau + 4 * g;
            st4(a.conv[0] + o, make_float4(cv[0], cv[1], cv[2], cv[3]));
            st4(a.conv[1] + o, make_float4(ct[0], ct[1], ct[2], ct[3]));
            st4(a.conv[2] + o, make_float4(cf[0], cf[1], cf[2], cf[3]));
        }
    }
}

template <int D>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void smore_spec_fwd(SpecFwdArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[kSpecLds<D>];
    spec_setup<D>(a, lds);
    spec_tile<D>(a, blockIdx.x, lds);
}

struct SpecBwdArgs {
    const float* spec;  // the forward's saved spectra [n][2][16 MT]
    const float* w[3];
    const float* g[3];  // d conv_v / conv_t / conv_f [n, d] (NULL = 0)
    int64_t n;
    float* gx[2];       // d img, d txt [n, d]
    float* gw;          // [gridDim.x][3][d/2+1][2] per-block partials
    float* dfreq;       // [waves][2][MT][64][4]: dFi, dFt between the two passes
};

// the sum over the 16 items (lanes n = 0..15 of lane group g) of x, in lane n == 0
__device__ __forceinline__ float sum16(float x) {
    x += __shfl_xor(x, 1, kWave);
    x += __shfl_xor(x, 2, kWave);
    x += __shfl_xor(x, 4, kWave);
    x += __shfl_xor(x, 8, kWave);
    return x;
}

// The backward in two passes, each small enough in live state to run two waves a SIMD
// (one pass holding every spectrum of 16 items needed 508 registers and 82 KB of LDS
// at d = 128: one wave a SIMD, 1.4 rounds of the chip at C5).
// 1. smore_spec_bwd_freq: dY_f, dY_v, dY_t = irfft^T(d conv_f / _v / _t) (k-step table of
//    the irfft matrix); dp = dY_f conj(wf) held in registers; dFi = dY_v conj(wv) +
//    dp conj(Ft), dFt = dY_t conj(wt) + dp conj(Fi) stored per wave, lane-contiguous
//    (each float4 store a 1 KB run); d w per block.
// 2. smore_spec_bwd_feat: d img = rfft^T(dFi), d txt = rfft^T(dFt) (output-tile table of
//    the rfft matrix).
template <int D>
__device__ __forceinline__ int64_t dfreq_off(int64_t gwave, int sig, int t, int lane) {
    return (((gwave * 2 + sig) * Spec<D>::MT + t) * 64 + lane) * 4;
}

template <int D>
constexpr int kBwdFreqLds = Tab<D>::kFloats + 2 * D;

// The frequency pass of 16 items on spectrum tiles T0 .. T0 + NT - 1 (one wave; the two
// halves of a block's 8 waves take the two tile ranges of the same items: twice the
// waves, each half the MFMA chain and registers)
template <int D, int T0, int NT>
__device__ __forceinline__ void freq_tiles(const SpecBwdArgs& a, const float4* __restrict__ tab,
                                           const float2 (*ws)[Spec<D>::NB], float2 (*dws)[Spec<D>::NB],
                                           int64_t gwave, int lane) {
    using S = Spec<D>;
    constexpr int MT = S::MT, NB = S::NB, SI = S::SI;
    const int n16 = lane & 15, g = lane >> 4;
    const int64_t item = gwave * 16 + n16;
    const bool iv = item < a.n;
    // the forward's spectra of tile t (lane (g, n): bins 8t + 2g, 8t + 2g + 1 of item n)
    auto spec4 = [&](int sig, int t) __attribute__((always_inline)) {
        const float4 v = iv ? ld4(a.spec + spec_off<D>(item, sig, t, g)) : f4(0.f);
        return floatx4{v.x, v.y, v.z, v.w};
    };
    // d w of bin b (summed over the wave's 16 items) into dws[m][b]
    auto put_dw = [&](int m, int b, bool bv, float2 dw) __attribute__((always_inline)) {
        dw.x = sum16(dw.x);
        dw.y = sum16(dw.y);
        if (n16 == 0 && bv) dws[m][b] = dw;
    };
    auto store_df = [&](int sig, const floatx4 (&v)[NT]) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
            st4(a.dfreq + dfreq_off<D>(gwave, sig, T0 + t, lane), make_float4(v[t][0], v[t][1], v[t][2], v[t][3]));
    };
    // dY = irfft^T(d conv_m) for the 16 items, in the spectrum layout
    auto irfft_t = [&](int m, floatx4 (&dy)[NT]) __attribute__((always_inline)) {
        ks_product_rows<D, T0, NT>(tab, a.g[m], item, iv, g, dy, lane);
    };
    floatx4 dy[NT], dp[NT];
    irfft_t(2, dy);
#pragma unroll
    for (int u = 0; u < NT; ++u) {
        const int t = T0 + u;
        const floatx4 fi4 = spec4(0, t), ft4 = spec4(1, t);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int b = 8 * t + 2 * g + p;
            const bool bv = b < NB;
            const float2 dY = pair(dy[u], p);
            put_dw(2, b, bv, cmulc(dY, cmul(pair(ft4, p), pair(fi4, p))));
            set_pair(dp[u], p, bv ? cmulc(dY, ws[2][bv ? b : 0]) : make_float2(0.f, 0.f));
        }
    }
    // image: dFi = dYv conj(wv) + dp conj(Ft)
    irfft_t(0, dy);
#pragma unroll
    for (int u = 0; u < NT; ++u) {
        const int t = T0 + u;
        const floatx4 fi4 = spec4(0, t), ft4 = spec4(1, t);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int b = 8 * t + 2 * g + p;
            const bool bv = b < NB;
            const float2 dY = pair(dy[u], p);
            put_dw(0, b, bv, cmulc(dY, pair(fi4, p)));
            const float2 uu = bv ? cmulc(dY, ws[0][bv ? b : 0]) : make_float2(0.f, 0.f);
            const float2 v = cmulc(pair(dp[u], p), pair(ft4, p));
            set_pair(dy[u], p, make_float2(uu.x + v.x, uu.y + v.y));
        }
    }
    store_df(0, dy);
    // text: dFt = dYt conj(wt) + dp conj(Fi)
    irfft_t(1, dy);
#pragma unroll
    for (int u = 0; u < NT; ++u) {
        const int t = T0 + u;
        const floatx4 fi4 = spec4(0, t), ft4 = spec4(1, t);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int b = 8 * t + 2 * g + p;
            const bool bv = b < NB;
            const float2 dY = pair(dy[u], p);
            put_dw(1, b, bv, cmulc(dY, pair(ft4, p)));
            const float2 uu = bv ? cmulc(dY, ws[1][bv ? b : 0]) : make_float2(0.f, 0.f);
            const float2 v = cmulc(pair(dp[u], p), pair(fi4, p));
            set_pair(dy[u], p, make_float2(uu.x + v.x, uu.y + v.y));
        }
    }
    store_df(1, dy);
    (void)MT;
    (void)SI;
}

template <int D>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void smore_spec_bwd_freq(SpecBwdArgs a) {
    using S = Spec<D>;
    constexpr int MT = S::MT, NB = S::NB, MTA = (MT + 1) / 2;
    __shared__ __attribute__((aligned(16))) float lds[kBwdFreqLds<D>];
    __shared__ float2 ws[3][NB];
    __shared__ float2 dws[4][3][NB];
    float* tw = lds + Tab<D>::kFloats;
    twiddles<D>(tw);
    for (int e = threadIdx.x; e < 3 * NB; e += blockDim.x)
        ws[e / NB][e % NB] = make_float2(a.w[e / NB][2 * (e % NB)], a.w[e / NB][2 * (e % NB) + 1]);
    __syncthreads();
    tab_ks<D>(reinterpret_cast<float4*>(lds), [&](int j, int f) { return inv_coef<D>(f, j, tw); });
    __syncthreads();
    const float4* tab = reinterpret_cast<const float4*>(lds);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, ig = wave & 3;
    const int64_t gwave = (int64_t)blockIdx.x * 4 + ig;
    if (wave < 4)  // wave-uniform: tiles 0 .. MTA-1, then MTA .. MT-1, of the same 16 items
        freq_tiles<D, 0, MTA>(a, tab, ws, dws[ig], gwave, lane);
    else
        freq_tiles<D, MTA, MT - MTA>(a, tab, ws, dws[ig], gwave, lane);
    __syncthreads();
    // per-block d weight partial, the four item groups added in order (deterministic; a
    // bin's dws entry comes from the one wave whose tiles hold it)
    for (int e = threadIdx.x; e < 3 * NB * 2; e += blockDim.x) {
        const int m = e / (2 * NB), k = (e / 2) % NB, c = e & 1;
        const float2 w0 = dws[0][m][k], w1 = dws[1][m][k], w2 = dws[2][m][k], w3 = dws[3][m][k];
        const float v = c ? ((w0.y + w1.y) + w2.y) + w3.y : ((w0.x + w1.x) + w2.x) + w3.x;
        a.gw[((int64_t)blockIdx.x * 3 + m) * NB * 2 + k * 2 + c] = v;
    }
}

template <int D>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void smore_spec_bwd_feat(SpecBwdArgs a) {
    constexpr int MT = Spec<D>::MT, OT = Spec<D>::OT, HT = OT / 2;  // output tiles per half
    __shared__ __attribute__((aligned(16))) float lds[kBwdFreqLds<D>];
    float* tw = lds + Tab<D>::kFloats;
    twiddles<D>(tw);
    __syncthreads();
    tab_ot<D>(reinterpret_cast<float4*>(lds), [&](int j, int o) { return fwd_coef<D>(j, o, tw); });
    __syncthreads();
    const float4* tab = reinterpret_cast<const float4*>(lds);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, n16 = lane & 15, g = lane >> 4;
    const int ig = wave & 3, h = wave >> 2;  // item group, half of the output tiles
    const int64_t gwave = (int64_t)blockIdx.x * 4 + ig;
    const int64_t item = gwave * 16 + n16;
    const bool iv = item < a.n;
#pragma unroll 1
    for (int sig = 0; sig < 2; ++sig) {
        floatx4 df[MT];
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            const float4 v = ld4(a.dfreq + dfreq_off<D>(gwave, sig, t, lane));
            df[t] = floatx4{v.x, v.y, v.z, v.w};
        }
        // d x = rfft^T(dF): output tiles in pairs (two independent accumulators), step
        // (t, i) <-> spectrum row 16t + 4g + i
#pragma unroll 1
        for (int tau = h * HT; tau < (h + 1) * HT; tau += 2) {  // rolled: one pair's coefficients live
            floatx4 a0{0.f, 0.f, 0.f, 0.f}, a1 = a0;
            float4 c[2] = {f4(0.f), f4(0.f)};
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                tie(c);
                const int base = opaque(lane);
                c[0] = ot_at<D>(tab, base, tau, t, lane);
                c[1] = ot_at<D>(tab, base, tau + 1, t, lane);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    a0 = mfma16(f4c(c[0], i), df[t][i], a0);
                    a1 = mfma16(f4c(c[1], i), df[t][i], a1);
                }
            }
            if (iv) {
                const int64_t o = item * D + 16 * tau + 4 * g;
                st4(a.gx[sig] + o, make_float4(a0[0], a0[1], a0[2], a0[3]));
                st4(a.gx[sig] + o + 16, make_float4(a1[0], a1[1], a1[2], a1[3]));
            }
        }
    }
}

// ---------------------------------------------------------------------------
// the item side in one launch: projection -> spectral part -> modality gates
// ---------------------------------------------------------------------------
// Every block runs its smore_proj share (an item tile x one modality x one K split) and
// then counts itself in at its tile; the tile's last arriver (release / acquire at agent
// scope: the other blocks' projection rows may sit in another XCD's L2) runs the
// spectral part of those 64 items and, with `item` set, the three modality gates
// (smore.py:262-272) on the conv rows its own lanes just stored.  The arithmetic is
// smore_proj + smore_spec_fwd + gates_fwd's, op for op: the results are bit-identical
// to the three-launch chain, without its two [n, d] round trips through HBM, two
// launch boundaries or the spectral part's tail (it runs while other tiles project).
struct ItemFwdArgs {
    SpecProjArgs p;
    SpecFwdArgs s;
    uint32_t* cnt;          // [tiles] arrival counters: zero, re-armed by each tile's last arriver
    const float* item;      // item_id embedding [n, D] (NULL: no gates)
    const float* gW[3];     // gate_v/t/f Linear weights [D, D] and biases
    const float* gb[3];
    float scale;            // inject_scale (residual mode)
    int32_t mul;            // inject_mode == "mul"
    float* gout[3];         // img_i, txt_i, fus_i
};

template <int D>
constexpr int kItemLds = kPjLds<D> > kSpecLds<D> ? (kPjLds<D> > D * sf::kLd<D> ? kPjLds<D> : D * sf::kLd<D>)
                                                 : (kSpecLds<D> > D * sf::kLd<D> ? kSpecLds<D> : D * sf::kLd<D>);

template <int D>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void smore_item_fwd(ItemFwdArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[kItemLds<D>];
    __shared__ int last;
    const int tile = proj_block<D>(a.p, blockIdx.x, lds);
    // publish (the split-K counter hand-off): every wave drains its projection stores, one
    // lane releases at agent scope for the block (one L2 write-back per block: a release in
    // every lane, or __threadfence(), costs several times the whole hand-off) then counts
    // the block in; the tile's last arriver acquires once and reads the other blocks' rows
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t need = (uint32_t)(a.p.S[0] + a.p.S[1]);
        const uint32_t prev = __hip_atomic_fetch_add(a.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev + 1 == need;
        if (last) {
            __hip_atomic_store(a.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!last) return;  // block-uniform
    spec_setup<D>(a.s, lds);
    spec_tile<D>(a.s, tile, lds);
    if (!a.item) return;
    // the gates: the conv rows this lane stored above (same lane, same addresses)
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int64_t r = ((int64_t)tile * 4 + (threadIdx.x >> 6)) * 16 + (lane & 15);
    const int64_t row = r < a.s.n ? r : -1;
    const sf::Fld<D> it = sf::fload<D>(a.item, row, g);
#pragma unroll 1
    for (int m = 0; m < 3; ++m) {
        const sf::Fld<D> cv = sf::fload<D>(a.s.conv[m], row, g);
        const float* W = sf::stage_w<D>(lds, a.gW[m]);  // (its barrier: the spectral part's LDS readers are done)
        const sf::Fld<D> sg = sf::fmap<D>(sf::mv_p<D, sf::kLd<D>>(W, a.gb[m], cv, lane), sf::sigm);
        const sf::Fld<D> o = a.mul ? sf::fmap2<D>(it, sg, [](float x, float y) { return x * y; })
                                   : sf::fmap2<D>(it, sg, [&](float x, float y) { return x + a.scale * y; });
        sf::fstore<D>(a.gout[m], row, g, o);
    }
}

}  // namespace rsx

using namespace rsx;

extern "C" size_t rsx_smore_spectral_spec_floats(int64_t n_items, int32_t d) {
    if (n_items <= 0) return 0;
    const int mt = d == 64 ? Spec<64>::MT : Spec<128>::MT;
    return (size_t)n_items * 2 * 16 * (size_t)mt;
}

// K splits of a projection: about 1536 blocks over both modalities, >= 512 of K per split
// (C5's 768-wide features: one split; two -- 1,440 blocks in 2.8 rounds of the 512 resident
// d = 128 blocks instead of 720 in 1.4 -- measured no faster once smore_spec_fwd sums them:
// proj 148.7 -> 138.3 us, spec_fwd 73.6 -> 82.5)
static int env_int(const char* name, int dflt) { return env_knob(name, dflt, 1, 1 << 20); }

static int proj_splits(int64_t n, int K) {
    static const int target = env_int("RSX_PROJ_TARGET", 1536), mink = env_int("RSX_PROJ_MINK", 512);
    const int64_t tiles = (n + kPjItems - 1) / kPjItems;
    int64_t s = (target + 2 * tiles - 1) / (2 * tiles);  // blocks per modality ~target (C3: 3.37 -> 3.31 ms/step at 1536 vs 512)
    const int64_t smax = K / mink > 0 ? K / mink : 1;
    if (s > smax) s = smax;
    if (s > 8) s = 8;
    return (int)(s < 1 ? 1 : s);
}

extern "C" size_t rsx_smore_spectral_fwd_ws_bytes(int64_t n_items, int32_t d, int32_t dv, int32_t dt) {
    if (n_items <= 0 || dv <= 0 || dt <= 0) return 0;
    const int64_t extra = (proj_splits(n_items, dv) - 1) + (proj_splits(n_items, dt) - 1);
    return (size_t)extra * (size_t)n_items * (size_t)d * sizeof(float);
}

// the launch arguments of the projection and the spectral part (rc != RSX_OK: invalid)
static int spectral_args(const float* V, int32_t dv, const float* Wv, const float* bv, const float* T, int32_t dt,
                         const float* Wt, const float* bt, const float* wv, const float* wt, const float* wf,
                         int64_t n_items, int32_t d, float* img, float* txt, float* conv_v, float* conv_t,
                         float* conv_f, float* spec, void* ws, size_t ws_bytes, SpecProjArgs& p, SpecFwdArgs& a) {
    if (n_items < 0 || dv <= 0 || dt <= 0 || (dv & 3) || (dt & 3)) return RSX_ERR_ARG;
    if (!V || !Wv || !bv || !T || !Wt || !bt || !wv || !wt || !wf || !img || !txt || !conv_v || !conv_t || !conv_f ||
        !spec)
        return RSX_ERR_ARG;
    if (d != 64 && d != 128) return RSX_ERR_UNSUPPORTED;
    if (ws_bytes < rsx_smore_spectral_fwd_ws_bytes(n_items, d, dv, dt) || (ws_bytes && !ws)) return RSX_ERR_WORKSPACE;
    p.X[0] = V;
    p.X[1] = T;
    p.K[0] = dv;
    p.K[1] = dt;
    p.W[0] = Wv;
    p.W[1] = Wt;
    p.n = n_items;
    p.tiles = (int)((n_items + kPjItems - 1) / kPjItems);
    float* outs[2] = {img, txt};
    float* w = static_cast<float*>(ws);
    for (int m = 0; m < 2; ++m) {
        p.S[m] = a.S[m] = proj_splits(n_items, p.K[m]);
        for (int sp = 0; sp < 8; ++sp) {
            float* o = nullptr;
            if (sp == 0) {
                o = outs[m];
            } else if (sp < p.S[m]) {
                o = w;
                w += n_items * d;
            }
            p.out[m][sp] = o;
            a.part[m][sp] = o;
        }
    }
    a.x[0] = img;
    a.x[1] = txt;
    a.b[0] = bv;
    a.b[1] = bt;
    a.w[0] = wv;
    a.w[1] = wt;
    a.w[2] = wf;
    a.n = n_items;
    a.conv[0] = conv_v;
    a.conv[1] = conv_t;
    a.conv[2] = conv_f;
    a.spec = spec;
    return RSX_OK;
}

extern "C" int rsx_smore_spectral_fwd(const float* V, int32_t dv, const float* Wv, const float* bv, const float* T,
                                      int32_t dt, const float* Wt, const float* bt, const float* wv, const float* wt,
                                      const float* wf, int64_t n_items, int32_t d, float* img, float* txt,
                                      float* conv_v, float* conv_t, float* conv_f, float* spec, void* ws,
                                      size_t ws_bytes, rsx_stream_t stream) {
    SpecProjArgs p;
    SpecFwdArgs a;
    const int rc = spectral_args(V, dv, Wv, bv, T, dt, Wt, bt, wv, wt, wf, n_items, d, img, txt, conv_v, conv_t,
                                 conv_f, spec, ws, ws_bytes, p, a);
    if (rc != RSX_OK || n_items == 0) return rc;
    const dim3 gp((unsigned)(p.tiles * (p.S[0] + p.S[1])));
    const dim3 gs((unsigned)((n_items + 63) / 64));
    hipStream_t s = as_stream(stream);
    if (d == 64) {
        hipLaunchKernelGGL(smore_proj<64>, gp, dim3(256), 0, s, p);
        hipLaunchKernelGGL(smore_spec_fwd<64>, gs, dim3(256), 0, s, a);
    } else {
        static const int half = env_knob("RSX_PROJ_HALF", 1, 0, 1);  // 0: one block per (tile, split) (A/B)
        const int nb = (int)(p.tiles * (p.S[0] + p.S[1]));
        if (half) hipLaunchKernelGGL(smore_proj_half<128>, dim3((unsigned)(16 * ((nb + 7) / 8))), dim3(256), 0, s, p, nb);
        else hipLaunchKernelGGL(smore_proj<128>, gp, dim3(256), 0, s, p);
        hipLaunchKernelGGL(smore_spec_fwd<128>, gs, dim3(256), 0, s, a);
    }
    return last_rc();
}

extern "C" size_t rsx_smore_item_tiles(int64_t n_items) {
    return n_items <= 0 ? 0 : (size_t)((n_items + kPjItems - 1) / kPjItems);
}

extern "C" int rsx_smore_item_fwd(const float* V, int32_t dv, const float* Wv, const float* bv, const float* T,
                                  int32_t dt, const float* Wt, const float* bt, const float* wv, const float* wt,
                                  const float* wf, int64_t n_items, int32_t d, float* img, float* txt, float* conv_v,
                                  float* conv_t, float* conv_f, float* spec, void* ws, size_t ws_bytes,
                                  uint32_t* tile_cnt, const float* item, const float* const* gate_W,
                                  const float* const* gate_b, float scale, int32_t mul, float* const* gate_out,
                                  rsx_stream_t stream) {
    ItemFwdArgs a;
    const int rc = spectral_args(V, dv, Wv, bv, T, dt, Wt, bt, wv, wt, wf, n_items, d, img, txt, conv_v, conv_t,
                                 conv_f, spec, ws, ws_bytes, a.p, a.s);
    if (rc != RSX_OK) return rc;
    if (!tile_cnt) return RSX_ERR_ARG;
    a.cnt = tile_cnt;
    a.item = item;
    a.scale = scale;
    a.mul = mul;
    if (item && (!gate_W || !gate_b || !gate_out)) return RSX_ERR_ARG;
    for (int m = 0; m < 3; ++m) {
        a.gW[m] = item ? gate_W[m] : nullptr;
        a.gb[m] = item ? gate_b[m] : nullptr;
        a.gout[m] = item ? gate_out[m] : nullptr;
        if (item && (!a.gW[m] || !a.gb[m] || !a.gout[m])) return RSX_ERR_ARG;
    }
    if (n_items == 0) return RSX_OK;
    const dim3 grid((unsigned)(a.p.tiles * (a.p.S[0] + a.p.S[1])));
    hipStream_t s = as_stream(stream);
    if (d == 64)
        hipLaunchKernelGGL(smore_item_fwd<64>, grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(smore_item_fwd<128>, grid, dim3(256), 0, s, a);
    return last_rc();
}

extern "C" size_t rsx_smore_spectral_bwd_partials(int64_t n_items, int32_t d) {
    return (size_t)((n_items + 63) / 64) * 3 * (size_t)(d / 2 + 1) * 2;
}

extern "C" size_t rsx_smore_spectral_bwd_ws_bytes(int64_t n_items, int32_t d) {
    if (n_items <= 0) return 0;
    const int mt = d == 64 ? Spec<64>::MT : Spec<128>::MT;
    const int64_t waves = (n_items + 63) / 64 * 4;
    return (size_t)waves * 2 * (size_t)mt * 64 * 4 * sizeof(float);
}

extern "C" int rsx_smore_spectral_bwd(const float* spec, const float* wv, const float* wt, const float* wf,
                                      const float* g_v, const float* g_t, const float* g_f, int64_t n_items, int32_t d,
                                      float* g_img, float* g_txt, float* g_w_partial, void* ws, size_t ws_bytes,
                                      rsx_stream_t stream) {
    if (n_items < 0 || !spec || !wv || !wt || !wf || !g_img || !g_txt || !g_w_partial) return RSX_ERR_ARG;
    if (d != 64 && d != 128) return RSX_ERR_UNSUPPORTED;
    if (n_items == 0) return RSX_OK;
    if (!ws || ws_bytes < rsx_smore_spectral_bwd_ws_bytes(n_items, d)) return RSX_ERR_WORKSPACE;
    SpecBwdArgs a;
    a.spec = spec;
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
    a.dfreq = static_cast<float*>(ws);
    const dim3 g((unsigned)((n_items + 63) / 64));
    hipStream_t s = as_stream(stream);
    if (d == 64) {
        hipLaunchKernelGGL(smore_spec_bwd_freq<64>, g, dim3(512), 0, s, a);
        hipLaunchKernelGGL(smore_spec_bwd_feat<64>, g, dim3(512), 0, s, a);
    } else {
        hipLaunchKernelGGL(smore_spec_bwd_freq<128>, g, dim3(512), 0, s, a);
        hipLaunchKernelGGL(smore_spec_bwd_feat<128>, g, dim3(512), 0, s, a);
    }
    return last_rc();
}

// smore_fuse.hip — SMORE's per-row MLP blocks, its InfoNCE terms and a
// multi-tensor Adam, each one launch (gfx950, f32 MFMA: exact f32 products, f32 sums).
//
// Replaces, per SMORE forward/backward (reference src/models/smore.py):
//  * the modality gates  g = sigmoid(Linear(conv)); item + 0.7 g     (:262-272)
//  * the preference block: softmax(query MLP(fusion)) * view, the dropout'd
//    sigmoid preference gates on the content rows, their mean, content + side
//                                                                     (:320-341)
//  * InfoNCE(side[pos], content[pos]) and InfoNCE(side[u], content[u]) (:380-387,
//    :398-404): L2-normalise, B x B similarity GEMM, exp, row sums, -log ratio
//  * torch.optim.Adam over every SMORE parameter tensor (trainer.py:133,238)
// which torch ran as ~30 elementwise / GEMM / reduction kernels each (per SMORE
// step under the mirror gradient, ~1000 launches of 5-20 us: C3 was launch-bound).
//
// Row fields (smore_fld.hpp).  A 16-row tile of [rows x D] lives in a wave as the accumulator
// layout of v_mfma_f32_16x16x4f32 transposed: lane l = n + 16 g holds row n0 + n,
// features 16 t + 4 g + r (t < D/16, r < 4) in register 4 t + r.  A row's D
// features are 4 lanes' registers (row reductions: registers, then xor 16, 32);
// loads and stores are float4s.  A matrix product z = W x of every row
// (nn.Linear) is Z^T = W X^T on the MFMA with A = W (lane (o, g) reads W[o][k] for
// the K slot k = 16 t + 4 g + r that its own B register x[n][k] holds: the K index
// of an MFMA may be permuted freely when A and B agree), so Z lands in the same
// field layout: a chain of Linears / activations never leaves registers.  W^T x
// (the backward) reads W by columns the same way.  Weights stay in global memory
// (a 16-64 KB matrix is L1/L2 resident; a float4 per lane feeds 4 MFMAs).
//
// Weight gradients: the backward kernels write each Linear's pre-activation
// gradient rows dZ (and the recomputed hidden rows the second Linear of a query
// MLP reads); rsx_smore_wgrad then forms dW = dZ^T X and db = colsum(dZ) for up
// to 8 (dZ, X) pairs in one launch of row-split partials plus one ordered
// reduction (deterministic).
#include <cmath>

#include "rsx_adam.hpp"
#include "rsx_common.hpp"
#include "smore_fld.hpp"

namespace rsx {
namespace sf {

// ---------------------------------------------------------------------------
// modality gates (smore.py:262-272)
// ---------------------------------------------------------------------------
struct GateArgs {
    const float* conv[3];   // conv_v, conv_t, conv_f [n, D]
    const float* item;      // item_id embedding [n, D]
    const float* W[3];      // gate_v/t/f Linear weights [D, D]
    const float* b[3];
    int64_t n;
    float scale;            // inject_scale (residual mode)
    int32_t mul;            // inject_mode == "mul"
    int32_t pad0;
    float* out[3];          // forward: img_i, txt_i, fus_i
    const float* gout[3];   // backward: their gradients (NULL = zero)
    float* g_item;          // backward outputs
    float* g_conv[3];
    float* dz[3];           // pre-activation gradients (wgrad rows)
    int64_t nbx;            // 64-row blocks of n (grid.x may be fewer: blocks stride over them)
    float* saved;           // optional [3][n][D]: the gates' sigmoid rows (forward writes them,
                            // gates_bwd_res_sv reads them instead of recomputing the product)
};

// Blocks stride over the 64-row blocks (grid.x <= a.nbx): a gate's weight is staged once
// per block (grid.y = 3: one gate per block row), not once per 64 rows.
template <int D>
__global__ __launch_bounds__(256) void gates_fwd(GateArgs a) {
    __shared__ __attribute__((aligned(16))) float wl[D * kLd<D>];
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const bool split = gridDim.y > 1;
    if (split) {  // one gate per block row: the next row block's rows load during this one's product
        const int m = (int)blockIdx.y;
        const float* W = stage_w<D>(wl, a.W[m]);
        auto row_of = [&](int64_t bx) {
            const int64_t r = (bx * 4 + (threadIdx.x >> 6)) * 16 + (lane & 15);
            return bx < a.nbx && r < a.n ? r : (int64_t)-1;
        };
        Fld<D> cvn = fload<D>(a.conv[m], row_of(blockIdx.x), g);
#pragma unroll 1
        for (int64_t bx = blockIdx.x; bx < a.nbx; bx += gridDim.x) {  // block-uniform
            const int64_t row = row_of(bx);
            const Fld<D> cv = cvn;
            const Fld<D> it = fload<D>(a.item, row, g);
            cvn = fload<D>(a.conv[m], row_of(bx + gridDim.x), g);
            const Fld<D> s = fmap<D>(mv_p<D, kLd<D>>(W, a.b[m], cv, lane), sigm);
            if (a.saved) fstore<D>(a.saved + (int64_t)m * a.n * D, row, g, s);
            const Fld<D> o = a.mul ? fmap2<D>(it, s, [](float x, float y) { return x * y; })
                                   : fmap2<D>(it, s, [&](float x, float y) { return x + a.scale * y; });
            fstore<D>(a.out[m], row, g, o);
        }
        return;
    }
#pragma unroll 1
    for (int64_t bx = blockIdx.x; bx < a.nbx; bx += gridDim.x) {  // block-uniform
        const int64_t n0 = (bx * 4 + (threadIdx.x >> 6)) * 16;
        const int64_t row = n0 + (lane & 15) < a.n ? n0 + (lane & 15) : -1;
        const Fld<D> it = fload<D>(a.item, row, g);
        const int m0 = split ? (int)blockIdx.y : 0, m1 = split ? m0 + 1 : 3;
#pragma unroll 1
        for (int m = m0; m < m1; ++m) {
            const Fld<D> cv = fload<D>(a.conv[m], row, g);
            const float* W = split ? wl : stage_w<D>(wl, a.W[m]);
            const Fld<D> s = fmap<D>(mv_p<D, kLd<D>>(W, a.b[m], cv, lane), sigm);
            if (a.saved) fstore<D>(a.saved + (int64_t)m * a.n * D, row, g, s);
            const Fld<D> o = a.mul ? fmap2<D>(it, s, [](float x, float y) { return x * y; })
                                   : fmap2<D>(it, s, [&](float x, float y) { return x + a.scale * y; });
            fstore<D>(a.out[m], row, g, o);
        }
    }
}

template <int D>
__global__ __launch_bounds__(256) void gates_bwd(GateArgs a) {
    __shared__ __attribute__((aligned(16))) float wl[D * kLd<D>];
    const int lane = threadIdx.x & 63, g = lane >> 4;
    // grid.y = 3 (residual mode): one gate per block row; g_item = sum of the three
    // upstream gradients (no sigmoid in it) is formed by the gate-0 blocks, in gate order
    const bool split = gridDim.y > 1;
    if (split) stage_w<D>(wl, a.W[blockIdx.y]);
#pragma unroll 1
    for (int64_t bx = blockIdx.x; bx < a.nbx; bx += gridDim.x) {  // block-uniform
    const int64_t n0 = (bx * 4 + (threadIdx.x >> 6)) * 16;
    const int64_t row = n0 + (lane & 15) < a.n ? n0 + (lane & 15) : -1;
    const Fld<D> it = fload<D>(a.item, row, g);
    Fld<D> gi = fzero<D>();
    const int m0 = split ? (int)blockIdx.y : 0, m1 = split ? m0 + 1 : 3;
    if (split && blockIdx.y == 0) {
#pragma unroll 1
        for (int m = 0; m < 3; ++m)
            gi = fmap2<D>(gi, a.gout[m] ? fload<D>(a.gout[m], row, g) : fzero<D>(),
                          [](float acc, float x) { return acc + x; });
        fstore<D>(a.g_item, row, g, gi);
    }
#pragma unroll 1
    for (int m = m0; m < m1; ++m) {
        const Fld<D> go = a.gout[m] ? fload<D>(a.gout[m], row, g) : fzero<D>();
        const Fld<D> cv = fload<D>(a.conv[m], row, g);
        const float* W = split ? wl : stage_w<D>(wl, a.W[m]);
        const Fld<D> s = fmap<D>(mv_p<D, kLd<D>>(W, a.b[m], cv, lane), sigm);
        Fld<D> ds;
        if (a.mul) {
            gi = fmap3<D>(gi, go, s, [](float acc, float x, float y) { return acc + x * y; });
            ds = fmap2<D>(go, it, [](float x, float y) { return x * y; });
        } else {
            gi = fmap2<D>(gi, go, [](float acc, float x) { return acc + x; });
            ds = fmap<D>(go, [&](float x) { return a.scale * x; });
        }
        const Fld<D> dz = fmap2<D>(ds, s, [](float x, float y) { return x * ((1.f - y) * y); });
        fstore<D>(a.dz[m], row, g, dz);
        fstore<D>(a.g_conv[m], row, g, mvt_p<D, kLd<D>>(W, dz, lane));
    }
    if (!split) fstore<D>(a.g_item, row, g, gi);
    }
}

// gates_bwd in residual mode (out = item + scale * sigmoid(Linear(conv)), one gate per
// block row): the same arithmetic with no item row or g_item accumulator held across the
// gate's two matrix products (the gate-0 blocks form g_item first), so fewer fields
// are live: d = 128 fits two waves a SIMD.
template <int D>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void gates_bwd_res(GateArgs a) {
    __shared__ __attribute__((aligned(16))) float wl[D * kLd<D>];
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int m = (int)blockIdx.y;
    const float* W = stage_w<D>(wl, a.W[m]);
    auto row_of = [&](int64_t bx) {
        const int64_t r = (bx * 4 + (threadIdx.x >> 6)) * 16 + (lane & 15);
        return bx < a.nbx && r < a.n ? r : (int64_t)-1;
    };
    // the next row block's conv rows are loaded while this one's products run
    Fld<D> cvn = fload<D>(a.conv[m], row_of(blockIdx.x), g);
#pragma unroll 1
    for (int64_t bx = blockIdx.x; bx < a.nbx; bx += gridDim.x) {  // block-uniform
        const int64_t row = row_of(bx);
        if (m == 0) {  // g_item = sum of the three upstream gradients, in gate order
            Fld<D> gi = fzero<D>();
#pragma unroll 1
            for (int q = 0; q < 3; ++q)
                gi = fmap2<D>(gi, a.gout[q] ? fload<D>(a.gout[q], row, g) : fzero<D>(),
                              [](float acc, float x) { return acc + x; });
            fstore<D>(a.g_item, row, g, gi);
        }
        Fld<D> dz;
        {
            const Fld<D> cv = cvn;
            const Fld<D> go = a.gout[m] ? fload<D>(a.gout[m], row, g) : fzero<D>();  // in flight during the product
            cvn = fload<D>(a.conv[m], row_of(bx + gridDim.x), g);
            const Fld<D> s = fmap<D>(mv_p<D, kLd<D>>(W, a.b[m], cv, lane), sigm);
            dz = fmap2<D>(fmap<D>(go, [&](float x) { return a.scale * x; }), s,
                          [](float x, float y) { return x * ((1.f - y) * y); });
        }
        fstore<D>(a.dz[m], row, g, dz);
        fstore<D>(a.g_conv[m], row, g, mvt_p<D, kLd<D>>(W, dz, lane));
    }
}

// gates_bwd_res from the forward's sigmoid rows (GateArgs::saved): one matrix product a
// row block (d conv = W^T dz) instead of two; the same element formulas.  The next row
// block's sigmoid and upstream-gradient rows load during this block's product.
template <int D>
__global__ __launch_bounds__(256) void gates_bwd_res_sv(GateArgs a) {
    __shared__ __attribute__((aligned(16))) float wl[D * kLd<D>];
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int m = (int)blockIdx.y;
    const float* W = stage_w<D>(wl, a.W[m]);
    const float* S = a.saved + (int64_t)m * a.n * D;
    auto row_of = [&](int64_t bx) {
        const int64_t r = (bx * 4 + (threadIdx.x >> 6)) * 16 + (lane & 15);
        return bx < a.nbx && r < a.n ? r : (int64_t)-1;
    };
    int64_t r0 = row_of(blockIdx.x);
    Fld<D> sn = fload<D>(S, r0, g);
    Fld<D> gn = a.gout[m] ? fload<D>(a.gout[m], r0, g) : fzero<D>();
#pragma unroll 1
    for (int64_t bx = blockIdx.x; bx < a.nbx; bx += gridDim.x) {  // block-uniform
        const int64_t row = row_of(bx);
        if (m == 0) {  // g_item = sum of the three upstream gradients, in gate order
            Fld<D> gi = fzero<D>();
#pragma unroll 1
            for (int q = 0; q < 3; ++q)
                gi = fmap2<D>(gi, a.gout[q] ? fload<D>(a.gout[q], row, g) : fzero<D>(),
                              [](float acc, float x) { return acc + x; });
            fstore<D>(a.g_item, row, g, gi);
        }
        const Fld<D> dz = fmap2<D>(fmap<D>(gn, [&](float x) { return a.scale * x; }), sn,
                                   [](float x, float y) { return x * ((1.f - y) * y); });
        const int64_t rn = row_of(bx + gridDim.x);
        sn = fload<D>(S, rn, g);
        gn = a.gout[m] ? fload<D>(a.gout[m], rn, g) : fzero<D>();
        fstore<D>(a.dz[m], row, g, dz);
        fstore<D>(a.g_conv[m], row, g, mvt_p<D, kLd<D>>(W, dz, lane));
    }
}

// ---------------------------------------------------------------------------
// preference block (smore.py:320-341)
// ---------------------------------------------------------------------------
enum { kW1v = 0, kW2v, kW1t, kW2t, kWip, kWtp, kWfp, kNW };

struct PrefArgs {
    const float* W[kNW];     // query_v.0, query_v.2, query_t.0, query_t.2, gate_{image,text,fusion}_prefer.0
    const float* b[kNW];     // biases (query_*.2 have none: NULL)
    const float* C;          // content rows [n, D]
    const float* IE;         // image_embeds
    const float* TE;         // text_embeds
    const float* FE;         // fusion_embeds
    int64_t n;
    float p_drop;            // dropout probability of the three preference gates (0 = eval / off)
    float drop_scale;        // 1 / (1 - p)
    const int64_t* seed;     // device word: the call's dropout seed
    float* all;              // forward outputs: content + side, side
    float* side;
    const float* g_all;      // backward inputs (g_side may be NULL)
    const float* g_side;
    float* gC;               // backward outputs
    float* gIE;
    float* gTE;
    float* gFE;
    float* hv;               // recomputed tanh rows of the query MLPs (wgrad inputs)
    float* ht;
    float* dz[kNW];          // pre-activation gradients (wgrad rows)
    // batch rows (rsx_smore_pref_rows): logical row r reads C / IE / TE / FE at rows[r];
    // row-r outputs (all, side, c_out, fe_out, dz, hv, ht) and inputs (g_all, g_side,
    // g_cin) are compact; gC / gIE / gTE / gFE are added into full tables at rows[r]
    const int64_t* rows;
    float* c_out;            // forward: the gathered content / fusion rows (optional)
    float* fe_out;
    const float* g_cin;      // backward: gradient of c_out (optional), added into gC
    // backward (batch rows, optional): [kOcc][n][D] per-occurrence row gradients instead of
    // float atomics into the tables; pref_segsum then sums them per table row in a fixed order
    float* occ;
    // batch rows, optional: [kSv][n][D] the forward's activations (written by pref_fwd_rows,
    // read by pref_bwd_rows_sv instead of recomputing 13 of the backward's 20 products)
    float* saved;
    // batch rows, optional: the occurrence plan the split forward builds for the backward's
    // per-row sums -- plan = [n] counts then [n][kPlanCap] occurrence lists (pref_segsum_plan),
    // lead = [1 + table rows] u64 scratch: word 0 the call counter, then one key per table row
    int32_t* plan;
    unsigned long long* lead;
};

// Occurrences listed per leading occurrence (more: that row falls back to segsum_one's scan)
constexpr int kPlanCap = 128;

// the saved activation slots: the fusion gate's sigmoid, then per view v (image 0, text 1)
// the query MLP's tanh row, its softmax row and the preference gate's sigmoid (all before
// the dropout mask, which the backward recomputes from the seed)
constexpr int kSvF = 0, kSv = 7;
__host__ __device__ constexpr int sv_h(int v) { return 1 + 3 * v; }
__host__ __device__ constexpr int sv_s(int v) { return 2 + 3 * v; }
__host__ __device__ constexpr int sv_p(int v) { return 3 + 3 * v; }
template <int D>
__device__ __forceinline__ float* sv_slot(const PrefArgs& a, int k) {
    return a.saved ? a.saved + (int64_t)k * a.n * D : nullptr;
}

// the per-occurrence slots of pref_bwd_rows (occ): the three gC shares (parts 0, 3, 4),
// the three gFE shares (parts 0, 1, 2), gIE, gTE
constexpr int kOccC0 = 0, kOccC3 = 1, kOccC4 = 2, kOccF0 = 3, kOccF1 = 4, kOccF2 = 5, kOccI = 6, kOccT = 7,
              kOcc = 8;

// the table row of logical row r (r < 0: none)
__device__ __forceinline__ int64_t src_row(const PrefArgs& a, int64_t r) { return (r >= 0 && a.rows) ? a.rows[r] : r; }

// Y[row] += x (float atomics: rows repeat within a batch).  RSX_PREF_PLAIN_STORES=1 (a timing
// variant only, tools/build_variant.py: wrong where rows repeat) stores instead, to price the atomics.
#ifndef RSX_PREF_PLAIN_STORES
#define RSX_PREF_PLAIN_STORES 0
#endif
template <int D>
__device__ __forceinline__ void fatomic(float* Y, int64_t row, int g, const Fld<D>& x) {
    if (row < 0 || !Y) return;
    if (RSX_PREF_PLAIN_STORES) {
        fstore<D>(Y, row, g, x);
        return;
    }
#pragma unroll
    for (int t = 0; t < D / 16; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) unsafeAtomicAdd(Y + row * D + 16 * t + 4 * g + r, x.f[t][r]);
}

// a row gradient of logical row `out` (table row `row`): into the per-occurrence slot, or
// added into the table
template <int D>
__device__ __forceinline__ void radd(const PrefArgs& a, int slot, float* Y, int64_t row, int64_t out, int g,
                                     const Fld<D>& x) {
    if (a.occ) fstore<D>(a.occ + (int64_t)slot * a.n * D, out, g, x);
    else fatomic<D>(Y, row, g, x);
}

template <int D>
__global__ __launch_bounds__(256) void pref_fwd(PrefArgs a) {
    __shared__ __attribute__((aligned(16))) float wl[D * kLd<D>];
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int64_t n0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
    const int64_t out = n0 + (lane & 15) < a.n ? n0 + (lane & 15) : -1;
    const int64_t row = src_row(a, out);
    const uint64_t seed = a.p_drop > 0.f ? (uint64_t)*a.seed : 0;
    const auto mul = [](float x, float y) { return x * y; };
    const auto lin = [&](int k, const Fld<D>& x) { return mv_p<D, kLd<D>>(stage_w<D>(wl, a.W[k]), a.b[k], x, lane); };
    const Fld<D> FE = fload<D>(a.FE, row, g);
    const Fld<D> C = fload<D>(a.C, row, g);
    fstore<D>(a.c_out, out, g, C);
    fstore<D>(a.fe_out, out, g, FE);
    // agg_img = ip * (softmax(query_v(FE)) * IE)
    Fld<D> h = fmap<D>(lin(kW1v, FE), tanh_);
    Fld<D> s = softmax_row<D>(lin(kW2v, h));
    Fld<D> ip = fmap<D>(lin(kWip, C), sigm);
    if (a.p_drop > 0.f) ip = fmap2<D>(ip, drop_scale<D>(seed, 0, row, g, a.p_drop, a.drop_scale), mul);
    const Fld<D> x1 = fmap3<D>(ip, s, fload<D>(a.IE, row, g), [](float p, float q, float e) { return p * (q * e); });
    h = fmap<D>(lin(kW1t, FE), tanh_);
    s = softmax_row<D>(lin(kW2t, h));
    Fld<D> tp = fmap<D>(lin(kWtp, C), sigm);
    if (a.p_drop > 0.f) tp = fmap2<D>(tp, drop_scale<D>(seed, 1, row, g, a.p_drop, a.drop_scale), mul);
    const Fld<D> x2 = fmap3<D>(tp, s, fload<D>(a.TE, row, g), [](float p, float q, float e) { return p * (q * e); });
    Fld<D> fp = fmap<D>(lin(kWfp, C), sigm);
    if (a.p_drop > 0.f) fp = fmap2<D>(fp, drop_scale<D>(seed, 2, row, g, a.p_drop, a.drop_scale), mul);
    // side = mean(stack([x1, x2, fp * FE]))  (sum, then * 1/3 as torch's mean)
    const Fld<D> sd = fmap3<D>(x1, x2, fmap2<D>(fp, FE, mul),
                               [](float u, float v, float w) { return ((u + v) + w) * (1.f / 3.f); });
    fstore<D>(a.side, out, g, sd);
    fstore<D>(a.all, out, g, fmap2<D>(C, sd, [](float u, float v) { return u + v; }));
}

template <int D>
__global__ __launch_bounds__(256) void pref_bwd(PrefArgs a) {
    __shared__ __attribute__((aligned(16))) float wl[D * kLd<D>];
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int64_t n0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
    const int64_t out = n0 + (lane & 15) < a.n ? n0 + (lane & 15) : -1;
    const int64_t row = src_row(a, out);
    const uint64_t seed = a.p_drop > 0.f ? (uint64_t)*a.seed : 0;
    const auto mul = [](float x, float y) { return x * y; };
    const auto add = [](float x, float y) { return x + y; };
    const auto sig_bwd = [](float gy, float y) { return gy * ((1.f - y) * y); };
    const Fld<D> gA = fload<D>(a.g_all, out, g);
    // d side = g_all + g_side;  each of the three stacked views gets d side / 3
    const Fld<D> g1 = a.g_side ? fmap2<D>(gA, fload<D>(a.g_side, out, g), [](float u, float v) { return (u + v) * (1.f / 3.f); })
                               : fmap<D>(gA, [](float u) { return u * (1.f / 3.f); });
    const Fld<D> FE = fload<D>(a.FE, row, g);
    const Fld<D> C = fload<D>(a.C, row, g);
    // batch-row mode: blockIdx.y = 0 the fusion view (+ the pass-through terms), 1 the
    // image view, 2 the text view, each adding its share of gC / gFE (atomics): three
    // shorter chains in parallel instead of one long one (otherwise part = -1: all)
    const int part = gridDim.y > 1 ? (int)blockIdx.y : -1;
    Fld<D> gC = part > 0 ? fzero<D>() : a.g_cin ? fmap2<D>(gA, fload<D>(a.g_cin, out, g), add) : gA;
    Fld<D> gFE = fzero<D>();
    if (part <= 0) {   // fusion view: x3 = fp * FE
        const float* W = stage_w<D>(wl, a.W[kWfp]);
        const Fld<D> sf = fmap<D>(mv_p<D, kLd<D>>(W, a.b[kWfp], C, lane), sigm);
        const Fld<D> mf = a.p_drop > 0.f ? drop_scale<D>(seed, 2, row, g, a.p_drop, a.drop_scale) : Fld<D>{};
        const Fld<D> fp = a.p_drop > 0.f ? fmap2<D>(sf, mf, mul) : sf;
        Fld<D> dp = fmap2<D>(g1, FE, mul);
        if (a.p_drop > 0.f) dp = fmap2<D>(dp, mf, mul);
        const Fld<D> dz = fmap2<D>(dp, sf, sig_bwd);
        fstore<D>(a.dz[kWfp], out, g, dz);
        gC = fmap2<D>(gC, mvt_p<D, kLd<D>>(W, dz, lane), add);
        gFE = fmap2<D>(g1, fp, mul);
    }
#pragma unroll 1
    for (int v = 0; v < 2; ++v) {  // v = 0: image view, 1: text view
        if (part >= 0 && part != v + 1) continue;  // block-uniform
        const int w1 = v ? kW1t : kW1v, w2 = v ? kW2t : kW2v, wp = v ? kWtp : kWip;
        const Fld<D> h = fmap<D>(mv_p<D, kLd<D>>(stage_w<D>(wl, a.W[w1]), a.b[w1], FE, lane), tanh_);
        fstore<D>(v ? a.ht : a.hv, out, g, h);
        const Fld<D> s = softmax_row<D>(mv_p<D, kLd<D>>(stage_w<D>(wl, a.W[w2]), nullptr, h, lane));
        const Fld<D> E = fload<D>(v ? a.TE : a.IE, row, g);
        Fld<D> pp;
        {
            const float* W = stage_w<D>(wl, a.W[wp]);
            const Fld<D> sp = fmap<D>(mv_p<D, kLd<D>>(W, a.b[wp], C, lane), sigm);
            const Fld<D> mp = a.p_drop > 0.f ? drop_scale<D>(seed, v, row, g, a.p_drop, a.drop_scale) : Fld<D>{};
            pp = a.p_drop > 0.f ? fmap2<D>(sp, mp, mul) : sp;
            // x = pp * (s * E)
            Fld<D> dpp = fmap3<D>(g1, s, E, [](float u, float q, float e) { return u * (q * e); });
            if (a.p_drop > 0.f) dpp = fmap2<D>(dpp, mp, mul);
            const Fld<D> dzp = fmap2<D>(dpp, sp, sig_bwd);
            fstore<D>(a.dz[wp], out, g, dzp);
            gC = fmap2<D>(gC, mvt_p<D, kLd<D>>(W, dzp, lane), add);
        }
        const Fld<D> da = fmap2<D>(g1, pp, mul);          // d (s * E)
        if (a.rows) fatomic<D>(v ? a.gTE : a.gIE, row, g, fmap2<D>(da, s, mul));
        else fstore<D>(v ? a.gTE : a.gIE, row, g, fmap2<D>(da, s, mul));
        const Fld<D> dsm = fmap2<D>(da, E, mul);          // d softmax output
        const float dot = rsum<D>(fmap2<D>(dsm, s, mul));
        const Fld<D> dq = fmap2<D>(s, dsm, [&](float y, float gy) { return y * (gy - dot); });
        fstore<D>(a.dz[w2], out, g, dq);
        const Fld<D> dh = mvt_p<D, kLd<D>>(stage_w<D>(wl, a.W[w2]), dq, lane);
        const Fld<D> dz1 = fmap2<D>(dh, h, [](float gy, float y) { return gy * (1.f - y * y); });
        fstore<D>(a.dz[w1], out, g, dz1);
        gFE = fmap2<D>(gFE, mvt_p<D, kLd<D>>(stage_w<D>(wl, a.W[w1]), dz1, lane), add);
    }
    if (a.rows) {
        fatomic<D>(a.gC, row, g, gC);
        fatomic<D>(a.gFE, row, g, gFE);
    } else {
        fstore<D>(a.gC, row, g, gC);
        fstore<D>(a.gFE, row, g, gFE);
    }
}

// The batch-row forward as three block rows (blockIdx.y): 0 the fusion view x3 = fp * FE
// (into `side`) and the gathered C / FE rows, 1 the image view x1 (into `all`), 2 the text
// view x2 (into the scratch `hv`): three chains of <= 3 matrix products instead of one
// of 7; pref_combine then forms side = ((x1 + x2) + x3) / 3 and all = C + side, pref_fwd's
// arithmetic element for element.
template <int D>
__global__ __launch_bounds__(256) void pref_fwd_rows(PrefArgs a) {
    __shared__ __attribute__((aligned(16))) float wl[D * kLd<D>];
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int64_t n0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
    const int64_t out = n0 + (lane & 15) < a.n ? n0 + (lane & 15) : -1;
    const int64_t row = src_row(a, out);
    const uint64_t seed = a.p_drop > 0.f ? (uint64_t)*a.seed : 0;
    const auto mul = [](float x, float y) { return x * y; };
    const auto lin = [&](int k, const Fld<D>& x) { return mv_p<D, kLd<D>>(stage_w<D>(wl, a.W[k]), a.b[k], x, lane); };
    const int part = (int)blockIdx.y;
    if (part == 0) {
        if (a.plan && out >= 0 && g == 0) {
            // occurrence plan, step 1: each table row's key keeps its first occurrence
            // (the largest key: this call's counter in the high word, ~j in the low one)
            const unsigned long long call = a.lead[0] + 1ull;
            atomicMax(a.lead + 1 + row, (call << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)out));
            a.plan[out] = 0;
        }
        const Fld<D> C = fload<D>(a.C, row, g);
        fstore<D>(a.c_out, out, g, C);
        Fld<D> fp = fmap<D>(lin(kWfp, C), sigm);
        fstore<D>(sv_slot<D>(a, kSvF), out, g, fp);
        if (a.p_drop > 0.f) fp = fmap2<D>(fp, drop_scale<D>(seed, 2, row, g, a.p_drop, a.drop_scale), mul);
        const Fld<D> FE = fload<D>(a.FE, row, g);
        fstore<D>(a.fe_out, out, g, FE);
        fstore<D>(a.side, out, g, fmap2<D>(fp, FE, mul));
        return;
    }
    const int v = part - 1;
    Fld<D> s;
    {
        const Fld<D> h = fmap<D>(lin(v ? kW1t : kW1v, fload<D>(a.FE, row, g)), tanh_);
        fstore<D>(sv_slot<D>(a, sv_h(v)), out, g, h);
        s = softmax_row<D>(lin(v ? kW2t : kW2v, h));
        fstore<D>(sv_slot<D>(a, sv_s(v)), out, g, s);
    }
    Fld<D> pg = fmap<D>(lin(v ? kWtp : kWip, fload<D>(a.C, row, g)), sigm);
    fstore<D>(sv_slot<D>(a, sv_p(v)), out, g, pg);
    if (a.p_drop > 0.f) pg = fmap2<D>(pg, drop_scale<D>(seed, v, row, g, a.p_drop, a.drop_scale), mul);
    const Fld<D> x = fmap3<D>(pg, s, fload<D>(v ? a.TE : a.IE, row, g), [](float p, float q, float e) { return p * (q * e); });
    fstore<D>(v ? a.hv : a.all, out, g, x);
}

// side = ((x1 + x2) + x3) * (1/3), all = C + side over the compact rows (float4 a thread)
template <int D>
__global__ __launch_bounds__(256) void pref_combine(PrefArgs a) {
    if (a.plan) {
        // occurrence plan, step 2: occurrence j joins its row's first occurrence l's list
        // (in any order: pref_segsum_plan sorts it); thread 0 advances the call counter
        // (nothing in this launch reads it)
        const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
        if (j < a.n) {
            const int64_t l = (int64_t)(0xFFFFFFFFu - (uint32_t)a.lead[1 + a.rows[j]]);
            const int pos = atomicAdd(a.plan + l, 1);
            if (pos < kPlanCap) a.plan[a.n + l * kPlanCap + pos] = (int32_t)j;
        }
        if (j == 0) atomicAdd(a.lead, 1ull);
    }
    const int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (e >= a.n * D) return;
    const int64_t r = e / D, f = e % D;
    const float4 x1 = ld4(a.all + e), x2 = ld4(a.hv + e), x3 = ld4(a.side + e);
    const float4 c = a.c_out ? ld4(a.c_out + e) : ld4(a.C + src_row(a, r) * D + f);
    const float4 sd = make_float4(((x1.x + x2.x) + x3.x) * (1.f / 3.f), ((x1.y + x2.y) + x3.y) * (1.f / 3.f),
                                  ((x1.z + x2.z) + x3.z) * (1.f / 3.f), ((x1.w + x2.w) + x3.w) * (1.f / 3.f));
    st4(a.side + e, sd);
    st4(a.all + e, make_float4(c.x + sd.x, c.y + sd.y, c.z + sd.z, c.w + sd.w));
}

// The batch-row backward (rsx_smore_pref_rows, gradients added by atomics): blockIdx.y = 0
// the fusion view + the pass-through terms, 1 / 2 the image / text view's query chain,
// 3 / 4 the image / text view's preference gate — the same arithmetic as pref_bwd's split
// form (each block row recomputes the forward values it needs), ordered so that few row
// fields are live at once
// (at d = 128 a field is 32 VGPRs a lane: pref_bwd's order keeps ~9 of them across its
// matrix products and spills): the gate product first (C then dead), the query MLP from
// FE (dead after), tanh rows reloaded from the hv / ht rows this kernel wrote, each view's
// gC / gFE share added as soon as it is formed.
template <int D>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void pref_bwd_rows(PrefArgs a) {
    __shared__ __attribute__((aligned(16))) float wl[D * kLd<D>];
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int64_t n0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
    const int64_t out = n0 + (lane & 15) < a.n ? n0 + (lane & 15) : -1;
    const int64_t row = src_row(a, out);
    const uint64_t seed = a.p_drop > 0.f ? (uint64_t)*a.seed : 0;
    const auto mul = [](float x, float y) { return x * y; };
    const auto add = [](float x, float y) { return x + y; };
    const auto sig_bwd = [](float gy, float y) { return gy * ((1.f - y) * y); };
    const auto g1_of = [&]() __attribute__((always_inline)) {  // d side / 3 (each stacked view's share)
        const Fld<D> gA = fload<D>(a.g_all, out, g);
        return a.g_side ? fmap2<D>(gA, fload<D>(a.g_side, out, g), [](float u, float v) { return (u + v) * (1.f / 3.f); })
                        : fmap<D>(gA, [](float u) { return u * (1.f / 3.f); });
    };
    const int part = (int)blockIdx.y;
    if (part == 0) {  // fusion view x3 = fp * FE, and d all -> d content
        const float* W = stage_w<D>(wl, a.W[kWfp]);
        const Fld<D> sf = fmap<D>(mv_p<D, kLd<D>>(W, a.b[kWfp], fload<D>(a.C, row, g), lane), sigm);
        const Fld<D> mf = a.p_drop > 0.f ? drop_scale<D>(seed, 2, row, g, a.p_drop, a.drop_scale) : Fld<D>{};
        const Fld<D> g1 = g1_of();
        Fld<D> dp = fmap2<D>(g1, fload<D>(a.FE, row, g), mul);
        if (a.p_drop > 0.f) dp = fmap2<D>(dp, mf, mul);
        const Fld<D> dz = fmap2<D>(dp, sf, sig_bwd);
        fstore<D>(a.dz[kWfp], out, g, dz);
        const Fld<D> fp = a.p_drop > 0.f ? fmap2<D>(sf, mf, mul) : sf;
        radd<D>(a, kOccF0, a.gFE, row, out, g, fmap2<D>(g1, fp, mul));
        const Fld<D> gA = fload<D>(a.g_all, out, g);
        const Fld<D> gC = a.g_cin ? fmap2<D>(gA, fload<D>(a.g_cin, out, g), add) : gA;
        radd<D>(a, kOccC0, a.gC, row, out, g, fmap2<D>(gC, mvt_p<D, kLd<D>>(W, dz, lane), add));
        return;
    }
    // parts 1 / 2: the image / text view's query chain (d IE / d TE, d FE); parts 3 / 4 the
    // same view's preference gate (d C): each recomputes the forward values it needs (the
    // gate sigmoid, resp. the softmax), so the longest chain is 5 products instead of 6
    const int v = (part - 1) & 1;  // 0: image view, 1: text view
    const bool gate_part = part >= 3;
    const int w1 = v ? kW1t : kW1v, w2 = v ? kW2t : kW2v, wp = v ? kWtp : kWip;
    // the view's preference gate on C (dropout mask applied after the sigmoid)
    const Fld<D> sp = fmap<D>(mv_p<D, kLd<D>>(stage_w<D>(wl, a.W[wp]), a.b[wp], fload<D>(a.C, row, g), lane), sigm);
    Fld<D> s;
    {
        const Fld<D> h = fmap<D>(mv_p<D, kLd<D>>(stage_w<D>(wl, a.W[w1]), a.b[w1], fload<D>(a.FE, row, g), lane), tanh_);
        if (!gate_part) fstore<D>(v ? a.ht : a.hv, out, g, h);
        s = softmax_row<D>(mv_p<D, kLd<D>>(stage_w<D>(wl, a.W[w2]), nullptr, h, lane));
    }
    const Fld<D> mp = a.p_drop > 0.f ? drop_scale<D>(seed, v, row, g, a.p_drop, a.drop_scale) : Fld<D>{};
    const Fld<D> g1 = g1_of();
    if (gate_part) {
        // x = pp * (s * E): d pp, through the dropout mask and the sigmoid
        Fld<D> dpp = fmap3<D>(g1, s, fload<D>(v ? a.TE : a.IE, row, g), [](float u, float q, float e) { return u * (q * e); });
        if (a.p_drop > 0.f) dpp = fmap2<D>(dpp, mp, mul);
        const Fld<D> dzp = fmap2<D>(dpp, sp, sig_bwd);
        fstore<D>(a.dz[wp], out, g, dzp);
        radd<D>(a, v ? kOccC4 : kOccC3, a.gC, row, out, g, mvt_p<D, kLd<D>>(stage_w<D>(wl, a.W[wp]), dzp, lane));
        return;
    }
    const Fld<D> pp = a.p_drop > 0.f ? fmap2<D>(sp, mp, mul) : sp;
    Fld<D> da = fmap2<D>(g1, pp, mul);  // d (s * E)
    radd<D>(a, v ? kOccT : kOccI, v ? a.gTE : a.gIE, row, out, g, fmap2<D>(da, s, mul));
    da = fmap2<D>(da, fload<D>(v ? a.TE : a.IE, row, g), mul);  // d softmax output
    const float dot = rsum<D>(fmap2<D>(da, s, mul));
    const Fld<D> dq = fmap2<D>(s, da, [&](float y, float gy) { return y * (gy - dot); });
    fstore<D>(a.dz[w2], out, g, dq);
    const Fld<D> dh = mvt_p<D, kLd<D>>(stage_w<D>(wl, a.W[w2]), dq, lane);
    const Fld<D> h = fload<D>(v ? a.ht : a.hv, out, g);  // this lane's own store above
    const Fld<D> dz1 = fmap2<D>(dh, h, [](float gy, float y) { return gy * (1.f - y * y); });
    fstore<D>(a.dz[w1], out, g, dz1);
    radd<D>(a, v ? kOccF2 : kOccF1, a.gFE, row, out, g, mvt_p<D, kLd<D>>(stage_w<D>(wl, a.W[w1]), dz1, lane));
}

// pref_bwd_rows from the forward's saved activations (PrefArgs::saved): the same block
// rows, occurrence slots and element formulas, but no forward product is recomputed --
// 7 matrix products (part 0: W_fp^T; parts 1 / 2: W_2^T then W_1^T; parts 3 / 4: W_p^T)
// instead of 20.  The tanh rows the weight gradients read are the saved ones.
template <int D>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void pref_bwd_rows_sv(PrefArgs a) {
    __shared__ __attribute__((aligned(16))) float wl[D * kLd<D>];
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int64_t n0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
    const int64_t out = n0 + (lane & 15) < a.n ? n0 + (lane & 15) : -1;
    const int64_t row = src_row(a, out);
    const uint64_t seed = a.p_drop > 0.f ? (uint64_t)*a.seed : 0;
    const auto mul = [](float x, float y) { return x * y; };
    const auto add = [](float x, float y) { return x + y; };
    const auto sig_bwd = [](float gy, float y) { return gy * ((1.f - y) * y); };
    const auto g1_of = [&]() __attribute__((always_inline)) {  // d side / 3 (each stacked view's share)
        const Fld<D> gA = fload<D>(a.g_all, out, g);
        return a.g_side ? fmap2<D>(gA, fload<D>(a.g_side, out, g), [](float u, float v) { return (u + v) * (1.f / 3.f); })
                        : fmap<D>(gA, [](float u) { return u * (1.f / 3.f); });
    };
    const int part = (int)blockIdx.y;
    if (part == 0) {  // fusion view x3 = fp * FE, and d all -> d content
        const Fld<D> sf = fload<D>(sv_slot<D>(a, kSvF), out, g);
        const Fld<D> mf = a.p_drop > 0.f ? drop_scale<D>(seed, 2, row, g, a.p_drop, a.drop_scale) : Fld<D>{};
        const Fld<D> g1 = g1_of();
        Fld<D> dp = fmap2<D>(g1, fload<D>(a.FE, row, g), mul);
        if (a.p_drop > 0.f) dp = fmap2<D>(dp, mf, mul);
        const Fld<D> dz = fmap2<D>(dp, sf, sig_bwd);
        fstore<D>(a.dz[kWfp], out, g, dz);
        const Fld<D> fp = a.p_drop > 0.f ? fmap2<D>(sf, mf, mul) : sf;
        radd<D>(a, kOccF0, a.gFE, row, out, g, fmap2<D>(g1, fp, mul));
        const Fld<D> gA = fload<D>(a.g_all, out, g);
        const Fld<D> gC = a.g_cin ? fmap2<D>(gA, fload<D>(a.g_cin, out, g), add) : gA;
        radd<D>(a, kOccC0, a.gC, row, out, g, fmap2<D>(gC, mvt_p<D, kLd<D>>(stage_w<D>(wl, a.W[kWfp]), dz, lane), add));
        return;
    }
    const int v = (part - 1) & 1;  // 0: image view, 1: text view
    const bool gate_part = part >= 3;
    const int w1 = v ? kW1t : kW1v, w2 = v ? kW2t : kW2v, wp = v ? kWtp : kWip;
    const Fld<D> sp = fload<D>(sv_slot<D>(a, sv_p(v)), out, g);
    const Fld<D> s = fload<D>(sv_slot<D>(a, sv_s(v)), out, g);
    const Fld<D> mp = a.p_drop > 0.f ? drop_scale<D>(seed, v, row, g, a.p_drop, a.drop_scale) : Fld<D>{};
    const Fld<D> g1 = g1_of();
    if (gate_part) {
        Fld<D> dpp = fmap3<D>(g1, s, fload<D>(v ? a.TE : a.IE, row, g), [](float u, float q, float e) { return u * (q * e); });
        if (a.p_drop > 0.f) dpp = fmap2<D>(dpp, mp, mul);
        const Fld<D> dzp = fmap2<D>(dpp, sp, sig_bwd);
        fstore<D>(a.dz[wp], out, g, dzp);
        radd<D>(a, v ? kOccC4 : kOccC3, a.gC, row, out, g, mvt_p<D, kLd<D>>(stage_w<D>(wl, a.W[wp]), dzp, lane));
        return;
    }
    const Fld<D> pp = a.p_drop > 0.f ? fmap2<D>(sp, mp, mul) : sp;
    Fld<D> da = fmap2<D>(g1, pp, mul);  // d (s * E)
    radd<D>(a, v ? kOccT : kOccI, v ? a.gTE : a.gIE, row, out, g, fmap2<D>(da, s, mul));
    da = fmap2<D>(da, fload<D>(v ? a.TE : a.IE, row, g), mul);  // d softmax output
    const float dot = rsum<D>(fmap2<D>(da, s, mul));
    const Fld<D> dq = fmap2<D>(s, da, [&](float y, float gy) { return y * (gy - dot); });
    fstore<D>(a.dz[w2], out, g, dq);
    const Fld<D> dh = mvt_p<D, kLd<D>>(stage_w<D>(wl, a.W[w2]), dq, lane);
    const Fld<D> h = fload<D>(sv_slot<D>(a, sv_h(v)), out, g);
    const Fld<D> dz1 = fmap2<D>(dh, h, [](float gy, float y) { return gy * (1.f - y * y); });
    fstore<D>(a.dz[w1], out, g, dz1);
    radd<D>(a, v ? kOccF2 : kOccF1, a.gFE, row, out, g, mvt_p<D, kLd<D>>(stage_w<D>(wl, a.W[w1]), dz1, lane));
}

// The per-occurrence row gradients of pref_bwd_rows summed per table row, deterministic:
// one wave per occurrence j; the first occurrence of its row (no earlier j' with the same
// row: a ballot scan) sums every occurrence of the row in ascending order, each
// occurrence's shares in slot order, and stores the row of gC / gIE / gTE / gFE.  Both
// scans test U chunks of 64 rows per step (loads in flight together: a chunk at a time
// made every wave a chain of ~n / 64 dependent round trips).  The row ids come from
// `RowAt`: the global int64 array, or (pref_segsum_lds) the block's int32 copy in LDS.
constexpr int kSegList = 128;  // a wave's occurrence list (LDS int32)
#ifndef RSX_SEGSUM_UB
#define RSX_SEGSUM_UB 0  // 0: 8 occurrences a round at d = 64, 4 at d = 128 (16 at d = 64 spilled: 4x slower)
#endif
// RSX_SEGSUM_ABL (timing ablations, tools/build_variant.py only): 1 skips the occurrence
// loads of pref_segsum_plan, 2 its table stores
#ifndef RSX_SEGSUM_ABL
#define RSX_SEGSUM_ABL 0
#endif
template <int D>
constexpr int kSegUB = RSX_SEGSUM_UB ? RSX_SEGSUM_UB : (D <= 64 ? 8 : 4);  // occurrences summed per round
template <int D, typename RowAt>
__device__ __forceinline__ void segsum_one(int64_t j, int64_t n, RowAt row_at, const float* __restrict__ occ,
                                           float* __restrict__ gC, float* __restrict__ gIE, float* __restrict__ gTE,
                                           float* __restrict__ gFE, int32_t* lst) {
    constexpr int PL = D / 64;  // columns per lane: lane + 64 p
    // UB occurrences' loads in flight at once: a hot row's sum is ceil(count / UB) dependent
    // rounds (a batch's most popular item has ~80 occurrences)
    constexpr int UC = 8, US = 4, UB = kSegUB<D>;
    const int lane = threadIdx.x & 63;
    const int64_t x = row_at(j);
    for (int64_t c = 0; c < j; c += 64 * UC) {
        int64_t r[UC];
#pragma unroll
        for (int u = 0; u < UC; ++u) {
            const int64_t k = c + 64 * u + lane;
            r[u] = k < j ? row_at(k) : -1;
        }
        bool hit = false;
#pragma unroll
        for (int u = 0; u < UC; ++u) hit |= r[u] == x;
        if (__ballot(hit)) return;  // an earlier occurrence leads
    }
    const int64_t sl = n * D;
    float aC[PL], aF[PL], aI[PL], aT[PL];
#pragma unroll
    for (int p = 0; p < PL; ++p) aC[p] = aF[p] = aI[p] = aT[p] = 0.f;
    // the row's occurrences are listed (ascending) in the wave's LDS list, then summed UB
    // at a time with their loads issued together (a hot row's occurrences one by one were
    // a chain of dependent loads: the launch's tail)
    int cnt = 0;  // wave-uniform
    auto flush = [&]() __attribute__((always_inline)) {
        for (int i0 = 0; i0 < cnt; i0 += UB) {
            float v[UB][8][PL];
#pragma unroll
            for (int t = 0; t < UB; ++t) {
                const int64_t k = i0 + t < cnt ? (int64_t)lst[i0 + t] : j;  // (a padded slot reloads j, unused)
                const float* o = occ + k * D + lane;
#pragma unroll
                for (int p = 0; p < PL; ++p) {
                    const int64_t q = 64 * p;
                    v[t][0][p] = o[kOccC0 * sl + q];
                    v[t][1][p] = o[kOccC3 * sl + q];
                    v[t][2][p] = o[kOccC4 * sl + q];
                    v[t][3][p] = o[kOccF0 * sl + q];
                    v[t][4][p] = o[kOccF1 * sl + q];
                    v[t][5][p] = o[kOccF2 * sl + q];
                    v[t][6][p] = o[kOccI * sl + q];
                    v[t][7][p] = o[kOccT * sl + q];
                }
            }
#pragma unroll
            for (int t = 0; t < UB; ++t) {
                if (i0 + t >= cnt) break;
#pragma unroll
                for (int p = 0; p < PL; ++p) {
                    aC[p] = ((aC[p] + v[t][0][p]) + v[t][1][p]) + v[t][2][p];
                    aF[p] = ((aF[p] + v[t][3][p]) + v[t][4][p]) + v[t][5][p];
                    aI[p] += v[t][6][p];
                    aT[p] += v[t][7][p];
                }
            }
        }
        cnt = 0;
    };
    for (int64_t c0 = j; c0 < n; c0 += 64 * US) {
        uint64_t mu[US];
        {
            int64_t r[US];
#pragma unroll
            for (int u = 0; u < US; ++u) {
                const int64_t k = c0 + 64 * u + lane;
                r[u] = k < n ? row_at(k) : -1;
            }
#pragma unroll
            for (int u = 0; u < US; ++u) mu[u] = __ballot(r[u] == x);
        }
#pragma unroll
        for (int u = 0; u < US; ++u) {  // the chunks in order: occurrences ascending
            uint64_t m = mu[u];
            while (m) {
                const int b = __builtin_ctzll(m);
                m &= m - 1;
                if (lane == 0) lst[cnt] = (int32_t)(c0 + 64 * u + b);
                if (++cnt == kSegList) flush();
            }
        }
    }
    flush();
#pragma unroll
    for (int p = 0; p < PL; ++p) {
        const int64_t col = x * D + lane + 64 * p;
        gC[col] = aC[p];
        gFE[col] = aF[p];
        gIE[col] = aI[p];
        gTE[col] = aT[p];
    }
}

template <int D>
__global__ __launch_bounds__(256) void pref_segsum(const int64_t* __restrict__ rows, int64_t n,
                                                   const float* __restrict__ occ, float* __restrict__ gC,
                                                   float* __restrict__ gIE, float* __restrict__ gTE,
                                                   float* __restrict__ gFE) {
    __shared__ int32_t lst[4][kSegList];
    const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= n) return;
    segsum_one<D>(j, n, [&](int64_t k) { return rows[k]; }, occ, gC, gIE, gTE, gFE, lst[threadIdx.x >> 6]);
}

// 16 occurrences a block share one int32 copy of the row ids in LDS (n <= kSegLds):
// every wave's scans read LDS instead of re-reading the int64 ids from L2
constexpr int kSegLds = 16384, kSegWaves = 16;
template <int D>
__global__ __launch_bounds__(64 * kSegWaves) void pref_segsum_lds(const int64_t* __restrict__ rows, int64_t n,
                                                                  const float* __restrict__ occ,
                                                                  float* __restrict__ gC, float* __restrict__ gIE,
                                                                  float* __restrict__ gTE, float* __restrict__ gFE) {
    __shared__ int32_t rl[kSegLds];
    __shared__ int32_t lst[kSegWaves][kSegList];
    for (int64_t k = threadIdx.x; k < n; k += 64 * kSegWaves) rl[k] = (int32_t)rows[k];
    __syncthreads();
    const int64_t j = (int64_t)blockIdx.x * kSegWaves + (threadIdx.x >> 6);
    if (j >= n) return;
    segsum_one<D>(j, n, [&](int64_t k) { return (int64_t)rl[k]; }, occ, gC, gIE, gTE, gFE, lst[threadIdx.x >> 6]);
}

// The per-row sums from the forward's occurrence plan: one wave per occurrence j; j leads
// its row when its plan count is non-zero.  The leader sorts its (unordered) list into
// ascending occurrence order and sums it as segsum_one does (same order, same bits); a row
// with more than kPlanCap occurrences takes segsum_one's scan.  No row-id scan, no LDS copy
// of the ids: the launch is the gathers and the stores.
template <int D>
__global__ __launch_bounds__(256) void pref_segsum_plan(const int64_t* __restrict__ rows, int64_t n,
                                                        const int32_t* __restrict__ plan, const float* __restrict__ occ,
                                                        float* __restrict__ gC, float* __restrict__ gIE,
                                                        float* __restrict__ gTE, float* __restrict__ gFE) {
    __shared__ int32_t lst[4][kSegList];
    const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= n) return;
    const int cnt = plan[j];
    if (cnt == 0) return;  // not a first occurrence
    int32_t* L = lst[threadIdx.x >> 6];
    if (cnt > kPlanCap) {
        segsum_one<D>(j, n, [&](int64_t k) { return rows[k]; }, occ, gC, gIE, gTE, gFE, L);
        return;
    }
    constexpr int PL = D / 64;
    constexpr int UB = kSegUB<D>;
    static_assert(kPlanCap <= 128 && kPlanCap <= kSegList, "two list entries a lane");
    const int lane = threadIdx.x & 63;
    const int32_t* lp = plan + n + j * kPlanCap;
    const int32_t e0 = lane < cnt ? lp[lane] : 0x7fffffff;
    const int32_t e1 = 64 + lane < cnt ? lp[64 + lane] : 0x7fffffff;
    int r0 = 0, r1 = 0;  // ranks: the list sorted ascending (entries are distinct)
    for (int k = 0; k < cnt; ++k) {
        const int32_t x = k < 64 ? __shfl(e0, k) : __shfl(e1, k - 64);
        r0 += x < e0;
        r1 += x < e1;
    }
    if (lane < cnt) L[r0] = e0;
    if (64 + lane < cnt) L[r1] = e1;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the list stores before any lane reads it
    __builtin_amdgcn_wave_barrier();
    const int64_t sl = n * D;
    float aC[PL], aF[PL], aI[PL], aT[PL];
#pragma unroll
    for (int p = 0; p < PL; ++p) aC[p] = aF[p] = aI[p] = aT[p] = 0.f;
    for (int i0 = 0; i0 < cnt; i0 += UB) {
        float v[UB][8][PL];
#pragma unroll
        for (int t = 0; t < UB; ++t) {
            const int64_t k = i0 + t < cnt ? (int64_t)L[i0 + t] : j;
            const float* o = occ + k * D + lane;
#pragma unroll
            for (int p = 0; p < PL; ++p) {
                const int64_t q = 64 * p;
                if (RSX_SEGSUM_ABL == 1) {
#pragma unroll
                    for (int u = 0; u < 8; ++u) v[t][u][p] = (float)k;
                    continue;
                }
                v[t][0][p] = o[kOccC0 * sl + q];
                v[t][1][p] = o[kOccC3 * sl + q];
                v[t][2][p] = o[kOccC4 * sl + q];
                v[t][3][p] = o[kOccF0 * sl + q];
                v[t][4][p] = o[kOccF1 * sl + q];
                v[t][5][p] = o[kOccF2 * sl + q];
                v[t][6][p] = o[kOccI * sl + q];
                v[t][7][p] = o[kOccT * sl + q];
            }
        }
#pragma unroll
        for (int t = 0; t < UB; ++t) {
            if (i0 + t >= cnt) break;
#pragma unroll
            for (int p = 0; p < PL; ++p) {
                aC[p] = ((aC[p] + v[t][0][p]) + v[t][1][p]) + v[t][2][p];
                aF[p] = ((aF[p] + v[t][3][p]) + v[t][4][p]) + v[t][5][p];
                aI[p] += v[t][6][p];
                aT[p] += v[t][7][p];
            }
        }
    }
    const int64_t x = rows[j];
    if (RSX_SEGSUM_ABL == 2 && aC[0] != 12345.f) return;
#pragma unroll
    for (int p = 0; p < PL; ++p) {
        const int64_t col = x * D + lane + 64 * p;
        gC[col] = aC[p];
        gFE[col] = aF[p];
        gIE[col] = aI[p];
        gTE[col] = aT[p];
    }
}

// rsx_tag_rows_next: tag_rows_k with the tag bump in the same launch.  tag2 = {tag, ticket}:
// every thread tags with tag2[0] + 1; each block takes a ticket when its stores are issued,
// and the last block (every other block has read tag2[0] by then) stores the new tag and
// re-arms the ticket.  One launch instead of torch's add_ plus tag_rows_k.
__global__ __launch_bounds__(256) void tag_rows_next_k(int32_t* __restrict__ row_tag, const int64_t* __restrict__ rows,
                                                       int64_t n, int32_t* __restrict__ tag2) {
    const int32_t t1 = tag2[0] + 1;
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j < n) row_tag[rows[j]] = t1;
    __syncthreads();
    if (threadIdx.x == 0 && atomicAdd(tag2 + 1, 1) == (int)gridDim.x - 1) {
        atomicExch(tag2, t1);
        atomicExch(tag2 + 1, 0);
    }
}

// Batch-row tags (rsx_tag_rows): row_tag[rows[j]] = *tag_dev for every j (duplicates
// store the same value), one thread per row: torch's index_put of the same assignment
// took 11 us at 6,144 rows.
__global__ __launch_bounds__(256) void tag_rows_k(int32_t* __restrict__ row_tag, const int64_t* __restrict__ rows,
                                                  int64_t n, const int32_t* __restrict__ tag_dev) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j < n) row_tag[rows[j]] = *tag_dev;
}

// ---------------------------------------------------------------------------
// batched weight gradients: dW_p = dZ_p^T X_p, db_p = colsum(dZ_p)
// ---------------------------------------------------------------------------
constexpr int kWgPairs = 8, kWgRows = 512;

struct WgArgs {
    const float* dz[kWgPairs];  // [n, D]
    const float* x[kWgPairs];   // [n, D]
    float* dw[kWgPairs];        // [D, D]
    float* db[kWgPairs];        // [D] or NULL
    int32_t n_pairs;
    int32_t n_splits;
    int64_t n;
    int64_t rows;               // rows per split (wg_rows)
    float* part;                // [n_pairs][n_splits][D*D + D]
};

// rows per split: enough blocks to fill the chip (~512 over all pairs; the batch-row
// preference block has only 3B rows), at least 64 (d = 64) / 128 (d = 128) rows and
// at most kWgRows, a multiple of the 32-row chunk
inline int64_t wg_rows(int64_t n, int d, int n_pairs) {
    int64_t r = (n * (n_pairs > 0 ? n_pairs : 1) + 511) / 512;
    const int64_t lo = d <= 64 ? 64 : 128;
    if (r < lo) r = lo;
    if (r > kWgRows) r = kWgRows;
    return (r + 31) / 32 * 32;
}

// block (split, pair): rows [r0, r1) in chunks of 32, each chunk's dz and x rows
// staged in LDS (row stride D + 16: the 4 K-rows x 16 columns of an MFMA operand
// read fall in 64 distinct banks), the next chunk's float4s loaded into registers
// while this one is multiplied.  Wave w owns output row tiles to = w, w + 4, ..;
// D[o][k]: lane (k, g) reg r holds o = 16 to + 4 g + r, k = 16 tk + c.
constexpr int kWgChunk = 32;

template <int D>
__global__ __launch_bounds__(256) void wgrad_part(WgArgs a) {
    constexpr int T = D / 16, TPW = (T + 3) / 4, LD = D + 16;
    constexpr int Q = D / 4;                          // float4s per row
    constexpr int PER = kWgChunk * Q / 256;           // float4s per thread per array
    __shared__ __attribute__((aligned(16))) float zl[kWgChunk * LD];
    __shared__ __attribute__((aligned(16))) float xl[kWgChunk * LD];
    const int split = blockIdx.x, pr = blockIdx.y;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
    const float* __restrict__ dz = a.dz[pr];
    const float* __restrict__ x = a.x[pr];
    const int64_t r0 = (int64_t)split * a.rows, r1 = min(a.n, r0 + a.rows);
    float* out = a.part + ((int64_t)pr * a.n_splits + split) * (D * D + D);
    floatx4 acc[TPW][T];
#pragma unroll
    for (int q = 0; q < TPW; ++q)
#pragma unroll
        for (int tk = 0; tk < T; ++tk) acc[q][tk] = floatx4{0.f, 0.f, 0.f, 0.f};
    float bs[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) bs[q] = 0.f;
    float4 pz[PER], px[PER];
    auto fetch = [&](int64_t cb) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x + 256 * i;
            const int rr = e / Q, c4 = e - rr * Q;
            const bool ok = cb + rr < r1;
            pz[i] = ok ? ld4(dz + (cb + rr) * D + 4 * c4) : f4(0.f);
            px[i] = ok ? ld4(x + (cb + rr) * D + 4 * c4) : f4(0.f);
        }
    };
    if (r0 < r1) fetch(r0);
    for (int64_t cb = r0; cb < r1; cb += kWgChunk) {
        __syncthreads();  // the previous chunk's readers are done
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x + 256 * i;
            const int rr = e / Q, c4 = e - rr * Q;
            *reinterpret_cast<float4*>(zl + rr * LD + 4 * c4) = pz[i];
            *reinterpret_cast<float4*>(xl + rr * LD + 4 * c4) = px[i];
        }
        __syncthreads();
        if (cb + kWgChunk < r1) fetch(cb + kWgChunk);
#pragma unroll
        for (int s = 0; s < kWgChunk / 4; ++s) {
            const float* zr = zl + (4 * s + g) * LD + c;
            const float* xr = xl + (4 * s + g) * LD + c;
            float bv[T];
#pragma unroll
            for (int tk = 0; tk < T; ++tk) bv[tk] = xr[16 * tk];
#pragma unroll
            for (int q = 0; q < TPW; ++q) {
                const int to = w + 4 * q;
                if (to < T) {
                    const float av = zr[16 * to];  // A[o = 16to + c][K = row 4s + g]
                    bs[q] += av;
#pragma unroll
                    for (int tk = 0; tk < T; ++tk) acc[q][tk] = mfma4(av, bv[tk], acc[q][tk]);
                }
            }
        }
    }
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int to = w + 4 * q;
        if (to >= T) break;
#pragma unroll
        for (int tk = 0; tk < T; ++tk)
#pragma unroll
            for (int r = 0; r < 4; ++r) out[(16 * to + 4 * g + r) * D + 16 * tk + c] = acc[q][tk][r];
        float b = bs[q];
        b += __shfl_xor(b, 16, kWave);
        b += __shfl_xor(b, 32, kWave);
        if (g == 0) out[D * D + 16 * to + c] = b;
    }
}

// element e = blockIdx.x * 64 + lane of pair blockIdx.y: wave w adds splits
// [w S/4, (w+1) S/4) in order with 8 loads in flight, the four quarters are added in
// wave order (deterministic)
template <int D>
__global__ __launch_bounds__(256) void wgrad_reduce(WgArgs a) {
    constexpr int64_t SZ = D * D + D;
    __shared__ float q[4][64];
    const int pr = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t e = (int64_t)blockIdx.x * 64 + lane;
    const int S = a.n_splits;
    const int b = S * wave / 4, en = S * (wave + 1) / 4;
    float acc = 0.f;
    if (e < SZ) {
        const float* p = a.part + (int64_t)pr * S * SZ + e;
        int i = b;
        for (; i + 8 <= en; i += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)(i + u) * SZ];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += v[u];
        }
        for (; i < en; ++i) acc += p[(int64_t)i * SZ];
    }
    q[wave][lane] = acc;
    __syncthreads();
    if (wave != 0 || e >= SZ) return;
    const float s = ((q[0][lane] + q[1][lane]) + q[2][lane]) + q[3][lane];
    if (e < D * D) a.dw[pr][e] = s;
    else if (a.db[pr]) a.db[pr][e - D * D] = s;
}

// ---------------------------------------------------------------------------
// InfoNCE (smore.py:380-387) over two (view1, view2) row sets
// ---------------------------------------------------------------------------
// term t: view1 rows src1[idx_t[b] + off_t], view2 rows src2[idx_t[b] + off_t], b < B.
// Forward block (own tile of 16 rows, term): waves split the other tiles; each
// normalises what it loads (F.normalize: x / max(|x|, 1e-12)); S = n1 n2^T / tau on the
// MFMA (A = other rows, B = own rows: S^T lands with the own row per lane), row sums of
// exp(S) combined over waves in order; l_b = -log(pos_b / ttl_b).  The normalised rows,
// norms and ttl go to the workspace for the backward; the last block adds each term's
// l_b in order (mean).
// Backward block (own tile, mode, term): P = exp(S)/ttl_i; mode 0 (own = view1 rows i):
// O_i = sum_j P_ij n2_j; mode 1 (own = view2 rows j): O_j = sum_i P_ij n1_i (ttl by the
// other row).  d n = g/(B tau) (O - n_other_own); through F.normalize; atomically added
// into the row's gradient (pos items / users repeat within a batch).
constexpr int kNceWaves = 8;

struct NceArgs {
    const float* src1;       // side   [N, D]
    const float* src2;       // content [N, D]
    const int64_t* idx[2];   // [B] each
    int64_t off[2];
    int64_t B;
    float tau;
    int32_t pad0;
    float* nrm;              // ws: [2 terms][2 views][B][D] normalised rows
    float* norms;            // ws: [2][2][B] |x|
    float* ttl;              // ws: [2][B]
    float* lrow;             // ws: [2][B]
    float* loss;             // [2]: cl_items, cl_users
    const float* add_loss;   // forward (optional): total = add_loss[0] + cl * (cl_items + cl_users)
    float cl;
    float* total;
    const float* gloss;      // backward: upstream gradients of the two losses, gloss[term * gstride] * gscale
    int32_t gstride;
    float gscale;
    float* g1;               // d src1 [N, D] (accumulated)
    float* g2;               // d src2
    float* E;                // ws (B <= kNceStoreMax): [2][B][B] exp(S / tau), written by the forward,
                             // read by the backward instead of recomputing S (NULL: recompute)
    float* nrmT;             // ws (with E): [2 terms][2 views][ceil(B/16)][D][16] the normalised rows,
                             // each 16-row tile transposed (the backward's MFMA B operand as stored)
    // backward, the compact batch rows (rsx_smore_loss_rows_bwd): every (term, own row)
    // destination is distinct, so the rows are stored, not added; and two element-wise jobs
    // spread over the grid: xo = xg * gloss[0] (xn floats) and z1, z2 zeroed (zn floats each)
    int32_t rows;
    const float* xg;
    float* xo;
    int64_t xn;
    float* z1;
    float* z2;
    int64_t zn;
};

// the element-wise jobs of the compact-rows backward, grid-strided over every thread of the
// launch (uniform no-ops otherwise)
__device__ __forceinline__ void nce_extra(const NceArgs& a) {
    if (!a.xo && !a.z1) return;
    const int64_t nthr = (int64_t)gridDim.x * gridDim.y * gridDim.z * blockDim.x;
    const int64_t tid =
        (((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
    if (a.xo) {
        const float sc = a.gloss[0];
        for (int64_t i = tid; i < a.xn / 4; i += nthr) {
            const float4 v = ld4(a.xg + 4 * i);
            st4(a.xo + 4 * i, make_float4(v.x * sc, v.y * sc, v.z * sc, v.w * sc));
        }
    }
    if (a.z1) {
        for (int64_t i = tid; i < a.zn / 4; i += nthr) {
            st4(a.z1 + 4 * i, f4(0.f));
            st4(a.z2 + 4 * i, f4(0.f));
        }
    }
}
constexpr int64_t kNceStoreMax = 4096;

template <int D>
__device__ __forceinline__ Fld<D> nce_load_norm(const NceArgs& a, int term, int view, int64_t b, int g, float* nrm_out) {
    const int64_t row = b >= 0 ? a.idx[term][b] + a.off[term] : -1;
    Fld<D> x = fload<D>(view ? a.src2 : a.src1, row, g);
    const float n = sqrtf(rsum<D>(fmap<D>(x, [](float v) { return v * v; })));
    const float den = fmaxf(n, 1e-12f);
    if (nrm_out) *nrm_out = n;
    return fmap<D>(x, [&](float v) { return v / den; });
}

// The batch rows of both views normalised once (F.normalize, eps 1e-12): nrm[term][view]
// [B][D] and |x| (for the backward), and the positive pair's dot (n1 * n2).sum(-1) kept
// in lrow until nce_fwd turns it into the row loss.  One wave per 16 rows.
template <int D>
__global__ __launch_bounds__(64) void nce_norm(NceArgs a) {
    const int term = blockIdx.y;
    const int lane = threadIdx.x, g = lane >> 4;
    const int64_t B = a.B;
    const int64_t bo = (int64_t)blockIdx.x * 16 + (lane & 15) < B ? (int64_t)blockIdx.x * 16 + (lane & 15) : -1;
    float n1 = 0.f, n2 = 0.f;
    const Fld<D> X1 = nce_load_norm<D>(a, term, 0, bo, g, &n1);
    const Fld<D> X2 = nce_load_norm<D>(a, term, 1, bo, g, &n2);
    fstore<D>(a.nrm + ((int64_t)(term * 2 + 0) * B) * D, bo, g, X1);
    fstore<D>(a.nrm + ((int64_t)(term * 2 + 1) * B) * D, bo, g, X2);
    if (a.nrmT) {  // tile blockIdx.x transposed: [feature][16 rows] (rows past B are zeros)
        const int64_t nt = (B + 15) / 16;
        float* t1 = a.nrmT + (((int64_t)(term * 2 + 0) * nt + blockIdx.x) * D) * 16 + (lane & 15);
        float* t2 = a.nrmT + (((int64_t)(term * 2 + 1) * nt + blockIdx.x) * D) * 16 + (lane & 15);
#pragma unroll
        for (int t = 0; t < D / 16; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                t1[(16 * t + 4 * g + i) * 16] = X1.f[t][i];
                t2[(16 * t + 4 * g + i) * 16] = X2.f[t][i];
            }
    }
    const float dot = rsum<D>(fmap2<D>(X1, X2, [](float u, float v) { return u * v; }));
    if (g == 0 && bo >= 0) {
        a.norms[(term * 2 + 0) * B + bo] = n1;
        a.norms[(term * 2 + 1) * B + bo] = n2;
        a.lrow[term * B + bo] = dot;
    }
}

// ttl[own] = sum over the other rows m of exp(<n1[own], n2[m]> / tau): a block owns 16
// rows, its waves stride over the 16-row tiles of the other view (contiguous normalised
// rows, two tiles in flight ahead of the one being multiplied); then the row loss
// -log(exp(dot / tau) / ttl).
template <int D>
__global__ __launch_bounds__(64 * kNceWaves) void nce_fwd(NceArgs a) {
    __shared__ float part[kNceWaves][16];
    const int term = blockIdx.y;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
    const int64_t B = a.B;
    const int64_t n0 = (int64_t)blockIdx.x * 16;
    const int64_t bo = n0 + c < B ? n0 + c : -1;
    const float* n1 = a.nrm + ((int64_t)(term * 2 + 0) * B) * D;
    const float* n2 = a.nrm + ((int64_t)(term * 2 + 1) * B) * D;
    const Fld<D> X = fload<D>(n1, bo, g);  // own view1 rows (B operand)
    const int64_t ntile = (B + 15) / 16;
    auto row_of = [&](int64_t mt) { return (mt < ntile && mt * 16 + c < B) ? mt * 16 + c : (int64_t)-1; };
    float es = 0.f;  // exp sum of own row c over the other rows 4g + r of this wave's tiles
    Fld<D> Y0 = fload<D>(n2, row_of(w), g);
    Fld<D> Y1 = fload<D>(n2, row_of(w + kNceWaves), g);
    for (int64_t mt = w; mt < ntile; mt += kNceWaves) {
        const Fld<D> Y2 = fload<D>(n2, row_of(mt + 2 * kNceWaves), g);  // two tiles ahead, in flight
        const int64_t m0 = mt * 16;
        const floatx4 sv = tile_dot<D>(Y0, X);  // s[r] = <own c, other m0 + 4g + r>
        floatx4 ev;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            ev[r] = m0 + 4 * g + r < B ? expf(sv[r] / a.tau) : 0.f;
            es += ev[r];  // (+0 for a column past B: the sum is unchanged)
        }
        if (a.E && bo >= 0) {  // E[term][own][m0 + 4g .. +3] for the backward
            float* er = a.E + ((int64_t)term * B + bo) * B + m0 + 4 * g;
            if ((B & 3) == 0 && m0 + 4 * g + 3 < B) {
                *reinterpret_cast<floatx4*>(er) = ev;
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (m0 + 4 * g + r < B) er[r] = ev[r];
            }
        }
        Y0 = Y1;
        Y1 = Y2;
    }
    es += __shfl_xor(es, 16, kWave);
    es += __shfl_xor(es, 32, kWave);
    if (lane < 16) part[w][lane] = es;
    __syncthreads();
    if (w == 0 && lane < 16 && bo >= 0) {
        float ttl = 0.f;
#pragma unroll
        for (int i = 0; i < kNceWaves; ++i) ttl += part[i][lane];
        const float pos = expf(a.lrow[term * B + bo] / a.tau);
        a.ttl[term * B + bo] = ttl;
        a.lrow[term * B + bo] = -logf(pos / ttl);
    }
}

// the two means (cl_items, cl_users): one wave per term, rows summed in a fixed order;
// optionally the model's total loss add_loss + cl * (cl_items + cl_users) in f32, in
// the reference's order (smore.py:411: bpr + cl_loss * (cl_items + cl_users))
__global__ __launch_bounds__(128) void nce_mean(NceArgs a) {
    const int term = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const float* l = a.lrow + (int64_t)term * a.B;
    double acc = 0.0;
    // the same order as one row at a time (i = lane, lane + 64, ...), the loads of 32 rows
    // issued together (one at a time, each add waited on its load: ~10 us at B = 2048)
    int64_t i = lane;
    for (; i + 64 * 31 < a.B; i += 64 * 32) {
        float v[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) v[u] = l[i + 64 * u];
#pragma unroll
        for (int u = 0; u < 32; ++u) acc += (double)v[u];
    }
    for (; i < a.B; i += 64) acc += (double)l[i];
    acc = group_sum_d<64>(acc);
    __shared__ float m[2];
    if (lane == 0) {
        m[term] = (float)(acc / (double)a.B);
        a.loss[term] = m[term];
    }
    __syncthreads();
    if (threadIdx.x == 0 && a.total) a.total[0] = a.add_loss[0] + a.cl * (m[0] + m[1]);
}

template <int D>
__global__ __launch_bounds__(64 * kNceWaves) void nce_bwd(NceArgs a) {
    constexpr int T = D / 16;
    constexpr int TILE = 16 * kLd<D>;  // one wave's other-tile copy (rows padded)
    static_assert(kNceWaves * 64 * T * 4 <= kNceWaves * TILE, "reduction fits the tile buffer");
    __shared__ __attribute__((aligned(16))) float sm[kNceWaves * TILE];
    nce_extra(a);
    const int term = blockIdx.z, mode = blockIdx.y;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
    const int64_t B = a.B;
    const int64_t n0 = (int64_t)blockIdx.x * 16;
    const int64_t bo = n0 + c < B ? n0 + c : -1;
    const float* own_n = a.nrm + ((int64_t)(term * 2 + mode) * B) * D;
    const float* oth_n = a.nrm + ((int64_t)(term * 2 + (mode ^ 1)) * B) * D;
    const float* ttl = a.ttl + term * B;
    const float ttl_own = (mode == 0 && bo >= 0) ? ttl[bo] : 1.f;
    float* tl = sm + w * TILE;
    Fld<D> O = fzero<D>();
    const int64_t ntile = (B + 15) / 16;
    auto row_of = [&](int64_t mt) { return (mt < ntile && mt * 16 + c < B) ? mt * 16 + c : (int64_t)-1; };
    auto ttl_of = [&](int64_t mt) {  // mode 1: the divisor of the other rows 4g + r
        floatx4 t = {1.f, 1.f, 1.f, 1.f};
        if (mode == 1)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t m = mt * 16 + 4 * g + r;
                if (mt < ntile && m < B) t[r] = ttl[m];
            }
        return t;
    };
    // exp(S / tau) of own row c and other rows mt*16 + 4g + r as the forward wrote it
    // (E[term][view1 row][view2 row]; 0 past B or for a missing own row)
    const float* eb = a.E ? a.E + (int64_t)term * B * B : nullptr;
    auto e_of = [&](int64_t mt) {
        floatx4 ev = {0.f, 0.f, 0.f, 0.f};
        if (!eb || bo < 0 || mt >= ntile) return ev;
        const int64_t m0 = mt * 16 + 4 * g;
        if (mode == 0) {
            const float* er = eb + bo * B + m0;
            if ((B & 3) == 0 && m0 + 3 < B) {
                ev = *reinterpret_cast<const floatx4*>(er);
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) ev[r] = m0 + r < B ? er[r] : 0.f;
            }
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) ev[r] = m0 + r < B ? eb[(m0 + r) * B + bo] : 0.f;
        }
        return ev;
    };
    const Fld<D> X = fload<D>(own_n, bo, g);
    Fld<D> Y = fload<D>(oth_n, row_of(w), g);
    floatx4 tv = ttl_of(w);
    floatx4 ev = e_of(w);
    for (int64_t mt = w; mt < ntile; mt += kNceWaves) {
        const Fld<D> Yn = fload<D>(oth_n, row_of(mt + kNceWaves), g);  // next tile, in flight
        const floatx4 tvn = ttl_of(mt + kNceWaves);
        const floatx4 evn = e_of(mt + kNceWaves);
        const int64_t m0 = mt * 16;
        // P for own row c and other rows m0 + 4g + r
        floatx4 p;
        if (eb) {
#pragma unroll
            for (int r = 0; r < 4; ++r) p[r] = (bo >= 0 && m0 + 4 * g + r < B) ? ev[r] / (mode == 0 ? ttl_own : tv[r]) : 0.f;
        } else {
            const floatx4 s = tile_dot<D>(Y, X);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool ok = m0 + 4 * g + r < B;
                p[r] = ok ? expf(s[r] / a.tau) / (mode == 0 ? ttl_own : tv[r]) : 0.f;
            }
        }
        // O^T[k][own] += sum_m Y^T[k][m] P^T[m][own] (K slot (r, g) = other row m0 + 4g + r):
        // the A operand is the tile transposed, through this wave's LDS copy
#pragma unroll
        for (int t = 0; t < T; ++t)
            *reinterpret_cast<floatx4*>(tl + (lane & 15) * kLd<D> + 16 * t + 4 * g) = Y.f[t];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float* yr = tl + (4 * g + r) * kLd<D> + c;
#pragma unroll
            for (int tk = 0; tk < T; ++tk) O.f[tk] = mfma4(yr[16 * tk], p[r], O.f[tk]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        Y = Yn;
        tv = tvn;
        ev = evn;
    }
    __syncthreads();
    floatx4* red = reinterpret_cast<floatx4*>(sm);  // [wave][lane][T]
#pragma unroll
    for (int t = 0; t < T; ++t) red[(w * 64 + lane) * T + t] = O.f[t];
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int t = 0; t < T; ++t) {
        floatx4 s = red[lane * T + t];
#pragma unroll
        for (int i = 1; i < kNceWaves; ++i) s += red[(i * 64 + lane) * T + t];
        O.f[t] = s;
    }
    if (bo < 0) return;
    const float coef = (a.gloss[term * a.gstride] * a.gscale) * (1.f / a.tau) / (float)B;
    const Fld<D> Z = fload<D>(oth_n, bo, g);  // the own row's other view
    const Fld<D> dn = fmap2<D>(O, Z, [&](float o, float z) { return coef * (o - z); });
    // F.normalize backward: (dn - y <y, dn>) / |x|, or dn / eps when |x| <= eps
    const float nx = a.norms[(term * 2 + mode) * B + bo];
    Fld<D> dv;
    if (nx > 1e-12f) {
        const float yd = rsum<D>(fmap2<D>(X, dn, [](float u, float v) { return u * v; }));
        dv = fmap2<D>(dn, X, [&](float u, float y) { return (u - y * yd) / nx; });
    } else {
        dv = fmap<D>(dn, [](float u) { return u / 1e-12f; });
    }
    float* dst = (mode == 0 ? a.g1 : a.g2) + (a.idx[term][bo] + a.off[term]) * D;
    if (a.rows) {
#pragma unroll
        for (int t = 0; t < T; ++t) st4(dst + 16 * t + 4 * g, make_float4(dv.f[t][0], dv.f[t][1], dv.f[t][2], dv.f[t][3]));
        return;
    }
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) atomicAdd(dst + 16 * t + 4 * g + r, dv.f[t][r]);
}

// nce_bwd with the forward's stored exp tiles (a.E) and transposed row tiles (a.nrmT):
// O (own x features) += P (own x other) Y (other x features) with A = P as computed per
// lane (own c, other 4g + r) and B = the other tile read straight in the operand layout
// (lane (c, g): Y[other 4g .. 4g+3][feature 16 tk + c], one float4 per output tile), so a
// tile costs T float4 loads and 4T MFMAs: no per-tile LDS transpose, no wave barriers.
// The same products in the same K grouping and order as nce_bwd; the waves' partials are
// summed in wave order through LDS (transposed back to the row layout) and the epilogue
// is nce_bwd's.
template <int D, int NG>
__global__ __launch_bounds__(64 * kNceWaves) void nce_bwd_t(NceArgs a) {
    // NG own 16-row groups per block: every other-view tile a wave loads feeds NG groups'
    // MFMAs (NG = 2 halves the L2 reads of the other view's tiles; same K split over the
    // waves, same order, so the results are NG = 1's bit for bit)
    constexpr int T = D / 16;
    // The partials' tile red[w][row][col] is stored with row r's columns rotated by 8 sig(r)
    // floats (sig below).  Unrotated, the epilogue's ds_read_b128 of row c, columns 16 t + 4 g
    // put the 8 lanes of one g in a lane group on the same 4 banks (8-way: PMC conflict share
    // 0.75).  sig gives every ds_read_b128 lane group ({0-3,12-15,20-27}, ...)
    // 16 distinct 4-bank segments, and every ds_write_b32 half-wave (rows 4g + q, g = 0, 1)
    // 32 distinct banks (rows 4 apart rotate 16 banks apart): conflict-free both ways.
    __shared__ __attribute__((aligned(16))) float red[kNceWaves][16][D];
    auto rot = [](int r) { return 8 * ((2 * r + 2 * (r >> 2) + ((r >> 3) & 1)) & 7); };
    nce_extra(a);
    const int term = blockIdx.z, mode = blockIdx.y;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
    const int64_t B = a.B;
    int64_t bo[NG];
#pragma unroll
    for (int h = 0; h < NG; ++h) {
        const int64_t n0 = ((int64_t)blockIdx.x * NG + h) * 16;
        bo[h] = n0 + c < B ? n0 + c : -1;
    }
    const int64_t ntile = (B + 15) / 16;
    const float* own_n = a.nrm + ((int64_t)(term * 2 + mode) * B) * D;
    const float* oth_n = a.nrm + ((int64_t)(term * 2 + (mode ^ 1)) * B) * D;
    const float* othT = a.nrmT + ((int64_t)(term * 2 + (mode ^ 1)) * ntile) * D * 16 + c * 16 + 4 * g;
    const float* ttl = a.ttl + term * B;
    float ttl_own[NG];
#pragma unroll
    for (int h = 0; h < NG; ++h) ttl_own[h] = (mode == 0 && bo[h] >= 0) ? ttl[bo[h]] : 1.f;
    const float* eb = a.E + (int64_t)term * B * B;
    auto ttl_of = [&](int64_t mt) {
        floatx4 t = {1.f, 1.f, 1.f, 1.f};
        if (mode == 1)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t m = mt * 16 + 4 * g + r;
                if (mt < ntile && m < B) t[r] = ttl[m];
            }
        return t;
    };
    auto e_of = [&](int64_t mt, int64_t own) {
        floatx4 ev = {0.f, 0.f, 0.f, 0.f};
        if (own < 0 || mt >= ntile) return ev;
        const int64_t m0 = mt * 16 + 4 * g;
        if (mode == 0) {
            const float* er = eb + own * B + m0;
            if ((B & 3) == 0 && m0 + 3 < B) {
                ev = *reinterpret_cast<const floatx4*>(er);
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) ev[r] = m0 + r < B ? er[r] : 0.f;
            }
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) ev[r] = m0 + r < B ? eb[(m0 + r) * B + own] : 0.f;
        }
        return ev;
    };
    auto y_of = [&](int64_t mt, floatx4(&y)[T]) {
#pragma unroll
        for (int tk = 0; tk < T; ++tk)
            y[tk] = mt < ntile ? *reinterpret_cast<const floatx4*>(othT + (mt * D + 16 * tk) * 16)
                               : floatx4{0.f, 0.f, 0.f, 0.f};
    };
    floatx4 O[NG][T];
#pragma unroll
    for (int h = 0; h < NG; ++h)
#pragma unroll
        for (int tk = 0; tk < T; ++tk) O[h][tk] = floatx4{0.f, 0.f, 0.f, 0.f};
    floatx4 Y[T];
    y_of(w, Y);
    floatx4 tv = ttl_of(w);
    floatx4 ev[NG];
#pragma unroll
    for (int h = 0; h < NG; ++h) ev[h] = e_of(w, bo[h]);
    for (int64_t mt = w; mt < ntile; mt += kNceWaves) {
        floatx4 Yn[T];
        y_of(mt + kNceWaves, Yn);  // the next tile, in flight
        const floatx4 tvn = ttl_of(mt + kNceWaves);
        floatx4 evn[NG];
#pragma unroll
        for (int h = 0; h < NG; ++h) evn[h] = e_of(mt + kNceWaves, bo[h]);
        const int64_t m0 = mt * 16;
#pragma unroll
        for (int h = 0; h < NG; ++h) {
            floatx4 p;
#pragma unroll
            for (int r = 0; r < 4; ++r)
                p[r] = (bo[h] >= 0 && m0 + 4 * g + r < B) ? ev[h][r] / (mode == 0 ? ttl_own[h] : tv[r]) : 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int tk = 0; tk < T; ++tk) O[h][tk] = mfma4(p[r], Y[tk][r], O[h][tk]);
        }
#pragma unroll
        for (int tk = 0; tk < T; ++tk) Y[tk] = Yn[tk];
        tv = tvn;
#pragma unroll
        for (int h = 0; h < NG; ++h) ev[h] = evn[h];
    }
    // the waves' partials summed in wave order, one group at a time through `red`; wave h
    // finishes group h
    Fld<D> S;
#pragma unroll
    for (int h = 0; h < NG; ++h) {
        if (h) __syncthreads();  // wave h - 1 has read the previous group
        // lane (c, g) holds O[own 4g + q][feature 16 tk + c]
#pragma unroll
        for (int tk = 0; tk < T; ++tk)
#pragma unroll
            for (int q = 0; q < 4; ++q) red[w][4 * g + q][(16 * tk + c + rot(4 * g + q)) & (D - 1)] = O[h][tk][q];
        __syncthreads();
        if (w == h) {
#pragma unroll
            for (int t = 0; t < T; ++t) {
                const int col = (16 * t + 4 * g + rot(c)) & (D - 1);
                floatx4 s = *reinterpret_cast<const floatx4*>(&red[0][c][col]);
#pragma unroll
                for (int i = 1; i < kNceWaves; ++i) s += *reinterpret_cast<const floatx4*>(&red[i][c][col]);
                S.f[t] = s;
            }
        }
    }
    if (w >= NG) return;
    const int64_t own = bo[w];
    if (own < 0) return;
    const Fld<D> X = fload<D>(own_n, own, g);
    const float coef = (a.gloss[term * a.gstride] * a.gscale) * (1.f / a.tau) / (float)B;
    const Fld<D> Z = fload<D>(oth_n, own, g);  // the own row's other view
    const Fld<D> dn = fmap2<D>(S, Z, [&](float o, float z) { return coef * (o - z); });
    const float nx = a.norms[(term * 2 + mode) * B + own];
    Fld<D> dv;
    if (nx > 1e-12f) {
        const float yd = rsum<D>(fmap2<D>(X, dn, [](float u, float v) { return u * v; }));
        dv = fmap2<D>(dn, X, [&](float u, float y) { return (u - y * yd) / nx; });
    } else {
        dv = fmap<D>(dn, [](float u) { return u / 1e-12f; });
    }
    float* dst = (mode == 0 ? a.g1 : a.g2) + (a.idx[term][own] + a.off[term]) * D;
    if (a.rows) {
#pragma unroll
        for (int t = 0; t < T; ++t) st4(dst + 16 * t + 4 * g, make_float4(dv.f[t][0], dv.f[t][1], dv.f[t][2], dv.f[t][3]));
        return;
    }
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) atomicAdd(dst + 16 * t + 4 * g + r, dv.f[t][r]);
}

// ---------------------------------------------------------------------------
// multi-tensor Adam
// ---------------------------------------------------------------------------
constexpr int kAdamMax = 32, kAdamPerBlock = 2048;

struct AdamList {
    float* p[kAdamMax];
    const float* g[kAdamMax];
    float* m[kAdamMax];
    float* v[kAdamMax];
    const int64_t* step[kAdamMax];
    int64_t n[kAdamMax];
    int64_t blk[kAdamMax + 1];
    uint32_t vec4;       // bit i: tensor i is float4-aligned with n % 4 == 0
    int32_t count;
    float lr, beta1, beta2, eps, wd;
    float gscale;        // the gradient is g * gscale (f32 product, as torch's grad.mul_(s)); 1 = none
    const double* lr_dev;  // if non-NULL the learning rate is read here (graph replays across lr changes)
    const int32_t* halt;   // if non-NULL and *halt != 0 (a NaN loss, rsx_nan_gate) nothing is updated
    // the mirror gradient's restore folded in (rsx_adam_multi_mg): with ralpha non-NULL,
    // p = p + rx * float(*ralpha * rmult [* lr]) first (axpy_multi's two roundings), then Adam
    const float* rx[kAdamMax];
    const double* ralpha;
    double rmult;
};

// y + x * s with two roundings (torch's mul then add_; no contraction): axpy_multi's arithmetic
__device__ __forceinline__ float restore1(float y, float x, float s) {
#pragma clang fp contract(off)
    return y + x * s;
}

__global__ __launch_bounds__(256) void adam_multi(AdamList L) {
    if (L.halt && *L.halt) return;
    int t = 0;
    while (t + 1 < L.count && (int64_t)blockIdx.x >= L.blk[t + 1]) ++t;
    rsx_adam cfg;
    cfg.lr = L.lr_dev ? (float)*L.lr_dev : L.lr;
    cfg.beta1 = L.beta1;
    cfg.beta2 = L.beta2;
    cfg.eps = L.eps;
    cfg.weight_decay = L.wd;
    cfg.step_dev = L.step[t];
    cfg.step = 1;
    const AdamConst c = adam_const(cfg);
    float* __restrict__ p = L.p[t];
    const float* __restrict__ gr = L.g[t];
    float* __restrict__ m = L.m[t];
    float* __restrict__ v = L.v[t];
    const int64_t base = ((int64_t)blockIdx.x - L.blk[t]) * kAdamPerBlock;
    const int64_t n = L.n[t];
    const float* __restrict__ rx = L.ralpha ? L.rx[t] : nullptr;
    const float rs = rx ? (float)(*L.ralpha * (L.lr_dev ? L.rmult * *L.lr_dev : L.rmult)) : 0.f;
    if ((L.vec4 >> t) & 1u) {
#pragma unroll
        for (int k = 0; k < kAdamPerBlock / 1024; ++k) {
            const int64_t i = base + 4 * (k * 256 + threadIdx.x);
            if (i < n) {
                float4 pp = ld4(p + i), mm = ld4(m + i), vv = ld4(v + i);
                float4 gg = ld4(gr + i);
                if (rx) {
                    const float4 xx = ld4(rx + i);
                    pp = make_float4(restore1(pp.x, xx.x, rs), restore1(pp.y, xx.y, rs), restore1(pp.z, xx.z, rs),
                                     restore1(pp.w, xx.w, rs));
                }
                if (L.gscale != 1.f) gg = mul4(L.gscale, gg);
                adam_elem(c, pp.x, mm.x, vv.x, gg.x);
                adam_elem(c, pp.y, mm.y, vv.y, gg.y);
                adam_elem(c, pp.z, mm.z, vv.z, gg.z);
                adam_elem(c, pp.w, mm.w, vv.w, gg.w);
                st4(p + i, pp);
                st4(m + i, mm);
                st4(v + i, vv);
            }
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < kAdamPerBlock / 256; ++k) {
        const int64_t i = base + k * 256 + threadIdx.x;
        if (i < n) {
            float pp = p[i], mm = m[i], vv = v[i];
            if (rx) pp = restore1(pp, rx[i], rs);
            adam_elem(c, pp, mm, vv, L.gscale != 1.f ? gr[i] * L.gscale : gr[i]);
            p[i] = pp;
            m[i] = mm;
            v[i] = vv;
        }
    }
}

// the batch loss's NaN check (reference src/common/trainer.py:192-203) on the device:
// one lane counts the batch and, on the first NaN loss, records {1, its 1-based index}
__global__ void nan_gate(const float* loss, int32_t* halt, int32_t* counter) {
    if (threadIdx.x != 0) return;
    const int32_t c = counter[0] + 1;
    counter[0] = c;
    const float x = loss[0];
    if (x != x && halt[0] == 0) {
        halt[1] = c;
        halt[0] = 1;
    }
}

// ---------------------------------------------------------------------------
// model-level mirror gradient (reference src/common/trainer.py:268-348)
// ---------------------------------------------------------------------------
// The scale alpha_eff = clamp(max(base, rel * rms(p) / (lr * rms(g) + 1e-12)), base * max)
// from ONE pass over every (p, g) pair (per-block f64 sums of squares, reduced in
// block order: deterministic), and p += float(alpha * mult) * g over the list in one
// launch (the reference's per-parameter p.add_(-alpha * lr * g) and its restore).
struct PairList {
    float* y[kAdamMax];
    const float* x[kAdamMax];
    int64_t n[kAdamMax];
    int64_t blk[kAdamMax + 1];
    int32_t count;
    uint32_t vec4;  // bit i: pair i is float4-aligned with n % 4 == 0
};

__device__ __forceinline__ int list_slot(const PairList& L) {
    int t = 0;
    while (t + 1 < L.count && (int64_t)blockIdx.x >= L.blk[t + 1]) ++t;
    return t;
}

// partial[block] = (sum g^2, sum p^2) over the block's 2048 elements (x = g, y = p)
__global__ __launch_bounds__(256) void mg_sumsq(PairList L, double* partial) {
    const int t = list_slot(L);
    const int64_t base = ((int64_t)blockIdx.x - L.blk[t]) * kAdamPerBlock;
    double sg = 0.0, sp = 0.0;
    if ((L.vec4 >> t) & 1u) {  // float4 loads, both of a thread's chunks in flight together
        float4 gv[kAdamPerBlock / 1024], pv[kAdamPerBlock / 1024];
#pragma unroll
        for (int k = 0; k < kAdamPerBlock / 1024; ++k) {
            const int64_t i = base + 4 * (k * 256 + threadIdx.x);
            const bool ok = i < L.n[t];
            gv[k] = ok ? ld4(L.x[t] + i) : f4(0.f);
            pv[k] = ok ? ld4(L.y[t] + i) : f4(0.f);
        }
#pragma unroll
        for (int k = 0; k < kAdamPerBlock / 1024; ++k) {
            sg += (double)gv[k].x * gv[k].x + (double)gv[k].y * gv[k].y + (double)gv[k].z * gv[k].z +
                  (double)gv[k].w * gv[k].w;
            sp += (double)pv[k].x * pv[k].x + (double)pv[k].y * pv[k].y + (double)pv[k].z * pv[k].z +
                  (double)pv[k].w * pv[k].w;
        }
    } else {
        for (int k = 0; k < kAdamPerBlock / 256; ++k) {
            const int64_t i = base + k * 256 + threadIdx.x;
            if (i < L.n[t]) {
                const double gv = L.x[t][i], pv = L.y[t][i];
                sg += gv * gv;
                sp += pv * pv;
            }
        }
    }
    __shared__ double red[2][4];
    sg = group_sum_d<64>(sg);
    sp = group_sum_d<64>(sp);
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = sg;
        red[1][threadIdx.x >> 6] = sp;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        partial[2 * blockIdx.x] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
        partial[2 * blockIdx.x + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    }
}

// one 1024-thread block: the block sums thread-strided (independent loads in flight),
// then a fixed tree (deterministic), then the reference's scalar arithmetic: rms
// values as f32 tensor results, the rest in f64
constexpr int kMgFinal = 1024;
__global__ __launch_bounds__(kMgFinal) void mg_alpha_final(const double* partial, int64_t n_blocks, int64_t numel,
                                                           double base, double lr, double rel, double max_scale,
                                                           double* alpha, const double* lr_dev) {
    double sg0 = 0.0, sp0 = 0.0, sg1 = 0.0, sp1 = 0.0;
    int64_t b = threadIdx.x;
    for (; b + kMgFinal < n_blocks; b += 2 * kMgFinal) {
        sg0 += partial[2 * b];
        sp0 += partial[2 * b + 1];
        sg1 += partial[2 * (b + kMgFinal)];
        sp1 += partial[2 * (b + kMgFinal) + 1];
    }
    if (b < n_blocks) {
        sg0 += partial[2 * b];
        sp0 += partial[2 * b + 1];
    }
    double sg = group_sum_d<64>(sg0 + sg1);
    double sp = group_sum_d<64>(sp0 + sp1);
    __shared__ double red[2][kMgFinal / 64];
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = sg;
        red[1][threadIdx.x >> 6] = sp;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    sg = 0.0;
    sp = 0.0;
    for (int w = 0; w < kMgFinal / 64; ++w) {
        sg += red[0][w];
        sp += red[1][w];
    }
    const float sq = (float)sqrt((double)numel);
    const double grad_rms = (double)((float)sqrt(sg) / sq);
    const double param_rms = (double)((float)sqrt(sp) / sq + 1e-12f);
    if (lr_dev) lr = *lr_dev;
    double a = rel * param_rms / (lr * grad_rms + 1e-12);
    a = a > base ? a : base;  // Python max(base, x): keeps base when x is NaN
    const double cap = base * max_scale;
    *alpha = a < cap ? a : cap;
}

// y += float(alpha * mult) * x
__global__ __launch_bounds__(256) void axpy_multi(PairList L, const double* alpha, double mult, const double* lr_dev,
                                                   const int32_t* halt) {
#pragma clang fp contract(off)  // two roundings, as torch's mul then add_ (device code contracts by default)
    if (halt && *halt) return;
    const int t = list_slot(L);
    const float s = (float)(*alpha * (lr_dev ? mult * *lr_dev : mult));
    const int64_t base = ((int64_t)blockIdx.x - L.blk[t]) * kAdamPerBlock;
    float* __restrict__ y = L.y[t];
    const float* __restrict__ x = L.x[t];
    if ((L.vec4 >> t) & 1u) {
#pragma unroll
        for (int k = 0; k < kAdamPerBlock / 1024; ++k) {
            const int64_t i = base + 4 * (k * 256 + threadIdx.x);
            if (i < L.n[t]) {
                const float4 yy = ld4(y + i), xx = ld4(x + i);
                st4(y + i, make_float4(yy.x + xx.x * s, yy.y + xx.y * s, yy.z + xx.z * s, yy.w + xx.w * s));
            }
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < kAdamPerBlock / 256; ++k) {
        const int64_t i = base + k * 256 + threadIdx.x;
        if (i < L.n[t]) y[i] = y[i] + x[i] * s;
    }
}

// ---------------------------------------------------------------------------
// spectral filter weights: unit normalisation w / (|w| + 1e-8) (smore.py:221-229)
// ---------------------------------------------------------------------------
// three [nb][2] (re, im) weights -> out [3][nb][2]
__global__ __launch_bounds__(256) void unit_w_fwd(const float* w0, const float* w1, const float* w2, int nb,
                                                  int normalize, float* out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= 3 * nb) return;
    const float* w = i < nb ? w0 : (i < 2 * nb ? w1 : w2);
    const int b = i % nb;
    const float re = w[2 * b], im = w[2 * b + 1];
    if (normalize) {
        const float den = hypotf(re, im) + 1e-8f;  // torch.abs(complex) + 1e-8, then a complex / real division
        out[2 * i] = re / den;
        out[2 * i + 1] = im / den;
    } else {
        out[2 * i] = re;
        out[2 * i + 1] = im;
    }
}

// d w from the spectral backward's per-block partials [nblk][3][nb][2] through the
// normalisation: w~ = w / den, den = |w| + eps:
// d w = g / den - <g, w> w / (|w| den^2)  (|w| = 0: torch's sgn(0) = 0, no second term).
// One block per weight entry i: the partials thread-strided over the blocks, then a
// fixed tree (deterministic).
__global__ __launch_bounds__(256) void unit_w_bwd(const float* part, int nblk, const float* w0, const float* w1,
                                                  const float* w2, int nb, int normalize, float* g0, float* g1,
                                                  float* g2) {
    const int i = blockIdx.x;
    float ga = 0.f, gb = 0.f;
    for (int k = threadIdx.x; k < nblk; k += 256) {
        const float2 v = *reinterpret_cast<const float2*>(part + ((int64_t)k * 3 * nb + i) * 2);
        ga += v.x;
        gb += v.y;
    }
    ga = group_sum<64>(ga);
    gb = group_sum<64>(gb);
    __shared__ float red[2][4];
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = ga;
        red[1][threadIdx.x >> 6] = gb;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    ga = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    gb = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    const int m = i / nb, b = i % nb;
    const float* w = m == 0 ? w0 : (m == 1 ? w1 : w2);
    float* g = m == 0 ? g0 : (m == 1 ? g1 : g2);
    if (normalize) {
        const float re = w[2 * b], im = w[2 * b + 1];
        const float r = hypotf(re, im), den = r + 1e-8f;
        float da = ga / den, db = gb / den;
        if (r > 0.f) {
            const float k = (ga * re + gb * im) / (den * den) / r;
            da -= k * re;
            db -= k * im;
        }
        ga = da;
        gb = db;
    }
    g[2 * b] = ga;
    g[2 * b + 1] = gb;
}

}  // namespace sf
}  // namespace rsx

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
using namespace rsx;


extern "C" {

int rsx_smore_gates(int32_t backward, const float* const* conv, const float* item, const float* const* W,
                    const float* const* b, int64_t n, int32_t d, float scale, int32_t mul, float* const* out,
                    const float* const* gout, float* g_item, float* const* g_conv, float* const* dz,
                    rsx_stream_t stream) {
    return rsx_smore_gates_saved(backward, conv, item, W, b, n, d, scale, mul, out, gout, g_item, g_conv, dz,
                                 nullptr, stream);
}

int rsx_smore_gates_saved(int32_t backward, const float* const* conv, const float* item, const float* const* W,
                          const float* const* b, int64_t n, int32_t d, float scale, int32_t mul, float* const* out,
                          const float* const* gout, float* g_item, float* const* g_conv, float* const* dz,
                          float* saved, rsx_stream_t stream) {
    if (n < 0 || !conv || !item || !W || !b) return RSX_ERR_ARG;
    if (n == 0) return RSX_OK;
    sf::GateArgs a{};
    for (int m = 0; m < 3; ++m) {
        a.conv[m] = conv[m];
        a.W[m] = W[m];
        a.b[m] = b[m];
        if (!conv[m] || !W[m]) return RSX_ERR_ARG;
        if (backward) {
            if (!g_conv || !dz || !g_conv[m] || !dz[m]) return RSX_ERR_ARG;
            a.gout[m] = gout ? gout[m] : nullptr;
            a.g_conv[m] = g_conv[m];
            a.dz[m] = dz[m];
        } else {
            if (!out || !out[m]) return RSX_ERR_ARG;
            a.out[m] = out[m];
        }
    }
    if (backward && !g_item) return RSX_ERR_ARG;
    a.item = item;
    a.n = n;
    a.scale = scale;
    a.mul = mul;
    a.g_item = g_item;
    a.saved = saved;  // the mul-mode backward (gates_bwd) recomputes the sigmoids regardless
    // one gate per block row, except the mul-mode backward (its g_item needs all three
    // sigmoids of a row: one block runs the three gates)
    a.nbx = ((n + 15) / 16 + 3) / 4;
    // blocks: the row blocks, at most RSX_GATE_BLOCKS (default: 2 per CU -- the LDS
    // weight copy allows two; each block then strides over its row blocks)
    const unsigned gy = (backward && mul) ? 1u : 3u;
    static const int64_t cap_env = env_knob("RSX_GATE_BLOCKS", 0, 1, 1 << 20);
    int64_t gx = a.nbx;
    const int64_t cap = cap_env > 0 ? cap_env : (int64_t)(2 * device_cus()) / gy;
    if (cap > 0 && gx > cap) gx = cap;
    const dim3 grid((unsigned)gx, gy);
    hipStream_t s = as_stream(stream);
    switch (d) {
        case 64:
            if (backward && !mul && saved) hipLaunchKernelGGL(sf::gates_bwd_res_sv<64>, grid, dim3(256), 0, s, a);
            else if (backward && !mul) hipLaunchKernelGGL(sf::gates_bwd_res<64>, grid, dim3(256), 0, s, a);
            else if (backward) hipLaunchKernelGGL(sf::gates_bwd<64>, grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL(sf::gates_fwd<64>, grid, dim3(256), 0, s, a);
            break;
        case 128:
            if (backward && !mul && saved) hipLaunchKernelGGL(sf::gates_bwd_res_sv<128>, grid, dim3(256), 0, s, a);
            else if (backward && !mul) hipLaunchKernelGGL(sf::gates_bwd_res<128>, grid, dim3(256), 0, s, a);
            else if (backward) hipLaunchKernelGGL(sf::gates_bwd<128>, grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL(sf::gates_fwd<128>, grid, dim3(256), 0, s, a);
            break;
        default: return RSX_ERR_UNSUPPORTED;
    }
    return last_rc();
}

int rsx_smore_pref(int32_t backward, const float* const* W, const float* const* b, const float* content,
                   const float* image_emb, const float* text_emb, const float* fusion_emb, int64_t n, int32_t d,
                   float p_drop, const int64_t* seed_dev, float* all_out, float* side_out, const float* g_all,
                   const float* g_side, float* g_content, float* g_image, float* g_text, float* g_fusion,
                   float* hv, float* ht, float* const* dz, rsx_stream_t stream) {
    return rsx_smore_pref_rows(backward, W, b, content, image_emb, text_emb, fusion_emb, nullptr, n, d, p_drop,
                               seed_dev, all_out, side_out, nullptr, nullptr, g_all, g_side, nullptr, g_content,
                               g_image, g_text, g_fusion, hv, ht, dz, nullptr, stream);
}

int rsx_tag_rows_next(int32_t* row_tag, const int64_t* rows, int64_t n, int32_t* tag2, rsx_stream_t stream) {
    if (n < 0 || !row_tag || !tag2 || (n > 0 && !rows)) return RSX_ERR_ARG;
    if (n == 0) n = 1, rows = nullptr;  // still one block: the bump
    const int64_t nb = (n + 255) / 256;
    if (nb > 0x7fffffffll) return RSX_ERR_UNSUPPORTED;
    if (!rows) {  // no rows: the bump alone (one thread's worth of work in one block)
        hipLaunchKernelGGL(sf::tag_rows_next_k, dim3(1), dim3(256), 0, as_stream(stream), row_tag, rows, (int64_t)0,
                           tag2);
        return last_rc();
    }
    hipLaunchKernelGGL(sf::tag_rows_next_k, dim3((unsigned)nb), dim3(256), 0, as_stream(stream), row_tag, rows, n, tag2);
    return last_rc();
}

int rsx_tag_rows(int32_t* row_tag, const int64_t* rows, int64_t n, const int32_t* tag_dev, rsx_stream_t stream) {
    if (!row_tag || !tag_dev || n < 0 || (n > 0 && !rows)) return RSX_ERR_ARG;
    if (n == 0) return RSX_OK;
    hipLaunchKernelGGL(sf::tag_rows_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), row_tag,
                       rows, n, tag_dev);
    return last_rc();
}

// RSX_SEGSUM_GLOBAL=1: the per-row sums read the row ids from global memory even when
// they fit the LDS copy (timing A/B; the two kernels give identical results)
static bool seg_global() {
    static const bool v = env_knob("RSX_SEGSUM_GLOBAL", 0, 0, 1) != 0;
    return v;
}

int rsx_smore_pref_rows(int32_t backward, const float* const* W, const float* const* b, const float* content,
                        const float* image_emb, const float* text_emb, const float* fusion_emb, const int64_t* rows,
                        int64_t n, int32_t d, float p_drop, const int64_t* seed_dev, float* all_out,
                        float* side_out, float* content_out, float* fusion_out, const float* g_all,
                        const float* g_side, const float* g_content_in, float* g_content, float* g_image,
                        float* g_text, float* g_fusion, float* hv, float* ht, float* const* dz, float* occ,
                        rsx_stream_t stream) {
    return rsx_smore_pref_rows_saved(backward, W, b, content, image_emb, text_emb, fusion_emb, rows, n, d, p_drop,
                                     seed_dev, all_out, side_out, content_out, fusion_out, g_all, g_side,
                                     g_content_in, g_content, g_image, g_text, g_fusion, hv, ht, dz, occ, nullptr,
                                     nullptr, nullptr, stream);
}

int rsx_smore_pref_rows_saved(int32_t backward, const float* const* W, const float* const* b, const float* content,
                              const float* image_emb, const float* text_emb, const float* fusion_emb,
                              const int64_t* rows, int64_t n, int32_t d, float p_drop, const int64_t* seed_dev,
                              float* all_out, float* side_out, float* content_out, float* fusion_out,
                              const float* g_all, const float* g_side, const float* g_content_in, float* g_content,
                              float* g_image, float* g_text, float* g_fusion, float* hv, float* ht, float* const* dz,
                              float* occ, float* saved, int32_t* plan, uint64_t* lead, rsx_stream_t stream) {
    if (n < 0 || !W || !b || !content || !image_emb || !text_emb || !fusion_emb) return RSX_ERR_ARG;
    if (occ && (!backward || !rows)) return RSX_ERR_ARG;
    // the saved activations exist for the batch-row split forward (scratch hv) and its backward
    if (saved && (!rows || (!backward && !hv))) return RSX_ERR_ARG;
    // the occurrence plan: built by the split forward (lead scratch needed), read by the backward's sums
    if (plan && (!rows || n > 0x7fffffffll || (backward ? !occ : (!hv || !lead)))) return RSX_ERR_ARG;
    if (p_drop < 0.f || p_drop >= 1.f || (p_drop > 0.f && !seed_dev)) return RSX_ERR_ARG;
    if (n == 0) return RSX_OK;
    sf::PrefArgs a{};
    for (int i = 0; i < sf::kNW; ++i) {
        if (!W[i]) return RSX_ERR_ARG;
        a.W[i] = W[i];
        a.b[i] = b[i];
        if (backward) {
            if (!dz || !dz[i]) return RSX_ERR_ARG;
            a.dz[i] = dz[i];
        }
    }
    if (backward ? (!g_all || !g_content || !g_image || !g_text || !g_fusion || (!saved && (!hv || !ht)))
                 : (!all_out || !side_out))
        return RSX_ERR_ARG;
    a.C = content;
    a.IE = image_emb;
    a.TE = text_emb;
    a.FE = fusion_emb;
    a.n = n;
    a.p_drop = p_drop;
    a.drop_scale = p_drop > 0.f ? (float)(1.0 / (1.0 - (double)p_drop)) : 1.f;
    a.seed = seed_dev;
    a.all = all_out;
    a.side = side_out;
    a.g_all = g_all;
    a.g_side = g_side;
    a.gC = g_content;
    a.gIE = g_image;
    a.gTE = g_text;
    a.gFE = g_fusion;
    a.hv = hv;
    a.ht = ht;
    a.rows = rows;
    a.c_out = backward ? nullptr : content_out;
    a.fe_out = backward ? nullptr : fusion_out;
    a.g_cin = backward ? g_content_in : nullptr;
    a.occ = occ;
    a.saved = saved;
    a.plan = backward ? nullptr : plan;  // the kernels build it in the forward only
    a.lead = reinterpret_cast<unsigned long long*>(lead);
    // batch-row backward: the three views' chains as three block rows (gradients are atomics
    // there); batch-row forward with the scratch hv: likewise, then pref_combine
    const bool split_fwd = !backward && rows && hv;
    const dim3 grid((unsigned)(((n + 15) / 16 + 3) / 4), backward && rows ? 5 : split_fwd ? 3 : 1);
    hipStream_t s = as_stream(stream);
    if (split_fwd) {
        if (n == 0) return RSX_OK;
        if (d == 64) hipLaunchKernelGGL(sf::pref_fwd_rows<64>, grid, dim3(256), 0, s, a);
        else if (d == 128) hipLaunchKernelGGL(sf::pref_fwd_rows<128>, grid, dim3(256), 0, s, a);
        else return RSX_ERR_UNSUPPORTED;
        const dim3 gc((unsigned)((n * d / 4 + 255) / 256));
        if (d == 64) hipLaunchKernelGGL(sf::pref_combine<64>, gc, dim3(256), 0, s, a);
        else hipLaunchKernelGGL(sf::pref_combine<128>, gc, dim3(256), 0, s, a);
        return last_rc();
    }
    switch (d) {
        case 64:
            if (backward && saved) hipLaunchKernelGGL(sf::pref_bwd_rows_sv<64>, grid, dim3(256), 0, s, a);
            else if (backward && rows) hipLaunchKernelGGL(sf::pref_bwd_rows<64>, grid, dim3(256), 0, s, a);
            else if (backward) hipLaunchKernelGGL(sf::pref_bwd<64>, grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL(sf::pref_fwd<64>, grid, dim3(256), 0, s, a);
            break;
        case 128:
            if (backward && saved) hipLaunchKernelGGL(sf::pref_bwd_rows_sv<128>, grid, dim3(256), 0, s, a);
            else if (backward && rows) hipLaunchKernelGGL(sf::pref_bwd_rows<128>, grid, dim3(256), 0, s, a);
            else if (backward) hipLaunchKernelGGL(sf::pref_bwd<128>, grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL(sf::pref_fwd<128>, grid, dim3(256), 0, s, a);
            break;
        default: return RSX_ERR_UNSUPPORTED;
    }
    if (occ) {  // the per-occurrence rows summed per table row (deterministic)
        if (n > 0x7fffffffll) return RSX_ERR_UNSUPPORTED;  // occurrence indices listed as int32
        if (plan) {  // the forward's occurrence plan
            const dim3 sg((unsigned)((n + 3) / 4));
            if (d == 64) hipLaunchKernelGGL(sf::pref_segsum_plan<64>, sg, dim3(256), 0, s, rows, n, plan, occ, g_content, g_image, g_text, g_fusion);
            else hipLaunchKernelGGL(sf::pref_segsum_plan<128>, sg, dim3(256), 0, s, rows, n, plan, occ, g_content, g_image, g_text, g_fusion);
        } else if (n <= sf::kSegLds && !seg_global()) {  // row ids < 2^31 (table rows)
            const dim3 sg((unsigned)((n + sf::kSegWaves - 1) / sf::kSegWaves)), sb(64 * sf::kSegWaves);
            if (d == 64) hipLaunchKernelGGL(sf::pref_segsum_lds<64>, sg, sb, 0, s, rows, n, occ, g_content, g_image, g_text, g_fusion);
            else hipLaunchKernelGGL(sf::pref_segsum_lds<128>, sg, sb, 0, s, rows, n, occ, g_content, g_image, g_text, g_fusion);
        } else {
            const dim3 sg((unsigned)((n + 3) / 4));
            if (d == 64) hipLaunchKernelGGL(sf::pref_segsum<64>, sg, dim3(256), 0, s, rows, n, occ, g_content, g_image, g_text, g_fusion);
            else hipLaunchKernelGGL(sf::pref_segsum<128>, sg, dim3(256), 0, s, rows, n, occ, g_content, g_image, g_text, g_fusion);
        }
    }
    return last_rc();
}

size_t rsx_smore_pref_rows_occ_floats(int64_t n, int32_t d) { return (size_t)sf::kOcc * (size_t)n * (size_t)d; }
size_t rsx_smore_pref_rows_saved_floats(int64_t n, int32_t d) { return (size_t)sf::kSv * (size_t)n * (size_t)d; }
size_t rsx_smore_pref_plan_words(int64_t n) { return (size_t)n * (size_t)(1 + sf::kPlanCap); }

size_t rsx_smore_wgrad_ws_bytes(int64_t n, int32_t d, int32_t n_pairs) {
    const int64_t rows = sf::wg_rows(n, d, n_pairs);
    const int64_t splits = (n + rows - 1) / rows;
    return (size_t)(n_pairs > 0 ? n_pairs : 0) * (size_t)(splits > 0 ? splits : 1) * (size_t)(d * d + d) * 4;
}

int rsx_smore_wgrad(int32_t n_pairs, const float* const* dz, const float* const* x, float* const* dw,
                    float* const* db, int64_t n, int32_t d, void* ws, size_t ws_bytes, rsx_stream_t stream) {
    if (n_pairs <= 0 || n_pairs > sf::kWgPairs || n < 0 || !dz || !x || !dw) return RSX_ERR_ARG;
    if (d != 64 && d != 128) return RSX_ERR_UNSUPPORTED;
    hipStream_t s = as_stream(stream);
    if (n == 0) {
        for (int i = 0; i < n_pairs; ++i) {
            if (hipMemsetAsync(dw[i], 0, (size_t)d * d * 4, s) != hipSuccess) return last_rc();
            if (db && db[i] && hipMemsetAsync(db[i], 0, (size_t)d * 4, s) != hipSuccess) return last_rc();
        }
        return RSX_OK;
    }
    if (ws_bytes < rsx_smore_wgrad_ws_bytes(n, d, n_pairs) || !ws) return RSX_ERR_WORKSPACE;
    sf::WgArgs a{};
    for (int i = 0; i < n_pairs; ++i) {
        if (!dz[i] || !x[i] || !dw[i]) return RSX_ERR_ARG;
        a.dz[i] = dz[i];
        a.x[i] = x[i];
        a.dw[i] = dw[i];
        a.db[i] = db ? db[i] : nullptr;
    }
    a.n_pairs = n_pairs;
    a.n = n;
    a.rows = sf::wg_rows(n, d, n_pairs);
    a.n_splits = (int32_t)((n + a.rows - 1) / a.rows);
    a.part = static_cast<float*>(ws);
    const dim3 g1((unsigned)a.n_splits, (unsigned)n_pairs);
    const dim3 g2((unsigned)((d * d + d + 63) / 64), (unsigned)n_pairs);
    if (d == 64) {
        hipLaunchKernelGGL(sf::wgrad_part<64>, g1, dim3(256), 0, s, a);
        hipLaunchKernelGGL(sf::wgrad_reduce<64>, g2, dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL(sf::wgrad_part<128>, g1, dim3(256), 0, s, a);
        hipLaunchKernelGGL(sf::wgrad_reduce<128>, g2, dim3(256), 0, s, a);
    }
    return last_rc();
}

size_t rsx_smore_infonce_ws_bytes(int64_t batch, int32_t d) {
    // the stored exp(S / tau) tiles and the transposed row tiles
    const int64_t e = batch <= sf::kNceStoreMax ? 2 * batch * batch + 4 * ((batch + 15) / 16) * 16 * d : 0;
    return (size_t)(4 * batch * d + 4 * batch + 2 * batch + 2 * batch + e) * 4;
}

static int nce_bwd_launch(sf::NceArgs& a, int64_t batch, int32_t d, hipStream_t s);

static int nce_setup(sf::NceArgs& a, const float* side, const float* content, const int64_t* users,
                     const int64_t* pos_items, int64_t n_users, int64_t batch, int32_t d, float tau, void* ws,
                     size_t ws_bytes) {
    if (!side || !content || !users || !pos_items || batch < 0 || n_users < 0 || !(tau > 0.f)) return RSX_ERR_ARG;
    if (d != 64 && d != 128) return RSX_ERR_UNSUPPORTED;
    if (!ws || ws_bytes < rsx_smore_infonce_ws_bytes(batch, d)) return RSX_ERR_WORKSPACE;
    a.src1 = side;
    a.src2 = content;
    a.idx[0] = pos_items;  // term 0: cl_items = InfoNCE(side_i[pos], content_i[pos])
    a.off[0] = n_users;
    a.idx[1] = users;      // term 1: cl_users = InfoNCE(side_u[u], content_u[u])
    a.off[1] = 0;
    a.B = batch;
    a.tau = tau;
    float* f = static_cast<float*>(ws);
    a.nrm = f;
    a.norms = a.nrm + 4 * batch * d;
    a.ttl = a.norms + 4 * batch;
    a.lrow = a.ttl + 2 * batch;
    a.E = batch <= sf::kNceStoreMax ? a.lrow + 2 * batch : nullptr;
    static const int t64 = env_knob("RSX_NCE_T64", 1, 0, 1);
    a.nrmT = a.E && (d == 128 || t64) ? a.E + 2 * batch * batch : nullptr;  // read by nce_bwd_t only
    return RSX_OK;
}

int rsx_smore_infonce_fwd(const float* side, const float* content, const int64_t* users, const int64_t* pos_items,
                          int64_t n_users, int64_t batch, int32_t d, float tau, float* loss_out, void* ws,
                          size_t ws_bytes, rsx_stream_t stream) {
    return rsx_smore_infonce_fwd_total(side, content, users, pos_items, n_users, batch, d, tau, loss_out, nullptr, 0.f,
                                       nullptr, ws, ws_bytes, stream);
}

int rsx_smore_infonce_fwd_total(const float* side, const float* content, const int64_t* users,
                                const int64_t* pos_items, int64_t n_users, int64_t batch, int32_t d, float tau,
                                float* loss_out, const float* add_loss, float cl, float* total_out, void* ws,
                                size_t ws_bytes, rsx_stream_t stream) {
    sf::NceArgs a{};
    int rc = nce_setup(a, side, content, users, pos_items, n_users, batch, d, tau, ws, ws_bytes);
    if (rc) return rc;
    if (!loss_out || (total_out && !add_loss)) return RSX_ERR_ARG;
    a.loss = loss_out;
    a.add_loss = add_loss;
    a.cl = cl;
    a.total = total_out;
    hipStream_t s = as_stream(stream);
    if (batch == 0) return hip_rc(hipMemsetAsync(loss_out, 0xff, 8, s));  // mean of nothing: NaN
    const dim3 grid((unsigned)((batch + 15) / 16), 2);
    if (d == 64) {
        hipLaunchKernelGGL(sf::nce_norm<64>, grid, dim3(64), 0, s, a);
        hipLaunchKernelGGL(sf::nce_fwd<64>, grid, dim3(64 * sf::kNceWaves), 0, s, a);
    } else {
        hipLaunchKernelGGL(sf::nce_norm<128>, grid, dim3(64), 0, s, a);
        hipLaunchKernelGGL(sf::nce_fwd<128>, grid, dim3(64 * sf::kNceWaves), 0, s, a);
    }
    hipLaunchKernelGGL(sf::nce_mean, dim3(1), dim3(128), 0, s, a);
    return last_rc();
}

int rsx_smore_infonce_bwd(const float* side, const float* content, const int64_t* users, const int64_t* pos_items,
                          int64_t n_users, int64_t batch, int32_t d, float tau, const float* g_loss, float* g_side,
                          float* g_content, void* ws, size_t ws_bytes, rsx_stream_t stream) {
    return rsx_smore_infonce_bwd_scaled(side, content, users, pos_items, n_users, batch, d, tau, g_loss, 1, 1.f,
                                        g_side, g_content, ws, ws_bytes, stream);
}

int rsx_smore_infonce_bwd_scaled(const float* side, const float* content, const int64_t* users,
                                 const int64_t* pos_items, int64_t n_users, int64_t batch, int32_t d, float tau,
                                 const float* g_loss, int32_t g_stride, float g_scale, float* g_side,
                                 float* g_content, void* ws, size_t ws_bytes, rsx_stream_t stream) {
    sf::NceArgs a{};
    int rc = nce_setup(a, side, content, users, pos_items, n_users, batch, d, tau, ws, ws_bytes);
    if (rc) return rc;
    if (!g_loss || !g_side || !g_content || g_stride < 0) return RSX_ERR_ARG;
    if (batch == 0) return RSX_OK;
    a.gloss = g_loss;
    a.gstride = g_stride;
    a.gscale = g_scale;
    a.g1 = g_side;
    a.g2 = g_content;
    return nce_bwd_launch(a, batch, d, as_stream(stream));
}

int rsx_smore_loss_rows_bwd(const float* side_c, const float* content_c, const int64_t* ar, int64_t batch, int32_t d,
                            float tau, const float* g_total, float cl, const float* g_bpr, float* g_all,
                            float* g_side, float* g_content, void* ws, size_t ws_bytes, rsx_stream_t stream) {
    sf::NceArgs a{};
    int rc = nce_setup(a, side_c, content_c, ar, ar, batch, batch, d, tau, ws, ws_bytes);
    if (rc) return rc;
    if (!g_total || !g_bpr || !g_all || !g_side || !g_content) return RSX_ERR_ARG;
    if (batch == 0) return RSX_OK;
    a.gloss = g_total;
    a.gstride = 0;
    a.gscale = cl;
    a.g1 = g_side;
    a.g2 = g_content;
    a.rows = 1;  // rows [users; positives] each written once (ar = arange(batch))
    a.xg = g_bpr;
    a.xo = g_all;
    a.xn = 3 * batch * d;
    a.z1 = g_side + 2 * batch * d;  // the negatives' rows: no InfoNCE term
    a.z2 = g_content + 2 * batch * d;
    a.zn = batch * d;
    return nce_bwd_launch(a, batch, d, as_stream(stream));
}

static int nce_bwd_launch(sf::NceArgs& a, int64_t batch, int32_t d, hipStream_t s) {
    const dim3 grid((unsigned)((batch + 15) / 16), 2, 2);
    if (a.E && a.nrmT) {  // the forward's exp tiles and transposed rows (same workspace, same batch);
        // d = 64 too since round 6 (its reduction tile conflict-free: C3's backward 81 -> 54 us;
        // RSX_NCE_T64=0 keeps nce_bwd<64> there, the round-5 form, for A/B)
        static const int ng = env_knob("RSX_NCE_GROUPS", 2, 1, 2);
        const dim3 g2((unsigned)((batch + 31) / 32), 2, 2);
        if (d == 128 && ng == 2) hipLaunchKernelGGL((sf::nce_bwd_t<128, 2>), g2, dim3(64 * sf::kNceWaves), 0, s, a);
        else if (d == 128) hipLaunchKernelGGL((sf::nce_bwd_t<128, 1>), grid, dim3(64 * sf::kNceWaves), 0, s, a);
        else if (ng == 2) hipLaunchKernelGGL((sf::nce_bwd_t<64, 2>), g2, dim3(64 * sf::kNceWaves), 0, s, a);
        else hipLaunchKernelGGL((sf::nce_bwd_t<64, 1>), grid, dim3(64 * sf::kNceWaves), 0, s, a);
    } else {
        if (d == 64) hipLaunchKernelGGL(sf::nce_bwd<64>, grid, dim3(64 * sf::kNceWaves), 0, s, a);
        else hipLaunchKernelGGL(sf::nce_bwd<128>, grid, dim3(64 * sf::kNceWaves), 0, s, a);
    }
    return last_rc();
}

int rsx_adam_multi(int32_t count, float* const* p, const float* const* g, float* const* m, float* const* v,
                   const int64_t* const* step_dev, const int64_t* n, float lr, float beta1, float beta2, float eps,
                   float weight_decay, rsx_stream_t stream) {
    return rsx_adam_multi_scaled(count, p, g, m, v, step_dev, n, lr, beta1, beta2, eps, weight_decay, 1.f, nullptr,
                                 nullptr, stream);
}

int rsx_nan_gate(const float* loss, int32_t* halt, int32_t* counter, rsx_stream_t stream) {
    if (!loss || !halt || !counter) return RSX_ERR_ARG;
    hipLaunchKernelGGL(sf::nan_gate, dim3(1), dim3(64), 0, as_stream(stream), loss, halt, counter);
    return last_rc();
}

int rsx_adam_multi_scaled(int32_t count, float* const* p, const float* const* g, float* const* m, float* const* v,
                          const int64_t* const* step_dev, const int64_t* n, float lr, float beta1, float beta2,
                          float eps, float weight_decay, float grad_scale, const double* lr_dev,
                          const int32_t* halt, rsx_stream_t stream) {
    return rsx_adam_multi_mg(count, p, g, m, v, step_dev, n, lr, beta1, beta2, eps, weight_decay, grad_scale, lr_dev,
                             halt, nullptr, nullptr, 0.0, stream);
}

int rsx_adam_multi_mg(int32_t count, float* const* p, const float* const* g, float* const* m, float* const* v,
                      const int64_t* const* step_dev, const int64_t* n, float lr, float beta1, float beta2, float eps,
                      float weight_decay, float grad_scale, const double* lr_dev, const int32_t* halt,
                      const float* const* rx, const double* ralpha, double rmult, rsx_stream_t stream) {
    if (count < 0 || (count > 0 && (!p || !g || !m || !v || !step_dev || !n))) return RSX_ERR_ARG;
    if ((rx != nullptr) != (ralpha != nullptr)) return RSX_ERR_ARG;
    hipStream_t s = as_stream(stream);
    for (int32_t c0 = 0; c0 < count; c0 += sf::kAdamMax) {
        sf::AdamList L{};
        L.lr = lr;
        L.beta1 = beta1;
        L.beta2 = beta2;
        L.eps = eps;
        L.wd = weight_decay;
        L.gscale = grad_scale;
        L.lr_dev = lr_dev;
        L.halt = halt;
        L.ralpha = ralpha;
        L.rmult = rmult;
        int64_t blocks = 0;
        int k = 0;
        // the chunk is tensors [c0, c0 + 32): empty ones are skipped, never carried into the next chunk
        for (int32_t i = c0; i < count && i < c0 + sf::kAdamMax; ++i) {
            if (n[i] < 0 || (n[i] > 0 && (!p[i] || !g[i] || !m[i] || !v[i] || !step_dev[i]))) return RSX_ERR_ARG;
            if (n[i] > 0 && rx && !rx[i]) return RSX_ERR_ARG;
            if (n[i] == 0) continue;
            L.p[k] = p[i];
            L.g[k] = g[i];
            L.m[k] = m[i];
            L.v[k] = v[i];
            L.rx[k] = rx ? rx[i] : nullptr;
            L.step[k] = step_dev[i];
            L.n[k] = n[i];
            L.blk[k] = blocks;
            const uintptr_t al = (uintptr_t)p[i] | (uintptr_t)g[i] | (uintptr_t)m[i] | (uintptr_t)v[i] |
                                 (uintptr_t)(rx ? rx[i] : nullptr);
            if ((n[i] & 3) == 0 && (al & 15) == 0) L.vec4 |= 1u << k;
            blocks += (n[i] + sf::kAdamPerBlock - 1) / sf::kAdamPerBlock;
            ++k;
        }
        L.blk[k] = blocks;
        L.count = k;
        if (blocks > 0) hipLaunchKernelGGL(sf::adam_multi, dim3((unsigned)blocks), dim3(256), 0, s, L);
        const int rc = last_rc();
        if (rc) return rc;
    }
    return RSX_OK;
}

// the pair lists of up to 32 tensors each, in launch order; returns blocks per list
static int build_pair_lists(int32_t count, float* const* y, const float* const* x, const int64_t* n,
                            sf::PairList* lists, int n_lists, int64_t* blocks_out) {
    int li = 0;
    for (int32_t c0 = 0; c0 < count; c0 += sf::kAdamMax, ++li) {
        if (li >= n_lists) return RSX_ERR_ARG;
        sf::PairList& L = lists[li];
        L = sf::PairList{};
        int64_t blocks = 0;
        int k = 0;
        for (int32_t i = c0; i < count && i < c0 + sf::kAdamMax; ++i) {
            if (n[i] < 0 || (n[i] > 0 && (!y[i] || !x[i]))) return RSX_ERR_ARG;
            if (n[i] == 0) continue;
            L.y[k] = y[i];
            L.x[k] = x[i];
            L.n[k] = n[i];
            L.blk[k] = blocks;
            if ((n[i] & 3) == 0 && (((uintptr_t)y[i] | (uintptr_t)x[i]) & 15) == 0) L.vec4 |= 1u << k;
            blocks += (n[i] + sf::kAdamPerBlock - 1) / sf::kAdamPerBlock;
            ++k;
        }
        L.blk[k] = blocks;
        L.count = k;
        blocks_out[li] = blocks;
    }
    return RSX_OK;
}

size_t rsx_mg_alpha_ws_bytes(int32_t count, const int64_t* n) {
    int64_t blocks = 0;
    for (int32_t i = 0; i < count; ++i) blocks += (n[i] + sf::kAdamPerBlock - 1) / sf::kAdamPerBlock;
    return (size_t)(blocks > 0 ? blocks : 1) * 2 * sizeof(double);
}

int rsx_mg_alpha(int32_t count, const float* const* params, const float* const* grads, const int64_t* n,
                 double base, double lr, double rel_step, double max_scale, double* alpha_out, void* ws,
                 size_t ws_bytes, const double* lr_dev, rsx_stream_t stream) {
    if (count <= 0 || count > 8 * sf::kAdamMax || !params || !grads || !n || !alpha_out) return RSX_ERR_ARG;
    if (!ws || ws_bytes < rsx_mg_alpha_ws_bytes(count, n)) return RSX_ERR_WORKSPACE;
    sf::PairList lists[8];
    int64_t blocks[8] = {0};
    const int rc = build_pair_lists(count, const_cast<float* const*>(params), grads, n, lists, 8, blocks);
    if (rc) return rc;
    hipStream_t s = as_stream(stream);
    double* part = static_cast<double*>(ws);
    int64_t off = 0, numel = 0;
    for (int32_t i = 0; i < count; ++i) numel += n[i];
    for (int li = 0; li * sf::kAdamMax < count; ++li) {
        if (blocks[li] > 0) hipLaunchKernelGGL(sf::mg_sumsq, dim3((unsigned)blocks[li]), dim3(256), 0, s, lists[li], part + 2 * off);
        off += blocks[li];
    }
    hipLaunchKernelGGL(sf::mg_alpha_final, dim3(1), dim3(sf::kMgFinal), 0, s, part, off, numel, base, lr, rel_step,
                       max_scale, alpha_out, lr_dev);
    return last_rc();
}

int rsx_axpy_multi(int32_t count, float* const* y, const float* const* x, const int64_t* n,
                   const double* alpha_dev, double mult, const double* lr_dev, const int32_t* halt,
                   rsx_stream_t stream) {
    if (count < 0 || count > 8 * sf::kAdamMax || !alpha_dev || (count > 0 && (!y || !x || !n))) return RSX_ERR_ARG;
    sf::PairList lists[8];
    int64_t blocks[8] = {0};
    const int rc = build_pair_lists(count, y, x, n, lists, 8, blocks);
    if (rc) return rc;
    hipStream_t s = as_stream(stream);
    for (int li = 0; li * sf::kAdamMax < count; ++li)
        if (blocks[li] > 0) hipLaunchKernelGGL(sf::axpy_multi, dim3((unsigned)blocks[li]), dim3(256), 0, s, lists[li], alpha_dev, mult, lr_dev,
                               halt);
    return last_rc();
}

int rsx_smore_unit_weights(const float* wv, const float* wt, const float* wf, int32_t d, int32_t normalize,
                           float* out, rsx_stream_t stream) {
    if (!wv || !wt || !wf || !out || d <= 0) return RSX_ERR_ARG;
    const int nb = d / 2 + 1;
    hipLaunchKernelGGL(sf::unit_w_fwd, dim3((3 * nb + 255) / 256), dim3(256), 0, as_stream(stream), wv, wt, wf, nb,
                       normalize, out);
    return last_rc();
}

int rsx_smore_unit_weights_bwd(const float* partials, int64_t n_blocks, const float* wv, const float* wt,
                               const float* wf, int32_t d, int32_t normalize, float* gv, float* gt, float* gf,
                               rsx_stream_t stream) {
    if (!partials || n_blocks < 0 || !wv || !wt || !wf || !gv || !gt || !gf || d <= 0) return RSX_ERR_ARG;
    const int nb = d / 2 + 1;
    hipLaunchKernelGGL(sf::unit_w_bwd, dim3(3 * nb), dim3(256), 0, as_stream(stream), partials,
                       (int)n_blocks, wv, wt, wf, nb, normalize, gv, gt, gf);
    return last_rc();
}

}  // extern "C"

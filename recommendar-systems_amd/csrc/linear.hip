// linear.hip — weight gradients with a long reduction:  dW = g^T x  with g [n, out],
// x [n, in], n >> out.  Two users in SMORE:
//   * the Linear(d, d) layers (reference src/models/smore.py:106-120: query_v / query_t
//     MLPs, gate_* and gate_*_prefer) applied to all 26k user+item rows: a 64 x 64
//     output with a 26k-long reduction;
//   * the modality projections image_trs / text_trs (:256-259) in the spectral
//     backward: d W_v = d img^T V, a 64 x 4096 output over the 7k items.
// A library GEMM sees a tiny output and runs the long reduction on a few
// workgroups.  Here the reduction is split (WgPlan): each wave computes a 32 x 32*IG
// strip over its rows (fp32 MFMA, exact f32 fma chains, next chunk prefetched, one
// g value feeding IG MFMAs) and writes it to its partial slot; a second pass adds
// the slots in a fixed order.  Deterministic: the result depends only on the shapes.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "rsx_common.hpp"

namespace rsx {

typedef float floatx16 __attribute__((ext_vector_type(16)));

// RSX_LBWD_ABL (timing ablations of the fused backward, tools/build_variant.py only; the
// product build leaves it 0): 1 skips the dx products, 2 skips the dW products, 3 drops the
// sched_group_barrier orderings (the compiler's schedule; results unchanged)
#ifndef RSX_LBWD_ABL
#define RSX_LBWD_ABL 0
#endif

constexpr int kWgChunk = 16;         // rows per wave step: 8 MFMA k-steps of 2 rows
constexpr int kWgTargetWaves = 2048; // two per SIMD (LDS-staged blocks interleave)

// Block geometry: a wave computes a 32 x (32*IG) strip of dW (one A value feeds IG
// MFMAs); the block's 4 waves take OTB strips of rows o (OTB = min(4, out/32)) and
// RW = 4/OTB row groups (16 rows each of every 16*RW-row block step).  Each row
// group of each block writes its own partial (slot s*RW + r); the reduce adds the
// slots in order.
struct WgPlan {
    int ig;        // i tiles per wave (1, 2 or 4)
    int otb, rw;   // o strips per block, row groups per block
    int64_t nob, nib;  // blocks along o and i
    int64_t rows;  // rows per block (multiple of kWgChunk * rw)
    int splits;    // S
    int slots() const { return splits * rw; }
};

static int lin_env(const char* name, int dflt) { return env_knob(name, dflt, 1, 1 << 20); }

// in_dim: a multiple of 4 (float4 rows); the i tiles cover ceil(in_dim / 32) * 32 columns and
// the kernel masks the columns past in_dim (loads as zeros, no stores)
static WgPlan wg_plan(int64_t n, int out_dim, int in_dim, int max_ig = 4, int64_t target_waves = kWgTargetWaves) {
    WgPlan p;
    const int it = (in_dim + 31) / 32, ot = out_dim / 32;
    p.ig = (it % 4 == 0 && max_ig >= 4) ? 4 : (it % 2 == 0 && max_ig >= 2) ? 2 : 1;
    p.otb = ot % 4 == 0 ? 4 : ot % 2 == 0 ? 2 : 1;
    p.rw = 4 / p.otb;
    p.nob = ot / p.otb;
    p.nib = it / p.ig;
    const int64_t grid_waves = p.nob * p.nib * 4;
    // splits rounded down: a grid just over the resident count pays a whole second
    // round for its last few blocks (C5's 768-wide projections: 516 blocks on 512 slots)
    int64_t s = target_waves / grid_waves;
    // partials: at most a quarter of the input bytes (or 4 MB)
    const int64_t in_bytes = n * (int64_t)(out_dim + in_dim) * 4;
    const int64_t slot_bytes = (int64_t)out_dim * in_dim * 4;
    const int64_t cap_bytes = in_bytes / 4 > (4 << 20) ? in_bytes / 4 : (4 << 20);
    const int64_t smax_bytes = cap_bytes / (slot_bytes * p.rw);
    if (s > smax_bytes) s = smax_bytes;
    const int64_t step = (int64_t)kWgChunk * p.rw;
    const int64_t smax_rows = (n + step - 1) / step;  // at least one chunk per row group
    if (s > smax_rows) s = smax_rows;
    if (s < 1) s = 1;
    int64_t rows = (n + s - 1) / s;
    rows = (rows + step - 1) / step * step;
    p.rows = rows;
    p.splits = (int)(n > 0 ? (n + rows - 1) / rows : 1);
    return p;
}

// One block step = CH = 16*RW rows: the block loads the chunk's g[:, o cols] and
// x[:, i cols] slices with float4 loads into LDS (double-buffered, the next chunk's
// loads in flight during this chunk's MFMAs), then row group r computes its 16
// rows from LDS: A = g[2u + h][wo + j], B_q = x[2u + h][32q + j].
//
// DX (the fused projection backward, one block column of o: nob == 1): the same
// pass also writes the input gradient dx = g W of the chunk's rows and the block's
// IC columns (W [out, in] row-major, its [out x IC] slice staged once in LDS;
// 16x16x4 f32 MFMA tiles from the g chunk already in LDS) and, in the blocks of
// the first i column, the bias-gradient partials colsum(g) (the av values the dW
// MFMAs read, summed per lane) into the slot's tail [out] floats.
template <int IG, int OTB, bool DX>
__device__ __forceinline__ void wgrad_partial_body(int64_t bid, const float* __restrict__ g, const float* __restrict__ x,
                                                   int64_t n, int out_dim, int in_dim, int64_t rows, int64_t nob,
                                                   int64_t nib, float* __restrict__ part, const float* __restrict__ W,
                                                   float* __restrict__ dx, int do_db);

template <int IG, int OTB, bool DX = false>
__global__ __launch_bounds__(256) void wgrad_partial(const float* __restrict__ g, const float* __restrict__ x,
                                                     int64_t n, int out_dim, int in_dim, int64_t rows, int64_t nob,
                                                     int64_t nib, float* __restrict__ part,
                                                     const float* __restrict__ W = nullptr, float* __restrict__ dx = nullptr,
                                                     int do_db = 0) {
    wgrad_partial_body<IG, OTB, DX>(blockIdx.x, g, x, n, out_dim, in_dim, rows, nob, nib, part, W, dx, do_db);
}

// Two fused projection backwards of the same rows and output width in one launch (SMORE's
// image and text projections, src/models/smore.py:256-259): blocks [0, nb0) are problem 0's,
// the rest problem 1's, each with its own plan (rows per split, i blocks, partial slots).
struct LbwdProb {
    const float* g;
    const float* x;
    const float* W;
    float* dx;
    float* part;
    int64_t rows, nib;
    int32_t in_dim, do_db;
};

template <int IG, int OTB>
__global__ __launch_bounds__(256) void wgrad_partial_pair(LbwdProb p0, LbwdProb p1, int64_t nb0, int64_t n,
                                                          int out_dim) {
    const bool first = (int64_t)blockIdx.x < nb0;
    const LbwdProb& q = first ? p0 : p1;
    wgrad_partial_body<IG, OTB, true>(first ? (int64_t)blockIdx.x : (int64_t)blockIdx.x - nb0, q.g, q.x, n, out_dim,
                                      q.in_dim, q.rows, 1, q.nib, q.part, q.W, q.dx, q.do_db);
}

template <int IG, int OTB, bool DX>
__device__ __forceinline__ void wgrad_partial_body(int64_t bid, const float* __restrict__ g, const float* __restrict__ x,
                                                   int64_t n, int out_dim, int in_dim, int64_t rows, int64_t nob,
                                                   int64_t nib, float* __restrict__ part, const float* __restrict__ W,
                                                   float* __restrict__ dx, int do_db) {
    constexpr int RW = 4 / OTB;
    constexpr int OC = 32 * OTB, IC = 32 * IG;   // block's o / i columns
    constexpr int CH = kWgChunk * RW;            // rows per block step
    constexpr int GP = OC + 4, XP = IC + 4;      // padded LDS rows
    constexpr int WPT = OC + 4;                  // W^T slice rows (a column of W: o contiguous, 16-B aligned)
    constexpr int NG = CH * OC / 4, NX = CH * IC / 4;  // float4s per step
    constexpr int PER = (NG + NX + 255) / 256;
    __shared__ __attribute__((aligned(16))) float gs[2][CH * GP];
    __shared__ __attribute__((aligned(16))) float xs[2][CH * XP];
    __shared__ __attribute__((aligned(16))) float wl[DX ? IC * WPT : 4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 31, h = lane >> 5;
    const int64_t bo = bid % nob, bi = (bid / nob) % nib, s = bid / (nob * nib);
    const int ob = (int)bo * OC, ib = (int)bi * IC;
    const int wo = (wave % OTB) * 32;  // wave's o strip within the block
    const int r = wave / OTB;          // row group
    const int64_t r0 = s * rows;
    const int64_t r1 = min(n, r0 + rows);
    const int64_t nst = (r1 - r0 + CH - 1) / CH;
    floatx16 acc[IG];
#pragma unroll
    for (int q = 0; q < IG; ++q)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[q][e] = 0.f;
    // global -> registers two steps ahead (st[k & 1]), registers -> LDS one step ahead
    float4 st[2][PER];
    auto gload = [&](int64_t c, float4(&v)[PER]) __attribute__((always_inline)) {
        const int64_t c0 = r0 + c * CH;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int e = threadIdx.x + 256 * k;
            float4 t = f4(0.f);
            if (e < NG) {
                const int rr = e / (OC / 4), cc = (e % (OC / 4)) * 4;
                const int64_t row = c0 + rr;
                if (row < r1) t = ld4(g + row * out_dim + ob + cc);
            } else if (e < NG + NX) {
                const int e2 = e - NG;
                const int rr = e2 / (IC / 4), cc = (e2 % (IC / 4)) * 4;
                const int64_t row = c0 + rr;
                if (row < r1 && ib + cc < in_dim) t = ld4(x + row * in_dim + ib + cc);
            }
            v[k] = t;
        }
    };
    auto sstore = [&](int b, const float4(&v)[PER]) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int e = threadIdx.x + 256 * k;
            float* d = nullptr;
            if (e < NG) {
                d = &gs[b][(e / (OC / 4)) * GP + (e % (OC / 4)) * 4];
            } else if (e < NG + NX) {
                const int e2 = e - NG;
                d = &xs[b][(e2 / (IC / 4)) * XP + (e2 % (IC / 4)) * 4];
            }
            if (d) {
                d[0] = v[k].x;
                d[1] = v[k].y;
                d[2] = v[k].z;
                d[3] = v[k].w;
            }
        }
    };
    if (nst > 0) {
        gload(0, st[0]);
        if (nst > 1) gload(1, st[1]);
        sstore(0, st[0]);
    }
    if constexpr (DX) {  // W[:, ib : ib + IC]^T (out_dim == OC): wl[col][o], lanes along o
        for (int e = threadIdx.x; e < OC * IC / 4; e += 256) {
            const int o = e % OC, c = (e / OC) * 4;
            const float4 v = ib + c < in_dim ? ld4(W + (int64_t)o * in_dim + ib + c) : f4(0.f);
            wl[(c + 0) * WPT + o] = v.x;
            wl[(c + 1) * WPT + o] = v.y;
            wl[(c + 2) * WPT + o] = v.z;
            wl[(c + 3) * WPT + o] = v.w;
        }
    }
    __syncthreads();
    const bool db_blk = DX && do_db && bi == 0;
    float dbacc = 0.f;
    // one block step on buffer / register slot B (a template constant: st[] stays in
    // registers); step c+1's data (loaded a step ago) goes to the other buffer after
    // this step's MFMAs, step c+2's loads are issued into the slot just freed
    auto step = [&](int64_t c, auto bc) __attribute__((always_inline)) {
        constexpr int B = decltype(bc)::value;
        if (c + 2 < nst) gload(c + 2, st[B]);
        const float* gb = gs[B] + (r * kWgChunk) * GP + wo + j;
        const float* xb = xs[B] + (r * kWgChunk) * XP + j;
        float av[8], bv[8][IG];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            av[u] = gb[(2 * u + h) * GP];
#pragma unroll
            for (int q = 0; q < IG; ++q) bv[u][q] = xb[(2 * u + h) * XP + 32 * q];
        }
        if (!(DX && RSX_LBWD_ABL == 2)) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int q = 0; q < IG; ++q)
                    acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u][q], acc[q], 0, 0, 0);
        }
        // every LDS operand read issued before the first MFMA (one latency per step, not
        // one per MFMA pair)
#if RSX_LBWD_ABL != 3
        __builtin_amdgcn_sched_group_barrier(0x100, 8 + 8 * IG, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 8 * IG, 0);
#endif
        if constexpr (DX && RSX_LBWD_ABL != 1) {
            if (db_blk) {
#pragma unroll
                for (int u = 0; u < 8; ++u) dbacc += av[u];
            }
            // dx[CH x IC] = g_chunk[CH x OC] W_slice[OC x IC]: CH/16 x IC/16 tiles of 16x16,
            // wave w takes tiles w, w + 4, ...; lane (n = lane & 15, q4 = lane >> 4).  Each
            // tile is computed transposed, dx^T = W_slice^T g_chunk^T (A = W^T from the
            // transposed LDS slice, B = g^T from the chunk), so a lane ends with 4 adjacent
            // columns of one row (one float4 store, not 4 dword stores); and the K order is
            // permuted (lane group q4 takes o = q4 OC/4 + k, A and B alike), so a lane's
            // operands are contiguous: OC/8 ds_read_b128 a tile instead of OC/2 ds_read_b32
            constexpr int NT = (CH / 16) * (IC / 16);
            constexpr int K4 = OC / 16;  // float4 operand groups per lane
            const int64_t c0 = r0 + c * CH;
            const int n16 = lane & 15, q4 = lane >> 4;
#pragma unroll 1
            for (int t = wave; t < NT; t += 4) {
                const int mt = t / (IC / 16), nt = t % (IC / 16);
                const float* gb4 = gs[B] + (mt * 16 + n16) * GP + q4 * (OC / 4);
                const float* wa4 = wl + (nt * 16 + n16) * WPT + q4 * (OC / 4);
                typedef float floatx4_t __attribute__((ext_vector_type(4)));
                floatx4_t d0 = {0.f, 0.f, 0.f, 0.f}, d1 = {0.f, 0.f, 0.f, 0.f};
                float4 A4[K4], B4[K4];
#pragma unroll
                for (int k = 0; k < K4; ++k) {
                    A4[k] = *reinterpret_cast<const float4*>(wa4 + 4 * k);
                    B4[k] = *reinterpret_cast<const float4*>(gb4 + 4 * k);
                }
#pragma unroll
                for (int k = 0; k < K4; ++k) {
                    d0 = __builtin_amdgcn_mfma_f32_16x16x4f32(A4[k].x, B4[k].x, d0, 0, 0, 0);
                    d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(A4[k].y, B4[k].y, d1, 0, 0, 0);
                    d0 = __builtin_amdgcn_mfma_f32_16x16x4f32(A4[k].z, B4[k].z, d0, 0, 0, 0);
                    d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(A4[k].w, B4[k].w, d1, 0, 0, 0);
                }
#if RSX_LBWD_ABL != 3
                __builtin_amdgcn_sched_group_barrier(0x100, 2 * K4, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 4 * K4, 0);
#endif
                const floatx4_t d = d0 + d1;
                // lane holds columns 4 q4 .. 4 q4 + 3 of the tile, row n16
                const int64_t row = c0 + mt * 16 + n16;
                const int col = ib + nt * 16 + 4 * q4;
                if (row < r1 && col < in_dim) st4(dx + row * in_dim + col, make_float4(d[0], d[1], d[2], d[3]));
            }
        }
        if (c + 1 < nst) sstore(B ^ 1, st[B ^ 1]);
        __syncthreads();
    };
    for (int64_t c = 0; c < nst; c += 2) {  // block-uniform
        step(c, std::integral_constant<int, 0>{});
        if (c + 1 < nst) step(c + 1, std::integral_constant<int, 1>{});
    }
    // C layout: lane holds column ib + 32q + j, rows ob + wo + (e&3) + 8(e>>2) + 4h
    const int64_t slot_sz = (int64_t)out_dim * in_dim + (DX && do_db ? out_dim : 0);
    float* dst = part + (s * RW + r) * slot_sz;
    if constexpr (DX) {
        if (db_blk) {  // the slot's bias partial: rows 2u + h summed per half, halves added
            dbacc += __shfl_xor(dbacc, 32, 64);
            if (h == 0) dst[(int64_t)out_dim * in_dim + wo + j] = dbacc;
        }
    }
#pragma unroll
    for (int q = 0; q < IG; ++q) {
        if (ib + 32 * q + j >= in_dim) continue;  // the padded columns of a ragged last i tile
#pragma unroll
        for (int e = 0; e < 16; ++e)
            dst[(int64_t)(ob + wo + (e & 3) + 8 * (e >> 2) + 4 * h) * in_dim + ib + 32 * q + j] = acc[q][e];
    }
}

// element e = blockIdx.x*64 + lane; wave w adds slots [w*S/4, (w+1)*S/4) in
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

// as wgrad_reduce with slots `stride` floats apart (the fused backward's slots carry
// the bias partials after the sz weight partials)
__global__ __launch_bounds__(256) void wgrad_reduce_strided(const float* __restrict__ part, int S, int64_t sz,
                                                            int64_t stride, float* __restrict__ out) {
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
            for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(p + u) * stride + e];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += v[u];
        }
        for (; p < en; ++p) acc += part[(int64_t)p * stride + e];
    }
    q[wave][lane] = acc;
    __syncthreads();
    if (wave == 0 && e < sz) out[e] = ((q[0][lane] + q[1][lane]) + q[2][lane]) + q[3][lane];
}

// dW and db of the fused backward in one launch: a slot is sz weight partials followed by
// out_dim bias partials (stride sz + out_dim), so element e < sz + out_dim of every slot
// adds up the same way; e < sz goes to dw, the rest to db (wgrad_reduce_strided's order)
__global__ __launch_bounds__(256) void wgrad_reduce_dwdb(const float* __restrict__ part, int S, int64_t sz,
                                                         int64_t stride, float* __restrict__ dw,
                                                         float* __restrict__ db) {
    __shared__ float q[4][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t e = (int64_t)blockIdx.x * 64 + lane;
    const int b = (int)((int64_t)S * wave / 4), en = (int)((int64_t)S * (wave + 1) / 4);
    float acc = 0.f;
    if (e < stride) {
        int p = b;
        for (; p + 8 <= en; p += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(p + u) * stride + e];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += v[u];
        }
        for (; p < en; ++p) acc += part[(int64_t)p * stride + e];
    }
    q[wave][lane] = acc;
    __syncthreads();
    if (wave == 0 && e < stride) {
        const float v = ((q[0][lane] + q[1][lane]) + q[2][lane]) + q[3][lane];
        if (e < sz) dw[e] = v;
        else db[e - sz] = v;
    }
}

// wgrad_reduce_dwdb of two problems in one launch: blocks [0, nb0) reduce problem 0's slots
struct DwdbProb {
    const float* part;
    int S;
    int64_t sz, stride;
    float* dw;
    float* db;
};

__global__ __launch_bounds__(256) void wgrad_reduce_dwdb_pair(DwdbProb p0, DwdbProb p1, int64_t nb0) {
    __shared__ float q[4][64];
    const bool first = (int64_t)blockIdx.x < nb0;
    const DwdbProb& r = first ? p0 : p1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t e = (first ? (int64_t)blockIdx.x : (int64_t)blockIdx.x - nb0) * 64 + lane;
    const int b = (int)((int64_t)r.S * wave / 4), en = (int)((int64_t)r.S * (wave + 1) / 4);
    float acc = 0.f;
    if (e < r.stride) {
        int p = b;
        for (; p + 8 <= en; p += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = r.part[(int64_t)(p + u) * r.stride + e];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += v[u];
        }
        for (; p < en; ++p) acc += r.part[(int64_t)p * r.stride + e];
    }
    q[wave][lane] = acc;
    __syncthreads();
    if (wave == 0 && e < r.stride) {
        const float v = ((q[0][lane] + q[1][lane]) + q[2][lane]) + q[3][lane];
        if (e < r.sz) r.dw[e] = v;
        else if (r.db) r.db[e - r.sz] = v;
    }
}

}  // namespace rsx

using namespace rsx;

extern "C" size_t rsx_linear_wgrad_ws_bytes(int64_t n, int32_t out_dim, int32_t in_dim) {
    if (n <= 0 || out_dim <= 0 || in_dim <= 0 || (out_dim % 32) || (in_dim % 4)) return 0;
    const WgPlan p = wg_plan(n, out_dim, in_dim);
    return (size_t)p.slots() * (size_t)out_dim * (size_t)in_dim * sizeof(float);
}

// the fused backward stages a W slice too: IC <= 64 keeps two blocks per CU in LDS
// (RSX_LBWD_IG / RSX_LBWD_WAVES: tuning overrides)
static int bwd_ig() {
    static const int v = lin_env("RSX_LBWD_IG", 2);
    return v;
}
static int64_t bwd_waves() {
    static const int v = lin_env("RSX_LBWD_WAVES", kWgTargetWaves);
    return v;
}

extern "C" size_t rsx_linear_bwd_ws_bytes(int64_t n, int32_t out_dim, int32_t in_dim) {
    if (n <= 0 || (out_dim != 32 && out_dim != 64 && out_dim != 128) || in_dim <= 0 || (in_dim % 4)) return 0;
    const WgPlan p = wg_plan(n, out_dim, in_dim, bwd_ig(), bwd_waves());
    return (size_t)p.slots() * ((size_t)out_dim * (size_t)in_dim + (size_t)out_dim) * sizeof(float);
}

// dW = g^T x, dx = g W, db = colsum(g) (db may be NULL) in one pass over the rows;
// out_dim in {32, 64, 128} (one block column of o), in_dim a multiple of 4.
extern "C" int rsx_linear_bwd(const float* g, const float* x, const float* W, int64_t n, int32_t out_dim,
                              int32_t in_dim, float* dw, float* dx, float* db, void* ws, size_t ws_bytes,
                              rsx_stream_t stream) {
    if (n < 0 || out_dim <= 0 || in_dim <= 0 || !dw || !W || (n > 0 && !dx)) return RSX_ERR_ARG;
    if ((out_dim != 32 && out_dim != 64 && out_dim != 128) || (in_dim % 4)) return RSX_ERR_UNSUPPORTED;
    if (n > 0 && (!g || !x)) return RSX_ERR_ARG;
    hipStream_t s = as_stream(stream);
    const int64_t sz = (int64_t)out_dim * in_dim;
    if (n == 0) {
        hipLaunchKernelGGL(wgrad_reduce, dim3((unsigned)((sz + 63) / 64)), dim3(256), 0, s, (const float*)nullptr, 0,
                           sz, dw);
        if (db) hipLaunchKernelGGL(wgrad_reduce, dim3((unsigned)((out_dim + 63) / 64)), dim3(256), 0, s,
                                   (const float*)nullptr, 0, (int64_t)out_dim, db);
        return last_rc();
    }
    if (ws_bytes < rsx_linear_bwd_ws_bytes(n, out_dim, in_dim) || !ws) return RSX_ERR_WORKSPACE;
    const WgPlan p = wg_plan(n, out_dim, in_dim, bwd_ig(), bwd_waves());
    if (p.nob != 1) return RSX_ERR_UNSUPPORTED;
    float* part = static_cast<float*>(ws);
    const dim3 grid((unsigned)(p.nob * p.nib * p.splits));
    const int do_db = db != nullptr;
#define RSX_WGX(IG, OTB)                                                                                        \
    hipLaunchKernelGGL((wgrad_partial<IG, OTB, true>), grid, dim3(256), 0, s, g, x, n, (int)out_dim, (int)in_dim,  \
                       p.rows, p.nob, p.nib, part, W, dx, do_db)
    const int key = p.ig * 8 + p.otb;
    switch (key) {
        case 4 * 8 + 4: RSX_WGX(4, 4); break;
        case 4 * 8 + 2: RSX_WGX(4, 2); break;
        case 4 * 8 + 1: RSX_WGX(4, 1); break;
        case 2 * 8 + 4: RSX_WGX(2, 4); break;
        case 2 * 8 + 2: RSX_WGX(2, 2); break;
        case 2 * 8 + 1: RSX_WGX(2, 1); break;
        case 1 * 8 + 4: RSX_WGX(1, 4); break;
        case 1 * 8 + 2: RSX_WGX(1, 2); break;
        default: RSX_WGX(1, 1); break;
    }
#undef RSX_WGX
    // slots of sz + out_dim floats: dw from the first sz, db from the tails (one launch)
    if (do_db) {
        const int64_t st = sz + out_dim;
        hipLaunchKernelGGL(wgrad_reduce_dwdb, dim3((unsigned)((st + 63) / 64)), dim3(256), 0, s, (const float*)part,
                           p.slots(), sz, st, dw, db);
    } else {
        hipLaunchKernelGGL(wgrad_reduce_strided, dim3((unsigned)((sz + 63) / 64)), dim3(256), 0, s,
                           (const float*)part, p.slots(), sz, sz, dw);
    }
    return last_rc();
}

// the pair's plans: the 2048-wave budget split by input width (the blocks of both problems
// then carry about the same rows x columns each, so they finish together)
static void pair_plans(int64_t n, int32_t out_dim, int32_t in0, int32_t in1, WgPlan& p0, WgPlan& p1) {
    const int64_t w = bwd_waves();
    const int64_t w0 = std::max<int64_t>(4, w * in0 / (in0 + in1)), w1 = std::max<int64_t>(4, w - w0);
    p0 = wg_plan(n, out_dim, in0, bwd_ig(), w0);
    p1 = wg_plan(n, out_dim, in1, bwd_ig(), w1);
}

extern "C" size_t rsx_linear_bwd_pair_ws_bytes(int64_t n, int32_t out_dim, int32_t in0, int32_t in1) {
    if (n <= 0 || (out_dim != 32 && out_dim != 64 && out_dim != 128) || in0 <= 0 || in1 <= 0 || (in0 % 4) || (in1 % 4))
        return 0;
    WgPlan p0, p1;
    pair_plans(n, out_dim, in0, in1, p0, p1);
    const size_t s0 = (size_t)p0.slots() * ((size_t)out_dim * (size_t)in0 + (size_t)out_dim);
    const size_t s1 = (size_t)p1.slots() * ((size_t)out_dim * (size_t)in1 + (size_t)out_dim);
    return (s0 + s1) * sizeof(float) + 256;
}

// rsx_linear_bwd of two Linears over the same n rows and out_dim in one launch pair (SMORE's
// image_trs / text_trs backward, src/models/smore.py:256-259): each problem's results equal
// its own rsx_linear_bwd's with the pair's plan (deterministic).  The image and text problems
// each filled the chip alone; the text one (a few hundred columns) was latency-bound behind
// the image one.  RSX_ERR_UNSUPPORTED when the two plans need different kernel shapes.
extern "C" int rsx_linear_bwd_pair(const float* g0, const float* x0, const float* W0, int32_t in0, float* dw0,
                                   float* dx0, float* db0, const float* g1, const float* x1, const float* W1,
                                   int32_t in1, float* dw1, float* dx1, float* db1, int64_t n, int32_t out_dim,
                                   void* ws, size_t ws_bytes, rsx_stream_t stream) {
    if (n <= 0 || in0 <= 0 || in1 <= 0 || !dw0 || !dw1 || !W0 || !W1 || !dx0 || !dx1 || !g0 || !g1 || !x0 || !x1)
        return RSX_ERR_ARG;
    if ((out_dim != 32 && out_dim != 64 && out_dim != 128) || (in0 % 4) || (in1 % 4)) return RSX_ERR_UNSUPPORTED;
    if (!ws || ws_bytes < rsx_linear_bwd_pair_ws_bytes(n, out_dim, in0, in1)) return RSX_ERR_WORKSPACE;
    WgPlan p0, p1;
    pair_plans(n, out_dim, in0, in1, p0, p1);
    if (p0.nob != 1 || p1.nob != 1 || p0.ig != p1.ig || p0.otb != p1.otb) return RSX_ERR_UNSUPPORTED;
    float* part0 = static_cast<float*>(ws);
    float* part1 = part0 + (size_t)p0.slots() * ((size_t)out_dim * (size_t)in0 + (size_t)out_dim);
    const LbwdProb a{g0, x0, W0, dx0, part0, p0.rows, p0.nib, in0, db0 != nullptr};
    const LbwdProb b{g1, x1, W1, dx1, part1, p1.rows, p1.nib, in1, db1 != nullptr};
    const int64_t nb0 = p0.nib * p0.splits, nb1 = p1.nib * p1.splits;
    hipStream_t s = as_stream(stream);
    const dim3 grid((unsigned)(nb0 + nb1));
#define RSX_WGP(IG, OTB) hipLaunchKernelGGL((wgrad_partial_pair<IG, OTB>), grid, dim3(256), 0, s, a, b, nb0, n, (int)out_dim)
    switch (p0.ig * 8 + p0.otb) {
        case 4 * 8 + 4: RSX_WGP(4, 4); break;
        case 4 * 8 + 2: RSX_WGP(4, 2); break;
        case 4 * 8 + 1: RSX_WGP(4, 1); break;
        case 2 * 8 + 4: RSX_WGP(2, 4); break;
        case 2 * 8 + 2: RSX_WGP(2, 2); break;
        case 2 * 8 + 1: RSX_WGP(2, 1); break;
        case 1 * 8 + 4: RSX_WGP(1, 4); break;
        case 1 * 8 + 2: RSX_WGP(1, 2); break;
        default: RSX_WGP(1, 1); break;
    }
#undef RSX_WGP
    const int64_t sz0 = (int64_t)out_dim * in0, sz1 = (int64_t)out_dim * in1;
    // a slot is the sz weight partials, then (with a bias) the out_dim bias partials
    const int64_t st0 = sz0 + (db0 ? out_dim : 0), st1 = sz1 + (db1 ? out_dim : 0);
    const DwdbProb r0{part0, p0.slots(), sz0, st0, dw0, db0};
    const DwdbProb r1{part1, p1.slots(), sz1, st1, dw1, db1};
    const int64_t rb0 = (st0 + 63) / 64, rb1 = (st1 + 63) / 64;
    hipLaunchKernelGGL(wgrad_reduce_dwdb_pair, dim3((unsigned)(rb0 + rb1)), dim3(256), 0, s, r0, r1, rb0);
    return last_rc();
}

extern "C" int rsx_linear_wgrad(const float* g, const float* x, int64_t n, int32_t out_dim, int32_t in_dim, float* dw,
                                void* ws, size_t ws_bytes, rsx_stream_t stream) {
    if (n < 0 || out_dim <= 0 || in_dim <= 0 || !dw) return RSX_ERR_ARG;
    if ((out_dim % 32) || (in_dim % 4)) return RSX_ERR_UNSUPPORTED;
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
    float* part = static_cast<float*>(ws);
    const dim3 grid((unsigned)(p.nob * p.nib * p.splits));
#define RSX_WG(IG, OTB)                                                                                        \
    hipLaunchKernelGGL((wgrad_partial<IG, OTB>), grid, dim3(256), 0, s, g, x, n, (int)out_dim, (int)in_dim, p.rows, \
                       p.nob, p.nib, part)
    const int key = p.ig * 8 + p.otb;
    switch (key) {
        case 4 * 8 + 4: RSX_WG(4, 4); break;
        case 4 * 8 + 2: RSX_WG(4, 2); break;
        case 4 * 8 + 1: RSX_WG(4, 1); break;
        case 2 * 8 + 4: RSX_WG(2, 4); break;
        case 2 * 8 + 2: RSX_WG(2, 2); break;
        case 2 * 8 + 1: RSX_WG(2, 1); break;
        case 1 * 8 + 4: RSX_WG(1, 4); break;
        case 1 * 8 + 2: RSX_WG(1, 2); break;
        default: RSX_WG(1, 1); break;
    }
#undef RSX_WG
    hipLaunchKernelGGL(wgrad_reduce, dim3((unsigned)((sz + 63) / 64)), dim3(256), 0, s, (const float*)part, p.slots(),
                       sz, dw);
    return last_rc();
}

// spmm.hip — nnz-balanced CSR SpMM with fused row epilogues (gfx950).
//
// Replaces torch.sparse.mm(norm_adj, E) of the reference's propagation loops
// (src/models/lightgcn.py:121-125, src/models/layergcn.py:132-138,
// src/models/smore.py:281-317) and the autograd backward of the same products.
//
// Layout: a row of X/Y is d f32 (d in {32,64,128,256}); a "group" of G = d/4
// lanes owns one output row, lane li holding columns [4li, 4li+4) as a float4, so
// every gathered neighbour row is one coalesced 16 B-per-lane read (a d=64 row is
// 16 lanes x float4 = 256 B; d=256 is one whole wavefront).  Work items carry at
// most `chunk` nonzeros (the schedule built by rsx_csr_schedule_host), so a hub
// row with 10^4..10^6 neighbours is spread over many groups; its partial sums go
// to a slab and a fixup pass adds them in chunk order and applies the epilogue:
// results are deterministic run to run.
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "rsx_adam.hpp"
#include "rsx_common.hpp"

namespace rsx {

// ---------------------------------------------------------------------------
// row epilogues
// ---------------------------------------------------------------------------
// RSX_ADAM_LATE=1 (since round 6): the ADAM epilogue loads p, m, v after the gathers rather
// than before them (102 instead of 115 VGPRs; the C2 ADAM launch 32.4-33.1 against
// 33.3-33.4 us in six alternating runs, profiles/r06/spmm_occ/)
#ifndef RSX_ADAM_LATE
#define RSX_ADAM_LATE 1
#endif
// RSX_FINAL_LATE (A/B): the FINAL epilogue's four stored layers loaded after the gathers
#ifndef RSX_FINAL_LATE
#define RSX_FINAL_LATE 0
#endif

// Row operands of an epilogue, loaded by epi_load right after the work item is
// known so that they are in flight during the neighbour gathers (the ADAM kind
// reads five rows: a whole extra dependent memory trip if loaded after the loop).
struct EpiIn {
    float4 a, b, c, d, e;
    float w;
    float regc;   // ADAM with reg_cnt: the row's regulariser scale (0 off the tagged rows)
    bool tagged;  // row_tag[row] == tag (true when no tag flag needs it)
};

// tag flags in effect (none without a tag array)
__device__ __forceinline__ int tag_flags(const rsx_epilogue& e) { return e.row_tag ? e.tag_flags : 0; }
__device__ __forceinline__ int32_t tag_of(const rsx_epilogue& e) { return e.tag_dev ? *e.tag_dev : e.tag; }

template <int KIND, int D>
__device__ __forceinline__ EpiIn epi_load(const rsx_epilogue& e, int64_t row, int li) {
    const int64_t off = row * D + li * 4;
    EpiIn in;
    in.a = in.b = in.c = in.d = in.e = f4(0.f);
    in.w = 0.f;
    in.regc = 0.f;
    const int tf = tag_flags(e);
    in.tagged = (tf & (RSX_TAG_SPARSE_S | RSX_TAG_SPARSE_R | RSX_TAG_ZERO)) ? e.row_tag[row] == tag_of(e) : true;
    // rows of s_in / r_add known to be zero off the tagged rows are not loaded
    const float* s_in = (!(tf & RSX_TAG_SPARSE_S) || in.tagged) ? e.s_in : nullptr;
    const float* r_add = (!(tf & RSX_TAG_SPARSE_R) || in.tagged) ? e.r_add : nullptr;
    if constexpr (KIND == RSX_EPI_LAYERSUM || KIND == RSX_EPI_AXPBY) {
        if (s_in) in.a = ld4(s_in + off);
    } else if constexpr (KIND == RSX_EPI_FINAL) {
        if (!RSX_FINAL_LATE) {
            if (s_in) in.a = ld4(s_in + off);
            if (r_add) in.b = ld4(r_add + off);
            if (e.aux) in.c = ld4(e.aux + off);
            if (e.e0) in.d = ld4(e.e0 + off);
        }
    } else if constexpr (KIND == RSX_EPI_ADD) {
        if (s_in) in.a = ld4(s_in + off);
        if (r_add) in.b = ld4(r_add + off);
    } else if constexpr (KIND == RSX_EPI_ADAM) {
        if (s_in) in.a = ld4(s_in + off);
        if (r_add) in.b = ld4(r_add + off);
        if (!RSX_ADAM_LATE) {
            in.c = ld4(e.p + off);
            in.d = ld4(e.m + off);
            in.e = ld4(e.v + off);
        }
        if (e.reg_cnt && (!(tf & RSX_TAG_SPARSE_R) || in.tagged)) {
            const int32_t* c = e.reg_cnt + 3 * row;
            in.regc = (float)c[0] * e.reg_k[0] + (float)c[1] * e.reg_k[1] + (float)c[2] * e.reg_k[2];
        }
    } else if constexpr (KIND == RSX_EPI_LAYERGCN) {
        in.a = ld4(e.e0 + off);
        if (e.s_in) in.b = ld4(e.s_in + off);
    } else if constexpr (KIND == RSX_EPI_LAYERGCN_BWD) {
        if (e.r_add) in.a = ld4(e.r_add + off);
        in.b = ld4(e.aux + off);
        in.c = ld4(e.e0 + off);
        if (e.s_in) in.d = ld4(e.s_in + off);
        in.w = e.aux_w[row];
    }
    return in;
}

// Adam's per-launch constants (two f64 pows of the step count): evaluated once per
// thread, not once per row
__device__ __forceinline__ float uniform_f(float x) {  // wave-uniform: lives in an SGPR
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}

template <int KIND>
__device__ __forceinline__ AdamConst adam_for(const rsx_epilogue& e) {
    if constexpr (KIND == RSX_EPI_ADAM) {
        AdamConst c = adam_const(e.adam);
        c.lr = uniform_f(c.lr);
        c.omb1 = uniform_f(c.omb1);
        c.b2 = uniform_f(c.b2);
        c.omb2 = uniform_f(c.omb2);
        c.eps = uniform_f(c.eps);
        c.wd = uniform_f(c.wd);
        c.step_size = uniform_f(c.step_size);
        c.bc2_sqrt = uniform_f(c.bc2_sqrt);
        return c;
    } else {
        return AdamConst{};
    }
}

template <int KIND, int D>
__device__ __forceinline__ void epilogue(const rsx_epilogue& e, int64_t row, float4 acc, int li, const EpiIn& in,
                                         const AdamConst& c) {
    constexpr int G = D / 4;
    const int64_t off = row * D + li * 4;
    acc = mul4(e.alpha, acc);
    if constexpr (KIND == RSX_EPI_STORE) {
        st4(e.y + off, acc);
    } else if constexpr (KIND == RSX_EPI_LAYERSUM) {
        if (e.y) st4(e.y + off, acc);
        const float4 s = e.s_in ? add4(in.a, acc) : acc;
        st4(e.s_out + off, s);
    } else if constexpr (KIND == RSX_EPI_FINAL) {
        // (((s_in + r_add) + aux) + e0) + acc: the stored layers summed in layer order
        float4 a4 = in.a, b4 = in.b, c4 = in.c, d4 = in.d;
        if (RSX_FINAL_LATE) {  // epi_load's operands, loaded here (the same rows, the same tag rules)
            const int tf = tag_flags(e);
            const float* s_in = (!(tf & RSX_TAG_SPARSE_S) || in.tagged) ? e.s_in : nullptr;
            const float* r_add = (!(tf & RSX_TAG_SPARSE_R) || in.tagged) ? e.r_add : nullptr;
            a4 = s_in ? ld4(s_in + off) : f4(0.f);
            b4 = r_add ? ld4(r_add + off) : f4(0.f);
            c4 = e.aux ? ld4(e.aux + off) : f4(0.f);
            d4 = e.e0 ? ld4(e.e0 + off) : f4(0.f);
        }
        float4 t = a4;
        if (e.r_add) t = add4(t, b4);
        if (e.aux) t = add4(t, c4);
        if (e.e0) t = add4(t, d4);
        const float4 s = (e.s_in || e.r_add || e.aux || e.e0) ? add4(t, acc) : acc;
        st4(e.f + off, mul4(e.beta, s));
    } else if constexpr (KIND == RSX_EPI_AXPBY) {
        float4 s = acc;
        if (e.s_in) s = fma4(e.beta, in.a, s);
        st4(e.y + off, s);
    } else if constexpr (KIND == RSX_EPI_ADD) {
        float4 s = acc;
        if (e.s_in) s = add4(s, in.a);
        if (e.reg_cnt) {  // sum over occurrences of k * ego row; loaded here, after the gathers
            // (only the sharded step's last item partial has counts: no registers held across the loop)
            int32_t* c = e.reg_cnt + 3 * row;
            const float regc = (float)c[0] * e.reg_k[0] + (float)c[1] * e.reg_k[1] + (float)c[2] * e.reg_k[2];
            s = add4(s, mul4(regc, ld4(e.p + off)));
            if (li == 0) {
                c[0] = 0;
                c[1] = 0;
                c[2] = 0;
            }
        } else if (e.r_add) {
            s = add4(s, in.b);
        }
        st4(e.y + off, mul4(e.beta, s));
    } else if constexpr (KIND == RSX_EPI_ADAM) {
        float4 p = in.c, m = in.d, v = in.e;
        if (RSX_ADAM_LATE) {  // moments loaded after the gathers (fewer registers live across them)
            p = ld4(e.p + off);
            m = ld4(e.m + off);
            v = ld4(e.v + off);
        }
        float4 g = e.s_in ? add4(in.a, acc) : acc;
        g = mul4(e.beta, g);
        if (e.reg_cnt) g = add4(g, mul4(in.regc, p));  // sum over occurrences of k * ego row
        else if (e.r_add) g = add4(g, in.b);
        g.x = adam_elem(c, p.x, m.x, v.x, g.x);
        g.y = adam_elem(c, p.y, m.y, v.y, g.y);
        g.z = adam_elem(c, p.z, m.z, v.z, g.z);
        g.w = adam_elem(c, p.w, m.w, v.w, g.w);
        if (!(e.halt && *e.halt)) {  // a NaN loss halted training: parameters stay as they are
            st4(e.p + off, p);
            st4(e.m + off, m);
            st4(e.v + off, v);
        }
        if (e.g_out) st4(e.g_out + off, g);
    } else if constexpr (KIND == RSX_EPI_LAYERGCN) {
        // F.cosine_similarity(z, e0, dim=-1, eps=1e-8) = <z/max(|z|,eps), e/max(|e|,eps)>
        const float4 e0 = in.a;
        const float zz = group_sum<G>(dot4(acc, acc));
        const float ee = group_sum<G>(dot4(e0, e0));
        const float ze = group_sum<G>(dot4(acc, e0));
        const float nz = fmaxf(sqrtf(zz), 1e-8f), ne = fmaxf(sqrtf(ee), 1e-8f);
        const float c = ze / (nz * ne);
        const float4 out = mul4(c, acc);
        if (e.aux) st4(e.aux + off, acc);
        if (e.aux_w && li == 0) e.aux_w[row] = c;
        if (e.y) st4(e.y + off, out);
        if (e.s_out) st4(e.s_out + off, e.s_in ? add4(in.b, out) : out);
    } else if constexpr (KIND == RSX_EPI_LAYERGCN_BWD) {
        float4 dE = acc;
        if (e.r_add) dE = add4(dE, in.a);
        const float4 z = in.b;
        const float4 e0 = in.c;
        const float c = in.w;
        const float zz = group_sum<G>(dot4(z, z));
        const float ee = group_sum<G>(dot4(e0, e0));
        const float gz = group_sum<G>(dot4(dE, z));
        const float rz = sqrtf(zz), re = sqrtf(ee);
        const float nz = fmaxf(rz, 1e-8f), ne = fmaxf(re, 1e-8f);
        const float inv = 1.f / (nz * ne);
        // d c / d z = e/(nz ne) - c z/|z|^2 ; d c / d e = z/(nz ne) - c e/|e|^2
        // (the clamped norm is a constant when |x| < eps: no second term then)
        const float kz = rz > 1e-8f ? c / (nz * nz) : 0.f;
        const float ke = re > 1e-8f ? c / (ne * ne) : 0.f;
        float4 dz = mul4(c, dE);
        dz = fma4(gz * inv, e0, dz);
        dz = fma4(-gz * kz, z, dz);
        if (e.y) st4(e.y + off, dz);
        if (e.s_out) {
            float4 de = mul4(gz * inv, z);
            de = fma4(-gz * ke, e0, de);
            st4(e.s_out + off, e.s_in ? add4(in.d, de) : de);
        }
    }
    if (!(tag_flags(e) & RSX_TAG_ZERO) || in.tagged) {
        if (e.zero0) st4(e.zero0 + off, f4(0.f));
        if (e.zero1) st4(e.zero1 + off, f4(0.f));
        if constexpr (KIND == RSX_EPI_ADAM) {
            if (e.reg_cnt && (tag_flags(e) & RSX_TAG_ZERO) && li == 0) {
                int32_t* c = e.reg_cnt + 3 * row;
                c[0] = 0;
                c[1] = 0;
                c[2] = 0;
            }
        }
    }
}

template <int KIND, int D>
__device__ __forceinline__ void epilogue(const rsx_epilogue& e, int64_t row, float4 acc, int li) {
    epilogue<KIND, D>(e, row, acc, li, epi_load<KIND, D>(e, row, li), adam_for<KIND>(e));
}

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
constexpr int kBlock = 256;
constexpr int kUnroll = 8;

// d = 64 helper: broadcast (col, val) entries 8H..8H+7 of the 16-lane row with
// row_newbcast and accumulate their neighbour rows (entries >= n are skipped).
template <int T>
__device__ __forceinline__ int row_bcast(int x) {
    return __builtin_amdgcn_update_dpp(0, x, 0x150 + T, 0xf, 0xf, false);
}
template <int H, int D = 64>
__device__ __forceinline__ float4 gather8(float4 acc, int cm, float vm, int n, const float* xl) {
    const int vi = __float_as_int(vm);
    int c[8];
    float v[8];
    c[0] = row_bcast<8 * H + 0>(cm); v[0] = __int_as_float(row_bcast<8 * H + 0>(vi));
    c[1] = row_bcast<8 * H + 1>(cm); v[1] = __int_as_float(row_bcast<8 * H + 1>(vi));
    c[2] = row_bcast<8 * H + 2>(cm); v[2] = __int_as_float(row_bcast<8 * H + 2>(vi));
    c[3] = row_bcast<8 * H + 3>(cm); v[3] = __int_as_float(row_bcast<8 * H + 3>(vi));
    c[4] = row_bcast<8 * H + 4>(cm); v[4] = __int_as_float(row_bcast<8 * H + 4>(vi));
    c[5] = row_bcast<8 * H + 5>(cm); v[5] = __int_as_float(row_bcast<8 * H + 5>(vi));
    c[6] = row_bcast<8 * H + 6>(cm); v[6] = __int_as_float(row_bcast<8 * H + 6>(vi));
    c[7] = row_bcast<8 * H + 7>(cm); v[7] = __int_as_float(row_bcast<8 * H + 7>(vi));
    float4 xv[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) xv[t] = (8 * H + t < n && c[t] >= 0) ? ld4(xl + (int64_t)c[t] * D) : f4(0.f);
#pragma unroll
    for (int t = 0; t < 8; ++t) acc = fma4(v[t], xv[t], acc);
    return acc;
}

// Fixup of long row `l` by one whole block, at the end of the same launch: thread 0
// waits until all of the row's chunk partials are counted (their blocks come
// earlier in dispatch order, so they are running or done and never wait
// themselves; the poll is bounded so the wave always exits), then the block's
// groups each sum a strided subset of the partials (4 independent accumulators),
// group 0 adds the group sums in a fixed order and applies the epilogue: the
// result does not depend on which chunk finished last.  Thread 0 re-arms the
// counter for the next launch.
template <int D, int KIND>
__device__ __forceinline__ void fixup_block(const rsx_csr& a, const rsx_epilogue& e, float* slab, int64_t l) {
    constexpr int G = D / 4;
    constexpr int GPB = kBlock / G;
    __shared__ float4 part[GPB][G];
    __shared__ int ok;
    const int li = threadIdx.x % G;
    const int gi = threadIdx.x / G;
    const int4 lr = reinterpret_cast<const int4*>(a.long_rows)[l];
    // an untagged row's chunks skipped too (nothing arrives; the counter stays 0)
    if ((tag_flags(e) & RSX_TAG_ROWS) && e.row_tag[lr.x] != tag_of(e)) return;
    EpiIn pre;
    if (gi == 0) pre = epi_load<KIND, D>(e, lr.x, li);
    int* cnt = reinterpret_cast<int*>(slab + a.n_slots * D) + l;
    if (threadIdx.x == 0) {
        int polls = 0;
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < lr.z && polls < (1 << 24)) {
            __builtin_amdgcn_s_sleep(2);
            ++polls;
        }
        ok = polls < (1 << 24);
    }
    __syncthreads();
    const float* base = slab + (int64_t)lr.y * D + li * 4;
    auto ldp = [&](int64_t s) {
        const float* q = base + s * D;
        return make_float4(__hip_atomic_load(q + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __hip_atomic_load(q + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    };
    float4 a0 = f4(0.f), a1 = f4(0.f), a2 = f4(0.f), a3 = f4(0.f);
    int s = gi;
    for (; s + 3 * GPB < lr.z; s += 4 * GPB) {
        a0 = add4(a0, ldp(s));
        a1 = add4(a1, ldp(s + GPB));
        a2 = add4(a2, ldp(s + 2 * GPB));
        a3 = add4(a3, ldp(s + 3 * GPB));
    }
    for (; s < lr.z; s += GPB) a0 = add4(a0, ldp(s));
    part[gi][li] = add4(add4(a0, a1), add4(a2, a3));
    __syncthreads();
    if (gi == 0) {
        float4 acc = part[0][li];
#pragma unroll 4
        for (int g = 1; g < GPB; ++g) acc = add4(acc, part[g][li]);
        if (!ok) acc = f4(__builtin_nanf(""));  // producers never arrived: poison the row
        epilogue<KIND, D>(e, lr.x, acc, li, pre, adam_for<KIND>(e));
    }
    if (threadIdx.x == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int H>
__device__ __forceinline__ void bcast8(int cm, int vi, int* c, float* v) {
    c[0] = row_bcast<8 * H + 0>(cm); v[0] = __int_as_float(row_bcast<8 * H + 0>(vi));
    c[1] = row_bcast<8 * H + 1>(cm); v[1] = __int_as_float(row_bcast<8 * H + 1>(vi));
    c[2] = row_bcast<8 * H + 2>(cm); v[2] = __int_as_float(row_bcast<8 * H + 2>(vi));
    c[3] = row_bcast<8 * H + 3>(cm); v[3] = __int_as_float(row_bcast<8 * H + 3>(vi));
    c[4] = row_bcast<8 * H + 4>(cm); v[4] = __int_as_float(row_bcast<8 * H + 4>(vi));
    c[5] = row_bcast<8 * H + 5>(cm); v[5] = __int_as_float(row_bcast<8 * H + 5>(vi));
    c[6] = row_bcast<8 * H + 6>(cm); v[6] = __int_as_float(row_bcast<8 * H + 6>(vi));
    c[7] = row_bcast<8 * H + 7>(cm); v[7] = __int_as_float(row_bcast<8 * H + 7>(vi));
}

// all 16 entries of the row at once: 16 neighbour loads in flight per lane
__device__ __forceinline__ float4 gather16(float4 acc, int cm, float vm, int n, const float* xl) {
    const int vi = __float_as_int(vm);
    int c[16];
    float v[16];
    bcast8<0>(cm, vi, c, v);
    bcast8<1>(cm, vi, c + 8, v + 8);
    float4 xv[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) xv[t] = (t < n && c[t] >= 0) ? ld4(xl + (int64_t)c[t] * 64) : f4(0.f);
#pragma unroll
    for (int t = 0; t < 16; ++t) acc = fma4(v[t], xv[t], acc);
    return acc;
}

#ifndef RSX_SPMM_G16
#define RSX_SPMM_G16 0
#endif
#ifndef RSX_SPMM_WAVES
#define RSX_SPMM_WAVES 0
#endif
#if RSX_SPMM_WAVES
#define RSX_SPMM_ATTR __attribute__((amdgpu_waves_per_eu(RSX_SPMM_WAVES, RSX_SPMM_WAVES)))
#else
#define RSX_SPMM_ATTR
#endif
// RSX_ADAM_WAVES (tuning): the minimum waves a SIMD for the ADAM kind alone
#ifndef RSX_ADAM_WAVES
#define RSX_ADAM_WAVES 0
#endif

// One group of G lanes per work item {row, slot, begin, end}.
typedef float v4f __attribute__((ext_vector_type(4)));

// 16-B write-through store (the whole 128-B line comes from one instruction of one
// wave, MI355X_MICROARCH.md hand-off table); the caller drains with vmcnt(0).
__device__ __forceinline__ void st4_sc1(float* p, float4 v) {
    const v4f t = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(t) : "memory");
}

#ifndef RSX_SPMM_PF
#define RSX_SPMM_PF 1
#endif
// d >= 128: (col, val) loaded 16 entries per lane-row and DPP-broadcast (0: the
// per-entry wave-uniform loads; a compile-time A/B switch, tools/build_variant.py)
#ifndef RSX_SPMM_WIDE_BCAST
#define RSX_SPMM_WIDE_BCAST 1
#endif

// (col, val) of the next work item's first 16 nonzeros, loaded while the current
// item's first gathers are in flight (d = 64): the next item starts with its
// gathers instead of a dependent (col, val) trip.
struct NextCV {
    int cm;
    float vm;
    bool ok;
};

// One work item {row, slot, begin, end} by a group of G lanes.
template <int D, int KIND>
__device__ __forceinline__ void spmm_item(const rsx_csr& a, const float* __restrict__ x, const rsx_epilogue& e,
                                          float* __restrict__ slab, int4 wk, int li, NextCV& pf, int4 nxt,
                                          bool has_nxt, const AdamConst& ac) {
    const int tf = tag_flags(e);
    const bool have_pf = pf.ok;
    pf.ok = false;
    if (tf & RSX_TAG_ROWS) {  // whole group leaves together (one row per group)
        const int64_t r = wk.y < 0 ? wk.x : reinterpret_cast<const int4*>(a.long_rows)[wk.x].x;
        if (e.row_tag[r] != tag_of(e)) return;
    }
    const bool sparse_x = tf & RSX_TAG_SPARSE_X;
    const int32_t* __restrict__ xtag = e.x_tag ? e.x_tag : e.row_tag;
    EpiIn pre;
    if (wk.y < 0) {
        pre = epi_load<KIND, D>(e, wk.x, li);
    } else {
        pre.a = pre.b = pre.c = pre.d = pre.e = f4(0.f);
        pre.w = 0.f;
        pre.regc = 0.f;
        pre.tagged = true;
    }
    const int32_t* __restrict__ col = a.col;
    const float* __restrict__ val = a.val;
    const float* xl = x + li * 4;
    float4 acc = f4(0.f);
    int j = wk.z;
    const int end = wk.w;
    if constexpr (D == 64) {
        // d = 64: a group is exactly one 16-lane DPP row.  Lane li loads the
        // (col, val) of nonzero j+li (one coalesced load per 16 nonzeros) and
        // row_newbcast:t hands entry t to the whole row in one VALU op, so the
        // memory pipe only sees the neighbour-row gathers.
        for (; j < end; j += 16) {
            const bool mine = j + li < end;
            int cm;
            float vm;
            if (RSX_SPMM_PF && j == wk.z && have_pf) {
                cm = mine ? pf.cm : 0;
                vm = mine ? pf.vm : 0.f;
            } else {
                cm = mine ? col[j + li] : 0;
                vm = mine ? val[j + li] : 0.f;
            }
            if (sparse_x && mine && xtag[cm] != tag_of(e)) cm = -1;  // zero X row: no gather
            const int n = end - j;
#if RSX_SPMM_G16
            acc = gather16(acc, cm, vm, n, xl);
#else
#if RSX_SPMM_PF
            if (j == wk.z && has_nxt) {
                // issue this chunk's first 8 gathers, then the next item's (col, val), then add
                const int vi = __float_as_int(vm);
                int c[8];
                float v[8];
                bcast8<0>(cm, vi, c, v);
                float4 xv[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) xv[t] = (t < n && c[t] >= 0) ? ld4(xl + (int64_t)c[t] * 64) : f4(0.f);
                const bool nm = nxt.z + li < nxt.w;
                pf.cm = nm ? col[nxt.z + li] : 0;
                pf.vm = nm ? val[nxt.z + li] : 0.f;
                pf.ok = true;
#pragma unroll
                for (int t = 0; t < 8; ++t) acc = fma4(v[t], xv[t], acc);
            } else {
                acc = gather8<0>(acc, cm, vm, n, xl);
            }
#else
            acc = gather8<0>(acc, cm, vm, n, xl);
#endif
            if (n > 8) acc = gather8<1>(acc, cm, vm, n, xl);
#endif
        }
    } else if constexpr (RSX_SPMM_WIDE_BCAST && D >= 128) {
        // d = 128 / 256: a group spans 2 / 4 DPP rows.  Lane li loads entry j + (li & 15):
        // the rows of a group load the same 16 (col, val) entries (one coalesced request
        // each), and row_newbcast:t hands entry t to every lane of its row -- two vector
        // loads per 16 nonzeros instead of two wave-uniform loads per nonzero, so the
        // memory pipe carries the neighbour-row gathers only.  Same fma chain in nonzero
        // order as the per-entry loop below: bit-identical results.
        const int q = li & 15;
        for (; j < end; j += 16) {
            const bool mine = j + q < end;
            int cm = mine ? col[j + q] : 0;
            const float vm = mine ? val[j + q] : 0.f;
            if (sparse_x && mine && xtag[cm] != tag_of(e)) cm = -1;  // zero X row: no gather
            const int n = end - j;
            acc = gather8<0, D>(acc, cm, vm, n, xl);
            if (n > 8) acc = gather8<1, D>(acc, cm, vm, n, xl);
        }
    } else {
        for (; j + kUnroll <= end; j += kUnroll) {
            int c[kUnroll];
            float v[kUnroll];
#pragma unroll
            for (int t = 0; t < kUnroll; ++t) {
                c[t] = col[j + t];
                v[t] = val[j + t];
            }
            if (sparse_x) {
#pragma unroll
                for (int t = 0; t < kUnroll; ++t)
                    if (xtag[c[t]] != tag_of(e)) c[t] = -1;
            }
            float4 xv[kUnroll];
#pragma unroll
            for (int t = 0; t < kUnroll; ++t) xv[t] = c[t] >= 0 ? ld4(xl + (int64_t)c[t] * D) : f4(0.f);
#pragma unroll
            for (int t = 0; t < kUnroll; ++t) acc = fma4(v[t], xv[t], acc);
        }
        if (j < end) {
            int c[kUnroll];
            float v[kUnroll];
#pragma unroll
            for (int t = 0; t < kUnroll; ++t) {
                const bool ok = j + t < end;
                c[t] = ok ? col[j + t] : 0;
                v[t] = ok ? val[j + t] : 0.f;
                if (sparse_x && ok && xtag[c[t]] != tag_of(e)) c[t] = -1;
            }
            float4 xv[kUnroll];
#pragma unroll
            for (int t = 0; t < kUnroll; ++t) xv[t] = (j + t < end && c[t] >= 0) ? ld4(xl + (int64_t)c[t] * D) : f4(0.f);
#pragma unroll
            for (int t = 0; t < kUnroll; ++t)
                if (j + t < end) acc = fma4(v[t], xv[t], acc);
        }
    }
    if (wk.y < 0) {
        epilogue<KIND, D>(e, wk.x, acc, li, pre, ac);
    } else {
        // partial of long row wk.x: written through the (per-XCD, non-coherent) L2,
        // drained (vmcnt(0)), then counted by one lane of the group; the row's fixup
        // block polls the count with sc1 loads and reads the partials with sc1 loads
        st4_sc1(slab + (int64_t)wk.y * D + li * 4, acc);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (li == 0) {
            int* cnt = reinterpret_cast<int*>(slab + a.n_slots * D) + wk.x;
            __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <int D, int KIND>
__device__ __forceinline__ void spmm_main_body(const rsx_csr& a, const float* __restrict__ x, const rsx_epilogue& e,
                                               float* __restrict__ slab, int64_t n_main, int64_t bid);

// Work blocks [0, n_main): each group walks work items w, w + n_main*GPB, ...
// (the next descriptor is loaded before the current item is processed); blocks
// [n_main, n_main + n_long) are the long rows' fixups (fix_only: every block is one).
template <int D, int KIND>
__global__ RSX_SPMM_ATTR __launch_bounds__(kBlock)
__attribute__((amdgpu_waves_per_eu(KIND == RSX_EPI_ADAM && RSX_ADAM_WAVES ? RSX_ADAM_WAVES : 1))) void spmm_main(rsx_csr a, const float* __restrict__ x,
                                                                  rsx_epilogue e, float* __restrict__ slab,
                                                                  int64_t n_main, int fix_only, TagJob tj) {
    constexpr int G = D / 4;
    constexpr int GPB = kBlock / G;
    const int li = threadIdx.x % G;
    if (tj.batch > 0) {  // the last blocks tag the batch rows (nothing in this launch reads row_tag)
        const int64_t n_tag = (3 * tj.batch + kBlock - 1) / kBlock;
        const int64_t tb = (int64_t)blockIdx.x - ((int64_t)gridDim.x - n_tag);
        if (tb >= 0) {
            const int64_t t = tb * kBlock + threadIdx.x;
            if (t < 3 * tj.batch) {
                const int64_t id = tj.trip[t];
                tj.row_tag[t < tj.batch ? id : tj.n_users + id] = tj.tag_dev ? *tj.tag_dev : tj.tag;
            }
            return;
        }
    }
    if (fix_only) {
        fixup_block<D, KIND>(a, e, slab, (int64_t)blockIdx.x);
        return;
    }
    if ((int64_t)blockIdx.x >= n_main) {
        fixup_block<D, KIND>(a, e, slab, (int64_t)blockIdx.x - n_main);
        return;
    }
    spmm_main_body<D, KIND>(a, x, e, slab, n_main, (int64_t)blockIdx.x);
}

// Up to kBatchMax independent products of one epilogue kind and width in ONE launch
// (SMORE's three item views through their kNN graphs, or through R): every
// problem's work blocks first, then every problem's hub-row fixup blocks, so no
// fixup can be dispatched ahead of the partials it waits for.
constexpr int kBatchMax = 4;
struct SpmmBatch {
    rsx_csr a[kBatchMax];
    const float* x[kBatchMax];
    rsx_epilogue e[kBatchMax];
    float* slab[kBatchMax];
    int64_t n_main[kBatchMax];
    int64_t main_off[kBatchMax + 1];
    int64_t fix_off[kBatchMax + 1];
    int32_t count;
};

template <int D, int KIND>
__global__ __launch_bounds__(kBlock) void spmm_batch(SpmmBatch b, int fix_only) {
    int64_t bid = blockIdx.x;
    const int64_t nm = fix_only ? 0 : b.main_off[b.count];
    int p = 0;
    if (bid < nm) {
        while (p + 1 < b.count && bid >= b.main_off[p + 1]) ++p;
        spmm_main_body<D, KIND>(b.a[p], b.x[p], b.e[p], b.slab[p], b.n_main[p], bid - b.main_off[p]);
        return;
    }
    bid -= nm;
    while (p + 1 < b.count && bid >= b.fix_off[p + 1]) ++p;
    fixup_block<D, KIND>(b.a[p], b.e[p], b.slab[p], bid - b.fix_off[p]);
}

// The work blocks of spmm_main: block `bid` of n_main walks work items w, w + n_main*GPB, ...
template <int D, int KIND>
__device__ __forceinline__ void spmm_main_body(const rsx_csr& a, const float* __restrict__ x, const rsx_epilogue& e,
                                               float* __restrict__ slab, int64_t n_main, int64_t bid) {
    constexpr int G = D / 4;
    constexpr int GPB = kBlock / G;
    const int li = threadIdx.x % G;
    const int64_t stride = n_main * GPB;
    int64_t w = bid * GPB + threadIdx.x / G;
    if (w >= a.n_work) return;  // whole groups leave together
    const int4* work = reinterpret_cast<const int4*>(a.work);
    int4 wk = work[w];
    NextCV pf = {0, 0.f, false};
    const AdamConst ac = adam_for<KIND>(e);
    for (;;) {
        const int64_t wn = w + stride;
        const int4 nxt = wn < a.n_work ? work[wn] : make_int4(0, 0, 0, 0);
        spmm_item<D, KIND>(a, x, e, slab, wk, li, pf, nxt, wn < a.n_work, ac);
        if (wn >= a.n_work) break;
        w = wn;
        wk = nxt;
    }
}

// The schedule of a CSR whose rows are a subset of a template's nonzeros (every row's
// degree <= the template's: an edge-dropout graph of the template) in the template's
// work layout: whole rows keep their item, a long row keeps its chunk items and its
// fixup (the chunks past the row's new end become empty items: zero partials).
__global__ __launch_bounds__(256) void schedule_rebind_kernel(rsx_csr t, const int64_t* __restrict__ rp,
                                                              int32_t* __restrict__ work) {
    const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (w >= t.n_work) return;
    const int4 wk = reinterpret_cast<const int4*>(t.work)[w];
    int4 out;
    if (wk.y < 0) {
        out = make_int4(wk.x, -1, (int)rp[wk.x], (int)rp[wk.x + 1]);
    } else {
        const int4 lr = reinterpret_cast<const int4*>(t.long_rows)[wk.x];
        const int64_t e = rp[lr.x + 1];
        int64_t b = rp[lr.x] + (int64_t)(wk.y - lr.y) * t.chunk;
        if (b > e) b = e;
        out = make_int4(wk.x, wk.y, (int)b, (int)(b + t.chunk < e ? b + t.chunk : e));
    }
    reinterpret_cast<int4*>(work)[w] = out;
}

// acc = 0 for every row (stand-alone Adam, K = 0 forward, first LayerGCN backward step).
template <int D, int KIND>
__global__ __launch_bounds__(kBlock) void rowwise_kernel(int64_t n_rows, rsx_epilogue e) {
    constexpr int G = D / 4;
    constexpr int GPB = kBlock / G;
    const int li = threadIdx.x % G;
    const int64_t row = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
    if (row >= n_rows) return;
    if ((tag_flags(e) & RSX_TAG_ROWS) && e.row_tag[row] != tag_of(e)) return;
    epilogue<KIND, D>(e, row, f4(0.f), li);
}

// Work blocks per launch (n = the blocks the work list would need): enough to fill
// the chip once, later items walked by the same groups.  A d = 64 list needing more
// than one 2,048-block round gets 1,536 longer-lived blocks (C2 step 133.6-135.0 us
// against 135.8-137.8 at 2,048 and 152 at 1,024; its ADAM layer 33.5 vs 35.2-35.9
// us), while a list that fits one round launches whole (baby: 111 us/step whole,
// 115 capped at 1,536; tools/gpu/maxb_sweep.sh, ab_legs.sh).  RSX_SPMM_MAXB
// overrides (tuning), RSX_SPMM_MAXB_ADAM for the Adam-epilogue kind alone.
static int64_t env_blocks(const char* name) { return env_knob(name, 0, 1, 1 << 20); }
static int64_t spmm_max_blocks(int kind, int d, int64_t n) {
    static const int64_t all = env_blocks("RSX_SPMM_MAXB");
    static const int64_t adam = env_blocks("RSX_SPMM_MAXB_ADAM");
    if (kind == RSX_EPI_ADAM && adam > 0) return adam;
    if (all > 0) return all;
    return d <= 64 && n > 2048 ? 1536 : 2048;
}

// Fixup blocks ride in the same launch only while they cannot fill the chip (so
// the partials' blocks always find room whatever the dispatch order); beyond that
// they get a launch of their own.
constexpr int64_t kInlineFixups = 1024;

template <int D, int KIND>
static int launch_spmm(const rsx_csr& a, const float* x, const rsx_epilogue& e, float* slab,
                       hipStream_t s, const TagJob& tj) {
    constexpr int GPB = kBlock / (D / 4);
    int64_t n_main = (a.n_work + GPB - 1) / GPB;
    n_main = std::min(n_main, spmm_max_blocks(KIND, D, n_main));
    const bool inl = a.n_long <= kInlineFixups;
    const int64_t n_tag = tj.batch > 0 ? (3 * tj.batch + kBlock - 1) / kBlock : 0;
    const int64_t nb = n_main + (inl ? a.n_long : 0) + n_tag;
    if (nb > 0)
        hipLaunchKernelGGL((spmm_main<D, KIND>), dim3((unsigned)nb), dim3(kBlock), 0, s, a, x, e, slab, n_main, 0,
                           tj);
    if (!inl)
        hipLaunchKernelGGL((spmm_main<D, KIND>), dim3((unsigned)a.n_long), dim3(kBlock), 0, s, a, x, e, slab,
                           n_main, 1, TagJob{});
    return last_rc();
}

template <int D, int KIND>
static int launch_batch(SpmmBatch& b, hipStream_t s) {
    constexpr int GPB = kBlock / (D / 4);
    int64_t nm = 0, nf = 0;
    for (int p = 0; p < b.count; ++p) {
        int64_t n_main = (b.a[p].n_work + GPB - 1) / GPB;
        n_main = std::min(n_main, spmm_max_blocks(KIND, D, n_main));
        b.n_main[p] = n_main;
        b.main_off[p] = nm;
        b.fix_off[p] = nf;
        nm += n_main;
        nf += b.a[p].n_long;
    }
    b.main_off[b.count] = nm;
    b.fix_off[b.count] = nf;
    if (nf > kInlineFixups) {  // too many fixup blocks to ride along: every product's fixups in a second launch
        if (nm > 0) {
            const int64_t f = b.fix_off[b.count];
            b.fix_off[b.count] = 0;  // (the first launch has no fixup blocks: nm blocks only)
            hipLaunchKernelGGL((spmm_batch<D, KIND>), dim3((unsigned)nm), dim3(kBlock), 0, s, b, 0);
            b.fix_off[b.count] = f;
        }
        hipLaunchKernelGGL((spmm_batch<D, KIND>), dim3((unsigned)nf), dim3(kBlock), 0, s, b, 1);
        return last_rc();
    }
    if (nm + nf > 0) hipLaunchKernelGGL((spmm_batch<D, KIND>), dim3((unsigned)(nm + nf)), dim3(kBlock), 0, s, b, 0);
    return last_rc();
}

template <int D>
static int batch_d(SpmmBatch& b, int kind, hipStream_t s) {
    switch (kind) {
        case RSX_EPI_STORE: return launch_batch<D, RSX_EPI_STORE>(b, s);
        case RSX_EPI_ADD: return launch_batch<D, RSX_EPI_ADD>(b, s);
        case RSX_EPI_AXPBY: return launch_batch<D, RSX_EPI_AXPBY>(b, s);
        default: return RSX_ERR_UNSUPPORTED;
    }
}

template <int D, int KIND>
static int launch_rowwise(int64_t n, const rsx_epilogue& e, hipStream_t s) {
    constexpr int GPB = kBlock / (D / 4);
    if (n <= 0) return 0;
    hipLaunchKernelGGL((rowwise_kernel<D, KIND>), dim3((unsigned)((n + GPB - 1) / GPB)), dim3(kBlock), 0,
                       s, n, e);
    return last_rc();
}

template <int D>
static int spmm_d(const rsx_csr& a, const float* x, const rsx_epilogue& e, float* slab, hipStream_t s,
                  const TagJob& tj) {
    switch (e.kind) {
        case RSX_EPI_STORE: return launch_spmm<D, RSX_EPI_STORE>(a, x, e, slab, s, tj);
        case RSX_EPI_LAYERSUM: return launch_spmm<D, RSX_EPI_LAYERSUM>(a, x, e, slab, s, tj);
        case RSX_EPI_FINAL: return launch_spmm<D, RSX_EPI_FINAL>(a, x, e, slab, s, tj);
        case RSX_EPI_ADAM: return launch_spmm<D, RSX_EPI_ADAM>(a, x, e, slab, s, tj);
        case RSX_EPI_LAYERGCN: return launch_spmm<D, RSX_EPI_LAYERGCN>(a, x, e, slab, s, tj);
        case RSX_EPI_AXPBY: return launch_spmm<D, RSX_EPI_AXPBY>(a, x, e, slab, s, tj);
        case RSX_EPI_LAYERGCN_BWD: return launch_spmm<D, RSX_EPI_LAYERGCN_BWD>(a, x, e, slab, s, tj);
        case RSX_EPI_ADD: return launch_spmm<D, RSX_EPI_ADD>(a, x, e, slab, s, tj);
        default: return RSX_ERR_ARG;
    }
}

template <int D>
static int rowwise_d(int64_t n, const rsx_epilogue& e, hipStream_t s) {
    switch (e.kind) {
        case RSX_EPI_STORE: return launch_rowwise<D, RSX_EPI_STORE>(n, e, s);
        case RSX_EPI_LAYERSUM: return launch_rowwise<D, RSX_EPI_LAYERSUM>(n, e, s);
        case RSX_EPI_FINAL: return launch_rowwise<D, RSX_EPI_FINAL>(n, e, s);
        case RSX_EPI_ADAM: return launch_rowwise<D, RSX_EPI_ADAM>(n, e, s);
        case RSX_EPI_LAYERGCN: return launch_rowwise<D, RSX_EPI_LAYERGCN>(n, e, s);
        case RSX_EPI_AXPBY: return launch_rowwise<D, RSX_EPI_AXPBY>(n, e, s);
        case RSX_EPI_LAYERGCN_BWD: return launch_rowwise<D, RSX_EPI_LAYERGCN_BWD>(n, e, s);
        case RSX_EPI_ADD: return launch_rowwise<D, RSX_EPI_ADD>(n, e, s);
        default: return RSX_ERR_ARG;
    }
}

// `tj`: the launch also tags the batch rows (internal: the step's first forward layer)
int spmm_dispatch_tagging(const rsx_csr& a, const float* x, int d, const rsx_epilogue& e, float* slab,
                          hipStream_t s, const TagJob& tj) {
    if (a.n_long > 0 && !slab) return RSX_ERR_WORKSPACE;
    if (tj.batch > 0 && (!tj.trip || !tj.row_tag)) return RSX_ERR_ARG;
    switch (d) {
        case 32: return spmm_d<32>(a, x, e, slab, s, tj);
        case 64: return spmm_d<64>(a, x, e, slab, s, tj);
        case 128: return spmm_d<128>(a, x, e, slab, s, tj);
        case 256: return spmm_d<256>(a, x, e, slab, s, tj);
        default: return RSX_ERR_UNSUPPORTED;
    }
}

int spmm_dispatch(const rsx_csr& a, const float* x, int d, const rsx_epilogue& e, float* slab,
                  hipStream_t s) {
    return spmm_dispatch_tagging(a, x, d, e, slab, s, TagJob{});
}

int rowwise_dispatch(int64_t n, int d, const rsx_epilogue& e, hipStream_t s) {
    switch (d) {
        case 32: return rowwise_d<32>(n, e, s);
        case 64: return rowwise_d<64>(n, e, s);
        case 128: return rowwise_d<128>(n, e, s);
        case 256: return rowwise_d<256>(n, e, s);
        default: return RSX_ERR_UNSUPPORTED;
    }
}

}  // namespace rsx

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char* rsx_version(void) { return "rsx 0.1.0 gfx950"; }

int rsx_csr_schedule_host(const int64_t* rowptr_host, int64_t n_rows, int32_t chunk, int32_t* work_host,
                          int32_t* long_host, int64_t* n_work, int64_t* n_long, int64_t* n_slots) {
    if (!rowptr_host || n_rows < 0 || chunk <= 0 || !n_work || !n_long || !n_slots) return RSX_ERR_ARG;
    if (rowptr_host[n_rows] >= (int64_t(1) << 31)) return RSX_ERR_ARG;
    int64_t nw = 0, nl = 0, ns = 0;
    // pass 1: the chunks of long rows (slab items) come first, so that every block
    // producing a partial is dispatched before the fixup blocks that consume it
    for (int64_t r = 0; r < n_rows; ++r) {
        const int64_t b = rowptr_host[r], e = rowptr_host[r + 1];
        const int64_t deg = e - b;
        if (deg <= chunk) continue;
        const int64_t nc = (deg + chunk - 1) / chunk;
        if (long_host) {
            int32_t* l = long_host + 4 * nl;
            l[0] = (int32_t)r; l[1] = (int32_t)ns; l[2] = (int32_t)nc; l[3] = 0;
        }
        for (int64_t c = 0; c < nc; ++c) {
            if (work_host) {
                int32_t* w = work_host + 4 * nw;
                const int64_t cb = b + c * chunk;
                const int64_t ce = cb + chunk < e ? cb + chunk : e;
                w[0] = (int32_t)nl; w[1] = (int32_t)(ns + c); w[2] = (int32_t)cb; w[3] = (int32_t)ce;
            }
            ++nw;
        }
        ns += nc;
        ++nl;
    }
    // pass 2: whole rows
    for (int64_t r = 0; r < n_rows; ++r) {
        const int64_t b = rowptr_host[r], e = rowptr_host[r + 1];
        if (e - b > chunk) continue;
        if (work_host) {
            int32_t* w = work_host + 4 * nw;
            w[0] = (int32_t)r; w[1] = -1; w[2] = (int32_t)b; w[3] = (int32_t)e;
        }
        ++nw;
    }
    *n_work = nw;
    *n_long = nl;
    *n_slots = ns;
    return RSX_OK;
}

int rsx_csr_schedule_rebind(const rsx_csr* tmpl, const int64_t* rowptr, int32_t* work, rsx_stream_t stream) {
    if (!tmpl || !rowptr || !work || !tmpl->work || (tmpl->n_long > 0 && !tmpl->long_rows)) return RSX_ERR_ARG;
    if (tmpl->n_work == 0) return RSX_OK;
    hipLaunchKernelGGL(rsx::schedule_rebind_kernel, dim3((unsigned)((tmpl->n_work + 255) / 256)), dim3(256), 0,
                       rsx::as_stream(stream), *tmpl, rowptr, work);
    return rsx::last_rc();
}

int rsx_spmm(const rsx_csr* a, const float* x, int32_t d, const rsx_epilogue* epi, float* slab,
             rsx_stream_t stream) {
    if (!a || !x || !epi) return RSX_ERR_ARG;
    return rsx::spmm_dispatch(*a, x, d, *epi, slab, rsx::as_stream(stream));
}

int rsx_spmm_batch(int32_t count, const rsx_csr* const* a, const float* const* x, int32_t d, const rsx_epilogue* epis,
                   float* const* slabs, rsx_stream_t stream) {
    using namespace rsx;
    if (count < 0 || count > kBatchMax || (count > 0 && (!a || !x || !epis || !slabs))) return RSX_ERR_ARG;
    if (count == 0) return RSX_OK;
    SpmmBatch b{};
    b.count = count;
    const int kind = epis[0].kind;
    for (int p = 0; p < count; ++p) {
        if (!a[p] || !x[p] || epis[p].kind != kind) return RSX_ERR_ARG;
        if (a[p]->n_long > 0 && !slabs[p]) return RSX_ERR_WORKSPACE;
        b.a[p] = *a[p];
        b.x[p] = x[p];
        b.e[p] = epis[p];
        b.slab[p] = slabs[p];
    }
    hipStream_t s = as_stream(stream);
    switch (d) {
        case 32: return batch_d<32>(b, kind, s);
        case 64: return batch_d<64>(b, kind, s);
        case 128: return batch_d<128>(b, kind, s);
        case 256: return batch_d<256>(b, kind, s);
        default: return RSX_ERR_UNSUPPORTED;
    }
}

int rsx_rowwise(int64_t n_rows, int32_t d, const rsx_epilogue* epi, rsx_stream_t stream) {
    if (!epi || n_rows < 0) return RSX_ERR_ARG;
    return rsx::rowwise_dispatch(n_rows, d, *epi, rsx::as_stream(stream));
}

}  // extern "C"

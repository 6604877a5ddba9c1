// fullsort.hip — full-sort user x item scoring fused with train-item masking and top-K (gfx950).
//
// Replaces, per evaluation batch (reference src/common/trainer.py:509-528):
//     scores = u_emb[users] @ item_emb.T          (src/models/lightgcn.py:164, layergcn.py:186,
//                                                  smore.py:420)
//     scores[mask[0], mask[1]] = -1e10             (trainer.py:524)
//     _, topk = torch.topk(scores, k, dim=-1)      (trainer.py:526)
// without materialising the [B_u, n_items] score matrix.
//
// Kernel 1 (fs_tiles): grid = (blocks of 32 users) x (item chunks), one wavefront
// per block, no LDS candidate buffers and no barriers, so two waves share every
// SIMD (d <= 64) and the hardware overlaps one wave's selection work with the
// other's MFMA chain.  A 32x32 score tile is D/2 v_mfma_f32_32x32x2_f32 — exact f32
// fma chains, A = item rows (straight from L2 into double-buffered registers),
// B = user rows (registers), reduction index permuted so lane-half h reads the
// contiguous half of its row.  Lanes j and j+32 hold the tile's 32 scores of user
// j.  Scores above the user's running threshold are appended, as 64-bit keys
// (ordered score bits << 32 | ~item: one u64 order = score desc, index asc), to the
// user's candidate row in the workspace (L2-resident); a lane walks only its set
// bits, reading its scores back from a small LDS scratch.  When a row may overflow,
// the wave radix-selects its k-th key with ballots, compacts the row to the top k
// and raises the threshold.  Items arrive in ascending index order within a chunk,
// so the strict "> threshold" filter drops nothing the canonical order would keep.
// Kernel 2 (fs_select): one wavefront per user takes the exact top-K over every
// chunk's list (each already cut to its top k) and rank-sorts it.
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "rsx_common.hpp"

// Profiling ablations (RSX_FS_MODE 1, 4, 5, 6, 8, 9: scores only, pass 1 only, no exact dots,
// no candidates, candidate counters in out_idx ...) return wrong top-k lists by design: they
// exist only in an ablation build (tools/build_variant.py fs_abl -DRSX_FS_ABLATION=1).  The
// product library compiles every FS_ABL(x) to false, and refuses a set RSX_FS_MODE.
#ifndef RSX_FS_ABLATION
#define RSX_FS_ABLATION 0
#endif
#define FS_ABL(x) (RSX_FS_ABLATION && a.mode == (x))

namespace rsx {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef unsigned long long u64;

#ifndef RSX_FS_CAP
#define RSX_FS_CAP 256
#endif
constexpr int kCap = RSX_FS_CAP;  // candidate slots per (user, chunk) row; compaction when > kCap - 32
constexpr int kNK = kCap / 64;  // candidate keys per lane while compacting
constexpr int kMaxK = 96;     // k limit: a chunk's final list (<= k) is <= 2 keys per lane in fs_select

__device__ __forceinline__ unsigned ord_f32(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_f32(unsigned o) {
    const unsigned u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
    return __uint_as_float(u);
}
__device__ __forceinline__ u64 make_key(float s, int idx) {
    return ((u64)ord_f32(s) << 32) | (u64)(0xffffffffu - (unsigned)idx);
}
__device__ __forceinline__ float key_score(u64 k) { return unord_f32((unsigned)(k >> 32)); }
__device__ __forceinline__ int key_index(u64 k) { return (int)(0xffffffffu - (unsigned)(k & 0xffffffffu)); }

__device__ __forceinline__ u64 shfl_xor_u64(u64 v, int m) {
    const unsigned lo = __shfl_xor((unsigned)(v & 0xffffffffu), m, kWave);
    const unsigned hi = __shfl_xor((unsigned)(v >> 32), m, kWave);
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 shfl_u64(u64 v, int src) {
    const unsigned lo = __shfl((unsigned)(v & 0xffffffffu), src, kWave);
    const unsigned hi = __shfl((unsigned)(v >> 32), src, kWave);
    return ((u64)hi << 32) | lo;
}

// Descending bitonic sort of 128 keys held by one wavefront: element e = lane + 64*q.
__device__ __forceinline__ void bitonic128_desc(u64& e0, u64& e1, int lane) {
#pragma unroll
    for (int size = 2; size <= 128; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride == 64) {
                const u64 mx = e0 > e1 ? e0 : e1;
                const u64 mn = e0 > e1 ? e1 : e0;
                e0 = mx;
                e1 = mn;
            } else {
                const bool lower = (lane & stride) == 0;
                {
                    const u64 pv = shfl_xor_u64(e0, stride);
                    const bool desc = ((lane & size) == 0);
                    const bool keep_max = (lower == desc);
                    e0 = keep_max ? (e0 > pv ? e0 : pv) : (e0 > pv ? pv : e0);
                }
                {
                    const u64 pv = shfl_xor_u64(e1, stride);
                    const bool desc = (((lane + 64) & size) == 0);
                    const bool keep_max = (lower == desc);
                    e1 = keep_max ? (e1 > pv ? e1 : pv) : (e1 > pv ? pv : e1);
                }
            }
        }
    }
}

struct FsArgs {
    const float* U;
    const int64_t* users;
    int64_t nb;
    const float* I;
    int64_t ni;
    const int64_t* mrp;
    const int32_t* mcol;
    int k;
    int n_chunks;
    int64_t chunk_items;
    u64* cand;    // [nb][n_chunks][kCap] raw candidate keys
    int* ccount;  // [nb][n_chunks]
    float* out_val;
    int64_t* out_idx;
    int mode;  // profiling ablation (RSX_FS_MODE, ablation builds only, see FS_ABL): 0 = the product
    const __bf16* Ib;  // fs_screen: bf16 item rows + norm block (kScreenRow), padded to whole 32-item tiles
    int n_lists;       // candidate lists per user: n_chunks (fs_tiles), n_chunks * seg_slots (fs_screen)
    int seg_slots;     // fs_screen: segments per (user block, chunk) (1: unsegmented)
    int64_t seg_waves; // fs_screen: waves per chunk of the balanced split (0: one per user block)
    unsigned* lbound;  // fs_screen two-phase: [nb] the user's L as an ordered word (fs_thresh)
    uint16_t* samp;    // two-phase pass 1: [nb][n_lists][96] the segments' samples (ordered words' high halves)
    uint16_t* mcnt1;   // two-phase pass 1: [nb][n_lists] masked items sampled by value (0xffff: no segment)
};


__device__ __forceinline__ int popc64(u64 x) { return __popcll(x); }
__device__ __forceinline__ u64 lanemask_lt(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

__device__ __forceinline__ u64 ld_u64_l2(const u64* p) {  // bypasses the CU's L1 (L2-served)
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


// Shrink one user's buffer (k < n <= kCap unique nonzero keys, in global memory) to
// exactly its top k, compacted to the front, and return the k-th key's score (the
// new threshold).  The wave loads the buffer coalesced (two keys per lane; empty
// slots read as 0, which no valid key is) and finds the k-th largest key by a
// bitwise radix search with ballots: 32 rounds on the ordered-score word (one VALU
// compare per key pair and scalar counting per round), and 32 more on the index
// word only when several keys share the boundary score.  Every round is a handful
// of instructions, so the selection costs a fraction of an all-pairs rank count.
// slack >= 0 (running compactions): stop the search as soon as the keys at or above
// the current score-word bound number k..k+slack and keep them all (no tie pass):
// the returned bound's score is then a valid strict filter for later (higher-index)
// items, since at least k kept keys outrank any later key of that score or less.
// slack < 0: exactly the top k (the final per-chunk cut fs_select relies on).
__device__ __forceinline__ float compact_slot(u64* buf, int n, int k, int lane, int* new_cnt, unsigned lo,
                                              unsigned hi, int slack = -1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's inserts are in L2
    u64 x[kNK];
    unsigned hw[kNK];
#pragma unroll
    for (int q = 0; q < kNK; ++q) {
        x[q] = lane + 64 * q < n ? ld_u64_l2(buf + lane + 64 * q) : 0ull;
        hw[q] = (unsigned)(x[q] >> 32);
    }
    // every buffered score word lies in [lo, hi] (lo = ord(threshold): the kept k-th key sits on it; hi = the
    // row's maximum), so the answer shares their common high bits: search below them
    const unsigned diff = lo ^ hi;
    const int top = diff ? 31 - __builtin_clz(diff) : -1;
    unsigned th = top >= 31 ? 0u : (hi >> (top + 1)) << (top + 1);
    for (int bit = top; bit >= 0; --bit) {
        const unsigned c = th | (1u << bit);
        int m = 0;
#pragma unroll
        for (int q = 0; q < kNK; ++q) m += popc64(__ballot(hw[q] >= c));
        if (m >= k) {
            th = c;
            if (m <= k + slack) {  // early stop: keep every key whose score word is >= th
                const u64 lt = lanemask_lt(lane);
                int base = 0;
#pragma unroll
                for (int q = 0; q < kNK; ++q) {
                    const bool kp = x[q] != 0ull && hw[q] >= th;
                    const u64 bq = __ballot(kp);
                    if (kp) buf[base + popc64(bq & lt)] = x[q];
                    base += popc64(bq);
                }
                *new_cnt = base;
                return unord_f32(th);
            }
        }
    }
    // th = the k-th largest score word
    int gt = 0, eq = 0;
#pragma unroll
    for (int q = 0; q < kNK; ++q) {
        gt += popc64(__ballot(hw[q] > th));
        eq += popc64(__ballot(hw[q] == th));
    }
    const int need = k - gt;  // keys with score word th that are kept
    unsigned tl = 0;          // keep (th, lo >= tl); 0 keeps the whole tie group
    if (eq != need) {
        for (int bit = 31; bit >= 0; --bit) {
            const unsigned c = tl | (1u << bit);
            int m = 0;
#pragma unroll
            for (int q = 0; q < kNK; ++q) m += popc64(__ballot(hw[q] == th && (unsigned)x[q] >= c));
            if (m >= need) tl = c;
        }
    }
    const u64 T = ((u64)th << 32) | tl;
    const u64 lt = lanemask_lt(lane);
    int base = 0;
#pragma unroll
    for (int q = 0; q < kNK; ++q) {
        const bool kp = x[q] != 0ull && x[q] >= T;
        const u64 bq = __ballot(kp);
        if (kp) buf[base + popc64(bq & lt)] = x[q];
        base += popc64(bq);
    }
    *new_cnt = base;
    return key_score(T);
}

// One wavefront per block, no barriers: the wave owns 32 users and walks its item
// chunk in 32-item tiles.  A operands (item rows) come straight from L2 into a
// double-buffered register set (lane l: item l&31, floats [h*D/2 + CW*c, +CW)),
// prefetched one chunk ahead of the MFMAs that consume the current one; rows past
// the chunk are clamped to a valid row and zeroed, so the load is branch-free.
#ifndef RSX_FS_FULLLOAD
#define RSX_FS_FULLLOAD 1
#endif
#ifndef RSX_FS_GUARD
#define RSX_FS_GUARD 1
#endif
#ifndef RSX_FS_SLACK
#define RSX_FS_SLACK 16  // running compactions keep up to k + this many keys (-1: exact top k)
#endif
#ifndef RSX_FS_WARM
#define RSX_FS_WARM 8  // tiles scored up front for the warm-up threshold (0: off)
#endif
template <int D, int CW>
__device__ __forceinline__ void load_chunk(float (&r)[CW], const float* I, int64_t item, int64_t i1, int64_t ni,
                                           int off, bool full = false) {
    if (RSX_FS_FULLLOAD && full) {  // the whole 32-item tile is inside the chunk (wave-uniform): no clamps, no selects
        const float* p = I + item * D + off;
#pragma unroll
        for (int q = 0; q < CW / 4; ++q) {
            const float4 v = ld4(p + 4 * q);
            r[4 * q] = v.x;
            r[4 * q + 1] = v.y;
            r[4 * q + 2] = v.z;
            r[4 * q + 3] = v.w;
        }
        return;
    }
    const bool ok = item < i1;
    const float* p = I + (ok ? item : ni - 1) * D + off;
#pragma unroll
    for (int q = 0; q < CW / 4; ++q) {
        const float4 v = ld4(p + 4 * q);
        r[4 * q] = ok ? v.x : 0.f;
        r[4 * q + 1] = ok ? v.y : 0.f;
        r[4 * q + 2] = ok ? v.z : 0.f;
        r[4 * q + 3] = ok ? v.w : 0.f;
    }
}

template <int V>
struct IntC {
    static constexpr int value = V;
};

// No LDS and no block barrier: the candidate buffers live in the workspace (one
// [kCap] row per (user, chunk), L2-resident), so two wavefronts fit on every SIMD
// (VGPRs permitting) and the hardware interleaves them: one wave's filtering and
// compaction issue while the other's MFMA chain runs.  Mask cursor and compaction
// are per-lane / per-user branches; the MFMA chain of tile t is issued before the
// filter of tile t-1 so the VALU work starts as soon as the previous scores exist.
template <int D, int MODE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(D <= 64 ? 2 : 1))) void fs_tiles(FsArgs a) {
    constexpr int HALF = D / 2;
    constexpr int CW = HALF < 32 ? HALF : 32;  // floats per operand chunk
    constexpr int NCH = HALF / CW;             // chunks per lane-half row

    const int lane = threadIdx.x, j = lane & 31, h = lane >> 5;
    __shared__ __attribute__((aligned(16))) float sscr[64 * 16];
    float* scratch = sscr + lane * 4;  // score r of this lane: scratch[256 * (r >> 2) + (r & 3)] (conflict-free float4 rows)
    // block -> (user block, chunk).  Blocks are dealt round-robin to the 8 XCDs, so
    // when the chunk count divides 8 the blocks of one XCD all work on the same
    // chunk and its L2 holds that chunk's item rows (placement is a speed matter only)
    const int64_t n_ub = (a.nb + 31) / 32;
    int64_t ub;
    int chunk;
    if ((8 % a.n_chunks) == 0) {
        const int64_t b = blockIdx.x, xcd = b & 7, slot = b >> 3;
        chunk = (int)(xcd % a.n_chunks);
        ub = slot * (8 / a.n_chunks) + xcd / a.n_chunks;
    } else {
        chunk = (int)(blockIdx.x % a.n_chunks);
        ub = blockIdx.x / a.n_chunks;
    }
    if (ub >= n_ub) return;
    const int64_t ublock = ub * 32;
    const int64_t bslot = ublock + j;
    const bool uvalid = bslot < a.nb;
    const int64_t urow = uvalid ? (a.users ? a.users[bslot] : bslot) : 0;
    const int64_t i0 = (int64_t)chunk * a.chunk_items;
    const int64_t i1 = min(a.ni, i0 + a.chunk_items);
    const int ntiles = (int)((i1 - i0 + 31) / 32);
    // candidate row of (user, chunk); the row of user jj is base + jj * rowstep
    u64* const base = a.cand + (ublock * a.n_chunks + chunk) * (int64_t)kCap;
    const int64_t rowstep = (int64_t)a.n_chunks * kCap;
    u64* mybuf = base + (int64_t)j * rowstep;

    float bu[HALF];
    {
        const float* ur = a.U + urow * D + h * HALF;
#pragma unroll
        for (int s = 0; s < HALF; s += 4) {
            const float4 v = uvalid ? ld4(ur + s) : f4(0.f);
            bu[s] = v.x;
            bu[s + 1] = v.y;
            bu[s + 2] = v.z;
            bu[s + 3] = v.w;
        }
    }
    int64_t mp = 0, me = 0;
    int64_t next_mask = LLONG_MAX;
    if (uvalid && a.mrp) {
        int64_t lo = a.mrp[urow], hi = a.mrp[urow + 1];
        me = hi;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if ((int64_t)a.mcol[mid] < i0) lo = mid + 1; else hi = mid;
        }
        mp = lo;
        next_mask = mp < me ? (int64_t)a.mcol[mp] : LLONG_MAX;
    }
    int cnt = 0;
    float tau = -INFINITY;
    unsigned omax = 0;  // max ordered score word this lane inserted (the row max is the pair's max)
    u64 prof[6] = {0, 0, 0, 0, 0, 0};  // MODE 4: memtime per segment (mfma issue, -, filter, compact, mask+copy, tiles)
    const int64_t nsteps = (int64_t)ntiles * NCH;
    float ra[CW], rb[CW];
    if (ntiles > 0) load_chunk<D, CW>(ra, a.I, i0 + j, i1, a.ni, h * HALF, i0 + 32 <= i1);

    auto mask_bits = [&](int64_t tb) __attribute__((always_inline)) -> unsigned {  // train items of this user in [tb, tb+32)
        unsigned mb = 0;
        while (next_mask < tb + 32) {
            mb |= 1u << (unsigned)(next_mask - tb);
            ++mp;
            next_mask = mp < me ? (int64_t)a.mcol[mp] : LLONG_MAX;
        }
        return mb;
    };
    auto mfma_tile = [&](auto par, int t, floatx16& acc) __attribute__((always_inline)) {
        constexpr int P = decltype(par)::value;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
        if constexpr (NCH == 1) {
            // one operand buffer: once the chain has read it, it is refilled with the
            // next tile's rows (the loads land while this tile is filtered)
#pragma unroll
            for (int q = 0; q < CW; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[q], bu[q], acc, 0, 0, 0);
            if (!RSX_FS_GUARD || t + 1 < ntiles)  // the chain has read ra: refill it with the next tile (none after the last)
                load_chunk<D, CW>(ra, a.I, i0 + (int64_t)(t + 1) * 32 + j, i1, a.ni, h * HALF,
                                  i0 + (int64_t)(t + 2) * 32 <= i1);
        } else {
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
                float(&cur)[CW] = ((P + c) & 1) ? rb : ra;
                float(&nxt)[CW] = ((P + c) & 1) ? ra : rb;
                const int64_t s1 = (int64_t)t * NCH + c + 1;
                const int t1 = (int)(s1 / NCH), c1 = (int)(s1 % NCH);
                load_chunk<D, CW>(nxt, a.I, s1 < nsteps ? i0 + (int64_t)t1 * 32 + j : i1, i1, a.ni,
                                  h * HALF + CW * c1, s1 < nsteps && i0 + (int64_t)(t1 + 1) * 32 <= i1);
#pragma unroll
                for (int q = 0; q < CW; ++q)
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q], bu[CW * c + q], acc, 0, 0, 0);
            }
        }
    };
    // FULL: all 32 items of the tile are in the chunk; MASKED: some lane has train
    // items in it (both wave-uniform, so the common tile takes the leanest variant)
    auto filter_v = [&](auto full_c, auto masked_c, const floatx16& sv, unsigned mb, int64_t tb) __attribute__((always_inline)) {
        constexpr bool FULL = decltype(full_c)::value != 0, MASKED = decltype(masked_c)::value != 0;
        if constexpr (FULL && !MASKED) {
            // the common tile once the threshold has settled: one max over the 16
            // scores decides whether this lane (and, by ballot, the wave) has anything
            float mx = sv[0];
#pragma unroll
            for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sv[r]);
            if (__ballot(uvalid && mx > tau) == 0ull) return;
        }
        unsigned m = 0;
        const int rem = (int)(i1 - tb);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int ii = (r & 3) + 8 * (r >> 2) + 4 * h;
            const float sc = (MASKED && ((mb >> ii) & 1u)) ? -1e10f : sv[r];
            m |= ((FULL || ii < rem) && sc > tau) ? (1u << r) : 0u;
        }
        if (!uvalid) m = 0;
        const u64 ci0 = MODE == 4 ? __builtin_amdgcn_s_memtime() : 0;
        if (__ballot(m != 0u)) {
            // a lane takes ~1 score per tile on average: stage the 16 scores in the
            // lane's LDS scratch and insert only the set bits (per-lane index = address)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *reinterpret_cast<float4*>(scratch + 256 * q) = make_float4(sv[4 * q], sv[4 * q + 1], sv[4 * q + 2], sv[4 * q + 3]);
            const unsigned pm = (unsigned)__shfl_xor((int)m, 32, kWave);
            int pos = cnt + (h ? __popc(pm) : 0);
            cnt += __popc(m) + __popc(pm);
            unsigned mm = m;
            while (mm) {
                const int r = __ffs(mm) - 1;
                mm &= mm - 1;
                const int ii = (r & 3) + 8 * (r >> 2) + 4 * h;
                const float raw = scratch[256 * (r >> 2) + (r & 3)];
                const float sc = (MASKED && ((mb >> ii) & 1u)) ? -1e10f : raw;
                const u64 key = make_key(sc, (int)(tb + ii));
                omax = max(omax, (unsigned)(key >> 32));
                mybuf[pos++] = key;
            }
        }
        if constexpr (MODE == 4) prof[1] += __builtin_amdgcn_s_memtime() - ci0;
    };
    auto filter = [&](const floatx16& sv, unsigned mb, int64_t tb) __attribute__((always_inline)) {
        if constexpr (MODE == 1) {
            float sink = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) sink += sv[r];
            if (sink == 1234.5f) a.out_val[0] = sink;  // keep the MFMAs live
            return;
        }
        const bool full = tb + 32 <= i1;
        const bool masked = __ballot(mb != 0u) != 0ull;
        if (full) {
            if (masked) filter_v(IntC<1>{}, IntC<1>{}, sv, mb, tb);
            else filter_v(IntC<1>{}, IntC<0>{}, sv, mb, tb);
        } else {
            filter_v(IntC<0>{}, IntC<1>{}, sv, mb, tb);
        }
    };
    auto compact = [&]() __attribute__((always_inline)) {
        if constexpr (MODE == 1) return;
        u64 need = __ballot(h == 0 && cnt > kCap - 32);
        while (need) {
            const int jj = __ffsll((long long)need) - 1;
            need &= need - 1;
            const int n = __builtin_amdgcn_readlane(cnt, jj);
            const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)ord_f32(tau), jj);
            const unsigned hi = max((unsigned)__builtin_amdgcn_readlane((int)omax, jj),
                                    (unsigned)__builtin_amdgcn_readlane((int)omax, jj + 32));
            int kept;
            const float nt = compact_slot(base + (int64_t)jj * rowstep, n, a.k, lane, &kept, lo, hi, RSX_FS_SLACK);
            if (j == jj) {
                tau = nt;
                cnt = kept;
            }
        }
    };

    // Warm-up threshold (d <= 64): score the chunk's first RSX_FS_WARM tiles once
    // without inserting anything, keeping per lane the two largest (masked) scores of
    // each of its 16 accumulator slots -- 64 distinct items per user, so for k <= 64
    // the k-th largest of those scores bounds the chunk's k-th best score from below
    // -- then restart at tile 0 keeping only scores >= that bound.  This replaces the
    // warm-up's unfiltered inserts and every user's first compaction with
    // RSX_FS_WARM extra tiles of MFMA.
    if constexpr (NCH == 1 && MODE != 1) {
        if (RSX_FS_WARM > 0 && ntiles > RSX_FS_WARM && a.k <= 64) {
            const int64_t mp0 = mp, nm0 = next_mask;
            float t1[16], t2[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) t1[r] = t2[r] = -INFINITY;
            for (int t = 0; t < RSX_FS_WARM; ++t) {
                floatx16 acc;
                mfma_tile(IntC<0>{}, t, acc);
                const unsigned mb = mask_bits(i0 + (int64_t)t * 32);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int ii = (r & 3) + 8 * (r >> 2) + 4 * h;
                    const float sc = ((mb >> ii) & 1u) ? -1e10f : acc[r];
                    const float lo = fminf(t1[r], sc);
                    t1[r] = fmaxf(t1[r], sc);
                    t2[r] = fmaxf(t2[r], lo);
                }
            }
            // the k-th largest of the lane pair's 64 scores (radix search on ordered words)
            unsigned th = 0;
            for (int bit = 31; bit >= 0; --bit) {
                const unsigned c = th | (1u << bit);
                int n = 0;
#pragma unroll
                for (int r = 0; r < 16; ++r) n += (int)(ord_f32(t1[r]) >= c) + (int)(ord_f32(t2[r]) >= c);
                n += __shfl_xor(n, 32, kWave);
                if (n >= a.k) th = c;
            }
            // keep ord(score) >= th, i.e. score > unord(th - 1): ties with the bound stay
            // (items before the bound's own item rank above it in (score, index) order)
            // (-0.0 == +0.0 as floats: a bound at +0.0 filters with a negative denormal)
            if (uvalid && th > 0) {
                const float tb = unord_f32(th - 1);
                tau = tb == 0.f ? -__FLT_DENORM_MIN__ : tb;
            }
            mp = mp0;
            next_mask = nm0;
            load_chunk<D, CW>(ra, a.I, i0 + j, i1, a.ni, h * HALF, i0 + 32 <= i1);
        }
    }

    if (ntiles > 0) {
        // one tile per iteration: the chain of tile t is issued before the filter of
        // tile t-1; the accumulator rotates by a register copy, so filter and
        // compaction have one call site each
        floatx16 prev, cur;
        mfma_tile(IntC<0>{}, 0, prev);
        unsigned mb = mask_bits(i0);
        for (int t = 1; t < ntiles; ++t) {
            const u64 c0 = MODE == 4 ? __builtin_amdgcn_s_memtime() : 0;
            mfma_tile(IntC<0>{}, t, cur);
            const u64 c1 = MODE == 4 ? __builtin_amdgcn_s_memtime() : 0;
            filter(prev, mb, i0 + (int64_t)(t - 1) * 32);
            const u64 c2 = MODE == 4 ? __builtin_amdgcn_s_memtime() : 0;
            compact();
            const u64 c3 = MODE == 4 ? __builtin_amdgcn_s_memtime() : 0;
            mb = mask_bits(i0 + (int64_t)t * 32);
            prev = cur;
            if constexpr (MODE == 4) {
                const u64 c4 = __builtin_amdgcn_s_memtime();
                prof[0] += c1 - c0;
                prof[2] += c2 - c1;
                prof[3] += c3 - c2;
                prof[4] += c4 - c3;
                prof[5] += 1;
            }
        }
        filter(prev, mb, i0 + (int64_t)(ntiles - 1) * 32);
        compact();
    }
    if constexpr (MODE == 4) {
        if (lane == 0) {
            unsigned long long* dbg = reinterpret_cast<unsigned long long*>(a.out_idx);
#pragma unroll
            for (int q = 0; q < 6; ++q) atomicAdd(dbg + q, (unsigned long long)prof[q]);
        }
        return;
    }
    if constexpr (MODE == 1) return;
    if (a.n_chunks > 2) {  // lists cut to their top k: fs_select then reads <= k <= 96 keys per chunk
        u64 need = __ballot(h == 0 && cnt > a.k);
        while (need) {
            const int jj = __ffsll((long long)need) - 1;
            need &= need - 1;
            const int n = __builtin_amdgcn_readlane(cnt, jj);
            const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)ord_f32(tau), jj);
            const unsigned hi = max((unsigned)__builtin_amdgcn_readlane((int)omax, jj),
                                    (unsigned)__builtin_amdgcn_readlane((int)omax, jj + 32));
            int kept;
            compact_slot(base + (int64_t)jj * rowstep, n, a.k, lane, &kept, lo, hi);
            if (j == jj) cnt = kept;
        }
    }
    if (uvalid && h == 0) a.ccount[bslot * a.n_chunks + chunk] = cnt;
}

// ---------------------------------------------------------------------------
// Screened full-sort (k <= 64): bf16 MFMA bounds, exact f32 scores for the
// candidates only.
//
// fs_tiles spends most of its time on f32 MFMA (1/16 of the bf16 rate) and on
// inserting scores that a low running threshold lets through.  fs_screen scores
// every (user, item) pair twice with v_mfma_f32_32x32x16_bf16 and computes the
// exact f32 score only for the few items that can reach the user's top k:
//  * bound: with bf16 (round-to-nearest) operands, exact products and f32
//    accumulation, |s~ - s| <= eps * sum_j |u_j||v_j| <= eps * |u| * |v_i| for the
//    exact f32 score s (an fmaf chain) and eps = 2^-7 + 2^-16 + 2 D 2^-23 < kScreenEps;
//    the margin eps |u| |v_i| rides in the MFMA as one more K block: the item's bf16
//    row carries |v_i| and the user's carries -+eps |u|, both rounded up, so the
//    accumulator holds the bound itself;
//  * pass 1: each lane keeps, per accumulator slot, the three largest lower bounds
//    s~ - eps |u||v_i| (masked items: exactly -1e10) -- 96 distinct items per user --
//    and the k-th largest of them, L, is a lower bound of the user's exact k-th
//    score (k items are known to score >= L);
//  * pass 2: an item whose upper bound s~ + eps |u||v_i| is >= L (> the running
//    threshold) gets its exact score by an fmaf chain over d in order (bitwise the
//    score_dense kernel's; the user row from LDS), and enters the candidate row as
//    fs_tiles' 64-bit key if that score is >= L; rows that fill up are compacted
//    exactly as in fs_tiles.
// The candidate rows, counts and fs_select are fs_tiles'; the top k is exact.
//
// Invariants the exactness rests on (a change to either pass must keep every one;
// tests/test_gpu_realshape.py::test_fullsort_screen_exact_vs_cpu_fmaf anchors them on
// the CPU's fmaf scores, test_gpu_kernels.py::test_fullsort_screen_exact_vs_dense_scores
// on score_dense's):
//  (i)   bound: for every unmasked item, lo_i <= s_i <= hi_i with lo/hi the pass-1 /
//        pass-2 accumulators (the margin block rounds |v_i| and eps |u| up);
//  (ii)  key score: a masked item's score is exactly -1e10 in both passes (not its
//        bound), an item past the chunk end is -inf in pass 1 and never queued;
//  (iii) threshold: L = the k-th largest of >= k DISTINCT items' lower scores (pass 1
//        samples distinct items per slot), so at least k items score >= L and every
//        top-k item scores >= L; tau starts just below L and only rises to a k-th
//        largest exact key of the user's row, so "score > tau" never rejects a top-k item;
//  (iv)  queue completeness: pass 2 queues EVERY item whose upper score (hi_i, or -1e10
//        for a masked item) exceeds the user's tau when its tile is scanned -- masked
//        items included: a user whose unmasked items number fewer than k in the chunk
//        has L = -1e10 and needs its masked items in the candidate row (they fill the
//        top k as -1e10 in index order).  The round-2 "leaner masked-tile branch" that
//        was reverted skipped masked items in pass 2 and broke exactly this: pass 1 stays
//        correct, the row misses its -1e10 entries.  Rebuilt (tools/fs_lean_variant.py)
//        and run on the GPU: it fails the CPU-anchored test on the masked-heavy users only
//        (rows 1, 2 at every plan, k 50 / 64) and the dense-scores test on its masked-heavy
//        user at k 50 / 64 only (30 unmasked items: k 1 / 17 need no -1e10 entry); every
//        other row stays exact (profiles/r03/fs_invariant/);
//  (v)   drain order: a queued item is scored against the user's tau at drain time
//        (tau only rises), and a row is compacted to its exact top k+slack keys before
//        it could overflow; fs_select then merges the user's lists exactly.
// Round 3 refinements, each keeping (i)-(v):
//  * two phases (default; RSX_FS_2PHASE=0: one launch): pass 1 of every segment max-es its
//    L into a per-user word, pass 2 starts every segment of the user from the largest --
//    each segment's L is a lower bound of the user's k-th score (iii), so their max is;
//  * mask-free pass 1 (when every user of the wave has k + m <= 32 * RSX_FS_TOP, m = its
//    masked items in the segment): masked items are sampled by their bounds and L is the
//    (k + m)-th largest sample -- at most m of the k + m distinct items above it are
//    masked, so (iii) holds without a per-slot mask select;
//  * pass 2 with every tau >= -1e10 (wave-uniform test): a masked item's key -1e10 never
//    exceeds tau, so (iv) needs no masked entry; items are tested by their raw upper
//    bound (a masked hit is queued with its mask bit and scored -1e10 at the drain, below
//    tau); a wave with some tau < -1e10 takes the exact masked select of (iv).
// ---------------------------------------------------------------------------
#ifndef RSX_FS_SCREEN_WPE
#define RSX_FS_SCREEN_WPE 2  // fs_screen waves per SIMD requested at d <= 64
#endif
#ifndef RSX_FS_ABUF
#define RSX_FS_ABUF 2  // fs_screen item-operand buffers at d <= 64 (a ring: loads NB - 1 tiles ahead; 1 at d > 64)
#endif
#ifndef RSX_FS_P1PIPE
#define RSX_FS_P1PIPE 0  // 1: fs_screen pass 1 software-pipelined over two accumulators (A/B variant)
#endif
#ifndef RSX_FS_TOP
#define RSX_FS_TOP 3  // fs_screen pass-1 samples per accumulator slot (2 or 3): 32 * TOP distinct items a user
#endif
template <int D>
constexpr int kAbuf = D <= 64 ? RSX_FS_ABUF : 1;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr float kScreenEps = 0.0080f;

template <int D>
constexpr int kScreenRow = D + 16;  // bf16 elements per screened item row: the row, then |v| and 15 zeros
constexpr int kScreenPadTiles = 2;  // 32-row tiles past ni_pad in the bf16 copy (read ahead, never used)

__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
    const bf16x2 v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(unsigned, v);
}
__device__ __forceinline__ bf16x8 pack_bf16x8(float4 p, float4 q) {
    const u32x4 w = {pack_bf16x2(p.x, p.y), pack_bf16x2(p.z, p.w), pack_bf16x2(q.x, q.y), pack_bf16x2(q.z, q.w)};
    return __builtin_bit_cast(bf16x8, w);
}
// v_max_f32 / v_med3_f32 as single instructions: the builtins' IEEE-mode lowering adds a
// canonicalising max per operand (scores are finite here)
__device__ __forceinline__ float vmax(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vmed3(float a, float b, float c) {
    float r;
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// bf16 bits of the smallest bf16 >= x (x >= 0 finite)
__device__ __forceinline__ unsigned bf16_up(float x) { return (__float_as_uint(x) + 0xffffu) >> 16; }

// bf16 copy of every item row with its L2 norm appended (rounded up); rows [ni, ni_pad)
// are zero.  D/4 threads a row.
template <int D>
__global__ __launch_bounds__(256) void fs_prep(const float* __restrict__ I, int64_t ni, int64_t ni_pad,
                                               __bf16* __restrict__ Ib) {
    constexpr int G = D / 4;
    constexpr int DP = kScreenRow<D>;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t row = t / G;
    const int c = (int)(t % G);
    const float4 v = row < ni ? ld4(I + row * D + 4 * c) : f4(0.f);
    float ss = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) ss += __shfl_xor(ss, o, kWave);  // the row's G threads: one aligned lane group
    if (row >= ni_pad) return;
    __bf16* r = Ib + row * DP;
    *reinterpret_cast<uint2*>(r + 4 * c) = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
    if (c == 0) {
        const u32x4 z = {0u, 0u, 0u, 0u};
        u32x4 w = z;
        w[0] = bf16_up(sqrtf(ss) * 1.0001f);  // element D (low half of the first word)
        *reinterpret_cast<u32x4*>(r + D) = w;
        *reinterpret_cast<u32x4*>(r + D + 8) = z;
    }
}

// ND exact scores at once (one per candidate, the chains interleaved: each is exact_dot's
// fmaf chain over d in order, bit for bit; the interleave only hides the FMA latency)
template <int D, int ND>
__device__ __forceinline__ void exact_dots(const float* const (&u)[ND], const float* const (&v)[ND], float (&out)[ND]) {
    float acc[ND];
#pragma unroll
    for (int n = 0; n < ND; ++n) acc[n] = 0.f;
#pragma unroll 4
    for (int c = 0; c < D; c += 4) {
        float4 x[ND], y[ND];
#pragma unroll
        for (int n = 0; n < ND; ++n) {
            x[n] = *reinterpret_cast<const float4*>(u[n] + c);
            y[n] = ld4(v[n] + c);
        }
#pragma unroll
        for (int n = 0; n < ND; ++n) {
            acc[n] = fmaf(x[n].x, y[n].x, acc[n]);
            acc[n] = fmaf(x[n].y, y[n].y, acc[n]);
            acc[n] = fmaf(x[n].z, y[n].z, acc[n]);
            acc[n] = fmaf(x[n].w, y[n].w, acc[n]);
        }
    }
#pragma unroll
    for (int n = 0; n < ND; ++n) out[n] = acc[n];
}

// exact score <U row, I row>: fmaf chain over d in order (as score_dense)
template <int D>
__device__ __forceinline__ float exact_dot(const float* __restrict__ u, const float* __restrict__ v) {
    float acc = 0.f;
#pragma unroll 4  // blocks of 16 d: the loads of a block in flight together, few registers
    for (int c = 0; c < D; c += 4) {
        const float4 x = *reinterpret_cast<const float4*>(u + c), y = ld4(v + c);
        acc = fmaf(x.x, y.x, acc);
        acc = fmaf(x.y, y.y, acc);
        acc = fmaf(x.z, y.z, acc);
        acc = fmaf(x.w, y.w, acc);
    }
    return acc;
}

// One segment of fs_screen: user block ub, item tiles [ta, tz) of chunk `chunk`, into
// candidate list `li` of the block's users (lists per user: a.n_lists).
// train-item mask lists: a user's masked columns of the segment in LDS (up to kMaskCap,
// stride kMaskCap + 1: conflict-free; screen_segment's LDS form)
#ifndef RSX_FS_DRAIN
#define RSX_FS_DRAIN 1  // pass-2 candidates scored per lane per drain (interleaved exact dots; 2: same time)
#endif
constexpr int kDrainPer = RSX_FS_DRAIN;
constexpr int kQueueCap = 64 * kDrainPer + 1024;  // < 64 kDrainPer pending + one tile's (<= 16 per lane)
constexpr int kMaskCap = 32;
constexpr int kMaskStride = kMaskCap + 1;

// PH: 0 both passes in one launch (the segment's own L); 1 pass 1 only, the segment's L
// max-ed into a.lbound[user]; 2 pass 2 only, from tau = the user's a.lbound (every
// segment of the user: chunks and split ranges)
template <int D, int PH>
__device__ __forceinline__ void screen_segment(const FsArgs& a, int64_t ub, int chunk, int li, int ta, int tz,
                                               float* urows, unsigned* queue, int* lcnt, unsigned* lomax,
                                               int* mlds) {
    constexpr int HALF = D / 2;
    constexpr int NM = D / 16;  // bf16 MFMAs per 32x32 tile over the row (8 operand elements per lane each)
    constexpr int DP = kScreenRow<D>;
    constexpr int US = D + 4;   // LDS user row stride (floats)
    const int lane = threadIdx.x, j = lane & 31, h = lane >> 5;
    const int64_t ublock = ub * 32;
    const int64_t bslot = ublock + j;
    const bool uvalid = bslot < a.nb;
    const int64_t urow = uvalid ? (a.users ? a.users[bslot] : bslot) : 0;
    const int64_t c0 = (int64_t)chunk * a.chunk_items;
    const int64_t i0 = c0 + (int64_t)ta * 32;
    const int64_t i1 = min(min(a.ni, c0 + a.chunk_items), c0 + (int64_t)tz * 32);
    const int ntiles = tz - ta;
    u64* const base = a.cand + (ublock * a.n_lists + li) * (int64_t)kCap;
    const int64_t rowstep = (int64_t)a.n_lists * kCap;

    // B operand: lane (user j, half h) holds u_j[h D/2 + 8 s .. + 8) for MFMA s (the A
    // operand takes the item rows with the same split, so each MFMA sums 16 of the d);
    // the f32 row also goes to LDS for the exact scores
    u32x4 bu[NM + 1];
    float ss = 0.f;
    float* const myrow = urows + j * US;
#pragma unroll
    for (int s = 0; s < NM; ++s) {
        const float4 p = uvalid ? ld4(a.U + urow * D + h * HALF + 8 * s) : f4(0.f);
        const float4 q = uvalid ? ld4(a.U + urow * D + h * HALF + 8 * s + 4) : f4(0.f);
        ss += p.x * p.x + p.y * p.y + p.z * p.z + p.w * p.w + q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
        bu[s] = u32x4{pack_bf16x2(p.x, p.y), pack_bf16x2(p.z, p.w), pack_bf16x2(q.x, q.y), pack_bf16x2(q.z, q.w)};
        if constexpr (PH != 1) {  // the f32 row for the exact scores (pass 2)
            *reinterpret_cast<float4*>(myrow + h * HALF + 8 * s) = p;
            *reinterpret_cast<float4*>(myrow + h * HALF + 8 * s + 4) = q;
        }
    }
    ss += __shfl_xor(ss, 32, kWave);
    // margin block: element 0 of lane half 0 carries -eps |u| (pass 1; +eps |u| in pass 2)
    const unsigned cmb = bf16_up(kScreenEps * sqrtf(ss) * 1.0001f);
    bu[NM] = u32x4{h == 0 ? (cmb | 0x8000u) : 0u, 0u, 0u, 0u};
    __syncthreads();  // urows (the previous segment's readers are done: see the end)

    // train-item mask: the user's sorted columns; [mp, mq) are the segment's
    int64_t mp = 0, me = 0, mq = 0;
    if (uvalid && a.mrp) {
        int64_t lo = a.mrp[urow], hi = a.mrp[urow + 1];
        me = hi;
        auto first_ge = [&](int64_t l, int64_t r, int64_t x) __attribute__((always_inline)) {
            while (l < r) {
                const int64_t mid = (l + r) >> 1;
                if ((int64_t)a.mcol[mid] < x) l = mid + 1; else r = mid;
            }
            return l;
        };
        mp = first_ge(lo, hi, i0);
        mq = first_ge(mp, hi, i1);
    }
    // m = the user's masked items in [i0, i1).  MASK-FREE pass 1 (wave-uniform, when every
    // user has k + m <= the 32 * RSX_FS_TOP samples): masked items are sampled by their
    // bounds like any other, and L is the (k + m)-th largest sample -- of the k + m distinct
    // items at or above it at most m are masked, so k unmasked items score >= L
    const int64_t mcount = mq - mp;
    const int kk = a.k + (int)mcount;
    const bool mfree = __ballot(uvalid && kk > 32 * RSX_FS_TOP) == 0ull;
    // The mask cursor, in one of two forms chosen per segment (wave-uniform):
    //  LDS: every user's m <= kMaskCap -- the segment's columns staged once in the user's
    //       LDS list (both lane halves read it; INT_MAX-terminated): the tile loops then
    //       hold no global load besides the item operands, so their waits count those;
    //  GLOBAL: a per-lane cursor over the columns, the one after the current prefetched.
    const bool mlds_ok = __ballot(mcount > kMaskCap) == 0ull;
    int* const ml = mlds + j * kMaskStride;
    if (mlds_ok) {
        int v[kMaskCap / 2];  // lane half h loads entries h, h + 2, ..: every load before the first store
        if (mcount > 0) {
#pragma unroll
            for (int q = 0; q < kMaskCap / 2; ++q) v[q] = a.mcol[mp + min((int64_t)(2 * q + h), mcount - 1)];
        }
#pragma unroll
        for (int q = 0; q < kMaskCap / 2; ++q) ml[2 * q + h] = 2 * q + h < mcount ? v[q] : INT_MAX;
        if (h == 0) ml[kMaskCap] = INT_MAX;
    }
    const int64_t mp0 = mp;
    int next_mask = INT_MAX, after = INT_MAX, mcur = 0;
    auto mask_start = [&]() __attribute__((always_inline)) {  // (every variable assigned on every path)
        const int nm = mlds_ok ? ml[0] : (mp0 < me ? a.mcol[mp0] : INT_MAX);
        const int af = (!mlds_ok && mp0 + 1 < me) ? a.mcol[mp0 + 1] : INT_MAX;
        mcur = 0;
        mp = mp0;
        next_mask = nm;
        after = af;
    };
    __syncthreads();  // the lists (lanes read their partner half's entries)
    mask_start();
    // the tile's mask bits, form M: 0 none (mask-free pass 1), 1 LDS, 2 GLOBAL
    auto mask_bits = [&](auto form, int64_t tb) __attribute__((always_inline)) -> unsigned {
        constexpr int M = decltype(form)::value;
        unsigned mb = 0;
        if constexpr (M == 1) {
            while ((int64_t)next_mask < tb + 32) {
                mb |= 1u << (unsigned)((int64_t)next_mask - tb);
                next_mask = ml[++mcur];
            }
        } else if constexpr (M == 2) {
            while ((int64_t)next_mask < tb + 32) {
                mb |= 1u << (unsigned)((int64_t)next_mask - tb);
                ++mp;
                next_mask = after;
                after = mp + 1 < me ? a.mcol[mp + 1] : INT_MAX;
            }
        }
        return mb;
    };
    // A operand: item i0 + 32 t + j, half h (the padded bf16 copy: no clamps), loaded
    // in tile order through one stepping pointer.  NB > 1: a ring of NB buffers, tile
    // t's MFMAs preceded by the loads of tile t + NB - 1 (two tiles of latency cover at
    // two waves per SIMD); NB = 1: one buffer refilled with the next tile as soon as the
    // MFMAs have read it.  Every tile issues its load unconditionally (a conditional
    // load would make the compiler's wait before the MFMAs cover the prefetch too): the
    // last NB - 1 loads read past the segment, into the copy's kScreenPadTiles tiles
    constexpr int NB = kAbuf<D>;
    u32x4 ra[NB][NM + 1];
    const __bf16* const a0 = a.Ib + (i0 + j) * DP;
    const __bf16* anext = a0;
    auto load_a = [&](auto par) __attribute__((always_inline)) {
        constexpr int P = decltype(par)::value % NB;
        const u32x4* p = reinterpret_cast<const u32x4*>(anext + h * HALF);
#pragma unroll
        for (int s = 0; s < NM; ++s) ra[P][s] = p[s];
        ra[P][NM] = *reinterpret_cast<const u32x4*>(anext + D + 8 * h);
        anext += 32 * DP;
    };
    auto tile = [&](auto par, int t, floatx16& acc) __attribute__((always_inline)) {
        constexpr int P = decltype(par)::value % NB;
        if constexpr (NB > 1) load_a(IntC<(P + NB - 1) % NB>{});
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
        for (int s = 0; s <= NM; ++s)
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ra[P][s]),
                                                          __builtin_bit_cast(bf16x8, bu[s]), acc, 0, 0, 0);
        if constexpr (NB == 1) load_a(IntC<0>{});
    };
    // the first NB - 1 tiles' loads, then tiles in groups of NB (ring slots by template)
    auto prime = [&]() __attribute__((always_inline)) {
        anext = a0;
        if (ntiles <= 0) return;
        load_a(IntC<0>{});
        if constexpr (NB > 2) load_a(IntC<1>{});
    };
    auto sweep = [&](auto&& body) __attribute__((always_inline)) {
        for (int t = 0; t < ntiles; t += NB) {
            body(IntC<0>{}, t);
            if constexpr (NB > 1)
                if (t + 1 < ntiles) body(IntC<1>{}, t + 1);
            if constexpr (NB > 2)
                if (t + 2 < ntiles) body(IntC<2>{}, t + 2);
        }
    };

    // pass 1: the RSX_FS_TOP largest lower bounds per slot (t3 unused at 2)
    float t1[16], t2[16], t3[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) t1[r] = t2[r] = t3[r] = -INFINITY;
    // pass 1 of one tile in two halves: p1_issue (the mask cursor, then the tile's MFMAs)
    // and p1_update (the missing / masked slots' keys, the per-slot top three)
    auto p1_issue = [&](auto form, auto par, int t, floatx16& acc) __attribute__((always_inline)) -> unsigned {
        // the mask cursor first: its loads' waits then precede the next tile's prefetch
        const unsigned mb = mask_bits(form, i0 + (int64_t)t * 32);
        tile(par, t, acc);
        return mb;
    };
    auto p1_update = [&](auto form, int t, floatx16& acc, unsigned mb) __attribute__((always_inline)) {
        const int64_t tb = i0 + (int64_t)t * 32;
        const int rem = (int)(i1 - tb);
        // a tile with a missing item (the chunk's last) or, outside the mask-free form, a
        // masked one: those slots first take their key (-inf / -1e10) in place, then every
        // tile runs the same update (one code path: no register shuffles between forms)
        if (rem < 32 || (decltype(form)::value != 0 && __ballot(mb != 0u) != 0ull)) {  // wave-uniform
            // slot r <-> item io(r) + 4 h: shift the mask and the bound by 4 h once, so the
            // per-slot tests take immediates (no per-slot constants held in registers)
            const unsigned mbh = mb >> (4 * h);
            const int remh = rem - 4 * h;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int io = (r & 3) + 8 * (r >> 2);
                acc[r] = io >= remh ? -INFINITY : (((mbh >> io) & 1u) ? -1e10f : acc[r]);
            }
        }
        // top three by median-of-three (t1 >= t2 >= t3): t3 = med3(t2, t3, x),
        // t2 = med3(t1, t2, x), t1 = max(t1, x)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if constexpr (RSX_FS_TOP == 3) t3[r] = vmed3(t2[r], t3[r], acc[r]);
            t2[r] = vmed3(t1[r], t2[r], acc[r]);
            t1[r] = vmax(t1[r], acc[r]);
        }
    };
    auto pass1 = [&](auto form, auto par, int t) __attribute__((always_inline)) {
        floatx16 acc;
        const unsigned mb = p1_issue(form, par, t, acc);
        p1_update(form, t, acc, mb);
    };
    // Software-pipelined pass 1 (NB <= 2): tile t + 1's MFMAs are issued before tile t's
    // top-three update, into a second accumulator, so the update's VALU fills the matrix
    // pipe's dependent-MFMA gaps of the same wave instead of following the chain (one
    // accumulator serialises MFMA chain -> VALU -> next chain: ~48 VALU per tile behind
    // 5 dependent MFMAs).  Same tiles, same order of updates: the same samples.
    auto sweep1 = [&](auto form) __attribute__((always_inline)) {
        // the mask-free form of the two-phase pass-1 kernel at d <= 64 (the other forms and
        // kernels would spill past the two-waves-per-SIMD register budget)
        if constexpr (RSX_FS_P1PIPE && NB <= 2 && decltype(form)::value == 0 && PH == 1 && D <= 64) {
            if (ntiles <= 0) return;
            // every tile but the segment's last is full: the loop's tiles take the top-three
            // update with no masking (one basic block: the next tile's MFMAs and this tile's
            // VALU interleave, one MFMA per ~9 updates); the last tile the masked form
            auto upd = [&](floatx16& acc) __attribute__((always_inline)) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    if constexpr (RSX_FS_TOP == 3) t3[r] = vmed3(t2[r], t3[r], acc[r]);
                    t2[r] = vmed3(t1[r], t2[r], acc[r]);
                    t1[r] = vmax(t1[r], acc[r]);
                }
            };
#define RSX_P1_INTERLEAVE()                                     \
    do {                                                        \
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);      \
        __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);     \
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);      \
        __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);     \
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);      \
        __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);     \
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);      \
        __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);     \
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);      \
        __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);     \
    } while (0)
            floatx16 acc0, acc1;
            unsigned mb0 = p1_issue(form, IntC<0>{}, 0, acc0), mb1 = 0;
            int t = 0;
            for (; t + 2 < ntiles; t += 2) {  // tiles t, t + 1 full
                mb1 = p1_issue(form, IntC<1>{}, t + 1, acc1);
                upd(acc0);
                RSX_P1_INTERLEAVE();
                mb0 = p1_issue(form, IntC<0>{}, t + 2, acc0);
                upd(acc1);
                RSX_P1_INTERLEAVE();
            }
#undef RSX_P1_INTERLEAVE
            if (t + 1 < ntiles) {  // tiles t (full) and t + 1 (the last)
                mb1 = p1_issue(form, IntC<1>{}, t + 1, acc1);
                upd(acc0);
                p1_update(form, t + 1, acc1, mb1);
            } else {
                p1_update(form, t, acc0, mb0);
            }
        } else {
            sweep([&](auto par, int t) __attribute__((always_inline)) { pass1(form, par, t); });
        }
    };
    unsigned th = 0;
    if constexpr (PH != 2) {
        prime();
        if (mfree) sweep1(IntC<0>{});
        else if (mlds_ok) sweep1(IntC<1>{});
        else sweep1(IntC<2>{});
        if constexpr (PH == 1) {  // publish the samples; fs_thresh takes L over all the user's segments
            if (uvalid) {
                // high half of the ordered word (rounding down: a lower bound stays one); -inf
                // (a missing item) as 0, which counts as no sample
                auto s16 = [](float x) __attribute__((always_inline)) -> unsigned {
                    return x == -INFINITY ? 0u : ord_f32(x) >> 16;
                };
                uint4* dst = reinterpret_cast<uint4*>(a.samp + ((bslot * a.n_lists + li) * 96 + h * 48));
#pragma unroll
                for (int q = 0; q < 6; ++q) {
                    unsigned w[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int v0 = 8 * q + 2 * e, v1 = v0 + 1;  // sample v: t1 / t2 / t3 [v % 16] by v / 16
                        const float x0 = v0 < 16 ? t1[v0] : v0 < 32 ? t2[v0 - 16] : t3[v0 - 32];
                        const float x1 = v1 < 16 ? t1[v1] : v1 < 32 ? t2[v1 - 16] : t3[v1 - 32];
                        w[e] = s16(RSX_FS_TOP == 3 || v0 < 32 ? x0 : -INFINITY) |
                               (s16(RSX_FS_TOP == 3 || v1 < 32 ? x1 : -INFINITY) << 16);
                    }
                    dst[q] = make_uint4(w[0], w[1], w[2], w[3]);
                }
                if (h == 0) a.mcnt1[bslot * a.n_lists + li] = (uint16_t)(mfree ? min(mcount, (int64_t)0xfffe) : 0);
            }
            return;
        }
        // L = the k-th largest of the lane pair's 32 * RSX_FS_TOP bounds (radix search on
        // ordered words)
        for (int bit = 31; bit >= 0; --bit) {
            const unsigned c = th | (1u << bit);
            int n = 0;
#pragma unroll
            for (int r = 0; r < 16; ++r)
                n += (int)(ord_f32(t1[r]) >= c) + (int)(ord_f32(t2[r]) >= c) +
                     (RSX_FS_TOP == 3 ? (int)(ord_f32(t3[r]) >= c) : 0);
            n += __shfl_xor(n, 32, kWave);
            if (n >= (mfree ? kk : a.k)) th = c;
        }
    } else {
        th = uvalid ? a.lbound[bslot] : 0u;
    }
    // running strict filter "> tau" keeping every score >= L (the ordered word below L's;
    // -0.0 == +0.0 as floats, so a bound that lands on a zero filters with a negative denormal)
    float tau = -INFINITY;
    if (th > ord_f32(-INFINITY)) {
        const float tb = unord_f32(th - 1);
        tau = tb == 0.f ? -__FLT_DENORM_MIN__ : tb;
    }
    if (PH == 0 && FS_ABL(5)) {  // profiling ablation: pass 1 only
        if (uvalid && h == 0) a.ccount[bslot * a.n_lists + li] = 0;
        if (tau == 1234.5f) a.out_val[0] = tau;
        __syncthreads();
        return;
    }

    // pass 2: candidates by upper bound go to a queue in LDS (item << 6 | masked << 5 | user);
    // groups of 64 get their exact scores one per lane (all lanes busy), and the kept
    // keys enter the users' candidate rows (fs_tiles' rows and compaction), counts and
    // row maxima kept in LDS
    bu[NM] = u32x4{h == 0 ? cmb : 0u, 0u, 0u, 0u};
    mask_start();
    int cnt = 0;
    unsigned omax = 0;
    if (lane < 32) {
        lcnt[lane] = 0;
        lomax[lane] = 0u;
    }
    int qn = 0;  // queued candidates (wave-uniform)
    int nq = 0;  // mode 9 (profiling): candidates queued by this segment
    auto compact = [&]() __attribute__((always_inline)) {
        u64 need = __ballot(h == 0 && cnt > kCap - 64 * kDrainPer);  // room for a whole drain group after this
        while (need) {
            const int jj = __ffsll((long long)need) - 1;
            need &= need - 1;
            const int nn = __builtin_amdgcn_readlane(cnt, jj);
            const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)ord_f32(tau), jj);
            const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)omax, jj);
            int kept;
            const float nt = compact_slot(base + (int64_t)jj * rowstep, nn, a.k, lane, &kept, lo, hi, RSX_FS_SLACK);
            if (j == jj) {
                tau = nt;
                cnt = kept;
            }
            if (lane == jj) lcnt[jj] = kept;
        }
    };
    const u64 ltm = lanemask_lt(lane);
    auto drain = [&](bool all) __attribute__((always_inline)) {
        constexpr int G = 64 * kDrainPer;  // candidates per drain group: kDrainPer per lane
        int g = 0;
        while (qn - g >= G || (all && qn > g)) {
            const int n = min(G, qn - g);
            __syncthreads();  // queue writes, counts
            unsigned e[kDrainPer];
            int ju[kDrainPer];
            float tj[kDrainPer], sc[kDrainPer];
            const float* up[kDrainPer];
            const float* vp[kDrainPer];
#pragma unroll
            for (int q = 0; q < kDrainPer; ++q) {
                e[q] = lane + 64 * q < n ? queue[g + lane + 64 * q] : 0u;
                ju[q] = (int)(e[q] & 31u);
                tj[q] = __shfl(tau, ju[q], kWave);
                up[q] = urows + ju[q] * US;
                vp[q] = a.I + (int64_t)(e[q] >> 6) * D;
            }
            if (FS_ABL(6)) {  // profiling ablation: no dots
#pragma unroll
                for (int q = 0; q < kDrainPer; ++q) sc[q] = unord_f32(ord_f32(tj[q]) + 1u + (unsigned)lane);
            } else if (lane < n) {  // (lanes past n hold item 0: valid addresses, results unused)
                exact_dots<D, kDrainPer>(up, vp, sc);
            }
#pragma unroll
            for (int q = 0; q < kDrainPer; ++q) {
                const float v = (e[q] & 32u) ? -1e10f : sc[q];
                if (lane + 64 * q < n && v > tj[q]) {
                    const int pos = atomicAdd(&lcnt[ju[q]], 1);
                    const u64 key = make_key(v, (int)(e[q] >> 6));
                    atomicMax(&lomax[ju[q]], (unsigned)(key >> 32));
                    base[(int64_t)ju[q] * rowstep + pos] = key;
                }
            }
            __syncthreads();
            cnt = lcnt[j];
            omax = lomax[j];
            compact();
            g += n;
        }
        const int rest = qn - g;
        if (g > 0 && rest > 0) {  // rest < G: the unscored tail to the queue's front
            unsigned v[kDrainPer];
            __syncthreads();
#pragma unroll
            for (int q = 0; q < kDrainPer; ++q) v[q] = lane + 64 * q < rest ? queue[g + lane + 64 * q] : 0u;
            __syncthreads();
#pragma unroll
            for (int q = 0; q < kDrainPer; ++q)
                if (lane + 64 * q < rest) queue[lane + 64 * q] = v[q];
        }
        qn = rest;
    };
    auto pass2 = [&](auto form, auto par, int t) __attribute__((always_inline)) {
        const int64_t tb = i0 + (int64_t)t * 32;
        const unsigned mb = mask_bits(form, tb);
        floatx16 acc;
        tile(par, t, acc);
        const int rem = (int)(i1 - tb);
        const unsigned ebase = ((unsigned)(tb + 4 * h) << 6) | (unsigned)j;
        // one ballot per slot; its lanes append at queue[qn + their rank] (branch-free tests)
        auto push = [&](bool c, unsigned e) __attribute__((always_inline)) {
            const u64 bal = __ballot(c) & (FS_ABL(8) ? 0ull : ~0ull);  // 8: profiling ablation, no candidates
            if (bal) {
                const int rk = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
                if (c) queue[qn + rk] = e;
                qn += popc64(bal);
                if (FS_ABL(9)) nq += popc64(bal);
            }
        };
        const float tv = uvalid ? tau : INFINITY;  // invalid users take nothing
        // every tau >= -1e10 (wave-uniform): a masked item (key -1e10) never needs queueing,
        // so the items are tested by their raw upper bounds and a hit carries its mask bit
        // (the drain scores it -1e10, below tau); otherwise -- and on the chunk's last tile
        // -- masked slots take -1e10 and missing ones -inf in place first
        const unsigned mbh = mb >> (4 * h);
        if (rem < 32 || __ballot(tv < -1e10f) != 0ull) {
            const int remh = rem - 4 * h;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int io = (r & 3) + 8 * (r >> 2);
                acc[r] = io >= remh ? -INFINITY : (((mbh >> io) & 1u) ? -1e10f : acc[r]);
            }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int io = (r & 3) + 8 * (r >> 2);
            push(acc[r] > tv, (ebase + ((unsigned)io << 6)) | (((mbh >> io) & 1u) << 5));
        }
        if (qn >= 64 * kDrainPer) drain(false);
    };
    prime();
    if (mlds_ok) sweep([&](auto par, int t) __attribute__((always_inline)) { pass2(IntC<1>{}, par, t); });
    else sweep([&](auto par, int t) __attribute__((always_inline)) { pass2(IntC<2>{}, par, t); });
    drain(true);
    __syncthreads();
    cnt = lcnt[j];
    omax = lomax[j];
    if (a.n_lists > 8) {  // lists cut to their top k (fs_select<16, 2>)
        u64 need = __ballot(h == 0 && cnt > a.k);
        while (need) {
            const int jj = __ffsll((long long)need) - 1;
            need &= need - 1;
            const int nn = __builtin_amdgcn_readlane(cnt, jj);
            const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)ord_f32(tau), jj);
            const unsigned hi = max((unsigned)__builtin_amdgcn_readlane((int)omax, jj),
                                    (unsigned)__builtin_amdgcn_readlane((int)omax, jj + 32));
            int kept;
            compact_slot(base + (int64_t)jj * rowstep, nn, a.k, lane, &kept, lo, hi);
            if (j == jj) cnt = kept;
        }
    }
    if (uvalid && h == 0) a.ccount[bslot * a.n_lists + li] = cnt;
    if (FS_ABL(9) && lane == 0) {  // profiling: queued / kept candidate totals into out_idx[0], [1]
        atomicAdd(reinterpret_cast<unsigned long long*>(a.out_idx), (unsigned long long)nq);
        int kept = 0;
        for (int q = 0; q < 32; ++q) kept += lcnt[q];
        atomicAdd(reinterpret_cast<unsigned long long*>(a.out_idx) + 1, (unsigned long long)kept);
    }
    __syncthreads();  // LDS reuse by the next segment
}

// Balanced full-sort screening: the (user block, item tile) pairs of each chunk are
// split evenly over the chunk's waves (a.seg_waves of them; 0: one wave per (user
// block, chunk)), so that every SIMD gets the same work whatever the user count --
// 2,226 whole (block, chunk) waves on 2,048 resident slots would take two rounds.  A
// wave's range covers whole or partial tile ranges of consecutive user blocks; segment
// s of (block, chunk) writes list chunk * S + s (S = a.seg_slots), and the last segment
// of a (block, chunk) zeroes the counts of the lists after it.
template <int D, int PH>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(D <= 64 ? RSX_FS_SCREEN_WPE : 1))) void fs_screen(FsArgs a) {
    constexpr int US = D + 4;
    __shared__ __attribute__((aligned(16))) float urows[PH == 1 ? 4 : 32 * US];  // pass 2's f32 user rows
    __shared__ unsigned queue[PH == 1 ? 1 : kQueueCap];  // pass 2 candidates
    __shared__ int lcnt[32];
    __shared__ unsigned lomax[32];
    __shared__ int mlds[32 * kMaskStride];
    const int64_t n_ub = (a.nb + 31) / 32;
    const int64_t nper = a.seg_waves ? a.seg_waves : n_ub;  // waves per chunk
    int64_t w;
    int chunk;
    if ((8 % a.n_chunks) == 0) {  // one chunk per XCD: blocks are dealt round-robin to the 8 XCDs
        const int64_t b = blockIdx.x, xcd = b & 7, slot = b >> 3;
        chunk = (int)(xcd % a.n_chunks);
        w = slot * (8 / a.n_chunks) + xcd / a.n_chunks;
    } else {
        chunk = (int)(blockIdx.x % a.n_chunks);
        w = blockIdx.x / a.n_chunks;
    }
    if (w >= nper) return;
    const int64_t c0 = (int64_t)chunk * a.chunk_items;
    const int nt = (int)((min(a.ni, c0 + a.chunk_items) - c0 + 31) / 32);
    const int64_t T = n_ub * nt;
    const int64_t lo = a.seg_waves ? w * T / nper : w * nt, hi = a.seg_waves ? (w + 1) * T / nper : (w + 1) * nt;
    const int S = a.seg_slots;
    for (int64_t x = lo; x < hi;) {
        const int64_t ub = x / nt;
        const int t0 = (int)(x - ub * nt);
        const int t1 = (int)min((int64_t)nt, t0 + (hi - x));
        const int64_t wf = ((ub * nt + 1) * nper + T - 1) / T - 1;  // the wave whose range holds tile 0 of ub
        const int seg = a.seg_waves ? (int)(w - wf) : 0;
        screen_segment<D, PH>(a, ub, chunk, chunk * S + seg, t0, t1, urows, queue, lcnt, lomax, mlds);
        if (PH != 1 && t1 == nt) {  // the block's last segment in this chunk: the later lists are empty
            const int j = threadIdx.x & 31;
            const int64_t bslot = ub * 32 + j;
            if (threadIdx.x < 32 && bslot < a.nb)
                for (int q = seg + 1; q < S; ++q) a.ccount[bslot * a.n_lists + chunk * S + q] = 0;
        }
        x += t1 - t0;
    }
}

// The user's L of the two-phase screen: the (k + M)-th largest of every sample its pass-1
// segments published (M = their masked items sampled by value).  The segments cover
// disjoint item ranges, so the samples are distinct items and at most M of the k + M at
// or above L are masked: k unmasked items score >= L (invariant (iii) over the union).
// One wave per user; 16-bit radix search; fewer than k + M samples: no threshold (0).
// NW: sample pairs (u32 words) per lane, nl * 48 <= 64 NW
template <int NW>
__global__ __launch_bounds__(256) void fs_thresh(const uint16_t* __restrict__ samp, const uint16_t* __restrict__ mcnt,
                                                 int nl, int64_t nb, int k, unsigned* __restrict__ lbound) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= nb) return;  // whole waves
    const unsigned m = lane < nl ? (unsigned)mcnt[b * nl + lane] : 0xffffu;
    const u64 valid = __ballot(m != 0xffffu);  // bit l: list l has a segment
    int mm = m != 0xffffu ? (int)m : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mm += __shfl_xor(mm, o, kWave);
    const int kk = k + mm;
    const int nwords = nl * 48;
    const unsigned* __restrict__ w32 = reinterpret_cast<const unsigned*>(samp) + b * nwords;
    unsigned v[2 * NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) {  // every load before the first use
        const int e = lane + 64 * q;
        const unsigned x = e < nwords ? w32[e] : 0u;
        const bool ok = e < nwords && ((valid >> (e / 48)) & 1ull);
        v[2 * q] = ok ? (x & 0xffffu) : 0u;
        v[2 * q + 1] = ok ? (x >> 16) : 0u;
    }
    unsigned th = 0;
    for (int bit = 15; bit >= 0; --bit) {
        const unsigned c = th | (1u << bit);
        int n = 0;
#pragma unroll
        for (int q = 0; q < 2 * NW; ++q) n += popc64(__ballot(v[q] >= c));
        if (n >= kk) th = c;
    }
    if (lane == 0) lbound[b] = th << 16;
}

// Exact k-th largest of the nonzero keys held E per lane (radix search with ballots,
// score word first, index word only for a tie at the boundary).
template <int E>
__device__ __forceinline__ u64 kth_largest_n(const u64 (&e)[E], int k) {
    // the nonzero keys' score words lie in [lo, hi] (wave min / max), so the answer
    // shares their common high bits: search only below them (as compact_slot)
    unsigned hi = 0u, lo = 0xffffffffu;
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const unsigned w = (unsigned)(e[m] >> 32);
        if (e[m] != 0ull) {
            hi = max(hi, w);
            lo = min(lo, w);
        }
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        hi = max(hi, (unsigned)__shfl_xor((int)hi, o, kWave));
        lo = min(lo, (unsigned)__shfl_xor((int)lo, o, kWave));
    }
    const unsigned diff = lo ^ hi;
    const int top = diff ? 31 - __builtin_clz(diff) : -1;
    unsigned th = top >= 31 ? 0u : (hi >> (top + 1)) << (top + 1);
    for (int bit = top; bit >= 0; --bit) {
        const unsigned c = th | (1u << bit);
        int n = 0;
#pragma unroll
        for (int m = 0; m < E; ++m) n += popc64(__ballot((unsigned)(e[m] >> 32) >= c));
        if (n >= k) th = c;
    }
    int gt = 0, eq = 0;
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const unsigned h = (unsigned)(e[m] >> 32);
        gt += popc64(__ballot(h > th));
        eq += popc64(__ballot(h == th && e[m] != 0ull));
    }
    const int need = k - gt;
    if (eq == need) return (u64)th << 32;
    unsigned tl = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const unsigned c = tl | (1u << bit);
        int n = 0;
#pragma unroll
        for (int m = 0; m < E; ++m)
            n += popc64(__ballot((unsigned)(e[m] >> 32) == th && (unsigned)e[m] >= c));
        if (n >= need) tl = c;
    }
    return ((u64)th << 32) | tl;
}

// The user's candidate lists as one virtual array: key p lives in list c(p) at offset
// p - off[c] (off[] the lists' prefix sums, wave-uniform).
template <int SMAX>
struct FsLists {
    const u64* src;  // the user's first list; list c at src + c * kCap
    int off[SMAX + 1];
    __device__ __forceinline__ u64 at(int p) const {
        int c = 0;
#pragma unroll
        for (int q = 1; q < SMAX; ++q) c += p >= off[q];
        int o = off[0];
#pragma unroll
        for (int q = 1; q < SMAX; ++q) o = c == q ? off[q] : o;
        return src[c * kCap + (p - o)];
    }
};

__device__ __forceinline__ unsigned wave_sum_u(unsigned x) {
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) x += (unsigned)__shfl_xor((int)x, o, kWave);
    return x;
}

// Exact k-th largest of `total` keys of the lists (any count): the radix search of
// kth_largest_n re-reading the keys (L2) each round -- users with very many keys.
template <int SMAX>
__device__ u64 kth_largest_lists(const FsLists<SMAX>& Ls, int total, int k, int lane) {
    unsigned hi = 0u, lo = 0xffffffffu;
    for (int p = lane; p < total; p += 64) {
        const unsigned w = (unsigned)(Ls.at(p) >> 32);
        hi = max(hi, w);
        lo = min(lo, w);
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        hi = max(hi, (unsigned)__shfl_xor((int)hi, o, kWave));
        lo = min(lo, (unsigned)__shfl_xor((int)lo, o, kWave));
    }
    const unsigned diff = lo ^ hi;
    const int top = diff ? 31 - __builtin_clz(diff) : -1;
    unsigned th = top >= 31 ? 0u : (hi >> (top + 1)) << (top + 1);
    for (int bit = top; bit >= 0; --bit) {
        const unsigned c = th | (1u << bit);
        unsigned n = 0;
        for (int p = lane; p < total; p += 64) n += (unsigned)(Ls.at(p) >> 32) >= c;
        if ((int)wave_sum_u(n) >= k) th = c;
    }
    unsigned gt = 0, eq = 0;
    for (int p = lane; p < total; p += 64) {
        const unsigned w = (unsigned)(Ls.at(p) >> 32);
        gt += w > th;
        eq += w == th;
    }
    const int need = k - (int)wave_sum_u(gt);
    if ((int)wave_sum_u(eq) == need) return (u64)th << 32;
    unsigned tl = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const unsigned c = tl | (1u << bit);
        unsigned n = 0;
        for (int p = lane; p < total; p += 64) {
            const u64 x = Ls.at(p);
            n += (unsigned)(x >> 32) == th && (unsigned)x >= c;
        }
        if ((int)wave_sum_u(n) >= need) tl = c;
    }
    return ((u64)th << 32) | tl;
}

// One wavefront per user: the exact top-k over the user's candidate lists (a.n_lists
// <= SMAX of them: raw rows of <= kCap keys, or rows cut to the top k), ordered by
// (score desc, index asc).  The lists are read as one array of the keys that exist:
// <= 512 of them (<= 4 lists; 1024 for more) go to 8 (16) registers a lane in one round
// trip and the k-th key is searched there; more are searched in place.
template <int SMAX>
__global__ __launch_bounds__(256) void fs_select(FsArgs a) {
    constexpr int kDenseE = SMAX <= 4 ? 8 : 16;  // keys per lane held in registers
    __shared__ u64 top[4][kCap];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t b = (int64_t)blockIdx.x * 4 + wv;
    if (b >= a.nb) return;  // wave-uniform
    FsLists<SMAX> Ls;
    Ls.src = a.cand + b * a.n_lists * (int64_t)kCap;
    int total = 0;
#pragma unroll
    for (int c = 0; c < SMAX; ++c) {
        Ls.off[c] = total;
        total += c < a.n_lists ? a.ccount[b * a.n_lists + c] : 0;
    }
    Ls.off[SMAX] = total;
    const int k = a.k;
    const bool dense = total <= 64 * kDenseE;
    u64 e[kDenseE];
#pragma unroll
    for (int m = 0; m < kDenseE; ++m) e[m] = dense && lane + 64 * m < total ? Ls.at(lane + 64 * m) : 0ull;
    u64 T = 1ull;
    if (total > k) T = dense ? kth_largest_n<kDenseE>(e, k) : kth_largest_lists<SMAX>(Ls, total, k, lane);
    // gather the winners (exactly min(k, total)) into LDS
    const u64 lt = lanemask_lt(lane);
    int base = 0;
    if (dense) {
#pragma unroll
        for (int m = 0; m < kDenseE; ++m) {
            const bool kp = e[m] != 0ull && e[m] >= T;
            const u64 bal = __ballot(kp);
            if (kp) top[wv][base + popc64(bal & lt)] = e[m];
            base += popc64(bal);
        }
    } else {
        for (int p0 = 0; p0 < total; p0 += 64) {
            const u64 x = p0 + lane < total ? Ls.at(p0 + lane) : 0ull;
            const bool kp = x != 0ull && x >= T;
            const u64 bal = __ballot(kp);
            if (kp) top[wv][base + popc64(bal & lt)] = x;
            base += popc64(bal);
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // rank-sort the winners (keys unique): position = number of larger keys
    const int kept = base;
    for (int q = lane; q < kept; q += 64) {
        const u64 mine = top[wv][q];
        int r = 0;
        for (int t = 0; t < kept; ++t) r += top[wv][t] > mine;
        a.out_val[b * k + r] = key_score(mine);
        a.out_idx[b * k + r] = (int64_t)key_index(mine);
    }
    for (int q = kept + lane; q < k; q += 64) {
        a.out_val[b * k + q] = -INFINITY;
        a.out_idx[b * k + q] = -1;
    }
}

static void fs_plan(int64_t nb, int64_t ni, int d, int* nw, int* n_chunks, int64_t* chunk_items) {
    *nw = 1;
    const int64_t waves = (nb + 31) / 32;
    // item chunks per 32-user wave: enough waves for two per SIMD (2048 on the chip:
    // one wave's filtering/compaction overlaps the other's MFMA chain), no more
    // (every extra chunk re-pays the threshold warm-up)
    const int64_t target = d <= 64 ? 1900 : 950;  // fs_tiles occupancy: 2 waves/SIMD at d <= 64, else 1
    int64_t s = (target + waves - 1) / waves;
    if (s < 1) s = 1;
    if (s > 16) s = 16;
    {  // tuning override
        static const int v = env_knob("RSX_FS_CHUNKS", 0, 1, 16);
        if (v) s = v;
    }
    int64_t per = (ni + s - 1) / s;
    per = (per + 31) / 32 * 32;
    if (per < 32) per = 32;
    *chunk_items = per;
    *n_chunks = (int)((ni + per - 1) / per);
}

static bool fs_use_screen(int k, int d, int64_t ni) {
    static const int on = env_knob("RSX_FS_SCREEN", 1, 0, 1);  // 0: the f32-MFMA fs_tiles path
    return on && k <= 64 && (d == 32 || d == 64 || d == 128 || d == 256) && ni < (1ll << 26);  // queue entry: item << 6
}

static size_t fs_align(size_t x) { return (x + 255) / 256 * 256; }

// The lists layout of a call: fs_tiles keeps one list per (user, chunk); fs_screen
// splits each chunk's (user block, tile) pairs evenly over the resident wave slots
// when there are more (block, chunk) waves than slots (SEGMENTS, fs_screen's header).
struct FsLayout {
    int n_chunks;
    int64_t chunk_items;
    bool screen;
    int n_lists, seg_slots;
    int64_t seg_waves;  // waves per chunk (0: one per user block)
    int64_t blocks;
};

static int fs_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0, v = 0;
        n = (hipGetDevice(&dev) == hipSuccess &&
             hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
                ? v
                : 256;
        (void)hipGetLastError();
    }
    return n;
}

// fs_screen's item chunks: the most chunks that still fit every (32-user block, chunk)
// wave in one round of resident slots, when that fills >= 80 % of them (one list per
// chunk, no split); otherwise enough chunks to exceed the slots, split evenly below
// (fs_layout).  At most 16 chunks.
static void screen_plan(int64_t nb, int64_t ni, int wps, int* n_chunks, int64_t* chunk_items) {
    const int64_t n_ub = (nb + 31) / 32;
    const int64_t slots = (int64_t)fs_cus() * 4 * wps;
    int64_t c = slots / n_ub;
    if (c < 1 || n_ub * c * 5 < slots * 4) c = (slots + n_ub - 1) / n_ub;
    if (c < 1) c = 1;
    if (c > 16) c = 16;
    int64_t per = (ni + c - 1) / c;
    per = (per + 31) / 32 * 32;
    *chunk_items = per;
    *n_chunks = (int)((ni + per - 1) / per);
}

// resident fs_screen waves per SIMD a layout plans for: pass 1 (and the one-launch form)
// 2 at d <= 128 (register budget), 1 at d = 256; the pass-2 launch of the two-phase form
// holds no pass-1 samples (fewer registers): RSX_FS_WPS2 (tuning)
static int fs_wps(int d, int phase) {
    static const int w2 = env_knob("RSX_FS_WPS2", 0, 1, 4);
    if (phase == 2 && w2 > 0) return w2;
    return d <= 128 ? 2 : 1;
}

static FsLayout fs_layout(int64_t nb, int64_t ni, int k, int d, int wps) {
    FsLayout L{};
    int nw;
    L.screen = fs_use_screen(k, d, ni);
    if (L.screen) screen_plan(nb, ni, wps, &L.n_chunks, &L.chunk_items);
    else fs_plan(nb, ni, d, &nw, &L.n_chunks, &L.chunk_items);
    L.n_lists = L.n_chunks;
    L.seg_slots = 1;
    const int64_t n_ub = (nb + 31) / 32;
    const int C = L.n_chunks;
    L.blocks = n_ub * C;
    static const int seg_env = env_knob("RSX_FS_SEG", 1, 0, 1);  // 0: no balanced split (tuning)
    if (L.screen && seg_env && (8 % C) == 0) {
        const int64_t slots = (int64_t)fs_cus() * 4 * wps;
        const int64_t wc = slots / C;
        if (n_ub * C > slots && wc >= 1) {
            int S = 1;
            bool ok = true;
            for (int c = 0; c < C; ++c) {
                const int64_t nt = (std::min(ni, (int64_t)(c + 1) * L.chunk_items) - (int64_t)c * L.chunk_items + 31) / 32;
                const int64_t m = n_ub * nt / wc;  // shortest wave range (tiles)
                if (m < 1) ok = false;
                else S = (int)std::max<int64_t>(S, (nt + m - 1) / m + 1);
            }
            if (ok && C * S <= 8) {
                L.seg_waves = wc;
                L.seg_slots = S;
                L.n_lists = C * S;
                L.blocks = wc * C;
            }
        }
    }
    if ((8 % C) == 0) L.blocks = (L.blocks + 7) / 8 * 8;  // whole rounds of the XCD-aware mapping
    return L;
}

// workspace: candidate rows | counts | (screen) bf16 item copy
// candidate lists per user: the pass-2 layout's (two-phase) or the one-launch layout's
static int fs_lists(int64_t nb, int64_t ni, int k, int d) {
    return std::max(fs_layout(nb, ni, k, d, fs_wps(d, 1)).n_lists, fs_layout(nb, ni, k, d, fs_wps(d, 2)).n_lists);
}

size_t fs_ws(int64_t nb, int64_t ni, int k, int d) {
    const FsLayout L = fs_layout(nb, ni, k, d, fs_wps(d, 1));
    const int nl = fs_lists(nb, ni, k, d);
    size_t bytes = fs_align((size_t)nb * nl * kCap * sizeof(u64) + (size_t)nb * nl * sizeof(int) + 512);
    if (L.screen) {
        const size_t ni_pad = (size_t)(ni + 31) / 32 * 32;
        bytes += fs_align((ni_pad + 32 * kScreenPadTiles) * (d + 16) * sizeof(__bf16));
        bytes += fs_align((size_t)nb * sizeof(unsigned));  // lbound
        bytes += fs_align((size_t)nb * L.n_lists * 96 * sizeof(uint16_t));  // samp (pass-1 layout)
        bytes += fs_align((size_t)nb * L.n_lists * sizeof(uint16_t));       // mcnt1
    }
    return bytes;
}

// L: the one-launch / pass-1 layout; L2: the pass-2 layout of the two-phase form (its own
// chunks and segments: pass 1 only publishes per-user thresholds, pass 2 writes the lists)
template <int D>
static int launch_fs(FsArgs& a, const FsLayout& L, const FsLayout& L2, hipStream_t s) {
    const dim3 grid((unsigned)L.blocks);
    if (a.Ib) {  // screened path
        const int64_t ni_pad = (a.ni + 31) / 32 * 32;
        const int64_t nthr = ni_pad * (D / 4);
        hipLaunchKernelGGL((fs_prep<D>), dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, s, a.I, a.ni, ni_pad,
                           const_cast<__bf16*>(a.Ib));
        if (FS_ABL(9)) (void)hipMemsetAsync(a.out_idx, 0, 2 * sizeof(int64_t), s);  // profiling counters
        if (a.lbound) {  // two phases: every segment of a user filters by the user's L over all of them
            (void)hipMemsetAsync(a.mcnt1, 0xff, (size_t)a.nb * L.n_lists * sizeof(uint16_t), s);
            hipLaunchKernelGGL((fs_screen<D, 1>), grid, dim3(64), 0, s, a);
            {
                const dim3 tg((unsigned)((a.nb + 3) / 4));
                const uint16_t* sp = a.samp;
                const uint16_t* mc = a.mcnt1;
                const int nl = L.n_lists;  // <= 16
                if (nl <= 4) hipLaunchKernelGGL((fs_thresh<3>), tg, dim3(256), 0, s, sp, mc, nl, a.nb, a.k, a.lbound);
                else if (nl <= 8) hipLaunchKernelGGL((fs_thresh<6>), tg, dim3(256), 0, s, sp, mc, nl, a.nb, a.k, a.lbound);
                else hipLaunchKernelGGL((fs_thresh<12>), tg, dim3(256), 0, s, sp, mc, nl, a.nb, a.k, a.lbound);
            }
            if (FS_ABL(5)) return last_rc();
            a.n_chunks = L2.n_chunks;
            a.chunk_items = L2.chunk_items;
            a.n_lists = L2.n_lists;
            a.seg_slots = L2.seg_slots;
            a.seg_waves = L2.seg_waves;
            hipLaunchKernelGGL((fs_screen<D, 2>), dim3((unsigned)L2.blocks), dim3(64), 0, s, a);
        } else {
            hipLaunchKernelGGL((fs_screen<D, 0>), grid, dim3(64), 0, s, a);
        }
    } else if (FS_ABL(4)) {
        hipLaunchKernelGGL((fs_tiles<D, 4>), grid, dim3(64), 0, s, a);
    } else if (FS_ABL(1)) {
        hipLaunchKernelGGL((fs_tiles<D, 1>), grid, dim3(64), 0, s, a);
    } else {
        hipLaunchKernelGGL((fs_tiles<D, 0>), grid, dim3(64), 0, s, a);
    }
    const dim3 sg((unsigned)((a.nb + 3) / 4));
    if (FS_ABL(9)) return last_rc();  // profiling: out_idx holds the candidate counts
    if (a.Ib || !RSX_FS_ABLATION || a.mode == 0) {
        const int n = a.n_lists;
        if (n <= 2) hipLaunchKernelGGL((fs_select<2>), sg, dim3(256), 0, s, a);
        else if (n <= 4) hipLaunchKernelGGL((fs_select<4>), sg, dim3(256), 0, s, a);
        else if (n <= 8) hipLaunchKernelGGL((fs_select<8>), sg, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((fs_select<16>), sg, dim3(256), 0, s, a);
    }
    return last_rc();
}

int fs_call(const float* U, const int64_t* users, int64_t nb, const float* I, int64_t ni, int d,
            const int64_t* mrp, const int32_t* mcol, int k, float* out_val, int64_t* out_idx, void* ws,
            size_t ws_bytes, hipStream_t s) {
    if (!U || !I || !out_val || !out_idx || nb < 0 || ni <= 0 || k <= 0) return RSX_ERR_ARG;
    if (k > ni) return RSX_ERR_ARG;
    if (k > kMaxK) return RSX_ERR_UNSUPPORTED;
    if (nb == 0) return RSX_OK;
    if (!ws || ws_bytes < fs_ws(nb, ni, k, d)) return RSX_ERR_WORKSPACE;
    FsArgs a;
    const FsLayout L = fs_layout(nb, ni, k, d, fs_wps(d, 1));
    const int nl = fs_lists(nb, ni, k, d);
    a.n_chunks = L.n_chunks;
    a.chunk_items = L.chunk_items;
    a.n_lists = L.n_lists;
    a.seg_slots = L.seg_slots;
    a.seg_waves = L.seg_waves;
    a.U = U;
    a.users = users;
    a.nb = nb;
    a.I = I;
    a.ni = ni;
    a.mrp = mrp;
    a.mcol = mcol;
    a.k = k;
    a.cand = static_cast<u64*>(ws);
    a.ccount = reinterpret_cast<int*>(static_cast<char*>(ws) + (size_t)nb * nl * kCap * sizeof(u64));
    a.out_val = out_val;
    a.out_idx = out_idx;
    a.Ib = nullptr;
    a.lbound = nullptr;
    a.samp = nullptr;
    a.mcnt1 = nullptr;
    if (L.screen) {
        char* p = static_cast<char*>(ws) + fs_align((size_t)nb * nl * kCap * sizeof(u64) + (size_t)nb * nl * sizeof(int) + 512);
        a.Ib = reinterpret_cast<const __bf16*>(p);
        const size_t ni_pad = (size_t)(ni + 31) / 32 * 32;
        static const int two = env_knob("RSX_FS_2PHASE", 1, 0, 1);  // 0: both passes in one launch, per-segment thresholds
        char* q = p + fs_align((ni_pad + 32 * kScreenPadTiles) * (d + 16) * sizeof(__bf16));
        a.lbound = two ? reinterpret_cast<unsigned*>(q) : nullptr;
        q += fs_align((size_t)nb * sizeof(unsigned));
        a.samp = reinterpret_cast<uint16_t*>(q);
        q += fs_align((size_t)nb * L.n_lists * 96 * sizeof(uint16_t));
        a.mcnt1 = reinterpret_cast<uint16_t*>(q);
    }
    {
        static const int mode = env_knob("RSX_FS_MODE", 0, 0, 9);
        if (mode != 0 && !RSX_FS_ABLATION) {
            fprintf(stderr, "librsx: RSX_FS_MODE=%d is a profiling ablation (wrong top-k by design); it runs only in "
                            "an ablation build (tools/build_variant.py NAME -DRSX_FS_ABLATION=1)\n", mode);
            return RSX_ERR_UNSUPPORTED;
        }
        a.mode = mode;
    }
    const FsLayout L2 = a.lbound ? fs_layout(nb, ni, k, d, fs_wps(d, 2)) : L;
    switch (d) {
        case 32: return launch_fs<32>(a, L, L2, s);
        case 64: return launch_fs<64>(a, L, L2, s);
        case 128: return launch_fs<128>(a, L, L2, s);
        case 256: return launch_fs<256>(a, L, L2, s);
        default: return RSX_ERR_UNSUPPORTED;
    }
}

// ---------------------------------------------------------------------------
// dense scores (full_sort_predict API path) and row gather
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void score_dense(const float* __restrict__ U, const int64_t* __restrict__ users,
                                                   int64_t nb, const float* __restrict__ I, int64_t ni,
                                                   float* __restrict__ out) {
    __shared__ float urow[D];
    const int64_t b = blockIdx.y;
    const int64_t ur = users ? users[b] : b;
    for (int c = threadIdx.x; c < D; c += 256) urow[c] = U[ur * D + c];
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= ni) return;
    const float* ir = I + i * D;
    float acc = 0.f;
#pragma unroll 8
    for (int c = 0; c < D; c += 4) {
        const float4 v = ld4(ir + c);
        acc = fmaf(urow[c], v.x, acc);
        acc = fmaf(urow[c + 1], v.y, acc);
        acc = fmaf(urow[c + 2], v.z, acc);
        acc = fmaf(urow[c + 3], v.w, acc);
    }
    out[b * ni + i] = acc;
}

__global__ void gather_rows_k(const float* __restrict__ src, const int64_t* __restrict__ idx, int64_t n,
                              int64_t offset, int d, float* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t r = t / d;
    if (r >= n) return;
    const int c = (int)(t % d);
    out[r * d + c] = src[(idx[r] + offset) * d + c];
}

}  // namespace rsx

extern "C" {

size_t rsx_fullsort_ws_bytes(int64_t n_batch, int64_t n_items, int32_t k) {
    // worst case over d (the plan's chunk count and the screened path's bf16 item copy depend on d)
    size_t w = 0;
    for (int d : {32, 64, 128, 256}) {
        const size_t b = rsx::fs_ws(n_batch, n_items, k, d);
        w = b > w ? b : w;
    }
    return w;
}

int rsx_fullsort_plan(int64_t n_batch, int64_t n_items, int32_t d, int32_t* n_chunks, int64_t* chunk_items) {
    if (!n_chunks || !chunk_items || n_batch < 0 || n_items <= 0) return RSX_ERR_ARG;
    const rsx::FsLayout L = rsx::fs_layout(n_batch, n_items, 50, d, rsx::fs_wps(d, 1));  // the plan of k <= 64 calls (pass 1)
    *n_chunks = L.n_chunks;
    *chunk_items = L.chunk_items;
    return RSX_OK;
}

int rsx_fullsort_topk(const float* user_emb, const int64_t* users, int64_t n_batch, const float* item_emb,
                      int64_t n_items, int32_t d, const int64_t* mask_rowptr, const int32_t* mask_col, int32_t k,
                      float* out_val, int64_t* out_idx, void* ws, size_t ws_bytes, rsx_stream_t stream) {
    return rsx::fs_call(user_emb, users, n_batch, item_emb, n_items, d, mask_rowptr, mask_col, k, out_val,
                        out_idx, ws, ws_bytes, rsx::as_stream(stream));
}

int rsx_score_dense(const float* user_emb, const int64_t* users, int64_t n_batch, const float* item_emb,
                    int64_t n_items, int32_t d, float* out, rsx_stream_t stream) {
    if (!user_emb || !item_emb || !out || n_batch < 0 || n_items <= 0) return RSX_ERR_ARG;
    if (n_batch == 0) return RSX_OK;
    hipStream_t s = rsx::as_stream(stream);
    dim3 grid((unsigned)((n_items + 255) / 256), (unsigned)n_batch);
    switch (d) {
        case 32: hipLaunchKernelGGL(rsx::score_dense<32>, grid, dim3(256), 0, s, user_emb, users, n_batch, item_emb, n_items, out); break;
        case 64: hipLaunchKernelGGL(rsx::score_dense<64>, grid, dim3(256), 0, s, user_emb, users, n_batch, item_emb, n_items, out); break;
        case 128: hipLaunchKernelGGL(rsx::score_dense<128>, grid, dim3(256), 0, s, user_emb, users, n_batch, item_emb, n_items, out); break;
        case 256: hipLaunchKernelGGL(rsx::score_dense<256>, grid, dim3(256), 0, s, user_emb, users, n_batch, item_emb, n_items, out); break;
        default: return RSX_ERR_UNSUPPORTED;
    }
    return rsx::last_rc();
}

int rsx_gather_rows(const float* src, const int64_t* idx, int64_t n, int64_t offset, int32_t d, float* out,
                    rsx_stream_t stream) {
    if (!src || !idx || !out || n < 0 || d <= 0) return RSX_ERR_ARG;
    if (n == 0) return RSX_OK;
    const int64_t tot = n * d;
    hipLaunchKernelGGL(rsx::gather_rows_k, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                       rsx::as_stream(stream), src, idx, n, offset, d, out);
    return rsx::last_rc();
}

}  // extern "C"

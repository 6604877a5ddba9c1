// fullsort.hip — full-sort user x item scoring fused with train-item masking and top-K (gfx950).
//
// Replaces, per evaluation batch (reference src/common/trainer.py:509-528):
//     scores = u_emb[users] @ item_emb.T          (src/models/lightgcn.py:164, layergcn.py:186,
//                                                  smore.py:420)
//     scores[mask[0], mask[1]] = -1e10             (trainer.py:524)
//     _, topk = torch.topk(scores, k, dim=-1)      (trainer.py:526)
// without materialising the [B_u, n_items] score matrix.
//
// Kernel 1 (fs_tiles): grid = (user blocks of 32*NW users) x (item chunks).  Each
// wavefront owns 32 users; the NW waves of a block share 32-item tiles staged in
// LDS (double buffered, row stride D+4 floats so the 32 lanes of a half-wave hit
// 32 distinct 4-bank slots).  A 32x32 score tile is D/2 v_mfma_f32_32x32x2_f32 —
// exact f32 fma chains, A = item rows, B = user rows, with the reduction index k
// permuted so that lane-half h reads the contiguous half [h*D/2, (h+1)*D/2) of its
// row.  The C/D layout puts user j = lane&31 on the lane and 16 items in the
// registers, so lanes j and j+32 together hold the tile's 32 scores of user j.
// Scores above the user's running threshold go into a per-user LDS candidate
// buffer as 64-bit keys (ordered score bits << 32 | ~item), so one u64 order is
// (score desc, index asc); when a buffer may overflow the wave bitonic-sorts it
// and keeps the top K, which also raises the threshold.  Items arrive in
// ascending index order within a chunk, so the strict "> threshold" filter drops
// nothing that the canonical order would keep.
// Kernel 2 (fs_merge): 16 lanes per user merge the chunks' sorted top-K lists.
#include <climits>

#include "rsx_common.hpp"

namespace rsx {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef unsigned long long u64;

constexpr int kCap = 128;  // candidate slots per user (>= K + 32)
constexpr int kMaxK = kCap - 32;

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
    u64* cand;  // [nb][n_chunks][k]
    float* out_val;
    int64_t* out_idx;
};

constexpr int kStride = kCap + 1;  // u64 slots per user row in LDS (+1: spreads the 32 users over banks)

__device__ __forceinline__ int popc64(u64 x) { return __popcll(x); }
__device__ __forceinline__ u64 lanemask_lt(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

// Exact k-th largest of the (unique, nonzero) keys e0/e1 held by the wave, by a
// bitwise binary search with ballots: 32 steps on the score half, and 32 more on
// the index half only when scores tie at the boundary.  Zero keys are padding.
__device__ __forceinline__ u64 kth_largest(u64 e0, u64 e1, int k) {
    const unsigned h0 = (unsigned)(e0 >> 32), h1 = (unsigned)(e1 >> 32);
    unsigned th = 0;
#pragma unroll 4
    for (int bit = 31; bit >= 0; --bit) {
        const unsigned c = th | (1u << bit);
        const int n = popc64(__ballot(h0 >= c)) + popc64(__ballot(h1 >= c));
        if (n >= k) th = c;
    }
    // th = largest score-word with at least k keys >= it
    const int gt = popc64(__ballot(h0 > th)) + popc64(__ballot(h1 > th));
    const int need = k - gt;  // how many of the keys with score-word == th are kept
    const int eq = popc64(__ballot(h0 == th)) + popc64(__ballot(h1 == th));
    if (eq == need) return ((u64)th << 32);  // every tie kept: threshold = lowest key of the tie group
    const unsigned l0 = (unsigned)e0, l1 = (unsigned)e1;
    unsigned tl = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const unsigned c = tl | (1u << bit);
        const int n = popc64(__ballot(h0 == th && l0 >= c)) + popc64(__ballot(h1 == th && l1 >= c));
        if (n >= need) tl = c;
    }
    return ((u64)th << 32) | tl;
}

// Keep the k largest keys of one user's buffer (n > k entries), compacted to the
// front; returns the new score threshold.  Whole wave, no sort.
__device__ __forceinline__ float compact_slot(u64* buf, int n, int k, int lane) {
    const u64 e0 = lane < n ? buf[lane] : 0ull;
    const u64 e1 = lane + 64 < n ? buf[lane + 64] : 0ull;
    const u64 T = kth_largest(e0, e1, k);
    const bool k0 = e0 != 0ull && e0 >= T;
    const bool k1 = e1 != 0ull && e1 >= T;
    const u64 b0 = __ballot(k0), b1 = __ballot(k1);
    const u64 lt = lanemask_lt(lane);
    const int p0 = popc64(b0 & lt);
    const int p1 = popc64(b0) + popc64(b1 & lt);
    __builtin_amdgcn_wave_barrier();
    if (k0) buf[p0] = e0;
    if (k1) buf[p1] = e1;
    __builtin_amdgcn_wave_barrier();
    return key_score(T);
}

// Write the top-min(n,k) keys of one user's buffer to dst[0..k) in descending
// order (rank by counting: every lane compares its key with all others via
// readlane; no LDS round trips), zero-padded.  n <= kCap.
__device__ __forceinline__ void emit_sorted(const u64* buf, int n, int k, int lane, u64* dst) {
    u64 e0 = lane < n ? buf[lane] : 0ull;
    u64 e1 = lane + 64 < n ? buf[lane + 64] : 0ull;
    if (n > k) {
        const u64 T = kth_largest(e0, e1, k);
        if (e0 < T) e0 = 0ull;
        if (e1 < T) e1 = 0ull;
    }
    int r0 = 0, r1 = 0;
    const int m = n < 64 ? n : 64;
    for (int t = 0; t < m; ++t) {
        const unsigned lo = __builtin_amdgcn_readlane((unsigned)(e0 & 0xffffffffu), t);
        const unsigned hi = __builtin_amdgcn_readlane((unsigned)(e0 >> 32), t);
        const u64 x = ((u64)hi << 32) | lo;
        r0 += x > e0;
        r1 += x > e1;
    }
    for (int t = 0; t < n - 64; ++t) {
        const unsigned lo = __builtin_amdgcn_readlane((unsigned)(e1 & 0xffffffffu), t);
        const unsigned hi = __builtin_amdgcn_readlane((unsigned)(e1 >> 32), t);
        const u64 x = ((u64)hi << 32) | lo;
        r0 += x > e0;
        r1 += x > e1;
    }
    if (e0 != 0ull && r0 < k) dst[r0] = e0;
    if (e1 != 0ull && r1 < k) dst[r1] = e1;
    const int kept = n < k ? n : k;
    for (int e = kept + lane; e < k; e += 64) dst[e] = 0ull;
}

template <int D, int NW>
__global__ __launch_bounds__(64 * NW) void fs_tiles(FsArgs a) {
    constexpr int LD = D + 4;
    constexpr int HALF = D / 2;
    constexpr int PER = (32 * D / 4) / (64 * NW);  // float4 loads per thread per tile
    static_assert(PER >= 1, "tile too small for block");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* tiles = reinterpret_cast<float*>(smem);                           // [2][32][LD]
    u64* cbuf = reinterpret_cast<u64*>(smem + 2 * 32 * LD * sizeof(float));  // [NW*32][kStride]

    const int tid = threadIdx.x;
    const int wv = tid >> 6, lane = tid & 63, j = lane & 31, h = lane >> 5;
    const int slot = wv * 32 + j;
    const int64_t bslot = (int64_t)blockIdx.x * (32 * NW) + slot;
    const bool uvalid = bslot < a.nb;
    const int64_t urow = uvalid ? (a.users ? a.users[bslot] : bslot) : 0;
    const int chunk = blockIdx.y;
    const int64_t i0 = (int64_t)chunk * a.chunk_items;
    const int64_t i1 = min(a.ni, i0 + a.chunk_items);
    const int ntiles = (int)((i1 - i0 + 31) / 32);
    u64* mybuf = cbuf + slot * kStride;

    // user fragment: B[k][j] for k in this lane-half's contiguous half of the row
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
    // mask cursor: first training item >= i0 (columns sorted)
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
    int cnt = 0;  // candidates of user j (same value in lanes j and j+32)
    float tau = -INFINITY;

    float4 pre[PER];
    auto load_tile = [&](int t) {
        const int64_t base = i0 + (int64_t)t * 32;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int f = tid + q * 64 * NW;  // float4 index within the tile
            const int r = f / (D / 4), c4 = f % (D / 4);
            const int64_t item = base + r;
            pre[q] = item < i1 ? ld4(a.I + item * D + c4 * 4) : f4(0.f);
        }
    };
    auto store_tile = [&](int buf) {
        float* tb = tiles + buf * 32 * LD;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int f = tid + q * 64 * NW;
            const int r = f / (D / 4), c4 = f % (D / 4);
            st4(tb + r * LD + c4 * 4, pre[q]);
        }
    };
    if (ntiles > 0) {
        load_tile(0);
        store_tile(0);
    }
    __syncthreads();

    for (int t = 0; t < ntiles; ++t) {
        const int buf = t & 1;
        if (t + 1 < ntiles) load_tile(t + 1);
        // 32x32 score tile
        floatx16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
        const float* ar = tiles + buf * 32 * LD + j * LD + h * HALF;
#pragma unroll
        for (int s = 0; s < HALF; s += 4) {
            const float4 av = ld4(ar + s);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bu[s], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bu[s + 1], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bu[s + 2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bu[s + 3], acc, 0, 0, 0);
        }
        if (t + 1 < ntiles) store_tile(buf ^ 1);
        // masked items of this tile for user j
        const int64_t tb = i0 + (int64_t)t * 32;
        unsigned mbits = 0;
        while (next_mask < tb + 32) {
            mbits |= 1u << (unsigned)(next_mask - tb);
            ++mp;
            next_mask = mp < me ? (int64_t)a.mcol[mp] : LLONG_MAX;
        }
        // which of my 16 scores pass the threshold
        unsigned m = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int ii = (r & 3) + 8 * (r >> 2) + 4 * h;
            const float sc = ((mbits >> ii) & 1u) ? -1e10f : acc[r];
            if (uvalid && tb + ii < i1 && sc > tau) m |= 1u << r;
        }
        if (__ballot(m != 0u)) {
            const unsigned pm = (unsigned)__shfl_xor((int)m, 32, kWave);  // partner half's mask
            int pos = cnt + (h ? __popc(pm) : 0);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if ((m >> r) & 1u) {
                    const int ii = (r & 3) + 8 * (r >> 2) + 4 * h;
                    const float sc = ((mbits >> ii) & 1u) ? -1e10f : acc[r];
                    mybuf[pos++] = make_key(sc, (int)(tb + ii));
                }
            }
            cnt += __popc(m) + __popc(pm);
        }
        // keep room for the next tile (at most 32 new candidates per user)
        u64 need = __ballot(h == 0 && cnt > kCap - 32);
        if (need) {
            __builtin_amdgcn_wave_barrier();
            while (need) {
                const int jj = __ffsll((long long)need) - 1;
                need &= need - 1;
                const int n = __builtin_amdgcn_readlane(cnt, jj);
                const float nt = compact_slot(cbuf + (wv * 32 + jj) * kStride, n, a.k, lane);
                if (j == jj) {
                    tau = nt;
                    cnt = a.k;
                }
            }
        }
        __syncthreads();
    }
    // final: this chunk's top-k of every user, sorted, to the workspace
    __builtin_amdgcn_wave_barrier();
    for (int jj = 0; jj < 32; ++jj) {
        const int64_t b2 = (int64_t)blockIdx.x * (32 * NW) + wv * 32 + jj;
        if (b2 >= a.nb) break;  // wave-uniform
        const int n = __builtin_amdgcn_readlane(cnt, jj);
        emit_sorted(cbuf + (wv * 32 + jj) * kStride, n, a.k, lane, a.cand + ((b2 * a.n_chunks) + chunk) * a.k);
    }
}

// 16 lanes per user: k-way merge of n_chunks sorted lists (n_chunks <= 16).
__global__ __launch_bounds__(256) void fs_merge(FsArgs a) {
    const int li = threadIdx.x & 15;
    const int64_t b = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
    if (b >= a.nb) return;
    const u64* src = a.cand + b * a.n_chunks * a.k + (int64_t)li * a.k;
    const bool has = li < a.n_chunks;
    int ptr = 0;
    u64 head = has ? src[0] : 0ull;
    for (int o = 0; o < a.k; ++o) {
        u64 m = head;
#pragma unroll
        for (int s = 8; s > 0; s >>= 1) {
            const u64 pv = shfl_xor_u64(m, s);
            m = m > pv ? m : pv;
        }
        if (has && head == m && m != 0ull) {
            ++ptr;
            head = ptr < a.k ? src[ptr] : 0ull;
        }
        if (li == 0) {
            a.out_val[b * a.k + o] = m ? key_score(m) : -INFINITY;
            a.out_idx[b * a.k + o] = m ? (int64_t)key_index(m) : -1;
        }
    }
}

static void fs_plan(int64_t nb, int64_t ni, int d, int* nw, int* n_chunks, int64_t* chunk_items) {
    *nw = d <= 64 ? 4 : 2;
    const int64_t ublocks = (nb + 32 * (*nw) - 1) / (32 * (*nw));
    int64_t s = (256 + ublocks - 1) / ublocks;  // about one block per CU
    if (s < 1) s = 1;
    if (s > 16) s = 16;
    int64_t per = (ni + s - 1) / s;
    per = (per + 31) / 32 * 32;
    if (per < 32) per = 32;
    *chunk_items = per;
    *n_chunks = (int)((ni + per - 1) / per);
}

size_t fs_ws(int64_t nb, int64_t ni, int k, int d) {
    int nw, nc;
    int64_t per;
    fs_plan(nb, ni, d, &nw, &nc, &per);
    return (size_t)nb * nc * k * sizeof(u64) + 256;
}

template <int D, int NW>
static int launch_fs(FsArgs& a, hipStream_t s) {
    const size_t lds = 2 * 32 * (D + 4) * sizeof(float) + NW * 32 * kStride * sizeof(u64);
    const int64_t ublocks = (a.nb + 32 * NW - 1) / (32 * NW);
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)fs_tiles<D, NW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr_set = true;
    }
    hipLaunchKernelGGL((fs_tiles<D, NW>), dim3((unsigned)ublocks, (unsigned)a.n_chunks), dim3(64 * NW), lds, s,
                       a);
    hipLaunchKernelGGL(fs_merge, dim3((unsigned)((a.nb + 15) / 16)), dim3(256), 0, s, a);
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
    int nw;
    fs_plan(nb, ni, d, &nw, &a.n_chunks, &a.chunk_items);
    a.U = U;
    a.users = users;
    a.nb = nb;
    a.I = I;
    a.ni = ni;
    a.mrp = mrp;
    a.mcol = mcol;
    a.k = k;
    a.cand = static_cast<u64*>(ws);
    a.out_val = out_val;
    a.out_idx = out_idx;
    switch (d) {
        case 32: return launch_fs<32, 4>(a, s);
        case 64: return launch_fs<64, 4>(a, s);
        case 128: return launch_fs<128, 2>(a, s);
        case 256: return launch_fs<256, 2>(a, s);
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
    // worst case over d (the plan depends on d only through NW)
    size_t a = rsx::fs_ws(n_batch, n_items, k, 64), b = rsx::fs_ws(n_batch, n_items, k, 128);
    return a > b ? a : b;
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

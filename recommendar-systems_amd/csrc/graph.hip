// graph.hip — the normalised user-item adjacencies built on the device (gfx950).
//
// Replaces the reference's Python dok loops (hours and >100 GB of RAM at the C4
// graph's 10^8 edges):
//  * LightGCN.get_norm_adj_mat (src/models/lightgcn.py:65-103; LayerGCN's eval graph,
//    src/models/layergcn.py:91-117): binary symmetric A = [[0, R], [R^T, 0]] with
//    duplicate interactions collapsed, d_v = deg_v + 1e-7 and d_r^-1/2 d_c^-1/2 in
//    float64, cast to float32;
//  * SMORE.get_adj_mat (src/models/smore.py:176-207): float32 degrees, ^-1/2 with
//    inf -> 0 (no epsilon), d_r * 1 * d_c in float32;
//  * LayerGCN's per-epoch edge-dropout graph (src/models/layergcn.py:51-81): float32
//    1/sqrt(1e-7 + kept degree) products of the kept edges, compacted from the
//    symmetric template.
// Output: CSR (rowptr int64, col int32, val f32), columns sorted inside each row —
// the layout rsx/graph.py's host builders produce (tests compare them bit for bit).
//
// Build: keys u<<32|i radix-sorted and de-duplicated (hipCUB), integer degrees by
// atomics (exact in any order), rowptr by an exclusive scan; the user rows are the
// unique keys in order; the item rows are the keys i<<32|u radix-sorted.  x^-1/2 comes
// from the caller's table of the host pow's values per degree (numpy's, as the
// reference), with the device's float64 pow only beyond the table.
#include <hipcub/hipcub.hpp>

#include "rsx_common.hpp"

#define RSX_TRY_HIP(x)                                  \
    do {                                                \
        const hipError_t e_ = (x);                      \
        if (e_ != hipSuccess) return rsx::hip_rc(e_);   \
    } while (0)

namespace rsx {
namespace gb {

__global__ __launch_bounds__(256) void make_keys(const int64_t* u, const int64_t* i, int64_t E, uint64_t* keys) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e < E) keys[e] = ((uint64_t)u[e] << 32) | (uint64_t)(uint32_t)i[e];
}

__global__ __launch_bounds__(256) void degrees(const uint64_t* uk, const int64_t* n_unique, int64_t cap,
                                               int64_t nu, int64_t* deg) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= cap || j >= *n_unique) return;
    const uint64_t k = uk[j];
    atomicAdd(reinterpret_cast<unsigned long long*>(deg + (k >> 32)), 1ull);
    atomicAdd(reinterpret_cast<unsigned long long*>(deg + nu + (k & 0xFFFFFFFFull)), 1ull);
}

// d^-1/2 per node: mode 0 float64 (deg + 1e-7), mode 1 float32 (inf -> 0), stored as double;
// from the caller's host-computed table where the degree is in it (bit-equal to the
// reference's numpy pow by construction), else the device's float64 pow
__global__ __launch_bounds__(256) void dinv_k(const int64_t* deg, int64_t n, int mode, const double* table,
                                              int64_t table_len, double* dinv) {
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (v >= n) return;
    if (table && deg[v] < table_len) {
        dinv[v] = table[deg[v]];
    } else if (mode == 0) {
        dinv[v] = pow((double)deg[v] + 1e-7, -0.5);
    } else {
        const float x = (float)deg[v];
        const float d = x == 0.f ? INFINITY : (float)pow((double)x, -0.5);
        dinv[v] = isinf(d) ? 0.0 : (double)d;
    }
}

__device__ __forceinline__ float edge_val(const double* dinv, int64_t r, int64_t c, int mode) {
    if (mode == 0) return (float)(dinv[r] * dinv[c]);
    return ((float)dinv[r] * 1.f) * (float)dinv[c];
}

// user rows: entry j = unique key j; item keys for the second sort (pad: all ones)
__global__ __launch_bounds__(256) void user_rows(const uint64_t* uk, const int64_t* n_unique, int64_t cap,
                                                 int64_t nu, const double* dinv, int mode, int32_t* col, float* val,
                                                 uint64_t* ikeys) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= cap) return;
    if (j >= *n_unique) {
        ikeys[j] = ~0ull;
        return;
    }
    const uint64_t k = uk[j];
    const int64_t u = (int64_t)(k >> 32), i = (int64_t)(k & 0xFFFFFFFFull);
    col[j] = (int32_t)(nu + i);
    val[j] = edge_val(dinv, u, nu + i, mode);
    ikeys[j] = ((uint64_t)i << 32) | (uint64_t)u;
}

__global__ __launch_bounds__(256) void item_rows(const uint64_t* ik, const int64_t* n_unique, int64_t cap,
                                                 int64_t nu, const double* dinv, int mode, int32_t* col, float* val) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t U = *n_unique;
    if (j >= cap || j >= U) return;
    const uint64_t k = ik[j];
    const int64_t i = (int64_t)(k >> 32), u = (int64_t)(k & 0xFFFFFFFFull);
    col[U + j] = (int32_t)u;
    val[U + j] = edge_val(dinv, nu + i, u, mode);
}

// ---- edge dropout ----------------------------------------------------------------
__global__ __launch_bounds__(256) void kept_degrees(const int64_t* u, const int64_t* i, const uint8_t* keep,
                                                    int64_t E, int64_t nu, int32_t* cnt) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= E || !keep[e]) return;
    atomicAdd(cnt + u[e], 1);
    atomicAdd(cnt + nu + i[e], 1);
}

// float32 1/sqrt(1e-7 + kept degree) (the reference's _normalize_adj_m, layergcn.py:72-81)
__global__ __launch_bounds__(256) void kept_inv(const int32_t* cnt, int64_t n, float* inv) {
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (v < n) inv[v] = 1.f / sqrtf(1e-7f + (float)cnt[v]);
}

__global__ __launch_bounds__(256) void template_flags(const int64_t* t_eid, const uint8_t* keep, int64_t T,
                                                      int64_t* flags) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t < T) flags[t] = keep[t_eid[t]] ? 1 : 0;
    if (t == T) flags[t] = 0;
}

__global__ __launch_bounds__(256) void compact(const int64_t* t_rowptr, int64_t n, const int32_t* t_col,
                                               const int64_t* t_eid, const uint8_t* keep, const int64_t* pos,
                                               int64_t T, const int64_t* e_u, const int64_t* e_i, int64_t nu,
                                               const float* inv, int64_t* rowptr, int32_t* col, float* val) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t <= n) rowptr[t] = pos[t_rowptr[t]];
    if (t >= T) return;
    const int64_t e = t_eid[t];
    if (!keep[e]) return;
    const int64_t p = pos[t];
    col[p] = t_col[t];
    val[p] = inv[e_u[e]] * inv[nu + e_i[e]];
}

inline unsigned blocks(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace gb
}  // namespace rsx

using namespace rsx;

namespace {

struct AdjWs {
    uint64_t *k0, *k1, *k2;
    int64_t *deg, *n_unique;
    double* dinv;
    void* temp;
    size_t temp_bytes;
};

size_t temp_need(int64_t E, int64_t n) {
    size_t a = 0, b = 0, c = 0;
    (void)hipcub::DeviceRadixSort::SortKeys(nullptr, a, (uint64_t*)nullptr, (uint64_t*)nullptr, (int)E);
    (void)hipcub::DeviceSelect::Unique(nullptr, b, (uint64_t*)nullptr, (uint64_t*)nullptr, (int64_t*)nullptr, (int)E);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, (int64_t*)nullptr, (int64_t*)nullptr, (int)(n + 1));
    return std::max(a, std::max(b, c));
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t adj_layout(int64_t E, int64_t n, AdjWs* w, void* base) {
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* p = base ? static_cast<char*>(base) + off : nullptr;
        off += align256(bytes);
        return p;
    };
    const size_t tb = temp_need(E, n);
    AdjWs x;
    x.k0 = (uint64_t*)take((size_t)E * 8);
    x.k1 = (uint64_t*)take((size_t)E * 8);
    x.k2 = (uint64_t*)take((size_t)E * 8);
    x.deg = (int64_t*)take((size_t)(n + 1) * 8);
    x.n_unique = (int64_t*)take(8);
    x.dinv = (double*)take((size_t)n * 8);
    x.temp = take(tb);
    x.temp_bytes = tb;
    if (w) *w = x;
    return off;
}

}  // namespace

extern "C" {

size_t rsx_adj_build_ws_bytes(int64_t n_edges, int64_t n_users, int64_t n_items) {
    if (n_edges < 1) n_edges = 1;
    return adj_layout(n_edges, n_users + n_items, nullptr, nullptr);
}

int rsx_adj_build(const int64_t* u, const int64_t* i, int64_t n_edges, int64_t n_users, int64_t n_items,
                  int32_t mode, const double* dinv_table, int64_t table_len, int64_t* rowptr, int32_t* col,
                  float* val, void* ws, size_t ws_bytes, rsx_stream_t stream) {
    if (n_edges < 0 || (n_edges > 0 && (!u || !i || !col || !val)) || n_users < 0 || n_items < 0 ||
        (mode != 0 && mode != 1) || !rowptr || table_len < 0 || (table_len > 0 && !dinv_table))
        return RSX_ERR_ARG;
    if (n_users >= (int64_t(1) << 31) || n_items >= (int64_t(1) << 31) || 2 * n_edges >= (int64_t(1) << 31) ||
        n_edges >= INT32_MAX)
        return RSX_ERR_ARG;
    const int64_t n = n_users + n_items, E = n_edges > 0 ? n_edges : 1;
    if (!ws || ws_bytes < rsx_adj_build_ws_bytes(n_edges, n_users, n_items)) return RSX_ERR_WORKSPACE;
    hipStream_t s = as_stream(stream);
    AdjWs w;
    adj_layout(E, n, &w, ws);
    RSX_TRY_HIP(hipMemsetAsync(w.deg, 0, (size_t)(n + 1) * 8, s));
    if (n_edges == 0) {
        RSX_TRY_HIP(hipMemsetAsync(rowptr, 0, (size_t)(n + 1) * 8, s));
        return RSX_OK;
    }
    hipLaunchKernelGGL(gb::make_keys, dim3(gb::blocks(E)), dim3(256), 0, s, u, i, E, w.k0);
    size_t tb = w.temp_bytes;
    if (hipcub::DeviceRadixSort::SortKeys(w.temp, tb, w.k0, w.k1, (int)E, 0, 64, s) != hipSuccess) return last_rc();
    tb = w.temp_bytes;
    if (hipcub::DeviceSelect::Unique(w.temp, tb, w.k1, w.k0, w.n_unique, (int)E, s) != hipSuccess) return last_rc();
    hipLaunchKernelGGL(gb::degrees, dim3(gb::blocks(E)), dim3(256), 0, s, w.k0, w.n_unique, E, n_users, w.deg);
    tb = w.temp_bytes;
    if (hipcub::DeviceScan::ExclusiveSum(w.temp, tb, w.deg, rowptr, (int)(n + 1), s) != hipSuccess) return last_rc();
    hipLaunchKernelGGL(gb::dinv_k, dim3(gb::blocks(n)), dim3(256), 0, s, w.deg, n, mode,
                       table_len > 0 ? dinv_table : nullptr, table_len, w.dinv);
    hipLaunchKernelGGL(gb::user_rows, dim3(gb::blocks(E)), dim3(256), 0, s, w.k0, w.n_unique, E, n_users, w.dinv,
                       mode, col, val, w.k2);
    tb = w.temp_bytes;
    if (hipcub::DeviceRadixSort::SortKeys(w.temp, tb, w.k2, w.k1, (int)E, 0, 64, s) != hipSuccess) return last_rc();
    hipLaunchKernelGGL(gb::item_rows, dim3(gb::blocks(E)), dim3(256), 0, s, w.k1, w.n_unique, E, n_users, w.dinv,
                       mode, col, val);
    return last_rc();
}

size_t rsx_edge_dropout_ws_bytes(int64_t n_edges, int64_t n_users, int64_t n_items) {
    const int64_t n = n_users + n_items, T = 2 * (n_edges > 0 ? n_edges : 1);
    size_t c = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, (int64_t*)nullptr, (int64_t*)nullptr, (int)(T + 1));
    return align256((size_t)n * 4) + align256((size_t)n * 4) + 2 * align256((size_t)(T + 1) * 8) + align256(c);
}

int rsx_edge_dropout_build(const int64_t* e_u, const int64_t* e_i, const uint8_t* keep, int64_t n_edges,
                           int64_t n_users, int64_t n_items, const int64_t* t_rowptr, const int32_t* t_col,
                           const int64_t* t_eid, int64_t* rowptr, int32_t* col, float* val, void* ws,
                           size_t ws_bytes, rsx_stream_t stream) {
    if (!e_u || !e_i || !keep || n_edges < 0 || !t_rowptr || !t_col || !t_eid || !rowptr || !col || !val)
        return RSX_ERR_ARG;
    if (2 * n_edges >= (int64_t(1) << 31)) return RSX_ERR_ARG;
    if (!ws || ws_bytes < rsx_edge_dropout_ws_bytes(n_edges, n_users, n_items)) return RSX_ERR_WORKSPACE;
    const int64_t n = n_users + n_items, T = 2 * n_edges;
    hipStream_t s = as_stream(stream);
    char* p = static_cast<char*>(ws);
    int32_t* cnt = reinterpret_cast<int32_t*>(p);
    p += align256((size_t)n * 4);
    float* inv = reinterpret_cast<float*>(p);
    p += align256((size_t)n * 4);
    int64_t* flags = reinterpret_cast<int64_t*>(p);
    p += align256((size_t)(T + 1) * 8);
    int64_t* pos = reinterpret_cast<int64_t*>(p);
    p += align256((size_t)(T + 1) * 8);
    size_t tb = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (int64_t*)nullptr, (int64_t*)nullptr, (int)(T + 1));
    RSX_TRY_HIP(hipMemsetAsync(cnt, 0, (size_t)n * 4, s));
    if (n_edges > 0)
        hipLaunchKernelGGL(gb::kept_degrees, dim3(gb::blocks(n_edges)), dim3(256), 0, s, e_u, e_i, keep, n_edges,
                           n_users, cnt);
    hipLaunchKernelGGL(gb::kept_inv, dim3(gb::blocks(n)), dim3(256), 0, s, cnt, n, inv);
    hipLaunchKernelGGL(gb::template_flags, dim3(gb::blocks(T + 1)), dim3(256), 0, s, t_eid, keep, T, flags);
    if (hipcub::DeviceScan::ExclusiveSum(p, tb, flags, pos, (int)(T + 1), s) != hipSuccess) return last_rc();
    hipLaunchKernelGGL(gb::compact, dim3(gb::blocks(std::max(T, n + 1))), dim3(256), 0, s, t_rowptr, n, t_col, t_eid,
                       keep, pos, T, e_u, e_i, n_users, inv, rowptr, col, val);
    return last_rc();
}

}  // extern "C"

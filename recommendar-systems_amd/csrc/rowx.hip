// rowx.hip — the batch-row gradient exchange of data-parallel SMORE (gfx950).
//
// Data-parallel SMORE (rsx.smore, scheme "dp") keeps every table
// replicated and gives each rank its own batch; the objective is the sum over ranks of
// the reference loss of each rank's batch (src/models/smore.py:366-411).  Every path
// from a rank's loss to the parameters runs through the preference block on the batch
// rows (smore.py:320-341), whose backward leaves four [N, d] table gradients (content,
// image, text, fusion views) defined on the rank's batch rows only.  Those rows are the
// exchange: each rank packs its rows (one entry per occurrence, a flag on the first
// occurrence of each row), one all-gather of the packed entries, then every rank
// rebuilds the same four tables on the union of the ranks' rows -- zero the union rows,
// then add rank 0's rows, rank 1's, ... in rank order (within one rank a row is added
// once, so no float atomics and no race) -- and runs the rest of the backward (UI
// backbone, views, item side) on identical inputs: identical gradients, replicas that
// stay bit-identical under the per-element Adam.  The union row list is written out for
// the tag-aware consumers (the batch-row tags of the backbone and the views).
//
// The work is HBM-bound byte movement: per occurrence 16 + 4 T d bytes packed (T = 4
// tables), gathered W-fold, then read once and added into the tables.
#include "rsx_common.hpp"

namespace rsx {
namespace rowx {

constexpr int kHead = 4;  // header floats of an entry: row (two words), first flag, pad

__global__ void bump_tag(int32_t* tag_dev) { tag_dev[0] += 1; }

// lead[rows[j]] = max over j of (tag << 32 | ~j): the smallest occurrence index of each
// row under this call's tag (earlier calls' keys carry a smaller tag)
__global__ __launch_bounds__(256) void lead_k(const int64_t* __restrict__ rows, int64_t n,
                                              unsigned long long* __restrict__ lead,
                                              const int32_t* __restrict__ tag_dev) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const unsigned long long key =
        ((unsigned long long)(uint32_t)tag_dev[0] << 32) | (unsigned long long)(0xffffffffu - (uint32_t)j);
    atomicMax(lead + rows[j], key);
}

struct Tables {
    float* t[8];
};

// one thread per float4 of an entry: float4 0 = header, then the T tables' rows
__global__ __launch_bounds__(256) void pack_k(const int64_t* __restrict__ rows, int64_t n, int64_t n_max, Tables tb,
                                              int32_t T, int32_t d, const unsigned long long* __restrict__ lead,
                                              const int32_t* __restrict__ tag_dev, float* __restrict__ packed) {
    const int64_t q4 = 1 + (int64_t)T * (d / 4);  // float4s per entry
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= n_max * q4) return;
    const int64_t j = g / q4;
    const int64_t q = g - j * q4;
    const bool real = j < n;
    const int64_t row = rows[real ? j : 0];  // a padding entry names a real row, flag 0
    float* e = packed + j * (kHead + (int64_t)T * d);
    if (q == 0) {
        bool first = false;
        if (real) {
            const unsigned long long key =
                ((unsigned long long)(uint32_t)tag_dev[0] << 32) | (unsigned long long)(0xffffffffu - (uint32_t)j);
            first = lead[row] == key;
        }
        const uint64_t r = (uint64_t)row;
        st4(e, make_float4(__uint_as_float((uint32_t)r), __uint_as_float((uint32_t)(r >> 32)), first ? 1.f : 0.f,
                           0.f));
        return;
    }
    const int64_t c = q - 1;
    const int t = (int)(c / (d / 4));
    const int64_t col = (c - (int64_t)t * (d / 4)) * 4;
    st4(e + kHead + (int64_t)t * d + col, real ? ld4(tb.t[t] + row * d + col) : f4(0.f));
}

__device__ __forceinline__ int64_t head_row(const float* e) {
    return (int64_t)((uint64_t)__float_as_uint(e[0]) | ((uint64_t)__float_as_uint(e[1]) << 32));
}

// every entry of every rank: union_rows[e] = its row; the row zeroed in each table
__global__ __launch_bounds__(256) void zero_k(const float* __restrict__ packed, int64_t n_all, Tables tb, int32_t T,
                                              int32_t d, int64_t* __restrict__ union_rows) {
    const int64_t q4 = 1 + (int64_t)T * (d / 4);
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= n_all * q4) return;
    const int64_t j = g / q4;
    const int64_t q = g - j * q4;
    const float* e = packed + j * (kHead + (int64_t)T * d);
    const int64_t row = head_row(e);
    if (q == 0) {
        union_rows[j] = row;
        return;
    }
    const int64_t c = q - 1;
    const int t = (int)(c / (d / 4));
    const int64_t col = (c - (int64_t)t * (d / 4)) * 4;
    st4(tb.t[t] + row * d + col, f4(0.f));
}

// one rank's entries: the first occurrence of each of its rows added into the tables
__global__ __launch_bounds__(256) void add_k(const float* __restrict__ packed, int64_t n_max, Tables tb, int32_t T,
                                             int32_t d) {
    const int64_t q4 = (int64_t)T * (d / 4);
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= n_max * q4) return;
    const int64_t j = g / q4;
    const int64_t c = g - j * q4;
    const float* e = packed + j * (kHead + (int64_t)T * d);
    if (e[2] == 0.f) return;
    const int64_t row = head_row(e);
    const int t = (int)(c / (d / 4));
    const int64_t col = (c - (int64_t)t * (d / 4)) * 4;
    float* dst = tb.t[t] + row * d + col;
    st4(dst, add4(ld4(dst), ld4(e + kHead + (int64_t)t * d + col)));
}

inline bool tables_ok(const float* const* tables, int32_t T, int32_t d) {
    if (!tables || T < 1 || T > 8 || d <= 0 || d % 4) return false;
    for (int t = 0; t < T; ++t)
        if (!tables[t]) return false;
    return true;
}

}  // namespace rowx
}  // namespace rsx

using namespace rsx;

size_t rsx_rowx_entry_floats(int32_t n_tables, int32_t d) { return (size_t)rowx::kHead + (size_t)n_tables * d; }

int rsx_rowx_pack(const int64_t* rows, int64_t n, int64_t n_max, const float* const* tables, int32_t n_tables,
                  int32_t d, uint64_t* lead, int32_t* tag_dev, float* packed, rsx_stream_t stream) {
    if (!rows || n < 1 || n_max < n || !lead || !tag_dev || !packed || !rowx::tables_ok(tables, n_tables, d))
        return RSX_ERR_ARG;
    hipStream_t s = as_stream(stream);
    rowx::Tables tb{};
    for (int t = 0; t < n_tables; ++t) tb.t[t] = const_cast<float*>(tables[t]);
    hipLaunchKernelGGL(rowx::bump_tag, dim3(1), dim3(1), 0, s, tag_dev);
    hipLaunchKernelGGL(rowx::lead_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, rows, n,
                       reinterpret_cast<unsigned long long*>(lead), tag_dev);
    const int64_t work = n_max * (1 + (int64_t)n_tables * (d / 4));
    hipLaunchKernelGGL(rowx::pack_k, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s, rows, n, n_max, tb,
                       n_tables, d, reinterpret_cast<const unsigned long long*>(lead), tag_dev, packed);
    return last_rc();
}

int rsx_rowx_combine(const float* packed, int32_t world, int64_t n_max, float* const* tables, int32_t n_tables,
                     int32_t d, int64_t* union_rows, rsx_stream_t stream) {
    if (!packed || world < 1 || n_max < 1 || !union_rows || !rowx::tables_ok(tables, n_tables, d))
        return RSX_ERR_ARG;
    hipStream_t s = as_stream(stream);
    rowx::Tables tb{};
    for (int t = 0; t < n_tables; ++t) tb.t[t] = tables[t];
    const int64_t n_all = (int64_t)world * n_max;
    const int64_t zw = n_all * (1 + (int64_t)n_tables * (d / 4));
    hipLaunchKernelGGL(rowx::zero_k, dim3((unsigned)((zw + 255) / 256)), dim3(256), 0, s, packed, n_all, tb, n_tables,
                       d, union_rows);
    const int64_t aw = n_max * (int64_t)n_tables * (d / 4);
    const int64_t stride = n_max * (int64_t)rsx_rowx_entry_floats(n_tables, d);
    for (int r = 0; r < world; ++r)  // rank order: the same float sums on every rank
        hipLaunchKernelGGL(rowx::add_k, dim3((unsigned)((aw + 255) / 256)), dim3(256), 0, s, packed + r * stride,
                           n_max, tb, n_tables, d);
    return last_rc();
}

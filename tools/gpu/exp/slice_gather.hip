// Experiment (round 6): does an XCD-sliced table layout make the C2 SpMM's neighbour
// gathers L2-resident?  A sports-shaped random bipartite graph (35,598 users x 18,357
// items, 214,654 interactions, power-law item popularity), its symmetric normalised
// adjacency, d = 64 f32.
//   row    : the production layout, 16 lanes x float4 per row (256 B), one row per group
//   slice  : the table as 8 column slices [8][N][8] (32 B a row-slice); block b works on
//            slice b % 8 (blocks b, b + 8 share an XCD: one XCD gathers from one 1.7 MB
//            slice, which fits its 4 MiB L2); a 16-lane group = one row, 8 lane pairs
//            each gathering every 8th neighbour, reduced across pairs at the end
//   slice_x: the same kernel with slice = b / (blocks per slice) (no XCD affinity)
// Prints us per product and the max |difference| of the two results.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 fma4(float a, float4 x, float4 y) {
    return make_float4(fmaf(a, x.x, y.x), fmaf(a, x.y, y.y), fmaf(a, x.z, y.z), fmaf(a, x.w, y.w));
}

__global__ __launch_bounds__(256) void k_row(const int64_t* rp, const int* col, const float* val, const float* x,
                                             float* y, int n) {
    const int li = threadIdx.x & 15;
    const int r = blockIdx.x * 16 + (threadIdx.x >> 4);
    if (r >= n) return;
    const int b = (int)rp[r], e = (int)rp[r + 1];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int j = b; j < e; j += 16) {
        const bool mine = j + li < e;
        const int cm = mine ? col[j + li] : 0;
        const float vm = mine ? val[j + li] : 0.f;
        const int m = min(16, e - j);
        float4 xv[16];
        float vv[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int c = __shfl(cm, t, 16);
            vv[t] = __shfl(vm, t, 16);
            xv[t] = t < m ? ld4(x + (int64_t)c * 64 + li * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int t = 0; t < 16; ++t)
            if (t < m) acc = fma4(vv[t], xv[t], acc);
    }
    *reinterpret_cast<float4*>(y + (int64_t)r * 64 + li * 4) = acc;
}

template <bool AFFINE>
__global__ __launch_bounds__(256) void k_slice(const int64_t* rp, const int* col, const float* val, const float* xs,
                                               float* ys, int n, int nrb) {
    const int s = AFFINE ? (blockIdx.x & 7) : (blockIdx.x / nrb);
    const int rb = AFFINE ? (blockIdx.x >> 3) : (blockIdx.x % nrb);
    const int li = threadIdx.x & 15, pr = li >> 1, h = li & 1;
    const int r = rb * 16 + (threadIdx.x >> 4);
    if (r >= n) return;
    const float* xb = xs + (int64_t)s * n * 8 + h * 4;
    const int b = (int)rp[r], e = (int)rp[r + 1];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int j = b; j < e; j += 16) {
        const bool mine = j + li < e;
        const int cm = mine ? col[j + li] : 0;
        const float vm = mine ? val[j + li] : 0.f;
        const int c0 = __shfl(cm, pr, 16), c1 = __shfl(cm, pr + 8, 16);
        const float v0 = __shfl(vm, pr, 16), v1 = __shfl(vm, pr + 8, 16);
        const float4 x0 = j + pr < e ? ld4(xb + (int64_t)c0 * 8) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 x1 = j + pr + 8 < e ? ld4(xb + (int64_t)c1 * 8) : make_float4(0.f, 0.f, 0.f, 0.f);
        acc = fma4(v0, x0, acc);
        acc = fma4(v1, x1, acc);
    }
#pragma unroll
    for (int m = 2; m <= 8; m <<= 1) {
        acc.x += __shfl_xor(acc.x, m, 16);
        acc.y += __shfl_xor(acc.y, m, 16);
        acc.z += __shfl_xor(acc.z, m, 16);
        acc.w += __shfl_xor(acc.w, m, 16);
    }
    if (pr == 0) *reinterpret_cast<float4*>(ys + (int64_t)s * n * 8 + (int64_t)r * 8 + h * 4) = acc;
}

// nnz-balanced forms: work items {row, begin, end} of <= 32 nonzeros (hub rows split),
// one item per 16-lane group, each item's partial written to its own output row (no
// fixup: this measures the gathers, not the combine)
__global__ __launch_bounds__(256) void k_row_items(const int4* it, int nit, const int* col, const float* val,
                                                   const float* x, float* y) {
    const int li = threadIdx.x & 15;
    const int w = blockIdx.x * 16 + (threadIdx.x >> 4);
    if (w >= nit) return;
    const int4 wk = it[w];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int j = wk.y; j < wk.z; j += 16) {
        const bool mine = j + li < wk.z;
        const int cm = mine ? col[j + li] : 0;
        const float vm = mine ? val[j + li] : 0.f;
        const int m = min(16, wk.z - j);
        float4 xv[16];
        float vv[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int c = __shfl(cm, t, 16);
            vv[t] = __shfl(vm, t, 16);
            xv[t] = t < m ? ld4(x + (int64_t)c * 64 + li * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int t = 0; t < 16; ++t)
            if (t < m) acc = fma4(vv[t], xv[t], acc);
    }
    *reinterpret_cast<float4*>(y + (int64_t)w * 64 + li * 4) = acc;
}

template <bool AFFINE>
__global__ __launch_bounds__(256) void k_slice_items(const int4* it, int nit, const int* col, const float* val,
                                                     const float* xs, float* ys, int n, int nrb) {
    const int s = AFFINE ? (blockIdx.x & 7) : (blockIdx.x / nrb);
    const int rb = AFFINE ? (blockIdx.x >> 3) : (blockIdx.x % nrb);
    const int li = threadIdx.x & 15, pr = li >> 1, h = li & 1;
    const int w = rb * 16 + (threadIdx.x >> 4);
    if (w >= nit) return;
    const int4 wk = it[w];
    const float* xb = xs + (int64_t)s * n * 8 + h * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int j = wk.y; j < wk.z; j += 16) {
        const bool mine = j + li < wk.z;
        const int cm = mine ? col[j + li] : 0;
        const float vm = mine ? val[j + li] : 0.f;
        const int c0 = __shfl(cm, pr, 16), c1 = __shfl(cm, pr + 8, 16);
        const float v0 = __shfl(vm, pr, 16), v1 = __shfl(vm, pr + 8, 16);
        const float4 x0 = j + pr < wk.z ? ld4(xb + (int64_t)c0 * 8) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 x1 = j + pr + 8 < wk.z ? ld4(xb + (int64_t)c1 * 8) : make_float4(0.f, 0.f, 0.f, 0.f);
        acc = fma4(v0, x0, acc);
        acc = fma4(v1, x1, acc);
    }
#pragma unroll
    for (int m = 2; m <= 8; m <<= 1) {
        acc.x += __shfl_xor(acc.x, m, 16);
        acc.y += __shfl_xor(acc.y, m, 16);
        acc.z += __shfl_xor(acc.z, m, 16);
        acc.w += __shfl_xor(acc.w, m, 16);
    }
    if (pr == 0) *reinterpret_cast<float4*>(ys + (int64_t)s * nit * 8 + (int64_t)w * 8 + h * 4) = acc;
}

int main() {
    const int U = 35598, I = 18357, E = 214654, N = U + I, D = 64;
    std::mt19937_64 rng(7);
    // item popularity ~ 1 / (rank + 20)^0.9, users >= 1 interaction each
    std::vector<double> w(I);
    for (int i = 0; i < I; ++i) w[i] = 1.0 / std::pow(i + 20.0, 0.9);
    std::discrete_distribution<int> pick_item(w.begin(), w.end());
    std::vector<std::pair<int, int>> ed;
    ed.reserve(E * 2);
    for (int u = 0; u < U; ++u) ed.push_back({u, pick_item(rng)});
    std::uniform_int_distribution<int> pick_user(0, U - 1);
    while ((int)ed.size() < E * 11 / 10) ed.push_back({pick_user(rng), pick_item(rng)});
    std::sort(ed.begin(), ed.end());
    ed.erase(std::unique(ed.begin(), ed.end()), ed.end());
    if ((int)ed.size() > E) ed.resize(E);
    std::vector<int> deg(N, 0);
    for (auto& p : ed) ++deg[p.first], ++deg[U + p.second];
    std::vector<std::vector<int>> adj(N);
    for (auto& p : ed) adj[p.first].push_back(U + p.second), adj[U + p.second].push_back(p.first);
    std::vector<int64_t> rp(N + 1, 0);
    std::vector<int> col;
    std::vector<float> val;
    for (int r = 0; r < N; ++r) {
        std::shuffle(adj[r].begin(), adj[r].end(), rng);
        for (int c : adj[r]) col.push_back(c), val.push_back((float)(1.0 / std::sqrt((double)deg[r] * deg[c])));
        rp[r + 1] = (int64_t)col.size();
    }
    const int64_t nnz = (int64_t)col.size();
    int maxd = 0;
    for (int r = 0; r < N; ++r) maxd = std::max(maxd, deg[r]);
    printf("graph: %d rows, %ld nnz, max degree %d\n", N, (long)nnz, maxd);
    std::vector<float> x((size_t)N * D), xs((size_t)N * D);
    std::normal_distribution<float> nd(0.f, 1.f);
    for (auto& v : x) v = nd(rng);
    for (int r = 0; r < N; ++r)
        for (int c = 0; c < D; ++c) xs[(size_t)(c / 8) * N * 8 + (size_t)r * 8 + c % 8] = x[(size_t)r * D + c];
    int64_t* d_rp;
    int* d_col;
    float *d_val, *d_x, *d_xs, *d_y, *d_ys;
    CK(hipMalloc(&d_rp, (N + 1) * 8));
    CK(hipMalloc(&d_col, nnz * 4));
    CK(hipMalloc(&d_val, nnz * 4));
    CK(hipMalloc(&d_x, (size_t)N * D * 4));
    CK(hipMalloc(&d_xs, (size_t)N * D * 4));
    CK(hipMalloc(&d_y, (size_t)N * D * 4));
    CK(hipMalloc(&d_ys, (size_t)N * D * 4));
    CK(hipMemcpy(d_rp, rp.data(), (N + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_col, col.data(), nnz * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_val, val.data(), nnz * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_x, x.data(), (size_t)N * D * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_xs, xs.data(), (size_t)N * D * 4, hipMemcpyHostToDevice));
    const int nrb = (N + 15) / 16;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time = [&](const char* name, auto launch) {
        for (int i = 0; i < 20; ++i) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        const int reps = 200;
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-8s %8.2f us\n", name, 1e3 * ms / reps);
    };
    for (int rep = 0; rep < 2; ++rep) {
        time("row", [&] { hipLaunchKernelGGL(k_row, dim3(nrb), dim3(256), 0, 0, d_rp, d_col, d_val, d_x, d_y, N); });
        time("slice", [&] {
            hipLaunchKernelGGL(k_slice<true>, dim3(8 * nrb), dim3(256), 0, 0, d_rp, d_col, d_val, d_xs, d_ys, N, nrb);
        });
        time("slice_x", [&] {
            hipLaunchKernelGGL(k_slice<false>, dim3(8 * nrb), dim3(256), 0, 0, d_rp, d_col, d_val, d_xs, d_ys, N, nrb);
        });
    }
    // nnz-balanced items
    std::vector<int4> items;
    for (int r = 0; r < N; ++r)
        for (int64_t b = rp[r]; b < rp[r + 1] || b == rp[r]; b += 32) {
            const int64_t e = std::min<int64_t>(b + 32, rp[r + 1]);
            items.push_back(make_int4(r, (int)b, (int)e, 0));
            if (e >= rp[r + 1]) break;
        }
    const int nit = (int)items.size();
    int4* d_it;
    float *d_yi, *d_ysi;
    CK(hipMalloc(&d_it, (size_t)nit * 16));
    CK(hipMalloc(&d_yi, (size_t)nit * D * 4));
    CK(hipMalloc(&d_ysi, (size_t)nit * D * 4));
    CK(hipMemcpy(d_it, items.data(), (size_t)nit * 16, hipMemcpyHostToDevice));
    const int nib = (nit + 15) / 16;
    printf("items (<= 32 nonzeros): %d\n", nit);
    for (int rep = 0; rep < 2; ++rep) {
        time("row_it", [&] { hipLaunchKernelGGL(k_row_items, dim3(nib), dim3(256), 0, 0, d_it, nit, d_col, d_val, d_x, d_yi); });
        time("slice_it", [&] {
            hipLaunchKernelGGL(k_slice_items<true>, dim3(8 * nib), dim3(256), 0, 0, d_it, nit, d_col, d_val, d_xs, d_ysi, N, nib);
        });
        time("slicex_it", [&] {
            hipLaunchKernelGGL(k_slice_items<false>, dim3(8 * nib), dim3(256), 0, 0, d_it, nit, d_col, d_val, d_xs, d_ysi, N, nib);
        });
    }
    {
        std::vector<float> a((size_t)nit * D), b((size_t)nit * D);
        CK(hipMemcpy(a.data(), d_yi, (size_t)nit * D * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), d_ysi, (size_t)nit * D * 4, hipMemcpyDeviceToHost));
        double md = 0;
        for (int w = 0; w < nit; ++w)
            for (int c = 0; c < D; ++c)
                md = std::max(md, (double)std::fabs(a[(size_t)w * D + c] - b[(size_t)(c / 8) * nit * 8 + (size_t)w * 8 + c % 8]));
        printf("items: max |row - slice| = %.3g\n", md);
    }
    CK(hipGetLastError());
    std::vector<float> y((size_t)N * D), ys((size_t)N * D);
    CK(hipMemcpy(y.data(), d_y, (size_t)N * D * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ys.data(), d_ys, (size_t)N * D * 4, hipMemcpyDeviceToHost));
    double md = 0;
    for (int r = 0; r < N; ++r)
        for (int c = 0; c < D; ++c)
            md = std::max(md, (double)std::fabs(y[(size_t)r * D + c] - ys[(size_t)(c / 8) * N * 8 + (size_t)r * 8 + c % 8]));
    printf("max |row - slice| = %.3g\n", md);
    return 0;
}

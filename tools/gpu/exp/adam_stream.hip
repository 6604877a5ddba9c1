// Micro: how fast can the dense Adam pass stream on MI355X at the sports size?
// variants: (0) one 16-lane group per row (rsx rowwise layout), (1) flat float4 per
// thread, grid-stride, (2) flat, 4 float4 per thread per iteration (loads first).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

struct AdamC { float lr, omb1, b2, omb2, eps, step_size, bc2_sqrt; };

__device__ __forceinline__ void adam4(const AdamC& c, float4& p, float4& m, float4& v, float4 g) {
#define E(x) { m.x = m.x + c.omb1 * (g.x - m.x); v.x = v.x * c.b2 + (c.omb2 * g.x) * g.x; \
    const float den = sqrtf(v.x) / c.bc2_sqrt + c.eps; p.x = p.x + (-c.step_size) * m.x / den; }
    E(x) E(y) E(z) E(w)
#undef E
}

__global__ void k_rows(int64_t n4, AdamC c, float4* p, float4* m, float4* v, const float4* g, const float4* r) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    float4 pp = p[i], mm = m[i], vv = v[i], gg = g[i], rr = r[i];
    float4 gt = make_float4(gg.x + rr.x, gg.y + rr.y, gg.z + rr.z, gg.w + rr.w);
    adam4(c, pp, mm, vv, gt);
    p[i] = pp; m[i] = mm; v[i] = vv;
}

template <int U>
__global__ void k_flat(int64_t n4, AdamC c, float4* p, float4* m, float4* v, const float4* g, const float4* r) {
    const int64_t stride = (int64_t)gridDim.x * 256 * U;
    for (int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride) {
        float4 pp[U], mm[U], vv[U], gg[U], rr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + u * 256;
            if (i < n4) { pp[u] = p[i]; mm[u] = m[i]; vv[u] = v[i]; gg[u] = g[i]; rr[u] = r[i]; }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + u * 256;
            if (i < n4) {
                float4 gt = make_float4(gg[u].x + rr[u].x, gg[u].y + rr[u].y, gg[u].z + rr[u].z, gg[u].w + rr[u].w);
                adam4(c, pp[u], mm[u], vv[u], gt);
                p[i] = pp[u]; m[i] = mm[u]; v[i] = vv[u];
            }
        }
    }
}

__global__ void k_copy(int64_t n4, const float4* a, float4* b) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n4) b[i] = a[i];
}

int main() {
    const int64_t rows = 53955, d = 64, n4 = rows * d / 4;
    std::vector<float4*> buf(8);
    for (auto& b : buf) { hipMalloc(&b, n4 * 16); hipMemset(b, 0, n4 * 16); }
    AdamC c{1e-3f, 0.1f, 0.999f, 0.001f, 1e-8f, 1e-2f, 0.05f};
    hipEvent_t s, e;
    hipEventCreate(&s); hipEventCreate(&e);
    auto time = [&](const char* name, auto fn, double bytes) {
        for (int i = 0; i < 10; ++i) fn();
        hipEventRecord(s);
        const int reps = 200;
        for (int i = 0; i < reps; ++i) fn();
        hipEventRecord(e);
        hipEventSynchronize(e);
        float ms; hipEventElapsedTime(&ms, s, e);
        const double us = ms * 1e3 / reps;
        printf("%-28s %8.2f us  %6.2f TB/s\n", name, us, bytes / (us * 1e-6) / 1e12);
    };
    const double B = n4 * 16.0;
    time("copy 13.8MB", [&] { hipLaunchKernelGGL(k_copy, dim3((n4 + 255) / 256), dim3(256), 0, 0, n4, buf[0], buf[1]); }, 2 * B);
    time("adam rows (1 float4/thr)", [&] { hipLaunchKernelGGL(k_rows, dim3((n4 + 255) / 256), dim3(256), 0, 0, n4, c, buf[0], buf[1], buf[2], buf[3], buf[4]); }, 8 * B);
    for (int g : {512, 1024, 2048, 4096}) {
        char nm[64];
        snprintf(nm, 64, "adam flat U=1 grid %d", g);
        time(nm, [&] { hipLaunchKernelGGL(k_flat<1>, dim3(g), dim3(256), 0, 0, n4, c, buf[0], buf[1], buf[2], buf[3], buf[4]); }, 8 * B);
        snprintf(nm, 64, "adam flat U=2 grid %d", g);
        time(nm, [&] { hipLaunchKernelGGL(k_flat<2>, dim3(g), dim3(256), 0, 0, n4, c, buf[0], buf[1], buf[2], buf[3], buf[4]); }, 8 * B);
        snprintf(nm, 64, "adam flat U=4 grid %d", g);
        time(nm, [&] { hipLaunchKernelGGL(k_flat<4>, dim3(g), dim3(256), 0, 0, n4, c, buf[0], buf[1], buf[2], buf[3], buf[4]); }, 8 * B);
    }
    // 3 streams (p, m, v) only: the tagged step's Adam traffic
    time("adam rows, g=r=same buf", [&] { hipLaunchKernelGGL(k_rows, dim3((n4 + 255) / 256), dim3(256), 0, 0, n4, c, buf[0], buf[1], buf[2], buf[5], buf[5]); }, 7 * B);
    return 0;
}

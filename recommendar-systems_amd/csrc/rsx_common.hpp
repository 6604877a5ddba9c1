// rsx_common.hpp — shared device helpers for the gfx950 kernels of librsx.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "rsx.h"

namespace rsx {

constexpr int kWave = 64;  // CDNA wavefront

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float4 f4(float a) { return make_float4(a, a, a, a); }
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 mul4(float s, float4 a) {
    return make_float4(s * a.x, s * a.y, s * a.z, s * a.w);
}
__device__ __forceinline__ float4 fma4(float s, float4 a, float4 c) {
    return make_float4(fmaf(s, a.x, c.x), fmaf(s, a.y, c.y), fmaf(s, a.z, c.z), fmaf(s, a.w, c.w));
}
__device__ __forceinline__ float dot4(float4 a, float4 b) {
    return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}

// Sum over the G lanes of an aligned lane group (G a power of two <= 64).
template <int G>
__device__ __forceinline__ float group_sum(float x) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) x += __shfl_xor(x, o, kWave);
    return x;
}
template <int G>
__device__ __forceinline__ double group_sum_d(double x) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) x += __shfl_xor(x, o, kWave);
    return x;
}

inline int hip_rc(hipError_t e) { return static_cast<int>(e); }
inline int last_rc() { return static_cast<int>(hipGetLastError()); }
inline hipStream_t as_stream(rsx_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
// the current device's CU count (cached per process; 256 when the query fails)
inline int device_cus() {
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

// A tuning knob read from the environment: unset -> dflt; an integer in [lo, hi] -> that
// value; anything else (not an integer, out of range) aborts with the knob's name.
// Knobs only re-plan launches (grid sizes, splits, phases); none changes a result.
inline int env_knob(const char* name, int dflt, int lo, int hi) {
    const char* v = getenv(name);
    if (!v || !*v) return dflt;
    char* end = nullptr;
    const long long x = strtoll(v, &end, 10);
    if (*end != '\0' || x < lo || x > hi) {
        fprintf(stderr, "librsx: %s=%s is not a valid value (an integer in [%d, %d])\n", name, v, lo, hi);
        abort();
    }
    return (int)x;
}

// Batch-row tagging carried by an SpMM launch (extra blocks after the work and
// fixup blocks): row_tag[u] = row_tag[n_users + i] = tag for every triplet.
struct TagJob {
    const int64_t* trip = nullptr;  // [3, batch]
    int64_t batch = 0;
    int64_t n_users = 0;
    int32_t* row_tag = nullptr;
    int32_t tag = 0;
    const int32_t* tag_dev = nullptr;  // device tag word (graph replays), else `tag`
};

}  // namespace rsx

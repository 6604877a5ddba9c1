// Micro: dependent v_add_f64 chain latency on gfx950 (one wave), vs an LDS-fed chain.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void chain_reg(double* out, int n, double a0) {
    double s = 0.0, x = a0;
    for (int i = 0; i < n; i += 8) {
#pragma unroll
        for (int q = 0; q < 8; ++q) s += x * (double)(q + 1);  // the mul is independent of s
    }
    out[threadIdx.x] = s;
}
__global__ void chain_reg_pure(double* out, int n, double a0) {
    double s = 0.0;
    double x0 = a0, x1 = a0 * 2, x2 = a0 * 3, x3 = a0 * 4;
    for (int i = 0; i < n; i += 4) {
        s += x0; s += x1; s += x2; s += x3;
    }
    out[threadIdx.x] = s;
}
int main() {
    double* o;
    hipMalloc(&o, 4096);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int n : {35600 * 2, 35600 * 8}) {
        for (int k = 0; k < 2; ++k) {
            hipLaunchKernelGGL(chain_reg_pure, dim3(1), dim3(64), 0, 0, o, n, 1.0000001);
            hipEventRecord(a);
            hipLaunchKernelGGL(chain_reg_pure, dim3(1), dim3(64), 0, 0, o, n, 1.0000001);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            printf("pure f64 add chain n=%d: %.3f ms = %.2f ns/add\n", n, ms, ms * 1e6 / n);
        }
    }
    return 0;
}

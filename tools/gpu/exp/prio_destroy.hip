// Round-6 diagnosis of the greatest-priority capture fault: is it the HIP
// runtime?  No RCCL, no torch.  Each round: a comm-like stream P (greatest priority, or the
// default with PRIO 0), optionally used eagerly first (EAGER), then a graph captured on S that
// forks onto P and joins back, instantiated and launched 5 times; with DESTROY the graph, its
// exec and P are destroyed before the next round creates a new P.
//   prio_destroy PRIO DESTROY EAGER
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

__global__ void bump(float* p, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += 1.f;
}

int main(int argc, char** argv) {
    const int prio = argc > 1 ? atoi(argv[1]) : 1, destroy = argc > 2 ? atoi(argv[2]) : 1,
              eager = argc > 3 ? atoi(argv[3]) : 1;
    const int n = 1 << 16;
    float* buf;
    CK(hipMalloc(&buf, n * sizeof(float)));
    CK(hipMemset(buf, 0, n * sizeof(float)));
    int least = 0, greatest = 0;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    hipStream_t S;
    CK(hipStreamCreateWithFlags(&S, hipStreamNonBlocking));
    int launches = 0;
    for (int round = 0; round < 3; ++round) {
        hipStream_t P;
        if (prio) CK(hipStreamCreateWithPriority(&P, hipStreamNonBlocking, greatest));
        else CK(hipStreamCreateWithFlags(&P, hipStreamNonBlocking));
        hipEvent_t f, j;
        CK(hipEventCreateWithFlags(&f, hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
        if (eager) {
            hipLaunchKernelGGL(bump, dim3(n / 256), dim3(256), 0, P, buf, n);
            CK(hipStreamSynchronize(P));
        }
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(S, hipStreamCaptureModeThreadLocal));
        hipLaunchKernelGGL(bump, dim3(n / 256), dim3(256), 0, S, buf, n);
        CK(hipEventRecord(f, S));
        CK(hipStreamWaitEvent(P, f, 0));
        hipLaunchKernelGGL(bump, dim3(n / 256), dim3(256), 0, P, buf, n);
        CK(hipEventRecord(j, P));
        CK(hipStreamWaitEvent(S, j, 0));
        hipLaunchKernelGGL(bump, dim3(n / 256), dim3(256), 0, S, buf, n);
        CK(hipStreamEndCapture(S, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int r = 0; r < 5; ++r) {
            CK(hipGraphLaunch(ge, S));
            CK(hipStreamSynchronize(S));
            ++launches;
        }
        printf("prio=%d destroy=%d eager=%d round %d: 5 launches ok\n", prio, destroy, eager, round);
        fflush(stdout);
        if (destroy) {
            CK(hipGraphExecDestroy(ge));
            CK(hipGraphDestroy(g));
            CK(hipStreamDestroy(P));
            CK(hipEventDestroy(f));
            CK(hipEventDestroy(j));
        }
    }
    float h = 0.f;
    CK(hipMemcpy(&h, buf, sizeof(float), hipMemcpyDeviceToHost));
    printf("prio=%d destroy=%d eager=%d: %d launches, buf[0] = %.0f (expected %d)\n", prio, destroy, eager, launches, h,
           3 * launches + (eager ? 3 : 0));
    return 0;
}

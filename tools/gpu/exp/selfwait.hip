// selfwait.hip — does a captured stream waiting on an event recorded on ITSELF break a
// HIP graph?  (round-4 sharded-step faults: csrc/dist.hip issued such waits on the comm
// stream between 4d71443 and 34a5abd; see DESIGN.md §6 "The round-4 faults").
//
// Graph, captured from origin stream s with a second stream c (forked, then joined):
//   s: A  x[i] = gen                       (gen = the launch number, from a device counter)
//   c: B  sleep ~200 us, y[i] = x[i] + 1    (waits on A through the fork event)
//   c: [variant 1: record e on c, c waits on e -- the self-wait]
//   c: C  z[i] = y[i] + 1
//   s: D  (after the join) err += (z[i] != gen + 2)
// With `rounds` > 1 the fork / B / C / join pattern repeats that many times in the one
// graph (each round's B on the side stream overlapping an A-like kernel on s), the shape
// of a captured sharded step: many short joins of a long-running side-stream kernel.
// Usage: selfwait <self_wait 0|1> <priority 0|1> [launches] [rounds]; prints the error count.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            printf("FAIL %s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            return 2;                                                             \
        }                                                                         \
    } while (0)

constexpr int N = 1 << 16;

__global__ void k_a(int* x, int* gen) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    __shared__ int g;
    if (threadIdx.x == 0) g = gen[0] + 1;
    __syncthreads();
    if (i < N) x[i] = g;
    if (i == 0) gen[1] = g;  // published for D (read after the join)
}

__global__ void k_b(const int* x, int* y) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < 20000) __builtin_amdgcn_s_sleep(16);  // ~200 us at 100 MHz
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) y[i] = x[i] + 1;
}

__global__ void k_c(const int* y, int* z) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) z[i] = y[i] + 1;
}

__global__ void k_d(const int* z, int* gen, int* err) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N && z[i] != gen[1] + 2) atomicAdd(err, 1);
    if (i == 0) gen[0] = gen[1];
}

int main(int argc, char** argv) {
    const int self_wait = argc > 1 ? atoi(argv[1]) : 0;
    const int prio = argc > 2 ? atoi(argv[2]) : 0;
    const int launches = argc > 3 ? atoi(argv[3]) : 200;
    const int rounds = argc > 4 ? atoi(argv[4]) : 1;
    int *x, *y, *z, *gen, *err;
    CK(hipMalloc(&x, N * 4));
    CK(hipMalloc(&y, N * 4));
    CK(hipMalloc(&z, N * 4));
    CK(hipMalloc(&gen, 8));
    CK(hipMalloc(&err, 4));
    CK(hipMemset(gen, 0, 8));
    CK(hipMemset(err, 0, 4));
    hipStream_t s, c;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    if (prio) {
        int least = 0, greatest = 0;
        CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
        CK(hipStreamCreateWithPriority(&c, hipStreamNonBlocking, greatest));
    } else {
        CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
    }
    hipEvent_t fork, self, join;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&self, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    const dim3 g(N / 256), b(256);
    hipGraph_t graph;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int r = 0; r < rounds; ++r) {
        hipLaunchKernelGGL(k_a, g, b, 0, s, x, gen);
        CK(hipEventRecord(fork, s));
        CK(hipStreamWaitEvent(c, fork, 0));
        hipLaunchKernelGGL(k_b, g, b, 0, c, x, y);
        if (self_wait) {
            CK(hipEventRecord(self, c));
            CK(hipStreamWaitEvent(c, self, 0));
        }
        hipLaunchKernelGGL(k_c, g, b, 0, c, y, z);
        CK(hipEventRecord(join, c));
        CK(hipStreamWaitEvent(s, join, 0));
        hipLaunchKernelGGL(k_d, g, b, 0, s, z, gen, err);
    }
    CK(hipStreamEndCapture(s, &graph));
    size_t nodes = 0;
    CK(hipGraphGetNodes(graph, nullptr, &nodes));
    hipGraphExec_t exec;
    CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    for (int i = 0; i < launches; ++i) CK(hipGraphLaunch(exec, s));
    CK(hipStreamSynchronize(s));
    int h_err = -1, h_gen[2] = {0, 0};
    CK(hipMemcpy(&h_err, err, 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h_gen, gen, 8, hipMemcpyDeviceToHost));
    printf("self_wait=%d priority=%d rounds=%d nodes=%zu launches=%d generations=%d wrong_elements=%d\n", self_wait,
           prio, rounds, nodes, launches, h_gen[0], h_err);
    return h_err == 0 && h_gen[0] == launches * rounds ? 0 : 1;
}

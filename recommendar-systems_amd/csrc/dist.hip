// dist.hip — row-sharded LightGCN step over RCCL (gfx950, one process per GPU).
//
// The reference is single-process; this is the build's scaling
// axis.  A = [[0, R], [R^T, 0]] is bipartite: with users split in
// contiguous per-rank blocks and the item rows replicated,
//     users^k = R_g items^{k-1}             local (items^{k-1} is replicated)
//     items^k = sum_g R_g^T users_g^{k-1}   per-rank partial + one all-reduce
// so a K-layer step exchanges 2K+1 item blocks of n_items*d floats (K forward
// layers, G's item rows + K-1 backward layers, the item gradient).  The
// sequence is the one rsx/dist.py:ShardedLightGCNEngine states in Python (the
// gloo-tested restatement of the partitioning); here the whole step is issued
// from C++ so the host never falls behind the device: every exchange goes to the
// communicator's own stream as soon as its partial exists (fork event from the
// compute stream), and the compute stream waits for it (join event) only where
// the reduced rows are read.  The user-row SpMM of a layer and the next layer's
// item partial run on the compute stream meanwhile.
//
// RCCL is resolved at run time from the copy the process already loaded (torch's
// ProcessGroupNCCL loads librccl.so.1), so librsx has no link-time dependency on
// it and loads on machines without RCCL; rsx_comm_* return RSX_ERR_COMM then.
#include <dlfcn.h>

#include <cstring>

#include <rccl/rccl.h>

#include "rsx_common.hpp"

namespace rsx {

int spmm_dispatch(const rsx_csr& a, const float* x, int d, const rsx_epilogue& e, float* slab, hipStream_t s);
int spmm_dispatch_tagging(const rsx_csr& a, const float* x, int d, const rsx_epilogue& e, float* slab,
                          hipStream_t s, const TagJob& tj);
int rowwise_dispatch(int64_t n, int d, const rsx_epilogue& e, hipStream_t s);
int bpr_call(int32_t variant, const float* fin, const float* ego, int64_t n_users, int64_t n_items, int32_t d,
             const int64_t* trip, int64_t batch, float reg, float batch_cfg, float* g_fin, float* g_ego,
             float* loss_out, double* loss_acc, void* ws, size_t ws_bytes, hipStream_t s, float g_div = 1.f,
             int32_t* halt = nullptr, int32_t tag = 0);
int bpr_fused_call(const float* fin, const float* ego, int64_t n_users, int64_t n_items, int32_t d,
                   const int64_t* trip, int64_t batch, float reg, float g_div, float* g_fin, int32_t* reg_cnt,
                   float* loss_out, double* loss_acc, void* ws, size_t ws_bytes, hipStream_t s, int32_t* halt = nullptr,
                   int32_t tag = 0);

namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclReduceScatter) reduce_scatter = nullptr;
    bool ok = false;
};

const Rccl& rccl() {
    static Rccl r = [] {
        Rccl x;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // torch's copy, if loaded
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return x;
        x.get_unique_id = reinterpret_cast<decltype(&ncclGetUniqueId)>(dlsym(h, "ncclGetUniqueId"));
        x.init_rank = reinterpret_cast<decltype(&ncclCommInitRank)>(dlsym(h, "ncclCommInitRank"));
        x.destroy = reinterpret_cast<decltype(&ncclCommDestroy)>(dlsym(h, "ncclCommDestroy"));
        x.all_reduce = reinterpret_cast<decltype(&ncclAllReduce)>(dlsym(h, "ncclAllReduce"));
        x.all_gather = reinterpret_cast<decltype(&ncclAllGather)>(dlsym(h, "ncclAllGather"));
        x.reduce_scatter = reinterpret_cast<decltype(&ncclReduceScatter)>(dlsym(h, "ncclReduceScatter"));
        x.ok = x.get_unique_id && x.init_rank && x.destroy && x.all_reduce && x.all_gather && x.reduce_scatter;
        return x;
    }();
    return r;
}

constexpr int kJoinEvents = 64;  // > 2K+2 exchanges in flight per step for any K <= 30

}  // namespace

}  // namespace rsx

struct rsx_comm_s {
    ncclComm_t nccl = nullptr;
    hipStream_t stream = nullptr;  // exchanges run here, ordered (eagerly issued steps)
    // exchanges of a step being captured into a hipGraph run here instead: a stream at
    // the default priority (nullptr when `stream` is one).  A captured fork / join on a
    // greatest-priority stream made graph replays segfault in hipGraphLaunch (round 4 /
    // round 5: the latency-injected sharded step, DESIGN.md §6 "The round-4 faults"),
    // and a replayed graph's kernels do not run on the captured streams anyway
    hipStream_t stream_cap = nullptr;
    hipEvent_t fork = nullptr;     // compute -> comm (waited right after it is recorded)
    hipEvent_t join[rsx::kJoinEvents] = {};
    int next = 0;
    int32_t rank = 0, world = 1;
    rsx_host_collective_fn host_fn = nullptr;  // test hook: host-side collective instead of RCCL
    void* host_ctx = nullptr;
    // latency-injected one-rank communicator (rsx_comm_init_sim): every collective is the
    // identity on the data (world 1) and a comm-stream kernel that holds `sim_blocks`
    // workgroups and streams the collective's HBM bytes for the modelled time at sim_world
    hipEvent_t pending = nullptr;  // the join event of the last rsx_comm_allreduce_f32_start
    int32_t sim_world = 0;
    double sim_busbw = 0.0;   // bytes/s per rank, the model's bus bandwidth at sim_world
    double sim_lat = 0.0;     // seconds per collective
    int32_t sim_blocks = 0;
    double sim_tick_hz = 0.0; // the device wall clock
    float* sim_scratch = nullptr;
    int64_t sim_scratch_floats = 0;
    // RSX_COMM_SIM_POISON=1 (tests): each stand-in collective overwrites its buffer with
    // poison (f32 NaN / i64 -1) for the modelled time and restores it at the end, so a
    // reader not ordered after the join sees NaN / an out-of-range id and a writer not
    // ordered before the fork is overwritten by the restore: a stream-order race detector
    int32_t sim_poison = 0;
    float* sim_save = nullptr;  // [scratch floats / 2]: the poisoned buffer's saved words
};

namespace rsx {

// The communicator's stream at the device's greatest priority (RSX_COMM_PRIORITY=0: the
// default priority): a collective queued behind a chip-filling product gets its
// workgroups dispatched as soon as slots free up, instead of after that product's queued
// blocks (RCCL's kernels, and the latency-injected stand-in, hold a few dozen CUs).
// Correctness never depends on it: every cross-stream read / write is fenced by the
// fork / join events (tests/test_gpu_dist.py runs the poisoned stand-in with it on).
hipError_t comm_streams_create(rsx_comm_s* c) {
    const int prio_on = env_knob("RSX_COMM_PRIORITY", 1, 0, 1);  // read per communicator
    // diagnosis only (tools/gpu/diag_priority.py): captured collectives on the priority stream
    // too, the round-4 configuration whose graph replays segfaulted
    const int cap_prio = env_knob("RSX_COMM_CAPTURE_PRIORITY", 0, 0, 1);
    int least = 0, greatest = 0;
    if (prio_on && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess && greatest != least) {
        hipError_t e = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, greatest);
        if (e == hipSuccess && !cap_prio) e = hipStreamCreateWithFlags(&c->stream_cap, hipStreamNonBlocking);
        return e;
    }
    return hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
}

int comm_rank(rsx_comm_t c) { return c->rank; }
int comm_world(rsx_comm_t c) { return c->world; }
// The modelled world of a latency-injected communicator (0 for a real or host-hook one).
int comm_sim_world(rsx_comm_t c) { return c->sim_world; }
// The stream the communicator's exchanges run on, for work issued from `s` (host-hook
// communicators: `s` itself): the priority stream for eager issue, the capture stream
// while `s` is being captured; a call issued on either comm stream stays on it.  Small
// kernels that only feed later exchanges can run there, off the compute stream.
hipStream_t comm_stream(rsx_comm_t c, hipStream_t s) {
    if (c->host_fn || s == c->stream || (c->stream_cap && s == c->stream_cap)) return s;
    if (c->stream_cap) {
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cap) == hipSuccess && cap == hipStreamCaptureStatusActive) return c->stream_cap;
    }
    return c->stream;
}
// The next event of the communicator's ring (for a fence the caller records itself).
hipEvent_t comm_event(rsx_comm_t c) {
    hipEvent_t j = c->join[c->next];
    c->next = (c->next + 1) % kJoinEvents;
    return j;
}

// The latency-injection stand-in for one collective: `blocks` workgroups copy `floats`
// floats of the scratch (half read, half written: the collective's HBM traffic) and
// then hold their slots until `ticks` of the device wall clock have passed since the
// kernel started (each block measures from its own start; all start together).
// Poison mode (`save` != nullptr, tests): each thread first saves its words of the
// collective's buffer and overwrites them with `poison` (published device-wide by a
// release fence), and restores them after the wait, so for the modelled time the
// buffer holds NaN (f32) / -1 (i64 ids) — what an unfenced reader would see.
__global__ __launch_bounds__(256) void sim_collective(float* __restrict__ scratch, int64_t half, int64_t floats,
                                                      uint64_t ticks, uint32_t* __restrict__ buf,
                                                      uint32_t* __restrict__ save, int64_t words, uint32_t poison) {
    const uint64_t t0 = wall_clock64();
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * 256;
    if (save) {
        for (int64_t i = tid; i < words; i += stride) {
            save[i] = buf[i];
            buf[i] = poison;
        }
        __threadfence();
    }
    // float4 copies, four in flight per lane, in passes over the scratch's halves (a
    // per-element loop with one dependent load at a time ran at ~0.2 TB/s on 32 blocks
    // and took several times the modelled collective time at C4's 1 GB item block)
    const int64_t h4 = half / 4;
    const float4* __restrict__ src = reinterpret_cast<const float4*>(scratch);
    float4* __restrict__ dst = reinterpret_cast<float4*>(scratch + half);
    for (int64_t todo = floats / 8; todo > 0;) {
        const int64_t n = todo < h4 ? todo : h4;
        int64_t i = tid;
        for (; i + 3 * stride < n; i += 4 * stride) {
            const float4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], e = src[i + 3 * stride];
            dst[i] = add4(a, f4(1.f));
            dst[i + stride] = add4(b, f4(1.f));
            dst[i + 2 * stride] = add4(c, f4(1.f));
            dst[i + 3 * stride] = add4(e, f4(1.f));
        }
        for (; i < n; i += stride) dst[i] = add4(src[i], f4(1.f));
        todo -= n;
    }
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
    if (save)
        for (int64_t i = tid; i < words; i += stride) buf[i] = save[i];
}

// Modelled time of one collective of `bytes` (the whole buffer: all-reduce X, all-gather
// / reduce-scatter world * count) over sim_world ranks: a ring moves 2 (W-1)/W X per rank
// for an all-reduce, (W-1)/W X for the others, at the model's per-rank bus bandwidth.
static double sim_seconds(const rsx_comm_s* c, int op, double bytes) {
    const double w = c->sim_world;
    const double moved = (op == RSX_COLL_ALLREDUCE ? 2.0 : 1.0) * (w - 1.0) / w * bytes;
    return moved / c->sim_busbw + c->sim_lat;
}

// In-place collective `op` (RSX_COLL_*) on buf over the communicator, after the
// work queued so far on `s`; returns the join event the reader must wait on
// (nullptr on error, rc set).  A host-hook communicator synchronises `s`, calls the
// hook and returns an event recorded on `s`.
hipEvent_t collective(rsx_comm_t c, int op, void* buf, int64_t count, int dtype, hipStream_t s, int* rc) {
    hipError_t e;
    hipEvent_t j = c->join[c->next];
    c->next = (c->next + 1) % kJoinEvents;
    const hipStream_t cs = comm_stream(c, s);
    // a call issued on the comm stream itself (work queued behind an earlier exchange) needs no
    // fork: a captured stream waiting on an event recorded on itself makes the graph's replay
    // segfault in hipGraphLaunch (tools/gpu/exp/selfwait.hip)
    const bool fork = s != cs;
    if (c->sim_world) {  // one rank: the data is already the result; the time is injected
        if (fork && ((e = hipEventRecord(c->fork, s)) != hipSuccess ||
                     (e = hipStreamWaitEvent(cs, c->fork, 0)) != hipSuccess)) {
            *rc = hip_rc(e);
            return nullptr;
        }
        const double es = dtype == RSX_COLL_I64 ? 8.0 : 4.0;
        const double bytes = (double)count * es;  // world 1: the whole buffer
        const double sec = sim_seconds(c, op, bytes);
        const double moved = (op == RSX_COLL_ALLREDUCE ? 2.0 : 1.0) * (c->sim_world - 1.0) / c->sim_world * bytes;
        int64_t floats = (int64_t)(2.0 * moved / 4.0);  // the moved bytes read once and written once
        const int64_t half = c->sim_scratch_floats / 2;
        // poison mode: the whole buffer the collective writes (world 1: count elements)
        const int64_t words = (int64_t)bytes / 4;
        const bool poison = c->sim_poison && words <= c->sim_scratch_floats / 2;
        hipLaunchKernelGGL(sim_collective, dim3((unsigned)c->sim_blocks), dim3(256), 0, cs, c->sim_scratch,
                           half, floats, (uint64_t)(sec * c->sim_tick_hz), poison ? static_cast<uint32_t*>(buf) : nullptr,
                           poison ? reinterpret_cast<uint32_t*>(c->sim_save) : nullptr, words,
                           dtype == RSX_COLL_I64 ? 0xffffffffu : 0x7fc00000u);
        if ((e = hipGetLastError()) != hipSuccess || (e = hipEventRecord(j, cs)) != hipSuccess) {
            *rc = hip_rc(e);
            return nullptr;
        }
        return j;
    }
    if (c->host_fn) {
        if ((e = hipStreamSynchronize(s)) != hipSuccess) {
            *rc = hip_rc(e);
            return nullptr;
        }
        if (c->host_fn(op, buf, count, dtype, c->host_ctx)) {
            *rc = RSX_ERR_COMM;
            return nullptr;
        }
        if ((e = hipEventRecord(j, s)) != hipSuccess) {
            *rc = hip_rc(e);
            return nullptr;
        }
        return j;
    }
    if (fork && ((e = hipEventRecord(c->fork, s)) != hipSuccess ||
                 (e = hipStreamWaitEvent(cs, c->fork, 0)) != hipSuccess)) {
        *rc = hip_rc(e);
        return nullptr;
    }
    const ncclDataType_t ty = dtype == RSX_COLL_I64 ? ncclInt64 : ncclFloat32;
    const size_t es = dtype == RSX_COLL_I64 ? 8 : 4;
    char* own = static_cast<char*>(buf) + (size_t)c->rank * (size_t)count * es;
    ncclResult_t r;
    if (op == RSX_COLL_ALLGATHER) r = rccl().all_gather(own, buf, (size_t)count, ty, c->nccl, cs);
    else if (op == RSX_COLL_REDUCESCATTER) r = rccl().reduce_scatter(buf, own, (size_t)count, ty, ncclSum, c->nccl, cs);
    else r = rccl().all_reduce(buf, buf, (size_t)count, ty, ncclSum, c->nccl, cs);
    if (r != ncclSuccess) {
        *rc = RSX_ERR_COMM;
        return nullptr;
    }
    if ((e = hipEventRecord(j, cs)) != hipSuccess) {
        *rc = hip_rc(e);
        return nullptr;
    }
    return j;
}

hipEvent_t exchange(rsx_comm_t c, float* a, int64_t n, hipStream_t s, int* rc) {
    return collective(c, RSX_COLL_ALLREDUCE, a, n, RSX_COLL_F32, s, rc);
}

namespace {

// ---- row lists of the sparse exchange -------------------------------------------
__global__ __launch_bounds__(256) void tag_rows_k(const int64_t* ids, int64_t n, int32_t* tag_arr,
                                                  const int32_t* tag_dev, int32_t tag, int64_t n_rows, int32_t* err) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const int64_t i = ids[j];
    if (i < 0 || i >= n_rows) {
        if (err) atomicOr(err, 1);
        return;
    }
    tag_arr[i] = tag_dev ? *tag_dev : tag;
}

// mode 0: dst[j] = src[ids[j]] (gather), 1: dst[ids[j]] = src[j] (scatter; duplicate
// ids carry identical rows), 2: dst[ids[j]] = 0.  An id outside [0, n_rows) is never
// dereferenced: it sets err bit 0 (rsx_sharded_lgcn_step.err) instead of faulting.
__global__ __launch_bounds__(256) void rows_k(const float* src, float* dst, const int64_t* ids, int64_t n, int d,
                                              int mode, int64_t n_rows, int32_t* err) {
    const int q = d / 4;
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= n * q) return;
    const int64_t j = e / q;
    const int c = (int)(e - j * q) * 4;
    const int64_t i = ids[j];
    if (i < 0 || i >= n_rows) {
        if (err) atomicOr(err, 1);
        return;
    }
    if (mode == 0) st4(dst + j * d + c, ld4(src + i * d + c));
    else if (mode == 1) st4(dst + i * d + c, ld4(src + j * d + c));
    else st4(dst + i * d + c, f4(0.f));
}

// This rank's list for the sparse last-layer exchange: its (pos, neg) items (the union
// share), then every neighbour item of its DISTINCT batch users (A_U row u: cols =
// n_users + item), appended at a claimed position; the caller zero-fills the slice first
// (unused slots stay item 0).  One wave per triplet; a user repeated in the batch is
// listed once: the wave that swaps the step's tag into row_tag[u] first lists it (the
// first item partial's tag blocks later write the same tags), so the list holds at most
// 2 batch + the sum of the batch's distinct users' degrees <= the host bound (2 union_cap
// + the union_cap largest degrees).  A claim past `cap` is dropped and sets err bit 1.
__global__ __launch_bounds__(256) void nbr_list_k(const int64_t* __restrict__ trip, int64_t batch,
                                                  const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                                  int64_t n_users, int64_t* __restrict__ out, int64_t cap,
                                                  int32_t* __restrict__ cnt, int32_t* __restrict__ row_tag,
                                                  const int32_t* __restrict__ tag_dev, int32_t tag,
                                                  int32_t* __restrict__ err) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= batch) return;
    if (lane < 2) out[2 * w + lane] = trip[(1 + lane) * batch + w];  // pos, neg of triplet w
    const int64_t u = trip[w];
    const int64_t b = rowptr[u], e = rowptr[u + 1];
    int32_t base = -1;
    if (lane == 0) {
        const int32_t t = tag_dev ? *tag_dev : tag;
        if (atomicExch(row_tag + u, t) != t) {
            base = atomicAdd(cnt, (int32_t)(e - b));
            if (2 * batch + base + (e - b) > cap && err) atomicOr(err, 2);
        }
    }
    base = __shfl(base, 0, 64);
    if (base < 0) return;  // a repeated user: listed by its first triplet's wave
    for (int64_t j = b + lane; j < e; j += 64) {
        const int64_t p = 2 * batch + base + (j - b);
        if (p < cap) out[p] = (int64_t)col[j] - n_users;
    }
}

int rows_op(const float* src, float* dst, const int64_t* ids, int64_t n, int d, int mode, int64_t n_rows,
            int32_t* err, hipStream_t s) {
    if (n <= 0) return 0;
    const int64_t tot = n * (d / 4);
    hipLaunchKernelGGL(rows_k, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, src, dst, ids, n, d, mode,
                       n_rows, err);
    return last_rc();
}

int wait(hipStream_t s, hipEvent_t j) { return hip_rc(hipStreamWaitEvent(s, j, 0)); }

rsx_epilogue epi(int kind) {
    rsx_epilogue e = {};
    e.kind = kind;
    e.alpha = 1.f;
    e.beta = 1.f;
    return e;
}

#define RSX_TRY(x)                 \
    do {                           \
        const int rc_ = (x);       \
        if (rc_) return rc_;       \
    } while (0)

// Forward layers (rsx/dist.py:_propagate).  Item rows of layer k live in
// bufs[(k-1)&1] + nu*d; they are summed across ranks before anything reads them.
int sharded_forward(const rsx_sharded_lgcn_step& st, bool zero_grads, hipStream_t s) {
    const int d = st.d, K = st.n_layers;
    const int64_t nu = st.n_users, ni = st.n_items, off = nu * (int64_t)d;
    const float beta = 1.f / (float)(K + 1);
    float* bufs[2] = {st.h0, st.h1};
    auto ys = [&](int k) -> float* { return k == 0 ? st.p : bufs[(k - 1) & 1]; };
    hipEvent_t joins[64] = {};
    int rc = 0;
    auto item_partial = [&](int k) -> int {  // items^k partial = R_g^T users^{k-1}; exchange queued
        rsx_epilogue e = epi(RSX_EPI_STORE);
        e.y = ys(k) + off;
        RSX_TRY(spmm_dispatch(*st.adj_i, ys(k - 1), d, e, st.slab_i, s));
        joins[k] = exchange(st.comm, ys(k) + off, ni * d, s, &rc);
        return joins[k] ? 0 : rc;
    };
    RSX_TRY(item_partial(1));
    for (int k = 1; k <= K; ++k) {
        const float* s_in = k == 1 ? st.p : st.s;
        if (k < K) {
            rsx_epilogue e = epi(RSX_EPI_LAYERSUM);
            e.y = ys(k);
            e.s_in = s_in;
            e.s_out = st.s;
            RSX_TRY(spmm_dispatch(*st.adj_u, ys(k - 1), d, e, st.slab_u, s));
            RSX_TRY(item_partial(k + 1));
        } else {
            rsx_epilogue e = epi(RSX_EPI_FINAL);
            e.beta = beta;
            e.f = st.final_emb;
            e.s_in = s_in;
            if (zero_grads) {
                e.zero0 = st.g;
                e.zero1 = st.r;
            }
            RSX_TRY(spmm_dispatch(*st.adj_u, ys(k - 1), d, e, st.slab_u, s));
        }
        RSX_TRY(wait(s, joins[k]));
        rsx_epilogue e = epi(RSX_EPI_ADD);
        e.s_in = s_in + off;
        e.r_add = ys(k) + off;
        if (k < K) {
            e.y = st.s + off;
        } else {
            e.beta = beta;
            e.y = st.final_emb + off;
            if (zero_grads) {
                e.zero0 = st.g + off;
                e.zero1 = st.r + off;
            }
        }
        RSX_TRY(rowwise_dispatch(ni, d, e, s));
    }
    return 0;
}

// Stored-layer step for K = 2, 3 (the sharded twin of step.hip's
// lgcn_step_stored_layers).  Forward: E^k user rows local, item rows = the sum of
// the ranks' partials (one exchange per layer); the last layer writes the mean
// directly: on rank 0 the item partial's epilogue adds the (already summed)
// E^0..E^{K-1} item rows, so one exchange of the final item rows gives the mean
// (scaled by 1/(K+1) before the sum), and the user rows' mean is computed on the
// batch rows only.  Backward: Horner on G' = dL/dfinal / (K+1) (BPR's g_div),
//   H^k = G' + A H^{k-1},  H^0 = G',  Adam on g = H^K + R,
// with G''s item rows summed once and added to the item partials by rank 0 only;
// the last item partial carries (rank 0) G'_I and (every rank) its own R_I, so one
// exchange gives the whole item gradient.  2K+1 exchanges of n_items*d floats per
// step, 2K SpMM launches + 1 item Adam launch, no layer-sum passes.  `train` false: forward only, every final row (evaluation).
int sharded_stored_layers(const rsx_sharded_lgcn_step& st, bool train, hipStream_t s) {
    const int d = st.d, K = st.n_layers;
    const int64_t nu = st.n_users, ni = st.n_items, off = nu * (int64_t)d;
    const bool root = st.comm->rank == 0;
    const float beta = 1.f / (float)(K + 1);
    const int32_t tag = (int32_t)st.tag;
    float* bufs[2] = {st.h0, st.h1};
    hipEvent_t joins[4] = {};
    int rc = 0;
    // sparse exchange: the union of every rank's (pos, neg) items, gathered first
    const bool sparse = train && st.union_items;
    const int64_t cap = st.union_cap;
    const int64_t nU = sparse ? (int64_t)st.comm->world * 2 * cap : 0;
    hipEvent_t jU = nullptr;
    if (sparse) {
        int64_t* mine = st.union_items + (int64_t)st.comm->rank * 2 * cap;
        RSX_TRY(hip_rc(hipMemcpyAsync(mine, st.triplets + st.batch, (size_t)(2 * st.batch) * sizeof(int64_t),
                                      hipMemcpyDeviceToDevice, s)));
        if (cap > st.batch)  // a partial batch: item 0 stands in (its rows come out right anyway)
            RSX_TRY(hip_rc(hipMemsetAsync(mine + 2 * st.batch, 0, (size_t)(2 * (cap - st.batch)) * sizeof(int64_t), s)));
        if (!(jU = collective(st.comm, RSX_COLL_ALLGATHER, st.union_items, 2 * cap, RSX_COLL_I64, s, &rc)))
            return rc;
    }
    // sparse last forward layer: this rank's (pos, neg) + batch users' neighbour items, gathered
    const bool nbr = sparse && st.nbr_items;  // (valid() checked the buffers and the cap)
    const int64_t nQ = nbr ? (int64_t)st.comm->world * st.nbr_cap : 0;
    hipEvent_t jN = nullptr;
    if (nbr) {
        int64_t* mine = st.nbr_items + (int64_t)st.comm->rank * st.nbr_cap;
        RSX_TRY(hip_rc(hipMemsetAsync(mine, 0, (size_t)st.nbr_cap * sizeof(int64_t), s)));
        RSX_TRY(hip_rc(hipMemsetAsync(st.nbr_count, 0, sizeof(int32_t), s)));
        hipLaunchKernelGGL(nbr_list_k, dim3((unsigned)((st.batch + 3) / 4)), dim3(256), 0, s, st.triplets, st.batch,
                           st.adj_u->rowptr, st.adj_u->col, nu, mine, st.nbr_cap, st.nbr_count, st.row_tag,
                           st.tag_dev, tag, st.err);
        RSX_TRY(last_rc());
        if (!(jN = collective(st.comm, RSX_COLL_ALLGATHER, st.nbr_items, st.nbr_cap, RSX_COLL_I64, s, &rc))) return rc;
    }
    // the previous step's owner rows, all-gathered while the first item partial runs (that
    // product reads user rows only); waited on before the first product reading item rows
    hipEvent_t jAG = nullptr;
    if (sparse && st.defer_ag) {
        const int64_t q = st.n_items_pad / st.comm->world;
        if (!(jAG = collective(st.comm, RSX_COLL_ALLGATHER, st.p + off, q * d, RSX_COLL_F32, s, &rc))) return rc;
    }
    // ---- forward (the first item partial's launch also tags the batch rows when training)
    const float* x = st.p;
    for (int k = 1; k < K; ++k) {
        rsx_epilogue e = epi(RSX_EPI_STORE);
        e.y = bufs[k - 1] + off;
        TagJob tj;
        if (train && k == 1) {
            tj.trip = st.triplets;
            tj.batch = st.batch;
            tj.n_users = nu;
            tj.row_tag = st.row_tag;
            tj.tag = tag;
            tj.tag_dev = st.tag_dev;
        }
        if (k == K - 1 && nbr) {
            // E^{K-1}_I is read on the listed rows only (the batch users' final rows gather
            // their neighbour items, the union items' final rows add it): summed there alone
            RSX_TRY(spmm_dispatch_tagging(*st.adj_i, x, d, e, st.slab_i, s, tj));
            RSX_TRY(wait(s, jN));
            RSX_TRY(rows_op(bufs[k - 1] + off, st.cbufN, st.nbr_items, nQ, d, 0, ni, st.err, s));
            if (!(joins[k] = exchange(st.comm, st.cbufN, nQ * d, s, &rc))) return rc;
        } else if (k == 1 && st.n_head > 1) {
            // the step's head: nothing but this product can run before the first exchange,
            // so it goes in row pieces, each piece's item rows summed as soon as they exist
            // (the comm stream is in order: the last piece's join covers every piece)
            for (int32_t p = 0; p < st.n_head; ++p) {
                const int64_t r0 = st.head_row0[p], r1 = st.head_row0[p + 1];
                e.y = bufs[0] + off + r0 * d;
                RSX_TRY(spmm_dispatch_tagging(st.head_i[p], x, d, e, st.head_slab[p], s, p == 0 ? tj : TagJob{}));
                if (!(joins[1] = exchange(st.comm, e.y, (r1 - r0) * d, s, &rc))) return rc;
            }
        } else {
            RSX_TRY(spmm_dispatch_tagging(*st.adj_i, x, d, e, st.slab_i, s, tj));   // item partial of E^k
            if (!(joins[k] = exchange(st.comm, bufs[k - 1] + off, ni * d, s, &rc))) return rc;
        }
        if (k >= 2) RSX_TRY(wait(s, joins[k - 1]));                  // E^{k-1} items summed
        if (k == 1 && jAG) RSX_TRY(wait(s, jAG));                     // p's item rows current
        e.y = bufs[k - 1];
        RSX_TRY(spmm_dispatch(*st.adj_u, x, d, e, st.slab_u, s));   // E^k user rows
        x = bufs[k - 1];
    }
    RSX_TRY(wait(s, joins[K - 1]));
    if (nbr) RSX_TRY(rows_op(st.cbufN, bufs[K - 2] + off, st.nbr_items, nQ, d, 1, ni, st.err, s));  // summed rows back
    {
        rsx_epilogue e = epi(RSX_EPI_FINAL);
        e.beta = beta;
        e.f = st.final_emb + off;
        if (root) {
            e.s_in = st.p + off;
            e.r_add = st.h0 + off;
            e.aux = K == 3 ? st.h1 + off : nullptr;
        }
        if (sparse) {  // only the union rows: tagged, computed, gathered, summed, scattered
            RSX_TRY(wait(s, jU));
            hipLaunchKernelGGL(tag_rows_k, dim3((unsigned)((nU + 255) / 256)), dim3(256), 0, s, st.union_items, nU,
                               st.item_tag, st.tag_dev, tag, ni, st.err);
            RSX_TRY(last_rc());
            // the union items in row_tag's item block as well: after the compact exchange G'_I
            // is nonzero exactly there, so the first backward user-row product gathers only
            // those item rows (RSX_TAG_SPARSE_X) -- the item block of row_tag is read by no
            // other product of this step (its user block holds this rank's batch users)
            hipLaunchKernelGGL(tag_rows_k, dim3((unsigned)((nU + 255) / 256)), dim3(256), 0, s, st.union_items, nU,
                               st.row_tag + nu, st.tag_dev, tag, ni, st.err);
            RSX_TRY(last_rc());
            e.row_tag = st.item_tag;
            e.tag = tag;
            e.tag_dev = st.tag_dev;
            e.tag_flags = RSX_TAG_ROWS;
            RSX_TRY(spmm_dispatch(*st.adj_i, x, d, e, st.slab_i, s));
            RSX_TRY(rows_op(st.final_emb + off, st.cbuf0, st.union_items, nU, d, 0, ni, st.err, s));
            if (!(joins[K] = exchange(st.comm, st.cbuf0, nU * d, s, &rc))) return rc;
            e.row_tag = nullptr;
            e.tag_dev = nullptr;
            e.tag_flags = 0;
        } else {
            RSX_TRY(spmm_dispatch(*st.adj_i, x, d, e, st.slab_i, s));
            if (!(joins[K] = exchange(st.comm, st.final_emb + off, ni * d, s, &rc))) return rc;
        }
        e.f = st.final_emb;
        e.s_in = st.p;
        e.r_add = st.h0;
        e.aux = K == 3 ? st.h1 : nullptr;
        if (train) {
            e.row_tag = st.row_tag;
            e.tag = tag;
            e.tag_dev = st.tag_dev;
            e.tag_flags = RSX_TAG_ROWS;
        }
        RSX_TRY(spmm_dispatch(*st.adj_u, x, d, e, st.slab_u, s));
        RSX_TRY(wait(s, joins[K]));
        if (sparse) RSX_TRY(rows_op(st.cbuf0, st.final_emb + off, st.union_items, nU, d, 1, ni, st.err, s));
    }
    if (!train) return 0;
    // ---- loss: G' = dL/dfinal / (K+1), R = d reg / d ego on this rank's batch rows
    // (with reg_cnt: one launch, the regulariser left as per-row occurrence counts)
    const float* reg_k = st.reg_cnt ? reinterpret_cast<const float*>(st.reg_cnt + 3 * (nu + ni) + 1) : nullptr;
    if (st.reg_cnt)
        RSX_TRY(bpr_fused_call(st.final_emb, st.p, nu, ni, d, st.triplets, st.batch, st.reg, (float)(K + 1), st.g,
                               st.reg_cnt, st.loss_out, st.loss_acc, st.ws, st.ws_bytes, s));
    else
        RSX_TRY(bpr_call(RSX_BPR_LIGHTGCN, st.final_emb, st.p, nu, ni, d, st.triplets, st.batch, st.reg,
                         (float)st.batch, st.g, st.r, st.loss_out, st.loss_acc, st.ws, st.ws_bytes, s,
                         (float)(K + 1)));
    // G'_I summed (R_I is not: every rank adds its own R_I to its last item partial,
    // whose exchange then sums them; one n_items*d exchange less per step)
    if (sparse) {  // G'_I is nonzero on this rank's batch items only: sum the union rows
        RSX_TRY(rows_op(st.g + off, st.cbuf1, st.union_items, nU, d, 0, ni, st.err, s));
        hipEvent_t j0 = exchange(st.comm, st.cbuf1, nU * d, s, &rc);
        if (!j0) return rc;
        RSX_TRY(wait(s, j0));
        RSX_TRY(rows_op(st.cbuf1, st.g + off, st.union_items, nU, d, 1, ni, st.err, s));
    } else {
        hipEvent_t j0 = exchange(st.comm, st.g + off, ni * d, s, &rc);
        if (!j0) return rc;
        RSX_TRY(wait(s, j0));
    }
    // ---- backward
    x = st.g;
    for (int k = 1; k < K; ++k) {
        rsx_epilogue e = epi(RSX_EPI_ADD);
        e.y = bufs[k - 1] + off;
        if (root) e.s_in = st.g + off;  // + G'_I once
        if (k == 1) {                   // X = G': only this rank's batch users are nonzero
            e.row_tag = st.row_tag;
            e.tag = tag;
            e.tag_dev = st.tag_dev;
            e.tag_flags = RSX_TAG_SPARSE_X;
        }
        if (k == 1 && st.n_head > 1) {
            // the backward's head: its first exchange waits for this product alone, so it
            // goes in the same row pieces as the forward's (the pieces' epilogue rows are
            // local: y and G'_I offset by the piece's first row; SPARSE_X reads columns)
            float* y0 = e.y;
            const float* s0 = e.s_in;
            for (int32_t p = 0; p < st.n_head; ++p) {
                const int64_t r0 = st.head_row0[p], r1 = st.head_row0[p + 1];
                e.y = y0 + r0 * d;
                if (s0) e.s_in = s0 + r0 * d;
                RSX_TRY(spmm_dispatch(st.head_i[p], x, d, e, st.head_slab[p], s));
                if (!(joins[1] = exchange(st.comm, e.y, (r1 - r0) * d, s, &rc))) return rc;
            }
        } else {
            RSX_TRY(spmm_dispatch(*st.adj_i, x, d, e, st.slab_i, s));
            if (!(joins[k] = exchange(st.comm, bufs[k - 1] + off, ni * d, s, &rc))) return rc;
        }
        if (k >= 2) RSX_TRY(wait(s, joins[k - 1]));
        rsx_epilogue u = epi(RSX_EPI_ADD);  // H^k users = G'_U + A_U H^{k-1}_I (G'_U on batch users only)
        u.y = bufs[k - 1];
        u.s_in = st.g;
        u.row_tag = st.row_tag;
        u.tag = tag;
        u.tag_dev = st.tag_dev;
        // k = 1, sparse schedule: X = G' whose item rows are nonzero on the union items only
        u.tag_flags = RSX_TAG_SPARSE_S | (k == 1 && sparse ? RSX_TAG_SPARSE_X : 0);
        RSX_TRY(spmm_dispatch(*st.adj_u, x, d, u, st.slab_u, s));
        x = bufs[k - 1];
    }
    {
        rsx_epilogue e = epi(RSX_EPI_ADD);  // item gradient partial: A_I H^{K-1}_U + own R_I (+ G'_I on rank 0)
        e.y = st.t;
        if (root) e.s_in = st.g + off;
        if (st.reg_cnt) {  // own R_I from the counts (cleared here), as the single-GPU Adam layer does
            e.reg_cnt = st.reg_cnt + 3 * nu;
            e.reg_k = reg_k;
            e.p = st.p + off;
        } else {
            e.r_add = st.r + off;
        }
        RSX_TRY(spmm_dispatch(*st.adj_i, x, d, e, st.slab_i, s));
        const int64_t q = sparse ? st.n_items_pad / st.comm->world : 0;  // item rows per owner
        hipEvent_t jt;
        if (sparse) {
            // G'_I and R_I live on the union rows only: cleared there, after their last reader
            RSX_TRY(rows_op(nullptr, st.g + off, st.union_items, nU, d, 2, ni, st.err, s));
            if (!st.reg_cnt) RSX_TRY(rows_op(nullptr, st.r + off, st.union_items, nU, d, 2, ni, st.err, s));
            jt = collective(st.comm, RSX_COLL_REDUCESCATTER, st.t, q * d, RSX_COLL_F32, s, &rc);
        } else {
            jt = exchange(st.comm, st.t, ni * d, s, &rc);
        }
        if (!jt) return rc;
        if (K >= 2) RSX_TRY(wait(s, joins[K - 1]));
        rsx_epilogue u = epi(RSX_EPI_ADAM);  // user rows: g = (G'_U + A_U H^{K-1}_I) + R_U
        u.s_in = st.g;
        u.r_add = st.r;
        u.p = st.p;
        u.m = st.m;
        u.v = st.v;
        u.adam = st.adam;
        u.zero0 = st.g;  // G'_U, R_U cleared on the batch users (nothing reads them later)
        u.zero1 = st.r;
        if (st.reg_cnt) {  // R_U from the counts (cleared on the batch users)
            u.r_add = nullptr;
            u.zero1 = nullptr;
            u.reg_cnt = st.reg_cnt;
            u.reg_k = reg_k;
        }
        u.row_tag = st.row_tag;
        u.tag = tag;
        u.tag_dev = st.tag_dev;
        u.tag_flags = RSX_TAG_SPARSE_S | RSX_TAG_SPARSE_R | RSX_TAG_ZERO;
        RSX_TRY(spmm_dispatch(*st.adj_u, x, d, u, st.slab_u, s));
        if (!sparse) RSX_TRY(wait(s, jt));  // (sparse: the owner Adam runs behind jt on the comm stream)
        if (sparse) {
            // this rank's item rows [rank q, (rank+1) q) ∩ [0, n_items): Adam on the owner only,
            // then every replica receives the updated rows
            const int64_t r0 = (int64_t)st.comm->rank * q;
            int64_t nown = r0 < ni ? (ni - r0 < q ? ni - r0 : q) : 0;
            // latency injection with RSX_COMM_SIM_SHARE=1 (bench.py): the one rank times ITS
            // share of the modelled W-rank job, so the owner Adam covers ceil(n_items / W) rows
            // (the parameters then differ from a one-rank run: a timing mode, not a training one)
            static const int64_t sim_share = env_knob("RSX_COMM_SIM_SHARE", 0, 0, 1);
            if (sim_share && st.comm->sim_world > 1) nown = (ni + st.comm->sim_world - 1) / st.comm->sim_world;
            rsx_epilogue a = epi(RSX_EPI_ADAM);
            a.s_in = st.t + r0 * d;
            a.p = st.p + off + r0 * d;
            a.m = st.m + off + r0 * d;
            a.v = st.v + off + r0 * d;
            a.adam = st.adam;
            // the owner Adam and the all-gather follow the reduce-scatter on the comm stream:
            // they read only its output and the item rows of p / m / v, which nothing on the
            // compute stream touches now (the user Adam there updates user rows), so the
            // all-gather no longer waits for the user-row Adam product
            const int on_comm = env_knob("RSX_SHARDED_COMM_ADAM", 1, 0, 1);  // read per issue (tests flip it)
            hipStream_t cs = on_comm ? comm_stream(st.comm, s) : s;  // (jt completes on cs itself)
            if (cs == s) RSX_TRY(wait(s, jt));
            if (nown > 0) RSX_TRY(rowwise_dispatch(nown, d, a, cs));
            if (st.defer_ag) {  // the all-gather opens the next step (or rsx_sharded_lightgcn_flush)
                if (cs != s) {
                    hipEvent_t ja = comm_event(st.comm);
                    RSX_TRY(hip_rc(hipEventRecord(ja, cs)));
                    RSX_TRY(wait(s, ja));
                }
            } else {
                hipEvent_t jp = collective(st.comm, RSX_COLL_ALLGATHER, st.p + off, q * d, RSX_COLL_F32, cs, &rc);
                if (!jp) return rc;
                RSX_TRY(wait(s, jp));  // the next step (and any reader) sees every updated replica
            }
        } else {
            rsx_epilogue a = epi(RSX_EPI_ADAM);  // item rows, identical on every rank
            a.s_in = st.t;
            a.p = st.p + off;
            a.m = st.m + off;
            a.v = st.v + off;
            a.adam = st.adam;
            a.zero0 = st.g + off;  // the summed G'_I and this rank's R_I: cleared densely
            a.zero1 = st.reg_cnt ? nullptr : st.r + off;
            RSX_TRY(rowwise_dispatch(ni, d, a, s));
        }
    }
    return 0;
}

// Fused-round step for K = 2, 3 (dense schedule, batch-row tags; st.xch = [2 n_items, d]).
// The bipartite graph splits each K-layer chain into two interleaved ones: an item
// partial needs only the rank's own user rows, so two layers' partials can be summed in
// ONE collective.  Forward: [E^1_I | E^2_I] then the final item rows (K = 3), or
// [E^1_I | final item rows] (K = 2: the final partial adds the rank's OWN E^1 partial,
// the sum over ranks is then the mean's E^1 term).  Backward (Horner on G' = dL/dfinal
// / (K+1)): [sum G'_I | H^1_I] then [H^2_I | item gradient] (K = 3) or the item gradient
// (K = 2); every item partial adds the rank's own G'_I, so the sums carry G'_I once.
// 4 collectives per step at K = 3 (3 at K = 2) instead of 2K+1, the same bytes; the
// summed halves are copied to the layer buffers the next products read.
int sharded_fused_rounds(const rsx_sharded_lgcn_step& st, hipStream_t s) {
    const int d = st.d, K = st.n_layers;
    const int64_t nu = st.n_users, ni = st.n_items, off = nu * (int64_t)d, X = ni * (int64_t)d;
    const bool root = st.comm->rank == 0;
    const float beta = 1.f / (float)(K + 1);
    const int32_t tag = (int32_t)st.tag;
    float* A = st.xch;
    float* B = st.xch + X;
    int rc = 0;
    auto copy = [&](float* dst, const float* src) -> int {
        return hip_rc(hipMemcpyAsync(dst, src, (size_t)X * sizeof(float), hipMemcpyDeviceToDevice, s));
    };
    auto tags = [&](rsx_epilogue& e, int flags) {
        e.row_tag = st.row_tag;
        e.tag = tag;
        e.tag_dev = st.tag_dev;
        e.tag_flags = flags;
    };
    // ---- forward
    {
        rsx_epilogue e = epi(RSX_EPI_STORE);  // E^1 item partial (this launch also tags the batch rows)
        e.y = A;
        TagJob tj;
        tj.trip = st.triplets;
        tj.batch = st.batch;
        tj.n_users = nu;
        tj.row_tag = st.row_tag;
        tj.tag = tag;
        tj.tag_dev = st.tag_dev;
        RSX_TRY(spmm_dispatch_tagging(*st.adj_i, st.p, d, e, st.slab_i, s, tj));
        rsx_epilogue u = epi(RSX_EPI_STORE);  // E^1 user rows (local: E^0 items are replicated)
        u.y = st.h0;
        RSX_TRY(spmm_dispatch(*st.adj_u, st.p, d, u, st.slab_u, s));
    }
    if (K == 3) {
        rsx_epilogue e = epi(RSX_EPI_STORE);  // E^2 item partial from the own E^1 user rows
        e.y = B;
        RSX_TRY(spmm_dispatch(*st.adj_i, st.h0, d, e, st.slab_i, s));
        hipEvent_t j1 = exchange(st.comm, A, 2 * X, s, &rc);
        if (!j1) return rc;
        RSX_TRY(wait(s, j1));
        RSX_TRY(copy(st.h0 + off, A));  // E^1 items
        RSX_TRY(copy(st.h1 + off, B));  // E^2 items
        rsx_epilogue u = epi(RSX_EPI_STORE);  // E^2 user rows
        u.y = st.h1;
        RSX_TRY(spmm_dispatch(*st.adj_u, st.h0, d, u, st.slab_u, s));
        rsx_epilogue f = epi(RSX_EPI_FINAL);  // final item partial; rank 0 adds the summed E^0..E^2 rows
        f.beta = beta;
        f.f = st.final_emb + off;
        if (root) {
            f.s_in = st.p + off;
            f.r_add = st.h0 + off;
            f.aux = st.h1 + off;
        }
        RSX_TRY(spmm_dispatch(*st.adj_i, st.h1, d, f, st.slab_i, s));
        hipEvent_t j2 = exchange(st.comm, st.final_emb + off, X, s, &rc);
        if (!j2) return rc;
        rsx_epilogue fu = epi(RSX_EPI_FINAL);  // final user rows, batch rows only
        fu.beta = beta;
        fu.f = st.final_emb;
        fu.s_in = st.p;
        fu.r_add = st.h0;
        fu.aux = st.h1;
        tags(fu, RSX_TAG_ROWS);
        RSX_TRY(spmm_dispatch(*st.adj_u, st.h1, d, fu, st.slab_u, s));
        RSX_TRY(wait(s, j2));
    } else {
        rsx_epilogue f = epi(RSX_EPI_FINAL);  // final item partial: (rank 0: E^0) + own E^1 partial + own E^2 partial
        f.beta = beta;
        f.f = B;
        if (root) f.s_in = st.p + off;
        f.r_add = A;
        RSX_TRY(spmm_dispatch(*st.adj_i, st.h0, d, f, st.slab_i, s));
        hipEvent_t j1 = exchange(st.comm, A, 2 * X, s, &rc);
        if (!j1) return rc;
        RSX_TRY(wait(s, j1));
        RSX_TRY(copy(st.h0 + off, A));             // E^1 items
        RSX_TRY(copy(st.final_emb + off, B));      // the final item rows
        rsx_epilogue fu = epi(RSX_EPI_FINAL);
        fu.beta = beta;
        fu.f = st.final_emb;
        fu.s_in = st.p;
        fu.r_add = st.h0;
        tags(fu, RSX_TAG_ROWS);
        RSX_TRY(spmm_dispatch(*st.adj_u, st.h0, d, fu, st.slab_u, s));
    }
    // ---- loss: G' (this rank's batch rows), R (counts with reg_cnt)
    const float* reg_k = st.reg_cnt ? reinterpret_cast<const float*>(st.reg_cnt + 3 * (nu + ni) + 1) : nullptr;
    if (st.reg_cnt)
        RSX_TRY(bpr_fused_call(st.final_emb, st.p, nu, ni, d, st.triplets, st.batch, st.reg, (float)(K + 1), st.g,
                               st.reg_cnt, st.loss_out, st.loss_acc, st.ws, st.ws_bytes, s));
    else
        RSX_TRY(bpr_call(RSX_BPR_LIGHTGCN, st.final_emb, st.p, nu, ni, d, st.triplets, st.batch, st.reg,
                         (float)st.batch, st.g, st.r, st.loss_out, st.loss_acc, st.ws, st.ws_bytes, s,
                         (float)(K + 1)));
    // ---- backward round 1: [sum G'_I | H^1_I = sum (G'_I + A_I G'_U)]
    RSX_TRY(copy(A, st.g + off));
    {
        rsx_epilogue e = epi(RSX_EPI_ADD);
        e.y = B;
        e.s_in = st.g + off;  // own G'_I
        tags(e, RSX_TAG_SPARSE_X);  // X = G': this rank's batch users only
        RSX_TRY(spmm_dispatch(*st.adj_i, st.g, d, e, st.slab_i, s));
    }
    hipEvent_t b1 = exchange(st.comm, A, 2 * X, s, &rc);
    if (!b1) return rc;
    RSX_TRY(wait(s, b1));
    RSX_TRY(copy(st.h1 + off, A));  // sum G'_I (h1's item rows are free in the backward)
    RSX_TRY(copy(st.h0 + off, B));  // H^1_I
    auto h_users = [&](float* y, const float* x) -> int {  // H users = G'_U + A_U (x's item rows)
        rsx_epilogue u = epi(RSX_EPI_ADD);
        u.y = y;
        u.s_in = st.g;
        tags(u, RSX_TAG_SPARSE_S);
        return spmm_dispatch(*st.adj_u, x, d, u, st.slab_u, s);
    };
    auto item_grad = [&](float* y, const float* x) -> int {  // own G'_I + A_I (x's user rows) + own R_I
        rsx_epilogue e = epi(RSX_EPI_ADD);
        e.y = y;
        e.s_in = st.g + off;
        if (st.reg_cnt) {  // own R_I from the counts (cleared here)
            e.reg_cnt = st.reg_cnt + 3 * nu;
            e.reg_k = reg_k;
            e.p = st.p + off;
        } else {
            e.r_add = st.r + off;
        }
        return spmm_dispatch(*st.adj_i, x, d, e, st.slab_i, s);
    };
    RSX_TRY(h_users(st.h0, st.h1));  // H^1_U = G'_U + A_U sum G'_I
    const float* gI;                  // the summed item gradient
    const float* xa;                  // the buffer whose item rows the user Adam layer reads
    if (K == 3) {
        RSX_TRY(h_users(st.h1, st.h0));  // H^2_U = G'_U + A_U H^1_I (h1's item rows: sum G'_I, read above)
        rsx_epilogue e = epi(RSX_EPI_ADD);  // H^2_I partial: own G'_I + A_I H^1_U
        e.y = A;
        e.s_in = st.g + off;
        RSX_TRY(spmm_dispatch(*st.adj_i, st.h0, d, e, st.slab_i, s));
        RSX_TRY(item_grad(B, st.h1));  // own G'_I + A_I H^2_U + own R_I
        hipEvent_t b2 = exchange(st.comm, A, 2 * X, s, &rc);
        if (!b2) return rc;
        RSX_TRY(wait(s, b2));
        RSX_TRY(copy(st.h1 + off, A));  // H^2_I
        gI = B;
        xa = st.h1;
    } else {
        RSX_TRY(item_grad(A, st.h0));  // own G'_I + A_I H^1_U + own R_I
        hipEvent_t b2 = exchange(st.comm, A, X, s, &rc);
        if (!b2) return rc;
        RSX_TRY(wait(s, b2));
        gI = A;
        xa = st.h0;
    }
    {
        rsx_epilogue u = epi(RSX_EPI_ADAM);  // user rows: g = (G'_U + A_U H^{K-1}_I) + R_U
        u.s_in = st.g;
        u.r_add = st.r;
        u.p = st.p;
        u.m = st.m;
        u.v = st.v;
        u.adam = st.adam;
        u.zero0 = st.g;
        u.zero1 = st.r;
        if (st.reg_cnt) {
            u.r_add = nullptr;
            u.zero1 = nullptr;
            u.reg_cnt = st.reg_cnt;
            u.reg_k = reg_k;
        }
        tags(u, RSX_TAG_SPARSE_S | RSX_TAG_SPARSE_R | RSX_TAG_ZERO);
        RSX_TRY(spmm_dispatch(*st.adj_u, xa, d, u, st.slab_u, s));
        rsx_epilogue a = epi(RSX_EPI_ADAM);  // item rows, identical on every rank
        a.s_in = gI;
        a.p = st.p + off;
        a.m = st.m + off;
        a.v = st.v + off;
        a.adam = st.adam;
        a.zero0 = st.g + off;  // own G'_I and R_I: cleared densely
        a.zero1 = st.reg_cnt ? nullptr : st.r + off;
        RSX_TRY(rowwise_dispatch(ni, d, a, s));
    }
    return 0;
}

bool valid(const rsx_sharded_lgcn_step* st) {
    if (!st || !st->adj_u || !st->adj_i || !st->comm || !st->p || !st->final_emb || st->n_layers < 1 ||
        st->n_layers > 30 || st->n_users < 0 || st->n_items <= 0)
        return false;
    if (st->adj_u->n_rows != st->n_users || st->adj_i->n_rows != st->n_items) return false;
    if (st->adj_u->n_cols != st->n_users + st->n_items || st->adj_i->n_cols != st->n_users + st->n_items) return false;
    if (st->n_layers >= 2 && (!st->s || !st->h0 || !st->h1)) return false;
    if (st->n_layers == 1 && !st->h0) return false;
    if ((st->adj_u->n_long > 0 && !st->slab_u) || (st->adj_i->n_long > 0 && !st->slab_i)) return false;
    if (st->union_items) {
        const int64_t w = st->comm->world;
        if (!st->item_tag || !st->cbuf0 || !st->cbuf1 || st->n_items_pad < st->n_items || st->n_items_pad % w ||
            st->union_cap < st->batch ||
            !st->row_tag || (st->n_layers != 2 && st->n_layers != 3) || st->d % 4)
            return false;
    }
    if (st->nbr_items && (!st->union_items || !st->nbr_count || !st->cbufN || st->nbr_cap < 2 * st->union_cap))
        return false;
    if (st->n_head > 1) {  // the head pieces tile adj_i's rows in order
        if (!st->head_i || !st->head_row0 || !st->head_slab || st->head_row0[0] != 0 ||
            st->head_row0[st->n_head] != st->n_items)
            return false;
        for (int32_t p = 0; p < st->n_head; ++p) {
            const rsx_csr& h = st->head_i[p];
            if (st->head_row0[p + 1] <= st->head_row0[p] || h.n_rows != st->head_row0[p + 1] - st->head_row0[p] ||
                h.n_cols != st->adj_i->n_cols || h.col != st->adj_i->col || h.val != st->adj_i->val ||
                (h.n_long > 0 && !st->head_slab[p]))
                return false;
        }
    }
    return true;
}

}  // namespace
}  // namespace rsx

extern "C" {

size_t rsx_comm_unique_id_bytes(void) { return sizeof(ncclUniqueId); }

int rsx_comm_get_unique_id(void* id_host) {
    if (!id_host) return RSX_ERR_ARG;
    if (!rsx::rccl().ok) return RSX_ERR_COMM;
    ncclUniqueId id;
    if (rsx::rccl().get_unique_id(&id) != ncclSuccess) return RSX_ERR_COMM;
    memcpy(id_host, &id, sizeof(id));
    return RSX_OK;
}

int rsx_comm_init(rsx_comm_t* out, const void* id_host, int32_t rank, int32_t world) {
    if (!out || !id_host || world < 1 || rank < 0 || rank >= world) return RSX_ERR_ARG;
    if (!rsx::rccl().ok) return RSX_ERR_COMM;
    rsx_comm_s* c = new rsx_comm_s();
    c->rank = rank;
    c->world = world;
    ncclUniqueId id;
    memcpy(&id, id_host, sizeof(id));
    hipError_t e = rsx::comm_streams_create(c);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork, hipEventDisableTiming);
    for (int i = 0; e == hipSuccess && i < rsx::kJoinEvents; ++i)
        e = hipEventCreateWithFlags(&c->join[i], hipEventDisableTiming);
    if (e != hipSuccess) {
        rsx_comm_destroy(c);
        return rsx::hip_rc(e);
    }
    if (rsx::rccl().init_rank(&c->nccl, world, id, rank) != ncclSuccess) {
        c->nccl = nullptr;
        rsx_comm_destroy(c);
        return RSX_ERR_COMM;
    }
    *out = c;
    return RSX_OK;
}

int rsx_comm_init_host(rsx_comm_t* out, int32_t rank, int32_t world, rsx_host_collective_fn fn, void* ctx) {
    if (!out || !fn || world < 1 || rank < 0 || rank >= world) return RSX_ERR_ARG;
    rsx_comm_s* c = new rsx_comm_s();
    c->rank = rank;
    c->world = world;
    c->host_fn = fn;
    c->host_ctx = ctx;
    hipError_t e = hipSuccess;
    for (int i = 0; e == hipSuccess && i < rsx::kJoinEvents; ++i)
        e = hipEventCreateWithFlags(&c->join[i], hipEventDisableTiming);
    if (e != hipSuccess) {
        rsx_comm_destroy(c);
        return rsx::hip_rc(e);
    }
    *out = c;
    return RSX_OK;
}

int rsx_comm_init_sim(rsx_comm_t* out, int32_t sim_world, double busbw_gbs, double latency_us, int32_t blocks,
                      int64_t scratch_mb) {
    if (!out || sim_world < 2 || busbw_gbs <= 0 || latency_us < 0 || blocks < 1 || scratch_mb < 1)
        return RSX_ERR_ARG;
    rsx_comm_s* c = new rsx_comm_s();
    c->rank = 0;
    c->world = 1;
    c->sim_world = sim_world;
    c->sim_busbw = busbw_gbs * 1e9;
    c->sim_lat = latency_us * 1e-6;
    c->sim_blocks = blocks;
    int dev = 0, khz = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
    c->sim_tick_hz = (khz > 0 ? khz : 100000) * 1e3;
    c->sim_scratch_floats = scratch_mb * (1 << 20) / 4;
    if (e == hipSuccess) e = hipMalloc(&c->sim_scratch, (size_t)c->sim_scratch_floats * 4);
    if (e == hipSuccess) e = hipMemset(c->sim_scratch, 0, (size_t)c->sim_scratch_floats * 4);
    c->sim_poison = (int32_t)rsx::env_knob("RSX_COMM_SIM_POISON", 0, 0, 1);
    if (e == hipSuccess && c->sim_poison) e = hipMalloc(&c->sim_save, (size_t)(c->sim_scratch_floats / 2) * 4);
    if (e == hipSuccess) e = rsx::comm_streams_create(c);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork, hipEventDisableTiming);
    for (int i = 0; e == hipSuccess && i < rsx::kJoinEvents; ++i)
        e = hipEventCreateWithFlags(&c->join[i], hipEventDisableTiming);
    if (e != hipSuccess) {
        rsx_comm_destroy(c);
        return rsx::hip_rc(e);
    }
    *out = c;
    return RSX_OK;
}

double rsx_comm_sim_seconds(rsx_comm_t c, int32_t op, double bytes) {
    if (!c || !c->sim_world) return -1.0;
    return rsx::sim_seconds(c, op, bytes);
}

int rsx_comm_destroy(rsx_comm_t c) {
    if (!c) return RSX_OK;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->stream_cap) (void)hipStreamSynchronize(c->stream_cap);
    if (c->sim_scratch) (void)hipFree(c->sim_scratch);
    if (c->sim_save) (void)hipFree(c->sim_save);
    // diagnosis only (tools/gpu/diag_priority3.py): leak the comm stream (1),
    // the RCCL communicator (2) or the fork / join events (4) instead of destroying them
    const int keep = rsx::env_knob("RSX_COMM_DIAG_KEEP", 0, 0, 7);
    if (c->nccl && !(keep & 2)) rsx::rccl().destroy(c->nccl);
    for (int i = 0; i < rsx::kJoinEvents; ++i)
        if (c->join[i] && !(keep & 4)) (void)hipEventDestroy(c->join[i]);
    if (c->fork && !(keep & 4)) (void)hipEventDestroy(c->fork);
    if (c->stream && !(keep & 1)) (void)hipStreamDestroy(c->stream);
    if (c->stream_cap) (void)hipStreamDestroy(c->stream_cap);
    delete c;
    return RSX_OK;
}

int rsx_comm_allreduce_f32(rsx_comm_t c, float* buf, int64_t n, rsx_stream_t stream) {
    if (!c || (!buf && n > 0) || n < 0) return RSX_ERR_ARG;
    int rc = 0;
    hipStream_t s = rsx::as_stream(stream);
    hipEvent_t j = rsx::exchange(c, buf, n, s, &rc);
    if (!j) return rc;
    return rsx::wait(s, j);
}

int rsx_comm_allreduce_f32_start(rsx_comm_t c, float* buf, int64_t n, rsx_stream_t stream) {
    if (!c || (!buf && n > 0) || n < 0) return RSX_ERR_ARG;
    if (c->pending) return RSX_ERR_ARG;  // one exchange in flight: every start pairs with one rsx_comm_wait
    int rc = 0;
    hipEvent_t j = rsx::exchange(c, buf, n, rsx::as_stream(stream), &rc);
    if (!j) return rc;
    c->pending = j;
    return RSX_OK;
}

int rsx_comm_wait(rsx_comm_t c, rsx_stream_t stream) {
    if (!c) return RSX_ERR_ARG;
    if (!c->pending) return RSX_OK;
    const int rc = rsx::wait(rsx::as_stream(stream), c->pending);
    c->pending = nullptr;
    return rc;
}

int rsx_comm_allgather_f32(rsx_comm_t c, float* buf, int64_t count, rsx_stream_t stream) {
    if (!c || (!buf && count > 0) || count < 0) return RSX_ERR_ARG;
    int rc = 0;
    hipStream_t s = rsx::as_stream(stream);
    hipEvent_t j = rsx::collective(c, RSX_COLL_ALLGATHER, buf, count, RSX_COLL_F32, s, &rc);
    if (!j) return rc;
    return rsx::wait(s, j);
}

int rsx_sharded_lightgcn_forward(const rsx_sharded_lgcn_step* st, rsx_stream_t stream) {
    if (!rsx::valid(st)) return RSX_ERR_ARG;
    if (st->row_tag && (st->n_layers == 2 || st->n_layers == 3))
        return rsx::sharded_stored_layers(*st, false, rsx::as_stream(stream));
    return rsx::sharded_forward(*st, false, rsx::as_stream(stream));
}

int rsx_sharded_lightgcn_flush(const rsx_sharded_lgcn_step* st, rsx_stream_t stream) {
    using namespace rsx;
    if (!valid(st)) return RSX_ERR_ARG;
    if (!st->union_items || !st->defer_ag) return RSX_OK;  // nothing is ever deferred
    hipStream_t s = as_stream(stream);
    int rc = 0;
    const int64_t q = st->n_items_pad / st->comm->world;
    hipEvent_t j = collective(st->comm, RSX_COLL_ALLGATHER, st->p + st->n_users * (int64_t)st->d, q * st->d,
                              RSX_COLL_F32, s, &rc);
    if (!j) return rc;
    return wait(s, j);
}

int rsx_sharded_lightgcn_step(const rsx_sharded_lgcn_step* st, rsx_stream_t stream) {
    using namespace rsx;
    if (!valid(st) || !st->m || !st->v || !st->g || !st->r || !st->t || !st->triplets || st->batch <= 0)
        return RSX_ERR_ARG;
    hipStream_t s = as_stream(stream);
    const int d = st->d, K = st->n_layers;
    if (st->row_tag && (K == 2 || K == 3)) {
        if (!st->tag_dev && (st->tag <= 0 || st->tag > INT32_MAX)) return RSX_ERR_ARG;
        if (st->xch && !st->union_items) return sharded_fused_rounds(*st, s);
        return sharded_stored_layers(*st, true, s);
    }
    const int64_t nu = st->n_users, ni = st->n_items, off = nu * (int64_t)d;
    const float beta = 1.f / (float)(K + 1);
    RSX_TRY(sharded_forward(*st, true, s));
    RSX_TRY(bpr_call(RSX_BPR_LIGHTGCN, st->final_emb, st->p, nu, ni, d, st->triplets, st->batch, st->reg,
                     (float)st->batch, st->g, st->r, st->loss_out, st->loss_acc, st->ws, st->ws_bytes, s));
    // backward: the same layer sums on H^0 = G = dL/dfinal (rsx/dist.py:step)
    float* bufs[2] = {st->h0, st->h1};
    auto ys = [&](int k) -> float* { return k == 0 ? st->g : bufs[(k - 1) & 1]; };
    hipEvent_t joins[64] = {};
    int rc = 0;
    hipEvent_t j0 = exchange(st->comm, st->g + off, ni * d, s, &rc);  // G's item rows: per-rank partials
    if (!j0) return rc;
    auto item_partial = [&](int k) -> int {
        if (k < K) {
            rsx_epilogue e = epi(RSX_EPI_STORE);
            e.y = ys(k) + off;
            RSX_TRY(spmm_dispatch(*st->adj_i, ys(k - 1), d, e, st->slab_i, s));
            joins[k] = exchange(st->comm, ys(k) + off, ni * d, s, &rc);
        } else {  // t = H_I^K/(K+1) + R_I: this rank's share of the item gradient beyond s_I/(K+1)
            rsx_epilogue e = epi(RSX_EPI_ADD);
            e.alpha = beta;
            e.y = st->t;
            e.r_add = st->r + off;
            RSX_TRY(spmm_dispatch(*st->adj_i, ys(k - 1), d, e, st->slab_i, s));
            joins[k] = exchange(st->comm, st->t, ni * d, s, &rc);
        }
        return joins[k] ? 0 : rc;
    };
    RSX_TRY(item_partial(1));
    RSX_TRY(wait(s, j0));
    for (int k = 1; k <= K; ++k) {
        const float* s_in = k == 1 ? st->g : st->s;
        if (k < K) {
            rsx_epilogue e = epi(RSX_EPI_LAYERSUM);
            e.y = ys(k);
            e.s_in = s_in;
            e.s_out = st->s;
            RSX_TRY(spmm_dispatch(*st->adj_u, ys(k - 1), d, e, st->slab_u, s));
            RSX_TRY(item_partial(k + 1));
            RSX_TRY(wait(s, joins[k]));
            rsx_epilogue a = epi(RSX_EPI_ADD);
            a.y = st->s + off;
            a.s_in = s_in + off;
            a.r_add = ys(k) + off;
            RSX_TRY(rowwise_dispatch(ni, d, a, s));
        } else {
            rsx_epilogue e = epi(RSX_EPI_ADAM);
            e.beta = beta;
            e.adam = st->adam;
            e.s_in = s_in;
            e.r_add = st->r;
            e.p = st->p;
            e.m = st->m;
            e.v = st->v;
            RSX_TRY(spmm_dispatch(*st->adj_u, ys(k - 1), d, e, st->slab_u, s));
            RSX_TRY(wait(s, joins[k]));
            rsx_epilogue a = epi(RSX_EPI_ADAM);
            a.beta = beta;
            a.adam = st->adam;
            a.s_in = s_in + off;
            a.r_add = st->t;
            a.p = st->p + off;
            a.m = st->m + off;
            a.v = st->v + off;
            RSX_TRY(rowwise_dispatch(ni, d, a, s));
        }
    }
    return 0;
}

}  // extern "C"

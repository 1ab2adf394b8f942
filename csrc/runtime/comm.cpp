// Native gradient-communication engine: RCCL over xGMI on a dedicated HIP stream
// (SURVEY T-L0c / N6).
//
// One Engine per process (one process per GPU).  The Python reducer hands it
// contiguous slices of the flat gradient arena ("buckets") as they become
// ready during backward:
//
//   allreduce(buf)  : event on the compute stream -> comm stream waits on it ->
//                     ncclAllReduce on the comm stream.  No host sync: the
//                     collective runs under the rest of backward.
//   wait()          : event on the comm stream -> the compute stream waits on it
//                     (the optimizer launched afterwards sees reduced grads).
//
// RCCL is resolved with dlopen/dlsym from the library path the caller passes
// (the librccl.so PyTorch itself loaded), so the process holds a single RCCL
// instance whichever ROCm install the headers came from.  Only the RCCL types
// are taken from <rccl/rccl.h>.
//
// Failure detection: every collective records a start event and a host
// launch time; ddl_comm_async_error() surfaces RCCL's asynchronous error state and
// ddl_comm_oldest_pending_ms() how long the oldest unfinished collective has been on the
// comm stream.  The Python watchdog (parallel/comm.py) polls both from a thread and calls
// ddl_comm_abort() (ncclCommAbort: RCCL kernels stuck on a dead peer return) when a peer
// fails or a collective exceeds its timeout; every later call then fails with the reason.
// ddl_comm_collective_ms() reads a finished collective's device time (per-bucket timing).
//
// The reference has no communication layer at all; BASELINE.json
// mandates "data-parallel all-reduce ... RCCL ring/tree over xGMI ... overlapped
// with backward on HIP streams".
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#define DDL_API extern "C" __attribute__((visibility("default")))

namespace {

struct Rccl {
    void* so = nullptr;
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclCommAbort) commAbort = nullptr;
    decltype(&ncclAllReduce) allReduce = nullptr;
    decltype(&ncclBroadcast) broadcast = nullptr;
    decltype(&ncclReduceScatter) reduceScatter = nullptr;
    decltype(&ncclAllGather) allGather = nullptr;
    decltype(&ncclGroupStart) groupStart = nullptr;
    decltype(&ncclGroupEnd) groupEnd = nullptr;
    decltype(&ncclGetErrorString) errorString = nullptr;
    decltype(&ncclCommGetAsyncError) getAsyncError = nullptr;   // optional
};

Rccl g_rccl;
std::mutex g_mu;
char g_err[512] = {0};

void set_err(const char* what, const char* detail) {
    std::snprintf(g_err, sizeof(g_err), "%s: %s", what, detail ? detail : "");
}

template <typename F>
bool sym(F& f, const char* name) {
    f = reinterpret_cast<F>(dlsym(g_rccl.so, name));
    if (!f) set_err("dlsym", name);
    return f != nullptr;
}

bool load_rccl(const char* path) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_rccl.so) return true;
    void* so = dlopen(path && *path ? path : "librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!so) {
        set_err("dlopen", dlerror());
        return false;
    }
    g_rccl.so = so;
    return sym(g_rccl.getUniqueId, "ncclGetUniqueId") && sym(g_rccl.commInitRank, "ncclCommInitRank") &&
           sym(g_rccl.commDestroy, "ncclCommDestroy") && sym(g_rccl.commAbort, "ncclCommAbort") &&
           sym(g_rccl.allReduce, "ncclAllReduce") && sym(g_rccl.broadcast, "ncclBroadcast") &&
           sym(g_rccl.reduceScatter, "ncclReduceScatter") && sym(g_rccl.allGather, "ncclAllGather") &&
           sym(g_rccl.groupStart, "ncclGroupStart") && sym(g_rccl.groupEnd, "ncclGroupEnd") &&
           sym(g_rccl.errorString, "ncclGetErrorString") &&
           (g_rccl.getAsyncError = reinterpret_cast<decltype(&ncclCommGetAsyncError)>(
                dlsym(g_rccl.so, "ncclCommGetAsyncError")), true);
}

bool ok(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return true;
    set_err(what, g_rccl.errorString ? g_rccl.errorString(r) : "rccl error");
    return false;
}

bool hok(hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    set_err(what, hipGetErrorString(e));
    return false;
}

ncclDataType_t dtype_of(int code) {
    switch (code) {
        case 0: return ncclBfloat16;
        case 1: return ncclFloat32;
        case 2: return ncclFloat16;
        case 3: return ncclInt64;
        default: return ncclInt32;
    }
}

constexpr int RING = 64;
using Clock = std::chrono::steady_clock;

struct Engine {
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;    // collectives run here, concurrent with compute
    hipEvent_t produced = nullptr;   // compute -> comm ordering
    hipEvent_t drained = nullptr;    // comm -> compute ordering
    hipEvent_t start[RING] = {};     // start[i % RING] / done[i % RING]: around collective number i + 1
    hipEvent_t done[RING] = {};
    Clock::time_point t_launch[RING];
    int rank = 0, world = 1, device = 0;
    long launched = 0;
    long finished = 0;               // every collective numbered <= finished is known complete
    long bytes = 0;
    int injected = 0;                // test hook: reported as the async error
    bool aborted = false;
    std::mutex mu;                   // API calls vs the watchdog thread's abort
};

// collective number e->launched + 1 is about to go onto the comm stream
bool mark_start(Engine* e) {
    const long i = e->launched % RING;
    e->t_launch[i] = Clock::now();
    return hok(hipEventRecord(e->start[i], e->stream), "hipEventRecord");
}

// all-reduce number e->launched just went onto the comm stream: mark its completion
bool mark_done(Engine* e) {
    return hok(hipEventRecord(e->done[(e->launched - 1) % RING], e->stream), "hipEventRecord");
}

bool usable(Engine* e) {
    if (e->aborted || !e->comm) {
        set_err("comm", "communicator aborted");
        return false;
    }
    return true;
}

// compute stream -> comm stream dependency (the event is re-recorded per call;
// hipStreamWaitEvent binds to the record that precedes it)
bool order_after(Engine* e, hipStream_t compute) {
    return hok(hipEventRecord(e->produced, compute), "hipEventRecord") &&
           hok(hipStreamWaitEvent(e->stream, e->produced, 0), "hipStreamWaitEvent");
}

}  // namespace

DDL_API const char* ddl_comm_last_error() { return g_err; }

DDL_API int ddl_comm_unique_id(const char* rccl_path, char* out) {
    if (!load_rccl(rccl_path)) return -1;
    ncclUniqueId id;
    if (!ok(g_rccl.getUniqueId(&id), "ncclGetUniqueId")) return -2;
    std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return 0;
}

DDL_API void* ddl_comm_create(const char* rccl_path, const char* id_bytes, int world, int rank, int device) {
    if (!load_rccl(rccl_path)) return nullptr;
    if (!hok(hipSetDevice(device), "hipSetDevice")) return nullptr;
    Engine* e = new Engine();
    e->rank = rank;
    e->world = world;
    e->device = device;
    int lo = 0, hi = 0;
    // highest priority: gradient rings should not queue behind backward GEMMs
    if (!hok(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange") ||
        !hok(hipStreamCreateWithPriority(&e->stream, hipStreamNonBlocking, hi), "hipStreamCreateWithPriority") ||
        !hok(hipEventCreateWithFlags(&e->produced, hipEventDisableTiming), "hipEventCreate") ||
        !hok(hipEventCreateWithFlags(&e->drained, hipEventDisableTiming), "hipEventCreate")) {
        delete e;
        return nullptr;
    }
    for (int i = 0; i < RING; ++i)
        if (!hok(hipEventCreate(&e->start[i]), "hipEventCreate") || !hok(hipEventCreate(&e->done[i]), "hipEventCreate")) {
            delete e;
            return nullptr;
        }
    ncclUniqueId id;
    std::memcpy(id.internal, id_bytes, NCCL_UNIQUE_ID_BYTES);
    if (!ok(g_rccl.commInitRank(&e->comm, world, id, rank), "ncclCommInitRank")) {
        hipStreamDestroy(e->stream);
        delete e;
        return nullptr;
    }
    return e;
}

DDL_API int ddl_comm_allreduce(void* h, void* buf, long count, int dtype, int avg, hipStream_t compute) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || count <= 0) return count == 0 ? 0 : -1;
    std::lock_guard<std::mutex> lk(e->mu);
    if (!usable(e)) return -4;
    if (!order_after(e, compute) || !mark_start(e)) return -3;
    if (!ok(g_rccl.allReduce(buf, buf, (size_t)count, dtype_of(dtype), avg ? ncclAvg : ncclSum, e->comm, e->stream),
            "ncclAllReduce"))
        return -2;
    e->launched += 1;
    e->bytes += count * (dtype == 1 || dtype >= 4 ? 4 : dtype == 3 ? 8 : 2);
    return mark_done(e) ? 0 : -3;
}

// several buckets that became ready together: one fused RCCL group launch
DDL_API int ddl_comm_allreduce_many(void* h, void** bufs, const long* counts, int n, int dtype, int avg,
                                    hipStream_t compute) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    std::lock_guard<std::mutex> lk(e->mu);
    if (!usable(e)) return -4;
    if (!order_after(e, compute)) return -3;
    const long before = e->launched;
    // one start mark per member, all at the group's stream position
    for (int i = 0, k = 0; i < n; ++i) {
        if (counts[i] <= 0) continue;
        const long slot = (before + k++) % RING;
        e->t_launch[slot] = Clock::now();
        if (!hok(hipEventRecord(e->start[slot], e->stream), "hipEventRecord")) return -3;
    }
    if (!ok(g_rccl.groupStart(), "ncclGroupStart")) return -2;
    for (int i = 0; i < n; ++i) {
        if (counts[i] <= 0) continue;
        if (!ok(g_rccl.allReduce(bufs[i], bufs[i], (size_t)counts[i], dtype_of(dtype), avg ? ncclAvg : ncclSum,
                                 e->comm, e->stream),
                "ncclAllReduce")) {
            g_rccl.groupEnd();
            return -2;
        }
        e->launched += 1;
    }
    if (!ok(g_rccl.groupEnd(), "ncclGroupEnd")) return -2;
    // every number of the group completes at the same point of the comm stream
    for (long k = before; k < e->launched; ++k)
        if (!hok(hipEventRecord(e->done[k % RING], e->stream), "hipEventRecord")) return -3;
    return 0;
}

DDL_API int ddl_comm_broadcast(void* h, void* buf, long count, int dtype, int root, hipStream_t compute) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    std::lock_guard<std::mutex> lk(e->mu);
    if (!usable(e)) return -4;
    if (!order_after(e, compute)) return -3;
    if (!ok(g_rccl.broadcast(buf, buf, (size_t)count, dtype_of(dtype), root, e->comm, e->stream), "ncclBroadcast"))
        return -2;
    return 0;
}

// reduce-scatter / all-gather (ZeRO-1 buckets) are numbered with the all-reduces, so
// ddl_comm_wait_upto covers them: the optimizer waits on one bucket's shard, the next
// forward on one bucket's gathered parameters
DDL_API int ddl_comm_reduce_scatter(void* h, const void* send, void* recv, long recv_count, int dtype, int avg,
                                    hipStream_t compute) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || recv_count <= 0) return recv_count == 0 ? 0 : -1;
    std::lock_guard<std::mutex> lk(e->mu);
    if (!usable(e)) return -4;
    if (!order_after(e, compute) || !mark_start(e)) return -3;
    if (!ok(g_rccl.reduceScatter(send, recv, (size_t)recv_count, dtype_of(dtype), avg ? ncclAvg : ncclSum, e->comm,
                                 e->stream),
            "ncclReduceScatter"))
        return -2;
    e->launched += 1;
    e->bytes += recv_count * e->world * (dtype == 1 || dtype >= 4 ? 4 : dtype == 3 ? 8 : 2);
    return mark_done(e) ? 0 : -3;
}

DDL_API int ddl_comm_all_gather(void* h, const void* send, void* recv, long send_count, int dtype,
                                hipStream_t compute) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || send_count <= 0) return send_count == 0 ? 0 : -1;
    std::lock_guard<std::mutex> lk(e->mu);
    if (!usable(e)) return -4;
    if (!order_after(e, compute) || !mark_start(e)) return -3;
    if (!ok(g_rccl.allGather(send, recv, (size_t)send_count, dtype_of(dtype), e->comm, e->stream), "ncclAllGather"))
        return -2;
    e->launched += 1;
    e->bytes += send_count * e->world * (dtype == 1 || dtype >= 4 ? 4 : dtype == 3 ? 8 : 2);
    return mark_done(e) ? 0 : -3;
}

// compute stream waits for every collective issued so far
DDL_API int ddl_comm_wait(void* h, hipStream_t compute) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    std::lock_guard<std::mutex> lk(e->mu);
    if (!usable(e)) return -4;
    return hok(hipEventRecord(e->drained, e->stream), "hipEventRecord") &&
                   hok(hipStreamWaitEvent(compute, e->drained, 0), "hipStreamWaitEvent")
               ? 0
               : -3;
}

// compute stream waits for collective number `seq` (all-reduce / reduce-scatter / all-gather; 1-based, as counted by ddl_comm_stats(h, 0))
// and, the comm stream being in order, everything issued before it.  A number more than
// RING behind the newest waits for a later one instead (still correct, just later).
DDL_API int ddl_comm_wait_upto(void* h, long seq, hipStream_t compute) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    std::lock_guard<std::mutex> lk(e->mu);
    if (!usable(e)) return -4;
    if (seq < 1 || seq > e->launched) return -1;
    if (e->launched - seq >= RING) seq = e->launched;
    return hok(hipStreamWaitEvent(compute, e->done[(seq - 1) % RING], 0), "hipStreamWaitEvent") ? 0 : -3;
}

DDL_API int ddl_comm_synchronize(void* h) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        if (!usable(e)) return -4;
    }
    // (not under the lock: the watchdog must be able to abort a synchronize stuck on a dead peer)
    return hok(hipStreamSynchronize(e->stream), "hipStreamSynchronize") ? 0 : -3;
}

// RCCL's asynchronous error state of the communicator: 0 = fine (ncclInProgress counts as
// fine), otherwise the ncclResult_t code; -4 after an abort.  Thread-safe (the watchdog).
DDL_API int ddl_comm_async_error(void* h) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    std::lock_guard<std::mutex> lk(e->mu);
    if (e->aborted || !e->comm) return -4;
    if (e->injected) return e->injected;
    if (!g_rccl.getAsyncError) return 0;
    ncclResult_t r = ncclSuccess;
    if (g_rccl.getAsyncError(e->comm, &r) != ncclSuccess) return (int)ncclInternalError;
    return (r == ncclSuccess || r == ncclInProgress) ? 0 : (int)r;
}

// Milliseconds the oldest collective that has not finished has been on the comm stream
// (host clock since its launch call), -1 if every collective finished.  Only the RING newest
// are tracked: older ones count as finished (their events were recycled).
DDL_API double ddl_comm_oldest_pending_ms(void* h) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1.0;
    std::lock_guard<std::mutex> lk(e->mu);
    if (e->finished < e->launched - RING) e->finished = e->launched - RING;
    while (e->finished < e->launched) {
        const long slot = e->finished % RING;      // collective number finished + 1
        const hipError_t q = hipEventQuery(e->done[slot]);
        if (q == hipErrorNotReady)
            return std::chrono::duration<double, std::milli>(Clock::now() - e->t_launch[slot]).count();
        if (q != hipSuccess) return -2.0;
        ++e->finished;
    }
    return -1.0;
}

// Device time of finished collective number `seq` (start -> done events), -1 if it has not
// finished or its events were recycled.
DDL_API double ddl_comm_collective_ms(void* h, long seq) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1.0;
    std::lock_guard<std::mutex> lk(e->mu);
    if (seq < 1 || seq > e->launched || e->launched - seq >= RING) return -1.0;
    const long slot = (seq - 1) % RING;
    if (hipEventQuery(e->done[slot]) != hipSuccess) return -1.0;
    float ms = -1.f;
    if (hipEventElapsedTime(&ms, e->start[slot], e->done[slot]) != hipSuccess) return -1.0;
    return ms;
}

// Failure path from any thread: ncclCommAbort (kernels spinning on a dead peer return, the
// streams drain) and mark the engine unusable; the stream / events stay for destroy.
DDL_API int ddl_comm_abort(void* h) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    std::lock_guard<std::mutex> lk(e->mu);
    if (e->comm && !e->aborted) g_rccl.commAbort(e->comm);
    e->comm = nullptr;
    e->aborted = true;
    return 0;
}

// Test hook: make ddl_comm_async_error report `code` (0 clears), as RCCL does for a peer failure.
DDL_API int ddl_comm_inject_error(void* h, int code) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    std::lock_guard<std::mutex> lk(e->mu);
    e->injected = code;
    return 0;
}

DDL_API long ddl_comm_stats(void* h, int which) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    return which == 0 ? e->launched : e->bytes;
}

DDL_API void ddl_comm_destroy(void* h, int abort) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        if (e->comm) {
            if (abort) g_rccl.commAbort(e->comm);
            else {
                hipStreamSynchronize(e->stream);
                g_rccl.commDestroy(e->comm);
            }
            e->comm = nullptr;
        }
    }
    for (int i = 0; i < RING; ++i) {
        if (e->start[i]) hipEventDestroy(e->start[i]);
        if (e->done[i]) hipEventDestroy(e->done[i]);
    }
    if (e->produced) hipEventDestroy(e->produced);
    if (e->drained) hipEventDestroy(e->drained);
    if (e->stream) hipStreamDestroy(e->stream);
    delete e;
}

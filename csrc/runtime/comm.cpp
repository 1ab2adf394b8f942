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
// The reference has no communication layer at all; BASELINE.json
// mandates "data-parallel all-reduce ... RCCL ring/tree over xGMI ... overlapped
// with backward on HIP streams".
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

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
           sym(g_rccl.errorString, "ncclGetErrorString");
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

struct Engine {
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;    // collectives run here, concurrent with compute
    hipEvent_t produced = nullptr;   // compute -> comm ordering
    hipEvent_t drained = nullptr;    // comm -> compute ordering
    hipEvent_t done[RING] = {};      // done[i % RING]: recorded after all-reduce number i + 1
    int rank = 0, world = 1, device = 0;
    long launched = 0;
    long bytes = 0;
};

// all-reduce number e->launched just went onto the comm stream: mark its completion
bool mark_done(Engine* e) {
    return hok(hipEventRecord(e->done[(e->launched - 1) % RING], e->stream), "hipEventRecord");
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
        if (!hok(hipEventCreateWithFlags(&e->done[i], hipEventDisableTiming), "hipEventCreate")) {
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
    if (!order_after(e, compute)) return -3;
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
    if (!order_after(e, compute)) return -3;
    if (!ok(g_rccl.groupStart(), "ncclGroupStart")) return -2;
    const long before = e->launched;
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
    if (!order_after(e, compute)) return -3;
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
    if (!order_after(e, compute)) return -3;
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
    if (!e || seq < 1 || seq > e->launched) return -1;
    if (e->launched - seq >= RING) seq = e->launched;
    return hok(hipStreamWaitEvent(compute, e->done[(seq - 1) % RING], 0), "hipStreamWaitEvent") ? 0 : -3;
}

DDL_API int ddl_comm_synchronize(void* h) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    return hok(hipStreamSynchronize(e->stream), "hipStreamSynchronize") ? 0 : -3;
}

DDL_API long ddl_comm_stats(void* h, int which) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    return which == 0 ? e->launched : e->bytes;
}

DDL_API void ddl_comm_destroy(void* h, int abort) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return;
    if (e->comm) {
        if (abort) g_rccl.commAbort(e->comm);
        else {
            hipStreamSynchronize(e->stream);
            g_rccl.commDestroy(e->comm);
        }
    }
    for (int i = 0; i < RING; ++i)
        if (e->done[i]) hipEventDestroy(e->done[i]);
    if (e->produced) hipEventDestroy(e->produced);
    if (e->drained) hipEventDestroy(e->drained);
    if (e->stream) hipStreamDestroy(e->stream);
    delete e;
}

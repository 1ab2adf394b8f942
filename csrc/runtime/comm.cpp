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
// Locking: the watchdog's three calls never take the lock an API call holds while it is inside
// RCCL.  `api` serialises the API callers among themselves (collective enqueue order); `book`
// guards the launch bookkeeping (counters, event slots, launch times) and is held only around
// event records and counter updates, never across an RCCL call; the communicator pointer and
// the abort flag are atomics.
//
// Communicator lifetime: every use of the communicator (an enqueue, the watchdog's async-error
// read) runs inside an in-flight guard (count up, THEN load the pointer); ddl_comm_abort() sets
// the abort flag, swaps the pointer out, waits until the count is zero and only then calls
// ncclCommAbort() -- so the communicator is never freed under a thread still using it.  That
// wait is short because the communicator is created NON-BLOCKING (ncclCommInitRankConfig,
// blocking = 0): no RCCL call ever blocks (RCCL sets up peer connections on a communicator's
// first collective; with a dead peer a blocking enqueue would hang inside RCCL), it returns
// ncclInProgress instead and the engine polls ncclCommGetAsyncError from its own loop, which
// checks the abort flag between polls and leaves without touching the communicator again.
// An enqueue in that loop counts as pending for ddl_comm_oldest_pending_ms() from the moment it
// began.  (DDL_COMM_NONBLOCKING=0, or an RCCL without ncclCommInitRankConfig: blocking mode, where
// an abort that finds a thread still inside RCCL after 2 s aborts anyway -- the only way to
// unblock it -- which is the one case not covered.)
//
// The reference has no communication layer at all; BASELINE.json
// mandates "data-parallel all-reduce ... RCCL ring/tree over xGMI ... overlapped
// with backward on HIP streams".
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#define DDL_API extern "C" __attribute__((visibility("default")))

namespace {

struct Rccl {
    void* so = nullptr;
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
    decltype(&ncclCommInitRankConfig) commInitRankConfig = nullptr;   // optional: non-blocking mode
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
    decltype(&ncclCommFinalize) commFinalize = nullptr;         // optional (non-blocking teardown)
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
                dlsym(g_rccl.so, "ncclCommGetAsyncError")), true) &&
           (g_rccl.commInitRankConfig = reinterpret_cast<decltype(&ncclCommInitRankConfig)>(
                dlsym(g_rccl.so, "ncclCommInitRankConfig")), true) &&
           (g_rccl.commFinalize = reinterpret_cast<decltype(&ncclCommFinalize)>(
                dlsym(g_rccl.so, "ncclCommFinalize")), true);
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
    std::atomic<ncclComm_t> comm{nullptr};
    hipStream_t stream = nullptr;    // collectives run here, concurrent with compute
    hipEvent_t produced = nullptr;   // compute -> comm ordering
    hipEvent_t drained = nullptr;    // comm -> compute ordering
    hipEvent_t start[RING] = {};     // start[i % RING] / done[i % RING]: around collective number i + 1
    hipEvent_t done[RING] = {};
    Clock::time_point t_launch[RING];
    int rank = 0, world = 1, device = 0;
    long launched = 0;               // (book)
    long finished = 0;               // (book) every collective numbered <= finished is known complete
    long bytes = 0;                  // (book)
    // an enqueue in progress (host time it began; in_enqueue false otherwise) (book)
    bool in_enqueue = false;
    Clock::time_point t_enqueue;
    std::atomic<int> injected{0};    // test hook: reported as the async error
    std::atomic<int> stall_ms{0};    // test hook: the next enqueue blocks this long (a dead peer)
    std::atomic<bool> aborted{false};
    std::atomic<int> inflight{0};    // threads holding the communicator pointer (InUse)
    bool nonblocking = false;        // created with blocking = 0: RCCL calls return ncclInProgress
    std::mutex api;                  // API callers among themselves; never taken by the watchdog
    std::mutex book;                 // bookkeeping only; never held across an RCCL call
};

// collective number e->launched + 1 is about to go onto the comm stream
bool mark_start(Engine* e) {
    std::lock_guard<std::mutex> lk(e->book);
    const long i = e->launched % RING;
    e->t_launch[i] = Clock::now();
    return hok(hipEventRecord(e->start[i], e->stream), "hipEventRecord");
}

// a collective just went onto the comm stream: count it, mark its completion
bool mark_done(Engine* e, long nbytes) {
    std::lock_guard<std::mutex> lk(e->book);
    e->launched += 1;
    e->bytes += nbytes;
    return hok(hipEventRecord(e->done[(e->launched - 1) % RING], e->stream), "hipEventRecord");
}

// In-flight guard: counted BEFORE the pointer is loaded, so an abort that swapped the pointer out
// and then saw the count at zero knows no thread can still reach the old communicator.
struct InUse {
    Engine* e;
    ncclComm_t c;
    explicit InUse(Engine* en) : e(en) {
        e->inflight.fetch_add(1);
        c = e->aborted.load() ? nullptr : e->comm.load();
    }
    ~InUse() { e->inflight.fetch_sub(1); }
    InUse(const InUse&) = delete;
    InUse& operator=(const InUse&) = delete;
};

// Mark an enqueue pending (the watchdog sees it from here until end_enqueue()).  In blocking mode
// the test stall happens here, before the communicator is loaded; in non-blocking mode inside
// settle(), where a real dead-peer enqueue would spin.
void begin_enqueue(Engine* e) {
    {
        std::lock_guard<std::mutex> lk(e->book);
        e->in_enqueue = true;
        e->t_enqueue = Clock::now();
    }
    if (!e->nonblocking) {
        const int stall = e->stall_ms.exchange(0);
        if (stall > 0) std::this_thread::sleep_for(std::chrono::milliseconds(stall));
    }
}

void end_enqueue(Engine* e) {
    std::lock_guard<std::mutex> lk(e->book);
    e->in_enqueue = false;
}

// Non-blocking mode: wait until the RCCL call that returned `r` has been accepted (ncclInProgress
// -> poll the communicator's async state), leaving early -- without touching `c` again -- once
// the communicator is aborted.  Blocking mode: `r` is final.
ncclResult_t settle(Engine* e, ncclComm_t c, ncclResult_t r) {
    if (!e->nonblocking) return r;
    const int stall = e->stall_ms.exchange(0);        // test hook: "InProgress" for that long
    const auto until = Clock::now() + std::chrono::milliseconds(stall > 0 ? stall : 0);
    for (long spin = 0;; ++spin) {
        if (e->aborted.load()) return ncclInvalidUsage;
        const bool stalled = stall > 0 && Clock::now() < until;
        if (!stalled && r != ncclInProgress) return r;
        if (!stalled && g_rccl.getAsyncError(c, &r) != ncclSuccess) return ncclInternalError;
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
        else std::this_thread::yield();
    }
}

bool rccl_ok(Engine* e, ncclComm_t c, ncclResult_t r, const char* what) {
    r = settle(e, c, r);
    if (e->aborted.load()) {
        set_err(what, "communicator aborted");
        return false;
    }
    return ok(r, what);
}

bool usable(Engine* e) {
    if (e->aborted.load() || !e->comm.load()) {
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

long esize(int dtype) { return dtype == 1 || dtype >= 4 ? 4 : dtype == 3 ? 8 : 2; }

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
    ncclComm_t c = nullptr;
    const char* nb = getenv("DDL_COMM_NONBLOCKING");
    e->nonblocking = g_rccl.commInitRankConfig && g_rccl.getAsyncError && g_rccl.commFinalize && !(nb && nb[0] == '0');
    bool good;
    if (e->nonblocking) {
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        ncclResult_t r = g_rccl.commInitRankConfig(&c, world, id, rank, &cfg);
        while (r == ncclInProgress && c) {
            std::this_thread::sleep_for(std::chrono::microseconds(200));
            if (g_rccl.getAsyncError(c, &r) != ncclSuccess) r = ncclInternalError;
        }
        good = ok(r, "ncclCommInitRankConfig");
    } else {
        good = ok(g_rccl.commInitRank(&c, world, id, rank), "ncclCommInitRank");
    }
    if (!good) {
        if (c) g_rccl.commAbort(c);
        hipStreamDestroy(e->stream);
        delete e;
        return nullptr;
    }
    e->comm.store(c);
    return e;
}

DDL_API int ddl_comm_allreduce(void* h, void* buf, long count, int dtype, int avg, hipStream_t compute) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || count <= 0) return count == 0 ? 0 : -1;
    std::lock_guard<std::mutex> lk(e->api);
    if (!usable(e)) return -4;
    if (!order_after(e, compute) || !mark_start(e)) return -3;
    begin_enqueue(e);
    bool good;
    {
        InUse u(e);
        if (!u.c) { end_enqueue(e); set_err("comm", "communicator aborted"); return -4; }
        good = rccl_ok(e, u.c, g_rccl.allReduce(buf, buf, (size_t)count, dtype_of(dtype), avg ? ncclAvg : ncclSum,
                                                u.c, e->stream), "ncclAllReduce");
    }
    end_enqueue(e);
    if (!good) return -2;
    return mark_done(e, count * esize(dtype)) ? 0 : -3;
}

// several buckets that became ready together: one fused RCCL group launch
DDL_API int ddl_comm_allreduce_many(void* h, void** bufs, const long* counts, int n, int dtype, int avg,
                                    hipStream_t compute) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    std::lock_guard<std::mutex> lk(e->api);
    if (!usable(e)) return -4;
    if (!order_after(e, compute)) return -3;
    long before;
    int members = 0;
    long nbytes = 0;
    {
        // one start mark per member, all at the group's stream position
        std::lock_guard<std::mutex> bk(e->book);
        before = e->launched;
        for (int i = 0; i < n; ++i) {
            if (counts[i] <= 0) continue;
            const long slot = (before + members++) % RING;
            e->t_launch[slot] = Clock::now();
            nbytes += counts[i] * esize(dtype);
            if (!hok(hipEventRecord(e->start[slot], e->stream), "hipEventRecord")) return -3;
        }
    }
    if (!members) return 0;
    begin_enqueue(e);
    bool good;
    {
        InUse u(e);
        if (!u.c) { end_enqueue(e); set_err("comm", "communicator aborted"); return -4; }
        good = ok(g_rccl.groupStart(), "ncclGroupStart");
        for (int i = 0; good && i < n; ++i) {
            if (counts[i] <= 0) continue;
            good = ok(g_rccl.allReduce(bufs[i], bufs[i], (size_t)counts[i], dtype_of(dtype),
                                       avg ? ncclAvg : ncclSum, u.c, e->stream), "ncclAllReduce");
        }
        // (in a group the members' results are deferred: ncclGroupEnd's result is the group's)
        good = rccl_ok(e, u.c, g_rccl.groupEnd(), "ncclGroupEnd") && good;
    }
    end_enqueue(e);
    if (!good) return -2;
    // every number of the group completes at the same point of the comm stream
    std::lock_guard<std::mutex> bk(e->book);
    e->launched = before + members;
    e->bytes += nbytes;
    for (long k = before; k < e->launched; ++k)
        if (!hok(hipEventRecord(e->done[k % RING], e->stream), "hipEventRecord")) return -3;
    return 0;
}

// (numbered and timed like the reductions, so a hung broadcast is covered by the watchdog too)
DDL_API int ddl_comm_broadcast(void* h, void* buf, long count, int dtype, int root, hipStream_t compute) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || count <= 0) return count == 0 ? 0 : -1;
    std::lock_guard<std::mutex> lk(e->api);
    if (!usable(e)) return -4;
    if (!order_after(e, compute) || !mark_start(e)) return -3;
    begin_enqueue(e);
    bool good;
    {
        InUse u(e);
        if (!u.c) { end_enqueue(e); set_err("comm", "communicator aborted"); return -4; }
        good = rccl_ok(e, u.c, g_rccl.broadcast(buf, buf, (size_t)count, dtype_of(dtype), root, u.c, e->stream),
                       "ncclBroadcast");
    }
    end_enqueue(e);
    if (!good) return -2;
    return mark_done(e, count * esize(dtype)) ? 0 : -3;
}

// reduce-scatter / all-gather (ZeRO-1 buckets) are numbered with the all-reduces, so
// ddl_comm_wait_upto covers them: the optimizer waits on one bucket's shard, the next
// forward on one bucket's gathered parameters
DDL_API int ddl_comm_reduce_scatter(void* h, const void* send, void* recv, long recv_count, int dtype, int avg,
                                    hipStream_t compute) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || recv_count <= 0) return recv_count == 0 ? 0 : -1;
    std::lock_guard<std::mutex> lk(e->api);
    if (!usable(e)) return -4;
    if (!order_after(e, compute) || !mark_start(e)) return -3;
    begin_enqueue(e);
    bool good;
    {
        InUse u(e);
        if (!u.c) { end_enqueue(e); set_err("comm", "communicator aborted"); return -4; }
        good = rccl_ok(e, u.c, g_rccl.reduceScatter(send, recv, (size_t)recv_count, dtype_of(dtype),
                                                    avg ? ncclAvg : ncclSum, u.c, e->stream), "ncclReduceScatter");
    }
    end_enqueue(e);
    if (!good) return -2;
    return mark_done(e, recv_count * e->world * esize(dtype)) ? 0 : -3;
}

DDL_API int ddl_comm_all_gather(void* h, const void* send, void* recv, long send_count, int dtype,
                                hipStream_t compute) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || send_count <= 0) return send_count == 0 ? 0 : -1;
    std::lock_guard<std::mutex> lk(e->api);
    if (!usable(e)) return -4;
    if (!order_after(e, compute) || !mark_start(e)) return -3;
    begin_enqueue(e);
    bool good;
    {
        InUse u(e);
        if (!u.c) { end_enqueue(e); set_err("comm", "communicator aborted"); return -4; }
        good = rccl_ok(e, u.c, g_rccl.allGather(send, recv, (size_t)send_count, dtype_of(dtype), u.c, e->stream),
                       "ncclAllGather");
    }
    end_enqueue(e);
    if (!good) return -2;
    return mark_done(e, send_count * e->world * esize(dtype)) ? 0 : -3;
}

// compute stream waits for every collective issued so far
DDL_API int ddl_comm_wait(void* h, hipStream_t compute) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    std::lock_guard<std::mutex> lk(e->api);
    if (!usable(e)) return -4;
    return hok(hipEventRecord(e->drained, e->stream), "hipEventRecord") &&
                   hok(hipStreamWaitEvent(compute, e->drained, 0), "hipStreamWaitEvent")
               ? 0
               : -3;
}

// compute stream waits for collective number `seq` (all-reduce / reduce-scatter / all-gather /
// broadcast; 1-based, as counted by ddl_comm_stats(h, 0)) and, the comm stream being in order,
// everything issued before it.  A number more than RING behind the newest waits for a later one
// instead (still correct, just later).
DDL_API int ddl_comm_wait_upto(void* h, long seq, hipStream_t compute) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    std::lock_guard<std::mutex> lk(e->api);
    if (!usable(e)) return -4;
    std::lock_guard<std::mutex> bk(e->book);
    if (seq < 1 || seq > e->launched) return -1;
    if (e->launched - seq >= RING) seq = e->launched;
    return hok(hipStreamWaitEvent(compute, e->done[(seq - 1) % RING], 0), "hipStreamWaitEvent") ? 0 : -3;
}

DDL_API int ddl_comm_synchronize(void* h) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    if (!usable(e)) return -4;
    // (no lock: the watchdog must be able to abort a synchronize stuck on a dead peer)
    return hok(hipStreamSynchronize(e->stream), "hipStreamSynchronize") ? 0 : -3;
}

// RCCL's asynchronous error state of the communicator: 0 = fine (ncclInProgress counts as
// fine), otherwise the ncclResult_t code; -4 after an abort.  Lock-free (the watchdog).
DDL_API int ddl_comm_async_error(void* h) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    InUse u(e);
    if (!u.c) return -4;
    if (const int inj = e->injected.load()) return inj;
    if (!g_rccl.getAsyncError) return 0;
    ncclResult_t r = ncclSuccess;
    if (g_rccl.getAsyncError(u.c, &r) != ncclSuccess) return (int)ncclInternalError;
    return (r == ncclSuccess || r == ncclInProgress) ? 0 : (int)r;
}

// Milliseconds the oldest collective that has not finished has been pending (host clock since
// its launch call; an enqueue still inside RCCL counts from when it began), -1 if every
// collective finished.  Only the RING newest are tracked: older ones count as finished (their
// events were recycled).  Takes the bookkeeping lock only (never held across an RCCL call).
DDL_API double ddl_comm_oldest_pending_ms(void* h) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1.0;
    std::lock_guard<std::mutex> bk(e->book);
    const auto now = Clock::now();
    double age = e->in_enqueue ? std::chrono::duration<double, std::milli>(now - e->t_enqueue).count() : -1.0;
    if (e->finished < e->launched - RING) e->finished = e->launched - RING;
    while (e->finished < e->launched) {
        const long slot = e->finished % RING;      // collective number finished + 1
        const hipError_t q = hipEventQuery(e->done[slot]);
        if (q == hipErrorNotReady) {
            const double a = std::chrono::duration<double, std::milli>(now - e->t_launch[slot]).count();
            return a > age ? a : age;
        }
        if (q != hipSuccess) return -2.0;
        ++e->finished;
    }
    return age;
}

// Device time of finished collective number `seq` (start -> done events), -1 if it has not
// finished or its events were recycled.
DDL_API double ddl_comm_collective_ms(void* h, long seq) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1.0;
    std::lock_guard<std::mutex> bk(e->book);
    if (seq < 1 || seq > e->launched || e->launched - seq >= RING) return -1.0;
    const long slot = (seq - 1) % RING;
    if (hipEventQuery(e->done[slot]) != hipSuccess) return -1.0;
    float ms = -1.f;
    if (hipEventElapsedTime(&ms, e->start[slot], e->done[slot]) != hipSuccess) return -1.0;
    return ms;
}

// Failure path from any thread, lock-free: the abort flag is set and the communicator swapped
// out first (later uses see it gone, an enqueue polling in settle() leaves), then -- once no
// thread holds the old pointer (InUse count zero) -- ncclCommAbort (kernels spinning on a dead
// peer return, the streams drain); the stream / events stay for destroy.
void abort_engine(Engine* e) {
    e->aborted.store(true);
    ncclComm_t c = e->comm.exchange(nullptr);
    if (!c) return;
    const auto t0 = Clock::now();
    while (e->inflight.load() > 0) {
        // blocking mode only: a thread stuck INSIDE RCCL never comes back unless the abort runs
        if (!e->nonblocking && Clock::now() - t0 > std::chrono::seconds(2)) break;
        std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    g_rccl.commAbort(c);
}

DDL_API int ddl_comm_abort(void* h) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    abort_engine(e);
    return 0;
}

// 1: the communicator was created non-blocking (every RCCL call returns promptly; see above)
DDL_API int ddl_comm_nonblocking(void* h) {
    Engine* e = static_cast<Engine*>(h);
    return e && e->nonblocking ? 1 : 0;
}

// Test hook: make ddl_comm_async_error report `code` (0 clears), as RCCL does for a peer failure.
DDL_API int ddl_comm_inject_error(void* h, int code) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    e->injected.store(code);
    return 0;
}

// Test hook: the next collective enqueue blocks `ms` milliseconds inside the engine (holding the
// API lock, as an RCCL enqueue stuck in connection setup to a dead peer does), then fails with -4
// if the communicator was aborted meanwhile.  Non-blocking mode: the stall is an RCCL call that
// keeps answering ncclInProgress, polled while the enqueue holds the communicator (InUse), so an
// abort lands while a real enqueue is in progress.
DDL_API int ddl_comm_test_stall(void* h, int ms) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    e->stall_ms.store(ms);
    return 0;
}

DDL_API long ddl_comm_stats(void* h, int which) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return -1;
    std::lock_guard<std::mutex> bk(e->book);
    return which == 0 ? e->launched : e->bytes;
}

DDL_API void ddl_comm_destroy(void* h, int abort) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return;
    // failure path: abort first, lock-free, so an enqueue still polling releases the API lock
    if (abort) abort_engine(e);
    {
        std::lock_guard<std::mutex> lk(e->api);     // no API call in flight past this point
        e->aborted.store(true);
        ncclComm_t c = e->comm.exchange(nullptr);
        if (c) {
            while (e->inflight.load() > 0) std::this_thread::sleep_for(std::chrono::microseconds(100));
            hipStreamSynchronize(e->stream);
            if (e->nonblocking) {
                // non-blocking teardown: finalize (flushes outstanding work; may answer ncclInProgress,
                // polled while the communicator is still alive), THEN destroy, after which c is gone
                ncclResult_t r = g_rccl.commFinalize(c);
                while (r == ncclInProgress) {
                    std::this_thread::sleep_for(std::chrono::microseconds(200));
                    if (g_rccl.getAsyncError(c, &r) != ncclSuccess) break;
                }
            }
            g_rccl.commDestroy(c);
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

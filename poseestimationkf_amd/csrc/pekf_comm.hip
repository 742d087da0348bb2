// pekf_comm.hip -- the one collective of the sharded path: RCCL over xGMI,
// reached through the C ABI so the multi-GPU host needs no PyTorch on its data path.
//
// Filters are independent (ExtendedKalmanFilter.py:6-80 shares nothing between KalmanFilter
// instances), so a shard of the batch runs on each GPU with no per-record exchange; the only
// collective is ONE gather of the final quaternions to the root (ncclGather, rccl.h:745), plus a
// max all-reduce the benchmark uses for its slowest-rank time.
//
// RCCL is bound at run time (dlopen of librccl.so.1 on first use), not at link time: a process
// that never shards pays nothing for it, and in a process that already has an RCCL loaded (the
// one PyTorch-ROCm bundles) the loader hands back that same library, so there is one RCCL and
// one HIP runtime per process.
//
// Deadlines (PEKF_COMM_TIMEOUT_S, default 300 s):
//  * communicator creation -- ncclCommInitRank (one process per GPU) and ncclCommInitAll (one process
//    for several GPUs) -- runs on a helper thread that the caller waits for until the deadline;
//  * pekf_comm_wait drains a stream, and every collective enqueued on it through this file gets the
//    deadline from the moment the stream reaches it (its inputs are ready: the compute queued before
//    it has finished), so a long compute queue is never mistaken for a dead peer, while a collective
//    that a peer never joins is aborted (ncclCommAbort) at its deadline.
// Either way a rank that never joins or dies mid-run ends the job with PEKF_ERR_TIMEOUT instead of
// leaving every other rank blocked inside RCCL.
#include <dlfcn.h>

#include <atomic>
#include <chrono>
#include <deque>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <type_traits>
#include <vector>

#include <rccl/rccl.h>

#include "pekf_internal.hpp"

namespace pekf {
namespace {

struct Rccl {
    decltype(&::ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&::ncclCommInitRank) init_rank = nullptr;
    decltype(&::ncclCommInitAll) init_all = nullptr;
    decltype(&::ncclCommDestroy) destroy = nullptr;
    decltype(&::ncclGather) gather = nullptr;
    decltype(&::ncclAllReduce) all_reduce = nullptr;
    decltype(&::ncclGroupStart) group_start = nullptr;
    decltype(&::ncclGroupEnd) group_end = nullptr;
    decltype(&::ncclGetErrorString) error_string = nullptr;
    decltype(&::ncclGetVersion) get_version = nullptr;
    decltype(&::ncclCommGetAsyncError) async_error = nullptr;
    decltype(&::ncclCommAbort) abort = nullptr;
    char why[256] = "";
    bool ok = false;
};

Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        // the loaded RCCL if there is one (SONAME match), else the ROCm installation's
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            snprintf(r.why, sizeof(r.why), "cannot load librccl.so.1: %s", dlerror());
            return;
        }
        bool all = true;
        auto sym = [&](auto &fn, const char *name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn && all) {
                snprintf(r.why, sizeof(r.why), "librccl.so.1 lacks %s", name);
                all = false;
            }
        };
        sym(r.get_unique_id, "ncclGetUniqueId");
        sym(r.init_rank, "ncclCommInitRank");
        sym(r.init_all, "ncclCommInitAll");
        sym(r.destroy, "ncclCommDestroy");
        sym(r.gather, "ncclGather");
        sym(r.all_reduce, "ncclAllReduce");
        sym(r.group_start, "ncclGroupStart");
        sym(r.group_end, "ncclGroupEnd");
        sym(r.error_string, "ncclGetErrorString");
        sym(r.get_version, "ncclGetVersion");
        sym(r.async_error, "ncclCommGetAsyncError");
        sym(r.abort, "ncclCommAbort");
        r.ok = all;

    });
    return r;
}

int need_rccl() {
    if (int st = require_device()) return st;
    Rccl &r = rccl();
    if (!r.ok) return set_error(PEKF_ERR_COMM, "%s", r.why);
    return PEKF_OK;
}

int nccl_fail(ncclResult_t e, const char *what) {
    return set_error(PEKF_ERR_COMM, "%s: %s (%d)", what, rccl().error_string(e), (int)e);
}

#define PEKF_NCCL(call)                                                  \
    do {                                                                 \
        ncclResult_t e_ = (call);                                        \
        if (e_ != ncclSuccess) return ::pekf::nccl_fail(e_, #call);      \
    } while (0)

static_assert(sizeof(ncclUniqueId) == PEKF_COMM_ID_BYTES, "RCCL unique id size");

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// PEKF_COMM_TIMEOUT_S (seconds; <= 0 disables the deadline), default 300
double env_timeout_s() {
    const char *v = getenv("PEKF_COMM_TIMEOUT_S");
    if (!v || !*v) return 300.0;
    char *end = nullptr;
    const double t = strtod(v, &end);
    return (end && end != v) ? t : 300.0;
}

double deadline_after(double timeout_s) { return timeout_s > 0 ? now_s() + timeout_s : 0.0; }

// PEKF_COMM_DEBUG=1: a stderr line per step of communicator creation / teardown (diagnosing hangs)
bool comm_debug() {
    static const bool on = [] {
        const char *v = getenv("PEKF_COMM_DEBUG");
        return v && *v && *v != '0';
    }();
    return on;
}
#define PEKF_COMM_TRACE(...)                                                          \
    do {                                                                              \
        if (comm_debug()) {                                                           \
            fprintf(stderr, "[pekf_comm %.3f] ", now_s());                            \
            fprintf(stderr, __VA_ARGS__);                                             \
            fputc('\n', stderr);                                                      \
        }                                                                             \
    } while (0)

// Polls a non-blocking communicator until RCCL has finished the call in progress on it.
// Returns PEKF_OK, the RCCL error, or PEKF_ERR_TIMEOUT (*expired set) at the deadline (0 = none).
int settle(ncclComm_t nc, double deadline, const char *what, bool *expired) {
    *expired = false;
    for (;;) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t e = rccl().async_error(nc, &st);
        if (e != ncclSuccess) return nccl_fail(e, "ncclCommGetAsyncError");
        if (st == ncclSuccess) return PEKF_OK;
        if (st != ncclInProgress) return nccl_fail(st, what);
        if (deadline > 0 && now_s() > deadline) {
            *expired = true;
            PEKF_COMM_TRACE("%s: deadline passed", what);
            return PEKF_ERR_TIMEOUT;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(500));
    }
}

}  // namespace
}  // namespace pekf

struct pekf_comm {
    ncclComm_t nc;
    int nranks, rank, device;
    double timeout_s;  // deadline of each settle on this communicator (<= 0: none)
    // The collectives enqueued on this communicator through this file and not yet seen complete, oldest
    // first: an event recorded just before each (its inputs are ready once it completes) and one just
    // after (the collective has completed).  pekf_comm_wait starts a collective's deadline when it sees
    // the first event complete, so only the collective itself, never the compute ahead of it, is timed.
    struct Pending {
        hipEvent_t pre, post;
        hipStream_t stream;
        const char *what;
        double ready_at;  // when pekf_comm_wait first saw `pre` complete (0: not yet)
    };
    std::deque<Pending> pending{};
    std::vector<hipEvent_t> spare{};  // events of retired entries, for reuse (on `device`)
    // Streams holding a collective that was enqueued but could not be tracked (its completion event
    // could not be recorded): pekf_comm_wait bounds a drain of such a stream by a wall-clock deadline
    // from the wait call instead, until the stream has drained once.
    std::vector<hipStream_t> lost{};
};

namespace pekf {
namespace {

// Makes `dev` current for the scope (events and the null stream belong to the current device).
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int dev) {
        if (hipGetDevice(&prev) != hipSuccess || prev == dev) prev = -1;
        else (void)hipSetDevice(dev);
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Collectives a communicator tracks at once.  One more is refused (PEKF_ERR_COMM) rather than enqueued
// untracked: an untracked collective that a peer never joins would stall the stream with no deadline
// running (the next tracked one's inputs would never be ready).
constexpr size_t kMaxPending = 1024;

void release(pekf_comm *c, const pekf_comm::Pending &p) {
    c->spare.push_back(p.pre);
    c->spare.push_back(p.post);
}

// Drops the completed collectives at the front of c's list.
void retire(pekf_comm *c) {
    while (!c->pending.empty() && hipEventQuery(c->pending.front().post) == hipSuccess) {
        release(c, c->pending.front());
        c->pending.pop_front();
    }
}

// An event recorded on s now (nullptr if the runtime refused: the collective then goes untracked).
hipEvent_t mark(pekf_comm *c, hipStream_t s) {
    DeviceScope on(c->device);
    hipEvent_t ev = nullptr;
    if (!c->spare.empty()) {
        ev = c->spare.back();
        c->spare.pop_back();
    } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
        return nullptr;
    }
    if (hipEventRecord(ev, s) != hipSuccess) {
        c->spare.push_back(ev);
        return nullptr;
    }
    return ev;
}

bool is_lost(const pekf_comm *c, hipStream_t s) {
    for (hipStream_t x : c->lost)
        if (x == s) return true;
    return false;
}

// Tracks a collective just enqueued on s between pre (recorded before it) and post.  Without post the
// collective cannot be tracked: s is marked lost (pekf_comm_wait then bounds its drain by wall clock).
// The caller has checked room() before enqueueing, so nothing is ever evicted.
void track(pekf_comm *c, hipStream_t s, hipEvent_t pre, hipEvent_t post, const char *what) {
    if (!post || c->pending.size() >= kMaxPending) {
        if (pre) c->spare.push_back(pre);
        if (post) c->spare.push_back(post);
        if (!is_lost(c, s)) c->lost.push_back(s);
        return;
    }
    c->pending.push_back({pre, post, s, what, 0.0});
}

// Room to track one more collective on c (after dropping the completed ones), else PEKF_ERR_COMM.
int room(pekf_comm *c) {
    retire(c);
    if (c->pending.size() < kMaxPending) return PEKF_OK;
    return set_error(PEKF_ERR_COMM,
                     "rank %d of %d: %zu collectives already in flight on this communicator (the most it tracks "
                     "for pekf_comm_wait's deadline); wait for them before enqueueing more",
                     c->rank, c->nranks, c->pending.size());
}

void drop_events(pekf_comm *c) {
    DeviceScope on(c->device);
    for (const auto &p : c->pending) release(c, p);
    c->pending.clear();
    c->lost.clear();
    for (hipEvent_t e : c->spare) (void)hipEventDestroy(e);
    c->spare.clear();
}

// Aborts c's RCCL communicator (kernels of it still in flight give up) and leaves c destroy-only.
void abort_comm(pekf_comm *c) {
    if (c->nc) (void)rccl().abort(c->nc);
    c->nc = nullptr;
}

// Result of an enqueue on c: ncclInProgress (non-blocking communicator) is settled against c's
// deadline; an expired deadline aborts c.
int enqueued(pekf_comm *c, ncclResult_t e, const char *what) {
    if (e == ncclSuccess) return PEKF_OK;
    if (e != ncclInProgress) return nccl_fail(e, what);
    bool expired = false;
    const int st = settle(c->nc, deadline_after(c->timeout_s), what, &expired);
    if (expired) {
        abort_comm(c);
        return set_error(PEKF_ERR_TIMEOUT, "%s: still in progress after %.0f s; communicator aborted", what,
                         c->timeout_s);
    }
    return st;
}

// Enqueues one collective of c on s between the two tracking events.
template <class Enqueue>
int tracked(pekf_comm *c, hipStream_t s, const char *what, Enqueue enqueue) {
    if (int st = room(c)) return st;
    hipEvent_t pre = mark(c, s);
    if (!pre) return set_error(PEKF_ERR_HIP, "%s: cannot record the event that times it; not enqueued", what);
    const int st = enqueued(c, enqueue(), what);
    if (st != PEKF_OK || !c->nc) {
        if (pre) c->spare.push_back(pre);
        return st;
    }
    track(c, s, pre, mark(c, s), what);
    return PEKF_OK;
}

// Communicator creations abandoned at their deadline whose helper thread is still blocked inside RCCL.
// While there is one, RCCL's bootstrap state is not to be trusted: later creations fail at once.
std::atomic<int> g_abandoned_inits{0};

enum class InitEnd { done, timed_out };

// Runs `init` (a blocking RCCL communicator creation filling n communicators) on a helper thread and
// waits for it at most timeout_s (<= 0: inline, no deadline).  On expiry the helper is abandoned: it
// stays blocked inside RCCL until the process exits, and if the creation completes after all it
// aborts the communicators it got.  *res is RCCL's result when the creation ended in time.
template <class Init>
InitEnd init_with_deadline(double timeout_s, int n, Init init, std::vector<ncclComm_t> *comms, ncclResult_t *res) {
    comms->assign(n, nullptr);
    if (timeout_s <= 0) {
        *res = init(comms->data());
        return InitEnd::done;
    }
    struct Job {
        std::mutex m;
        std::condition_variable cv;
        bool done = false, abandoned = false;
        ncclResult_t res = ncclSuccess;
        std::vector<ncclComm_t> nc;
    };
    auto job = std::make_shared<Job>();
    job->nc.assign(n, nullptr);
    std::thread([job, init] {
        std::vector<ncclComm_t> nc(job->nc.size(), nullptr);
        const ncclResult_t r = init(nc.data());
        std::lock_guard<std::mutex> g(job->m);
        if (job->abandoned) {
            for (ncclComm_t x : nc)
                if (x) (void)rccl().abort(x);
            g_abandoned_inits.fetch_sub(1);
            return;
        }
        job->res = r;
        job->nc = nc;
        job->done = true;
        job->cv.notify_all();
    }).detach();
    std::unique_lock<std::mutex> lk(job->m);
    if (!job->cv.wait_for(lk, std::chrono::duration<double>(timeout_s), [&] { return job->done; })) {
        job->abandoned = true;
        g_abandoned_inits.fetch_add(1);
        return InitEnd::timed_out;
    }
    *res = job->res;
    *comms = job->nc;
    return InitEnd::done;
}

int refuse_after_abandoned_init() {
    if (g_abandoned_inits.load() > 0)
        return set_error(PEKF_ERR_COMM,
                         "an earlier RCCL communicator creation passed its deadline and is still blocked inside "
                         "RCCL; this process must exit before it can create another communicator");
    return PEKF_OK;
}

}  // namespace
}  // namespace pekf

using namespace pekf;

extern "C" {

int pekf_comm_version(int *version) {
    PEKF_CHECK_ARG(version, "null pointer");
    if (int st = need_rccl()) return st;
    PEKF_NCCL(rccl().get_version(version));
    return PEKF_OK;
}

int pekf_comm_unique_id(void *id) {
    PEKF_CHECK_ARG(id, "null pointer");
    if (int st = need_rccl()) return st;
    ncclUniqueId u;
    PEKF_NCCL(rccl().get_unique_id(&u));
    memcpy(id, &u, sizeof(u));
    return PEKF_OK;
}

int pekf_comm_init_timeout(const void *id, int nranks, int rank, double timeout_s, pekf_comm **out) {
    PEKF_CHECK_ARG(id && out, "null pointer");
    PEKF_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "need 0 <= rank < nranks");
    *out = nullptr;
    if (int st = need_rccl()) return st;
    if (int st = refuse_after_abandoned_init()) return st;
    int dev = 0;
    PEKF_HIP(hipGetDevice(&dev));
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    // RCCL 2.27's "non-blocking" init (ncclCommInitRankConfig, blocking = 0) still waits in the calling
    // thread for every rank to reach the bootstrap root (measured on the box: it never returned with a
    // rank missing, scripts/comm_timeout_probe.py), so the deadline is kept here, on a helper thread.
    PEKF_COMM_TRACE("rank %d/%d on device %d: ncclCommInitRank (deadline %.0f s)", rank, nranks, dev, timeout_s);
    std::vector<ncclComm_t> nc;
    ncclResult_t res = ncclSuccess;
    const auto init = [nranks, u, rank, dev](ncclComm_t *c) {
        if (hipSetDevice(dev) != hipSuccess) return ncclUnhandledCudaError;
        return rccl().init_rank(c, nranks, u, rank);
    };
    if (init_with_deadline(timeout_s, 1, init, &nc, &res) == InitEnd::timed_out) {
        PEKF_COMM_TRACE("rank %d/%d: deadline passed; init abandoned", rank, nranks);
        return set_error(PEKF_ERR_TIMEOUT,
                         "RCCL communicator init (ncclCommInitRank, rank %d of %d, device %d): not all %d ranks "
                         "joined within %.0f s (PEKF_COMM_TIMEOUT_S); init abandoned",
                         rank, nranks, dev, nranks, timeout_s);
    }
    PEKF_COMM_TRACE("rank %d/%d: ncclCommInitRank returned %d", rank, nranks, (int)res);
    if (res != ncclSuccess) return nccl_fail(res, "ncclCommInitRank");
    *out = new pekf_comm{nc[0], nranks, rank, dev, timeout_s > 0 ? timeout_s : 0.0};
    return PEKF_OK;
}

int pekf_comm_init(const void *id, int nranks, int rank, pekf_comm **out) {
    return pekf_comm_init_timeout(id, nranks, rank, env_timeout_s(), out);
}

int pekf_comm_init_all_timeout(int ndev, const int *devices, double timeout_s, pekf_comm **out) {
    PEKF_CHECK_ARG(out && ndev >= 1, "need ndev >= 1 and an output array");
    for (int i = 0; i < ndev; ++i) out[i] = nullptr;
    if (int st = need_rccl()) return st;
    if (int st = refuse_after_abandoned_init()) return st;
    int visible = 0;
    PEKF_HIP(hipGetDeviceCount(&visible));
    std::vector<int> devs(ndev);
    for (int i = 0; i < ndev; ++i) {
        devs[i] = devices ? devices[i] : i;
        PEKF_CHECK_ARG(devs[i] >= 0 && devs[i] < visible, "device index out of range");
    }
    PEKF_COMM_TRACE("ncclCommInitAll over %d devices (deadline %.0f s)", ndev, timeout_s);
    std::vector<ncclComm_t> nc;
    ncclResult_t res = ncclSuccess;
    const auto init = [ndev, devs](ncclComm_t *c) { return rccl().init_all(c, ndev, devs.data()); };
    if (init_with_deadline(timeout_s, ndev, init, &nc, &res) == InitEnd::timed_out) {
        PEKF_COMM_TRACE("ncclCommInitAll: deadline passed; init abandoned");
        return set_error(PEKF_ERR_TIMEOUT,
                         "RCCL communicator init (ncclCommInitAll over %d devices): not done within %.0f s "
                         "(PEKF_COMM_TIMEOUT_S); init abandoned",
                         ndev, timeout_s);
    }
    PEKF_COMM_TRACE("ncclCommInitAll returned %d", (int)res);
    if (res != ncclSuccess) return nccl_fail(res, "ncclCommInitAll");
    for (int i = 0; i < ndev; ++i) out[i] = new pekf_comm{nc[i], ndev, i, devs[i], timeout_s > 0 ? timeout_s : 0.0};
    return PEKF_OK;
}

int pekf_comm_init_all(int ndev, const int *devices, pekf_comm **out) {
    return pekf_comm_init_all_timeout(ndev, devices, env_timeout_s(), out);
}

int pekf_comm_destroy(pekf_comm *c) {
    if (!c) return PEKF_OK;
    drop_events(c);
    if (!c->nc) {  // aborted: nothing left to destroy
        delete c;
        return PEKF_OK;
    }
    ncclResult_t e = rccl().destroy(c->nc);
    if (e == ncclInProgress) {  // non-blocking communicator: wait for the teardown
        bool expired = false;
        if (settle(c->nc, deadline_after(c->timeout_s), "ncclCommDestroy", &expired) == PEKF_OK) e = ncclSuccess;
        else (void)rccl().abort(c->nc);
    }
    delete c;
    if (e != ncclSuccess && e != ncclInProgress) return nccl_fail(e, "ncclCommDestroy");
    return PEKF_OK;
}

int pekf_comm_abort(pekf_comm *c) {
    if (!c) return PEKF_OK;
    abort_comm(c);
    drop_events(c);
    delete c;
    return PEKF_OK;
}

int pekf_comm_wait(pekf_comm *c, void *stream, double timeout_s) {
    PEKF_CHECK_ARG(c, "null communicator");
    PEKF_CHECK_ARG(c->nc, "communicator was aborted");
    const hipStream_t s = as_stream(stream);
    const double called_at = now_s();
    for (;;) {
        const hipError_t q = hipStreamQuery(s);
        if (q == hipSuccess) {
            retire(c);
            for (auto it = c->lost.begin(); it != c->lost.end(); ++it)
                if (*it == s) {
                    c->lost.erase(it);
                    break;
                }
            return PEKF_OK;
        }
        if (q != hipErrorNotReady) return hip_fail(q, "hipStreamQuery");
        ncclResult_t st = ncclSuccess;
        if (rccl().async_error(c->nc, &st) == ncclSuccess && st != ncclSuccess && st != ncclInProgress) {
            abort_comm(c);
            return set_error(PEKF_ERR_COMM, "RCCL asynchronous error on rank %d of %d: %s (%d); communicator aborted",
                             c->rank, c->nranks, rccl().error_string(st), (int)st);
        }
        // the oldest collective of this stream that has not completed: is the stream at it yet?
        pekf_comm::Pending *head = nullptr;
        for (auto it = c->pending.begin(); it != c->pending.end();) {
            if (it->stream != s) {
                ++it;
            } else if (hipEventQuery(it->post) == hipSuccess) {
                release(c, *it);
                it = c->pending.erase(it);
            } else {
                head = &*it;
                break;
            }
        }
        // a collective on s went untracked: no per-collective clock can be trusted, so the whole drain
        // gets the deadline from this call (compute queued on s is then charged too)
        if (timeout_s > 0 && is_lost(c, s) && now_s() - called_at > timeout_s) {
            abort_comm(c);
            return set_error(PEKF_ERR_TIMEOUT,
                             "rank %d of %d: a stream holding an untracked collective did not drain within %.0f s "
                             "of the wait (a peer rank gone?); communicator aborted",
                             c->rank, c->nranks, timeout_s);
        }
        if (head && timeout_s > 0 && hipEventQuery(head->pre) == hipSuccess) {
            const double t = now_s();
            if (head->ready_at == 0.0) {
                head->ready_at = t;
            } else if (t - head->ready_at > timeout_s) {
                const char *what = head->what;
                abort_comm(c);
                return set_error(PEKF_ERR_TIMEOUT,
                                 "rank %d of %d: %s did not complete within %.0f s of its inputs being ready (a peer "
                                 "rank gone?); communicator aborted",
                                 c->rank, c->nranks, what, timeout_s);
            }
        }
        std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
}

int pekf_comm_rank(const pekf_comm *c, int *rank, int *nranks, int *device) {
    PEKF_CHECK_ARG(c, "null communicator");
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->nranks;
    if (device) *device = c->device;
    return PEKF_OK;
}

int pekf_gather_dev(pekf_comm *c, const double *send, int64_t count, double *recv, int root, void *stream) {
    PEKF_CHECK_ARG(c && send, "null pointer");
    PEKF_CHECK_ARG(count >= 0, "negative size");
    PEKF_CHECK_ARG(root >= 0 && root < c->nranks, "root out of range");
    PEKF_CHECK_ARG(c->rank != root || recv, "the root needs a receive buffer of nranks * count doubles");
    PEKF_CHECK_ARG(c->nc, "communicator was aborted");
    const hipStream_t s = as_stream(stream);
    return tracked(c, s, "ncclGather", [&] { return rccl().gather(send, recv, (size_t)count, ncclFloat64, root, c->nc, s); });
}

int pekf_gather_multi_dev(int ndev, pekf_comm *const *comms, const double *const *send, int64_t count,
                          double *recv, int root, void *const *streams) {
    PEKF_CHECK_ARG(ndev >= 1 && comms && send && streams, "null pointer");
    PEKF_CHECK_ARG(count >= 0, "negative size");
    PEKF_CHECK_ARG(root >= 0 && root < ndev && recv, "root out of range or no receive buffer");
    for (int i = 0; i < ndev; ++i) PEKF_CHECK_ARG(comms[i] && comms[i]->nc, "null or aborted communicator");
    for (int i = 0; i < ndev; ++i)
        if (int st = room(comms[i])) return st;
    std::vector<hipEvent_t> pre(ndev);
    for (int i = 0; i < ndev; ++i) pre[i] = mark(comms[i], as_stream(streams[i]));
    const auto untrack = [&] {
        for (int i = 0; i < ndev; ++i)
            if (pre[i]) comms[i]->spare.push_back(pre[i]);
    };
    for (int i = 0; i < ndev; ++i)
        if (!pre[i]) {
            untrack();
            return set_error(PEKF_ERR_HIP, "ncclGather (grouped): cannot record the event that times it on device "
                             "%d; not enqueued", comms[i]->device);
        }
    ncclResult_t e = rccl().group_start();
    if (e != ncclSuccess) {
        untrack();
        return nccl_fail(e, "ncclGroupStart");
    }
    for (int i = 0; i < ndev; ++i) {
        e = rccl().gather(send[i], i == root ? recv : nullptr, (size_t)count, ncclFloat64, root, comms[i]->nc,
                          as_stream(streams[i]));
        if (e != ncclSuccess) {
            (void)rccl().group_end();
            untrack();
            return nccl_fail(e, "ncclGather");
        }
    }
    e = rccl().group_end();
    if (e != ncclSuccess) {
        untrack();
        return nccl_fail(e, "ncclGroupEnd");
    }
    for (int i = 0; i < ndev; ++i)
        track(comms[i], as_stream(streams[i]), pre[i], mark(comms[i], as_stream(streams[i])), "ncclGather (grouped)");
    return PEKF_OK;
}

int pekf_allreduce_max_dev(pekf_comm *c, double *buf, int64_t count, void *stream) {
    PEKF_CHECK_ARG(c && buf, "null pointer");
    PEKF_CHECK_ARG(count >= 0, "negative size");
    PEKF_CHECK_ARG(c->nc, "communicator was aborted");
    const hipStream_t s = as_stream(stream);
    return tracked(c, s, "ncclAllReduce",
                   [&] { return rccl().all_reduce(buf, buf, (size_t)count, ncclFloat64, ncclMax, c->nc, s); });
}

}  // extern "C"

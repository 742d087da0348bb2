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
// Deadlines: communicator creation waits for the (blocking) ncclCommInitRank on a helper thread for at
// most PEKF_COMM_TIMEOUT_S, and pekf_comm_wait drains a stream of collectives against a deadline,
// aborting the communicator (ncclCommAbort) on expiry, so a rank that never joins or dies mid-run ends
// the job with PEKF_ERR_TIMEOUT instead of leaving every other rank blocked inside RCCL.
#include <dlfcn.h>

#include <chrono>
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
    double timeout_s;  // deadline of each settle / wait on this communicator (<= 0: none)
};

namespace pekf {
namespace {

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
    int dev = 0;
    PEKF_HIP(hipGetDevice(&dev));
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    Rccl &r = rccl();
    if (timeout_s <= 0) {
        ncclComm_t nc = nullptr;
        PEKF_NCCL(r.init_rank(&nc, nranks, u, rank));  // collective over the nranks processes, no deadline
        *out = new pekf_comm{nc, nranks, rank, dev, 0.0};
        return PEKF_OK;
    }
    // RCCL 2.27's "non-blocking" init (ncclCommInitRankConfig, blocking = 0) still waits in the calling
    // thread for every rank to reach the bootstrap root (measured on the box: it never returned with a
    // rank missing, scripts/comm_timeout_probe.py), so the deadline is kept here instead: the blocking
    // init runs on a helper thread and this thread waits for it until the deadline.  On expiry the
    // helper is abandoned -- it stays blocked inside RCCL until the process exits, and if the missing
    // rank turns up after all it aborts the communicator it gets -- and PEKF_ERR_TIMEOUT is returned.
    struct Job {
        std::mutex m;
        std::condition_variable cv;
        bool done = false, abandoned = false;
        ncclResult_t res = ncclSuccess;
        ncclComm_t nc = nullptr;
    };
    auto job = std::make_shared<Job>();
    PEKF_COMM_TRACE("rank %d/%d on device %d: ncclCommInitRank on a helper thread (deadline %.0f s)", rank, nranks,
                    dev, timeout_s);
    std::thread([job, nranks, u, rank, dev] {
        ncclComm_t nc = nullptr;
        ncclResult_t res = ncclSuccess;
        if (hipSetDevice(dev) != hipSuccess) res = ncclUnhandledCudaError;
        else res = rccl().init_rank(&nc, nranks, u, rank);
        std::lock_guard<std::mutex> g(job->m);
        if (job->abandoned) {
            if (nc) (void)rccl().abort(nc);
            return;
        }
        job->res = res;
        job->nc = nc;
        job->done = true;
        job->cv.notify_all();
    }).detach();
    std::unique_lock<std::mutex> lk(job->m);
    const bool finished = job->cv.wait_for(lk, std::chrono::duration<double>(timeout_s), [&] { return job->done; });
    if (!finished) {
        job->abandoned = true;
        PEKF_COMM_TRACE("rank %d/%d: deadline passed; init abandoned", rank, nranks);
        return set_error(PEKF_ERR_TIMEOUT,
                         "RCCL communicator init (ncclCommInitRank, rank %d of %d, device %d): not all %d ranks "
                         "joined within %.0f s (PEKF_COMM_TIMEOUT_S); init abandoned",
                         rank, nranks, dev, nranks, timeout_s);
    }
    PEKF_COMM_TRACE("rank %d/%d: ncclCommInitRank returned %d", rank, nranks, (int)job->res);
    if (job->res != ncclSuccess) return nccl_fail(job->res, "ncclCommInitRank");
    *out = new pekf_comm{job->nc, nranks, rank, dev, timeout_s};
    return PEKF_OK;
}

int pekf_comm_init(const void *id, int nranks, int rank, pekf_comm **out) {
    return pekf_comm_init_timeout(id, nranks, rank, env_timeout_s(), out);
}

int pekf_comm_init_all(int ndev, const int *devices, pekf_comm **out) {
    PEKF_CHECK_ARG(out && ndev >= 1, "need ndev >= 1 and an output array");
    if (int st = need_rccl()) return st;
    int visible = 0;
    PEKF_HIP(hipGetDeviceCount(&visible));
    std::vector<int> devs(ndev);
    for (int i = 0; i < ndev; ++i) {
        devs[i] = devices ? devices[i] : i;
        PEKF_CHECK_ARG(devs[i] >= 0 && devs[i] < visible, "device index out of range");
    }
    std::vector<ncclComm_t> nc(ndev, nullptr);
    PEKF_NCCL(rccl().init_all(nc.data(), ndev, devs.data()));
    for (int i = 0; i < ndev; ++i) out[i] = new pekf_comm{nc[i], ndev, i, devs[i], env_timeout_s()};
    return PEKF_OK;
}

int pekf_comm_destroy(pekf_comm *c) {
    if (!c) return PEKF_OK;
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
    delete c;
    return PEKF_OK;
}

int pekf_comm_wait(pekf_comm *c, void *stream, double timeout_s) {
    PEKF_CHECK_ARG(c, "null communicator");
    PEKF_CHECK_ARG(c->nc, "communicator was aborted");
    const hipStream_t s = as_stream(stream);
    const double deadline = deadline_after(timeout_s);
    for (;;) {
        const hipError_t q = hipStreamQuery(s);
        if (q == hipSuccess) return PEKF_OK;
        if (q != hipErrorNotReady) return hip_fail(q, "hipStreamQuery");
        ncclResult_t st = ncclSuccess;
        if (rccl().async_error(c->nc, &st) == ncclSuccess && st != ncclSuccess && st != ncclInProgress) {
            abort_comm(c);
            return set_error(PEKF_ERR_COMM, "RCCL asynchronous error on rank %d of %d: %s (%d); communicator aborted",
                             c->rank, c->nranks, rccl().error_string(st), (int)st);
        }
        if (deadline > 0 && now_s() > deadline) {
            abort_comm(c);
            return set_error(PEKF_ERR_TIMEOUT,
                             "rank %d of %d: the stream's collectives did not complete within %.0f s (a peer rank "
                             "gone?); communicator aborted",
                             c->rank, c->nranks, timeout_s);
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
    return enqueued(c, rccl().gather(send, recv, (size_t)count, ncclFloat64, root, c->nc, as_stream(stream)),
                    "ncclGather");
}

int pekf_gather_multi_dev(int ndev, pekf_comm *const *comms, const double *const *send, int64_t count,
                          double *recv, int root, void *const *streams) {
    PEKF_CHECK_ARG(ndev >= 1 && comms && send && streams, "null pointer");
    PEKF_CHECK_ARG(count >= 0, "negative size");
    PEKF_CHECK_ARG(root >= 0 && root < ndev && recv, "root out of range or no receive buffer");
    for (int i = 0; i < ndev; ++i) PEKF_CHECK_ARG(comms[i] && comms[i]->nc, "null or aborted communicator");
    PEKF_NCCL(rccl().group_start());
    for (int i = 0; i < ndev; ++i) {
        const ncclResult_t e = rccl().gather(send[i], i == root ? recv : nullptr, (size_t)count, ncclFloat64, root,
                                             comms[i]->nc, as_stream(streams[i]));
        if (e != ncclSuccess) {
            (void)rccl().group_end();
            return nccl_fail(e, "ncclGather");
        }
    }
    PEKF_NCCL(rccl().group_end());
    return PEKF_OK;
}

int pekf_allreduce_max_dev(pekf_comm *c, double *buf, int64_t count, void *stream) {
    PEKF_CHECK_ARG(c && buf, "null pointer");
    PEKF_CHECK_ARG(count >= 0, "negative size");
    PEKF_CHECK_ARG(c->nc, "communicator was aborted");
    return enqueued(c, rccl().all_reduce(buf, buf, (size_t)count, ncclFloat64, ncclMax, c->nc, as_stream(stream)),
                    "ncclAllReduce");
}

}  // extern "C"

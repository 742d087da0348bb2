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
#include <dlfcn.h>

#include <cstdio>
#include <cstring>
#include <mutex>
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

}  // namespace
}  // namespace pekf

struct pekf_comm {
    ncclComm_t nc;
    int nranks, rank, device;
};

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

int pekf_comm_init(const void *id, int nranks, int rank, pekf_comm **out) {
    PEKF_CHECK_ARG(id && out, "null pointer");
    PEKF_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "need 0 <= rank < nranks");
    *out = nullptr;
    if (int st = need_rccl()) return st;
    int dev = 0;
    PEKF_HIP(hipGetDevice(&dev));
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t nc = nullptr;
    PEKF_NCCL(rccl().init_rank(&nc, nranks, u, rank));  // collective over the nranks processes
    *out = new pekf_comm{nc, nranks, rank, dev};
    return PEKF_OK;
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
    for (int i = 0; i < ndev; ++i) out[i] = new pekf_comm{nc[i], ndev, i, devs[i]};
    return PEKF_OK;
}

int pekf_comm_destroy(pekf_comm *c) {
    if (!c) return PEKF_OK;
    const ncclResult_t e = rccl().destroy(c->nc);
    delete c;
    if (e != ncclSuccess) return nccl_fail(e, "ncclCommDestroy");
    return PEKF_OK;
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
    PEKF_NCCL(rccl().gather(send, recv, (size_t)count, ncclFloat64, root, c->nc, as_stream(stream)));
    return PEKF_OK;
}

int pekf_gather_multi_dev(int ndev, pekf_comm *const *comms, const double *const *send, int64_t count,
                          double *recv, int root, void *const *streams) {
    PEKF_CHECK_ARG(ndev >= 1 && comms && send && streams, "null pointer");
    PEKF_CHECK_ARG(count >= 0, "negative size");
    PEKF_CHECK_ARG(root >= 0 && root < ndev && recv, "root out of range or no receive buffer");
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
    PEKF_NCCL(rccl().all_reduce(buf, buf, (size_t)count, ncclFloat64, ncclMax, c->nc, as_stream(stream)));
    return PEKF_OK;
}

}  // extern "C"

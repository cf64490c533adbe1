// comm.cpp -- the communicator of the sharded solve behind the C ABI (mgdp_comm_*): RCCL over xGMI,
// called from the library instead of torch.distributed's ProcessGroupNCCL.  librccl is loaded at
// the first call (dlopen), not linked: a process that never shards does not need it, and in a
// PyTorch process the copy torch already mapped is reused (one RCCL, one HIP runtime).  The
// communicator owns a small device buffer for the protocol's words (include/mgdp.h).
#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <string>

#include <rccl/rccl.h>

#include "comm.h"

struct mgdp_comm {
    ncclComm_t nc = nullptr;
    int nranks = 0, rank = 0, device = 0;
    int64_t *d_proto = nullptr;  // int64[8] device: the device protocol's words
    int64_t *h_word = nullptr;   // pinned int64[8]: host-driven collectives stage through it
    hipStream_t stream = nullptr;  // host-driven collectives (mgdp_comm_allreduce_max)
    int64_t calls = 0;             // all-reduces issued (mgdp_comm_stats)
};

namespace mgdp {
namespace {

struct Rccl {
    void *h = nullptr;
    std::string path;
    ncclResult_t (*getUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*commInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*allReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    const char *(*errorString)(ncclResult_t) = nullptr;
};

// The librccl already mapped into this process (e.g. PyTorch's bundled copy), if any.
std::string mapped_rccl() {
    FILE *f = std::fopen("/proc/self/maps", "r");
    if (!f) return {};
    char line[4096];
    std::string found;
    while (std::fgets(line, sizeof(line), f)) {
        const char *p = std::strchr(line, '/');
        if (p && std::strstr(p, "librccl")) {
            found = p;
            while (!found.empty() && (found.back() == '\n' || found.back() == ' ')) found.pop_back();
            break;
        }
    }
    std::fclose(f);
    return found;
}

Rccl *rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        std::string cands[3];
        if (const char *ev = std::getenv("MGDP_RCCL_LIB")) cands[0] = ev;
        cands[1] = mapped_rccl();
        cands[2] = "librccl.so.1";
        for (const auto &c : cands) {
            if (c.empty()) continue;
            if ((r.h = dlopen(c.c_str(), RTLD_NOW | RTLD_LOCAL))) { r.path = c; break; }
        }
        if (!r.h) return;
        r.getUniqueId = reinterpret_cast<decltype(r.getUniqueId)>(dlsym(r.h, "ncclGetUniqueId"));
        r.commInitRank = reinterpret_cast<decltype(r.commInitRank)>(dlsym(r.h, "ncclCommInitRank"));
        r.allReduce = reinterpret_cast<decltype(r.allReduce)>(dlsym(r.h, "ncclAllReduce"));
        r.commDestroy = reinterpret_cast<decltype(r.commDestroy)>(dlsym(r.h, "ncclCommDestroy"));
        r.errorString = reinterpret_cast<decltype(r.errorString)>(dlsym(r.h, "ncclGetErrorString"));
        if (!r.getUniqueId || !r.commInitRank || !r.allReduce || !r.commDestroy || !r.errorString) {
            dlclose(r.h);
            r.h = nullptr;
        }
    });
    return r.h ? &r : nullptr;
}

int nccl_fail(ncclResult_t e, const char *what) {
    Rccl *r = rccl();
    set_error("%s failed: %s", what, r ? r->errorString(e) : "librccl not loaded");
    return MGDP_E_HIP;
}

}  // namespace

int comm_allreduce_max_dev(mgdp_comm *c, int64_t *d, size_t n, hipStream_t stream) {
    Rccl *r = rccl();
    MGDP_CHECK(r && c && c->nc, MGDP_E_INVALID, "no communicator");
    const ncclResult_t e = r->allReduce(d, d, n, ncclInt64, ncclMax, c->nc, stream);
    if (e != ncclSuccess) return nccl_fail(e, "ncclAllReduce");
    ++c->calls;
    return 0;
}
int64_t *comm_proto(mgdp_comm *c) { return c->d_proto; }
int64_t *comm_host_word(mgdp_comm *c) { return c->h_word; }
int comm_device(const mgdp_comm *c) { return c->device; }

}  // namespace mgdp

extern "C" {

int mgdp_comm_unique_id(uint8_t *id_out) {
    MGDP_CHECK(id_out, MGDP_E_INVALID, "null argument");
    mgdp::Rccl *r = mgdp::rccl();
    MGDP_CHECK(r, MGDP_E_HIP, "librccl could not be loaded (MGDP_RCCL_LIB, a mapped copy, librccl.so.1)");
    ncclUniqueId id;
    const ncclResult_t e = r->getUniqueId(&id);
    if (e != ncclSuccess) return mgdp::nccl_fail(e, "ncclGetUniqueId");
    std::memcpy(id_out, &id, sizeof(id));
    return 0;
}

int mgdp_comm_create(const uint8_t *id, int32_t nranks, int32_t rank, int32_t device, mgdp_comm **out) {
    MGDP_CHECK(id && out, MGDP_E_INVALID, "null argument");
    MGDP_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, MGDP_E_INVALID, "rank %d of %d", rank, nranks);
    *out = nullptr;
    mgdp::Rccl *r = mgdp::rccl();
    MGDP_CHECK(r, MGDP_E_HIP, "librccl could not be loaded (MGDP_RCCL_LIB, a mapped copy, librccl.so.1)");
    mgdp::DeviceGuard guard(device);
    MGDP_CHECK(guard.ok, MGDP_E_HIP, "hipSetDevice(%d) failed", device);
    auto *c = new mgdp_comm;
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    hipError_t he = hipMalloc((void **)&c->d_proto, 8 * sizeof(int64_t));
    if (he == hipSuccess) he = hipMemset(c->d_proto, 0, 8 * sizeof(int64_t));
    if (he == hipSuccess) he = hipHostMalloc((void **)&c->h_word, 8 * sizeof(int64_t), hipHostMallocDefault);
    if (he == hipSuccess) he = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (he != hipSuccess) {
        mgdp_comm_destroy(c);
        return mgdp::hip_fail(he, "communicator buffers", __FILE__, __LINE__);
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    const ncclResult_t e = r->commInitRank(&c->nc, nranks, uid, rank);
    if (e != ncclSuccess) {
        c->nc = nullptr;
        mgdp_comm_destroy(c);
        return mgdp::nccl_fail(e, "ncclCommInitRank");
    }
    *out = c;
    return 0;
}

int mgdp_comm_destroy(mgdp_comm *c) {
    if (!c) return 0;
    mgdp::DeviceGuard guard(c->device);
    if (c->nc) {
        if (mgdp::Rccl *r = mgdp::rccl()) (void)r->commDestroy(c->nc);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->d_proto) (void)hipFree(c->d_proto);
    if (c->h_word) (void)hipHostFree(c->h_word);
    delete c;
    return 0;
}

int mgdp_comm_allreduce_max(mgdp_comm *c, int64_t *vals, int32_t n) {
    MGDP_CHECK(c && vals && n >= 1 && n <= 8, MGDP_E_INVALID, "bad argument (n <= 8 words)");
    mgdp::DeviceGuard guard(c->device);
    std::memcpy(c->h_word, vals, sizeof(int64_t) * n);
    int64_t *d = c->d_proto + 8 - n;  // the tail words: never the device protocol's live ones
    MGDP_HIP(hipMemcpyAsync(d, c->h_word, sizeof(int64_t) * n, hipMemcpyHostToDevice, c->stream));
    if (int rc = mgdp::comm_allreduce_max_dev(c, d, (size_t)n, c->stream)) return rc;
    MGDP_HIP(hipMemcpyAsync(c->h_word, d, sizeof(int64_t) * n, hipMemcpyDeviceToHost, c->stream));
    MGDP_HIP(hipStreamSynchronize(c->stream));
    std::memcpy(vals, c->h_word, sizeof(int64_t) * n);
    return 0;
}

int mgdp_comm_stats(const mgdp_comm *c, int64_t *allreduces, int32_t *nranks, int32_t *rank) {
    MGDP_CHECK(c, MGDP_E_INVALID, "null communicator");
    if (allreduces) *allreduces = c->calls;
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    return 0;
}

}  // extern "C"

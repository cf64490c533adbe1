// comm.cpp -- the communicator of the sharded solve behind the C ABI (mgdp_comm_*): RCCL over xGMI,
// called from the library instead of torch.distributed's ProcessGroupNCCL.  librccl is loaded at
// the first call (dlopen), not linked: a process that never shards does not need it, and in a
// PyTorch process the copy torch already mapped is reused (one RCCL, one HIP runtime).  The
// communicator owns a small device buffer for the protocol's words (include/mgdp.h).
// A second kind, the host communicator (mgdp_comm_create_host), all-reduces through a shared-memory
// segment between the processes of one host instead: RCCL refuses two ranks on one GPU, and that kind
// lets tests run the unchanged mgdp_vi_solve_sharded at world > 1 on a one-GPU box (each device
// all-reduce becomes a stream synchronisation, a host MAX and a copy back: a test path, not xGMI).
#include <dlfcn.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <string>

#include <rccl/rccl.h>

#include "comm.h"

namespace mgdp {
constexpr int kShmMaxRanks = 64;
// The host communicator's shared segment: every rank writes its words into its row of the call's
// slot (two slots alternate by call parity), then adds one to `arrived`; the rank whose add completes
// the call folds the MAX into res[slot] and publishes `gen` = calls done.  A rank can only start call
// g + 1 after call g's publication, which needs every rank's arrival at g, so slot g & 1 is never
// rewritten while a rank still reads call g's result.
struct ShmState {
    std::atomic<uint64_t> arrived;
    std::atomic<uint64_t> gen;
    uint64_t pad[14];
    int64_t vals[2][kShmMaxRanks][8];
    int64_t res[2][8];
};
static_assert(std::atomic<uint64_t>::is_always_lock_free, "process-shared atomics need lock-free words");
}  // namespace mgdp

struct mgdp_comm {
    int kind = 0;                  // 0 = RCCL, 1 = host shared memory (mgdp_comm_create_host)
    ncclComm_t nc = nullptr;
    mgdp::ShmState *shm = nullptr;  // kind 1: the mapped segment
    uint64_t shm_calls = 0;        // kind 1: this rank's calls so far (every rank issues the same sequence)
    int nranks = 0, rank = 0, device = 0;
    int64_t *d_proto = nullptr;  // int64[16] device: [0..7] the device protocol's words, [8..15] host-driven staging
    int64_t *h_word = nullptr;   // pinned int64[8]: host-driven collectives stage through it
    int64_t *h_stage = nullptr;  // pinned int64[8]: kind 1's device all-reduces stage through it
    hipStream_t stream = nullptr;  // host-driven collectives (mgdp_comm_allreduce_max)
    int64_t calls = 0;             // all-reduces issued (mgdp_comm_stats)
    int64_t host_waits = 0;        // host waits on the GPU inside the communicator and the sharded solve
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

// kind 1: MAX of n words over every rank through the shared segment (blocking; 120 s limit)
int shm_allreduce(mgdp_comm *c, int64_t *v, int n) {
    ShmState *s = c->shm;
    const uint64_t g = c->shm_calls++;
    const int slot = (int)(g & 1);
    for (int i = 0; i < n; ++i) s->vals[slot][c->rank][i] = v[i];
    const uint64_t a = s->arrived.fetch_add(1, std::memory_order_acq_rel) + 1;
    if (a == (g + 1) * (uint64_t)c->nranks) {
        for (int i = 0; i < n; ++i) {
            int64_t m = s->vals[slot][0][i];
            for (int r = 1; r < c->nranks; ++r) m = s->vals[slot][r][i] > m ? s->vals[slot][r][i] : m;
            s->res[slot][i] = m;
        }
        s->gen.store(g + 1, std::memory_order_release);
    } else {
        const auto t0 = std::chrono::steady_clock::now();
        while (s->gen.load(std::memory_order_acquire) < g + 1) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) {
                set_error("host communicator: rank %d waited 120 s in all-reduce %llu (a peer is gone or "
                          "issued a different collective sequence)", c->rank, (unsigned long long)g);
                return MGDP_E_INVALID;
            }
            sched_yield();
        }
    }
    for (int i = 0; i < n; ++i) v[i] = s->res[slot][i];
    ++c->calls;
    return 0;
}

}  // namespace

void comm_note_host_wait(mgdp_comm *c) { ++c->host_waits; }

int comm_allreduce_max_dev(mgdp_comm *c, int64_t *d, size_t n, hipStream_t stream) {
    MGDP_CHECK(c && n >= 1 && n <= 8, MGDP_E_INVALID, "no communicator / bad word count");
    if (c->kind == 1) {  // the same in-place device all-reduce, staged through the host
        MGDP_HIP(hipMemcpyAsync(c->h_stage, d, sizeof(int64_t) * n, hipMemcpyDeviceToHost, stream));
        MGDP_HIP(hipStreamSynchronize(stream));
        ++c->host_waits;
        if (int rc = shm_allreduce(c, c->h_stage, (int)n)) return rc;
        MGDP_HIP(hipMemcpyAsync(d, c->h_stage, sizeof(int64_t) * n, hipMemcpyHostToDevice, stream));
        MGDP_HIP(hipStreamSynchronize(stream));  // h_stage is reused by the next call
        return 0;
    }
    Rccl *r = rccl();
    MGDP_CHECK(r && c->nc, MGDP_E_INVALID, "no communicator");
    const ncclResult_t e = r->allReduce(d, d, n, ncclInt64, ncclMax, c->nc, stream);
    if (e != ncclSuccess) return nccl_fail(e, "ncclAllReduce");
    ++c->calls;
    return 0;
}
int64_t *comm_proto(mgdp_comm *c) { return c->d_proto; }
int64_t *comm_host_word(mgdp_comm *c) { return c->h_word; }
int comm_device(const mgdp_comm *c) { return c->device; }

namespace {
// device words, pinned words and the host-driven stream of a new communicator (both kinds)
int comm_buffers(mgdp_comm *c) {
    hipError_t he = hipMalloc((void **)&c->d_proto, 16 * sizeof(int64_t));
    if (he == hipSuccess) he = hipMemset(c->d_proto, 0, 16 * sizeof(int64_t));
    if (he == hipSuccess) he = hipHostMalloc((void **)&c->h_word, 8 * sizeof(int64_t), hipHostMallocDefault);
    if (he == hipSuccess) he = hipHostMalloc((void **)&c->h_stage, 8 * sizeof(int64_t), hipHostMallocDefault);
    if (he == hipSuccess) he = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (he != hipSuccess) return mgdp::hip_fail(he, "communicator buffers", __FILE__, __LINE__);
    return 0;
}
}  // namespace
}  // namespace mgdp

extern "C" {

int mgdp_comm_available(void) {
    MGDP_CHECK(mgdp::rccl(), MGDP_E_HIP, "librccl could not be loaded (MGDP_RCCL_LIB, a mapped copy, librccl.so.1)");
    return 0;
}

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
    if (int rc = mgdp::comm_buffers(c)) {
        mgdp_comm_destroy(c);
        return rc;
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

int mgdp_comm_create_host(const char *name, int32_t nranks, int32_t rank, int32_t device, mgdp_comm **out) {
    MGDP_CHECK(name && out && name[0] == '/' && !std::strchr(name + 1, '/') && std::strlen(name) < 200, MGDP_E_INVALID,
               "segment name: \"/\" then no further \"/\"");
    MGDP_CHECK(nranks >= 1 && nranks <= mgdp::kShmMaxRanks && rank >= 0 && rank < nranks, MGDP_E_INVALID,
               "rank %d of %d (at most %d ranks)", rank, nranks, mgdp::kShmMaxRanks);
    *out = nullptr;
    mgdp::DeviceGuard guard(device);
    MGDP_CHECK(guard.ok, MGDP_E_HIP, "hipSetDevice(%d) failed", device);
    // every rank opens (creating if needed) the same zero-filled segment: no rank waits for another
    const std::string path = std::string("/dev/shm") + name;
    const int fd = open(path.c_str(), O_RDWR | O_CREAT, 0600);
    MGDP_CHECK(fd >= 0, MGDP_E_INVALID, "open(%s) failed", path.c_str());
    const bool sized = ftruncate(fd, (off_t)sizeof(mgdp::ShmState)) == 0;
    void *m = sized ? mmap(nullptr, sizeof(mgdp::ShmState), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0) : MAP_FAILED;
    close(fd);
    MGDP_CHECK(m != MAP_FAILED, MGDP_E_INVALID, "mapping %s failed", path.c_str());
    auto *c = new mgdp_comm;
    c->kind = 1;
    c->shm = static_cast<mgdp::ShmState *>(m);
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    if (int rc = mgdp::comm_buffers(c)) {
        mgdp_comm_destroy(c);
        return rc;
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
    if (c->shm) (void)munmap(c->shm, sizeof(mgdp::ShmState));
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->d_proto) (void)hipFree(c->d_proto);
    if (c->h_word) (void)hipHostFree(c->h_word);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    delete c;
    return 0;
}

int mgdp_comm_allreduce_max(mgdp_comm *c, int64_t *vals, int32_t n) {
    MGDP_CHECK(c && vals && n >= 1 && n <= 8, MGDP_E_INVALID, "bad argument (n <= 8 words)");
    ++c->host_waits;
    if (c->kind == 1) return mgdp::shm_allreduce(c, vals, n);
    mgdp::DeviceGuard guard(c->device);
    std::memcpy(c->h_word, vals, sizeof(int64_t) * n);
    // staged in words [8..15]: never the device protocol's ([0..7]), which a sharded solve of another
    // handle in this process may be all-reducing on its own stream
    int64_t *d = c->d_proto + 8;
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

int mgdp_comm_host_waits(const mgdp_comm *c, int64_t *waits, int32_t *kind) {
    MGDP_CHECK(c, MGDP_E_INVALID, "null communicator");
    if (waits) *waits = c->host_waits;
    if (kind) *kind = c->kind;
    return 0;
}

}  // extern "C"

// sv_comm.cpp — RCCL communicators for the multi-GPU modes.
//
// The reference has no distributed code; the build's multi-GPU step is a gather of the
// finished disparity rows / frames to one device over xGMI.  RCCL (librccl.so.1, ROCm) is
// loaded with dlopen on first use, so a single-GPU process never maps it.  Two set-ups:
//   * one process per GPU (bench.py under torch.distributed.run): sv_comm_init_rank with a
//     unique id that rank 0 publishes (stereovision_amd/distributed.py: a file rendezvous);
//   * one process driving several GPUs: sv_comm_init_all (ncclCommInitAll), used by the
//     sv_*_multi entry points inside ncclGroupStart/End.
// Blocking helpers (barrier, max-allreduce) run on the communicator's own stream.
#include <dlfcn.h>

#include <chrono>
#include <cstring>
#include <thread>
#include <mutex>
#include <new>
#include <string>

#include <rccl/rccl.h>

#include "sv_internal.h"
#include "../../include/stereovision_amd.h"

struct sv_comm {
    int device = 0, rank = 0, nranks = 1;
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    void* scratch = nullptr;   // 64 B: barrier / allreduce operand
    bool nonblocking = false;  // initialised with ncclConfig.blocking = 0: calls may return
                               // ncclInProgress and are settled by polling (settle)
    std::mutex mu;
};

namespace {

struct Rccl {
    void* h = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    // non-blocking initialisation (optional symbols: without them init is the blocking call)
    decltype(&ncclCommInitRankConfig) init_rank_config = nullptr;
    decltype(&ncclCommGetAsyncError) async_error = nullptr;
    decltype(&ncclCommAbort) abort = nullptr;
    std::string load_error;
};

Rccl& rccl_state() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* names[] = {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"};
        for (const char* n : names) {
            r.h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
            if (r.h) break;
        }
        if (!r.h) {
            const char* e = dlerror();
            r.load_error = std::string("dlopen(librccl.so.1) failed: ") + (e ? e : "?");
            return;
        }
        auto sym = [&](const char* s) { return dlsym(r.h, s); };
        r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
        r.init_rank = reinterpret_cast<decltype(r.init_rank)>(sym("ncclCommInitRank"));
        r.init_all = reinterpret_cast<decltype(r.init_all)>(sym("ncclCommInitAll"));
        r.destroy = reinterpret_cast<decltype(r.destroy)>(sym("ncclCommDestroy"));
        r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(sym("ncclAllReduce"));
        r.send = reinterpret_cast<decltype(r.send)>(sym("ncclSend"));
        r.recv = reinterpret_cast<decltype(r.recv)>(sym("ncclRecv"));
        r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
        r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
        r.init_rank_config = reinterpret_cast<decltype(r.init_rank_config)>(sym("ncclCommInitRankConfig"));
        r.async_error = reinterpret_cast<decltype(r.async_error)>(sym("ncclCommGetAsyncError"));
        r.abort = reinterpret_cast<decltype(r.abort)>(sym("ncclCommAbort"));
        if (!r.get_unique_id || !r.init_rank || !r.init_all || !r.destroy || !r.all_reduce || !r.send ||
            !r.recv || !r.group_start || !r.group_end || !r.error_string) {
            r.load_error = "librccl.so.1 lacks an expected symbol";
            r.h = nullptr;
        }
    });
    return r;
}

Rccl* rccl() {
    Rccl& r = rccl_state();
    return r.h ? &r : nullptr;
}

int comm_fail(int code, const std::string& msg) { return sv::set_error(code, msg); }

int nccl_fail(Rccl* r, ncclResult_t e, const char* what) {
    return comm_fail(SV_EHIP, std::string(what) + ": " + (r ? r->error_string(e) : "rccl unavailable"));
}

#define SV_NCCL(r, call)                                              \
    do {                                                              \
        ncclResult_t e_ = (call);                                     \
        if (e_ != ncclSuccess) return nccl_fail((r), e_, #call);      \
    } while (0)

#define SV_CHIP(call)                                                 \
    do {                                                              \
        hipError_t e_ = (call);                                       \
        if (e_ != hipSuccess)                                         \
            return comm_fail(SV_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

Rccl* need_rccl(int* rc) {
    Rccl* r = rccl();
    if (!r) {
        const std::string& why = rccl_state().load_error;
        *rc = comm_fail(SV_ENODEV, why.empty() ? std::string("RCCL unavailable") : why);
    }
    return r;
}

// A call on a non-blocking communicator may return ncclInProgress: poll its state until it
// settles (timeout_s <= 0: no limit; the deadline returns ncclInProgress).
ncclResult_t settle(Rccl* r, ncclComm_t comm, ncclResult_t e, double timeout_s) {
    if (e != ncclInProgress || !r->async_error || !comm) return e;
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
    for (;;) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t q = r->async_error(comm, &st);
        if (q != ncclSuccess) return q;
        if (st != ncclInProgress) return st;
        if (timeout_s > 0 && std::chrono::steady_clock::now() > t_end) return ncclInProgress;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

// send / recv inside a group on a non-blocking communicator may report ncclInProgress: queued
inline ncclResult_t queued(ncclResult_t e) { return e == ncclInProgress ? ncclSuccess : e; }

int finish_comm(sv_comm* c) {
    SV_CHIP(hipSetDevice(c->device));
    SV_CHIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    SV_CHIP(hipMalloc(&c->scratch, 64));
    return 0;
}

}  // namespace

namespace sv {
// the multi-device entry points of sv_capi.cpp enqueue their transfers through these
int comm_group_start() {
    int rc = 0;
    Rccl* r = need_rccl(&rc);
    if (!r) return rc;
    SV_NCCL(r, r->group_start());
    return 0;
}
int comm_group_end() {
    int rc = 0;
    Rccl* r = need_rccl(&rc);
    if (!r) return rc;
    SV_NCCL(r, r->group_end());
    return 0;
}
int comm_send(sv_comm* c, const void* buf, size_t bytes, int peer, hipStream_t s) {
    int rc = 0;
    Rccl* r = need_rccl(&rc);
    if (!r) return rc;
    SV_NCCL(r, r->send(buf, bytes, ncclChar, peer, c->comm, s));
    return 0;
}
int comm_recv(sv_comm* c, void* buf, size_t bytes, int peer, hipStream_t s) {
    int rc = 0;
    Rccl* r = need_rccl(&rc);
    if (!r) return rc;
    SV_NCCL(r, r->recv(buf, bytes, ncclChar, peer, c->comm, s));
    return 0;
}
int comm_rank(const sv_comm* c) { return c->rank; }
int comm_size(const sv_comm* c) { return c->nranks; }
int comm_device(const sv_comm* c) { return c->device; }
}  // namespace sv

extern "C" {

int sv_comm_available(void) { return rccl() ? 1 : 0; }

int sv_comm_unique_id(uint8_t* id) {
    if (!id) return comm_fail(SV_EINVAL, "null id buffer");
    int rc = 0;
    Rccl* r = need_rccl(&rc);
    if (!r) return rc;
    ncclUniqueId u;
    SV_NCCL(r, r->get_unique_id(&u));
    static_assert(sizeof(u.internal) == SV_COMM_ID_BYTES, "unique id size");
    std::memcpy(id, u.internal, SV_COMM_ID_BYTES);
    return 0;
}

int sv_comm_init_rank(int device, int nranks, int rank, const uint8_t* id, double timeout_s, sv_comm** out) {
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks) return comm_fail(SV_EINVAL, "bad communicator arguments");
    *out = nullptr;
    int rc = 0;
    Rccl* r = need_rccl(&rc);
    if (!r) return rc;
    sv_comm* c = new (std::nothrow) sv_comm();
    if (!c) return comm_fail(SV_ENOMEM, "communicator allocation failed");
    c->device = device;
    c->rank = rank;
    c->nranks = nranks;
    ncclUniqueId u;
    std::memcpy(u.internal, id, SV_COMM_ID_BYTES);
    hipError_t he = hipSetDevice(device);
    if (he != hipSuccess) {
        delete c;
        return comm_fail(SV_EHIP, std::string("hipSetDevice: ") + hipGetErrorString(he));
    }
    ncclResult_t e;
    if (r->init_rank_config && r->async_error && r->abort) {
        // non-blocking: a rank whose peers died in bootstrap comes back at the deadline
        //  instead of blocking forever inside a collective initialisation
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        e = r->init_rank_config(&c->comm, nranks, u, rank, &cfg);
        e = settle(r, c->comm, e == ncclSuccess ? ncclInProgress : e, timeout_s);
        c->nonblocking = true;
    } else {
        e = r->init_rank(&c->comm, nranks, u, rank);
    }
    if (e != ncclSuccess) {
        if (c->comm && r->abort) r->abort(c->comm);
        delete c;
        if (e == ncclInProgress)
            return comm_fail(SV_EHIP, "ncclCommInitRank did not complete within " + std::to_string(timeout_s) +
                                          " s (a peer failed or never joined); aborted");
        return nccl_fail(r, e, "ncclCommInitRank");
    }
    rc = finish_comm(c);
    if (rc) {
        sv_comm_destroy(c);
        return rc;
    }
    *out = c;
    return 0;
}

int sv_comm_init_all(int ndev, const int* devices, sv_comm** comms) {
    if (ndev < 1 || !devices || !comms) return comm_fail(SV_EINVAL, "bad communicator arguments");
    for (int k = 0; k < ndev; ++k) {
        comms[k] = nullptr;
        for (int j = 0; j < k; ++j)
            if (devices[j] == devices[k]) return comm_fail(SV_EINVAL, "sv_comm_init_all: a device appears twice");
    }
    int rc = 0;
    Rccl* r = need_rccl(&rc);
    if (!r) return rc;
    ncclComm_t raw[64];
    if (ndev > 64) return comm_fail(SV_EINVAL, "at most 64 devices");
    SV_NCCL(r, r->init_all(raw, ndev, devices));
    for (int k = 0; k < ndev; ++k) {
        sv_comm* c = new (std::nothrow) sv_comm();
        if (c) {
            c->device = devices[k];
            c->rank = k;
            c->nranks = ndev;
            c->comm = raw[k];
            rc = finish_comm(c);
        }
        if (!c || rc) {
            if (c) sv_comm_destroy(c);
            else r->destroy(raw[k]);
            for (int j = k + 1; j < ndev; ++j) r->destroy(raw[j]);
            for (int j = 0; j < k; ++j) {
                sv_comm_destroy(comms[j]);
                comms[j] = nullptr;
            }
            return rc ? rc : comm_fail(SV_ENOMEM, "communicator allocation failed");
        }
        comms[k] = c;
    }
    return 0;
}

void sv_comm_destroy(sv_comm* c) {
    if (!c) return;
    Rccl* r = rccl();
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm && r) r->destroy(c->comm);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int sv_comm_rank(sv_comm* c, int* rank, int* nranks, int* device) {
    if (!c) return comm_fail(SV_EINVAL, "null communicator");
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->nranks;
    if (device) *device = c->device;
    return 0;
}

int sv_comm_barrier(sv_comm* c) {
    double v = 0.0;
    return sv_comm_allreduce_max_f64(c, &v);
}

int sv_comm_allreduce_max_f64(sv_comm* c, double* value) {
    if (!c || !value) return comm_fail(SV_EINVAL, "bad allreduce arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    Rccl* r = rccl();
    if (!r) return comm_fail(SV_ENODEV, "RCCL unavailable");
    SV_CHIP(hipSetDevice(c->device));
    SV_CHIP(hipMemcpyAsync(c->scratch, value, sizeof(double), hipMemcpyHostToDevice, c->stream));
    SV_NCCL(r, settle(r, c->comm, r->all_reduce(c->scratch, c->scratch, 1, ncclFloat64, ncclMax, c->comm, c->stream), 0));
    SV_CHIP(hipMemcpyAsync(value, c->scratch, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    SV_CHIP(hipStreamSynchronize(c->stream));
    return 0;
}

int sv_comm_gatherv(sv_comm* c, const void* d_send, uint64_t send_bytes, void* d_recv, const uint64_t* recv_offsets,
                    const uint64_t* recv_bytes, int root, void* stream) {
    if (!c || root < 0 || root >= c->nranks) return comm_fail(SV_EINVAL, "bad gather arguments");
    if (send_bytes && !d_send) return comm_fail(SV_EINVAL, "null send buffer");
    if (c->rank == root && (!d_recv || !recv_offsets || !recv_bytes)) return comm_fail(SV_EINVAL, "root needs recv layout");
    if (c->rank == root && recv_bytes[root] != send_bytes) return comm_fail(SV_EINVAL, "root's own block size differs");
    Rccl* r = rccl();
    if (!r) return comm_fail(SV_ENODEV, "RCCL unavailable");
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
    SV_CHIP(hipSetDevice(c->device));
    SV_NCCL(r, queued(r->group_start()));
    ncclResult_t e = ncclSuccess;
    if (c->rank == root) {
        for (int k = 0; k < c->nranks && e == ncclSuccess; ++k) {
            if (k == root || recv_bytes[k] == 0) continue;
            e = queued(r->recv(static_cast<uint8_t*>(d_recv) + recv_offsets[k], recv_bytes[k], ncclChar, k, c->comm, s));
        }
    } else if (send_bytes) {
        e = queued(r->send(d_send, send_bytes, ncclChar, root, c->comm, s));
    }
    ncclResult_t e2 = settle(r, c->comm, r->group_end(), 0);
    if (e != ncclSuccess) return nccl_fail(r, e, "ncclSend/ncclRecv");
    if (e2 != ncclSuccess) return nccl_fail(r, e2, "ncclGroupEnd");
    if (c->rank == root && send_bytes) {
        uint8_t* dst = static_cast<uint8_t*>(d_recv) + recv_offsets[root];
        if (dst != d_send) SV_CHIP(hipMemcpyAsync(dst, d_send, send_bytes, hipMemcpyDeviceToDevice, s));
    }
    return 0;
}

int sv_comm_scatterv(sv_comm* c, const void* d_send, const uint64_t* send_offsets, const uint64_t* send_bytes,
                     void* d_recv, uint64_t recv_bytes, int root, void* stream) {
    if (!c || root < 0 || root >= c->nranks) return comm_fail(SV_EINVAL, "bad scatter arguments");
    if (recv_bytes && !d_recv) return comm_fail(SV_EINVAL, "null receive buffer");
    if (c->rank == root && (!d_send || !send_offsets || !send_bytes)) return comm_fail(SV_EINVAL, "root needs send layout");
    if (c->rank == root && send_bytes[root] != recv_bytes) return comm_fail(SV_EINVAL, "root's own block size differs");
    Rccl* r = rccl();
    if (!r) return comm_fail(SV_ENODEV, "RCCL unavailable");
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
    SV_CHIP(hipSetDevice(c->device));
    SV_NCCL(r, queued(r->group_start()));
    ncclResult_t e = ncclSuccess;
    if (c->rank == root) {
        for (int k = 0; k < c->nranks && e == ncclSuccess; ++k) {
            if (k == root || send_bytes[k] == 0) continue;
            e = queued(r->send(static_cast<const uint8_t*>(d_send) + send_offsets[k], send_bytes[k], ncclChar, k, c->comm, s));
        }
    } else if (recv_bytes) {
        e = queued(r->recv(d_recv, recv_bytes, ncclChar, root, c->comm, s));
    }
    ncclResult_t e2 = settle(r, c->comm, r->group_end(), 0);
    if (e != ncclSuccess) return nccl_fail(r, e, "ncclSend/ncclRecv");
    if (e2 != ncclSuccess) return nccl_fail(r, e2, "ncclGroupEnd");
    if (c->rank == root && recv_bytes) {
        const uint8_t* src = static_cast<const uint8_t*>(d_send) + send_offsets[root];
        if (src != d_recv) SV_CHIP(hipMemcpyAsync(d_recv, src, recv_bytes, hipMemcpyDeviceToDevice, s));
    }
    return 0;
}

int sv_comm_synchronize(sv_comm* c) {
    if (!c) return comm_fail(SV_EINVAL, "null communicator");
    SV_CHIP(hipSetDevice(c->device));
    SV_CHIP(hipStreamSynchronize(c->stream));
    return 0;
}

}  // extern "C"

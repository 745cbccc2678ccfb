// Process-per-GPU communicators for prove_shard.
//
//   CallbackComm  the caller's transport (lsp_comm_ops: host-buffer allgather
//                 and broadcast), e.g. a torch.distributed gloo group or the
//                 Rust prover's own channel.  Device data is staged through
//                 host memory.
//   RcclComm      RCCL over xGMI, device buffers on the context's stream.
//                 librccl is opened with dlopen when a context attaches it,
//                 so the library itself has no RCCL dependency.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "comm.hpp"
#include "prove_internal.hpp"

namespace lsp {

namespace {
struct CallbackComm : Comm {
    lsp_comm_ops ops;
    std::vector<uint8_t> hs, hr;
    explicit CallbackComm(const lsp_comm_ops& o) : ops(o) {
        rank = o.rank;
        size = o.size;
    }

  protected:
    void do_allgather(lsp_ctx* ctx, const void* send, void* recv, size_t bytes) override {
        hs.resize(bytes);
        hr.resize(bytes * (size_t)size);
        LSP_HIP(hipMemcpyAsync(hs.data(), send, bytes, hipMemcpyDeviceToHost, ctx->stream));
        LSP_HIP(hipStreamSynchronize(ctx->stream));
        LSP_REQUIRE(ops.allgather(ops.user, hs.data(), hr.data(), bytes) == 0, LSP_E_STATE,
                    "communicator allgather failed");
        LSP_HIP(hipMemcpyAsync(recv, hr.data(), hr.size(), hipMemcpyHostToDevice, ctx->stream));
        LSP_HIP(hipStreamSynchronize(ctx->stream));
    }
    void do_bcast(lsp_ctx* ctx, void* buf, size_t bytes, int root) override {
        hs.resize(bytes);
        if (rank == root) {
            LSP_HIP(hipMemcpyAsync(hs.data(), buf, bytes, hipMemcpyDeviceToHost, ctx->stream));
            LSP_HIP(hipStreamSynchronize(ctx->stream));
        }
        LSP_REQUIRE(ops.bcast(ops.user, hs.data(), bytes, root) == 0, LSP_E_STATE, "communicator bcast failed");
        if (rank != root) {
            LSP_HIP(hipMemcpyAsync(buf, hs.data(), bytes, hipMemcpyHostToDevice, ctx->stream));
            LSP_HIP(hipStreamSynchronize(ctx->stream));
        }
    }
};

struct Rccl {
    void* so = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

const Rccl& rccl() {
    static Rccl r = [] {
        Rccl x;
        // LSP_RCCL_LIB first: the RCCL built against the HIP/HSA runtime already in
        // the process (the Python layer points it at torch's bundled copy, because
        // torch's runtime is the one this library binds when torch is loaded first)
        const char* env = std::getenv("LSP_RCCL_LIB");
        if (env && *env) x.so = dlopen(env, RTLD_NOW | RTLD_LOCAL);
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            if (x.so) break;
            x.so = dlopen(name, RTLD_NOW | RTLD_LOCAL);
        }
        if (!x.so) return x;
        x.get_unique_id = (decltype(x.get_unique_id))dlsym(x.so, "ncclGetUniqueId");
        x.init_rank = (decltype(x.init_rank))dlsym(x.so, "ncclCommInitRank");
        x.destroy = (decltype(x.destroy))dlsym(x.so, "ncclCommDestroy");
        x.all_gather = (decltype(x.all_gather))dlsym(x.so, "ncclAllGather");
        x.broadcast = (decltype(x.broadcast))dlsym(x.so, "ncclBroadcast");
        x.error_string = (decltype(x.error_string))dlsym(x.so, "ncclGetErrorString");
        return x;
    }();
    LSP_REQUIRE(r.so && r.get_unique_id && r.init_rank && r.destroy && r.all_gather && r.broadcast && r.error_string,
                LSP_E_STATE, "RCCL (librccl.so.1) is not loadable");
    return r;
}

#define LSP_RCCL(x)                                                                                       \
    do {                                                                                                  \
        ncclResult_t r_ = (x);                                                                            \
        if (r_ != ncclSuccess) throw LspError(LSP_E_STATE, std::string(#x) + " -> " + rccl().error_string(r_)); \
    } while (0)

struct RcclComm : Comm {
    ncclComm_t comm = nullptr;
    RcclComm(const ncclUniqueId& id, int r, int n) {
        rank = r;
        size = n;
        const auto t0 = std::chrono::steady_clock::now();
        LSP_RCCL(rccl().init_rank(&comm, n, id, r));
        init_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    ~RcclComm() override {
        if (comm) rccl().destroy(comm);
    }
    // Payloads are whole field elements (32-byte multiples): 64-bit words keep
    // the element counts small (a 2^26-row proof's coefficient blocks are 2 GiB
    // per rank), and broadcasts go in <= 1 GiB pieces
    static ncclDataType_t dtype(size_t bytes, size_t& count) {
        if (bytes % 8 == 0) {
            count = bytes / 8;
            return ncclUint64;
        }
        count = bytes;
        return ncclUint8;
    }

  protected:
    void do_allgather(lsp_ctx* ctx, const void* send, void* recv, size_t bytes) override {
        size_t n;
        const ncclDataType_t t = dtype(bytes, n);
        LSP_RCCL(rccl().all_gather(send, recv, n, t, comm, ctx->stream));
    }
    void do_bcast(lsp_ctx* ctx, void* buf, size_t bytes, int root) override {
        constexpr size_t piece = (size_t)1 << 30;
        for (size_t off = 0; off < bytes; off += piece) {
            size_t n;
            const ncclDataType_t t = dtype(std::min(piece, bytes - off), n);
            char* p = (char*)buf + off;
            LSP_RCCL(rccl().broadcast(p, p, n, t, root, comm, ctx->stream));
        }
    }
};
}  // namespace

Comm* make_callback_comm(const lsp_comm_ops& ops) { return new CallbackComm(ops); }

void rccl_unique_id(uint8_t out[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId id;
    LSP_RCCL(rccl().get_unique_id(&id));
    std::memcpy(out, &id, 128);
}

Comm* make_rccl_comm(const uint8_t id[128], int rank, int size) {
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    return new RcclComm(u, rank, size);
}

}  // namespace lsp

// Exchange layer of the sharded prover.  A proof over G ranks
// needs only two collectives, both on device buffers and both small except
// the quotient-chunk exchange: allgather (subtree roots, the FRI vector once
// it is short, query openings) and broadcast (the quotient chunks, one
// broadcast per holding rank; opened values from rank 0).  The transcript
// runs redundantly on every rank, so no challenge is ever sent.
//
//   SoloComm     G = 1 (the single-GPU prover; allgather is a copy)
//   ThreadComm   G ranks of one process, one thread and one lsp_ctx each:
//                distinct GPUs of the node (device-to-device copies over
//                xGMI with peer access on) or the same GPU repeated
//                ("virtual ranks", how the sharded path is tested on one GPU)
//   RcclComm     one process per GPU over RCCL (comm_rccl.cpp)
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <string>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include "host.hpp"

namespace lsp {

// One collective of a proof, as the communicator's log keeps it
// (lsp_comm_log): op 'A' allgather (bytes = each rank's share) or 'B'
// broadcast (bytes = the buffer, root), what it carried, and the device time
// between events recorded on the context's stream around it -- the wait for
// the slowest peer included
struct CommRec {
    char op;
    size_t bytes;
    int root;
    std::string tag;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    double ms = -1;
};

struct Comm {
    int rank = 0, size = 1;
    double init_ms = 0;          // communicator creation (RCCL: ncclCommInitRank), wall ms
    std::vector<CommRec> log;    // the collectives since the last begin_log()
    // Exchange calibration (lsp_comm_selftest, calibrate_exchange in prove.cpp),
    // the minimum over the ranks so every rank plans the same collectives:
    // allgather bandwidth into one rank ((G - 1) shares / wall time, GB/s), the
    // inverse NTT's rate on this GPU (G elements/s), and the probe's size.
    // 0 = not measured (then the split inverse is the default).
    double ag_gbs = 0, intt_gelem_s = 0;
    size_t ag_probe_bytes = 0;
    // every rank's own probe results, rank order, 3 per rank: allgather GB/s of
    // the 4 MiB probe, of the 256 MiB probe (0: not run), inverse-NTT G
    // elements/s (lsp_comm_calibration) -- so a biased minimum can be seen
    std::vector<double> calib_raw;
    std::string calib_status = "not calibrated";
    virtual ~Comm() {
        for (CommRec& r : log) {
            if (r.e0) (void)hipEventDestroy(r.e0);
            if (r.e1) (void)hipEventDestroy(r.e1);
        }
    }
    // LoopbackComm: peers' data is fabricated, so the proof's self-checks
    // (the FRI final polynomial's degree) cannot hold and are skipped
    virtual bool rehearsal() const { return false; }
    // recv[r * bytes ...] = rank r's send (device buffers, ordered on ctx->stream)
    void allgather(lsp_ctx* ctx, const void* send, void* recv, size_t bytes, const char* tag = "") {
        const size_t k = rec_begin(ctx, 'A', bytes, -1, tag);
        do_allgather(ctx, send, recv, bytes);
        rec_end(ctx, k);
    }
    // every rank's buf = root's buf (device buffer)
    void bcast(lsp_ctx* ctx, void* buf, size_t bytes, int root, const char* tag = "") {
        const size_t k = rec_begin(ctx, 'B', bytes, root, tag);
        do_bcast(ctx, buf, bytes, root);
        rec_end(ctx, k);
    }
    // a new proof: drop the previous log (its events go back to the context's pool)
    void begin_log(lsp_ctx* ctx) {
        for (CommRec& r : log) {
            if (r.e0) ctx->event_pool.push_back(r.e0);
            if (r.e1) ctx->event_pool.push_back(r.e1);
        }
        log.clear();
    }
    // the device times of the logged collectives (waits for the last event)
    void resolve_log() {
        for (CommRec& r : log) {
            if (r.ms >= 0 || !r.e0 || !r.e1) continue;
            float ms = 0;
            LSP_HIP(hipEventSynchronize(r.e1));
            LSP_HIP(hipEventElapsedTime(&ms, r.e0, r.e1));
            r.ms = ms;
        }
    }

    // host-vector conveniences over the device collectives
    std::vector<Fr> allgather_fr(lsp_ctx* ctx, const Fr* host, size_t n, const char* tag = "") {
        Fr* s = ctx->fbuf("comm_send", n);
        Fr* r = ctx->fbuf("comm_recv", n * (size_t)size);
        LSP_HIP(hipMemcpyAsync(s, host, n * sizeof(Fr), hipMemcpyHostToDevice, ctx->stream));
        allgather(ctx, s, r, n * sizeof(Fr), tag);
        std::vector<Fr> out(n * (size_t)size);
        LSP_HIP(hipMemcpyAsync(out.data(), r, out.size() * sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
        LSP_HIP(hipStreamSynchronize(ctx->stream));
        return out;
    }

  protected:
    virtual void do_allgather(lsp_ctx* ctx, const void* send, void* recv, size_t bytes) = 0;
    virtual void do_bcast(lsp_ctx* ctx, void* buf, size_t bytes, int root) = 0;
    // SoloComm (one rank) keeps no log: its "collectives" are local copies
    virtual bool logs() const { return size > 1; }

  private:
    hipEvent_t take_event(lsp_ctx* ctx) {
        hipEvent_t e;
        if (!ctx->event_pool.empty()) {
            e = ctx->event_pool.back();
            ctx->event_pool.pop_back();
        } else {
            LSP_HIP(hipEventCreate(&e));
        }
        return e;
    }
    size_t rec_begin(lsp_ctx* ctx, char op, size_t bytes, int root, const char* tag) {
        if (!logs() || log.size() >= 4096) return SIZE_MAX;
        CommRec r;
        r.op = op;
        r.bytes = bytes;
        r.root = root;
        r.tag = tag ? tag : "";
        r.e0 = take_event(ctx);
        LSP_HIP(hipEventRecord(r.e0, ctx->stream));
        log.push_back(std::move(r));
        return log.size() - 1;
    }
    void rec_end(lsp_ctx* ctx, size_t k) {
        if (k == SIZE_MAX) return;
        log[k].e1 = take_event(ctx);
        LSP_HIP(hipEventRecord(log[k].e1, ctx->stream));
    }
};

struct SoloComm : Comm {
  protected:
    void do_allgather(lsp_ctx* ctx, const void* send, void* recv, size_t bytes) override {
        if (send != recv)
            LSP_HIP(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    }
    void do_bcast(lsp_ctx*, void*, size_t, int) override {}
};

// Rehearsal of ONE rank of a G-rank proof on one GPU (lsp_ctx_attach_loopback):
// rank g runs its own share of every phase at full size, and the peers' parts
// of each exchange are fabricated locally -- allgather slots of other ranks get
// a copy of this rank's payload, a broadcast from another root leaves zeros (a
// valid field element).  The proof it returns is not a valid proof; what it
// measures is rank g's device memory and per-phase time at the real shapes,
// e.g. one rank of BASELINE configs[3] (2^26 rows over 8 GPUs) on a single GPU.
struct LoopbackComm : Comm {
    LoopbackComm(int r, int n) {
        rank = r;
        size = n;
    }
    bool rehearsal() const override { return true; }

  protected:
    void do_allgather(lsp_ctx* ctx, const void* send, void* recv, size_t bytes) override {
        for (int r = 0; r < size; ++r) {
            void* dst = (char*)recv + (size_t)r * bytes;
            if (dst != send) LSP_HIP(hipMemcpyAsync(dst, send, bytes, hipMemcpyDeviceToDevice, ctx->stream));
        }
    }
    void do_bcast(lsp_ctx* ctx, void* buf, size_t bytes, int root) override {
        if (root != rank) LSP_HIP(hipMemsetAsync(buf, 0, bytes, ctx->stream));
    }
};

// Shared state of an in-process group: a generation barrier that any rank can
// abort (a rank that throws must not leave the others waiting forever).
struct ThreadGroup {
    int size;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool aborted = false;
    std::vector<const void*> slot;
    std::vector<int> device;
    explicit ThreadGroup(int n) : size(n), slot(n, nullptr), device(n, 0) {}
    void barrier() {
        std::unique_lock<std::mutex> lk(m);
        if (aborted) throw LspError(LSP_E_STATE, "another rank of the group failed");
        const uint64_t g = gen;
        if (++arrived == size) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return;
        }
        cv.wait(lk, [&] { return gen != g || aborted; });
        if (aborted) throw LspError(LSP_E_STATE, "another rank of the group failed");
    }
    void abort() {
        std::lock_guard<std::mutex> lk(m);
        aborted = true;
        cv.notify_all();
    }
};

struct ThreadComm : Comm {
    ThreadGroup* grp;
    ThreadComm(ThreadGroup* g, int r) : grp(g) {
        rank = r;
        size = g->size;
    }

  protected:
    void do_allgather(lsp_ctx* ctx, const void* send, void* recv, size_t bytes) override {
        LSP_HIP(hipStreamSynchronize(ctx->stream));  // send is complete
        grp->slot[rank] = send;
        grp->barrier();
        for (int r = 0; r < size; ++r) {
            void* dst = (char*)recv + (size_t)r * bytes;
            if (grp->device[r] == ctx->device)
                LSP_HIP(hipMemcpyAsync(dst, grp->slot[r], bytes, hipMemcpyDeviceToDevice, ctx->stream));
            else
                LSP_HIP(hipMemcpyPeerAsync(dst, ctx->device, grp->slot[r], grp->device[r], bytes, ctx->stream));
        }
        LSP_HIP(hipStreamSynchronize(ctx->stream));
        grp->barrier();  // peers may reuse their send buffers only after every copy
    }
    void do_bcast(lsp_ctx* ctx, void* buf, size_t bytes, int root) override {
        LSP_HIP(hipStreamSynchronize(ctx->stream));
        if (rank == root) grp->slot[root] = buf;
        grp->barrier();
        if (rank != root) {
            if (grp->device[root] == ctx->device)
                LSP_HIP(hipMemcpyAsync(buf, grp->slot[root], bytes, hipMemcpyDeviceToDevice, ctx->stream));
            else
                LSP_HIP(hipMemcpyPeerAsync(buf, ctx->device, grp->slot[root], grp->device[root], bytes, ctx->stream));
            LSP_HIP(hipStreamSynchronize(ctx->stream));
        }
        grp->barrier();
    }
};

}  // namespace lsp

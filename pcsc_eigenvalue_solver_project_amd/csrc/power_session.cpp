// Power-iteration session: the host side of the fused device loop (include/eigsol_hip.h).
//
// Mirrors powerMethodImpl (src/power_method/power_method.hpp:47-99): begin() plays :60-66
// (x0 normalisation, lambda = 0, counters), each step() enqueues fused iterations of :68-96,
// finish() returns the EigenResult fields of :98.  The termination logic runs on the device
// (power_decide in internal.hpp), so the host only polls a done word between chunks.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#include <cxxabi.h>

#include "kernels_common.hpp"

namespace eigsol {
int csr_grid(eigsol_csr* A, int* grid, bool peer = false);
const void* csr_power_kernel(const eigsol_csr* A, bool peer);
int csr_power_launch(eigsol_csr* A, int64_t xlen, void* buf0, void* buf1, PowerCtl* ctl,
                     const void* rank_part, int nranks, void* my_part, void* blk_part, void* trace,
                     int parity, int grid, const dev::PeerArgs* peer = nullptr, int part = -1);
int64_t csr_bin_split_row(const eigsol_csr* A);
int dist_exchange_part(eigsol_csr* A, void* y, void* rank_part, int part, const std::vector<int64_t>& split,
                       hipStream_t comm_st, hipEvent_t* ev);
int peer_begin_launch(eigsol_ctx* ctx, int dtype, const dev::PeerArgs& pa, const void* x_own, int64_t npush,
                      const void* mine);
int coll_allgather(eigsol_ctx* ctx, const void* mine, size_t bytes, void* all);
int coll_barrier(eigsol_ctx* ctx);
int dense_grid(eigsol_dense* A, int* grid);
int dense_power_launch(eigsol_dense* A, void* buf0, void* buf1, PowerCtl* ctl,
                       const void* rank_part, int nranks, void* my_part, void* blk_part,
                       void* trace, int parity, int grid);
int norm_partial_launch(eigsol_ctx* ctx, int dtype, const void* x, int64_t n, PowerCtl* ctl,
                        void* blk_part, void* out, int grid);
int scale_out_launch(eigsol_ctx* ctx, int dtype, const void* src, double nrm, void* dst, int64_t n);
int dist_exchange(eigsol_csr* A, void* y, void* rank_part);
struct ShiftFactor;
int shift_factor_csr(eigsol_csr* A, const void* sigma, ShiftFactor** out);
int shift_factor_dense(eigsol_dense* A, const void* sigma, ShiftFactor** out);
void shift_factor_free(ShiftFactor* f);
int shift_grid(const ShiftFactor* f);
void* shift_aux(const ShiftFactor* f, int j);
int shift_error(ShiftFactor* f);
void shift_lag_reset(ShiftFactor* f);
int shift_iter_launch(ShiftFactor* f, void* buf0, void* buf1, PowerCtl* ctl, const void* rank_part,
                      void* my_part, void* trace, int parity, int first);
int shift_solve_launch(ShiftFactor* f, const void* b_dev, void* y_dev);
void shift_info(const ShiftFactor* f, double* bytes, int32_t* variant, int32_t* tiles);
// extended precision (EIGSOL_DD / EIGSOL_CDD, wide.hip): the same session interface, host-driven
struct WideSession;
int wide_session_create(eigsol_ctx* ctx, eigsol_csr* csr, eigsol_dense* dense, const void* sigma, int32_t trace_cap,
                        WideSession** out);
void wide_session_free(WideSession* s);
int wide_begin(WideSession* s, const eigsol_solver_options* opts, const void* x0, int on_dev);
int wide_step(WideSession* s, int32_t nsteps);
int wide_query(WideSession* s, int32_t* done, int32_t* launches);
int wide_finish(WideSession* s, void* lambda_out, void* x_out, int x_on_dev, int32_t* iterations, int32_t* converged);
int wide_trace(WideSession* s, void* trace_host, int32_t capacity, int32_t* count);
void wide_info(const WideSession* s, double* bytes, int32_t* variant, int32_t* tiles, int32_t* grid);
int wide_solve_shifted(eigsol_csr* csr, eigsol_dense* dense, const void* sigma, const void* b, int64_t nb, void* x);
}  // namespace eigsol

using namespace eigsol;

// Device-side peer exchange of a row-sharded session (EIGSOL_TRANSPORT_PEER): the own inbox, the
// peers' inboxes mapped into this process, and the push plan.
struct PeerState {
    dev::PeerArgs args{};
    void* inbox = nullptr;
    size_t inbox_bytes = 0;
    std::vector<void*> opened;    // IPC-opened peer inboxes (closed at destroy)
    void* peers_dev = nullptr;    // device table of P inbox pointers
    void* push_dev = nullptr;     // int4 push entries
    void* slice_push_dev = nullptr;
    int64_t npush = 0;
    bool agreed = false;          // every rank finished setup: destroy is collective from here on
};

struct eigsol_power {
    eigsol_ctx* ctx = nullptr;
    eigsol_csr* csr = nullptr;
    eigsol_dense* dense = nullptr;
    ShiftFactor* shift = nullptr;   // shifted inverse iteration: factor of A - sigma I
    int dtype = EIGSOL_F64;
    int64_t n = 0;            // rows owned (= vector length on one GPU)
    int64_t nbuf = 0;         // own + ghost entries (x-space)
    int64_t xoff = 0;         // x-space index of own row 0 (row-sharded: lower ghosts first)
    bool dist = false;
    void* buf[2] = {nullptr, nullptr};
    PowerCtl* ctl = nullptr;
    void* rank_part = nullptr;   // part4[nranks]
    void* my_part = nullptr;     // part4 (== rank_part on one GPU)
    void* blk_part = nullptr;    // part4[grid]
    void* trace = nullptr;
    int32_t trace_cap = 0;
    int grid = 8;
    int parity = 0;
    int launches = 0;
    bool begun = false;
    bool trivial = false;     // maxIterations <= 0
    PowerCtl* host_ctl = nullptr;   // pinned mirror for polling
    eigsol_solver_options opts{1000, 1e-10};
    int transport = EIGSOL_TRANSPORT_LOCAL;
    PeerState* peer = nullptr;
    int same_device = 1;      // ranks (of any process) sharing this rank's device
    // Split iteration (row-sharded, all-gather exchange, binned layout): two launches over the
    // first and second halves of the own chunks; the first half's all-gather runs on `comm`
    // while the second half computes.  split_rows[q]: rank q's rows in its first half.
    bool split = false;
    std::vector<int64_t> split_rows;
    hipStream_t comm = nullptr;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    WideSession* wide = nullptr;   // EIGSOL_DD / EIGSOL_CDD: the double-double session (wide.hip)
};

static constexpr size_t kPart = 32;

static int session_alloc(eigsol_power* s, int32_t trace_cap) {
    const size_t sb = scalar_bytes(s->dtype);
    EIGSOL_HIP(hipSetDevice(s->ctx->device));
    for (int i = 0; i < 2; ++i) EIGSOL_HIP(hipMalloc(&s->buf[i], std::max<int64_t>(s->nbuf, 1) * sb + 64));
    EIGSOL_HIP(hipMalloc(&s->ctl, sizeof(PowerCtl)));
    EIGSOL_HIP(hipMalloc(&s->rank_part, kPart * std::max(1, s->ctx->nranks)));
    // rank partials are all-gathered in place: this rank's slot is rank_part[rank]
    s->my_part = static_cast<char*>(s->rank_part) + kPart * (s->dist ? s->ctx->rank : 0);
    EIGSOL_HIP(hipMalloc(&s->blk_part, kPart * std::max(8, s->grid)));
    if (trace_cap > 0) EIGSOL_HIP(hipMalloc(&s->trace, (size_t)trace_cap * sb));
    s->trace_cap = std::max(0, trace_cap);
    EIGSOL_HIP(hipHostMalloc(&s->host_ctl, sizeof(PowerCtl), hipHostMallocDefault));
    std::memset(s->host_ctl, 0, sizeof(PowerCtl));
    EIGSOL_HIP(hipMemsetAsync(s->ctl, 0, sizeof(PowerCtl), s->ctx->stream));
    EIGSOL_HIP(hipMemsetAsync(s->blk_part, 0, kPart * std::max(8, s->grid), s->ctx->stream));
    return EIGSOL_OK;
}

static void peer_free(eigsol_power* s) {
    PeerState* p = s->peer;
    if (!p) return;
    // collective: no rank releases its inbox while a peer may still store into it
    if (p->agreed) (void)coll_barrier(s->ctx);
    for (void* q : p->opened) (void)hipIpcCloseMemHandle(q);
    for (void* q : {p->inbox, p->peers_dev, p->push_dev, p->slice_push_dev})
        if (q) (void)hipFree(q);
    delete p;
    s->peer = nullptr;
}

static void session_free(eigsol_power* s) {
    if (!s) return;
    if (s->wide) {
        wide_session_free(s->wide);
        delete s;
        return;
    }
    hipSetDevice(s->ctx->device);
    hipStreamSynchronize(s->ctx->stream);
    if (s->comm) {
        hipStreamSynchronize(s->comm);
        hipStreamDestroy(s->comm);
    }
    for (hipEvent_t e : s->ev)
        if (e) hipEventDestroy(e);
    peer_free(s);
    hipFree(s->buf[0]);
    hipFree(s->buf[1]);
    hipFree(s->ctl);
    hipFree(s->rank_part);
    hipFree(s->blk_part);
    if (s->trace) hipFree(s->trace);
    if (s->host_ctl) hipHostFree(s->host_ctl);
    if (s->shift) shift_factor_free(s->shift);
    if (s->csr) csr_release(s->csr);
    if (s->dense) dense_release(s->dense);
    delete s;
}

static int launch_iteration(eigsol_power* s) {
    if (s->peer)   // one launch: the epilogue delivers the halo and the partial to the peers
        return csr_power_launch(s->csr, s->nbuf, s->buf[0], s->buf[1], s->ctl, s->rank_part, s->ctx->nranks,
                                s->my_part, s->blk_part, s->trace, s->parity, s->grid, &s->peer->args);
    if (s->shift)
        return shift_iter_launch(s->shift, s->buf[0], s->buf[1], s->ctl, s->rank_part, s->my_part,
                                 s->trace, s->parity, s->launches == 0);
    if (s->csr && s->dist && s->split) {
        // launch t writes y_t into buf[t & 1]: the first half's rows go out while the second half computes
        for (int part = 0; part < 2; ++part) {
            EIGSOL_TRY(csr_power_launch(s->csr, s->nbuf, s->buf[0], s->buf[1], s->ctl, s->rank_part,
                                        s->ctx->nranks, s->my_part, s->blk_part, s->trace, s->parity, s->grid,
                                        nullptr, part));
            EIGSOL_TRY(dist_exchange_part(s->csr, s->buf[s->parity], s->rank_part, part, s->split_rows, s->comm,
                                          s->ev));
        }
        return EIGSOL_OK;
    }
    if (s->csr && s->dist) {
        EIGSOL_TRY(csr_power_launch(s->csr, s->nbuf, s->buf[0], s->buf[1], s->ctl, s->rank_part,
                                    s->ctx->nranks, s->my_part, s->blk_part, s->trace, s->parity, s->grid));
        // launch t wrote y_t into buf[t & 1]: halo exchange + all-gather of the rank partials
        return dist_exchange(s->csr, s->buf[s->parity], s->rank_part);
    }
    if (s->csr)
        return csr_power_launch(s->csr, s->nbuf, s->buf[0], s->buf[1], s->ctl, s->rank_part,
                                s->ctx->nranks, s->my_part, s->blk_part, s->trace, s->parity, s->grid);
    return dense_power_launch(s->dense, s->buf[0], s->buf[1], s->ctl, s->rank_part, s->ctx->nranks,
                              s->my_part, s->blk_part, s->trace, s->parity, s->grid);
}

static int pull_ctl(eigsol_power* s) {
    EIGSOL_HIP(hipMemcpyAsync(s->host_ctl, s->ctl, sizeof(PowerCtl), hipMemcpyDeviceToHost, s->ctx->stream));
    EIGSOL_HIP(hipStreamSynchronize(s->ctx->stream));
    return EIGSOL_OK;
}

// Inbox memory: uncached device memory by default (every access of the handed-off bytes is
// system-scope anyway); EIGSOL_PEER_MEM=finegrained|coarse for experiments.
static hipError_t peer_alloc(void** p, size_t bytes) {
    const char* m = std::getenv("EIGSOL_PEER_MEM");
    if (m && !std::strcmp(m, "coarse")) return hipMalloc(p, bytes);
    if (m && !std::strcmp(m, "finegrained")) return hipExtMallocWithFlags(p, bytes, hipDeviceMallocFinegrained);
    return hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached);
}

// Local part of the peer setup (allocation, address exchange, plan upload).  Returns EIGSOL_OK or
// an error; the caller makes the outcome collective.
static int peer_setup_local(eigsol_power* s) {
    eigsol_csr* A = s->csr;
    eigsol_ctx* ctx = s->ctx;
    const int P = ctx->nranks, me = ctx->rank;
    auto* p = new PeerState();
    s->peer = p;
    const size_t sb = scalar_bytes(s->dtype);
    // one ghost-area stride for every rank: a pusher addresses the peer's parity-1 area with it
    int64_t gmax = 1;
    for (int q = 0; q < P; ++q) {
        int64_t g = 0;
        for (int r = 0; r < P; ++r) g += A->ghost_counts[(size_t)q * P + r];
        gmax = std::max(gmax, g);
    }
    const int64_t stride = ((gmax + 15) / 16) * 16;
    p->inbox_bytes = sizeof(dev::PeerInbox) + 2 * (size_t)stride * sb;
    EIGSOL_HIP(peer_alloc(&p->inbox, p->inbox_bytes));
    EIGSOL_HIP(hipMemset(p->inbox, 0, p->inbox_bytes));
    std::vector<void*> table(P, nullptr);
    if (ctx->loop) {
        // one process: the other ranks' inboxes are plain device pointers
        std::vector<uintptr_t> all(P);
        const uintptr_t mine = reinterpret_cast<uintptr_t>(p->inbox);
        EIGSOL_TRY(coll_allgather(ctx, &mine, sizeof(mine), all.data()));
        for (int q = 0; q < P; ++q) table[q] = reinterpret_cast<void*>(all[q]);
    } else {
        hipIpcMemHandle_t h;
        std::memset(&h, 0, sizeof(h));
        const hipError_t e = hipIpcGetMemHandle(&h, p->inbox);
        // a rank whose export failed still takes part in the all-gather (zero handle)
        std::vector<hipIpcMemHandle_t> all(P);
        EIGSOL_TRY(coll_allgather(ctx, &h, sizeof(h), all.data()));
        if (e != hipSuccess) return fail(EIGSOL_E_HIP, std::string("hipIpcGetMemHandle: ") + hipGetErrorString(e));
        for (int q = 0; q < P; ++q) {
            if (q == me) { table[q] = p->inbox; continue; }
            void* ptr = nullptr;
            EIGSOL_HIP(hipIpcOpenMemHandle(&ptr, all[q], hipIpcMemLazyEnablePeerAccess));
            p->opened.push_back(ptr);
            table[q] = ptr;
        }
    }
    // push plan: {local row, peer, slot} sorted by row, and each slice's range of it
    p->npush = A->nsend;
    std::vector<int32_t> push(4 * std::max<int64_t>(p->npush, 1), 0);
    EIGSOL_TRY(eigsol_peer_plan(P, me, A->row_begins.data(), A->ghost_counts.data(), A->requests.data(),
                                A->nsend, push.data()));
    std::vector<int32_t> sp(2 * std::max<int32_t>(A->nslices, 1), 0);
    int64_t e = 0;
    for (int32_t sl = 0; sl < A->nslices; ++sl) {
        sp[2 * sl] = (int32_t)e;
        while (e < p->npush && push[4 * e] < (sl + 1) * 64) ++e;
        sp[2 * sl + 1] = (int32_t)e;
    }
    EIGSOL_HIP(hipMalloc(&p->peers_dev, sizeof(void*) * P));
    EIGSOL_HIP(hipMalloc(&p->push_dev, push.size() * sizeof(int32_t)));
    EIGSOL_HIP(hipMalloc(&p->slice_push_dev, sp.size() * sizeof(int32_t)));
    EIGSOL_HIP(hipMemcpy(p->peers_dev, table.data(), sizeof(void*) * P, hipMemcpyHostToDevice));
    EIGSOL_HIP(hipMemcpy(p->push_dev, push.data(), push.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    EIGSOL_HIP(hipMemcpy(p->slice_push_dev, sp.data(), sp.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    p->args.peers = static_cast<dev::PeerInbox* const*>(p->peers_dev);
    p->args.inbox = static_cast<dev::PeerInbox*>(p->inbox);
    p->args.push = static_cast<const int4*>(p->push_dev);
    p->args.slice_push = static_cast<const int2*>(p->slice_push_dev);
    p->args.ghost_stride = stride;
    p->args.me = me;
    p->args.P = P;
    if (std::getenv("EIGSOL_PEER_DEBUG")) {
        std::fprintf(stderr, "[peer] rank %d/%d inbox %p table", me, P, p->inbox);
        for (int q = 0; q < P; ++q) std::fprintf(stderr, " %p", table[q]);
        std::fprintf(stderr, " npush %lld nghost %lld stride %lld slices %d\n", (long long)p->npush,
                     (long long)A->nghost, (long long)stride, A->nslices);
    }
    EIGSOL_TRY(csr_grid(A, &s->grid, true));
    if (ctx->loop) {
        // loopback ranks share one device: each rank's blocks must stay co-resident with the
        // others' (a waiting launch must not keep a peer's producing launch off the CUs)
        s->grid = std::max(8, (s->grid / P) / 8 * 8);
    } else if (s->same_device > 1) {
        // ranks of other processes on this device (choose_transport's device-identity gather):
        // the same co-residency rule, split among the ranks that share the CUs
        s->grid = std::max(8, (s->grid / s->same_device) / 8 * 8);
    }
    return EIGSOL_OK;
}

// Frees the per-session device buffers only (a session falling back from the peer transport
// re-allocates them for the collective grid).
static void session_bufs_free(eigsol_power* s) {
    for (void** q : {&s->buf[0], &s->buf[1], reinterpret_cast<void**>(&s->ctl), &s->rank_part, &s->blk_part,
                     &s->trace}) {
        if (*q) (void)hipFree(*q);
        *q = nullptr;
    }
    if (s->host_ctl) (void)hipHostFree(s->host_ctl);
    s->host_ctl = nullptr;
}

// Number of ranks (this one included) whose device has this rank's PCI bus id.  Host-collective
// (every rank calls it).  Loopback worlds share one device by construction and return 1.
static int ranks_on_my_device(eigsol_ctx* ctx, int& out) {
    out = 1;
    if (ctx->loop || ctx->nranks <= 1) return EIGSOL_OK;
    char id[64];
    std::memset(id, 0, sizeof(id));
    if (hipDeviceGetPCIBusId(id, (int)sizeof(id) - 1, ctx->device) != hipSuccess)
        std::snprintf(id, sizeof(id), "unknown-%p", static_cast<void*>(ctx));   // unique: counted alone
    std::vector<char> all((size_t)ctx->nranks * sizeof(id));
    EIGSOL_TRY(coll_allgather(ctx, id, sizeof(id), all.data()));
    int same = 0;
    for (int q = 0; q < ctx->nranks; ++q)
        if (!std::memcmp(all.data() + (size_t)q * sizeof(id), id, sizeof(id))) ++same;
    out = std::max(1, same);
    return EIGSOL_OK;
}

// Collective choice of the per-iteration transport of a row-sharded CSR session.
// The session buffers are allocated inside the agreement (peer path), so that a rank whose
// allocation fails makes every rank fail or fall back together: a peer session's teardown is
// collective, and a rank tearing down alone would leave the others in an unmatched barrier.
static int choose_transport(eigsol_power* s, int32_t trace_cap) {
    eigsol_csr* A = s->csr;
    eigsol_ctx* ctx = s->ctx;
    const int P = ctx->nranks;
    const bool host_only = !ctx->comm && !ctx->loop;
    EIGSOL_TRY(ranks_on_my_device(ctx, s->same_device));
    int cand = (A->sliced && A->exchange == EIGSOL_EXCHANGE_HALO && P <= dev::kMaxPeerRanks) ? 1 : 0;
    if (const char* e = std::getenv("EIGSOL_DIST_TRANSPORT"))
        if (!std::strcmp(e, "collective") && !host_only) cand = 0;
    if (ctx->loop) {
        // Loopback ranks share one device: a waiting launch sits at the head of its stream's
        // hardware queue, so every rank needs a queue of its own, or a rank's launch can queue
        // behind a waiting one (a 10 s peer-wait fault).  HIP maps streams onto GPU_MAX_HW_QUEUES
        // queues (default 4) by use, so other live streams of the process can pair two ranks on
        // one queue whatever the count: the peer transport of a loopback world is opt-in
        // (EIGSOL_DIST_TRANSPORT=peer, for protocol tests and probes), the collective one the default.
        const char* t = std::getenv("EIGSOL_DIST_TRANSPORT");
        const char* q = std::getenv("GPU_MAX_HW_QUEUES");
        if (!(t && !std::strcmp(t, "peer")) || (q ? std::atoi(q) : 4) < P + 1) cand = 0;
    }
    std::vector<int> all(P);
    EIGSOL_TRY(coll_allgather(ctx, &cand, sizeof(int), all.data()));
    bool peer = true;
    for (int v : all) peer = peer && v;
    if (!peer) {
        if (host_only)
            return fail(EIGSOL_E_UNSUPPORTED, "row-sharded session on a host-bootstrapped context needs the "
                                              "peer exchange (halo matrix in the sliced layout on every rank)");
        s->transport = EIGSOL_TRANSPORT_COLLECTIVE;
        return EIGSOL_OK;
    }
    int rc = peer_setup_local(s);
    if (rc == EIGSOL_OK) rc = session_alloc(s, trace_cap);
    int ok = rc == EIGSOL_OK ? 1 : 0;
    const std::string why = ok ? "" : eigsol_last_error();
    EIGSOL_TRY(coll_allgather(ctx, &ok, sizeof(int), all.data()));
    bool all_ok = true;
    for (int v : all) all_ok = all_ok && v;
    if (all_ok) {
        s->peer->agreed = true;
        s->transport = EIGSOL_TRANSPORT_PEER;
        return EIGSOL_OK;
    }
    peer_free(s);   // not agreed: local teardown only
    session_bufs_free(s);
    if (host_only)
        return fail(EIGSOL_E_HIP, "peer exchange setup failed on some rank: " + why);
    s->transport = EIGSOL_TRANSPORT_COLLECTIVE;   // RCCL / loopback copies
    EIGSOL_TRY(csr_grid(A, &s->grid));
    return EIGSOL_OK;
}

// Collective: split every iteration in two row parts when every rank's shard is binned, uses the
// all-gather exchange and has >= 2 chunks (EIGSOL_DIST_SPLIT=0 disables).  The first part's
// all-gather then overlaps the second part's product (RCCL on a stream of its own).
static int choose_split(eigsol_power* s) {
    eigsol_csr* A = s->csr;
    eigsol_ctx* ctx = s->ctx;
    const int P = ctx->nranks;
    int cand = (A->binned && A->nchunks >= 2 && A->exchange == EIGSOL_EXCHANGE_ALLGATHER &&
                (ctx->comm || ctx->loop)) ? 1 : 0;
    if (const char* e = std::getenv("EIGSOL_DIST_SPLIT")) if (!std::atoi(e)) cand = 0;
    std::vector<int> all(P);
    EIGSOL_TRY(coll_allgather(ctx, &cand, sizeof(int), all.data()));
    for (int v : all) if (!v) return EIGSOL_OK;
    const int64_t mine = csr_bin_split_row(A);
    s->split_rows.assign(P, 0);
    EIGSOL_TRY(coll_allgather(ctx, &mine, sizeof(mine), s->split_rows.data()));
    if (!ctx->loop) {
        EIGSOL_HIP(hipStreamCreateWithFlags(&s->comm, hipStreamNonBlocking));
        for (hipEvent_t& e : s->ev) EIGSOL_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    s->split = true;
    return EIGSOL_OK;
}

// a session handle around a double-double session (power method when sigma is null)
static int wide_wrap(eigsol_ctx* ctx, eigsol_csr* csr, eigsol_dense* dense, const void* sigma, int32_t trace_cap,
                     eigsol_power** out) {
    EIGSOL_HIP(hipSetDevice(ctx->device));
    WideSession* w = nullptr;
    EIGSOL_TRY(wide_session_create(ctx, csr, dense, sigma, trace_cap, &w));
    auto* s = new eigsol_power();
    s->ctx = ctx;
    s->dtype = csr ? csr->dtype : dense->dtype;
    s->n = csr ? csr->nrows : dense->nrows;
    s->nbuf = s->n;
    s->wide = w;
    *out = s;
    return EIGSOL_OK;
}

extern "C" {

int eigsol_power_create_csr(eigsol_csr* A, int32_t trace_capacity, eigsol_power** out) {
    if (!A || !out) return fail(EIGSOL_E_INVALID, "eigsol_power_create_csr: null pointer");
    *out = nullptr;
    if (!A->dist && A->nrows != A->ncols) return fail(EIGSOL_E_NOT_SQUARE, "powerMethod: matrix must be square");
    if (A->dist ? A->n_global == 0 : A->nrows == 0) return fail(EIGSOL_E_ZERO_SIZE, "powerMethod: matrix has zero size");
    if (dtype_wide(A->dtype)) return wide_wrap(A->ctx, A, nullptr, nullptr, trace_capacity, out);
    auto* s = new eigsol_power();
    s->ctx = A->ctx;
    s->csr = A;
    s->dist = A->dist != 0;
    s->xoff = A->xoff;
    csr_retain(A);
    s->dtype = A->dtype;
    s->n = A->nrows;
    s->nbuf = A->ncols;
    int rc = csr_grid(A, &s->grid);
    if (rc == EIGSOL_OK && s->dist) rc = choose_transport(s, trace_capacity);
    if (rc == EIGSOL_OK && s->dist && s->transport == EIGSOL_TRANSPORT_COLLECTIVE) rc = choose_split(s);
    if (rc == EIGSOL_OK && !s->buf[0]) rc = session_alloc(s, trace_capacity);
    if (rc != EIGSOL_OK) { session_free(s); return rc; }
    *out = s;
    return EIGSOL_OK;
}

int eigsol_power_create_dense(eigsol_dense* A, int32_t trace_capacity, eigsol_power** out) {
    if (!A || !out) return fail(EIGSOL_E_INVALID, "eigsol_power_create_dense: null pointer");
    *out = nullptr;
    if (A->nrows != A->ncols) return fail(EIGSOL_E_NOT_SQUARE, "powerMethod: matrix must be square");
    if (A->nrows == 0) return fail(EIGSOL_E_ZERO_SIZE, "powerMethod: matrix has zero size");
    if (dtype_wide(A->dtype)) return wide_wrap(A->ctx, nullptr, A, nullptr, trace_capacity, out);
    auto* s = new eigsol_power();
    s->ctx = A->ctx;
    s->dense = A;
    dense_retain(A);
    s->dtype = A->dtype;
    s->n = A->nrows;
    s->nbuf = A->ncols;
    int rc = dense_grid(A, &s->grid);
    if (rc == EIGSOL_OK) rc = session_alloc(s, trace_capacity);
    if (rc != EIGSOL_OK) { session_free(s); return rc; }
    *out = s;
    return EIGSOL_OK;
}

int eigsol_power_destroy(eigsol_power* s) {
    session_free(s);
    return EIGSOL_OK;
}

int eigsol_power_begin(eigsol_power* s, const eigsol_solver_options* opts, const void* x0,
                       int x0_on_device) {
    if (!s || !opts || !x0) return fail(EIGSOL_E_INVALID, "eigsol_power_begin: null pointer");
    if (s->wide) return wide_begin(s->wide, opts, x0, x0_on_device);
    EIGSOL_HIP(hipSetDevice(s->ctx->device));
    hipStream_t st = s->ctx->stream;
    const size_t sb = scalar_bytes(s->dtype);
    if (s->shift) shift_lag_reset(s->shift);
    s->opts = *opts;
    s->trivial = opts->max_iterations <= 0;
    // y_{-1} = x0 lives in buf[1] (launch t reads buf[(t-1)&1]); own rows at x-space offset xoff
    char* x0dst = static_cast<char*>(s->buf[1]) + (size_t)s->xoff * sb;
    EIGSOL_HIP(hipMemcpyAsync(x0dst, x0, s->n * sb,
                              x0_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
    PowerCtl init;
    std::memset(&init, 0, sizeof(init));
    init.max_iter = opts->max_iterations;
    init.tol = opts->tolerance;
    init.trace_cap = s->trace_cap;
    init.nranks = s->ctx->nranks;
    init.st[0].t = -1;
    init.st[1].t = -1;
    std::memcpy(s->host_ctl, &init, sizeof(init));
    EIGSOL_HIP(hipMemcpyAsync(s->ctl, s->host_ctl, sizeof(PowerCtl), hipMemcpyHostToDevice, st));
    if (s->peer) {
        // fresh epochs: every rank's previous launches (and their stores into this inbox) are over
        // before the inbox is cleared, and every inbox is clear before anyone publishes again
        EIGSOL_HIP(hipStreamSynchronize(st));
        EIGSOL_TRY(coll_barrier(s->ctx));
        EIGSOL_HIP(hipMemsetAsync(s->peer->inbox, 0, s->peer->inbox_bytes, st));
        EIGSOL_HIP(hipStreamSynchronize(st));
        EIGSOL_TRY(coll_barrier(s->ctx));
    }
    // ||x0||^2 partials -> the input norm of launch 0 (x.normalize(), power_method.hpp:62)
    EIGSOL_TRY(norm_partial_launch(s->ctx, s->dtype, x0dst, s->n, s->ctl, s->blk_part, s->my_part, s->grid));
    if (s->peer)   // x0 halo + partial into every inbox (parity 1), epoch 1
        EIGSOL_TRY(peer_begin_launch(s->ctx, s->dtype, s->peer->args, x0dst, s->peer->npush, s->my_part));
    else if (s->dist)
        EIGSOL_TRY(dist_exchange(s->csr, s->buf[1], s->rank_part));   // x0 ghosts + partials
    EIGSOL_HIP(hipStreamSynchronize(st));   // host_ctl is reused by query()
    s->parity = 0;
    s->launches = 0;
    s->begun = true;
    return EIGSOL_OK;
}

int eigsol_power_step(eigsol_power* s, int32_t nsteps) {
    if (s && s->wide) return wide_step(s->wide, nsteps);
    if (!s || !s->begun) return fail(EIGSOL_E_INVALID, "eigsol_power_step: session not begun");
    if (s->trivial) return EIGSOL_OK;
    EIGSOL_HIP(hipSetDevice(s->ctx->device));
    for (int32_t i = 0; i < nsteps; ++i) {
        EIGSOL_TRY(launch_iteration(s));
        s->parity ^= 1;
        ++s->launches;
    }
    return EIGSOL_OK;
}

int eigsol_power_query(eigsol_power* s, int32_t* done, int32_t* launches) {
    if (s && s->wide) return wide_query(s->wide, done, launches);
    if (!s || !s->begun) return fail(EIGSOL_E_INVALID, "eigsol_power_query: session not begun");
    if (s->trivial) {
        if (done) *done = 1;
        if (launches) *launches = 0;
        return EIGSOL_OK;
    }
    EIGSOL_HIP(hipSetDevice(s->ctx->device));
    EIGSOL_TRY(pull_ctl(s));
    if (s->shift) EIGSOL_TRY(shift_error(s->shift));
    if (s->host_ctl->fault) {
        std::string flags;
        if (s->peer) {
            dev::PeerInbox box;
            if (hipMemcpy(&box, s->peer->inbox, sizeof(box), hipMemcpyDeviceToHost) == hipSuccess)
                for (int q = 0; q < s->ctx->nranks; ++q) flags += (q ? "," : "") + std::to_string(box.flag[q]);
        }
        return fail(EIGSOL_E_RCCL, "row-sharded peer exchange: inbox flags [" + flags + "]; rank " +
                                       std::to_string(s->ctx->rank) +
                                       " waited 10 s for peer " + std::to_string((s->host_ctl->fault & 0xff) - 1) +
                                       " at launch " + std::to_string(s->host_ctl->fault >> 8) +
                                       " (ranks stepping unevenly, or a peer failed)");
    }
    if (done) *done = s->host_ctl->done;
    if (launches) *launches = s->host_ctl->launches;
    return EIGSOL_OK;
}

int eigsol_power_finish(eigsol_power* s, void* lambda_out, void* x_out, int x_out_on_device,
                        int32_t* iterations, int32_t* converged) {
    if (s && s->wide) return wide_finish(s->wide, lambda_out, x_out, x_out_on_device, iterations, converged);
    if (!s || !s->begun) return fail(EIGSOL_E_INVALID, "eigsol_power_finish: session not begun");
    EIGSOL_HIP(hipSetDevice(s->ctx->device));
    hipStream_t st = s->ctx->stream;
    const size_t sb = scalar_bytes(s->dtype);
    double lam[2] = {0.0, 0.0};
    int parity = 1;
    double fnorm = 0.0;
    int32_t it = 0, conv = 0;
    if (s->trivial) {
        // maxIterations <= 0: lambda = 0, x = normalised x0, 0 iterations (power_method.hpp:61-68)
        const int P = s->dist ? s->ctx->nranks : 1;
        std::vector<double> part(4 * P);
        if (s->peer) {
            // the peers' x0 partials arrive in the inbox (parity 1) with epoch 1
            dev::PeerInbox box;
            const auto t0 = std::chrono::steady_clock::now();
            for (;;) {
                EIGSOL_HIP(hipMemcpy(&box, s->peer->inbox, sizeof(box), hipMemcpyDeviceToHost));
                bool all = true;
                for (int q = 0; q < P; ++q) all = all && (q == s->ctx->rank || box.flag[q] >= 1);
                if (all) break;
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10))
                    return fail(EIGSOL_E_RCCL, "row-sharded peer exchange: start-vector partials did not arrive");
                std::this_thread::sleep_for(std::chrono::microseconds(50));
            }
            for (int q = 0; q < P; ++q) {
                part[4 * q] = box.part[1][q].a;
                part[4 * q + 1] = box.part[1][q].b;
                part[4 * q + 2] = box.part[1][q].c;
            }
        } else {
            EIGSOL_HIP(hipMemcpyAsync(part.data(), s->rank_part, sizeof(double) * 4 * P, hipMemcpyDeviceToHost, st));
            EIGSOL_HIP(hipStreamSynchronize(st));
        }
        double n2 = 0.0;
        for (int r = 0; r < P; ++r) n2 += part[4 * r];   // rank order, as on the device
        fnorm = std::sqrt(n2);
        parity = 1;
    } else {
        EIGSOL_TRY(pull_ctl(s));
        if (!s->host_ctl->done)
            return fail(EIGSOL_E_INVALID, "eigsol_power_finish: iteration has not terminated");
        lam[0] = s->host_ctl->lam_re;
        lam[1] = s->host_ctl->lam_im;
        parity = s->host_ctl->final_parity;
        fnorm = s->host_ctl->final_norm;
        it = s->host_ctl->iters;
        conv = s->host_ctl->converged;
    }
    if (lambda_out) store_scalar(lambda_out, s->dtype, lam[0], lam[1]);
    if (iterations) *iterations = it;
    if (converged) *converged = conv;
    if (x_out) {
        // final_parity 2 + j: solve j of a multi-solve launch (the triangular factor's buffer aux[j])
        void* src = parity >= 2 ? shift_aux(s->shift, parity - 2)
                                : static_cast<char*>(s->buf[parity]) + (size_t)s->xoff * sb;
        if (parity >= 2) parity = 1;   // scratch below: buf[0]
        if (x_out_on_device) {
            EIGSOL_TRY(scale_out_launch(s->ctx, s->dtype, src, fnorm, x_out, s->n));
            EIGSOL_HIP(hipStreamSynchronize(st));
        } else {
            void* tmp = s->buf[parity ^ 1];
            EIGSOL_TRY(scale_out_launch(s->ctx, s->dtype, src, fnorm, tmp, s->n));
            EIGSOL_HIP(hipMemcpyAsync(x_out, tmp, s->n * sb, hipMemcpyDeviceToHost, st));
            EIGSOL_HIP(hipStreamSynchronize(st));
        }
    }
    return EIGSOL_OK;
}

int eigsol_power_trace(eigsol_power* s, void* trace_host, int32_t capacity, int32_t* count) {
    if (s && s->wide) return wide_trace(s->wide, trace_host, capacity, count);
    if (!s || !s->begun) return fail(EIGSOL_E_INVALID, "eigsol_power_trace: session not begun");
    int32_t n = 0;
    if (!s->trivial && s->trace) {
        EIGSOL_TRY(pull_ctl(s));
        n = s->host_ctl->ntrace;
        n = std::min(n, s->trace_cap);
        if (trace_host && capacity > 0) {
            const int32_t m = std::min(n, capacity);
            EIGSOL_HIP(hipMemcpy(trace_host, s->trace, (size_t)m * scalar_bytes(s->dtype), hipMemcpyDeviceToHost));
        }
    }
    if (count) *count = n;
    return EIGSOL_OK;
}

int eigsol_power_transport(const eigsol_power* s, int* transport) {
    if (!s || !transport) return fail(EIGSOL_E_INVALID, "eigsol_power_transport: null pointer");
    *transport = s->transport;
    return EIGSOL_OK;
}

int eigsol_power_kernel_info(eigsol_power* s, double* bytes, int32_t* grid, int32_t* tiles,
                             int32_t* variant) {
    if (!s) return fail(EIGSOL_E_INVALID, "eigsol_power_kernel_info: null session");
    if (s->wide) {
        wide_info(s->wide, bytes, variant, tiles, grid);
        return EIGSOL_OK;
    }
    const double sb = (double)scalar_bytes(s->dtype);
    if (s->shift) {
        shift_info(s->shift, bytes, variant, tiles);
    } else if (s->csr) {
        // values + int32 columns + int32 row pointers + x read once + y written once
        const double nnz = (double)s->csr->nnz, n = (double)s->csr->nrows;
        if (bytes) *bytes = (sb + 4.0) * nnz + 4.0 * (n + 1.0) + 2.0 * sb * n;
        if (tiles) *tiles = s->csr->sliced ? s->csr->nslices : s->csr->ntiles;
        if (variant) *variant = s->csr->sliced ? 5 : dtype_single(s->dtype) ? 6 : (s->csr->windowed ? 1 : 0);
        if (!s->csr->cblk.empty() && !s->peer) {   // column-blocked passes (tiles = blocks)
            if (variant) *variant = 9;
            if (tiles) *tiles = (int32_t)s->csr->cblk.size();
        }
        if (s->csr->binned && !s->peer) {   // column-binned chunks (tiles = chunks)
            if (variant) *variant = s->split ? 11 : 10;
            if (tiles) *tiles = s->csr->nchunks;
        }
    } else {
        const double n = (double)s->dense->nrows;
        if (bytes) *bytes = sb * n * n + 2.0 * sb * n;
        if (tiles) *tiles = 0;
        if (variant) *variant = 2;
    }
    if (grid) *grid = s->grid;
    return EIGSOL_OK;
}

// Demangled name of the fused power-iteration kernel a CSR session launches (the string rocprofv3
// prints for it), so roofline figures can be matched to the exact template instantiation.
int eigsol_power_kernel_name(eigsol_power* s, char* buf, size_t cap) {
    if (!s || !buf || cap == 0) return fail(EIGSOL_E_INVALID, "eigsol_power_kernel_name: null argument");
    buf[0] = 0;
    if (s->wide || s->shift || !s->csr) return EIGSOL_OK;   // named for CSR power sessions only
    const void* k = csr_power_kernel(s->csr, s->transport == EIGSOL_TRANSPORT_PEER);
    const char* m = k ? hipKernelNameRefByPtr(k, s->ctx->stream) : nullptr;
    if (!m) return EIGSOL_OK;
    int st = 0;
    char* d = abi::__cxa_demangle(m, nullptr, nullptr, &st);
    std::snprintf(buf, cap, "%s", (st == 0 && d) ? d : m);
    std::free(d);
    return EIGSOL_OK;
}

// One-shot solves: begin / step in doubling chunks until the device reports termination / finish.
static int run_to_completion(eigsol_power* s, const eigsol_solver_options* opts, const void* x0,
                             void* lambda_out, void* x_out, int32_t* iterations, int32_t* converged) {
    EIGSOL_TRY(eigsol_power_begin(s, opts, x0, 0));
    if (!s->trivial) {
        // Upper bound on launches: maxIterations + 2 (launch maxIter+1 only decides).
        const int64_t cap = (int64_t)opts->max_iterations + 2;
        int64_t issued = 0;
        int32_t chunk = 4;
        int32_t done = 0;
        while (!done) {
            const int32_t k = (int32_t)std::min<int64_t>(chunk, std::max<int64_t>(1, cap - issued));
            EIGSOL_TRY(eigsol_power_step(s, k));
            issued += k;
            EIGSOL_TRY(eigsol_power_query(s, &done, nullptr));
            chunk = std::min(chunk * 2, 64);
            if (!done && issued >= cap + 4)
                return fail(EIGSOL_E_SOLVER, "power iteration did not terminate (internal error)");
        }
    }
    return eigsol_power_finish(s, lambda_out, x_out, 0, iterations, converged);
}

int eigsol_power_csr(eigsol_csr* A, const eigsol_solver_options* opts, const void* x0,
                     void* lambda_out, void* x_out, int32_t* iterations, int32_t* converged) {
    if (!opts || !x0) return fail(EIGSOL_E_INVALID, "eigsol_power_csr: null opts/x0");
    eigsol_power* s = nullptr;
    EIGSOL_TRY(eigsol_power_create_csr(A, 0, &s));
    const int rc = run_to_completion(s, opts, x0, lambda_out, x_out, iterations, converged);
    session_free(s);
    return rc;
}

int eigsol_power_dense(eigsol_dense* A, const eigsol_solver_options* opts, const void* x0,
                       void* lambda_out, void* x_out, int32_t* iterations, int32_t* converged) {
    if (!opts || !x0) return fail(EIGSOL_E_INVALID, "eigsol_power_dense: null opts/x0");
    eigsol_power* s = nullptr;
    EIGSOL_TRY(eigsol_power_create_dense(A, 0, &s));
    const int rc = run_to_completion(s, opts, x0, lambda_out, x_out, iterations, converged);
    session_free(s);
    return rc;
}


// ---------------------------------------------------------------- shifted inverse iteration
// shiftedInversePowerMethod<S> (shifted_inverse_power_solver.hpp:112-125): the session factors
// A - sigma I once at creation and runs one fused solve launch per iteration.
static int shifted_create(eigsol_ctx* ctx, eigsol_csr* csr, eigsol_dense* dense, int dtype,
                          int64_t n, const void* sigma, int32_t trace_capacity, eigsol_power** out) {
    if (dtype_wide(dtype)) return wide_wrap(ctx, csr, dense, sigma, trace_capacity, out);
    auto* s = new eigsol_power();
    s->ctx = ctx;
    s->dtype = dtype;
    s->n = n;
    s->nbuf = n;
    int rc = csr ? shift_factor_csr(csr, sigma, &s->shift) : shift_factor_dense(dense, sigma, &s->shift);
    if (rc == EIGSOL_OK) {
        if (csr) { s->csr = csr; csr_retain(csr); }
        else { s->dense = dense; dense_retain(dense); }
        s->grid = std::max(64, shift_grid(s->shift));
        rc = session_alloc(s, trace_capacity);
    }
    if (rc != EIGSOL_OK) { session_free(s); return rc; }
    *out = s;
    return EIGSOL_OK;
}

int eigsol_shifted_create_csr(eigsol_csr* A, const void* sigma, int32_t trace_capacity, eigsol_power** out) {
    if (!A || !sigma || !out) return fail(EIGSOL_E_INVALID, "eigsol_shifted_create_csr: null pointer");
    *out = nullptr;
    if (A->dist || A->nrows != A->ncols)
        return fail(EIGSOL_E_NOT_SQUARE, "shiftedInversePowerMethod: matrix must be square");
    if (A->nrows == 0) return fail(EIGSOL_E_ZERO_SIZE, "shiftedInversePowerMethod: matrix has zero size");
    return shifted_create(A->ctx, A, nullptr, A->dtype, A->nrows, sigma, trace_capacity, out);
}

int eigsol_shifted_create_dense(eigsol_dense* A, const void* sigma, int32_t trace_capacity, eigsol_power** out) {
    if (!A || !sigma || !out) return fail(EIGSOL_E_INVALID, "eigsol_shifted_create_dense: null pointer");
    *out = nullptr;
    if (A->nrows != A->ncols) return fail(EIGSOL_E_NOT_SQUARE, "shiftedInversePowerMethod: matrix must be square");
    if (A->nrows == 0) return fail(EIGSOL_E_ZERO_SIZE, "shiftedInversePowerMethod: matrix has zero size");
    return shifted_create(A->ctx, nullptr, A, A->dtype, A->nrows, sigma, trace_capacity, out);
}

int eigsol_shifted_inverse_csr(eigsol_csr* A, const void* sigma, const eigsol_solver_options* opts,
                               const void* x0, void* lambda_out, void* x_out, int32_t* iterations,
                               int32_t* converged) {
    if (!opts || !x0) return fail(EIGSOL_E_INVALID, "eigsol_shifted_inverse_csr: null opts/x0");
    eigsol_power* s = nullptr;
    EIGSOL_TRY(eigsol_shifted_create_csr(A, sigma, 0, &s));
    const int rc = run_to_completion(s, opts, x0, lambda_out, x_out, iterations, converged);
    session_free(s);
    return rc;
}

int eigsol_shifted_inverse_dense(eigsol_dense* A, const void* sigma, const eigsol_solver_options* opts,
                                 const void* x0, void* lambda_out, void* x_out, int32_t* iterations,
                                 int32_t* converged) {
    if (!opts || !x0) return fail(EIGSOL_E_INVALID, "eigsol_shifted_inverse_dense: null opts/x0");
    eigsol_power* s = nullptr;
    EIGSOL_TRY(eigsol_shifted_create_dense(A, sigma, 0, &s));
    const int rc = run_to_completion(s, opts, x0, lambda_out, x_out, iterations, converged);
    session_free(s);
    return rc;
}

// solve_shifted<S> (solve_shifted.hpp:48-118): x = (A - sigma I)^{-1} b, host buffers.
static int solve_once(ShiftFactor* f, eigsol_ctx* ctx, size_t sb, int64_t n, const void* b, void* x) {
    void* d = nullptr;
    EIGSOL_HIP(hipMalloc(&d, 2 * n * sb));
    char* bd = static_cast<char*>(d);
    char* yd = bd + n * sb;
    int rc = EIGSOL_OK;
    if (hipMemcpyAsync(bd, b, n * sb, hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "solve_shifted: upload");
    if (rc == EIGSOL_OK) rc = shift_solve_launch(f, bd, yd);
    if (rc == EIGSOL_OK && hipMemcpyAsync(x, yd, n * sb, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "solve_shifted: download");
    if (rc == EIGSOL_OK && hipStreamSynchronize(ctx->stream) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "solve_shifted: synchronize");
    if (rc == EIGSOL_OK) rc = shift_error(f);
    hipFree(d);
    return rc;
}

int eigsol_solve_shifted_csr(eigsol_csr* A, const void* sigma, const void* b, int64_t nb, void* x) {
    if (!A || !sigma || !b || !x) return fail(EIGSOL_E_INVALID, "eigsol_solve_shifted_csr: null pointer");
    if (A->dist || A->nrows != A->ncols)
        return fail(EIGSOL_E_NOT_SQUARE, "solve_shifted: A must be square (sparse case)");
    if (A->nrows != nb)
        return fail(EIGSOL_E_SIZE_MISMATCH, "solve_shifted: size mismatch between A and b (sparse case)");
    if (nb == 0) return EIGSOL_OK;
    EIGSOL_HIP(hipSetDevice(A->ctx->device));
    if (dtype_wide(A->dtype)) return wide_solve_shifted(A, nullptr, sigma, b, nb, x);
    ShiftFactor* f = nullptr;
    EIGSOL_TRY(shift_factor_csr(A, sigma, &f));
    const int rc = solve_once(f, A->ctx, scalar_bytes(A->dtype), nb, b, x);
    shift_factor_free(f);
    return rc;
}

int eigsol_solve_shifted_dense(eigsol_dense* A, const void* sigma, const void* b, int64_t nb, void* x) {
    if (!A || !sigma || !b || !x) return fail(EIGSOL_E_INVALID, "eigsol_solve_shifted_dense: null pointer");
    if (A->nrows != A->ncols) return fail(EIGSOL_E_NOT_SQUARE, "solve_shifted: A must be square (dense case)");
    if (A->nrows != nb)
        return fail(EIGSOL_E_SIZE_MISMATCH, "solve_shifted: size mismatch between A and b (dense case)");
    if (nb == 0) return EIGSOL_OK;
    EIGSOL_HIP(hipSetDevice(A->ctx->device));
    if (dtype_wide(A->dtype)) return wide_solve_shifted(nullptr, A, sigma, b, nb, x);
    ShiftFactor* f = nullptr;
    EIGSOL_TRY(shift_factor_dense(A, sigma, &f));
    const int rc = solve_once(f, A->ctx, scalar_bytes(A->dtype), nb, b, x);
    shift_factor_free(f);
    return rc;
}

}  // extern "C"

// Row-sharded (multi-GPU) power iteration: one process per GPU, RCCL over xGMI.
//
// The reference is single-threaded (no distribution anywhere); this file adds the
// scale-out of powerMethodImpl's loop (src/power_method/power_method.hpp:68-96) that north_star
// asks for.  Rank p owns a contiguous block of rows.  Its CSR keeps global column indices on the
// host; at setup they are remapped to local columns [own rows | ghosts], where ghosts are the
// remote x entries the rank reads, grouped by owner rank in ascending global order.  Per
// iteration, after the fused SpMV launch:
//   pack      send_buf[k] = y[send_idx[k]]          (the rows each peer reads from us)
//   group {   ncclSend/ncclRecv per peer with traffic -> the ghost segment of the next input
//             ncclAllGather of this rank's partial sums (||y||^2, x^H y) }
// and the next launch sums the P rank partials in rank order, so every rank takes bitwise
// identical termination decisions without any host round trip.  For banded/locality-ordered
// matrices a rank only talks to its neighbours (halo of the band width); for unstructured ones
// the same code degenerates into an all-to-all of the needed entries.
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "internal.hpp"

namespace eigsol {

int csr_upload(eigsol_ctx* ctx, int dtype, int64_t nrows, int64_t ncols, int64_t nnz,
               const int32_t* rowptr, const int32_t* colidx, const void* values, eigsol_csr** out,
               int64_t xoff);

#define EIGSOL_RCCL(expr)                                                                       \
    do {                                                                                        \
        ncclResult_t _r = (expr);                                                               \
        if (_r != ncclSuccess)                                                                  \
            return ::eigsol::fail(EIGSOL_E_RCCL, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
    } while (0)

// ------------------------------------------------------------------------- loopback world
// Test transport: P ranks of one process, one host thread each, all on the same device.  Every
// communication step is a list of sends and receives; a step posts this rank's sends, records an
// event after everything the sends read, meets the other ranks at a host barrier, copies each
// receive from the matching send (k-th receive from q = k-th send from q to this rank, NCCL's
// per-pair order) on its own stream after the sender's event, records a second event, meets them
// again and waits for every peer's copies before the stream moves on (so no rank overwrites a
// buffer a peer still reads).  RCCL's collectives are expressed as sends and receives: an in-place
// all-gather is a send of the own block to, and a receive of every other block from, each peer.
// It exercises every device-side piece of the row-sharded path except RCCL itself.
struct LoopSend {
    int peer;
    const void* p;
    size_t bytes;
};
struct LoopRecv {
    int peer;
    void* p;
    size_t bytes;
};
struct LoopWorld {
    int P = 0;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    long gen = 0;
    int joined = 0;
    std::vector<std::vector<LoopSend>> sends;
    std::vector<hipEvent_t> ready, done;
    std::vector<std::vector<char>> hbuf;   // host all-gather slots
};
static std::mutex g_loop_m;
static std::map<std::string, std::shared_ptr<LoopWorld>> g_loop_worlds;
static const char kLoopMagic[] = "EIGSOL-LOOPBACK:";

static void loop_barrier(LoopWorld* w) {
    std::unique_lock<std::mutex> lk(w->m);
    const long g = w->gen;
    if (++w->arrived == w->P) {
        w->arrived = 0;
        ++w->gen;
        w->cv.notify_all();
    } else {
        w->cv.wait(lk, [&] { return w->gen != g; });
    }
}

static int loop_step(eigsol_ctx* ctx, const std::vector<LoopSend>& sends, const std::vector<LoopRecv>& recvs) {
    auto* w = static_cast<LoopWorld*>(ctx->loop);
    const int me = ctx->rank;
    hipStream_t st = ctx->stream;
    {
        std::lock_guard<std::mutex> lk(w->m);
        w->sends[me] = sends;
    }
    EIGSOL_HIP(hipEventRecord(w->ready[me], st));
    loop_barrier(w);
    std::vector<int> seen(w->P, 0);
    int rc = EIGSOL_OK;
    for (const LoopRecv& r : recvs) {
        int k = seen[r.peer]++, idx = -1;
        const std::vector<LoopSend>& ps = w->sends[r.peer];
        for (size_t j = 0; j < ps.size(); ++j)
            if (ps[j].peer == me && k-- == 0) { idx = (int)j; break; }
        if (idx < 0 || ps[idx].bytes != r.bytes) {
            rc = fail(EIGSOL_E_RCCL, "loopback: unmatched receive (internal error)");
            break;
        }
        if (hipStreamWaitEvent(st, w->ready[r.peer], 0) != hipSuccess ||
            (r.bytes && hipMemcpyAsync(r.p, ps[idx].p, r.bytes, hipMemcpyDeviceToDevice, st) != hipSuccess)) {
            rc = fail(EIGSOL_E_HIP, "loopback: copy");
            break;
        }
    }
    if (hipEventRecord(w->done[me], st) != hipSuccess && rc == EIGSOL_OK) rc = fail(EIGSOL_E_HIP, "loopback: event");
    loop_barrier(w);   // every rank reaches it, also after an error, so nobody waits forever
    for (int q = 0; q < w->P; ++q)
        if (q != me && hipStreamWaitEvent(st, w->done[q], 0) != hipSuccess && rc == EIGSOL_OK)
            rc = fail(EIGSOL_E_HIP, "loopback: event wait");
    return rc;
}

// in-place all-gather of `count` bytes per rank as loopback sends/receives
static void loop_allgather(eigsol_ctx* ctx, void* buf, size_t bytes, std::vector<LoopSend>& s,
                           std::vector<LoopRecv>& r) {
    char* b = static_cast<char*>(buf);
    for (int q = 0; q < ctx->nranks; ++q) {
        if (q == ctx->rank) continue;
        s.push_back({q, b + (size_t)ctx->rank * bytes, bytes});
        r.push_back({q, b + (size_t)q * bytes, bytes});
    }
}

// ------------------------------------------------------------------------- host collectives
// Setup-time all-gather of host bytes over whatever the context was bootstrapped with: the
// caller's callback (eigsol_ctx_create_dist_host), the loopback world, or RCCL (staged through a
// device buffer).  Never used per iteration.
int coll_allgather(eigsol_ctx* ctx, const void* mine, size_t bytes, void* all) {
    const int P = ctx->nranks, me = ctx->rank;
    char* out = static_cast<char*>(all);
    if (P == 1 || bytes == 0) {
        if (bytes) std::memcpy(out, mine, bytes);
        return EIGSOL_OK;
    }
    if (ctx->hcoll) {
        if (ctx->hcoll(mine, all, bytes, ctx->hcoll_user) != 0)
            return fail(EIGSOL_E_RCCL, "host all-gather callback failed");
        return EIGSOL_OK;
    }
    if (ctx->loop) {
        auto* w = static_cast<LoopWorld*>(ctx->loop);
        {
            std::lock_guard<std::mutex> lk(w->m);
            w->hbuf[me].assign(static_cast<const char*>(mine), static_cast<const char*>(mine) + bytes);
        }
        loop_barrier(w);
        int rc = EIGSOL_OK;
        for (int q = 0; q < P; ++q) {
            if (w->hbuf[q].size() != bytes) rc = fail(EIGSOL_E_RCCL, "loopback all-gather: size mismatch");
            else std::memcpy(out + (size_t)q * bytes, w->hbuf[q].data(), bytes);
        }
        loop_barrier(w);   // nobody overwrites a slot another rank still reads
        return rc;
    }
    if (!ctx->comm) return fail(EIGSOL_E_INVALID, "coll_allgather: context has no communicator");
    char* d = nullptr;
    EIGSOL_HIP(hipMalloc(&d, bytes * P));
    hipStream_t st = ctx->stream;
    int rc = EIGSOL_OK;
    if (hipMemcpyAsync(d + bytes * me, mine, bytes, hipMemcpyHostToDevice, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "coll_allgather: upload");
    ncclResult_t r = rc == EIGSOL_OK ? ncclAllGather(d + bytes * me, d, bytes, ncclChar,
                                                    static_cast<ncclComm_t>(ctx->comm), st)
                                     : ncclSuccess;
    if (r != ncclSuccess) rc = fail(EIGSOL_E_RCCL, std::string("coll_allgather: ") + ncclGetErrorString(r));
    if (rc == EIGSOL_OK && (hipMemcpyAsync(all, d, bytes * P, hipMemcpyDeviceToHost, st) != hipSuccess ||
                            hipStreamSynchronize(st) != hipSuccess))
        rc = fail(EIGSOL_E_HIP, "coll_allgather: download");
    hipFree(d);
    return rc;
}

int coll_barrier(eigsol_ctx* ctx) {
    const char one = 1;
    std::vector<char> all(ctx->nranks);
    return coll_allgather(ctx, &one, 1, all.data());
}

void dist_release_comm(eigsol_ctx* ctx) {
    if (ctx && ctx->comm) {
        ncclCommDestroy(static_cast<ncclComm_t>(ctx->comm));
        ctx->comm = nullptr;
    }
    if (ctx && ctx->loop) {
        auto* w = static_cast<LoopWorld*>(ctx->loop);
        std::lock_guard<std::mutex> g(g_loop_m);
        for (auto it = g_loop_worlds.begin(); it != g_loop_worlds.end(); ++it)
            if (it->second.get() == w && --w->joined == 0) {
                for (hipEvent_t e : w->ready) hipEventDestroy(e);
                for (hipEvent_t e : w->done) hipEventDestroy(e);
                g_loop_worlds.erase(it);
                break;
            }
        ctx->loop = nullptr;
    }
}

template <class S>
__global__ __launch_bounds__(256) void pack_kernel(const S* __restrict__ y, const int32_t* __restrict__ idx,
                                                   S* __restrict__ out, int64_t n) {
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256)
        out[k] = y[idx[k]];
}

// Halo exchange of the vector `y` (local layout [own | ghosts]) + all-gather of the rank partials
// (part4 = 4 doubles per rank, in place at rank_part[rank]).  Stream-ordered on ctx->stream.
int dist_exchange(eigsol_csr* A, void* y, void* rank_part) {
    eigsol_ctx* ctx = A->ctx;
    const size_t sb = scalar_bytes(A->dtype);
    hipStream_t st = ctx->stream;
    if (A->nsend > 0) {
        const int grid = (int)std::min<int64_t>(1024, (A->nsend + 255) / 256);
        // the pack moves whole scalars: 16-byte complex<double> as cplx, 8-byte scalars
        // (double, complex<float>) as double, float as float
        if (sb == 16)
            hipLaunchKernelGGL(pack_kernel<cplx>, dim3(grid), dim3(256), 0, st, (const cplx*)y,
                               A->send_idx, (cplx*)A->send_buf, A->nsend);
        else if (sb == 8)
            hipLaunchKernelGGL(pack_kernel<double>, dim3(grid), dim3(256), 0, st, (const double*)y,
                               A->send_idx, (double*)A->send_buf, A->nsend);
        else
            hipLaunchKernelGGL(pack_kernel<float>, dim3(grid), dim3(256), 0, st, (const float*)y,
                               A->send_idx, (float*)A->send_buf, A->nsend);
        EIGSOL_HIP(hipGetLastError());
    }
    ncclComm_t comm = static_cast<ncclComm_t>(ctx->comm);
    // RCCL element type of the vector payload: fp64 words for double / complex<double>, fp32 words
    // for float / complex<float> (the rank partials are always 4 doubles)
    const ncclDataType_t vty = dtype_single(A->dtype) ? ncclFloat32 : ncclFloat64;
    const size_t dpe = dtype_single(A->dtype) ? sb / 4 : sb / 8;   // RCCL elements per scalar
    char* xs = static_cast<char*>(y);   // x-space: [lower ghosts | own rows | upper ghosts]
    double* rpart = static_cast<double*>(rank_part);
    if (ctx->loop) {
        std::vector<LoopSend> ls;
        std::vector<LoopRecv> lr;
        if (A->exchange == EIGSOL_EXCHANGE_ALLGATHER) {
            const std::vector<int64_t>& rb = A->row_begins;
            for (int q = 0; q < ctx->nranks; ++q) {
                if (q == ctx->rank) continue;
                ls.push_back({q, xs + (size_t)rb[ctx->rank] * sb, (size_t)(rb[ctx->rank + 1] - rb[ctx->rank]) * sb});
                lr.push_back({q, xs + (size_t)rb[q] * sb, (size_t)(rb[q + 1] - rb[q]) * sb});
            }
        } else {
            for (int q = 0; q < ctx->nranks; ++q) {
                if (q == ctx->rank) continue;
                if (A->send_counts[q] > 0)
                    ls.push_back({q, static_cast<char*>(A->send_buf) + (size_t)A->send_offs[q] * sb,
                                  (size_t)A->send_counts[q] * sb});
                if (A->recv_counts[q] > 0)
                    lr.push_back({q, xs + (size_t)(A->recv_offs[q] + (q > ctx->rank ? A->nrows : 0)) * sb,
                                  (size_t)A->recv_counts[q] * sb});
            }
        }
        loop_allgather(ctx, rpart, 4 * sizeof(double), ls, lr);
        return loop_step(ctx, ls, lr);
    }
    if (A->exchange == EIGSOL_EXCHANGE_ALLGATHER) {
        // x-space = the global index space: every rank's own block lands in place on every rank
        const std::vector<int64_t>& rb = A->row_begins;
        const int P = ctx->nranks;
        bool equal = true;
        for (int q = 0; q < P; ++q) equal = equal && (rb[q + 1] - rb[q] == rb[1] - rb[0]);
        EIGSOL_RCCL(ncclGroupStart());
        if (equal) {
            EIGSOL_RCCL(ncclAllGather(xs + (size_t)rb[ctx->rank] * sb, xs, (size_t)(rb[1] - rb[0]) * dpe,
                                      vty, comm, st));
        } else {
            for (int q = 0; q < P; ++q)
                if (rb[q + 1] > rb[q])
                    EIGSOL_RCCL(ncclBroadcast(xs + (size_t)rb[q] * sb, xs + (size_t)rb[q] * sb,
                                              (size_t)(rb[q + 1] - rb[q]) * dpe, vty, q, comm, st));
        }
        EIGSOL_RCCL(ncclAllGather(rpart + 4 * ctx->rank, rpart, 4, ncclFloat64, comm, st));
        EIGSOL_RCCL(ncclGroupEnd());
        return EIGSOL_OK;
    }
    EIGSOL_RCCL(ncclGroupStart());
    for (int q = 0; q < ctx->nranks; ++q) {
        if (q == ctx->rank) continue;
        if (A->send_counts[q] > 0)
            EIGSOL_RCCL(ncclSend(static_cast<char*>(A->send_buf) + (size_t)A->send_offs[q] * sb,
                                 (size_t)A->send_counts[q] * dpe, vty, q, comm, st));
        if (A->recv_counts[q] > 0)
            EIGSOL_RCCL(ncclRecv(xs + (size_t)(A->recv_offs[q] + (q > ctx->rank ? A->nrows : 0)) * sb,
                                 (size_t)A->recv_counts[q] * dpe, vty, q, comm, st));
    }
    double* rp = static_cast<double*>(rank_part);
    EIGSOL_RCCL(ncclAllGather(rp + 4 * ctx->rank, rp, 4, ncclFloat64, comm, st));
    EIGSOL_RCCL(ncclGroupEnd());
    return EIGSOL_OK;
}

// All-gather exchange of an iteration split in two row parts (binned shards): part 0 moves rows
// [rb_q, rb_q + split[q]) of every rank q, part 1 the rest and the rank partials.  With RCCL the
// parts run on `comm` after an event on the compute stream, so part 0's transfer overlaps the
// second part's product; after part 1 the compute stream waits for `comm`.  The loopback world
// copies on the compute stream (same data movement, no overlap).
int dist_exchange_part(eigsol_csr* A, void* y, void* rank_part, int part, const std::vector<int64_t>& split,
                       hipStream_t comm_st, hipEvent_t* ev) {
    eigsol_ctx* ctx = A->ctx;
    const size_t sb = scalar_bytes(A->dtype);
    const int P = ctx->nranks, me = ctx->rank;
    const std::vector<int64_t>& rb = A->row_begins;
    char* xs = static_cast<char*>(y);
    double* rpart = static_cast<double*>(rank_part);
    auto seg = [&](int q, int64_t& lo, int64_t& hi) {
        lo = part == 0 ? rb[q] : rb[q] + split[q];
        hi = part == 0 ? rb[q] + split[q] : rb[q + 1];
    };
    if (ctx->loop) {
        std::vector<LoopSend> ls;
        std::vector<LoopRecv> lr;
        int64_t mlo, mhi;
        seg(me, mlo, mhi);
        for (int q = 0; q < P; ++q) {
            if (q == me) continue;
            int64_t lo, hi;
            seg(q, lo, hi);
            ls.push_back({q, xs + (size_t)mlo * sb, (size_t)(mhi - mlo) * sb});
            lr.push_back({q, xs + (size_t)lo * sb, (size_t)(hi - lo) * sb});
        }
        if (part == 1) loop_allgather(ctx, rpart, 4 * sizeof(double), ls, lr);
        return loop_step(ctx, ls, lr);
    }
    ncclComm_t comm = static_cast<ncclComm_t>(ctx->comm);
    const ncclDataType_t vty = dtype_single(A->dtype) ? ncclFloat32 : ncclFloat64;
    const size_t dpe = dtype_single(A->dtype) ? sb / 4 : sb / 8;
    EIGSOL_HIP(hipEventRecord(ev[part], ctx->stream));
    EIGSOL_HIP(hipStreamWaitEvent(comm_st, ev[part], 0));
    EIGSOL_RCCL(ncclGroupStart());
    for (int q = 0; q < P; ++q) {
        int64_t lo, hi;
        seg(q, lo, hi);
        if (hi > lo)
            EIGSOL_RCCL(ncclBroadcast(xs + (size_t)lo * sb, xs + (size_t)lo * sb, (size_t)(hi - lo) * dpe, vty, q,
                                      comm, comm_st));
    }
    if (part == 1) EIGSOL_RCCL(ncclAllGather(rpart + 4 * me, rpart, 4, ncclFloat64, comm, comm_st));
    EIGSOL_RCCL(ncclGroupEnd());
    if (part == 1) {
        EIGSOL_HIP(hipEventRecord(ev[2], comm_st));
        EIGSOL_HIP(hipStreamWaitEvent(ctx->stream, ev[2], 0));
    }
    return EIGSOL_OK;
}

}  // namespace eigsol

using namespace eigsol;

extern "C" {

// Pure host planning (no device, no communication): remap a rank's global column indices to the
// local x-space [ghosts of lower ranks | own rows | ghosts of higher ranks] — monotone in the global
// index, so banded row blocks keep compact column windows — and list the ghosts per owner
// (ascending global index; the lower-rank ghosts come first).  Exported for callers that exchange
// the request lists with their own transport, and for the CPU tests.
int eigsol_ghost_plan(int nranks, const int64_t* row_begins, int rank, int64_t nnz_local,
                      const int32_t* colidx_global, int32_t* colidx_local, int64_t* nghost,
                      int64_t* ghost_global, int64_t* recv_counts) {
    if (nranks < 1 || rank < 0 || rank >= nranks || !row_begins || !nghost || !recv_counts ||
        (nnz_local && (!colidx_global || !colidx_local || !ghost_global)))
        return fail(EIGSOL_E_INVALID, "eigsol_ghost_plan: invalid argument");
    for (int q = 0; q < nranks; ++q)
        if (row_begins[q + 1] < row_begins[q])
            return fail(EIGSOL_E_INVALID, "eigsol_ghost_plan: row_begins not monotone");
    const int64_t r0 = row_begins[rank], r1 = row_begins[rank + 1], n_global = row_begins[nranks];
    std::vector<int64_t> g;
    g.reserve(64);
    for (int64_t k = 0; k < nnz_local; ++k) {
        const int64_t c = colidx_global[k];
        if (c < 0 || c >= n_global) return fail(EIGSOL_E_INVALID, "eigsol_ghost_plan: column out of range");
        if (c < r0 || c >= r1) g.push_back(c);
    }
    std::sort(g.begin(), g.end());
    g.erase(std::unique(g.begin(), g.end()), g.end());
    // owners are contiguous row blocks, so sorting by global index groups ghosts by owner
    for (int q = 0; q < nranks; ++q) recv_counts[q] = 0;
    int q = 0;
    for (int64_t c : g) {
        while (c >= row_begins[q + 1]) ++q;
        recv_counts[q]++;
    }
    *nghost = (int64_t)g.size();
    std::copy(g.begin(), g.end(), ghost_global);
    const int64_t nown = r1 - r0;
    const int64_t nlow = std::lower_bound(g.begin(), g.end(), r0) - g.begin();
    for (int64_t k = 0; k < nnz_local; ++k) {
        const int64_t c = colidx_global[k];
        if (c >= r0 && c < r1) {
            colidx_local[k] = (int32_t)(nlow + c - r0);
        } else {
            const int64_t pos = std::lower_bound(g.begin(), g.end(), c) - g.begin();
            colidx_local[k] = (int32_t)(pos < nlow ? pos : nown + pos);
        }
    }
    return EIGSOL_OK;
}

int eigsol_exchange_mode(int nranks, const int64_t* row_begins, const int64_t* ghost_counts, int* mode) {
    if (nranks < 1 || !row_begins || !ghost_counts || !mode)
        return fail(EIGSOL_E_INVALID, "eigsol_exchange_mode: invalid argument");
    const int64_t n_global = row_begins[nranks];
    int m = EIGSOL_EXCHANGE_HALO;
    for (int r = 0; r < nranks; ++r) {
        int64_t g = 0;
        for (int q = 0; q < nranks; ++q) g += q == r ? 0 : ghost_counts[(size_t)r * nranks + q];
        const int64_t remote = n_global - (row_begins[r + 1] - row_begins[r]);
        if (remote > 0 && 4 * g >= remote) m = EIGSOL_EXCHANGE_ALLGATHER;
    }
    if (const char* e = std::getenv("EIGSOL_DIST_EXCHANGE")) {
        if (!std::strcmp(e, "halo")) m = EIGSOL_EXCHANGE_HALO;
        else if (!std::strcmp(e, "allgather")) m = EIGSOL_EXCHANGE_ALLGATHER;
    }
    *mode = m;
    return EIGSOL_OK;
}

int eigsol_csr_dist_info(const eigsol_csr* A, int* mode, int64_t* nghost) {
    if (!A) return fail(EIGSOL_E_INVALID, "eigsol_csr_dist_info: null matrix");
    if (mode) *mode = A->dist ? A->exchange : EIGSOL_EXCHANGE_HALO;
    if (nghost) *nghost = A->dist ? A->nghost : 0;
    return EIGSOL_OK;
}

int eigsol_dist_get_unique_id(void* id_out) {
    if (!id_out) return fail(EIGSOL_E_INVALID, "eigsol_dist_get_unique_id: null pointer");
    ncclUniqueId id;
    EIGSOL_RCCL(ncclGetUniqueId(&id));
    std::memcpy(id_out, &id, sizeof(id));
    return EIGSOL_OK;
}

int eigsol_dist_unique_id_bytes(void) { return NCCL_UNIQUE_ID_BYTES; }

int eigsol_dist_loopback_id(int nranks, void* id_out) {
    if (!id_out || nranks < 1) return fail(EIGSOL_E_INVALID, "eigsol_dist_loopback_id: invalid argument");
    static std::atomic<long> serial{0};
    char buf[NCCL_UNIQUE_ID_BYTES] = {0};
    std::snprintf(buf, sizeof(buf), "%s%d:%ld:%p", kLoopMagic, nranks, serial.fetch_add(1), (void*)&serial);
    std::memcpy(id_out, buf, sizeof(buf));
    return EIGSOL_OK;
}

int eigsol_ctx_create_dist(int device, int rank, int nranks, const void* unique_id,
                           eigsol_ctx** out) {
    if (!out || !unique_id || nranks < 1 || rank < 0 || rank >= nranks)
        return fail(EIGSOL_E_INVALID, "eigsol_ctx_create_dist: invalid argument");
    EIGSOL_TRY(eigsol_ctx_create(device, out));
    if (std::strncmp(static_cast<const char*>(unique_id), kLoopMagic, sizeof(kLoopMagic) - 1) == 0) {
        const std::string key(static_cast<const char*>(unique_id),
                              strnlen(static_cast<const char*>(unique_id), NCCL_UNIQUE_ID_BYTES));
        std::shared_ptr<LoopWorld> w;
        {
            std::lock_guard<std::mutex> g(g_loop_m);
            auto& slot = g_loop_worlds[key];
            if (!slot) {
                slot = std::make_shared<LoopWorld>();
                slot->P = nranks;
                slot->sends.resize(nranks);
                slot->hbuf.resize(nranks);
                slot->ready.resize(nranks);
                slot->done.resize(nranks);
                for (int q = 0; q < nranks; ++q) {
                    hipEventCreateWithFlags(&slot->ready[q], hipEventDisableTiming);
                    hipEventCreateWithFlags(&slot->done[q], hipEventDisableTiming);
                }
            }
            w = slot;
            ++w->joined;
        }
        if (w->P != nranks) {
            eigsol_ctx_destroy(*out);
            *out = nullptr;
            return fail(EIGSOL_E_INVALID, "eigsol_ctx_create_dist: loopback world size mismatch");
        }
        (*out)->loop = w.get();
        (*out)->rank = rank;
        (*out)->nranks = nranks;
        return EIGSOL_OK;
    }
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    ncclComm_t comm = nullptr;
    ncclResult_t r = ncclCommInitRank(&comm, nranks, id, rank);
    if (r != ncclSuccess) {
        eigsol_ctx_destroy(*out);
        *out = nullptr;
        return fail(EIGSOL_E_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    (*out)->comm = comm;
    (*out)->rank = rank;
    (*out)->nranks = nranks;
    return EIGSOL_OK;
}

// Collective over the context's communicator: every rank passes its own row block.  The setup
// exchanges (ghost counts, request lists) are host all-gathers (coll_allgather), so the same code
// serves RCCL, loopback and host-bootstrapped contexts.
int eigsol_csr_create_dist(eigsol_ctx* ctx, eigsol_dtype dtype, const int64_t* row_begins,
                           int64_t nnz_local, const int32_t* rowptr_local,
                           const int32_t* colidx_global, const void* values, eigsol_csr** out) {
    if (!ctx || !out || !row_begins || !rowptr_local)
        return fail(EIGSOL_E_INVALID, "eigsol_csr_create_dist: null argument");
    if (!ctx->comm && !ctx->loop && !ctx->hcoll)
        return fail(EIGSOL_E_INVALID, "eigsol_csr_create_dist: context has no communicator");
    *out = nullptr;
    if (dtype_wide(dtype))
        return fail(EIGSOL_E_UNSUPPORTED, "eigsol_csr_create_dist: the row-sharded path has no double-double kernels");
    if (dtype != EIGSOL_F64 && dtype != EIGSOL_C128 && dtype != EIGSOL_F32 && dtype != EIGSOL_C64)
        return fail(EIGSOL_E_INVALID, "eigsol_csr_create_dist: unknown dtype");
    const int P = ctx->nranks, me = ctx->rank;
    if (row_begins[0] != 0 || nnz_local < 0)
        return fail(EIGSOL_E_INVALID, "eigsol_csr_create_dist: row_begins must start at 0 and nnz be >= 0");
    for (int q = 0; q < P; ++q)
        if (row_begins[q + 1] < row_begins[q])
            return fail(EIGSOL_E_INVALID, "eigsol_csr_create_dist: row_begins not monotone");
    const int64_t n_global = row_begins[P];
    const int64_t nrows = row_begins[me + 1] - row_begins[me];
    if (n_global > INT32_MAX - 1)
        return fail(EIGSOL_E_INVALID, "eigsol_csr_create_dist: dimension exceeds int32 storage index");
    if (rowptr_local[0] != 0 || rowptr_local[nrows] != nnz_local)
        return fail(EIGSOL_E_INVALID, "eigsol_csr_create_dist: rowptr must start at 0 and end at nnz");
    std::vector<int32_t> col_local(std::max<int64_t>(nnz_local, 1));
    std::vector<int64_t> ghosts(std::max<int64_t>(nnz_local, 1)), recv(P), nghost(1);
    EIGSOL_TRY(eigsol_ghost_plan(P, row_begins, me, nnz_local, colidx_global, col_local.data(),
                                 nghost.data(), ghosts.data(), recv.data()));
    EIGSOL_HIP(hipSetDevice(ctx->device));
    // every rank learns how many entries each peer requests from it (P x P counts)
    std::vector<int64_t> all((size_t)P * P);
    EIGSOL_TRY(coll_allgather(ctx, recv.data(), sizeof(int64_t) * P, all.data()));
    int mode = EIGSOL_EXCHANGE_HALO;
    EIGSOL_TRY(eigsol_exchange_mode(P, row_begins, all.data(), &mode));   // same decision on every rank
    if (mode == EIGSOL_EXCHANGE_ALLGATHER) {
        // replicated x: local columns are the global ones, own rows sit at their global slots
        eigsol_csr* A = nullptr;
        EIGSOL_TRY(csr_upload(ctx, dtype, nrows, n_global, nnz_local, rowptr_local, colidx_global, values, &A,
                              row_begins[me]));
        A->dist = 1;
        A->exchange = EIGSOL_EXCHANGE_ALLGATHER;
        A->n_global = n_global;
        A->row_begin = row_begins[me];
        A->nghost = n_global - nrows;
        A->row_begins.assign(row_begins, row_begins + P + 1);
        A->send_counts.assign(P, 0);
        A->recv_counts.assign(P, 0);
        A->send_offs.assign(P, 0);
        A->recv_offs.assign(P, 0);
        *out = A;
        return EIGSOL_OK;
    }
    std::vector<int64_t> send(P), soff(P + 1, 0), roff(P + 1, 0);
    for (int q = 0; q < P; ++q) send[q] = (q == me) ? 0 : all[(size_t)q * P + me];
    for (int q = 0; q < P; ++q) {
        soff[q + 1] = soff[q] + send[q];
        roff[q + 1] = roff[q] + recv[q];
    }
    const int64_t nsend = soff[P];
    // request lists (global indices) to their owners: every rank's whole ghost list, padded to the
    // longest, all-gathered; each rank keeps the part addressed to it (ghost lists are grouped by
    // owner, so q's requests to me start at sum_{p < me} all[q][p])
    int64_t maxg = 0;
    for (int q = 0; q < P; ++q) {
        int64_t g = 0;
        for (int p = 0; p < P; ++p) g += all[(size_t)q * P + p];
        maxg = std::max(maxg, g);
    }
    std::vector<int64_t> mine(std::max<int64_t>(maxg, 1), -1), lists((size_t)P * std::max<int64_t>(maxg, 1));
    std::copy(ghosts.begin(), ghosts.begin() + nghost[0], mine.begin());
    EIGSOL_TRY(coll_allgather(ctx, mine.data(), sizeof(int64_t) * mine.size(), lists.data()));
    std::vector<int64_t> req(std::max<int64_t>(nsend, 1));
    for (int q = 0; q < P; ++q) {
        if (q == me || !send[q]) continue;
        int64_t off = 0;
        for (int p = 0; p < me; ++p) off += all[(size_t)q * P + p];
        std::copy_n(lists.begin() + (size_t)q * mine.size() + off, send[q], req.begin() + soff[q]);
    }
    int64_t nlow = 0;
    for (int q = 0; q < me; ++q) nlow += recv[q];
    std::vector<int32_t> send_idx(std::max<int64_t>(nsend, 1));
    for (int64_t k = 0; k < nsend; ++k) {
        const int64_t loc = req[k] - row_begins[me];
        if (loc < 0 || loc >= nrows)
            return fail(EIGSOL_E_RCCL, "eigsol_csr_create_dist: peer requested a row this rank does not own");
        send_idx[k] = (int32_t)(loc + nlow);   // x-space slot of the requested own row
    }
    eigsol_csr* A = nullptr;
    EIGSOL_TRY(csr_upload(ctx, dtype, nrows, nrows + nghost[0], nnz_local, rowptr_local,
                          col_local.data(), values, &A, nlow));
    A->dist = 1;
    A->n_global = n_global;
    A->row_begin = row_begins[me];
    A->nghost = nghost[0];
    A->row_begins.assign(row_begins, row_begins + P + 1);
    A->send_counts = send;
    A->recv_counts = recv;
    A->send_offs.assign(soff.begin(), soff.end() - 1);
    A->recv_offs.assign(roff.begin(), roff.end() - 1);
    A->nsend = nsend;
    A->h_send_idx.assign(send_idx.begin(), send_idx.begin() + nsend);
    A->peer_dst_off.assign(P, 0);
    for (int q = 0; q < P; ++q)
        for (int p = 0; p < me; ++p) A->peer_dst_off[q] += all[(size_t)q * P + p];
    A->ghost_counts = all;
    A->requests.assign(req.begin(), req.begin() + nsend);
    const size_t sb = scalar_bytes(dtype);
    hipStream_t st = ctx->stream;
    hipError_t e = hipMalloc(&A->send_idx, sizeof(int32_t) * std::max<int64_t>(nsend, 1));
    if (e == hipSuccess) e = hipMalloc(&A->send_buf, sb * std::max<int64_t>(nsend, 1));
    if (e == hipSuccess && nsend)
        e = hipMemcpyAsync(A->send_idx, send_idx.data(), sizeof(int32_t) * nsend, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        eigsol_csr_destroy(A);
        return fail(EIGSOL_E_HIP, std::string("eigsol_csr_create_dist: ") + hipGetErrorString(e));
    }
    *out = A;
    return EIGSOL_OK;
}

int eigsol_peer_plan(int nranks, int rank, const int64_t* row_begins, const int64_t* ghost_counts,
                     const int64_t* requests, int64_t nreq, int32_t* push_out) {
    if (nranks < 1 || rank < 0 || rank >= nranks || !row_begins || !ghost_counts || nreq < 0 ||
        (nreq && (!requests || !push_out)))
        return fail(EIGSOL_E_INVALID, "eigsol_peer_plan: invalid argument");
    const int P = nranks;
    const int64_t r0 = row_begins[rank], nrows = row_begins[rank + 1] - r0;
    std::vector<std::array<int32_t, 4>> ent;
    ent.reserve(nreq);
    int64_t k = 0;
    for (int q = 0; q < P; ++q) {
        if (q == rank) continue;
        const int64_t cnt = ghost_counts[(size_t)q * P + rank];
        int64_t base = 0;   // where this rank's rows start in q's ghost list
        for (int p = 0; p < rank; ++p) base += ghost_counts[(size_t)q * P + p];
        for (int64_t j = 0; j < cnt; ++j, ++k) {
            if (k >= nreq) return fail(EIGSOL_E_INVALID, "eigsol_peer_plan: fewer requests than ghost counts");
            const int64_t loc = requests[k] - r0;
            if (loc < 0 || loc >= nrows) return fail(EIGSOL_E_INVALID, "eigsol_peer_plan: request outside own rows");
            ent.push_back({(int32_t)loc, (int32_t)q, (int32_t)(base + j), 0});
        }
    }
    if (k != nreq) return fail(EIGSOL_E_INVALID, "eigsol_peer_plan: more requests than ghost counts");
    std::stable_sort(ent.begin(), ent.end(), [](const auto& x, const auto& y) { return x[0] < y[0]; });
    for (size_t i = 0; i < ent.size(); ++i)
        for (int c = 0; c < 4; ++c) push_out[4 * i + c] = ent[i][c];
    return EIGSOL_OK;
}

int eigsol_ctx_create_dist_host(int device, int rank, int nranks, eigsol_allgather_fn allgather,
                                void* user, eigsol_ctx** out) {
    if (!out || !allgather || nranks < 1 || rank < 0 || rank >= nranks)
        return fail(EIGSOL_E_INVALID, "eigsol_ctx_create_dist_host: invalid argument");
    EIGSOL_TRY(eigsol_ctx_create(device, out));
    (*out)->hcoll = allgather;
    (*out)->hcoll_user = user;
    (*out)->rank = rank;
    (*out)->nranks = nranks;
    return EIGSOL_OK;
}

}  // extern "C"

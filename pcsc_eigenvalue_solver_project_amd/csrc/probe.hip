// Device bandwidth probe (measurement only; bench.py reports it beside the 8 TB/s spec as the
// box's practical HBM ceiling, SURVEY §8d "verify with a STREAM-like kernel on the box").
//
// Hand-written gfx950 streams over one buffer of `bytes` (>= 2 GiB, so neither the 4 MB L2s nor
// the 256 MB Infinity Cache hold it): non-temporal loads / stores, four in flight per lane,
// grid-stride over 256-thread workgroups.  Three shapes:
//   read  - load only, 16-byte (dwordx4) and 8-byte (dwordx2) loads, the better of the two (the
//           loads feed an xor reduction that is stored only if it matches a sentinel, so the
//           compiler keeps every load and nothing is written; round 4, tools/width_probe.hip:
//           8-byte loads at 4 workgroups per CU read 7.3 TB/s, 16-byte ones 6.9 TB/s);
//   copy  - load + store to a second buffer (read + write bytes counted);
//   write - store only.
// Each is timed with HIP events on the context's stream over `reps` launches, for grids of 1, 2,
// 4 and 8 workgroups per CU; the best of those is reported.
#include <algorithm>
#include <vector>

#include "internal.hpp"

namespace eigsol {
namespace pdev {

using u4 = __attribute__((ext_vector_type(4))) unsigned int;
using u2 = __attribute__((ext_vector_type(2))) unsigned int;

constexpr int kT = 256;
constexpr int kU = 4;   // 16-byte accesses in flight per lane

__global__ __launch_bounds__(kT) void read_kernel(const u4* __restrict__ a, size_t n16, unsigned int* out) {
    const size_t stride = (size_t)gridDim.x * kT * kU;
    u4 acc = {0u, 0u, 0u, 0u};
    for (size_t base = (size_t)blockIdx.x * kT * kU + threadIdx.x; base < n16; base += stride) {
        u4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const size_t i = base + (size_t)u * kT;
            v[u] = i < n16 ? __builtin_nontemporal_load(a + i) : u4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) acc ^= v[u];
    }
    const unsigned int r = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (r == 0x9e3779b9u) out[0] = r;   // never true for the probe's zero-filled buffer
}

__global__ __launch_bounds__(kT) void read8_kernel(const u2* __restrict__ a, size_t n8, unsigned int* out) {
    const size_t stride = (size_t)gridDim.x * kT * kU;
    u2 acc = {0u, 0u};
    for (size_t base = (size_t)blockIdx.x * kT * kU + threadIdx.x; base < n8; base += stride) {
        u2 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const size_t i = base + (size_t)u * kT;
            v[u] = i < n8 ? __builtin_nontemporal_load(a + i) : u2{0u, 0u};
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) acc ^= v[u];
    }
    const unsigned int r = acc.x ^ acc.y;
    if (r == 0x9e3779b9u) out[0] = r;
}

__global__ __launch_bounds__(kT) void copy_kernel(const u4* __restrict__ a, u4* __restrict__ b, size_t n16) {
    const size_t stride = (size_t)gridDim.x * kT * kU;
    for (size_t base = (size_t)blockIdx.x * kT * kU + threadIdx.x; base < n16; base += stride) {
        u4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const size_t i = base + (size_t)u * kT;
            v[u] = i < n16 ? __builtin_nontemporal_load(a + i) : u4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const size_t i = base + (size_t)u * kT;
            if (i < n16) __builtin_nontemporal_store(v[u], b + i);
        }
    }
}

__global__ __launch_bounds__(kT) void write_kernel(u4* __restrict__ b, size_t n16) {
    const size_t stride = (size_t)gridDim.x * kT * kU;
    const u4 z = {0u, 0u, 0u, 0u};
    for (size_t base = (size_t)blockIdx.x * kT * kU + threadIdx.x; base < n16; base += stride)
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const size_t i = base + (size_t)u * kT;
            if (i < n16) __builtin_nontemporal_store(z, b + i);
        }
}

// read / write mix of the headline SpMV (reads 1.0 GB, writes y's 80 MB: ~12.5 : 1): every lane
// loads kMixR 16-byte words from `a` (kU in flight) and stores their xor as one 16-byte word to
// `b`, non-temporal like the other shapes
constexpr int kMixR = 12;
__global__ __launch_bounds__(kT) void mix_kernel(const u4* __restrict__ a, u4* __restrict__ b, size_t nout) {
    for (size_t o = (size_t)blockIdx.x * kT + threadIdx.x; o < nout; o += (size_t)gridDim.x * kT) {
        const size_t blk = (o / kT) * (size_t)kT * kMixR + (o % kT);   // coalesced: 12 wave-wide loads
        u4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int r = 0; r < kMixR; ++r) acc ^= __builtin_nontemporal_load(a + blk + (size_t)r * kT);
        __builtin_nontemporal_store(acc, b + o);
    }
}

}  // namespace pdev
}  // namespace eigsol

using namespace eigsol;

extern "C" {

int eigsol_hbm_probe(eigsol_ctx* ctx, size_t bytes, int reps, double* read_gbps, double* copy_gbps,
                     double* write_gbps, int* best_blocks_per_cu) {
    if (!ctx || bytes < 16) return fail(EIGSOL_E_INVALID, "eigsol_hbm_probe: null ctx or empty buffer");
    reps = std::max(1, reps);
    EIGSOL_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const size_t n16 = bytes / 16;
    void *a = nullptr, *b = nullptr, *o = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = EIGSOL_OK;
    if (hipMalloc(&a, n16 * 16) != hipSuccess || hipMalloc(&b, n16 * 16) != hipSuccess || hipMalloc(&o, 64) != hipSuccess ||
        hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "eigsol_hbm_probe: allocation (2 x " + std::to_string(bytes) + " bytes)");
    double best[3] = {0.0, 0.0, 0.0};
    int best_bpc = 0;
    if (rc == EIGSOL_OK) {
        (void)hipMemsetAsync(a, 0, n16 * 16, st);
        (void)hipMemsetAsync(b, 0, n16 * 16, st);
        const auto* ap = static_cast<const pdev::u4*>(a);
        auto* bp = static_cast<pdev::u4*>(b);
        for (int bpc : {1, 2, 4, 8}) {
            const unsigned grid = (unsigned)(bpc * ctx->num_cus);
            for (int kind = 0; kind < 4 && rc == EIGSOL_OK; ++kind) {   // read16, copy, write, read8
                auto launch = [&]() {
                    if (kind == 0)
                        hipLaunchKernelGGL(pdev::read_kernel, dim3(grid), dim3(pdev::kT), 0, st, ap, n16,
                                           static_cast<unsigned int*>(o));
                    else if (kind == 3)
                        hipLaunchKernelGGL(pdev::read8_kernel, dim3(grid), dim3(pdev::kT), 0, st,
                                           reinterpret_cast<const pdev::u2*>(ap), 2 * n16, static_cast<unsigned int*>(o));
                    else if (kind == 1)
                        hipLaunchKernelGGL(pdev::copy_kernel, dim3(grid), dim3(pdev::kT), 0, st, ap, bp, n16);
                    else
                        hipLaunchKernelGGL(pdev::write_kernel, dim3(grid), dim3(pdev::kT), 0, st, bp, n16);
                };
                launch();   // warm-up
                (void)hipEventRecord(e0, st);
                for (int r = 0; r < reps; ++r) launch();
                (void)hipEventRecord(e1, st);
                float ms = 0.0f;
                if (hipGetLastError() != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                    hipEventElapsedTime(&ms, e0, e1) != hipSuccess || ms <= 0.0f) {
                    rc = fail(EIGSOL_E_HIP, "eigsol_hbm_probe: timing");
                    break;
                }
                const double moved = (double)(n16 * 16) * (kind == 1 ? 2.0 : 1.0) * reps;
                const double gbps = moved / (ms * 1e-3) / 1e9;
                const int slot = kind == 3 ? 0 : kind;   // read: the better load width
                if (gbps > best[slot]) {
                    best[slot] = gbps;
                    if (slot == 0) best_bpc = bpc;
                }
            }
        }
    }
    if (read_gbps) *read_gbps = best[0];
    if (copy_gbps) *copy_gbps = best[1];
    if (write_gbps) *write_gbps = best[2];
    if (best_blocks_per_cu) *best_blocks_per_cu = best_bpc;
    (void)hipStreamSynchronize(st);
    for (void* p : {a, b, o})
        if (p) (void)hipFree(p);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    return rc;
}

// The read / write mix of the headline (12 reads : 1 write, 16-byte non-temporal accesses) over
// `bytes` of reads, best of 1/2/4/8 workgroups per CU: the practical ceiling for a kernel that
// streams a matrix and writes a vector, next to the read-only ceiling of eigsol_hbm_probe.
int eigsol_hbm_probe_mix(eigsol_ctx* ctx, size_t bytes, int reps, double* mix_gbps, int* best_blocks_per_cu) {
    if (!ctx || bytes < 16 * pdev::kMixR * pdev::kT) return fail(EIGSOL_E_INVALID, "eigsol_hbm_probe_mix: bad arguments");
    reps = std::max(1, reps);
    EIGSOL_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const size_t per = (size_t)16 * pdev::kMixR * pdev::kT;
    const size_t nblk = bytes / per;
    const size_t nin = nblk * pdev::kMixR * pdev::kT, nout = nblk * pdev::kT;
    void *a = nullptr, *b = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = EIGSOL_OK;
    if (hipMalloc(&a, nin * 16) != hipSuccess || hipMalloc(&b, nout * 16) != hipSuccess ||
        hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "eigsol_hbm_probe_mix: allocation");
    double best = 0.0;
    int best_bpc = 0;
    if (rc == EIGSOL_OK) {
        (void)hipMemsetAsync(a, 0, nin * 16, st);
        for (int bpc : {1, 2, 4, 8}) {
            const unsigned grid = (unsigned)(bpc * ctx->num_cus);
            auto launch = [&]() {
                hipLaunchKernelGGL(pdev::mix_kernel, dim3(grid), dim3(pdev::kT), 0, st, static_cast<const pdev::u4*>(a),
                                   static_cast<pdev::u4*>(b), nout);
            };
            launch();
            (void)hipEventRecord(e0, st);
            for (int r = 0; r < reps; ++r) launch();
            (void)hipEventRecord(e1, st);
            float ms = 0.0f;
            if (hipGetLastError() != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                hipEventElapsedTime(&ms, e0, e1) != hipSuccess || ms <= 0.0f) {
                rc = fail(EIGSOL_E_HIP, "eigsol_hbm_probe_mix: timing");
                break;
            }
            const double gbps = (double)(nin + nout) * 16.0 * reps / (ms * 1e-3) / 1e9;
            if (gbps > best) {
                best = gbps;
                best_bpc = bpc;
            }
        }
    }
    if (mix_gbps) *mix_gbps = best;
    if (best_blocks_per_cu) *best_blocks_per_cu = best_bpc;
    (void)hipStreamSynchronize(st);
    for (void* p : {a, b})
        if (p) (void)hipFree(p);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    return rc;
}

// This context's place in a multi-GPU world: rank, ranks, and how it exchanges (0 none, 1 RCCL
// communicator, 2 in-process loopback world, 3 caller's host all-gather with device peer inboxes).
int eigsol_ctx_info(eigsol_ctx* ctx, int* device, int* rank, int* nranks, int* comm_kind) {
    if (!ctx) return fail(EIGSOL_E_INVALID, "eigsol_ctx_info: null ctx");
    if (device) *device = ctx->device;
    if (rank) *rank = ctx->rank;
    if (nranks) *nranks = ctx->nranks;
    if (comm_kind) *comm_kind = ctx->comm ? 1 : ctx->loop ? 2 : ctx->hcoll ? 3 : 0;
    return EIGSOL_OK;
}

}  // extern "C"

// Device-resident dense (column-major) matrix and the fused power-iteration GEMV for gfx950.
//
// Dense branch of powerMethod<S> (src/power_method/power_method.hpp:141-143): y = A*x with A a
// column-major Eigen matrix (matrix.hpp:39-40).  HBM-bound (8 n^2 bytes per iteration), so the
// kernel streams A exactly once per iteration with coalesced 16-byte lane loads:
//
//   grid = row tiles (128 rows f64 / 64 rows c128) x column chunks.  In a block, lane l owns rows
//   (2l, 2l+1) (f64) of the tile and each of the 4 waves sweeps a quarter of the chunk's columns,
//   so every wave-load is one contiguous 1 KiB piece of a column.  Wave partials meet in LDS in a
//   fixed order; chunk partials meet through a per-tile last-arriver (write-through sc1 stores +
//   ticket, MI355X guide §6 G16), whose reducer sums the chunks in column order, writes y, and
//   feeds ||y||^2 and x^H y into the grid-level last-arriver shared with the CSR kernel.
#include <algorithm>
#include <cstring>
#include <type_traits>

#include "kernels_common.hpp"

// columns per load batch of dense_kernel (EIGSOL_DENSE_KU overrides at build time).  Round 6
// (tools/r06_dense_ku_ab.sh, 16384^2): f64 4 / 8 / 12 / 16 -> 0.324 / 0.324 / 0.343 / 0.334 ms,
// c128 0.660-0.667 / 0.661 / 0.663-0.667 / 0.647-0.649 ms: 8 for f64, 16 for 16-byte scalars
template <class S>
constexpr int dense_ku() {
#ifdef EIGSOL_DENSE_KU
    return EIGSOL_DENSE_KU;
#else
    return sizeof(S) == 16 ? 16 : 8;
#endif
}

namespace eigsol {
namespace dev {

// A lane owns 16 bytes of a column: 2 rows (f64, c64), 4 rows (f32) or 1 row (c128).
template <class S> struct DenseTile {
    static constexpr int kPerLane = 16 / (int)sizeof(S);
    static constexpr int kRows = 64 * kPerLane;
};

// the lane's 16 bytes of a column (non-temporal: A is read once per iteration)
template <class S, int PL>
__device__ __forceinline__ void load_col16(const S* p, S (&v)[PL]) {
    typedef double d2v __attribute__((ext_vector_type(2)));
    const d2v t = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
    __builtin_memcpy(&v[0], &t, 16);
}

// one 8-byte scalar, non-temporal (the bits through a double: cplxf is a struct)
template <class S>
__device__ __forceinline__ S load8_nt(const S* p) {
    static_assert(sizeof(S) == 8, "8-byte scalars");
    const double t = __builtin_nontemporal_load(reinterpret_cast<const double*>(p));
    S v;
    __builtin_memcpy(&v, &t, 8);
    return v;
}

template <class S>
struct DenseArgs {
    const S* a;            // column-major, leading dimension n
    int64_t n;             // rows (= cols for power)
    int64_t ncols;
    int32_t ntr;           // row tiles
    int32_t nchunk;        // column chunks
    int32_t cw;            // columns per chunk
    S* ypart;              // [nchunk][n] chunk partials
    uint32_t* tile_cnt;    // [ntr]
    const S* x_plain;
    S* y_plain;
    S* buf0;
    S* buf1;
    PowerCtl* ctl;
    const part4* rank_part;
    int32_t nranks;
    part4* my_part;
    part4* blk_part;
    S* trace;
};

__device__ __forceinline__ void st_agent_s(double* p, double v) { st_agent(p, v); }
__device__ __forceinline__ void st_agent_s(cplx* p, cplx v) {
    st_agent(&p->re, v.re);
    st_agent(&p->im, v.im);
}
__device__ __forceinline__ void st_agent_s(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent_s(cplxf* p, cplxf v) {
    st_agent_s(&p->re, v.re);
    st_agent_s(&p->im, v.im);
}
__device__ __forceinline__ float ld_agent_s(const float* p) {
    return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ cplxf ld_agent_s(const cplxf* p) { return cplxf{ld_agent_s(&p->re), ld_agent_s(&p->im)}; }
__device__ __forceinline__ double ld_agent_s(const double* p) { return ld_agent(p); }
__device__ __forceinline__ cplx ld_agent_s(const cplx* p) { return cplx{ld_agent(&p->re), ld_agent(&p->im)}; }

// kSplit (8-byte scalars, PL = 2): lane l owns rows l and l + 64 of the tile instead of 2l and
// 2l + 1, loaded by two 8-byte loads per column whose wave-instructions each cover 512 contiguous
// bytes (round 4, tools/width_probe.hip: 8-byte non-temporal streams read 7.3 TB/s at 4 workgroups
// per CU, 16-byte ones 6.7-6.9).  Every row is still summed over the columns in the same order.
template <class S, bool kPower, bool kSplit = false>
__global__ __launch_bounds__(kThreads) void dense_kernel(DenseArgs<S> a, int parity) {
    constexpr int R = DenseTile<S>::kRows;
    constexpr int PL = DenseTile<S>::kPerLane;
    __shared__ S wpart[kWaves][R];
    __shared__ double sm[3 * kWaves];
    __shared__ Prologue pro;
    __shared__ int s_last;
    __shared__ int s_tile_last;

    const S* xin;
    S* yout;
    double nrm = 0.0;
    if constexpr (kPower) {
        power_prologue<S>(a.ctl, a.rank_part, a.nranks, parity, a.trace, &pro);
        if (!__builtin_amdgcn_readfirstlane(pro.go)) return;   // block-uniform exit
        nrm = pro.nrm;
        xin = parity ? a.buf0 : a.buf1;
        yout = parity ? a.buf1 : a.buf0;
    } else {
        xin = a.x_plain;
        yout = a.y_plain;
    }
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    // block -> (row tile, column chunk); chunks of one tile are consecutive block ids
    const int rt = blockIdx.x / a.nchunk;
    const int ch = blockIdx.x % a.nchunk;
    static_assert(!kSplit || PL == 2, "split rows: two 8-byte rows per lane");
    const int64_t row0 = kSplit ? (int64_t)rt * R + lane : (int64_t)rt * R + (int64_t)lane * PL;
    // row of the lane's p-th value
    auto lrow = [&](int p) -> int64_t { return kSplit ? row0 + 64 * p : row0 + p; };
    const int64_t c0 = (int64_t)ch * a.cw;
    const int64_t c1 = min<int64_t>(a.ncols, c0 + a.cw);

    S acc[PL];
#pragma unroll
    for (int p = 0; p < PL; ++p) acc[p] = s_zero<S>();
    // the chunk's columns are split contiguously over the 4 waves
    const int64_t span = (c1 - c0 + kWaves - 1) / kWaves;
    const int64_t wc0 = c0 + w * span;
    const int64_t wc1 = min<int64_t>(c1, wc0 + span);
    // 16-byte column pieces need the tile inside the matrix and 16-byte aligned columns
    const bool vec = kSplit ? lrow(PL - 1) < a.n : (row0 + PL <= a.n && (a.n % PL) == 0);
    int64_t j = wc0;
    {
        // batches of kU columns, all loads issued before the products (A read once: non-temporal),
        // the same per-row summation order as the one-column loop below
        constexpr int kU = dense_ku<S>();
        if (vec) {
            for (; j + kU <= wc1; j += kU) {
                S xj[kU];
                S v[kU][PL];
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    xj[u] = xin[j + u];
                    if constexpr (kSplit) {
#pragma unroll
                        for (int p = 0; p < PL; ++p) v[u][p] = load8_nt(a.a + (j + u) * a.n + lrow(p));
                    } else {
                        load_col16<S, PL>(a.a + (j + u) * a.n + row0, v[u]);
                    }
                }
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    S x = xj[u];
                    if constexpr (kPower) x = scale_in(x, nrm);
#pragma unroll
                    for (int p = 0; p < PL; ++p) acc[p] = add(acc[p], mul(v[u][p], x));
                }
            }
        }
    }
    for (; j < wc1; ++j) {
        S xj = xin[j];
        if constexpr (kPower) xj = scale_in(xj, nrm);
        const S* col = a.a + j * a.n;
        if (vec) {
            S v[PL];
            if constexpr (kSplit) {
#pragma unroll
                for (int p = 0; p < PL; ++p) v[p] = load8_nt(col + lrow(p));
            } else {
                load_col16<S, PL>(col + row0, v);
            }
#pragma unroll
            for (int p = 0; p < PL; ++p) acc[p] = add(acc[p], mul(v[p], xj));
        } else {
#pragma unroll
            for (int p = 0; p < PL; ++p)
                if (lrow(p) < a.n) acc[p] = add(acc[p], mul(col[lrow(p)], xj));
        }
    }
#pragma unroll
    for (int p = 0; p < PL; ++p) wpart[w][kSplit ? lane + 64 * p : lane * PL + p] = acc[p];
    __syncthreads();
    // fixed-order wave combine, then publish the chunk partial write-through
    if (threadIdx.x < R) {
        S s = wpart[0][threadIdx.x];
#pragma unroll
        for (int q = 1; q < kWaves; ++q) s = add(s, wpart[q][threadIdx.x]);
        const int64_t row = (int64_t)rt * R + threadIdx.x;
        if (row < a.n) st_agent_s(a.ypart + (int64_t)ch * a.n + row, s);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t tk = __hip_atomic_fetch_add(a.tile_cnt + rt, 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
        s_tile_last = (tk == (uint32_t)a.nchunk - 1) ? 1 : 0;
        if (s_tile_last) __hip_atomic_store(a.tile_cnt + rt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    double n2 = 0.0, rr = 0.0, ri = 0.0;
    if (s_tile_last && threadIdx.x < R) {
        const int64_t row = (int64_t)rt * R + threadIdx.x;
        if (row < a.n) {
            S s = ld_agent_s(a.ypart + row);
            for (int q = 1; q < a.nchunk; ++q) s = add(s, ld_agent_s(a.ypart + (int64_t)q * a.n + row));
            yout[row] = s;
            if constexpr (kPower) {
                const S xi = scale_in(xin[row], nrm);
                n2 = sq_abs(s);
                acc_dot(rr, ri, xi, s);
            }
        }
    }
    if constexpr (kPower) {
        block_sum3(n2, rr, ri, sm);
        last_arriver_reduce(n2, rr, ri, a.blk_part, &a.ctl->counter, a.my_part, sm, &s_last);
    }
}

}  // namespace dev
}  // namespace eigsol

using namespace eigsol;
using namespace eigsol::dev;

namespace eigsol {

void dense_retain(eigsol_dense* A) { A->refs.fetch_add(1); }

void dense_release(eigsol_dense* A) {
    if (!A || A->refs.fetch_sub(1) != 1) return;
    (void)hipSetDevice(A->ctx->device);
    (void)hipStreamSynchronize(A->ctx->stream);
    if (A->ypart) (void)hipFree(A->ypart);
    if (A->tile_cnt) (void)hipFree(A->tile_cnt);
    if (A->a) (void)hipFree(A->a);
    if (A->shadow) dense_release(A->shadow);
    eigsol_ctx* c = A->ctx;
    delete A;
    ctx_release(c);
}

static void dense_layout(const eigsol_dense* A, int& ntr, int& nchunk, int& cw) {
    const int R = 64 * (16 / (int)scalar_bytes(A->dtype));   // DenseTile<S>::kRows
    ntr = (int)((A->nrows + R - 1) / R);
    // ~4 blocks per CU (EIGSOL_DENSE_TARGET overrides).  Round 4 (tools/dense_ab.sh, 16384^2): f64
    // 2048 / 1024 / 512 blocks 0.350 / 0.321 / 0.358 ms, c64 0.368 / 0.349 / 0.324 ms; the 8-byte
    // split-row loads (EIGSOL_DENSE_SPLIT=1, bitwise the same products) 0.343 / 0.337 / 0.316 ms f64
    int64_t target = 1024;
    if (const char* e = std::getenv("EIGSOL_DENSE_TARGET")) target = std::max<int64_t>(8, std::atoll(e));
    int64_t nch = std::max<int64_t>(1, target / std::max(1, ntr));
    nch = std::min<int64_t>(nch, std::max<int64_t>(1, (A->ncols + 15) / 16));
    nchunk = (int)nch;
    cw = (int)((A->ncols + nch - 1) / nch);
}

static int dense_work(eigsol_dense* A) {
    if (A->ypart) return EIGSOL_OK;
    dense_layout(A, A->ntr, A->nchunk, A->cw);
    const size_t sb = scalar_bytes(A->dtype);
    EIGSOL_HIP(hipMalloc(&A->ypart, (size_t)A->nchunk * std::max<int64_t>(1, A->nrows) * sb));
    EIGSOL_HIP(hipMalloc(&A->tile_cnt, sizeof(uint32_t) * std::max(1, A->ntr)));
    EIGSOL_HIP(hipMemsetAsync(A->tile_cnt, 0, sizeof(uint32_t) * std::max(1, A->ntr), A->ctx->stream));
    return EIGSOL_OK;
}

int dense_grid(eigsol_dense* A, int* grid) {
    int ntr, nchunk, cw;
    dense_layout(A, ntr, nchunk, cw);
    *grid = ntr * nchunk;
    return EIGSOL_OK;
}

template <class S>
static int dense_launch_t(eigsol_dense* A, bool power, const void* x, void* y,
                          void* buf0, void* buf1, PowerCtl* ctl, const void* rank_part, int nranks,
                          void* my_part, void* blk_part, void* trace, int parity) {
    DenseArgs<S> a{};
    a.a = (const S*)A->a;
    a.n = A->nrows;
    a.ncols = A->ncols;
    a.ntr = A->ntr;
    a.nchunk = A->nchunk;
    a.cw = A->cw;
    a.ypart = (S*)A->ypart;
    a.tile_cnt = A->tile_cnt;
    a.x_plain = (const S*)x;
    a.y_plain = (S*)y;
    a.buf0 = (S*)buf0;
    a.buf1 = (S*)buf1;
    a.ctl = ctl;
    a.rank_part = (const part4*)rank_part;
    a.nranks = nranks;
    a.my_part = (part4*)my_part;
    a.blk_part = (part4*)blk_part;
    a.trace = (S*)trace;
    const int grid = A->ntr * A->nchunk;
    hipStream_t s = A->ctx->stream;
    // EIGSOL_DENSE_SPLIT=1: the 8-byte split-row loads for 8-byte scalars (A/B)
    static const bool split = [] {
        const char* e = std::getenv("EIGSOL_DENSE_SPLIT");
        return e && std::atoi(e) != 0;
    }();
    if constexpr (sizeof(S) == 8) {
        if (split) {
            if (power)
                hipLaunchKernelGGL((dense_kernel<S, true, true>), dim3(grid), dim3(kThreads), 0, s, a, parity);
            else
                hipLaunchKernelGGL((dense_kernel<S, false, true>), dim3(grid), dim3(kThreads), 0, s, a, parity);
            EIGSOL_HIP(hipGetLastError());
            return EIGSOL_OK;
        }
    }
    if (power)
        hipLaunchKernelGGL((dense_kernel<S, true>), dim3(grid), dim3(kThreads), 0, s, a, parity);
    else
        hipLaunchKernelGGL((dense_kernel<S, false>), dim3(grid), dim3(kThreads), 0, s, a, parity);
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

int dense_power_launch(eigsol_dense* A, void* buf0, void* buf1, PowerCtl* ctl,
                       const void* rank_part, int nranks, void* my_part, void* blk_part,
                       void* trace, int parity, int /*grid*/) {
    EIGSOL_TRY(dense_work(A));
    auto run = [&](auto tag) {
        return dense_launch_t<decltype(tag)>(A, true, nullptr, nullptr, buf0, buf1, ctl, rank_part,
                                             nranks, my_part, blk_part, trace, parity);
    };
    switch (A->dtype) {
        case EIGSOL_C128: return run(cplx{});
        case EIGSOL_F32: return run(0.0f);
        case EIGSOL_C64: return run(cplxf{});
        default: return run(0.0);
    }
}

int wide_dense_gemv(eigsol_dense* A, const void* x, void* y);   // wide.hip

}  // namespace eigsol

extern "C" {

int eigsol_dense_create(eigsol_ctx* ctx, eigsol_dtype dtype, int64_t nrows, int64_t ncols,
                        const void* colmajor, eigsol_dense** out) {
    if (!ctx || !out) return fail(EIGSOL_E_INVALID, "eigsol_dense_create: null ctx/out");
    *out = nullptr;
    if (!dtype_valid(dtype) && !dtype_wide(dtype)) return fail(EIGSOL_E_INVALID, "eigsol_dense_create: unknown dtype");
    if (nrows < 0 || ncols < 0) return fail(EIGSOL_E_INVALID, "eigsol_dense_create: negative dimension");
    if (nrows * ncols > 0 && !colmajor) return fail(EIGSOL_E_INVALID, "eigsol_dense_create: null data");
    EIGSOL_HIP(hipSetDevice(ctx->device));
    const size_t sb = scalar_bytes(dtype);
    auto* A = new eigsol_dense();
    A->ctx = ctx;
    ctx_retain(ctx);
    A->dtype = dtype;
    A->nrows = nrows;
    A->ncols = ncols;
    const size_t bytes = (size_t)std::max<int64_t>(1, nrows * ncols) * sb + 64;
    hipError_t e = hipMalloc(&A->a, bytes);
    if (e == hipSuccess && nrows * ncols > 0)
        e = hipMemcpyAsync(A->a, colmajor, (size_t)nrows * ncols * sb, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
        dense_release(A);
        return fail(EIGSOL_E_HIP, std::string("eigsol_dense_create: ") + hipGetErrorString(e));
    }
    *out = A;
    return EIGSOL_OK;
}

int eigsol_dense_destroy(eigsol_dense* A) {
    dense_release(A);
    return EIGSOL_OK;
}

int eigsol_dense_gemv(eigsol_dense* A, const void* x_dev, void* y_dev) {
    if (!A || (!x_dev && A->ncols) || (!y_dev && A->nrows))
        return fail(EIGSOL_E_INVALID, "eigsol_dense_gemv: null pointer");
    if (A->nrows == 0) return EIGSOL_OK;
    EIGSOL_HIP(hipSetDevice(A->ctx->device));
    if (dtype_wide(A->dtype)) return wide_dense_gemv(A, x_dev, y_dev);
    EIGSOL_TRY(dense_work(A));
    auto run = [&](auto tag) {
        return dense_launch_t<decltype(tag)>(A, false, x_dev, y_dev, nullptr, nullptr, nullptr, nullptr, 1,
                                             nullptr, nullptr, nullptr, 0);
    };
    switch (A->dtype) {
        case EIGSOL_C128: return run(cplx{});
        case EIGSOL_F32: return run(0.0f);
        case EIGSOL_C64: return run(cplxf{});
        default: return run(0.0);
    }
}

}  // extern "C"

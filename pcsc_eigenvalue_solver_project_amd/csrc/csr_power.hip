// Device-resident CSR matrix and the fused power-iteration SpMV for gfx950.
//
// Replaces the numeric core behind powerMethod<S> (src/power_method/power_method.hpp:135-148):
// the two Eigen products per iteration (:69 and :81), y.norm() (:72), x = y/normY (:78), the
// Rayleigh dot (:81) and the is_close_relative test (:83-91, tolerance.hpp:28-33) become ONE
// kernel launch per iteration:
//
//   launch t:  x_t = y_{t-1} / ||y_{t-1}||  (division on the gather, bitwise the reference's x)
//              y_t = A x_t                 (row tiles staged through LDS, CSR-stream)
//              partials ||y_t||^2, x_t^H y_t  -> block partials -> last-arriver rank partial
//              prologue of launch t+1 turns the rank partials into the reference's decisions.
//
// Row tiles: consecutive rows whose nonzeros fit one LDS tile (4096 f64 / 2048 c128 products,
// <= 256 rows).  Phase 1 streams the tile's values/columns coalesced (16 B per lane), gathers x
// and writes the products to LDS; phase 2 gives each row to one lane, which sums its products
// sequentially in ascending column order — exactly the per-row order of the reference's
// Eigen CSC scatter, so every y_i is bitwise the reference's.  Rows longer than a tile get a tile
// of their own and a fixed-order strided block reduction (deterministic, tolerance-checked).
// Tiles are assigned XCD-contiguously (block b serves XCD group b % 8), so neighbouring row
// tiles — which gather overlapping x windows for banded matrices — share one XCD's L2.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <type_traits>
#include <vector>

#include "kernels_common.hpp"

namespace eigsol {
namespace dev {

template <class S> struct Tile;
// kNnz: LDS products per tile; kCap: nonzeros a tile may hold (f64 lanes load aligned pairs, so a
// tile starting at an odd index needs one spare slot).
template <> struct Tile<double> { static constexpr int kNnz = 2048; static constexpr int kCap = kNnz - 1; };
template <> struct Tile<cplx> { static constexpr int kNnz = 1024; static constexpr int kCap = kNnz; };
constexpr int kTileRows = 256;

// One pad element every 32 keeps the lane-per-row phase-2 reads spread over the 64 banks.
__device__ __forceinline__ int lds_idx(int k) { return k + (k >> 5); }

template <class S>
struct CsrArgs {
    const int32_t* rowptr;
    const int32_t* col;
    const S* val;
    const int4* tile_meta;   // per tile {r0, r1, e0, e1}
    int32_t ntiles;
    int32_t nrows;
    const S* x_plain;        // plain SpMV input (kPower == false)
    S* y_plain;              // plain SpMV output
    S* buf0;                 // power: y buffers, launch t reads buf[(t-1)&1], writes buf[t&1]
    S* buf1;
    PowerCtl* ctl;
    const part4* rank_part;
    int32_t nranks;
    part4* my_part;
    part4* blk_part;
    S* trace;
};

// Registers holding one tile's stream for one lane: P slots of (values, columns) plus the lane's
// row pointers.  f64 slots carry a 16-byte pair of values and an 8-byte pair of columns.
template <class S> struct Slot;
template <> struct Slot<double> {
    static constexpr int kNnz = 2;
    double2 v;
    int2 c;
};
template <> struct Slot<cplx> {
    static constexpr int kNnz = 1;
    cplx v;
    int c;
};
template <class S>
struct TileRegs {
    static constexpr int P = Tile<S>::kNnz / (Slot<S>::kNnz * kThreads);
    Slot<S> s[P];
    int rp0, rp1;
};

__device__ __forceinline__ bool short_tile(int4 m, int tn) { return m.w - m.z <= tn; }

// Issue every load of a tile's value/column stream and of the lane's row pointers.
template <class S>
__device__ __forceinline__ void load_tile(const CsrArgs<S>& a, int4 m, TileRegs<S>& R) {
    constexpr int P = TileRegs<S>::P;
    const int tid = threadIdx.x;
    if (short_tile(m, Tile<S>::kCap)) {
        if constexpr (std::is_same_v<S, double>) {
            const int q0 = m.z & ~1;
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const int q = q0 + 2 * (tid + p * kThreads);
                if (q < m.w) {
                    R.s[p].v = *reinterpret_cast<const double2*>(a.val + q);
                    R.s[p].c = *reinterpret_cast<const int2*>(a.col + q);
                }
            }
        } else {
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const int q = m.z + tid + p * kThreads;
                if (q < m.w) {
                    R.s[p].v = a.val[q];
                    R.s[p].c = a.col[q];
                }
            }
        }
    }
    if (tid < m.y - m.x) {
        R.rp0 = a.rowptr[m.x + tid];
        R.rp1 = a.rowptr[m.x + tid + 1];
    }
}

template <class S, bool kPower>
__global__ __launch_bounds__(kThreads) void csr_kernel(CsrArgs<S> a, int parity) {
    constexpr int TN = Tile<S>::kNnz;
    constexpr int P = TileRegs<S>::P;
    constexpr int NPS = Slot<S>::kNnz;
    __shared__ S prod[TN + TN / 32];
    __shared__ double sm[3 * kWaves];
    __shared__ Prologue pro;
    __shared__ int s_last;

    const S* xin;
    S* yout;
    double nrm = 0.0;
    if constexpr (kPower) {
        power_prologue<S>(a.ctl, a.rank_part, a.nranks, parity, a.trace, &pro);
        if (!pro.go) return;
        nrm = pro.nrm;
        xin = parity ? a.buf0 : a.buf1;
        yout = parity ? a.buf1 : a.buf0;
    } else {
        xin = a.x_plain;
        yout = a.y_plain;
    }
    (void)nrm;
    const int tid = threadIdx.x;
    double n2 = 0.0, rr = 0.0, ri = 0.0;

    // XCD-contiguous tile ranges: block b works in group b % 8 on tiles of that group's chunk.
    const int nb = gridDim.x >> 3;
    const int chunk = (a.ntiles + 7) >> 3;
    const int tbeg = (blockIdx.x & 7) * chunk;
    const int tend = min(a.ntiles, tbeg + chunk);
    int t = tbeg + (blockIdx.x >> 3);

    if (t < tend) {
        int4 m = a.tile_meta[t];
        TileRegs<S> R;
        load_tile(a, m, R);
        for (;;) {
            const int tn = t + nb;
            const bool has_next = tn < tend;
            int4 mn = m;
            if (has_next) mn = a.tile_meta[tn];
            const int nr = m.y - m.x;
            if (short_tile(m, Tile<S>::kCap)) {
                // ---- gathers of the current tile, all in flight together
                S xg[P][NPS];
                const int q0 = std::is_same_v<S, double> ? (m.z & ~1) : m.z;
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    const int qb = q0 + NPS * (tid + p * kThreads);
                    if constexpr (std::is_same_v<S, double>) {
                        if (qb >= m.z && qb < m.w) xg[p][0] = xin[R.s[p].c.x];
                        if (qb + 1 < m.w) xg[p][NPS - 1] = xin[R.s[p].c.y];
                    } else {
                        if (qb < m.w) xg[p][0] = xin[R.s[p].c];
                    }
                }
                S xrow = s_zero<S>();
                if (kPower && tid < nr) xrow = xin[m.x + tid];
                // ---- prefetch the next tile's stream while the gathers are in flight
                TileRegs<S> Rn;
                if (has_next) load_tile(a, mn, Rn);
                // ---- products -> LDS
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    const int qb = q0 + NPS * (tid + p * kThreads);
                    if constexpr (std::is_same_v<S, double>) {
                        if (qb >= m.z && qb < m.w) {
                            double xv = xg[p][0];
                            if constexpr (kPower) xv = scale_in(xv, nrm);
                            prod[lds_idx(qb - m.z)] = R.s[p].v.x * xv;
                        }
                        if (qb + 1 < m.w) {
                            double xv = xg[p][NPS - 1];
                            if constexpr (kPower) xv = scale_in(xv, nrm);
                            prod[lds_idx(qb + 1 - m.z)] = R.s[p].v.y * xv;
                        }
                    } else {
                        if (qb < m.w) {
                            S xv = xg[p][0];
                            if constexpr (kPower) xv = scale_in(xv, nrm);
                            prod[lds_idx(qb - m.z)] = mul(R.s[p].v, xv);
                        }
                    }
                }
                __syncthreads();
                // ---- one lane per row: sequential ascending-column sum (reference order)
                if (tid < nr) {
                    const int k0 = R.rp0 - m.z;
                    const int k1 = R.rp1 - m.z;
                    S sacc = s_zero<S>();
                    for (int k = k0; k < k1; ++k) sacc = add(sacc, prod[lds_idx(k)]);
                    yout[m.x + tid] = sacc;
                    if constexpr (kPower) {
                        const S xi = scale_in(xrow, nrm);
                        n2 += sq_abs(sacc);
                        acc_dot(rr, ri, xi, sacc);
                    }
                }
                __syncthreads();
                if (!has_next) break;
                R = Rn;
            } else {
                // ---- long row (m.y == m.x + 1): strided partial sums, fixed-order block reduction
                double pr = 0.0, pi = 0.0, dummy = 0.0;
                for (int q = m.z + tid; q < m.w; q += kThreads) {
                    S xv = xin[a.col[q]];
                    if constexpr (kPower) xv = scale_in(xv, nrm);
                    const S pq = mul(a.val[q], xv);
                    if constexpr (std::is_same_v<S, double>) {
                        pr += pq;
                    } else {
                        pr += pq.re;
                        pi += pq.im;
                    }
                }
                block_sum3(pr, pi, dummy, sm);
                if (tid == 0) {
                    S sacc;
                    set_re_im(sacc, pr, pi);
                    yout[m.x] = sacc;
                    if constexpr (kPower) {
                        const S xi = scale_in(xin[m.x], nrm);
                        n2 += sq_abs(sacc);
                        acc_dot(rr, ri, xi, sacc);
                    }
                }
                if (!has_next) break;
                load_tile(a, mn, R);
            }
            m = mn;
            t = tn;
        }
    }
    if constexpr (kPower) {
        block_sum3(n2, rr, ri, sm);
        last_arriver_reduce(n2, rr, ri, a.blk_part, &a.ctl->counter, a.my_part, sm, &s_last);
    }
}

// ||x||^2 partials of the start vector (x.normalize(), power_method.hpp:62).
template <class S>
__global__ __launch_bounds__(kThreads) void norm_partial_kernel(const S* x, int64_t n, PowerCtl* ctl,
                                                                part4* blk_part, part4* out) {
    __shared__ double sm[3 * kWaves];
    __shared__ int s_last;
    double n2 = 0.0, z1 = 0.0, z2 = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kThreads)
        n2 += sq_abs(x[i]);
    block_sum3(n2, z1, z2, sm);
    last_arriver_reduce(n2, z1, z2, blk_part, &ctl->counter, out, sm, &s_last);
}

// x_out = src / nrm (the reference's x = y / normY of the final iterate; unchanged if nrm == 0).
template <class S>
__global__ __launch_bounds__(kThreads) void scale_out_kernel(const S* src, double nrm, S* dst,
                                                             int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kThreads)
        dst[i] = scale_in(src[i], nrm);
}

}  // namespace dev
}  // namespace eigsol

using namespace eigsol;
using namespace eigsol::dev;

namespace eigsol {

void csr_retain(eigsol_csr* A) { A->refs.fetch_add(1); }

void csr_release(eigsol_csr* A) {
    if (!A || A->refs.fetch_sub(1) != 1) return;
    (void)hipSetDevice(A->ctx->device);
    (void)hipStreamSynchronize(A->ctx->stream);
    if (A->rowptr) (void)hipFree(A->rowptr);
    if (A->col) (void)hipFree(A->col);
    if (A->val) (void)hipFree(A->val);
    if (A->tile_meta) (void)hipFree(A->tile_meta);
    eigsol_ctx* c = A->ctx;
    delete A;
    ctx_release(c);
}

// ---------------------------------------------------------------- host: CSR build / upload
static int build_tiles(const int32_t* rowptr, int64_t nrows, int tile_nnz,
                       std::vector<int32_t>& meta, int32_t& long_tiles, int32_t& max_rows) {
    std::vector<int32_t> starts;
    starts.clear();
    starts.reserve(nrows / 64 + 2);
    long_tiles = 0;
    max_rows = 0;
    int64_t r = 0;
    while (r < nrows) {
        starts.push_back((int32_t)r);
        const int64_t len = rowptr[r + 1] - rowptr[r];
        if (len > tile_nnz) {
            ++long_tiles;
            ++r;
            max_rows = std::max(max_rows, 1);
            continue;
        }
        int64_t nz = len;
        int64_t rr = r + 1;
        while (rr < nrows && rr - r < kTileRows) {
            const int64_t l2 = rowptr[rr + 1] - rowptr[rr];
            if (nz + l2 > tile_nnz) break;
            nz += l2;
            ++rr;
        }
        max_rows = std::max(max_rows, (int32_t)(rr - r));
        r = rr;
    }
    starts.push_back((int32_t)nrows);
    const size_t nt = starts.size() - 1;
    meta.resize(4 * std::max<size_t>(nt, 1));
    for (size_t i = 0; i < nt; ++i) {
        meta[4 * i + 0] = starts[i];
        meta[4 * i + 1] = starts[i + 1];
        meta[4 * i + 2] = rowptr[starts[i]];
        meta[4 * i + 3] = rowptr[starts[i + 1]];
    }
    return (int)nt;
}

int csr_upload(eigsol_ctx* ctx, int dtype, int64_t nrows, int64_t ncols, int64_t nnz,
               const int32_t* rowptr, const int32_t* colidx, const void* values, eigsol_csr** out) {
    const size_t sb = scalar_bytes(dtype);
    // sort columns inside rows when needed (keeps the reference's ascending-column row order)
    std::vector<int32_t> col_sorted;
    std::vector<unsigned char> val_sorted;
    const int32_t* col_use = colidx;
    const void* val_use = values;
    bool sorted = true;
    for (int64_t i = 0; i < nrows && sorted; ++i)
        for (int32_t k = rowptr[i] + 1; k < rowptr[i + 1]; ++k)
            if (colidx[k] < colidx[k - 1]) { sorted = false; break; }
    if (!sorted) {
        col_sorted.assign(colidx, colidx + nnz);
        val_sorted.resize((size_t)nnz * sb);
        std::vector<int32_t> perm;
        for (int64_t i = 0; i < nrows; ++i) {
            const int32_t b = rowptr[i], e = rowptr[i + 1];
            perm.resize(e - b);
            std::iota(perm.begin(), perm.end(), b);
            std::stable_sort(perm.begin(), perm.end(),
                             [&](int32_t x, int32_t y) { return colidx[x] < colidx[y]; });
            for (int32_t k = b; k < e; ++k) {
                col_sorted[k] = colidx[perm[k - b]];
                std::memcpy(&val_sorted[(size_t)k * sb],
                            (const unsigned char*)values + (size_t)perm[k - b] * sb, sb);
            }
        }
        col_use = col_sorted.data();
        val_use = val_sorted.data();
    }
    std::vector<int32_t> meta;
    int32_t long_tiles = 0, max_rows = 0;
    const int ntiles = build_tiles(rowptr, nrows, dtype == EIGSOL_C128 ? Tile<cplx>::kCap : Tile<double>::kCap,
                                   meta, long_tiles, max_rows);

    auto* A = new eigsol_csr();
    A->ctx = ctx;
    ctx_retain(ctx);
    A->dtype = dtype;
    A->nrows = nrows;
    A->ncols = ncols;
    A->nnz = nnz;
    A->ntiles = ntiles;
    A->long_tiles = long_tiles;
    A->max_tile_rows = max_rows;
    const size_t pad = 8;   // 16-byte pair loads may touch one element past nnz
    auto cleanup = [&]() { csr_release(A); };
    hipError_t e;
    if ((e = hipMalloc(&A->rowptr, (nrows + 1) * sizeof(int32_t))) != hipSuccess ||
        (e = hipMalloc(&A->col, (nnz + pad) * sizeof(int32_t))) != hipSuccess ||
        (e = hipMalloc(&A->val, (nnz + pad) * sb)) != hipSuccess ||
        (e = hipMalloc(&A->tile_meta, meta.size() * sizeof(int32_t))) != hipSuccess) {
        cleanup();
        return fail(EIGSOL_E_HIP, std::string("eigsol_csr_create: hipMalloc: ") + hipGetErrorString(e));
    }
    hipStream_t s = ctx->stream;
    if ((e = hipMemsetAsync(A->col, 0, (nnz + pad) * sizeof(int32_t), s)) != hipSuccess ||
        (e = hipMemsetAsync(A->val, 0, (nnz + pad) * sb, s)) != hipSuccess ||
        (e = hipMemcpyAsync(A->rowptr, rowptr, (nrows + 1) * sizeof(int32_t), hipMemcpyHostToDevice, s)) != hipSuccess ||
        (nnz && (e = hipMemcpyAsync(A->col, col_use, nnz * sizeof(int32_t), hipMemcpyHostToDevice, s)) != hipSuccess) ||
        (nnz && (e = hipMemcpyAsync(A->val, val_use, nnz * sb, hipMemcpyHostToDevice, s)) != hipSuccess) ||
        (e = hipMemcpyAsync(A->tile_meta, meta.data(), meta.size() * sizeof(int32_t), hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess) {
        cleanup();
        return fail(EIGSOL_E_HIP, std::string("eigsol_csr_create: upload: ") + hipGetErrorString(e));
    }
    *out = A;
    return EIGSOL_OK;
}

static int validate_compressed(const char* who, int64_t nouter, int64_t ninner, int64_t nnz,
                               const int32_t* ptr, const int32_t* idx) {
    if (nouter < 0 || ninner < 0 || nnz < 0)
        return fail(EIGSOL_E_INVALID, std::string(who) + ": negative dimension");
    if (nnz > INT32_MAX - 16)
        return fail(EIGSOL_E_INVALID, std::string(who) + ": nnz exceeds int32 storage index");
    if (!ptr || (nnz && !idx)) return fail(EIGSOL_E_INVALID, std::string(who) + ": null array");
    if (ptr[0] != 0 || ptr[nouter] != nnz)
        return fail(EIGSOL_E_INVALID, std::string(who) + ": pointer array must start at 0 and end at nnz");
    for (int64_t i = 0; i < nouter; ++i)
        if (ptr[i + 1] < ptr[i])
            return fail(EIGSOL_E_INVALID, std::string(who) + ": pointer array not monotone");
    for (int64_t k = 0; k < nnz; ++k)
        if (idx[k] < 0 || idx[k] >= ninner)
            return fail(EIGSOL_E_INVALID, std::string(who) + ": index out of range");
    return EIGSOL_OK;
}

// ---------------------------------------------------------------- occupancy-derived grid
template <class S>
static int resident_grid(eigsol_ctx* ctx, int64_t ntiles, int* grid) {
    // Residency from the kernel's own resources (MI355X_MICROARCH.md § Register files: waves per
    // SIMD = floor(512 / VGPR allocation), 4 waves per block, 160 KiB LDS per CU).
    hipFuncAttributes fa;
    EIGSOL_HIP(hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(csr_kernel<S, true>)));
    const int vgpr_alloc = std::max(8, ((fa.numRegs + 7) / 8) * 8);
    const int by_vgpr = std::min(8, 512 / vgpr_alloc) * 4 / kWaves;
    const int by_lds = fa.sharedSizeBytes ? (int)(160 * 1024 / fa.sharedSizeBytes) : 8;
    int per_cu = std::max(1, std::min({by_vgpr, by_lds, 8}));
    if (const char* env = std::getenv("EIGSOL_CSR_BLOCKS_PER_CU")) per_cu = std::max(1, std::atoi(env));
    int64_t g = (int64_t)per_cu * ctx->num_cus;
    const int64_t need = ((ntiles + 7) / 8) * 8;
    g = std::min(g, std::max<int64_t>(need, 8));
    g = std::max<int64_t>(8, (g / 8) * 8);
    *grid = (int)g;
    return EIGSOL_OK;
}

int csr_grid(eigsol_csr* A, int* grid) {
    if (A->dtype == EIGSOL_C128) return resident_grid<cplx>(A->ctx, A->ntiles, grid);
    return resident_grid<double>(A->ctx, A->ntiles, grid);
}

template <class S>
static int launch_csr(eigsol_csr* A, const CsrArgs<S>& args, bool power, int parity, int grid) {
    hipStream_t s = A->ctx->stream;
    if (power)
        hipLaunchKernelGGL((csr_kernel<S, true>), dim3(grid), dim3(kThreads), 0, s, args, parity);
    else
        hipLaunchKernelGGL((csr_kernel<S, false>), dim3(grid), dim3(kThreads), 0, s, args, parity);
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

// entry points used by power_session.cpp
int csr_power_launch(eigsol_csr* A, void* buf0, void* buf1, PowerCtl* ctl, const void* rank_part,
                     int nranks, void* my_part, void* blk_part, void* trace, int parity, int grid) {
    if (A->dtype == EIGSOL_C128) {
        CsrArgs<cplx> a{A->rowptr, A->col, (const cplx*)A->val, (const int4*)A->tile_meta, A->ntiles,
                        (int32_t)A->nrows, nullptr, nullptr, (cplx*)buf0, (cplx*)buf1, ctl,
                        (const part4*)rank_part, nranks, (part4*)my_part, (part4*)blk_part,
                        (cplx*)trace};
        return launch_csr<cplx>(A, a, true, parity, grid);
    }
    CsrArgs<double> a{A->rowptr, A->col, (const double*)A->val, (const int4*)A->tile_meta, A->ntiles,
                      (int32_t)A->nrows, nullptr, nullptr, (double*)buf0, (double*)buf1, ctl,
                      (const part4*)rank_part, nranks, (part4*)my_part, (part4*)blk_part,
                      (double*)trace};
    return launch_csr<double>(A, a, true, parity, grid);
}

int norm_partial_launch(eigsol_ctx* ctx, int dtype, const void* x, int64_t n, PowerCtl* ctl,
                        void* blk_part, void* out, int grid) {
    hipStream_t s = ctx->stream;
    if (dtype == EIGSOL_C128)
        hipLaunchKernelGGL(norm_partial_kernel<cplx>, dim3(grid), dim3(kThreads), 0, s,
                           (const cplx*)x, n, ctl, (part4*)blk_part, (part4*)out);
    else
        hipLaunchKernelGGL(norm_partial_kernel<double>, dim3(grid), dim3(kThreads), 0, s,
                           (const double*)x, n, ctl, (part4*)blk_part, (part4*)out);
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

int scale_out_launch(eigsol_ctx* ctx, int dtype, const void* src, double nrm, void* dst, int64_t n) {
    hipStream_t s = ctx->stream;
    const int grid = (int)std::min<int64_t>(4096, std::max<int64_t>(1, (n + kThreads - 1) / kThreads));
    if (dtype == EIGSOL_C128)
        hipLaunchKernelGGL(scale_out_kernel<cplx>, dim3(grid), dim3(kThreads), 0, s, (const cplx*)src,
                           nrm, (cplx*)dst, n);
    else
        hipLaunchKernelGGL(scale_out_kernel<double>, dim3(grid), dim3(kThreads), 0, s,
                           (const double*)src, nrm, (double*)dst, n);
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

}  // namespace eigsol

// ---------------------------------------------------------------- C ABI
extern "C" {

int eigsol_csr_create(eigsol_ctx* ctx, eigsol_dtype dtype, int64_t nrows, int64_t ncols,
                      int64_t nnz, const int32_t* rowptr, const int32_t* colidx,
                      const void* values, eigsol_csr** out) {
    if (!ctx || !out) return fail(EIGSOL_E_INVALID, "eigsol_csr_create: null ctx/out");
    *out = nullptr;
    if (dtype != EIGSOL_F64 && dtype != EIGSOL_C128)
        return fail(EIGSOL_E_INVALID, "eigsol_csr_create: unknown dtype");
    if (nrows > INT32_MAX - 1 || ncols > INT32_MAX - 1)
        return fail(EIGSOL_E_INVALID, "eigsol_csr_create: dimension exceeds int32 storage index");
    EIGSOL_TRY(validate_compressed("eigsol_csr_create", nrows, ncols, nnz, rowptr, colidx));
    if (nnz && !values) return fail(EIGSOL_E_INVALID, "eigsol_csr_create: null values");
    EIGSOL_HIP(hipSetDevice(ctx->device));
    return csr_upload(ctx, dtype, nrows, ncols, nnz, rowptr, colidx, values, out);
}

int eigsol_csr_create_from_csc(eigsol_ctx* ctx, eigsol_dtype dtype, int64_t nrows, int64_t ncols,
                               int64_t nnz, const int32_t* colptr, const int32_t* rowidx,
                               const void* values, eigsol_csr** out) {
    if (!ctx || !out) return fail(EIGSOL_E_INVALID, "eigsol_csr_create_from_csc: null ctx/out");
    *out = nullptr;
    if (dtype != EIGSOL_F64 && dtype != EIGSOL_C128)
        return fail(EIGSOL_E_INVALID, "eigsol_csr_create_from_csc: unknown dtype");
    if (nrows > INT32_MAX - 1 || ncols > INT32_MAX - 1)
        return fail(EIGSOL_E_INVALID, "eigsol_csr_create_from_csc: dimension exceeds int32");
    EIGSOL_TRY(validate_compressed("eigsol_csr_create_from_csc", ncols, nrows, nnz, colptr, rowidx));
    if (nnz && !values) return fail(EIGSOL_E_INVALID, "eigsol_csr_create_from_csc: null values");
    // CSC -> CSR by counting sort; scanning columns in ascending order leaves every row's
    // columns ascending (the reference's CSC scatter order, power_method.hpp:69).
    const size_t sb = scalar_bytes(dtype);
    std::vector<int32_t> rp(nrows + 1, 0), ci(nnz);
    std::vector<unsigned char> v((size_t)nnz * sb);
    for (int64_t k = 0; k < nnz; ++k) rp[rowidx[k] + 1]++;
    for (int64_t i = 0; i < nrows; ++i) rp[i + 1] += rp[i];
    std::vector<int32_t> fill(rp.begin(), rp.end() - 1);
    for (int64_t j = 0; j < ncols; ++j)
        for (int32_t k = colptr[j]; k < colptr[j + 1]; ++k) {
            const int32_t d = fill[rowidx[k]]++;
            ci[d] = (int32_t)j;
            std::memcpy(&v[(size_t)d * sb], (const unsigned char*)values + (size_t)k * sb, sb);
        }
    EIGSOL_HIP(hipSetDevice(ctx->device));
    return csr_upload(ctx, dtype, nrows, ncols, nnz, rp.data(), ci.data(), v.data(), out);
}

int eigsol_csr_destroy(eigsol_csr* A) {
    csr_release(A);
    return EIGSOL_OK;
}

int eigsol_csr_info(eigsol_csr* A, int64_t* nrows, int64_t* ncols, int64_t* nnz, int* dtype) {
    if (!A) return fail(EIGSOL_E_INVALID, "eigsol_csr_info: null matrix");
    if (nrows) *nrows = A->nrows;
    if (ncols) *ncols = A->ncols;
    if (nnz) *nnz = A->nnz;
    if (dtype) *dtype = A->dtype;
    return EIGSOL_OK;
}

int eigsol_csr_spmv(eigsol_csr* A, const void* x_dev, void* y_dev) {
    if (!A || (!x_dev && A->ncols) || (!y_dev && A->nrows))
        return fail(EIGSOL_E_INVALID, "eigsol_csr_spmv: null pointer");
    if (A->nrows == 0) return EIGSOL_OK;
    EIGSOL_HIP(hipSetDevice(A->ctx->device));
    int grid = 8;
    EIGSOL_TRY(csr_grid(A, &grid));
    if (A->dtype == EIGSOL_C128) {
        CsrArgs<cplx> a{};
        a.rowptr = A->rowptr; a.col = A->col; a.val = (const cplx*)A->val; a.tile_meta = (const int4*)A->tile_meta;
        a.ntiles = A->ntiles; a.nrows = (int32_t)A->nrows;
        a.x_plain = (const cplx*)x_dev; a.y_plain = (cplx*)y_dev;
        return launch_csr<cplx>(A, a, false, 0, grid);
    }
    CsrArgs<double> a{};
    a.rowptr = A->rowptr; a.col = A->col; a.val = (const double*)A->val; a.tile_meta = (const int4*)A->tile_meta;
    a.ntiles = A->ntiles; a.nrows = (int32_t)A->nrows;
    a.x_plain = (const double*)x_dev; a.y_plain = (double*)y_dev;
    return launch_csr<double>(A, a, false, 0, grid);
}

}  // extern "C"

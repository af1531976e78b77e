// Internal header of libeigsol_hip.so (gfx950).  Host + device shared definitions.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <string>
#include <type_traits>
#include <vector>

#include "eigsol_hip.h"

struct eigsol_ctx;
struct eigsol_csr;
struct eigsol_dense;

namespace eigsol {

void ctx_retain(eigsol_ctx* c);
void ctx_release(eigsol_ctx* c);
void csr_retain(eigsol_csr* A);
void csr_release(eigsol_csr* A);
void dense_retain(eigsol_dense* A);
void dense_release(eigsol_dense* A);

// ------------------------------------------------------------------ errors
void set_error(const std::string& msg);
int fail(int status, const std::string& msg);

#define EIGSOL_HIP(expr)                                                                 \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess)                                                            \
            return ::eigsol::fail(EIGSOL_E_HIP, std::string(#expr) + ": " +              \
                                                    hipGetErrorString(_e));              \
    } while (0)

// Host wait for a stream inside a host-driven iteration (QR sweeps, GMRES steps):
// hipStreamSynchronize, or with EIGSOL_SYNC_SPIN=1 a busy poll of hipStreamQuery.  Round-4 A/B
// (tools/sync_ab.sh): QR 4096^2 real 1.187 / 1.208 s, complex 2.77 / 2.58 s, GMRES 1M 9.11 / 9.20
// ms per iteration (sync / spin) - within the run-to-run spread, so the default does not spin.
hipError_t stream_wait(hipStream_t st);

#define EIGSOL_TRY(expr)                  \
    do {                                  \
        int _s = (expr);                  \
        if (_s != EIGSOL_OK) return _s;   \
    } while (0)

// ------------------------------------------------------------------ scalars
// Complex values are (re, im) pairs, aligned to their size so one lane loads one value with a
// single 16-byte (cplx) or 8-byte (cplxf) load.  Arithmetic mirrors what g++ emits for
// std::complex<T> in the reference: products (ac-bd, ad+bc) with separate roundings (no FMA
// contraction: see the kernels' pragma).  float / cplxf are the reference's float and
// std::complex<float> instantiations (ScalarConcept, types.hpp:28-30): stored and multiplied in
// single precision; norm and Rayleigh partial sums accumulate in double (every single-precision
// square and product is exact in double).
struct alignas(16) cplx {
    double re, im;
};
struct alignas(8) cplxf {
    float re, im;
};

__host__ __device__ inline double sq_abs(double a) { return a * a; }
__host__ __device__ inline double sq_abs(cplx a) { return a.re * a.re + a.im * a.im; }
__host__ __device__ inline double sq_abs(float a) { return (double)a * (double)a; }
__host__ __device__ inline double sq_abs(cplxf a) {
    return (double)a.re * (double)a.re + (double)a.im * (double)a.im;
}

template <class S> __host__ __device__ inline S s_zero();
template <> __host__ __device__ inline double s_zero<double>() { return 0.0; }
template <> __host__ __device__ inline cplx s_zero<cplx>() { return cplx{0.0, 0.0}; }
template <> __host__ __device__ inline float s_zero<float>() { return 0.0f; }
template <> __host__ __device__ inline cplxf s_zero<cplxf>() { return cplxf{0.0f, 0.0f}; }

template <class S> struct dtype_of;
template <> struct dtype_of<double> { static constexpr int value = EIGSOL_F64; };
template <> struct dtype_of<cplx> { static constexpr int value = EIGSOL_C128; };
template <> struct dtype_of<float> { static constexpr int value = EIGSOL_F32; };
template <> struct dtype_of<cplxf> { static constexpr int value = EIGSOL_C64; };

// real scalars are packed in lane pairs by the sliced layout; complex ones one per lane
template <class S> inline constexpr bool is_real_v = std::is_same_v<S, double> || std::is_same_v<S, float>;
template <class S> inline constexpr bool is_cplx_v = !is_real_v<S>;

inline bool dtype_complex(int dtype) { return dtype == EIGSOL_C128 || dtype == EIGSOL_C64 || dtype == EIGSOL_CDD; }
inline bool dtype_single(int dtype) { return dtype == EIGSOL_F32 || dtype == EIGSOL_C64; }
// the fp64 / fp32 kernel families (every layout, factor and QR kernel); EIGSOL_DD / EIGSOL_CDD
// (long double carried as double-double) have their own kernels in wide.hip
inline bool dtype_valid(int dtype) { return dtype >= EIGSOL_F64 && dtype <= EIGSOL_C64; }
inline bool dtype_wide(int dtype) { return dtype == EIGSOL_DD || dtype == EIGSOL_CDD; }
inline size_t scalar_bytes(int dtype) {
    return dtype == EIGSOL_CDD ? 32 : (dtype == EIGSOL_C128 || dtype == EIGSOL_DD) ? 16 : dtype == EIGSOL_F32 ? 4 : 8;
}
// (re, im) in double -> one scalar of `dtype` at dst (results, traces, shifts)
inline void store_scalar(void* dst, int dtype, double re, double im) {
    switch (dtype) {
        case EIGSOL_F64: *static_cast<double*>(dst) = re; break;
        case EIGSOL_C128: static_cast<double*>(dst)[0] = re; static_cast<double*>(dst)[1] = im; break;
        case EIGSOL_F32: *static_cast<float*>(dst) = (float)re; break;
        default: static_cast<float*>(dst)[0] = (float)re; static_cast<float*>(dst)[1] = (float)im; break;
    }
}
inline void load_scalar(const void* src, int dtype, double& re, double& im) {
    im = 0.0;
    switch (dtype) {
        case EIGSOL_F64: re = *static_cast<const double*>(src); break;
        case EIGSOL_C128: re = static_cast<const double*>(src)[0]; im = static_cast<const double*>(src)[1]; break;
        case EIGSOL_F32: re = *static_cast<const float*>(src); break;
        default: re = static_cast<const float*>(src)[0]; im = static_cast<const float*>(src)[1]; break;
    }
}

// ------------------------------------------------------------------ power-iteration state
// Carried state, double-buffered by launch parity (launch with parity p reads st[p], writes st[p^1]).
struct alignas(16) PowerCarry {
    double rho_re, rho_im;   // Rayleigh quotient of x_{t-1}  (rho_{t-1})
    double nrm;              // ||y_{t-1}||  (norm of the launch's input vector)
    int32_t t;               // launch index that wrote this record
    int32_t pad;
};

// Device-resident control block of a session (zeroed / initialised by begin()).
struct alignas(64) PowerCtl {
    int32_t done;            // monotonic: set by block 0 of the launch that ends the reference loop
    uint32_t counter;        // last-arriver ticket for the block-partial reduction
    int32_t max_iter;
    int32_t trace_cap;
    double tol;
    int32_t nranks;
    int32_t ntrace;          // eigenvalue estimates completed so far (trace entries written)
    // result record (valid once done)
    double lam_re, lam_im;
    double final_norm;       // x_final = B[final_parity] / final_norm
    int32_t iters;
    int32_t converged;
    int32_t final_parity;
    int32_t launches;        // launches that passed the done-check (diagnostic)
    int32_t fault;           // row-sharded peer exchange: a wait for a peer timed out (host raises)
    int32_t pad_;
    PowerCarry st[2];
};

// Reference termination logic of powerMethodImpl (power_method.hpp:68-96) evaluated by the fused
// device loop.  Launch t computes y_t = A x_t with x_t = y_{t-1}/||y_{t-1}|| (y_{-1} = x0) and the
// partials of ||y_t||^2 and x_t^H y_t.  Its prologue therefore knows rho_{t-1} = x_{t-1}^H y_{t-1}
// (the reference's lambdaNew of iteration k = t-2, :81) and ||y_{t-1}|| (the normY of iteration
// k' = t-1, :72).  Identical on host and device, and evaluated redundantly by every block.
struct PowerDecision {
    bool done = false;
    bool converged = false;
    bool record = false;     // lambda_k completed: trace[k] = lam
    int32_t iters = 0;
    int32_t k = 0;
    double lam_re = 0.0, lam_im = 0.0;
};

__host__ __device__ inline double cabs_(double re, double im) {
#ifdef __HIP_DEVICE_COMPILE__
    return hypot(re, im);
#else
    return std::hypot(re, im);
#endif
}

// modulus that does not underflow where sq_abs does (|a| below ~1e-162 squares to 0): pivot
// searches and zero-pivot tests (the ordering is sq_abs's, up to rounding)
__host__ __device__ inline double mod_abs(double a) { return a < 0 ? -a : a; }
__host__ __device__ inline double mod_abs(cplx a) { return cabs_(a.re, a.im); }

// tolerance.hpp:28-33: |a - b| <= tol * (1 + |a|), a = lambdaNew (power_method.hpp:84).
__host__ __device__ inline bool close_rel(double are, double aim, double bre, double bim,
                                          double tol, bool is_complex) {
    const double dre = are - bre, dim = aim - bim;
    const double diff = is_complex ? cabs_(dre, dim) : (dre < 0 ? -dre : dre);
    const double scale = 1.0 + (is_complex ? cabs_(are, aim) : (are < 0 ? -are : are));
    return diff <= tol * scale;
}

__host__ __device__ inline PowerDecision power_decide(int32_t t, int32_t max_iter, double tol,
                                                      bool is_complex, double nrm_tm1,
                                                      double rho_tm1_re, double rho_tm1_im,
                                                      double rho_tm2_re, double rho_tm2_im) {
    PowerDecision d;
    if (t >= 2) {
        const int32_t k = t - 2;                 // reference iteration completing now
        d.record = true;
        d.k = k;
        d.lam_re = rho_tm1_re;
        d.lam_im = rho_tm1_im;
        if (k >= 1 && close_rel(rho_tm1_re, rho_tm1_im, rho_tm2_re, rho_tm2_im, tol, is_complex)) {
            d.done = true;                        // :83-90
            d.converged = true;
            d.iters = k + 1;
            return d;
        }
        if (k + 1 >= max_iter) {                  // loop bound :68
            d.done = true;
            d.iters = k + 1;
            return d;
        }
    }
    if (t >= 1 && nrm_tm1 == 0.0) {               // normY == 0 :73-76 (iteration k' = t-1)
        d.done = true;
        d.iters = t;
        if (t < 2) { d.lam_re = 0.0; d.lam_im = 0.0; }
        return d;
    }
    return d;
}

}  // namespace eigsol

// ------------------------------------------------------------------ opaque handle bodies
// Handles are reference counted: a matrix retains its context and a session retains its matrix,
// so destroying them in any order (e.g. from garbage-collected bindings) is safe.
struct eigsol_ctx {
    std::atomic<int> refs{1};
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;   // active stream (own or caller's)
    int num_cus = 256;
    // distributed (filled by eigsol_dist_* when a communicator is attached)
    void* comm = nullptr;
    void* loop = nullptr;   // in-process loopback world (tests: several ranks on one device), else null
    // host-collective bootstrap (eigsol_ctx_create_dist_host): the caller's all-gather of host
    // bytes, used for setup only; the per-iteration exchange then runs device to device
    eigsol_allgather_fn hcoll = nullptr;
    void* hcoll_user = nullptr;
    int rank = 0;
    int nranks = 1;
};

struct eigsol_csr {
    std::atomic<int> refs{1};
    eigsol_ctx* ctx = nullptr;
    int dtype = EIGSOL_F64;
    int64_t nrows = 0, ncols = 0, nnz = 0;
    int32_t* rowptr = nullptr;     // device, nrows+1
    int32_t* col = nullptr;        // device, nnz (+pad)
    uint16_t* col16 = nullptr;     // device, nnz (+pad): windowed tiles' column - window start
    void* val = nullptr;           // device, nnz (+pad)
    int32_t* tile_meta = nullptr;  // device, 4 ints per row tile: {r0, r1, e0, e1}
    int32_t* tile_win = nullptr;   // device, 2 ints per short tile: x window [w0, w1]
    int32_t windowed = 0;          // every short tile's window fits LDS: windowed kernel
    int32_t ntiles = 0;
    int32_t max_tile_rows = 0;
    int32_t nshort = 0;            // tiles [0, nshort) are short; the rest hold one long row each
    // sliced layout (csr_slice_kernel, preferred when every row has <= 64 entries)
    int32_t sliced = 0;
    int32_t nslices = 0;
    int32_t* slice_meta = nullptr; // device, 4 ints per slice
    void* sval = nullptr;          // device, 64 * K_s entries per slice
    uint32_t* scol8 = nullptr;     // device (window slices): 8-bit offsets, 4 per lane-dword
    int32_t slice_kb = 16;         // entries per row held in registers (kernel instantiation)
    int32_t slice_gather = 0;      // some slices gather x from global memory (kernel instantiation)
    int32_t* scol32 = nullptr;     // device (gather slices)
    uint8_t* slen = nullptr;       // device, per row (ragged slices)
    int32_t nseg = 1;              // stream segments (see kSliceSegShift): element offsets of each
    int64_t seg_val[16] = {0}, seg_c8[16] = {0}, seg_c32[16] = {0};
    // Row-sharded (multi-GPU) layout: this rank owns global rows [row_begin, row_begin + nrows);
    // local columns are [own rows | ghosts grouped by owner rank, ascending global index].
    int dist = 0;
    int64_t n_global = 0, row_begin = 0, nghost = 0;
    int64_t xoff = 0;              // x-space index of local row 0 (= ghosts owned by lower ranks)
    std::vector<int64_t> send_counts, send_offs, recv_counts, recv_offs;   // per peer (scalars)
    int exchange = 0;              // EIGSOL_EXCHANGE_HALO / _ALLGATHER
    std::vector<int64_t> row_begins;   // all ranks' row blocks (all-gather exchange)
    int32_t* send_idx = nullptr;   // device: local row of every entry sent, grouped by peer
    void* send_buf = nullptr;      // device: packed halo values
    int64_t nsend = 0;
    std::vector<int32_t> h_send_idx;     // host copy of send_idx (x-space slots of own rows)
    std::vector<int64_t> peer_dst_off;   // per peer q: where my rows start in q's ghost list
    std::vector<int64_t> ghost_counts;   // P x P: [r * P + q] = entries rank r reads from rank q
    std::vector<int64_t> requests;       // global rows the peers read from this rank (by peer)
    // Column blocks (gathered x larger than an XCD's L2): B sub-matrices holding the entries of
    // columns [c_b, c_{b+1}), all rows, tile layout; a product is B passes of csr_kernel, each
    // adding its block's entries to the row partials of the previous pass (the ascending-column
    // order of every row sum is kept), the last with the fused power epilogue.  Empty: off.
    std::vector<eigsol_csr*> cblk;
    // Column-binned layout (csr_bin_kernel; preferred over cblk where it is built): chunks of
    // kBinRows rows, entries ordered (column block, level, row), packed (row << bcbits | column).
    int32_t binned = 0;            // 0: not built; else KB of LDS row sums (kernel instantiation)
    int32_t bin_nt = 256;          // threads per workgroup (kernel instantiation)
    int32_t bin_rows = 0;          // rows per chunk (<= the instantiation's LDS row sums)
    int32_t nchunks = 0, bcbits = 0, nbsteps = 0;
    uint32_t* bpk = nullptr;
    void* bval = nullptr;
    int32_t* bstep = nullptr;      // 4 ints per step
    int32_t* blev = nullptr;       // 2 ints per level
    int32_t* bchunk = nullptr;     // nchunks + 1
    // extended precision (EIGSOL_DD / EIGSOL_CDD, wide.hip): plain CSR in rowptr / col / val (dd
    // values), plus the matrix rounded to fp64 for the shifted solves' factor (built on first use)
    eigsol_csr* shadow = nullptr;
};

struct eigsol_dense {
    std::atomic<int> refs{1};
    eigsol_ctx* ctx = nullptr;
    int dtype = EIGSOL_F64;
    int64_t nrows = 0, ncols = 0;
    void* a = nullptr;             // device, column-major, leading dimension nrows
    // GEMV workspace (allocated on first use): per-chunk row partials and per-tile tickets
    void* ypart = nullptr;
    uint32_t* tile_cnt = nullptr;
    int ntr = 0, nchunk = 1, cw = 1;
    eigsol_dense* shadow = nullptr;   // extended precision: the matrix rounded to fp64 (see eigsol_csr)
};

// Shifted inverse iteration and solve_shifted on gfx950: factor once, solve per iteration.
//
// Replaces the numeric core of shiftedInversePowerMethod<S>
// (src/power_method/shifted_inverse_power_solver.hpp:112-125, impl :21-79) and solve_shifted<S>
// (src/matrix/solve_shifted.hpp:48-118).  The reference refactors A - sigma I on every iteration
// (SparseLU with COLAMD, or dense PartialPivLU); the factorisation does not depend on the
// iterate, so the device path factors once per (A, sigma) and runs ONE solve launch per
// iteration.  The Rayleigh quotient on A (:62) needs no product with A:
// A y = x + sigma y, see shift_prologue (kernels_common.hpp).
//
// Factor kinds
//   * triangular CSR (upper or lower; config 5): the factor IS the matrix.  Pivots d_i - sigma
//     (coeffRef inserts a missing diagonal, solve_shifted.hpp:100-102), rows ordered by dependency
//     level, and a sync-free triangular solve: each 16-lane group solves one row, polling the
//     solved values of the rows it reads (an unsolved value is a sentinel NaN).
//   * dense (Matrix::Dense, and small non-triangular sparse matrices densified on the device):
//     right-looking blocked partial-pivot LU (panels of 64 real / 32 complex columns, trailing
//     update on the fp64 matrix cores; Eigen's PartialPivLU is blocked too), then a
//     single-workgroup forward/back substitution per iteration with the vector in LDS.
// Non-triangular sparse matrices too large to densify are reported as EIGSOL_E_UNSUPPORTED.
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "band_lu.hpp"
#include "kernels_common.hpp"
#include "mfma_rankk.hpp"

namespace eigsol {

struct GmresSolver;
// Adev: the device matrix A itself (same dtype and order), used for the products with M = A - sigma I
int gmres_create(eigsol_ctx* ctx, int dtype, int64_t n, const int32_t* rp, const int32_t* ci, const void* v,
                 double sre, double sim, GmresSolver** out, eigsol_csr* Adev = nullptr);
void gmres_free(GmresSolver* g);
int gmres_solve(GmresSolver* g, const void* b_dev, double bdiv, void* y_dev, const double* guess = nullptr);
int gmres_can_lag(const GmresSolver* g);
int gmres_solve_lag(GmresSolver* g, const void* b_dev, double bdiv, void* y_dev);
int gmres_lag_verdict(GmresSolver* g);
void gmres_lag_reset(GmresSolver* g);
void gmres_info(const GmresSolver* g, double* bytes, int32_t* steps);
int gmres_complete(const GmresSolver* g);

namespace dev {
constexpr int kMaxMulti = 4;      // solves per multi-solve launch (one head wave each)
}
static constexpr int kMultiDefault = 4;   // EIGSOL_TRSV_MULTI (config 5 per iteration: K = 1 0.674, 2 0.502, 3 0.439, 4 0.414 ms)

constexpr size_t kPinBytes = 256;   // ShiftFactor::hpin

struct ShiftFactor {
    eigsol_ctx* ctx = nullptr;
    int dtype = EIGSOL_F64;
    int64_t n = 0;
    int kind = 0;                 // 0 triangular CSR, 1 dense LU, 2 ILU(0)-preconditioned GMRES, 3 band LU
    GmresSolver* gm = nullptr;    // kind 2 (gmres.hip)
    bool lag_prev = false;        // kind 2 iteration: the previous launch's solve check is still to be read
    double lag_bdiv = 0.0;        // ... and that solve's divisor (||y_{t-1}||)
    void* promo = nullptr;        // kind 2 in single precision: [2][n] double-precision right-hand side and
                                  // solution of the GMRES family's solve (its factors are built in double)
    BandFactor* band = nullptr;   // kind 3 (band_lu.hip)
    void* hpin = nullptr;         // pinned host scratch for per-solve readbacks (pageable copies sleep ~1 ms)
    eigsol_csr* src = nullptr;    // kind 2: A, retained for the densified-LU fallback
    int fell_back = 0;            // kind 1 reached through the GMRES fallback
    double sig_re = 0.0, sig_im = 0.0;
    // triangular: everything indexed by solve position (rows sorted by level, levels padded)
    int upper = 1;
    int64_t nnz_total = 0;        // nonzeros of A (diagonal included), for roofline accounting
    int64_t nnz_off = 0;
    int32_t* order = nullptr;     // head position -> row (-1: level padding)
    void* z[2] = {nullptr, nullptr};   // solve values polled by readers; sentinel = not yet solved
    int32_t npos = 0, nchunks = 0, nlevels = 0;
    void* hval = nullptr;         // head, pass-major entries / columns / pivots
    int32_t* hcol = nullptr;
    void* hpiv = nullptr;
    int2* passes = nullptr;       // head passes {first position, end | barrier}
    int32_t npass = 0, hpos = 0, hlevels = 0;
    int wave_head = 1;            // head kernel: 1 one-wave (sptrsv_whead_kernel), 0 one workgroup
    void* wval = nullptr;         // one-wave head, pass-major (see sptrsv_whead_kernel)
    int32_t* wcol = nullptr;
    void* wrp = nullptr;
    int32_t* wdst = nullptr;
    int32_t nwpass = 0;
    int red_grid = 0;             // blocks of the partials reduction
    int2* smeta = nullptr;        // tail slices (see sptrsv_slice_kernel)
    int32_t* trow = nullptr;
    void* tpiv = nullptr;
    int32_t* tcol = nullptr;
    void* tval = nullptr;
    int32_t nslices = 0;
    int slice_b = 16;             // entries per lane held in registers (4, 8 or 16)
    int tail_chunks = 0;          // tail variant: 1 chunk kernel, 0 slice kernel
    int chunk_two = 0;            // chunk kernel with two entries per lane (tail rows longer than 16)
    int32_t* porder = nullptr;    // chunk variant (see sptrsv_chunk_kernel)
    int32_t* pptr = nullptr;
    int32_t* pcol = nullptr;
    void* pval = nullptr;
    void* ppiv = nullptr;
    int32_t chunk0 = 0;
    // tail polls without back-off (EIGSOL_TRSV_POLL_FAST, low 16 bits) and the back-off schedule
    // (EIGSOL_TRSV_POLL_SLOW, bits 16-18; poll_backoff).  Round 6 (tools/r06_trsv_backoff_ab.sh,
    // profiles/r06_trsv_backoff_ab.log, config 5 at K = 4): sleeps of 2 / 8 / 32 x 64 cycles
    // (growing with the spins) 0.4127-0.4134 ms per iteration; a constant 4 / 6 / 8 / 12 / 16:
    // 0.4072-0.4083 (the long sleeps woke late); 32: 0.415.  Default: a constant 8
    int poll_fast = 4 << 16;
    int poll_mode = 2;            // EIGSOL_TRSV_POLL_MODE (bit 0: slice tail, one re-poll per lane; bit 1: chunk tails, the second chunk's first polls after the first chunk: config 5 0.698 -> 0.674 ms, K = 4 0.419 -> 0.414)
    // multi-solve launches (sptrsv_chunk_role_kernel; EIGSOL_TRSV_MULTI=K, 1 disables): K reference
    // iterations per launch, solve j one dependency round behind solve j - 1
    int multi = 1;
    int grid_multi = 0;
    int hconc = 0;                // multi head: every solve's values fit the LDS (sptrsv_whead_kernel)
    void* aux[dev::kMaxMulti - 1] = {};           // w_0 .. w_{K-2} (n scalars each)
    void* zm[dev::kMaxMulti][2] = {};             // solve j >= 1: polled values (zm[0] unused: z)
    int32_t epoch_m = 0;
    void* kpart = nullptr;        // part4 per solve j >= 1: {||w_j||^2, w_{j-1}^H w_j}
    void* kblk = nullptr;         // part4 per block of those reductions
    uint32_t* work = nullptr;     // [2]: last-arriver ticket of the partials reduction
    int32_t* err = nullptr;
    void* wave_part = nullptr;    // part4 per wave
    int32_t epoch = 0;
    int grid = 0;
    // dense
    void* lu = nullptr;           // column-major n x n, L (unit) below, U on and above the diagonal
    int32_t* perm = nullptr;      // P b: b_perm[i] = b[perm[i]]
    int32_t* zero_pivot = nullptr;
    size_t lds_bytes = 0;
    // dense, multi-CU substitution (large n): epoch flags per block row, forward results
    int dense_multi = 0;
    int32_t* flag_f = nullptr;
    int32_t* flag_b = nullptr;
    void* zf = nullptr;
    void* tinv = nullptr;         // [nblk][2] inverted diagonal blocks inv(L_kk), inv(U_kk), 64 x 64 column-major
    void* tmul = nullptr;         // [nblk][2] premultiplied next-to-diagonal tiles (dense_tmul_kernel)
    int dense_v = 2;              // substitution kernel: 2 = dense_trsv2_kernel, 1 = dense_trsv_kernel (EIGSOL_DENSE_TRSV=1)
};

namespace dev {

#ifndef EIGSOL_TRSV_ROW_LANES
#define EIGSOL_TRSV_ROW_LANES 16
#endif
constexpr int kRowLanes = EIGSOL_TRSV_ROW_LANES;   // lanes per row: one row per 16-lane group
constexpr int kWaveRows = 64 / kRowLanes;          // positions per wave round (one chunk): levels are padded to this
constexpr int kSpinLimit = 1 << 20;   // polls (with back-off) before the wait is declared broken
// An unsolved entry of z holds this NaN in every 8-byte word.  A solved value never does: the
// producer maps it to the default quiet NaN (sanitize), so the value itself is the ready flag.
constexpr unsigned long long kSent = 0x7FF4DEAD7FF4DEADull;

template <class S>
struct TriArgs {
    const int32_t* order;  // head position -> row
    const S* hval;         // head, pass-major: entry k of group g of pass q at (q * 64 + g) * 16 + k
    const int32_t* hcol;   // LDS position of the column (padding: the zero slot hpos)
    const S* hpiv;         // pivot of group g of pass q at q * 64 + g
    const int2* passes;    // head passes
    int32_t npass, hpos;   // head passes, head positions
    const S* wval;         // one-wave head: entry k of lane l of pass q at (q * 4 + k) * 64 + l
    const int32_t* wcol;   // its LDS column position (padding: the zero slot hpos)
    const S* wrp;          // 1 / pivot of row group g of pass q at q * 16 + g
    const int32_t* wdst;   // LDS position that group g of pass q solves (-1: none)
    int32_t nwpass;
    const int2* smeta;     // tail slices: {entry offset, entries per lane}
    const int32_t* trow;   // row of lane l of slice s at s * 64 + l (-1: padding)
    const S* tpiv;
    const int32_t* tcol;   // entry k of lane l of slice s at off + 64 k + l (padding: the zero slot n)
    const S* tval;
    int32_t nslices;
    const int32_t* porder; // chunk variant, position-indexed: row (-1: padding), entries, pivots
    const int32_t* pptr;
    const int32_t* pcol;
    const S* pval;
    const S* ppiv;
    int32_t chunk0, nchunks;
    int32_t poll_fast;     // tail: polls re-issued without back-off
    int32_t poll_mode;     // bit 0: slice tail re-polls one dependency per lane; bit 1: late second-chunk polls
    int64_t n;
    S* zcur;            // polled by this launch
    S* znext;           // reset to the sentinel by this launch, for the next one
    uint32_t* work;
    int32_t* err;
    part4* wave_part;
    const S* b_plain;   // solve mode
    S* y_plain;
    S* buf0;            // iteration mode (same parity convention as the power loop)
    S* buf1;
    PowerCtl* ctl;
    const part4* rank_part;
    part4* my_part;
    S* trace;
    double sig_re, sig_im;
    // multi-solve launches (K solves; solve 0 polls zcur)
    int32_t K;
    S* zk[kMaxMulti];   // solve j's polled values (zk[0] = zcur)
    S* zkn[kMaxMulti];  // ... and the next launch's buffers (zkn[0] = znext)
    S* aux[kMaxMulti - 1];   // w_0 .. w_{K-2}
    part4* kpart;       // solves 1..K-1: {||w_j||^2, w_{j-1}^H w_j}
    part4* kblk;        // (K - 1) x red_grid block partials
    int32_t hconc;      // multi head: the K solves concurrently (K LDS value arrays)
};

// multiplication by an exact power of two (the pair launch's scaling of w1)
__device__ __forceinline__ double scale_r(double v, double s) { return v * s; }
__device__ __forceinline__ cplx scale_r(cplx v, double s) { return cplx{v.re * s, v.im * s}; }
__device__ __forceinline__ float scale_r(float v, double s) { return v * (float)s; }
__device__ __forceinline__ cplxf scale_r(cplxf v, double s) { return cplxf{v.re * (float)s, v.im * (float)s}; }

__device__ __forceinline__ void st_coh(double* p, double v) { st_agent(p, v); }
__device__ __forceinline__ void st_coh(cplx* p, cplx v) {
    st_agent(&p->re, v.re);
    st_agent(&p->im, v.im);
}
__device__ __forceinline__ void st_coh(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_coh(cplxf* p, cplxf v) {
    st_coh(&p->re, v.re);
    st_coh(&p->im, v.im);
}
__device__ __forceinline__ float ld_coh(const float* p) {
    return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ cplxf ld_coh(const cplxf* p) { return cplxf{ld_coh(&p->re), ld_coh(&p->im)}; }
__device__ __forceinline__ double ld_coh(const double* p) { return ld_agent(p); }
__device__ __forceinline__ cplx ld_coh(const cplx* p) { return cplx{ld_agent(&p->re), ld_agent(&p->im)}; }

// Indexed coherent access to a solve buffer (uniform base, element index): complex values move as
// ONE device-coherent (sc1) buffer load / store of 16 (8) bytes instead of two 8 (4) byte atomics,
// which halves the dependency polls' memory requests.  A torn read (one half still the sentinel)
// is simply unready: both halves are checked.  Buffer offsets are 32-bit (solve buffers < 4 GiB).
constexpr int kBufSc1 = 16;   // buffer cache policy: sc1 (device scope), as the agent-scope atomics use
__device__ __forceinline__ __amdgpu_buffer_rsrc_t coh_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, -1, 0x00020000);
}
template <class S>
__device__ __forceinline__ S ld_cohi(const S* base, int j) {
    if constexpr (std::is_same_v<S, cplx>) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(coh_rsrc(base), (uint32_t)j * 16u, 0, kBufSc1);
        return __builtin_bit_cast(cplx, v);
    } else if constexpr (std::is_same_v<S, cplxf>) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(coh_rsrc(base), (uint32_t)j * 8u, 0, kBufSc1);
        return __builtin_bit_cast(cplxf, v);
    } else {
        return ld_coh(base + j);
    }
}
template <class S>
__device__ __forceinline__ void st_cohi(S* base, int i, S v) {
    if constexpr (std::is_same_v<S, cplx>) {
        typedef unsigned int u4 __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), coh_rsrc(base), (uint32_t)i * 16u, 0,
                                               kBufSc1);
    } else if constexpr (std::is_same_v<S, cplxf>) {
        typedef unsigned int u2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), coh_rsrc(base), (uint32_t)i * 8u, 0,
                                              kBufSc1);
    } else {
        st_coh(base + i, v);
    }
}

__device__ __forceinline__ int ld_flag_err(const int32_t* p) {
    return __hip_atomic_load(const_cast<int32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool unready(double v) { return (unsigned long long)__double_as_longlong(v) == kSent; }
__device__ __forceinline__ bool unready(cplx v) { return unready(v.re) || unready(v.im); }
// single precision: every 32-bit word of an unsolved entry holds the low word of kSent (a NaN)
__device__ __forceinline__ bool unready(float v) { return __float_as_uint(v) == (uint32_t)(kSent & 0xffffffffu); }
__device__ __forceinline__ bool unready(cplxf v) { return unready(v.re) || unready(v.im); }
__device__ __forceinline__ double sanitize(double v) {
    return unready(v) ? __longlong_as_double(0x7FF8000000000000ll) : v;
}
__device__ __forceinline__ cplx sanitize(cplx v) { return cplx{sanitize(v.re), sanitize(v.im)}; }
__device__ __forceinline__ float sanitize(float v) { return unready(v) ? __uint_as_float(0x7FC00000u) : v; }
__device__ __forceinline__ cplxf sanitize(cplxf v) { return cplxf{sanitize(v.re), sanitize(v.im)}; }
template <class S>
__device__ __forceinline__ S sentinel() {
    const double s = __longlong_as_double((long long)kSent);
    const float sf = __uint_as_float((uint32_t)(kSent & 0xffffffffu));
    if constexpr (std::is_same_v<S, double>) return s;
    else if constexpr (std::is_same_v<S, cplx>) return cplx{s, s};
    else if constexpr (std::is_same_v<S, float>) return sf;
    else return cplxf{sf, sf};
}
template <class S>
__device__ __forceinline__ S s_one() {
    if constexpr (std::is_same_v<S, double>) return 1.0;
    else if constexpr (std::is_same_v<S, cplx>) return cplx{1.0, 0.0};
    else if constexpr (std::is_same_v<S, float>) return 1.0f;
    else return cplxf{1.0f, 0.0f};
}

// sum over the 16 lanes of a row group.  16 lanes: a DPP butterfly over the lane-index xor
// masks 15 (row_mirror), 7 (row_half_mirror), 3 and 1 (quad_perm), which span all 16 lanes:
// four VALU steps instead of four LDS-latency ds_bpermute round trips, and every lane of the
// group ends with the same bits (each step adds the same two values in both lanes).
template <int kCtrl>
__device__ __forceinline__ double dpp_f64(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), kCtrl, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), kCtrl, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
template <int kCtrl>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), kCtrl, 0xf, 0xf, false));
}
constexpr int kDppRowMirror = 0x140, kDppRowHalfMirror = 0x141, kDppQuad3210 = 0x1B, kDppQuad1032 = 0xB1;
__device__ __forceinline__ double group_sum(double v) {
    if constexpr (kRowLanes == 16) {
        v += dpp_f64<kDppRowMirror>(v);
        v += dpp_f64<kDppRowHalfMirror>(v);
        v += dpp_f64<kDppQuad3210>(v);
        v += dpp_f64<kDppQuad1032>(v);
    } else {
#pragma unroll
        for (int off = kRowLanes / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    }
    return v;
}
__device__ __forceinline__ cplx group_sum(cplx v) { return cplx{group_sum(v.re), group_sum(v.im)}; }
__device__ __forceinline__ float group_sum(float v) {
    if constexpr (kRowLanes == 16) {
        v += dpp_f32<kDppRowMirror>(v);
        v += dpp_f32<kDppRowHalfMirror>(v);
        v += dpp_f32<kDppQuad3210>(v);
        v += dpp_f32<kDppQuad1032>(v);
    } else {
#pragma unroll
        for (int off = kRowLanes / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    }
    return v;
}
__device__ __forceinline__ cplxf group_sum(cplxf v) { return cplxf{group_sum(v.re), group_sum(v.im)}; }

// poll z[j] until solved (bounded; a broken wait sets the sticky error word and gives up)
template <class S>
__device__ __forceinline__ S wait_value(const S* z, int j, int32_t* err) {
    S y = ld_cohi(z, j);
    int spins = 0;
    while (unready(y)) {
        // back off, exponentially: a wave far ahead of the dependency frontier must leave the
        // memory system to the producers
        if (spins < 4) __builtin_amdgcn_s_sleep(2);
        else if (spins < 16) __builtin_amdgcn_s_sleep(8);
        else __builtin_amdgcn_s_sleep(32);
        y = ld_cohi(z, j);
        if ((++spins & 255) == 0 && (spins > kSpinLimit || ld_flag_err(err) != 0)) {
            atomicOr(err, 1);
            break;
        }
    }
    return y;
}

// ---- head: the narrow leading levels, one workgroup, solved values in LDS.
// Levels [0, nhl) hold few rows each (the bottom of an upper-triangular DAG: the first 185 of
// config 5's 372 levels hold 9k of its 1M rows).  Through memory every level costs a coherent
// store + poll round trip (~1.1 us); here a level is a workgroup barrier and LDS reads.  Every
// column a head row reads is an earlier head row (lower level), so columns are LDS positions.
// Pass-major layout built at factor time: pass q (64 rows of one level, one per 16-lane group)
// stores entry k of its group g at hval/hcol[(q * 64 + g) * 16 + k] (padded: column -1) and the
// group's pivot at hpiv[q * 64 + g].  No load depends on another, so the loads of the next kHeadDepth
// passes are in flight (a register ring) while a pass computes: a pass costs its LDS and
// arithmetic latency, not a memory round trip.  zl starts as the scaled right-hand side.
// Padding entries read the zero slot zl[hpos] with value zero; the pass count is padded to a
// multiple of the ring depth with empty passes, so the ring loop is straight-line code.
constexpr int kHeadThreads = 1024;
constexpr int kHeadRows = kHeadThreads / kRowLanes;    // rows per pass
constexpr int kHeadDepth = 8;                          // passes in flight
constexpr int32_t kPassBarrier = 1 << 30;

template <class S, bool kIter>
__global__ __launch_bounds__(kHeadThreads) void sptrsv_head_kernel(TriArgs<S> a, int parity) {
    extern __shared__ __align__(16) unsigned char head_lds[];
    S* zl = reinterpret_cast<S*>(head_lds);
    // zl[hpos] is a zero (the column of padding entries, whose values are zero too)
    int2* pl = reinterpret_cast<int2*>(head_lds + (size_t)(a.hpos + 1) * sizeof(S));   // pass table
    __shared__ Prologue pro;
    const S* xin;
    S* yout;
    double nrm = 0.0;
    if constexpr (kIter) {
        shift_prologue<S>(a.ctl, a.rank_part, parity, a.trace, a.sig_re, a.sig_im, &pro);
        if (!__builtin_amdgcn_readfirstlane(pro.go)) return;   // the tail kernel resets z
        nrm = pro.nrm;
        xin = parity ? a.buf0 : a.buf1;
        yout = parity ? a.buf1 : a.buf0;
    } else {
        xin = a.b_plain;
        yout = a.y_plain;
    }
    const int tid = threadIdx.x;
    const int lane = tid & (kRowLanes - 1);
    const int grp = tid / kRowLanes;
    const int npass = a.npass;
    S rv[kHeadDepth], rp[kHeadDepth];
    int rc[kHeadDepth];
    auto load = [&](int q, S& v, int& c, S& p) {
        const uint32_t e = (uint32_t)(q < npass ? q : 0) * kHeadThreads + (uint32_t)tid;
        v = ldg_stream(a.hval, e);
        c = (int)ldg_stream(a.hcol, e);
        p = ldg_stream(a.hpiv, (uint32_t)(q < npass ? q : 0) * kHeadRows + (uint32_t)grp);
    };
#pragma unroll
    for (int u = 0; u < kHeadDepth; ++u) load(u, rv[u], rc[u], rp[u]);
    for (int p = tid; p < a.hpos; p += kHeadThreads) {
        const int i = a.order[p];
        S b = xin[i >= 0 ? i : 0];
        if constexpr (kIter) b = scale_in(b, nrm);
        zl[p] = b;
    }
    if (tid == 0) zl[a.hpos] = s_zero<S>();
    for (int q = tid; q < npass; q += kHeadThreads) pl[q] = a.passes[q];
    __syncthreads();
    for (int q0 = 0; q0 < npass; q0 += kHeadDepth) {
#pragma unroll
        for (int u = 0; u < kHeadDepth; ++u) {   // straight line: npass is a multiple of the depth
            const int q = q0 + u;
            const int2 pb = pl[q];   // LDS: a vector load here would wait for the ring (vmcnt is in order)
            S acc = group_sum(mul(rv[u], zl[rc[u]]));
            const int pos = pb.x + grp;
            if (lane == 0 && pos < (pb.y & ~kPassBarrier)) zl[pos] = sdiv(sub(zl[pos], acc), rp[u]);
            if (pb.y & kPassBarrier) __syncthreads();
            load(q + kHeadDepth, rv[u], rc[u], rp[u]);
            asm volatile("" ::: "memory");   // keep the refills in ring order (vmcnt retires in issue order)
        }
    }
    __syncthreads();
    // publish: the tail kernel (next in stream order) reads these through z
    for (int p = tid; p < a.hpos; p += kHeadThreads) {
        const int i = a.order[p];
        if (i < 0) continue;
        const S yi = sanitize(zl[p]);
        a.zcur[i] = yi;
        yout[i] = yi;
        a.znext[i] = sentinel<S>();
    }
}

// ---- head, one-wave form.  The narrow levels are a chain of short dependent steps; with a
// workgroup, every pass costs a barrier and the instruction issue of 16 waves (~0.6 us for 64
// rows).  Here ONE wave solves them with no barrier at all (a wave's LDS operations complete in
// issue order): 4 lanes per row, 4 entries per lane, 16 rows per pass, and the row's pivot applied
// as a multiplication by its reciprocal (computed at factor time).  A pass never spans two levels,
// so the rows of a pass are independent; the entries of the next kWHeadDepth passes are in flight
// in a register ring.  The other waves only help to stage the right-hand side into LDS and to
// publish the solved values.
constexpr int kWHeadThreads = 256;
constexpr int kWHeadDepth = 8;
constexpr int kWHeadRows = 16;   // rows per pass
constexpr int kDppQuad2301 = 0x4E;
__device__ __forceinline__ double quad_sum(double v) {
    v += dpp_f64<kDppQuad1032>(v);
    return v + dpp_f64<kDppQuad2301>(v);
}
__device__ __forceinline__ float quad_sum(float v) {
    v += dpp_f32<kDppQuad1032>(v);
    return v + dpp_f32<kDppQuad2301>(v);
}
__device__ __forceinline__ cplx quad_sum(cplx v) { return cplx{quad_sum(v.re), quad_sum(v.im)}; }
__device__ __forceinline__ cplxf quad_sum(cplxf v) { return cplxf{quad_sum(v.re), quad_sum(v.im)}; }

// kMulti: the multi-solve launch's head (shift_multi_prologue): the head is solved K times from
// LDS, solve j on s * (solve j-1's solution); solve j is published to zk[j] and, for the last
// one, to B[parity] (the earlier ones to aux[j]).
template <class S, bool kIter, bool kMulti = false>
__global__ __launch_bounds__(kWHeadThreads) void sptrsv_whead_kernel(TriArgs<S> a, int parity) {
    extern __shared__ __align__(16) unsigned char head_lds[];
    S* zl = reinterpret_cast<S*>(head_lds);
    __shared__ Prologue pro;
    const S* xin;
    S* yout;
    double nrm = 0.0, s2 = 1.0;
    const int K = kMulti ? a.K : 1;
    if constexpr (kIter) {
        if constexpr (kMulti)
            shift_multi_prologue<S>(a.ctl, a.rank_part, a.kpart, a.K, parity, a.trace, a.sig_re, a.sig_im, &pro);
        else
            shift_prologue<S>(a.ctl, a.rank_part, parity, a.trace, a.sig_re, a.sig_im, &pro);
        if (!__builtin_amdgcn_readfirstlane(pro.go)) return;   // the tail kernel resets z
        nrm = pro.nrm;
        s2 = pro.s;
        xin = parity ? a.buf0 : a.buf1;
        yout = parity ? a.buf1 : a.buf0;
    } else {
        xin = a.b_plain;
        yout = a.y_plain;
    }
    const int tid = threadIdx.x;
    // right-hand side of the head positions into LDS: 8 positions per thread per round, every
    // load of a round issued before the first is consumed
    constexpr int kB = 8;
    for (int p0 = 0; p0 < a.hpos; p0 += kWHeadThreads * kB) {
        int ii[kB];
        S bb[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            const int p = p0 + u * kWHeadThreads + tid;
            ii[u] = p < a.hpos ? a.order[p] : -1;
        }
#pragma unroll
        for (int u = 0; u < kB; ++u) bb[u] = xin[ii[u] >= 0 ? ii[u] : 0];
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            const int p = p0 + u * kWHeadThreads + tid;
            if (p < a.hpos) {
                if constexpr (kIter) zl[p] = scale_in(bb[u], nrm);
                else zl[p] = bb[u];
            }
        }
    }
    // multi-solve launch, concurrent head (a.hconc: every solve's values fit the LDS): wave j
    // solves system j in its own LDS array, one pass behind wave j - 1: before pass q it waits
    // for wave j - 1's progress word (LDS operations of one wave execute in order, so a progress
    // value q + 1 means pass q's values are in place), then takes its right-hand side s w_{j-1}
    // from wave j - 1's array.
    const int64_t pitch = a.hpos + 1;
    volatile int* prog = reinterpret_cast<volatile int*>(zl + K * pitch);
    const bool conc = kMulti && a.hconc;
    if (tid == 0) {
        zl[a.hpos] = s_zero<S>();
        if (conc)
            for (int j = 1; j < K; ++j) {
                zl[j * pitch + a.hpos] = s_zero<S>();
                prog[j - 1] = 0;
            }
    }
    __syncthreads();
    // which 0: values in zl, right-hand side in place; which j >= 1: values in array j, rhs s * array j-1
    auto passes = [&](const int which) {
        const int lane = tid & 63, grp = lane >> 2, slot = lane & 3;
        const int nw = a.nwpass;
        S* zs = zl + which * pitch;
        const S* zp = zl + (which ? which - 1 : 0) * pitch;
        S rv[kWHeadDepth][4], rq[kWHeadDepth];
        int rc[kWHeadDepth][4], rd[kWHeadDepth];
        auto load = [&](int q, S* v, int* c, S& r, int& d) {
            const uint32_t qq = (uint32_t)(q < nw ? q : 0);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t e = (qq * 4u + (uint32_t)k) * 64u + (uint32_t)lane;
                v[k] = ldg(a.wval, e);   // temporal loads: the head's data stays cached between solves
                c[k] = (int)ldg(a.wcol, e);
            }
            r = ldg(a.wrp, qq * (uint32_t)kWHeadRows + (uint32_t)grp);
            d = q < nw ? (int)ldg(a.wdst, qq * (uint32_t)kWHeadRows + (uint32_t)grp) : -1;
        };
#pragma unroll
        for (int u = 0; u < kWHeadDepth; ++u) load(u, rv[u], rc[u], rq[u], rd[u]);
        for (int q0 = 0; q0 < nw; q0 += kWHeadDepth) {
#pragma unroll
            for (int u = 0; u < kWHeadDepth; ++u) {   // straight line: nw is a multiple of the depth
                if (which) {
                    while (prog[which - 1] <= q0 + u) __builtin_amdgcn_s_sleep(1);
                    asm volatile("" ::: "memory");
                }
                S acc = mul(rv[u][0], zs[rc[u][0]]);
#pragma unroll
                for (int k = 1; k < 4; ++k) acc = add(acc, mul(rv[u][k], zs[rc[u][k]]));
                acc = quad_sum(acc);
                const int d = rd[u];
                if (slot == 0 && d >= 0) {
                    const S rhs = which ? scale_r(sanitize(zp[d]), s2) : zs[d];
                    zs[d] = mul(sub(rhs, acc), rq[u]);
                }
                asm volatile("" ::: "memory");   // this pass's store precedes the next pass's reads
                if (conc && which + 1 < K && lane == 0) prog[which] = q0 + u + 1;
                load(q0 + u + kWHeadDepth, rv[u], rc[u], rq[u], rd[u]);
            }
        }
    };
  for (int rep = 0; rep < K; ++rep) {
    if (!conc || rep == 0) {
        const int w = tid >> 6;
        if (w == 0 || (conc && w < K)) passes(w);
        __syncthreads();
    }
    // publish: the tail kernel (next in stream order) reads these through z
    S* zc = rep ? a.zk[rep] : a.zcur;
    S* zn = rep ? a.zkn[rep] : a.znext;
    S* yo = rep == K - 1 ? yout : a.aux[rep];
    const S* zsrc = zl + (conc ? rep : 0) * pitch;
    for (int p = tid; p < a.hpos; p += kWHeadThreads) {
        const int i = a.order[p];
        if (i < 0) continue;
        const S yi = sanitize(zsrc[p]);
        zc[i] = yi;
        yo[i] = yi;
        zn[i] = sentinel<S>();
        if (kMulti && !conc && rep + 1 < K) zl[p] = scale_r(yi, s2);   // the next solve's right-hand side
    }
    if (kMulti && !conc && rep + 1 < K) __syncthreads();
  }
}

// the chunk tails' back-off between re-polls of an unsolved value: pf = EIGSOL_TRSV_POLL_FAST in
// the low 16 bits (re-polls without a sleep), EIGSOL_TRSV_POLL_SLOW in bits 16-18 (the sleep
// schedule below, in units of 64 cycles: fewer re-poll requests against later wake-ups)
__device__ __forceinline__ void poll_backoff(int spins, int pf) {
    const int fast = pf & 0xffff, slow = pf >> 16;
    if (spins < fast) return;         // re-poll at once: the value is due within a round trip
    const int s = spins - fast;
    const int step = s < 4 ? 0 : (s < 16 ? 1 : 2);
    switch (slow * 3 + step) {        // s_sleep takes an immediate
        case 0: __builtin_amdgcn_s_sleep(2); break;     // 0: 2 / 8 / 32
        case 1: __builtin_amdgcn_s_sleep(8); break;
        case 2: __builtin_amdgcn_s_sleep(32); break;
        case 3: case 4: case 5: __builtin_amdgcn_s_sleep(4); break;       // 1: 4
        case 6: case 7: case 8: __builtin_amdgcn_s_sleep(6); break;       // 2: 6
        case 9: case 10: case 11: __builtin_amdgcn_s_sleep(16); break;    // 3: 16
        case 12: case 13: case 14: __builtin_amdgcn_s_sleep(8); break;    // 4: 8
        case 15: case 16: case 17: __builtin_amdgcn_s_sleep(32); break;   // 5: 32
        case 18: case 19: case 20: __builtin_amdgcn_s_sleep(12); break;   // 6: 12
        case 21: __builtin_amdgcn_s_sleep(16); break;   // 7: 16 / 24 / 32
        case 22: __builtin_amdgcn_s_sleep(24); break;
        default: __builtin_amdgcn_s_sleep(32); break;
    }
}

// first poll of a dependency is issued early (ld_coh); this finishes the wait
template <class S>
__device__ __forceinline__ S finish_wait(S y, const S* z, int j, int32_t* err, int pf) {
    int spins = 0;
    while (unready(y)) {
        poll_backoff(spins, pf);
        y = ld_cohi(z, j);
        if ((++spins & 255) == 0 && (spins > kSpinLimit || ld_flag_err(err) != 0)) {
            atomicOr(err, 1);
            break;
        }
    }
    return y;
}

// ---- tail: sync-free triangular solve over the remaining (wide) levels, one row per lane.
// The rows of each tail level are cut into slices of 64 (a level's last slice is padded with
// empty rows, so a slice never spans two levels and its lanes never wait on each other).  Slice
// s stores entry k of lane l at off_s + 64 k + l (coalesced), padded to at least B entries per
// lane with the zero slot z[n] (always 0) and value 0.  A lane computes its row exactly as the
// reference's back substitution does: s = b_i, s -= a_ij z_j in stored column order, y_i = s / d_i
// (oracle triu_shifted_solve_csr: bitwise equal when no FMA is contracted).
// Slices are dealt round-robin to the W waves, each taking its slices in increasing order.  A
// slice waits only on slices of strictly lower levels, i.e. earlier slices, so the earliest
// unfinished slice can always proceed provided every wave is resident: the kernel is launched
// cooperatively, so the runtime guarantees co-residency (or refuses the launch); a bounded spin
// plus a sticky error word still guarantee the grid drains.  (A ticket dispenser needs no
// co-residency, but 250k atomics on one word serialise: 3.3 ms against 0.9 ms.)
// Per slice: the B dependency loads (coherent; the solved value is its own ready flag, z starts
// as the sentinel NaN) and the B values are issued first, then the columns / row / pivot of the
// wave's next slice, so waiting on the dependencies does not wait on the prefetch (vmcnt retires
// in issue order).  Each launch resets the other z buffer row by row for the next launch (also
// when it exits early).  Norm / Rayleigh partials are reduced afterwards by shift_part_kernel.
template <class S, int B, bool kIter>
__global__ __launch_bounds__(kThreads) void sptrsv_slice_kernel(TriArgs<S> a, int parity) {
    __shared__ Prologue pro;
    const S* xin;
    S* yout;
    double nrm = 0.0;
    if constexpr (kIter) {
        shift_prologue<S>(a.ctl, a.rank_part, parity, a.trace, a.sig_re, a.sig_im, &pro);
        if (!__builtin_amdgcn_readfirstlane(pro.go)) {
            // nothing to solve, but the next launch still expects its z reset
            for (int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x; r < a.n; r += (int64_t)gridDim.x * kThreads)
                a.znext[r] = sentinel<S>();
            return;
        }
        nrm = pro.nrm;
        xin = parity ? a.buf0 : a.buf1;
        yout = parity ? a.buf1 : a.buf0;
    } else {
        xin = a.b_plain;
        yout = a.y_plain;
    }
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int W = gridDim.x * kWaves;
    const int ns = a.nslices;
    // consecutive slices (the slices of one level) go to consecutive workgroups, i.e. to
    // different CUs and XCDs, not to the four waves of one CU
    int s = wave * gridDim.x + blockIdx.x;

    int K, off, row;
    S piv;
    int col[B];
    auto fetch = [&](int s_, int& K_, int& off_, int* c, int& row_, S& piv_) {
        const bool in = s_ < ns;
        const int2 m = a.smeta[in ? s_ : 0];
        K_ = in ? m.y : 0;
        off_ = m.x;
#pragma unroll
        for (int k = 0; k < B; ++k) c[k] = (int)ldg_stream(a.tcol, (uint32_t)(off_ + 64 * k + lane));
        const uint32_t r = (uint32_t)((in ? s_ : 0) * 64 + lane);
        row_ = in ? (int)ldg_stream(a.trow, r) : -1;
        piv_ = ldg_stream(a.tpiv, r);
    };
    fetch(s, K, off, col, row, piv);
    for (; s < ns; s += W) {
        S z[B], v[B];
#pragma unroll
        for (int k = 0; k < B; ++k) z[k] = ld_cohi(a.zcur, col[k]);
#pragma unroll
        for (int k = 0; k < B; ++k) v[k] = ldg_stream(a.tval, (uint32_t)(off + 64 * k + lane));
        S bi = xin[row >= 0 ? row : 0];
        int Kn, offn, rown, coln[B];
        S pivn;
        fetch(s + W, Kn, offn, coln, rown, pivn);
        if constexpr (kIter) bi = scale_in(bi, nrm);
        S acc = bi;
        // dependencies not yet solved at the first load: poll them all together (one round trip
        // per poll round, not one per entry)
        bool pend = false;
#pragma unroll
        for (int k = 0; k < B; ++k) pend = pend || unready(z[k]);
        int spins = 0;
        while (pend) {
            if (spins >= (a.poll_fast & 0xffff)) {
                if (spins < (a.poll_fast & 0xffff) + 8) __builtin_amdgcn_s_sleep(2);
                else __builtin_amdgcn_s_sleep(16);
            }
            if (!(a.poll_mode & 1)) {
#pragma unroll
                for (int k = 0; k < B; ++k)
                    if (unready(z[k])) z[k] = ld_cohi(a.zcur, col[k]);
            } else {   // one poll per lane: its first unsolved dependency
                int kf = -1;
#pragma unroll
                for (int k = B - 1; k >= 0; --k)
                    if (unready(z[k])) kf = k;
                S zf = ld_cohi(a.zcur, kf >= 0 ? col[kf] : (int)a.n);
#pragma unroll
                for (int k = 0; k < B; ++k)
                    if (k == kf) z[k] = zf;
            }
            pend = false;
#pragma unroll
            for (int k = 0; k < B; ++k) pend = pend || unready(z[k]);
            if ((++spins & 255) == 0 && (spins > kSpinLimit || ld_flag_err(a.err) != 0)) {
                atomicOr(a.err, 1);
                break;
            }
        }
#pragma unroll
        for (int k = 0; k < B; ++k) acc = sub(acc, mul(v[k], z[k]));
        for (int k = B; k < K; ++k) {   // entries beyond B (long rows): one dependent round trip each
            const uint32_t e = (uint32_t)(off + 64 * k + lane);
            const int c = (int)a.tcol[e];
            acc = sub(acc, mul(a.tval[e], wait_value(a.zcur, c, a.err)));
        }
        if (row >= 0) {
            const S yi = sanitize(sdiv(acc, piv));
            st_cohi(a.zcur, row, yi);        // publish: readers poll this very word
            yout[row] = yi;
            a.znext[row] = sentinel<S>();
        }
        K = Kn;
        off = offn;
        row = rown;
        piv = pivn;
#pragma unroll
        for (int k = 0; k < B; ++k) col[k] = coln[k];
    }
}

// ---- tail, chunk variant: sync-free triangular solve, 16 lanes per row, 4 rows per chunk.
// Positions (level-ordered, every level padded to kWaveRows) form chunks of one wave round;
// chunk c belongs to wave (c - chunk0) mod W (consecutive chunks on consecutive workgroups), each
// wave taking its chunks in increasing order, two at a time: the dependency loads of a pair are
// issued at the end of the previous iteration (speculatively: a sentinel just means poll again),
// then the first chunk is solved and published, then the second (which may read the first).
// Progress needs every wave resident: launched cooperatively, like the slice variant.  Chosen
// for DAGs of many moderately wide levels (config 5: 0.86 ms against 1.3 ms for the slices,
// which wait on the slowest of 960 dependencies per wave); the slice variant wins on few, very
// wide levels (one 1M-row level: 74 us against 195 us).
template <class S>
struct RowMeta {
    int i, e0, len, j, j2;
    S v, v2, bi, pv;
};

// kTwo: rows of up to 2 x 16 entries (e.g. an LU factor with fill) keep a second entry per lane,
// whose dependency is polled together with the first instead of one round trip later
template <class S, bool kIter, bool kTwo = false>
__global__ __launch_bounds__(kThreads) void sptrsv_chunk_kernel(TriArgs<S> a, int parity) {
    __shared__ Prologue pro;
    const S* xin;
    S* yout;
    double nrm = 0.0;
    if constexpr (kIter) {
        shift_prologue<S>(a.ctl, a.rank_part, parity, a.trace, a.sig_re, a.sig_im, &pro);
        if (!__builtin_amdgcn_readfirstlane(pro.go)) {
            for (int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x; r < a.n; r += (int64_t)gridDim.x * kThreads)
                a.znext[r] = sentinel<S>();
            return;
        }
        nrm = pro.nrm;
        xin = parity ? a.buf0 : a.buf1;
        yout = parity ? a.buf1 : a.buf0;
    } else {
        xin = a.b_plain;
        yout = a.y_plain;
    }
    const int tid = threadIdx.x;
    const int lane = tid & (kRowLanes - 1);
    const int grp = (tid & 63) / kRowLanes;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int W = gridDim.x * kWaves;
    const int gw = a.chunk0 + wave * gridDim.x + blockIdx.x;

    auto fetch1 = [&](int c, RowMeta<S>& m) {   // position-indexed metadata: no dependent loads
        const bool in = c < a.nchunks;
        const int pos = (in ? c : 0) * kWaveRows + grp;
        m.i = in ? a.porder[pos] : -1;
        const int e0 = a.pptr[pos];
        m.e0 = e0;
        m.len = in ? a.pptr[pos + 1] - e0 : 0;
        m.pv = ldg_stream(a.ppiv, (uint32_t)pos);
    };
    auto fetch2 = [&](RowMeta<S>& m) {         // the row's first 16 entries and its right side
        const bool ok = lane < m.len;
        const int e = ok ? m.e0 + lane : 0;
        m.j = ok ? (int)ldg_stream(a.pcol, (uint32_t)e) : -1;
        m.v = ldg_stream(a.pval, (uint32_t)e);
        if constexpr (kTwo) {
            const bool ok2 = lane + kRowLanes < m.len;
            const int e2 = ok2 ? m.e0 + lane + kRowLanes : 0;
            m.j2 = ok2 ? (int)ldg_stream(a.pcol, (uint32_t)e2) : -1;
            m.v2 = ldg_stream(a.pval, (uint32_t)e2);
        }
        m.bi = xin[m.i >= 0 ? m.i : 0];
    };
    auto solve = [&](const RowMeta<S>& m, S z0, S z0b) {
        S acc = s_zero<S>();
        if (m.j >= 0) acc = mul(m.v, finish_wait(z0, a.zcur, m.j, a.err, a.poll_fast));
        if constexpr (kTwo)
            if (m.j2 >= 0) acc = add(acc, mul(m.v2, finish_wait(z0b, a.zcur, m.j2, a.err, a.poll_fast)));
        for (int k = lane + (kTwo ? 2 : 1) * kRowLanes; k < m.len; k += kRowLanes) {   // rows longer than 16 / 32
            const int e = m.e0 + k;
            acc = add(acc, mul(a.pval[e], wait_value(a.zcur, a.pcol[e], a.err)));
        }
        acc = group_sum(acc);
        if (m.i >= 0 && lane == 0) {
            S bi = m.bi;
            if constexpr (kIter) bi = scale_in(bi, nrm);
            const S yi = sanitize(sdiv(sub(bi, acc), m.pv));
            st_cohi(a.zcur, m.i, yi);        // publish: readers poll this very word
            if constexpr (!kIter) {          // iteration: shift_part_kernel<S, true> moves y out
                yout[m.i] = yi;
                a.znext[m.i] = sentinel<S>();
            }
        }
    };

    RowMeta<S> c0, c1, n0, n1;
    fetch1(gw, c0);
    fetch1(gw + W, c1);
    fetch2(c0);
    fetch2(c1);
    fetch1(gw + 2 * W, n0);
    fetch1(gw + 3 * W, n1);
    // EIGSOL_TRSV_POLL_MODE bit 1: the second chunk's first polls after the first chunk is solved
    const int late = a.poll_mode & 2;
    auto first_poll = [&](int j) { return j >= 0 ? ld_cohi(a.zcur, j) : s_zero<S>(); };
    S z0 = first_poll(c0.j), z1 = first_poll(c1.j);
    S z0b = s_zero<S>(), z1b = s_zero<S>();
    if constexpr (kTwo) {
        z0b = first_poll(c0.j2);
        z1b = first_poll(c1.j2);
    }
    for (int c = gw; c < a.nchunks; c += 2 * W) {
        fetch2(n0);
        fetch2(n1);
        RowMeta<S> m0, m1;
        fetch1(c + 4 * W, m0);
        fetch1(c + 5 * W, m1);
        solve(c0, z0, z0b);
        if (late) {
            z1 = first_poll(c1.j);
            if constexpr (kTwo) z1b = first_poll(c1.j2);
        }
        solve(c1, z1, z1b);
        z0 = first_poll(n0.j);
        if constexpr (kTwo) z0b = first_poll(n0.j2);
        if (!late) {
            z1 = first_poll(n1.j);
            if constexpr (kTwo) z1b = first_poll(n1.j2);
        }
        c0 = n0;
        c1 = n1;
        n0 = m0;
        n1 = m1;
    }
}

// ---- tail of a multi-solve launch (shift_multi_prologue), role split: the grid is K copies of
// the single-solve grid.  Blocks [jG, (j+1)G) run sptrsv_chunk_kernel's schedule for solve j:
// w_0 = (A - sigma I)^{-1} x, w_j = (A - sigma I)^{-1} (s w_{j-1}), taking each row's right-hand
// side s (w_{j-1})_i from solve j-1's polled value (its ready flag) and their dependencies from
// zk[j].  A wave waits only on its own solve's chains (and on the row of the solve before), so
// solve j trails solve j-1 by about one dependency round trip.  The matrix is read once per
// solve.  No deadlock: solve j-1 never waits on solve j, and every wave is resident (cooperative
// launch).  Measured on config 5 (pair launches, K = 2): 0.539 ms per iteration at one workgroup
// per CU per solve against 0.555 at two, and 0.58 ms for an interleaved schedule (each wave
// solving its chunks of round r for w_0, then those of round r - 1 for w_1: a wave's second-solve
// waits then add to its first-solve waits).
template <class S>
__global__ __launch_bounds__(kThreads) void sptrsv_chunk_role_kernel(TriArgs<S> a, int parity) {
    __shared__ Prologue pro;
    shift_multi_prologue<S>(a.ctl, a.rank_part, a.kpart, a.K, parity, a.trace, a.sig_re, a.sig_im, &pro);
    if (!__builtin_amdgcn_readfirstlane(pro.go)) {
        for (int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x; r < a.n; r += (int64_t)gridDim.x * kThreads)
            for (int j = 0; j < a.K; ++j) a.zkn[j][r] = sentinel<S>();
        return;
    }
    const int G = (int)gridDim.x / a.K;
    const int role = __builtin_amdgcn_readfirstlane((int)blockIdx.x / G);
    const int blk = (int)blockIdx.x - role * G;
    const double nrm = pro.nrm, s2 = pro.s;
    const S* xin = parity ? a.buf0 : a.buf1;
    S* zdep = a.zk[role];                          // dependencies and publication
    const S* zrhs = a.zk[role ? role - 1 : 0];     // solve j >= 1: the previous solve's values
    const int tid = threadIdx.x;
    const int lane = tid & (kRowLanes - 1);
    const int grp = (tid & 63) / kRowLanes;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int W = G * kWaves;
    const int gw = a.chunk0 + wave * G + blk;

    auto fetch1 = [&](int c, RowMeta<S>& m) {
        const bool in = c < a.nchunks;
        const int pos = (in ? c : 0) * kWaveRows + grp;
        m.i = in ? a.porder[pos] : -1;
        const int e0 = a.pptr[pos];
        m.e0 = e0;
        m.len = in ? a.pptr[pos + 1] - e0 : 0;
        m.pv = ldg_stream(a.ppiv, (uint32_t)pos);
    };
    auto fetch2 = [&](RowMeta<S>& m) {
        const bool ok = lane < m.len;
        const int e = ok ? m.e0 + lane : 0;
        m.j = ok ? (int)ldg_stream(a.pcol, (uint32_t)e) : -1;
        m.v = ldg_stream(a.pval, (uint32_t)e);
        // second solve: the first solve's value of the row, possibly not yet solved (polled below)
        m.bi = role ? ld_cohi(zrhs, (m.i >= 0 ? m.i : (int)a.n)) : xin[m.i >= 0 ? m.i : 0];
    };
    auto solve = [&](const RowMeta<S>& m, S z0) {
        S acc = s_zero<S>();
        S bv = m.bi;
        if (role) {
            // the dependency and (lane 0) the first solve's value of the row are polled in the same
            // loop: waiting for them one after the other would add a round trip to every level
            const bool nb = lane == 0 && m.i >= 0;
            S zv = m.j >= 0 ? z0 : s_zero<S>();
            int spins = 0;
            while (unready(zv) || (nb && unready(bv))) {
                poll_backoff(spins, a.poll_fast & ~0xffff);
                if (unready(zv)) zv = ld_cohi(zdep, m.j);
                if (nb && unready(bv)) bv = ld_cohi(zrhs, m.i);
                if ((++spins & 255) == 0 && (spins > kSpinLimit || ld_flag_err(a.err) != 0)) {
                    atomicOr(a.err, 1);
                    break;
                }
            }
            if (m.j >= 0) acc = mul(m.v, zv);
        } else if (m.j >= 0) {
            acc = mul(m.v, finish_wait(z0, zdep, m.j, a.err, a.poll_fast));
        }
        for (int k = lane + kRowLanes; k < m.len; k += kRowLanes) {
            const int e = m.e0 + k;
            acc = add(acc, mul(a.pval[e], wait_value(zdep, a.pcol[e], a.err)));
        }
        acc = group_sum(acc);
        if (m.i >= 0 && lane == 0) {
            S bi;
            if (role) bi = scale_r(bv, s2);
            else bi = scale_in(m.bi, nrm);
            const S yi = sanitize(sdiv(sub(bi, acc), m.pv));
            st_cohi(zdep, m.i, yi);        // moved out by shift_multi_part_kernel
        }
    };

    RowMeta<S> c0, c1, n0, n1;
    fetch1(gw, c0);
    fetch1(gw + W, c1);
    fetch2(c0);
    fetch2(c1);
    fetch1(gw + 2 * W, n0);
    fetch1(gw + 3 * W, n1);
    // EIGSOL_TRSV_POLL_MODE bit 1: the second chunk's first polls are issued after the first
    // chunk is solved instead of a round ahead (fewer polls of still-unsolved values); bit 2: both
    // chunks' first polls at the top of the round
    const int late = a.poll_mode;
    S z0 = c0.j >= 0 ? ld_cohi(zdep, c0.j) : s_zero<S>();
    S z1 = c1.j >= 0 ? ld_cohi(zdep, c1.j) : s_zero<S>();
    for (int c = gw; c < a.nchunks; c += 2 * W) {
        if (late & 4) {
            z0 = c0.j >= 0 ? ld_cohi(zdep, c0.j) : s_zero<S>();
            z1 = c1.j >= 0 ? ld_cohi(zdep, c1.j) : s_zero<S>();
        }
        fetch2(n0);
        fetch2(n1);
        RowMeta<S> m0, m1;
        fetch1(c + 4 * W, m0);
        fetch1(c + 5 * W, m1);
        solve(c0, z0);
        if (late & 2) z1 = c1.j >= 0 ? ld_cohi(zdep, c1.j) : s_zero<S>();
        solve(c1, z1);
        if (!(late & 4)) z0 = n0.j >= 0 ? ld_cohi(zdep, n0.j) : s_zero<S>();
        if (!(late & 6)) z1 = n1.j >= 0 ? ld_cohi(zdep, n1.j) : s_zero<S>();
        c0 = n0;
        c1 = n1;
        n0 = m0;
        n1 = m1;
    }
}

// Partials of a multi-solve launch, solve j: {||w_j||^2, w_{j-1}^H w_j} (w_{-1} = x) -> my_part
// (j = 0) or kpart[j - 1], each in a fixed order (grid-stride per thread, block sums, last-arriver
// sum in block order).  The solves left w_j only in their polled buffers: this kernel moves them
// out (aux[j], the last one to B[parity]) and resets the next launch's buffers, in coalesced
// streams.
template <class S>
__global__ __launch_bounds__(kThreads) void shift_multi_part_kernel(TriArgs<S> a, int parity) {
    __shared__ double sm[3 * kWaves];
    __shared__ int s_last[kMaxMulti];
    __shared__ int s_go;
    __shared__ double s_nrm;
    if (threadIdx.x == 0) {
        s_go = __hip_atomic_load(&a.ctl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 0 : 1;
        s_nrm = a.ctl->st[parity ^ 1].nrm;
    }
    __syncthreads();
    if (!s_go) return;
    const double nrm = s_nrm;
    const int K = a.K;
    const S* xin = parity ? a.buf0 : a.buf1;
    S* wlast = parity ? a.buf1 : a.buf0;
    double n2[kMaxMulti] = {}, dr[kMaxMulti] = {}, di[kMaxMulti] = {};
#pragma unroll 2
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * kThreads) {
        S prev = scale_in(xin[i], nrm);
#pragma unroll
        for (int j = 0; j < kMaxMulti; ++j) {
            if (j < K) {
                const S y = a.zk[j][i];
                (j == K - 1 ? wlast : a.aux[j])[i] = y;
                a.zkn[j][i] = sentinel<S>();
                n2[j] += sq_abs(y);
                acc_dot(dr[j], di[j], prev, y);
                prev = y;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < kMaxMulti; ++j) {
        if (j < K) {
            block_sum3(n2[j], dr[j], di[j], sm);
            last_arriver_reduce(n2[j], dr[j], di[j], j ? a.kblk + (size_t)(j - 1) * gridDim.x : a.wave_part,
                                a.work + 2 + j, j ? a.kpart + (j - 1) : a.my_part, sm, &s_last[j]);
        }
    }
}

// GMRES path: the launch prologue alone (the stop decision and ||y_{t-1}||), the solve follows on
// the host's word
template <class S>
__global__ __launch_bounds__(64) void shift_decide_kernel(TriArgs<S> a, int parity) {
    __shared__ Prologue pro;
    shift_prologue<S>(a.ctl, a.rank_part, parity, a.trace, a.sig_re, a.sig_im, &pro);
}

// Norm and Rayleigh partials of a solved iterate, in a fixed order (grid-stride per thread,
// block sums, last-arriver sum in block order): sum |y_i|^2 and sum conj(x_i) y_i with
// x = b / ||y_prev|| as the solve used it.  Skipped once the prologue has stopped the loop.
// kFromZ (triangular factors): the solve left y only in the polled buffer zcur; this kernel also
// moves it to B[parity] and resets znext to the sentinel for the next launch (coalesced streams,
// instead of two scattered 16-byte stores per row inside the latency-bound solve)
template <class S, bool kFromZ = false>
__global__ __launch_bounds__(kThreads) void shift_part_kernel(TriArgs<S> a, int parity) {
    __shared__ double sm[3 * kWaves];
    __shared__ int s_last;
    __shared__ int s_go;
    __shared__ double s_nrm;
    if (threadIdx.x == 0) {
        s_go = __hip_atomic_load(&a.ctl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 0 : 1;
        s_nrm = a.ctl->st[parity ^ 1].nrm;
    }
    __syncthreads();
    if (!s_go) return;
    const double nrm = s_nrm;
    const S* xin = parity ? a.buf0 : a.buf1;
    S* y = parity ? a.buf1 : a.buf0;
    double n2 = 0.0, pr = 0.0, pi = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * kThreads) {
        S yi;
        if constexpr (kFromZ) {
            yi = a.zcur[i];
            y[i] = yi;
            a.znext[i] = sentinel<S>();
        } else {
            yi = y[i];
        }
        n2 += sq_abs(yi);
        acc_dot(pr, pi, scale_in(xin[i], nrm), yi);   // p = sum conj(x_i) y_i
    }
    block_sum3(n2, pr, pi, sm);
    last_arriver_reduce(n2, pr, pi, a.wave_part, a.work + 2, a.my_part, sm, &s_last);
}

// ------------------------------------------------------------------ dense LU (factor once)
__device__ __forceinline__ double score(double v) { return fabs(v); }
__device__ __forceinline__ double score(cplx v) { return hypot(v.re, v.im); }
__device__ __forceinline__ double score(float v) { return fabs((double)v); }
__device__ __forceinline__ double score(cplxf v) { return hypot((double)v.re, (double)v.im); }

// Column k: pivot = first row of largest modulus in rows k..n-1, swap full rows, record the
// transposition, scale the subdiagonal column by the pivot (skipped for a zero pivot, as Eigen's
// partial_lu_impl does; the first zero pivot is recorded).
template <class S>
__global__ __launch_bounds__(1024) void lu_pivot_kernel(S* a, int64_t n, int64_t k, int64_t c0, int64_t c1,
                                                        int32_t* piv, int32_t* zero_pivot) {
    __shared__ double sv[1024];
    __shared__ int si[1024];
    __shared__ int s_p;
    const int tid = threadIdx.x;
    double best = -1.0;
    int bi = (int)k;
    for (int64_t i = k + tid; i < n; i += 1024) {
        const double s = score(a[k * n + i]);
        if (s > best) { best = s; bi = (int)i; }
    }
    sv[tid] = best;
    si[tid] = bi;
    __syncthreads();
    for (int off = 512; off > 0; off >>= 1) {
        if (tid < off) {
            const double o = sv[tid + off];
            const int oi = si[tid + off];
            if (o > sv[tid] || (o == sv[tid] && oi < si[tid])) { sv[tid] = o; si[tid] = oi; }
        }
        __syncthreads();
    }
    if (tid == 0) {
        s_p = si[0];
        piv[k] = si[0];
        if (sv[0] == 0.0 && *zero_pivot < 0) *zero_pivot = (int)k;
    }
    __syncthreads();
    const int64_t p = s_p;
    if (p != k)
        for (int64_t j = c0 + tid; j < c1; j += 1024) {
            const S t = a[j * n + k];
            a[j * n + k] = a[j * n + p];
            a[j * n + p] = t;
        }
    __syncthreads();
    const S d = a[k * n + k];
    if (score(d) != 0.0)
        for (int64_t i = k + 1 + tid; i < n; i += 1024) a[k * n + i] = sdiv(a[k * n + i], d);
}

// panel update a_ij -= l_ik u_kj, i > k, k < j < c1 (one thread per element, column-major coalesced)
template <class S>
__global__ __launch_bounds__(256) void lu_update_kernel(S* a, int64_t n, int64_t k, int64_t c1) {
    const int64_t m = n - k - 1, w = c1 - k - 1;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= m * w) return;
    const int64_t i = k + 1 + idx % m;
    const int64_t j = k + 1 + idx / m;
    a[j * n + i] = sub(a[j * n + i], mul(a[k * n + i], a[j * n + k]));
}

// the panel's row interchanges (rows j <-> piv[j], j = k0 .. k0 + kb - 1, in order) applied to every
// column outside the panel; one thread per column
template <class S>
__global__ __launch_bounds__(256) void lu_laswp_kernel(S* a, int64_t n, int64_t k0, int kb, const int32_t* piv) {
    int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= n - kb) return;
    if (c >= k0) c += kb;
    S* col = a + c * n;
    for (int j = 0; j < kb; ++j) {
        const int64_t r = k0 + j, p = piv[r];
        if (p != r) {
            const S t = col[r];
            col[r] = col[p];
            col[p] = t;
        }
    }
}

// U12 = L11^{-1} A12: L11 the panel's unit lower kb x kb block (LDS), one thread per column of A12
template <class S, int NB>
__global__ __launch_bounds__(256) void lu_trsm_kernel(S* a, int64_t n, int64_t k0, int kb) {
    __shared__ S l11[NB * NB];
    for (int e = threadIdx.x; e < kb * kb; e += 256) {
        const int i = e % kb, j = e / kb;
        l11[i + j * NB] = a[(k0 + i) + (k0 + j) * n];
    }
    __syncthreads();
    const int64_t c = k0 + kb + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= n) return;
    S* col = a + c * n + k0;
    S x[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) x[i] = i < kb ? col[i] : s_zero<S>();
#pragma unroll
    for (int j = 0; j < NB - 1; ++j) {
        if (j < kb) {   // kb < NB only for the last panel
#pragma unroll
            for (int i = j + 1; i < NB; ++i) x[i] = sub(x[i], mul(l11[i + j * NB], x[j]));
        }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
        if (i < kb) col[i] = x[i];
}

template <class S>
struct DenseSolveArgs {
    const S* lu;
    const int32_t* perm;
    int64_t n;
    const S* b_plain;
    S* y_plain;
    S* buf0;
    S* buf1;
    PowerCtl* ctl;
    const part4* rank_part;
    part4* my_part;
    S* trace;
    double sig_re, sig_im;
};

// One workgroup: z = P b (scaled by 1/||y_prev|| in iteration mode), L z = P b (unit lower),
// U y = z, all in LDS; column-oriented so every column access is coalesced.
template <class S, bool kIter>
__global__ __launch_bounds__(1024) void dense_lu_solve_kernel(DenseSolveArgs<S> a, int parity) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    S* z = reinterpret_cast<S*>(lds_raw);
    __shared__ Prologue pro;
    __shared__ double sm[3 * 16];
    const int tid = threadIdx.x;
    const int64_t n = a.n;
    const S* xin;
    S* yout;
    double nrm = 0.0;
    if constexpr (kIter) {
        shift_prologue<S>(a.ctl, a.rank_part, parity, a.trace, a.sig_re, a.sig_im, &pro);
        if (!__builtin_amdgcn_readfirstlane(pro.go)) return;   // block-uniform exit
        nrm = pro.nrm;
        xin = parity ? a.buf0 : a.buf1;
        yout = parity ? a.buf1 : a.buf0;
    } else {
        xin = a.b_plain;
        yout = a.y_plain;
    }
    for (int64_t i = tid; i < n; i += 1024) {
        S v = xin[a.perm[i]];
        if constexpr (kIter) v = scale_in(v, nrm);
        z[i] = v;
    }
    __syncthreads();
    // forward: for each column j, z_i -= L_ij z_j (i > j)
    for (int64_t j = 0; j < n; ++j) {
        const S zj = z[j];
        const S* colj = a.lu + j * n;
        for (int64_t i = j + 1 + tid; i < n; i += 1024) z[i] = sub(z[i], mul(colj[i], zj));
        __syncthreads();
    }
    // backward: for each column j from the last, z_j /= U_jj, z_i -= U_ij z_j (i < j)
    for (int64_t j = n - 1; j >= 0; --j) {
        const S* colj = a.lu + j * n;
        const S zj = sdiv(z[j], colj[j]);
        __syncthreads();
        if (tid == 0) z[j] = zj;
        for (int64_t i = tid; i < j; i += 1024) z[i] = sub(z[i], mul(colj[i], zj));
        __syncthreads();
    }
    double n2 = 0.0, pr = 0.0, pi = 0.0;
    for (int64_t i = tid; i < n; i += 1024) {
        const S yi = z[i];
        yout[i] = yi;
        if constexpr (kIter) {
            S xi = xin[i];
            xi = scale_in(xi, nrm);
            n2 += sq_abs(yi);
            acc_dot(pr, pi, xi, yi);
        }
    }
    if constexpr (kIter) {
        // 1024 threads = 16 waves: wave sums then a fixed-order sum by thread 0
        n2 = wave_sum(n2);
        pr = wave_sum(pr);
        pi = wave_sum(pi);
        const int w = tid >> 6;
        if ((tid & 63) == 0) { sm[w] = n2; sm[16 + w] = pr; sm[32 + w] = pi; }
        __syncthreads();
        if (tid == 0) {
            double s0 = 0.0, s1 = 0.0, s2 = 0.0;
            for (int i = 0; i < 16; ++i) { s0 += sm[i]; s1 += sm[16 + i]; s2 += sm[32 + i]; }
            a.my_part->a = s0;
            a.my_part->b = s1;
            a.my_part->c = s2;
            a.my_part->d = 0.0;
        }
    }
}

// ------------------------------------------------------------ multi-CU dense substitution
// L z = P b (L unit lower), then U y = z, for large dense factors: block rows of kDB rows, one
// persistent workgroup per resident slot taking block rows round-robin — all its forward rows in
// increasing order, then all its backward rows in decreasing order.  A block row accumulates the
// off-diagonal tiles L_rc z_c as the z_c it needs are published (epoch flags: no reset between
// launches), solves its kDB x kDB triangle in LDS, and publishes.  Forward rows wait only on
// smaller forward rows and backward rows only on forward rows and larger backward rows, and
// every workgroup finishes its forward list first, so with all workgroups resident the
// dependency graph always has a runnable item (bounded spins + an error word besides).
constexpr int kDB = 64;
__device__ __forceinline__ double readlane_s(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), src);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ cplx readlane_s(cplx v, int src) { return cplx{readlane_s(v.re, src), readlane_s(v.im, src)}; }
__device__ __forceinline__ float readlane_s(float v, int src) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src));
}
__device__ __forceinline__ cplxf readlane_s(cplxf v, int src) { return cplxf{readlane_s(v.re, src), readlane_s(v.im, src)}; }
template <class S>
struct DenseTriArgs {
    const S* lu;
    const int32_t* perm;
    int64_t n;
    int32_t nblk;
    int32_t epoch;
    int32_t* flag_f;     // [nblk] epoch when z of the block row is published
    int32_t* flag_b;     // [nblk] epoch when y of the block row is published
    const S* tinv;       // dense_trsv2_kernel: [nblk][2] inv(L_kk), inv(U_kk), 64 x 64 column-major
    const S* tmul;       // [nblk][2] inv(L_rr) L_{r,r-1}, inv(U_rr) U_{r,r+1} (dense_tmul_kernel)
    S* z;                // forward results (n)
    const S* b_plain;
    S* y_plain;
    S* buf0;
    S* buf1;
    PowerCtl* ctl;
    const part4* rank_part;
    part4* my_part;
    part4* wave_part;    // [grid] workgroup partials
    uint32_t* work;
    int32_t* err;
    S* trace;
    double sig_re, sig_im;
};

__device__ __forceinline__ void wait_flag(const int32_t* f, int32_t epoch, int32_t* err) {
    int spins = 0;
    while (__hip_atomic_load(const_cast<int32_t*>(f), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
        // back off: waves far ahead of the chain leave the memory system to the producers
        if (spins < 4) __builtin_amdgcn_s_sleep(2);
        else if (spins < 16) __builtin_amdgcn_s_sleep(8);
        else __builtin_amdgcn_s_sleep(32);
        if (++spins > (1 << 22)) { atomicOr(err, 1); break; }
    }
}

template <class S, bool kIter>
__global__ __launch_bounds__(256) void dense_trsv_kernel(DenseTriArgs<S> a, int parity) {
    __shared__ S tri[kDB * (kDB + 1)];     // the block row's diagonal tile (odd pitch)
    __shared__ S part[4][kDB];             // per-wave partial sums of the off-diagonal tiles
    __shared__ S zsh[4][kDB];              // per-wave copy of the block of z / y a tile multiplies
    __shared__ S vec[kDB];
    __shared__ Prologue pro;
    __shared__ int s_last;
    const S* xin;
    S* yout;
    double nrm = 0.0;
    if constexpr (kIter) {
        shift_prologue<S>(a.ctl, a.rank_part, parity, a.trace, a.sig_re, a.sig_im, &pro);
        if (!__builtin_amdgcn_readfirstlane(pro.go)) return;   // epoch flags: nothing to reset
        nrm = pro.nrm;
        xin = parity ? a.buf0 : a.buf1;
        yout = parity ? a.buf1 : a.buf0;
    } else {
        xin = a.b_plain;
        yout = a.y_plain;
    }
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t n = a.n;
    const int G = gridDim.x;
    double n2 = 0.0, pr = 0.0, pi = 0.0;
    for (int phase = 0; phase < 2; ++phase) {
        const bool fwd = phase == 0;
        // this workgroup's block rows: r = blockIdx.x + k G, forward increasing, backward decreasing
        const int cnt = a.nblk > (int)blockIdx.x ? (a.nblk - 1 - (int)blockIdx.x) / G + 1 : 0;
        for (int q = 0; q < cnt; ++q) {
            const int r = fwd ? (int)blockIdx.x + q * G : (int)blockIdx.x + (cnt - 1 - q) * G;
            const int64_t r0 = (int64_t)r * kDB;
            const int rn = (int)min<int64_t>(kDB, n - r0);
            // diagonal tile into LDS (column-major, pitch kDB + 1): all 16 loads of a thread first
            {
                constexpr int kPer = kDB * kDB / 256;
                S tv[kPer];
#pragma unroll
                for (int q = 0; q < kPer; ++q) {
                    const int e = tid + 256 * q, i = e % kDB, j = e / kDB;
                    tv[q] = a.lu[(r0 + min(i, rn - 1)) + (r0 + min(j, rn - 1)) * n];
                }
#pragma unroll
                for (int q = 0; q < kPer; ++q) {
                    const int e = tid + 256 * q, i = e % kDB, j = e / kDB;
                    tri[i + j * (kDB + 1)] = (i < rn && j < rn) ? tv[q] : s_zero<S>();
                }
            }
            // off-diagonal tiles: forward c < r (L), backward c > r (U); wave wv takes every 4th
            S acc = s_zero<S>();
            const int c_beg = fwd ? 0 : r + 1, c_end = fwd ? r : a.nblk;
            for (int c = c_beg + wv; c < c_end; c += 4) {
                wait_flag(fwd ? a.flag_f + c : a.flag_b + c, a.epoch, a.err);
                const int64_t c0 = (int64_t)c * kDB;
                const int cn = (int)min<int64_t>(kDB, n - c0);
                const S* src = fwd ? a.z : yout;
                // the published block of z (or y): one coherent load per lane, broadcast from LDS
                zsh[wv][lane] = lane < cn ? ld_coh(src + c0 + lane) : s_zero<S>();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const S* tile = a.lu + c0 * n + r0 + min(lane, max(rn - 1, 0));
                if (cn == kDB) {
                    // 16 tile columns in flight per lane before the FMAs consume them
#pragma unroll
                    for (int j0 = 0; j0 < kDB; j0 += 16) {
                        S tv[16];
#pragma unroll
                        for (int u = 0; u < 16; ++u) tv[u] = tile[(int64_t)(j0 + u) * n];
#pragma unroll
                        for (int u = 0; u < 16; ++u) acc = add(acc, mul(tv[u], zsh[wv][j0 + u]));
                    }
                } else {
                    for (int j = 0; j < cn; ++j) acc = add(acc, mul(tile[(int64_t)j * n], zsh[wv][j]));
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
            }
            part[wv][lane] = lane < rn ? acc : s_zero<S>();
            __syncthreads();
            if (wv == 0) {
                // right-hand side of the block row
                S rhs = s_zero<S>();
                if (lane < rn) {
                    if (fwd) {
                        rhs = xin[a.perm[r0 + lane]];
                        if constexpr (kIter) rhs = scale_in(rhs, nrm);
                    } else {
                        rhs = ld_coh(a.z + r0 + lane);   // published by this wave, read past L1
                    }
                    rhs = sub(rhs, add(add(part[0][lane], part[1][lane]), add(part[2][lane], part[3][lane])));
                }
                vec[lane] = rhs;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                // triangle: forward unit lower (column order), backward upper (reverse column order)
                // the solved entry travels by v_readlane (wave-uniform j), the tile column from LDS
                S v = vec[lane];
                auto step = [&](const int j) {
                    S zj;
                    if (!fwd && lane == j) v = sdiv(v, tri[j + j * (kDB + 1)]);
                    zj = readlane_s(v, j);
                    const bool below = fwd ? (lane > j) : (lane < j);
                    const S lij = tri[lane + j * (kDB + 1)];
                    if (below) v = sub(v, mul(lij, zj));
                };
                if (rn == kDB) {
                    if (fwd) {
#pragma unroll
                        for (int j = 0; j < kDB; ++j) step(j);
                    } else {
#pragma unroll
                        for (int j = kDB - 1; j >= 0; --j) step(j);
                    }
                } else {
                    for (int jj = 0; jj < rn; ++jj) step(fwd ? jj : rn - 1 - jj);
                }
                if (lane < rn) {
                    if (fwd) {
                        st_coh(a.z + r0 + lane, v);
                    } else {
                        const S yi = v;
                        st_coh(yout + r0 + lane, yi);
                        if constexpr (kIter) {
                            S xi = xin[r0 + lane];
                            xi = scale_in(xi, nrm);
                            n2 += sq_abs(yi);
                            acc_dot(pr, pi, xi, yi);
                        }
                    }
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0)
                    __hip_atomic_store(fwd ? a.flag_f + r : a.flag_b + r, a.epoch, __ATOMIC_RELEASE,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
            __syncthreads();
        }
    }
    // workgroup partials (wave 0 holds them), then the last arriver sums them in workgroup order
    if (wv == 0) {
        n2 = wave_sum(n2);
        pr = wave_sum(pr);
        pi = wave_sum(pi);
        if (lane == 0) {
            part4* p = a.wave_part + blockIdx.x;
            st_agent(&p->a, n2);
            st_agent(&p->b, pr);
            st_agent(&p->c, pi);
        }
    }
    __syncthreads();
    if (tid == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t tk = __hip_atomic_fetch_add(&a.work[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (tk == gridDim.x - 1) ? 1 : 0;
    }
    __syncthreads();
    if (!s_last) return;
    if constexpr (kIter) {
        if (tid == 0) {
            double sa = 0.0, sb = 0.0, sc = 0.0;
            for (int i = 0; i < G; ++i) {
                sa += ld_agent(&a.wave_part[i].a);
                sb += ld_agent(&a.wave_part[i].b);
                sc += ld_agent(&a.wave_part[i].c);
            }
            a.my_part->a = sa;
            a.my_part->b = sb;
            a.my_part->c = sc;
            a.my_part->d = 0.0;
        }
    }
    if (tid == 0) __hip_atomic_store(&a.work[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Inverted diagonal blocks of a dense LU factor (after the factorization; one workgroup per block and
// triangle): tinv + 4096 (2 k) = inv(L_kk) (unit lower), tinv + 4096 (2 k + 1) = inv(U_kk), 64 x 64
// column-major, the identity past a partial last block.  Wave w solves for the 16 unit vectors
// e_{16 w} .. e_{16 w + 15} at once, lane = row, the solved entry broadcast by v_readlane.
template <class S>
__global__ __launch_bounds__(256) void dense_tinv_kernel(const S* lu, int64_t n, S* tinv) {
    __shared__ S tri[kDB * (kDB + 1)];
    const int k = blockIdx.x, upper = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t r0 = (int64_t)k * kDB;
    const int rn = (int)min<int64_t>(kDB, n - r0);
    for (int e = tid; e < kDB * kDB; e += 256) {
        const int i = e % kDB, j = e / kDB;
        S v = s_zero<S>();
        if (i < rn && j < rn) v = lu[(r0 + i) + (r0 + j) * n];
        else if (i == j) set_re_im(v, 1.0, 0.0);
        tri[i + j * (kDB + 1)] = v;
    }
    __syncthreads();
    S v[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        v[t] = s_zero<S>();
        if (lane == 16 * wv + t) set_re_im(v[t], 1.0, 0.0);
    }
    if (!upper) {
        for (int j = 0; j < kDB; ++j) {
            const S lij = tri[lane + j * (kDB + 1)];
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const S zj = readlane_s(v[t], j);
                if (lane > j) v[t] = sub(v[t], mul(lij, zj));
            }
        }
    } else {
        for (int j = kDB - 1; j >= 0; --j) {
            const S ujj = tri[j + j * (kDB + 1)];
            const S uij = tri[lane + j * (kDB + 1)];
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                if (lane == j) v[t] = sdiv(v[t], ujj);
                const S zj = readlane_s(v[t], j);
                if (lane < j) v[t] = sub(v[t], mul(uij, zj));
            }
        }
    }
    S* out = tinv + (int64_t)(2 * k + upper) * kDB * kDB;
#pragma unroll
    for (int t = 0; t < 16; ++t) out[(16 * wv + t) * kDB + lane] = v[t];
}

// The premultiplied next-to-diagonal tiles of dense_trsv2_kernel's dense_pf 2: tmul + 4096 (2 r) =
// inv(L_rr) L_{r,r-1} (r >= 1), tmul + 4096 (2 r + 1) = inv(U_rr) U_{r,r+1} (r <= nblk - 2), 64 x 64
// column-major, rows past a partial last block and columns past a partial next block zero.  Thread =
// one column, 16 rows.
template <class S>
__global__ __launch_bounds__(256) void dense_tmul_kernel(const S* lu, const S* tinv, int64_t n, int nblk, S* tmul) {
    __shared__ S ti[kDB * (kDB + 1)];
    __shared__ S tl[kDB * (kDB + 1)];
    const int r = blockIdx.x, upper = blockIdx.y;
    const int tid = threadIdx.x;
    S* out = tmul + (int64_t)(2 * r + upper) * kDB * kDB;
    const int c = upper ? r + 1 : r - 1;
    if (c < 0 || c >= nblk) {
        for (int e = tid; e < kDB * kDB; e += 256) out[e] = s_zero<S>();
        return;
    }
    const int64_t r0 = (int64_t)r * kDB, c0 = (int64_t)c * kDB;
    const int rn = (int)min<int64_t>(kDB, n - r0), cn = (int)min<int64_t>(kDB, n - c0);
    const S* tv = tinv + (int64_t)(2 * r + upper) * kDB * kDB;
    for (int e = tid; e < kDB * kDB; e += 256) {
        const int i = e % kDB, j = e / kDB;
        ti[i + j * (kDB + 1)] = tv[e];
        tl[i + j * (kDB + 1)] = (i < rn && j < cn) ? lu[(r0 + i) + (c0 + j) * n] : s_zero<S>();
    }
    __syncthreads();
    const int j = tid & 63, i0 = (tid >> 6) * 16;
    S o[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) o[t] = s_zero<S>();
    for (int k = 0; k < kDB; ++k) {
        const S b = tl[k + j * (kDB + 1)];
#pragma unroll
        for (int t = 0; t < 16; ++t) o[t] = add(o[t], mul(ti[(i0 + t) + k * (kDB + 1)], b));
    }
#pragma unroll
    for (int t = 0; t < 16; ++t) out[(i0 + t) + j * kDB] = o[t];
}

// The multi-CU substitution with the diagonal blocks applied as products with their inverses
// (dense_tinv_kernel) and every off-diagonal tile loaded before its block's flag is awaited (the
// multifrontal row-block solve's scheme, mf_big_fwd_kernel).  A block row: each wave takes 16 columns
// of every column block - forward c = 0 .. r - 1, backward c = nblk - 1 .. r + 1 - loads its 64 x 16
// piece of the tile, polls the block's 16 published values (value flags, below), and accumulates;
// then t = rhs - sum, y = inv(T_rr) t as four 64 x 16 products from registers, published by 64
// write-through stores.  The per-block hand-off is one store and one poll instead of the 64-step
// triangle of dense_trsv_kernel and its epoch flag.  Workgroups take block rows round-robin like it.
// value flags of dense_trsv2_kernel: an unsolved entry holds this NaN in every 8-byte word, a solved one
// never does (a NaN result is stored as the default quiet NaN), so a waiting wave polls the values
// themselves.  Two buffers alternate by the launch's epoch: a launch solves in one and resets its own
// rows of the other for the next launch (no reader of the other buffer is running).
constexpr unsigned long long kDnSent = 0x7FF4DEAD7FF4DEADull;
__device__ __forceinline__ bool dn_unready(double v) { return (unsigned long long)__double_as_longlong(v) == kDnSent; }
__device__ __forceinline__ bool dn_unready(cplx v) { return dn_unready(v.re) || dn_unready(v.im); }
__device__ __forceinline__ bool dn_unready(float v) { return (unsigned)__float_as_int(v) == (unsigned)(kDnSent & 0xffffffffu); }
__device__ __forceinline__ bool dn_unready(cplxf v) { return dn_unready(v.re) || dn_unready(v.im); }
template <class S>
__device__ __forceinline__ S dn_sent() {
    S v;
    if constexpr (std::is_same_v<S, double>) v = __longlong_as_double((long long)kDnSent);
    else if constexpr (std::is_same_v<S, cplx>) v = cplx{__longlong_as_double((long long)kDnSent), __longlong_as_double((long long)kDnSent)};
    else if constexpr (std::is_same_v<S, float>) v = __int_as_float((int)(kDnSent & 0xffffffffu));
    else v = cplxf{__int_as_float((int)(kDnSent & 0xffffffffu)), __int_as_float((int)(kDnSent & 0xffffffffu))};
    return v;
}
__device__ __forceinline__ double dn_clean(double v) { return v != v ? __longlong_as_double(0x7FF8000000000000ll) : v; }
__device__ __forceinline__ cplx dn_clean(cplx v) { return cplx{dn_clean(v.re), dn_clean(v.im)}; }
__device__ __forceinline__ float dn_clean(float v) { return v != v ? __int_as_float(0x7FC00000) : v; }
__device__ __forceinline__ cplxf dn_clean(cplxf v) { return cplxf{dn_clean(v.re), dn_clean(v.im)}; }
template <class S>
__device__ __forceinline__ S dn_poll(const S* p, int32_t* err) {
    S v = ld_coh(p);
    int spins = 0;
    while (dn_unready(v)) {
        __builtin_amdgcn_s_sleep(1);
        v = ld_coh(p);
        if (++spins > (1 << 24)) {
            atomicOr(err, 1);
            break;
        }
    }
    return v;
}

template <class S, bool kIter, int kPf>
__global__ __launch_bounds__(256) void dense_trsv2_kernel(DenseTriArgs<S> a, int parity) {
    __shared__ S part[4][kDB];
    __shared__ S part2[4][kDB];
    __shared__ S zsh[4][16];
    __shared__ S vec[kDB];
    __shared__ Prologue pro;
    __shared__ int s_last;
    const S* xin;
    S* yout;
    double nrm = 0.0;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t n = a.n;
    const int G = gridDim.x;
    const int cnt = a.nblk > (int)blockIdx.x ? (a.nblk - 1 - (int)blockIdx.x) / G + 1 : 0;
    // a.z: [z | z' | y | y'] value buffers; this launch solves in (z, y) of its epoch's parity and
    // resets its own rows of the other pair for the next launch (also when the iteration has stopped)
    const int64_t pp = a.epoch & 1;
    S* zcur = a.z + pp * n;
    S* ycur = a.z + (2 + pp) * n;
    {
        S* znext = a.z + (1 - pp) * n;
        S* ynext = a.z + (3 - pp) * n;
        const S sent = dn_sent<S>();
        for (int q = 0; q < cnt; ++q) {
            const int64_t r0 = (int64_t)((int)blockIdx.x + q * G) * kDB;
            if (tid < kDB && r0 + tid < n) {
                st_coh(znext + r0 + tid, sent);
                st_coh(ynext + r0 + tid, sent);
            }
        }
    }
    if constexpr (kIter) {
        shift_prologue<S>(a.ctl, a.rank_part, parity, a.trace, a.sig_re, a.sig_im, &pro);
        if (!__builtin_amdgcn_readfirstlane(pro.go)) return;
        nrm = pro.nrm;
        xin = parity ? a.buf0 : a.buf1;
        yout = parity ? a.buf1 : a.buf0;
    } else {
        xin = a.b_plain;
        yout = a.y_plain;
    }
    double n2 = 0.0, pr = 0.0, pi = 0.0;
    for (int phase = 0; phase < 2; ++phase) {
        const bool fwd = phase == 0;
        for (int q = 0; q < cnt; ++q) {
            const int r = fwd ? (int)blockIdx.x + q * G : (int)blockIdx.x + (cnt - 1 - q) * G;
            const int64_t r0 = (int64_t)r * kDB;
            const int rn = (int)min<int64_t>(kDB, n - r0);
            const int64_t row = r0 + min(lane, rn - 1);
            // this wave's 16 columns of the inverted diagonal block, and the block row's right-hand side
            S iv[16];
            {
                const S* ti = a.tinv + (int64_t)(2 * r + (fwd ? 0 : 1)) * kDB * kDB + (16 * wv) * kDB + lane;
#pragma unroll
                for (int t = 0; t < 16; ++t) iv[t] = ti[t * kDB];
            }
            S rhs = s_zero<S>();
            if (wv == 0 && lane < rn) {
                if (fwd) {
                    rhs = xin[a.perm[r0 + lane]];
                    if constexpr (kIter) rhs = scale_in(rhs, nrm);
                } else {
                    rhs = dn_poll(zcur + r0 + lane, a.err);   // published by this workgroup in the forward phase
                }
            }
            S acc = s_zero<S>();
            const int nc = fwd ? r : a.nblk - 1 - r;
            // dense_pf 2: the block next to the diagonal enters as a product with the premultiplied tile
            // inv(T_rr) T_{r, r -/+ 1} (dense_tmul_kernel) after y' = inv(T_rr) (rhs - the other blocks)
            // is formed, so the chain's hand-off is followed by one 64 x 64 product instead of two
            const bool premul = kPf == 2 && nc > 0;
            const int nacc = premul ? nc - 1 : nc;
            const S* src = fwd ? zcur : ycur;
            const int j0 = 16 * wv;
            const S* tile = a.lu + row;
            // this wave's 64 x 16 piece of column block m's tile
            auto load_tile = [&](int m, S* tv) {
                const int c = fwd ? m : a.nblk - 1 - m;
                const int64_t c0 = (int64_t)c * kDB;
                const int cn = (int)min<int64_t>(kDB, n - c0);
#pragma unroll
                for (int t = 0; t < 16; ++t) tv[t] = tile[(c0 + min(j0 + t, cn - 1)) * n];
            };
            if constexpr (kPf >= 1) {
                // software-pipelined (default): the first poll of block m's values is issued before the
                // loads of tile m + 1, so the poll's wait leaves those in flight and a wave behind the
                // chain streams its tiles instead of paying one load latency per block; the same
                // products in the same order (bitwise the unpipelined loop)
                S tv[16], tn[16];
                if (nacc > 0) load_tile(0, tv);
                for (int m = 0; m < nacc; ++m) {
                    const int c = fwd ? m : a.nblk - 1 - m;
                    const int64_t c0 = (int64_t)c * kDB;
                    const int cn = (int)min<int64_t>(kDB, n - c0);
                    const bool mine = lane < 16 && j0 + lane < cn;
                    S zv = s_zero<S>();
                    if (mine) zv = ld_coh(src + c0 + j0 + lane);
                    if (m + 1 < nacc) load_tile(m + 1, tn);
                    if (mine) {
                        int spins = 0;
                        while (dn_unready(zv)) {
                            __builtin_amdgcn_s_sleep(1);
                            zv = ld_coh(src + c0 + j0 + lane);
                            if (++spins > (1 << 24)) {
                                atomicOr(a.err, 1);
                                break;
                            }
                        }
                    }
                    if (lane < 16) zsh[wv][lane] = zv;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                    for (int t = 0; t < 16; ++t) acc = add(acc, mul(tv[t], zsh[wv][t]));
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (int t = 0; t < 16; ++t) tv[t] = tn[t];
                }
            } else {
                for (int m = 0; m < nc; ++m) {
                    const int c = fwd ? m : a.nblk - 1 - m;
                    const int64_t c0 = (int64_t)c * kDB;
                    const int cn = (int)min<int64_t>(kDB, n - c0);
                    S tv[16];
                    load_tile(m, tv);
                    if (lane < 16) zsh[wv][lane] = j0 + lane < cn ? dn_poll(src + c0 + j0 + lane, a.err) : s_zero<S>();
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                    for (int t = 0; t < 16; ++t) acc = add(acc, mul(tv[t], zsh[wv][t]));
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                }
            }
            // premultiplied step: its tile piece and the first poll of its values issued now, under the
            // reductions below
            S tm[16];
            S zl = s_zero<S>();
            int64_t lc0 = 0;
            bool lmine = false;
            if (premul) {
                const int c = fwd ? r - 1 : r + 1;
                lc0 = (int64_t)c * kDB;
                const int cn = (int)min<int64_t>(kDB, n - lc0);
                lmine = lane < 16 && j0 + lane < cn;
                if (lmine) zl = ld_coh(src + lc0 + j0 + lane);
                const S* tmp = a.tmul + (int64_t)(2 * r + (fwd ? 0 : 1)) * kDB * kDB + j0 * kDB + lane;
#pragma unroll
                for (int t = 0; t < 16; ++t) tm[t] = tmp[t * kDB];
            }
            part[wv][lane] = acc;
            __syncthreads();
            if (wv == 0)
                vec[lane] = lane < rn ? sub(rhs, add(add(part[0][lane], part[1][lane]), add(part[2][lane], part[3][lane])))
                                      : s_zero<S>();
            __syncthreads();
            S p = s_zero<S>();
#pragma unroll
            for (int t = 0; t < 16; ++t) p = add(p, mul(iv[t], vec[16 * wv + t]));
            part[wv][lane] = p;
            __syncthreads();
            S y = s_zero<S>();
            if (wv == 0) y = add(add(part[0][lane], part[1][lane]), add(part[2][lane], part[3][lane]));
            if (premul) {
                if (lmine) {
                    int spins = 0;
                    while (dn_unready(zl)) {
                        __builtin_amdgcn_s_sleep(1);
                        zl = ld_coh(src + lc0 + j0 + lane);
                        if (++spins > (1 << 24)) {
                            atomicOr(a.err, 1);
                            break;
                        }
                    }
                }
                if (lane < 16) zsh[wv][lane] = zl;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                S q = s_zero<S>();
#pragma unroll
                for (int t = 0; t < 16; ++t) q = add(q, mul(tm[t], zsh[wv][t]));
                part2[wv][lane] = q;
                __syncthreads();
                if (wv == 0) y = sub(y, add(add(part2[0][lane], part2[1][lane]), add(part2[2][lane], part2[3][lane])));
            }
            if (wv == 0) {
                if (lane < rn) {
                    // publish (the value is its own flag)
                    if (fwd) {
                        st_coh(zcur + r0 + lane, dn_clean(y));
                    } else {
                        st_coh(ycur + r0 + lane, dn_clean(y));
                        yout[r0 + lane] = y;
                        if constexpr (kIter) {
                            S xi = xin[r0 + lane];
                            xi = scale_in(xi, nrm);
                            n2 += sq_abs(y);
                            acc_dot(pr, pi, xi, y);
                        }
                    }
                }
            }
            __syncthreads();
        }
    }
    // workgroup partials (wave 0 holds them), then the last arriver sums them in workgroup order
    if (wv == 0) {
        n2 = wave_sum(n2);
        pr = wave_sum(pr);
        pi = wave_sum(pi);
        if (lane == 0) {
            part4* pp = a.wave_part + blockIdx.x;
            st_agent(&pp->a, n2);
            st_agent(&pp->b, pr);
            st_agent(&pp->c, pi);
        }
    }
    __syncthreads();
    if (tid == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t tk = __hip_atomic_fetch_add(&a.work[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (tk == gridDim.x - 1) ? 1 : 0;
    }
    __syncthreads();
    if (!s_last) return;
    if constexpr (kIter) {
        if (tid == 0) {
            double sa = 0.0, sb = 0.0, sc = 0.0;
            for (int i = 0; i < G; ++i) {
                sa += ld_agent(&a.wave_part[i].a);
                sb += ld_agent(&a.wave_part[i].b);
                sc += ld_agent(&a.wave_part[i].c);
            }
            a.my_part->a = sa;
            a.my_part->b = sb;
            a.my_part->c = sc;
            a.my_part->d = 0.0;
        }
    }
    if (tid == 0) __hip_atomic_store(&a.work[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// CSR (device) -> dense column-major (device), for small non-triangular sparse matrices
template <class S>
__global__ void densify_kernel(const int32_t* rowptr, const int32_t* col, const S* val, int64_t n,
                               S* out) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    for (int e = rowptr[r]; e < rowptr[r + 1]; ++e) out[(int64_t)col[e] * n + r] = val[e];
}

template <class S>
__global__ void shift_diag_kernel(S* a, int64_t n, S sigma) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) a[i * n + i] = sub(a[i * n + i], sigma);
}

// ---- on-device analysis of a triangular CSR (factor_tri_device): the same level order and the same
// position-indexed chunk layout the host build produces, without moving the matrix off the device.

// Per row: pivot d_i - sigma (the diagonal entries summed in stored order, 0 where there is none),
// off-diagonal count, and the triangularity / zero-pivot flags (flags[0]: an entry left of the
// diagonal, [1]: right of it, [2]: a zero pivot), one atomic per wave.
template <class S>
__global__ __launch_bounds__(256) void tri_rows_kernel(const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                       const S* __restrict__ val, int64_t n, S sig,
                                                       S* __restrict__ pv, int32_t* __restrict__ offlen,
                                                       int32_t* __restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool lo = false, hi = false, zp = false;
    if (i < n) {
        S d = s_zero<S>();
        int32_t off = 0;
        for (int32_t e = rp[i]; e < rp[i + 1]; ++e) {
            const int32_t c = ci[e];
            if (c == i) d = add(d, val[e]);
            else {
                ++off;
                lo |= c < i;
                hi |= c > i;
            }
        }
        const S p = sub(d, sig);
        pv[i] = p;
        offlen[i] = off;
        if constexpr (std::is_same_v<S, double> || std::is_same_v<S, float>) zp = p == 0;
        else zp = p.re == 0 && p.im == 0;
    }
    const uint64_t bl = __ballot(lo), bh = __ballot(hi), bz = __ballot(zp);
    if ((threadIdx.x & 63) == 0) {
        if (bl) atomicOr(flags + 0, 1);
        if (bh) atomicOr(flags + 1, 1);
        if (bz) atomicOr(flags + 2, 1);
    }
}

// Dependency levels, sync-free: level(i) = 1 + max level of the rows row i reads (0 for none).
// Rows are claimed in dependency order through a ticket (upper: row n-1 first), four rows per wave
// (16 lanes per row); a row's dependencies always hold smaller tickets, claimed by waves that are
// already running, so every wait ends.  A wave re-polls its unfinished rows' dependencies
// (agent-scope loads, -1 = not yet known) and publishes a row as soon as all of them are known,
// inside the loop (a divergent group must never wait on a row its own wave publishes after the
// loop).  Per level: row count and longest row (atomics); maxlev = the deepest level.  A wait past
// ~2 s of the 100 MHz constant clock sets err and publishes level 0, so a broken analysis ends
// (the host then builds on the CPU).
__global__ __launch_bounds__(256) void tri_level_kernel(const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                        const int32_t* __restrict__ offlen, int64_t n, int upper,
                                                        int32_t* lev, uint32_t* ticket, int32_t* lcnt,
                                                        int32_t* lmax, int32_t* maxlev, int32_t* err) {
    const int lane = threadIdx.x & (kRowLanes - 1);
    const int grp = (threadIdx.x & 63) / kRowLanes;
    for (;;) {
        uint32_t t0 = 0;
        if ((threadIdx.x & 63) == 0) t0 = atomicAdd(ticket, (uint32_t)kWaveRows);
        t0 = __shfl(t0, 0, 64);
        if ((int64_t)t0 >= n) return;
        const int64_t t = (int64_t)t0 + grp;
        const bool live = t < n;
        const int64_t i = live ? (upper ? n - 1 - t : t) : 0;
        const int32_t e0 = live ? rp[i] : 0, e1 = live ? rp[i + 1] : 0;
        bool done = !live;
        const long long t_start = wall_clock64();
        for (;;) {
            int32_t m = -1;
            bool ready = true;
            if (!done)
                for (int32_t e = e0 + lane; e < e1; e += kRowLanes) {
                    const int32_t c = ci[e];
                    if (c == i) continue;
                    const int32_t l = __hip_atomic_load(lev + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (l < 0) ready = false;
                    m = max(m, l);
                }
            // the row's 16 lanes: all ready (ballot), and the largest dependency level (every lane
            // shuffles: a shuffle under a divergent mask would read inactive lanes' stale registers)
#pragma unroll
            for (int off = kRowLanes / 2; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off, 64));
            const uint64_t unready = __ballot(!ready);
            ready = ((unready >> (grp * kRowLanes)) & ((1ull << kRowLanes) - 1)) == 0;
            bool timeout = false;
            if (!done && !ready && wall_clock64() - t_start > 200000000ll) {
                timeout = true;
                ready = true;
                m = -1;
            }
            if (!done && ready) {
                if (lane == 0) {
                    if (timeout) atomicOr(err, 1);
                    const int32_t l = m + 1;
                    __hip_atomic_store(lev + i, l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    atomicAdd(lcnt + l, 1);
                    atomicMax(lmax + l, offlen[i]);
                    atomicMax(maxlev, l);
                }
                done = true;
            }
            if (__ballot(!done) == 0) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

// position -> row: the rows sorted by level (stable: ascending row inside a level) placed at their
// level's padded start; padding positions stay -1
__global__ __launch_bounds__(256) void tri_order_kernel(const int32_t* __restrict__ lev_sorted,
                                                        const int32_t* __restrict__ rows_sorted, int64_t n,
                                                        const int32_t* __restrict__ ustart,
                                                        const int32_t* __restrict__ pstart, int32_t* __restrict__ order) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    const int32_t l = lev_sorted[k];
    order[pstart[l] + (k - ustart[l])] = rows_sorted[k];
}

// per position: its row's off-diagonal count (plen[npos] = 0 closes the scan) and its pivot
template <class S>
__global__ __launch_bounds__(256) void tri_poslen_kernel(const int32_t* __restrict__ order, int64_t npos,
                                                         const int32_t* __restrict__ offlen, const S* __restrict__ pv,
                                                         S one, int32_t* __restrict__ plen, S* __restrict__ ppiv) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p > npos) return;
    if (p == npos) {
        plen[p] = 0;
        return;
    }
    const int32_t i = order[p];
    plen[p] = i >= 0 ? offlen[i] : 0;
    ppiv[p] = i >= 0 ? pv[i] : one;
}

// the position-ordered off-diagonal CSR: 16 lanes per position copy its row's entries (diagonal
// skipped, stored order kept) to pptr[p]
template <class S>
__global__ __launch_bounds__(256) void tri_gather_kernel(const int32_t* __restrict__ order, int64_t npos,
                                                         const int32_t* __restrict__ pptr,
                                                         const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                         const S* __restrict__ val, const int32_t* __restrict__ offlen,
                                                         int32_t* __restrict__ pcol, S* __restrict__ pval) {
    const int64_t p = ((int64_t)blockIdx.x * 256 + threadIdx.x) / kRowLanes;
    const int lane = threadIdx.x & (kRowLanes - 1);
    if (p >= npos) return;
    const int32_t i = order[p];
    if (i < 0) return;
    const int32_t e0 = rp[i], len = rp[i + 1] - e0, nd = len - offlen[i], base = pptr[p];
    for (int32_t k = lane; k < len; k += kRowLanes) {
        const int32_t c = ci[e0 + k];
        if (c == i) continue;
        const int32_t o = base + (c < i ? k : k - nd);
        pcol[o] = c;
        pval[o] = val[e0 + k];
    }
}

// head rows: row -> head position (their columns become LDS positions)
__global__ __launch_bounds__(256) void tri_rowpos_kernel(const int32_t* __restrict__ order, int32_t hpos,
                                                         int32_t* __restrict__ rowpos) {
    const int32_t p = blockIdx.x * 256 + threadIdx.x;
    if (p >= hpos) return;
    const int32_t i = order[p];
    if (i >= 0) rowpos[i] = p;
}

// 1 / pivot as the host build forms it (complex: in double, no contraction), for bitwise-equal heads
__device__ __forceinline__ double head_recip(double p) { return 1.0 / p; }
__device__ __forceinline__ float head_recip(float p) { return 1.0f / p; }
__device__ __forceinline__ cplx head_recip(cplx p) {
#pragma clang fp contract(off)
    const double d = p.re * p.re + p.im * p.im;
    return cplx{p.re / d, -p.im / d};
}
__device__ __forceinline__ cplxf head_recip(cplxf p) {
#pragma clang fp contract(off)
    const double re = p.re, im = p.im;
    const double d = re * re + im * im;
    return cplxf{(float)(re / d), (float)(-im / d)};
}

// one-wave head, pass-major (see sptrsv_whead_kernel): thread (q, u) fills row u of pass q; the
// arrays arrive pre-filled with the padding (values 0, columns hpos, pivots 1, targets -1)
template <class S>
__global__ __launch_bounds__(256) void tri_whead_kernel(const int2* __restrict__ ptab, int32_t nreal,
                                                        const int32_t* __restrict__ order, const int32_t* __restrict__ rp,
                                                        const int32_t* __restrict__ ci, const S* __restrict__ val,
                                                        const S* __restrict__ pv, const int32_t* __restrict__ rowpos,
                                                        S* __restrict__ wval, int32_t* __restrict__ wcol,
                                                        S* __restrict__ wrp, int32_t* __restrict__ wdst) {
    const int32_t g = blockIdx.x * 256 + threadIdx.x;
    const int32_t q = g / kWHeadRows, u = g % kWHeadRows;
    if (q >= nreal) return;
    const int2 pt = ptab[q];   // {first position, rows}
    if (u >= pt.y) return;
    const int32_t p = pt.x + u;
    const int32_t i = order[p];
    wrp[(size_t)q * kWHeadRows + u] = head_recip(pv[i]);
    wdst[(size_t)q * kWHeadRows + u] = p;
    int32_t idx = 0;
    for (int32_t e = rp[i]; e < rp[i + 1]; ++e) {
        const int32_t c = ci[e];
        if (c == i) continue;
        const size_t slot = ((size_t)q * 4 + (size_t)(idx % 4)) * 64 + (size_t)(4 * u + idx / 4);
        wcol[slot] = rowpos[c];
        wval[slot] = val[e];
        ++idx;
    }
}

template <class T>
__global__ __launch_bounds__(256) void fill_kernel(T* __restrict__ a, int64_t n, T v) {
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256) a[k] = v;
}

template <class S, class W>
__global__ __launch_bounds__(256) void convert_kernel(const S* __restrict__ in, W* __restrict__ out, int64_t n) {
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        if constexpr (is_real_v<S>) out[i] = static_cast<W>(in[i]);
        else out[i] = W{static_cast<decltype(W{}.re)>(in[i].re), static_cast<decltype(W{}.im)>(in[i].im)};
    }
}

}  // namespace dev

// ================================================================== host side
// dense_trsv2_kernel's loop form (EIGSOL_DENSE_PF, read per call): 0 one tile load per block, 1 tile
// loads one block ahead, 2 (default) also the premultiplied next-to-diagonal block; each form is its own
// instantiation so the others' registers do not bound it
template <class S>
static const void* dense_trsv2_ptr(bool iter, int pf) {
    if (pf <= 0) return iter ? reinterpret_cast<const void*>(dev::dense_trsv2_kernel<S, true, 0>)
                             : reinterpret_cast<const void*>(dev::dense_trsv2_kernel<S, false, 0>);
    if (pf == 1) return iter ? reinterpret_cast<const void*>(dev::dense_trsv2_kernel<S, true, 1>)
                             : reinterpret_cast<const void*>(dev::dense_trsv2_kernel<S, false, 1>);
    return iter ? reinterpret_cast<const void*>(dev::dense_trsv2_kernel<S, true, 2>)
                : reinterpret_cast<const void*>(dev::dense_trsv2_kernel<S, false, 2>);
}
template <class S>
static int dense_pf_mode() {
    const char* e = std::getenv("EIGSOL_DENSE_PF");
    return e ? std::max(0, std::min(2, std::atoi(e))) : 2;
}
// the dense LU (and the densified / banded general-sparse paths) is built for every scalar: single
// precision factors and solves in float (rank-NB updates on v_mfma_f32_16x16x4_f32); ILU(0)-GMRES
// stays double-only
template <class S> inline constexpr bool kDenseLU = true;
template <class S> inline constexpr bool kGmres = std::is_same_v<S, double> || std::is_same_v<S, cplx>;
// single-precision matrices take the GMRES family (exact / multifrontal LU, ILU(0) + GMRES) on their
// values widened to double: the factor, the residual checks and the refinement run in double, the
// iterate stays in the matrix's precision (dtype >= the reference's SparseLU<float>)
template <class S> using GmresScalar = std::conditional_t<is_real_v<S>, double, cplx>;
int resident_blocks(eigsol_ctx* ctx, const void* kernel, int threads, size_t dyn_lds, int* grid);

template <class S>
static S make_sigma(double re, double im) {
    if constexpr (std::is_same_v<S, double>) { (void)im; return re; }
    else if constexpr (std::is_same_v<S, cplx>) return cplx{re, im};
    else if constexpr (std::is_same_v<S, float>) { (void)im; return (float)re; }
    else return cplxf{(float)re, (float)im};
}
// host arithmetic of the factor set-up (pivots d_i - sigma) in the scalar's own precision
template <class S> static S h_add(S a, S b) {
    if constexpr (is_real_v<S>) return a + b;
    else return S{a.re + b.re, a.im + b.im};
}
template <class S> static S h_sub(S a, S b) {
    if constexpr (is_real_v<S>) return a - b;
    else return S{a.re - b.re, a.im - b.im};
}
template <class S> static bool h_zero(S a) {
    if constexpr (is_real_v<S>) return a == 0;
    else return a.re == 0 && a.im == 0;
}

static void shift_free(ShiftFactor* f) {
    if (!f) return;
    if (f->gm) gmres_free(f->gm);
    if (f->band) band_free(f->band);
    if (f->src) csr_release(f->src);
    hipSetDevice(f->ctx->device);
    hipStreamSynchronize(f->ctx->stream);
    for (void* p : {(void*)f->order, f->z[0], f->z[1],
                    f->hval, (void*)f->hcol, f->hpiv, (void*)f->passes, (void*)f->smeta, (void*)f->trow,
                    f->wval, (void*)f->wcol, f->wrp, (void*)f->wdst,
                    f->tpiv, (void*)f->tcol, f->tval, (void*)f->porder, (void*)f->pptr, (void*)f->pcol, f->pval,
                    f->ppiv,
                    (void*)f->work, (void*)f->err, f->wave_part, f->lu, (void*)f->perm,
                    (void*)f->zero_pivot, (void*)f->flag_f, (void*)f->flag_b, f->zf, f->tinv, f->tmul,
                    f->kpart, f->kblk, f->promo})
        if (p) hipFree(p);
    for (int j = 0; j < dev::kMaxMulti; ++j) {
        if (j < dev::kMaxMulti - 1 && f->aux[j]) hipFree(f->aux[j]);
        for (void* zb : f->zm[j]) if (zb) hipFree(zb);
    }
    if (f->hpin) hipHostFree(f->hpin);
    ctx_release(f->ctx);
    delete f;
}

void shift_factor_free(ShiftFactor* f) { shift_free(f); }

template <class S>
static int64_t kDenseSingleMax() {
    const char* e = std::getenv("EIGSOL_DENSE_TRSV_SINGLE_MAX");   // A/B: substitution crossover
    if (e) return std::atoll(e);
    // round 6 (profiles/r06_dense_small.log): the block-row substitution beats the one-workgroup one from
    // n = 128 on (0.080 -> 0.030 ms per iteration at 128, 0.332 -> 0.047 ms at 512)
    return 64;
}

template <class S>
static int dense_lu_factor(ShiftFactor* f, bool from_sparse) {
    hipStream_t st = f->ctx->stream;
    const int64_t n = f->n;
    S* a = static_cast<S*>(f->lu);
    int32_t* piv = nullptr;
    EIGSOL_HIP(hipMalloc(&piv, n * sizeof(int32_t)));
    EIGSOL_HIP(hipMalloc(&f->zero_pivot, sizeof(int32_t)));
    EIGSOL_HIP(hipMemsetAsync(f->zero_pivot, 0xff, sizeof(int32_t), st));
    hipLaunchKernelGGL((dev::shift_diag_kernel<S>), dim3((n + 255) / 256), dim3(256), 0, st, a, n,
                       make_sigma<S>(f->sig_re, f->sig_im));
    // right-looking blocked LU with partial pivoting (LAPACK getrf order): per panel of NB columns,
    // column-by-column pivoting and rank-1 updates inside the panel, the panel's interchanges on
    // the other columns, U12 = L11^-1 A12, and A22 -= L21 U12 on the fp64 matrix cores
    constexpr int NB = dev::RankKMax<S>::value;
    for (int64_t k0 = 0; k0 < n; k0 += NB) {
        const int kb = (int)std::min<int64_t>(NB, n - k0);
        const int64_t c1 = k0 + kb;
        for (int64_t k = k0; k < c1; ++k) {
            hipLaunchKernelGGL((dev::lu_pivot_kernel<S>), dim3(1), dim3(1024), 0, st, a, n, k, k0, c1, piv,
                               f->zero_pivot);
            const int64_t m = n - k - 1, w = c1 - k - 1;
            if (m > 0 && w > 0)
                hipLaunchKernelGGL((dev::lu_update_kernel<S>), dim3((m * w + 255) / 256), dim3(256), 0, st, a, n, k, c1);
        }
        if (n - kb > 0)
            hipLaunchKernelGGL((dev::lu_laswp_kernel<S>), dim3((n - kb + 255) / 256), dim3(256), 0, st, a, n, k0, kb, piv);
        const int64_t rest = n - c1;
        if (rest > 0) {
            hipLaunchKernelGGL((dev::lu_trsm_kernel<S, NB>), dim3((rest + 255) / 256), dim3(256), 0, st, a, n, k0, kb);
            rankk_update<S, true>(st, (int)rest, (int)rest, kb, -1.0, a + c1 + k0 * n, n, a + k0 + c1 * n, n,
                                  a + c1 + c1 * n, n);
        }
    }
    EIGSOL_HIP(hipGetLastError());
    std::vector<int32_t> hp(n);
    int32_t zp = -1;
    EIGSOL_HIP(hipMemcpyAsync(hp.data(), piv, n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    EIGSOL_HIP(hipMemcpyAsync(&zp, f->zero_pivot, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    EIGSOL_HIP(hipStreamSynchronize(st));
    hipFree(piv);
    // a sparse matrix goes through SparseLU in the reference, which reports a singular matrix
    if (from_sparse && zp >= 0)
        return fail(EIGSOL_E_SOLVER, "solve_shifted: SparseLU factorization failed");
    // transpositions -> permutation: (P b)[i] = b[perm[i]]
    std::vector<int32_t> perm(n);
    for (int64_t i = 0; i < n; ++i) perm[i] = (int32_t)i;
    for (int64_t k = 0; k < n; ++k) std::swap(perm[k], perm[hp[k]]);
    EIGSOL_HIP(hipMalloc(&f->perm, n * sizeof(int32_t)));
    EIGSOL_HIP(hipMemcpyAsync(f->perm, perm.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, st));
    EIGSOL_HIP(hipStreamSynchronize(st));
    f->kind = 1;
    f->lds_bytes = (size_t)n * sizeof(S);
    if (n > kDenseSingleMax<S>()) {
        // multi-CU substitution: one persistent workgroup per CU at most (all resident)
        const int nblk = (int)((n + dev::kDB - 1) / dev::kDB);
        f->dense_multi = 1;
        f->grid = std::max(1, std::min(nblk, 32));   // 16384^2 f64: 32 WGs 32 ms, 64: 37 ms, 256: 48 ms per solve
        if (const char* e = std::getenv("EIGSOL_DENSE_TRSV_GRID")) f->grid = std::max(1, std::min(nblk, std::atoi(e)));
        f->nchunks = nblk;
        EIGSOL_HIP(hipMalloc(&f->flag_f, sizeof(int32_t) * nblk));
        EIGSOL_HIP(hipMalloc(&f->flag_b, sizeof(int32_t) * nblk));
        EIGSOL_HIP(hipMalloc(&f->zf, sizeof(S) * n));
        EIGSOL_HIP(hipMalloc(&f->work, 64));
        EIGSOL_HIP(hipMalloc(&f->err, 64));
        EIGSOL_HIP(hipMalloc(&f->wave_part, sizeof(dev::part4) * f->grid));
        EIGSOL_HIP(hipMemsetAsync(f->flag_f, 0, sizeof(int32_t) * nblk, st));
        EIGSOL_HIP(hipMemsetAsync(f->flag_b, 0, sizeof(int32_t) * nblk, st));
        EIGSOL_HIP(hipMemsetAsync(f->work, 0, 64, st));
        EIGSOL_HIP(hipMemsetAsync(f->err, 0, 64, st));
        // EIGSOL_DENSE_TRSV=1: round 5's substitution (64-step triangles on one wave, 32 workgroups)
        const char* dv = std::getenv("EIGSOL_DENSE_TRSV");
        f->dense_v = (dv && std::atoi(dv) == 1) ? 1 : 2;
        if (f->dense_v == 2) {
            // value buffers [z | z' | y | y'] (dense_trsv2_kernel), all unsolved
            hipFree(f->zf);
            f->zf = nullptr;
            EIGSOL_HIP(hipMalloc(&f->zf, sizeof(S) * 4 * n));
            EIGSOL_HIP(hipMemsetD32Async(static_cast<hipDeviceptr_t>(f->zf), 0x7FF4DEADu, sizeof(S) * n, st));
            EIGSOL_HIP(hipMalloc(&f->tinv, sizeof(S) * (size_t)nblk * 2 * dev::kDB * dev::kDB));
            hipLaunchKernelGGL((dev::dense_tinv_kernel<S>), dim3(nblk, 2), dim3(256), 0, st, static_cast<const S*>(f->lu),
                               n, static_cast<S*>(f->tinv));
            EIGSOL_HIP(hipGetLastError());
            EIGSOL_HIP(hipMalloc(&f->tmul, sizeof(S) * (size_t)nblk * 2 * dev::kDB * dev::kDB));
            hipLaunchKernelGGL((dev::dense_tmul_kernel<S>), dim3(nblk, 2), dim3(256), 0, st, static_cast<const S*>(f->lu),
                               static_cast<const S*>(f->tinv), n, nblk, static_cast<S*>(f->tmul));
            EIGSOL_HIP(hipGetLastError());
            // one block row per workgroup while they all fit on the device at once (a cooperative launch)
            // (the fewest resident over the loop forms, so a later EIGSOL_DENSE_PF still fits the grid)
            int per_cu = 1 << 20;
            for (int pf = 0; pf < 3; ++pf)
                for (int it = 0; it < 2; ++it) {
                    int o = 1;
                    EIGSOL_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, dense_trsv2_ptr<S>(it != 0, pf), 256, 0));
                    per_cu = std::min(per_cu, o);
                }
            f->grid = std::max(1, std::min(nblk, std::max(1, per_cu) * f->ctx->num_cus));
            if (const char* e = std::getenv("EIGSOL_DENSE_TRSV_GRID")) f->grid = std::max(1, std::min(nblk, std::atoi(e)));
            hipFree(f->wave_part);
            f->wave_part = nullptr;
            EIGSOL_HIP(hipMalloc(&f->wave_part, sizeof(dev::part4) * f->grid));
        }
        EIGSOL_HIP(hipStreamSynchronize(st));
    }
    return EIGSOL_OK;
}

// dense factors up to this order (vector in one CU's LDS) use the single-workgroup substitution,
// larger ones the multi-CU block-row substitution (dense_trsv_kernel); their size is bounded by HBM
static int dense_limits(int dtype, int64_t n, const char* who) {
    const double bytes = (double)n * (double)n * (double)scalar_bytes(dtype);
    if (n > INT32_MAX / 2 || bytes > 0.9 * 288e9)
        return fail(EIGSOL_E_UNSUPPORTED, std::string(who) + ": dense factor of order " + std::to_string(n) +
                                              " does not fit the device memory");
    return EIGSOL_OK;
}

template <class S>
static int factor_dense_t(eigsol_dense* A, double sre, double sim, ShiftFactor** out) {
    EIGSOL_TRY(dense_limits(A->dtype, A->nrows, "shifted solve"));
    auto* f = new ShiftFactor();
    f->ctx = A->ctx;
    ctx_retain(f->ctx);
    f->dtype = A->dtype;
    f->n = A->nrows;
    f->sig_re = sre;
    f->sig_im = sim;
    const size_t bytes = (size_t)f->n * f->n * sizeof(S);
    int rc = EIGSOL_OK;
    if (hipMalloc(&f->lu, bytes) != hipSuccess) rc = fail(EIGSOL_E_HIP, "hipMalloc(LU)");
    if (rc == EIGSOL_OK && hipMemcpyAsync(f->lu, A->a, bytes, hipMemcpyDeviceToDevice, f->ctx->stream) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "hipMemcpyAsync(LU)");
    if (rc == EIGSOL_OK) rc = dense_lu_factor<S>(f, false);
    if (rc != EIGSOL_OK) { shift_free(f); return rc; }
    *out = f;
    return EIGSOL_OK;
}

int shift_factor_dense(eigsol_dense* A, const void* sigma, ShiftFactor** out) {
    double s[2] = {0.0, 0.0};
    load_scalar(sigma, A->dtype, s[0], s[1]);
    EIGSOL_HIP(hipSetDevice(A->ctx->device));
    switch (A->dtype) {
        case EIGSOL_C128: return factor_dense_t<cplx>(A, s[0], s[1], out);
        case EIGSOL_F32: return factor_dense_t<float>(A, s[0], 0.0, out);
        case EIGSOL_C64: return factor_dense_t<cplxf>(A, s[0], s[1], out);
        default: return factor_dense_t<double>(A, s[0], 0.0, out);
    }
}

// Level analysis of a triangular pattern (host, once per matrix): level(i) = 1 + max level of
// the rows it reads; positions sorted by level, each level padded to a multiple of kWaveRows.
static void level_order(const std::vector<int32_t>& rp, const std::vector<int32_t>& ci, int64_t n,
                        bool upper, std::vector<int32_t>& order, int32_t& nlevels,
                        std::vector<int64_t>& lstart, std::vector<int64_t>& lcount) {
    std::vector<int32_t> lev(n, 0);
    int32_t maxl = 0;
    auto visit = [&](int64_t i) {
        int32_t l = 0;
        for (int32_t e = rp[i]; e < rp[i + 1]; ++e) l = std::max(l, lev[ci[e]] + 1);
        lev[i] = l;
        maxl = std::max(maxl, l);
    };
    if (upper) for (int64_t i = n - 1; i >= 0; --i) visit(i);
    else for (int64_t i = 0; i < n; ++i) visit(i);
    nlevels = maxl + 1;
    std::vector<int64_t> cnt(nlevels + 1, 0);
    for (int64_t i = 0; i < n; ++i) ++cnt[lev[i] + 1];
    std::vector<int64_t> start(nlevels + 1, 0);
    constexpr int64_t W = dev::kWaveRows;
    for (int32_t l = 0; l < nlevels; ++l) start[l + 1] = start[l] + ((cnt[l + 1] + W - 1) / W) * W;
    order.assign(start[nlevels], -1);
    std::vector<int64_t> fill(start.begin(), start.end() - 1);
    for (int64_t i = 0; i < n; ++i) order[fill[lev[i]]++] = (int32_t)i;
    lstart = start;
    lcount.assign(cnt.begin() + 1, cnt.end());
}

// Head of the level order solved by one workgroup from LDS: the longest prefix of levels whose
// positions fit the LDS budget and whose levels are narrow (a wide level is cheaper spread over
// the whole GPU).  EIGSOL_TRSV_HEAD_ROWS / EIGSOL_TRSV_HEAD_WIDTH override (0 rows: no head).
template <class S>
static int32_t head_levels(const std::vector<int64_t>& lstart, const std::vector<int64_t>& lcount,
                           const std::vector<int32_t>& lmaxlen, int32_t nlevels, bool wave_head) {
    int64_t cap = (int64_t)(150 * 1024) / (int64_t)sizeof(S);
    // widest head level.  One-workgroup head: config 5 256 -> 0.861 ms, 1024 -> 0.872 ms per solve.
    // One-wave head (16 rows per pass, ~0.26 us a pass): 64 -> 0.833 ms, 256 -> 0.879 ms (a wider
    // level is cheaper in the tail, ~1.7 us a level)
    int64_t width = wave_head ? 64 : 256;
    if (const char* e = std::getenv("EIGSOL_TRSV_HEAD_ROWS")) cap = std::min<int64_t>(cap, std::atoll(e));
    if (const char* e = std::getenv("EIGSOL_TRSV_HEAD_WIDTH")) width = std::atoll(e);
    int32_t h = 0;
    int64_t npass = 0;   // the pass table shares the LDS budget (8 bytes a pass)
    while (h < nlevels && lcount[h] <= width && lmaxlen[h] <= dev::kRowLanes) {
        const int64_t np = npass + (lcount[h] + dev::kHeadRows - 1) / dev::kHeadRows;
        if ((lstart[h + 1] + 1) * (int64_t)sizeof(S) + (np + dev::kHeadDepth) * 8 > cap * (int64_t)sizeof(S)) break;
        npass = np;
        ++h;
    }
    return h;
}

template <class S>
static const void* slice_kernel_ptr(int b, bool iter) {
    if (b == 4) return iter ? reinterpret_cast<const void*>(dev::sptrsv_slice_kernel<S, 4, true>)
                            : reinterpret_cast<const void*>(dev::sptrsv_slice_kernel<S, 4, false>);
    if (b == 8) return iter ? reinterpret_cast<const void*>(dev::sptrsv_slice_kernel<S, 8, true>)
                            : reinterpret_cast<const void*>(dev::sptrsv_slice_kernel<S, 8, false>);
    return iter ? reinterpret_cast<const void*>(dev::sptrsv_slice_kernel<S, 16, true>)
                : reinterpret_cast<const void*>(dev::sptrsv_slice_kernel<S, 16, false>);
}

// General (non-triangular) sparse solver choice; EIGSOL_SPARSE_SOLVER=band|lu|gmres forces one.
//   band  - RCM + banded partial-pivot LU (band_lu.hip): a direct factor, like the reference's
//           SparseLU, chosen when the RCM band fits the solve kernel's LDS window and the device,
//           and (up to n = 16384) is smaller than the dense matrix;
//   lu    - the densified partial-pivot LU, up to n = 16384;
//   gmres - ILU(0) + GMRES for larger patterns whose RCM band is too wide.  A GMRES that stalls
//           (or an ILU(0) zero pivot) falls back to the densified LU wherever the dense factor fits
//           the device (EIGSOL_GMRES_FALLBACK=0 disables it); otherwise the solve fails with
//           EIGSOL_E_SOLVER, as SparseLU reports a failed solve (solve_shifted.hpp:112-114).
enum SparseSolver { kSolverBand, kSolverLU, kSolverGMRES };

static double device_free_bytes() {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 0.0;
    return (double)fr;
}

static bool general_sparse_forced(SparseSolver& out) {
    if (const char* e = std::getenv("EIGSOL_SPARSE_SOLVER")) {
        if (!std::strcmp(e, "gmres")) { out = kSolverGMRES; return true; }
        if (!std::strcmp(e, "lu")) { out = kSolverLU; return true; }
        if (!std::strcmp(e, "band")) { out = kSolverBand; return true; }
    }
    return false;
}

static SparseSolver general_sparse_solver(int64_t n, size_t sb, const BandPlan& plan, bool& forced) {
    forced = false;
    SparseSolver fs;
    if (general_sparse_forced(fs)) {
        forced = true;
        return fs;
    }
    const double dense = (double)n * (double)n * (double)sb;
    const bool band_fits = plan.ok && plan.bytes <= 0.6 * device_free_bytes();
    if (band_fits && (n > 16384 || plan.bytes < dense)) return kSolverBand;
    return n > 16384 ? kSolverGMRES : kSolverLU;
}

static bool gmres_fallback_enabled() {
    const char* e = std::getenv("EIGSOL_GMRES_FALLBACK");
    return !(e && !std::strcmp(e, "0"));
}

// GMRES failed (stalled solve, or ILU(0) zero pivot): switch the factor to the densified LU of A
// (retained in f->src) when it fits the device; otherwise keep GMRES's error.
template <class S>
static int gmres_dense_fallback(ShiftFactor* f, int rc_gmres) {
    if constexpr (!kDenseLU<S>) {
        return rc_gmres;
    } else {
        const int64_t n = f->n;
        const double bytes = (double)n * (double)n * (double)sizeof(S);
        if (!gmres_fallback_enabled() || !f->src || n > INT32_MAX / 2 || bytes > 0.8 * device_free_bytes())
            return rc_gmres;
        hipStream_t st = f->ctx->stream;
        EIGSOL_HIP(hipStreamSynchronize(st));
        // The densified LU is built in a scratch factor and moved into f only once it exists: a
        // failed allocation or a zero pivot leaves f a working GMRES factor (later launches and
        // shift_info still see f->gm) and frees the scratch.
        auto* g = new ShiftFactor();
        g->ctx = f->ctx;
        ctx_retain(g->ctx);
        g->dtype = f->dtype;
        g->n = n;
        g->sig_re = f->sig_re;
        g->sig_im = f->sig_im;
        int rc = EIGSOL_OK;
        if (hipMalloc(&g->lu, (size_t)bytes) != hipSuccess || hipMemsetAsync(g->lu, 0, (size_t)bytes, st) != hipSuccess)
            rc = fail(EIGSOL_E_HIP, "GMRES fallback: hipMalloc(dense LU)");
        if (rc == EIGSOL_OK) {
            hipLaunchKernelGGL((dev::densify_kernel<S>), dim3((n + 255) / 256), dim3(256), 0, st, f->src->rowptr,
                               f->src->col, static_cast<const S*>(f->src->val), n, static_cast<S*>(g->lu));
            rc = dense_lu_factor<S>(g, true);
        }
        if (rc != EIGSOL_OK) {
            shift_free(g);
            return rc;
        }
        if (f->gm) { gmres_free(f->gm); f->gm = nullptr; }
        for (void* p : {(void*)f->work, (void*)f->err, f->wave_part}) if (p) hipFree(p);
        f->kind = g->kind;
        f->lu = g->lu;
        f->perm = g->perm;
        f->zero_pivot = g->zero_pivot;
        f->lds_bytes = g->lds_bytes;
        f->dense_multi = g->dense_multi;
        f->grid = g->grid;
        f->nchunks = g->nchunks;
        f->flag_f = g->flag_f;
        f->flag_b = g->flag_b;
        f->zf = g->zf;
        f->tinv = g->tinv;
        f->tmul = g->tmul;
        f->dense_v = g->dense_v;
        f->work = g->work;
        f->err = g->err;
        f->wave_part = g->wave_part;
        ctx_release(g->ctx);
        delete g;   // its buffers now belong to f
        csr_release(f->src);
        f->src = nullptr;
        f->fell_back = 1;
        return EIGSOL_OK;
    }
}

template <class S>
static int factor_tri_host(eigsol_ctx* ctx, int dtype, int64_t n, std::vector<int32_t>& rp,
                           std::vector<int32_t>& ci, std::vector<S>& v, bool up, double sre, double sim,
                           ShiftFactor** out);

template <class S>
static int factor_tri_device(eigsol_csr* A, double sre, double sim, ShiftFactor** out, bool& declined);

template <class S>
static int factor_csr_t(eigsol_csr* A, double sre, double sim, ShiftFactor** out) {
    hipStream_t st = A->ctx->stream;
    const int64_t n = A->nrows, nnz = A->nnz;
    // triangular matrices: analysis and layout on the device (EIGSOL_TRSV_HOST=1: the host build)
    const char* host_env = std::getenv("EIGSOL_TRSV_HOST");
    if (n > 0 && !(host_env && std::atoi(host_env))) {
        bool declined = false;
        const int rc = factor_tri_device<S>(A, sre, sim, out, declined);
        if (!declined) return rc;
    }
    std::vector<int32_t> rp(n + 1), ci(nnz);
    std::vector<S> v(nnz);
    EIGSOL_HIP(hipMemcpyAsync(rp.data(), A->rowptr, (n + 1) * 4, hipMemcpyDeviceToHost, st));
    EIGSOL_HIP(hipMemcpyAsync(ci.data(), A->col, nnz * 4, hipMemcpyDeviceToHost, st));
    EIGSOL_HIP(hipMemcpyAsync(v.data(), A->val, nnz * sizeof(S), hipMemcpyDeviceToHost, st));
    EIGSOL_HIP(hipStreamSynchronize(st));
    bool up = true, lo = true;
    for (int64_t i = 0; i < n && (up || lo); ++i)
        for (int32_t e = rp[i]; e < rp[i + 1]; ++e) {
            if (ci[e] < i) up = false;
            if (ci[e] > i) lo = false;
        }
    if (up || lo) return factor_tri_host<S>(A->ctx, A->dtype, n, rp, ci, v, up, sre, sim, out);
    auto* f = new ShiftFactor();
    f->ctx = A->ctx;
    ctx_retain(f->ctx);
    f->dtype = A->dtype;
    f->n = n;
    f->sig_re = sre;
    f->sig_im = sim;
    f->nnz_total = nnz;
    int rc = EIGSOL_OK;
    {
        if constexpr (!kDenseLU<S>) {
            shift_free(f);
            return fail(EIGSOL_E_UNSUPPORTED, "solve_shifted: single-precision factors exist for triangular "
                                              "sparse matrices only");
        } else {
        // past n = 16384 the double / complex<double> factors take the GMRES family's direct
        // factors (exact no-pivot LU where the fill stays within 3 x nnz, else the nested-dissection
        // multifrontal LU, gmres.hip / multifrontal.hip; ILU(0) + GMRES when neither fits): the band
        // factor runs one panel kernel per 64 columns on one workgroup (round 5, config5_convdiff_1M:
        // 13.8 s, 1.37 s per solve).  Single precision takes the same family on values widened to
        // double (gm_solve_s).  The band stays for smaller orders, or forced.
        BandPlan plan;
        SparseSolver fs = kSolverBand;
        const bool pre_forced = general_sparse_forced(fs);
        // from n = 1024 (EIGSOL_SPARSE_FAMILY_MIN_N) too: on a 2-D stencil the band solve (one workgroup
        // walking the band) took 0.50 ms per iteration at n = 1024, 2.2 ms at 4096 and 9.5 ms at 16384, the
        // multifrontal LU 0.11 / 0.15 / 0.21 ms with a shorter set-up (round 6, tools/r06_small_sparse_paths.py,
        // profiles/r06_small_sparse_paths.log); the band LU stays the fallback for zero pivots
        static const int64_t family_min = [] {
            const char* e = std::getenv("EIGSOL_SPARSE_FAMILY_MIN_N");
            return e ? (int64_t)std::atoll(e) : (int64_t)1024;
        }();
        const bool large_gmres = !pre_forced && (n > 16384 || n >= family_min);
        if (!large_gmres && !(pre_forced && fs != kSolverBand)) band_plan(A->dtype, n, rp.data(), ci.data(), plan);
        bool forced = false;
        const SparseSolver solver = large_gmres ? kSolverGMRES : general_sparse_solver(n, sizeof(S), plan, forced);
        if (solver == kSolverBand) {
            if (!plan.ok) {
                shift_free(f);
                return fail(EIGSOL_E_UNSUPPORTED, "solve_shifted: the RCM band (kl " + std::to_string(plan.kl) +
                                                      ", ku " + std::to_string(plan.ku) +
                                                      ") is too wide for the band solve");
            }
            rc = band_create(A->ctx, A->dtype, n, rp.data(), ci.data(), v.data(), sre, sim, plan, &f->band);
            if (rc != EIGSOL_OK) { shift_free(f); return rc; }
            f->kind = 3;
            *out = f;
            return EIGSOL_OK;
        }
        if (solver == kSolverGMRES) {
            if constexpr (kGmres<S>) {
                rc = gmres_create(A->ctx, A->dtype, n, rp.data(), ci.data(), v.data(), sre, sim, &f->gm, A);
            } else {
                using W = GmresScalar<S>;
                std::vector<W> vw(v.size());
                for (size_t e = 0; e < v.size(); ++e) {
                    if constexpr (is_real_v<S>) vw[e] = static_cast<double>(v[e]);
                    else vw[e] = W{static_cast<double>(v[e].re), static_cast<double>(v[e].im)};
                }
                rc = gmres_create(A->ctx, dtype_complex(A->dtype) ? EIGSOL_C128 : EIGSOL_F64, n, rp.data(), ci.data(),
                                  vw.data(), sre, sim, &f->gm);
                if (rc == EIGSOL_OK && hipMalloc(&f->promo, 2 * (size_t)n * sizeof(W)) != hipSuccess)
                    rc = fail(EIGSOL_E_HIP, "solve_shifted: hipMalloc(single-precision GMRES vectors)");
            }
            f->red_grid = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n + 1023) / 1024));
            if (rc == EIGSOL_OK && (hipMalloc(&f->work, 64) != hipSuccess ||
                                    hipMalloc(&f->wave_part, (size_t)f->red_grid * sizeof(dev::part4)) != hipSuccess ||
                                    hipMemsetAsync(f->work, 0, 64, st) != hipSuccess))
                rc = fail(EIGSOL_E_HIP, "solve_shifted: GMRES work buffers");
            f->kind = 2;
            f->src = A;
            csr_retain(A);
            if (rc == EIGSOL_E_SOLVER && large_gmres) {
                // every factor of the family met a zero pivot (the no-pivot exact LU, the
                // multifrontal LU's front pivoting, ILU(0)): the partial-pivoting RCM band LU where
                // its band fits, as the reference's pivoting SparseLU would (solve_shifted.hpp:104-106)
                const std::string why = eigsol_last_error();
                BandPlan bp;
                band_plan(A->dtype, n, rp.data(), ci.data(), bp);
                if (bp.ok) {
                    auto* fb = new ShiftFactor();
                    fb->ctx = A->ctx;
                    ctx_retain(fb->ctx);
                    fb->dtype = A->dtype;
                    fb->n = n;
                    fb->sig_re = sre;
                    fb->sig_im = sim;
                    fb->nnz_total = nnz;
                    if (band_create(A->ctx, A->dtype, n, rp.data(), ci.data(), v.data(), sre, sim, bp, &fb->band) ==
                        EIGSOL_OK) {
                        fb->kind = 3;
                        shift_free(f);
                        *out = fb;
                        return EIGSOL_OK;
                    }
                    shift_free(fb);
                    (void)hipGetLastError();
                }
                rc = fail(EIGSOL_E_SOLVER, why);
            }
            if (rc == EIGSOL_E_SOLVER) rc = gmres_dense_fallback<S>(f, rc);   // ILU(0) zero pivot
            if (rc != EIGSOL_OK) { shift_free(f); return rc; }
            *out = f;
            return EIGSOL_OK;
        }
        // general sparse pattern: densify on the device and LU it (the reference's SparseLU)
        rc = dense_limits(A->dtype, n, "solve_shifted (non-triangular sparse)");
        const size_t bytes = (size_t)n * n * sizeof(S);
        if (rc == EIGSOL_OK && hipMalloc(&f->lu, bytes) != hipSuccess) rc = fail(EIGSOL_E_HIP, "hipMalloc(LU)");
        if (rc == EIGSOL_OK) {
            hipMemsetAsync(f->lu, 0, bytes, st);
            hipLaunchKernelGGL((dev::densify_kernel<S>), dim3((n + 255) / 256), dim3(256), 0, st,
                               A->rowptr, A->col, static_cast<const S*>(A->val), n, static_cast<S*>(f->lu));
            rc = dense_lu_factor<S>(f, true);
        }
        if (rc != EIGSOL_OK) { shift_free(f); return rc; }
        *out = f;
        return EIGSOL_OK;
        }
    }
}

template <class S>
static void tri_dump(const ShiftFactor* f);

static int dev_upload(hipStream_t st, void** dst, const void* src, size_t bytes) {
    EIGSOL_HIP(hipMalloc(dst, std::max<size_t>(bytes, 16)));
    if (bytes && src) EIGSOL_HIP(hipMemcpyAsync(*dst, src, bytes, hipMemcpyHostToDevice, st));
    return EIGSOL_OK;
}

// Launch geometry of a level-ordered triangular factor (host- or device-built): the tail grid (one
// residency round, cooperative launch), the multi-solve set-up and the partials grid.  Needs the
// layout fields (tail variant, chunk_two, slice_b, head, chunks / slices) already set.
template <class S>
static int tri_launch_setup(ShiftFactor* f) {
    int rc = EIGSOL_OK;
    // tail grid: one residency round (cooperative launch), capped at EIGSOL_TRSV_BLOCKS_PER_CU
    // blocks per CU and by the work
    {
        int per_cu_max = 0;
        const void* tk = f->tail_chunks ? (f->chunk_two ? reinterpret_cast<const void*>(dev::sptrsv_chunk_kernel<S, true, true>)
                                                        : reinterpret_cast<const void*>(dev::sptrsv_chunk_kernel<S, true>))
                                        : slice_kernel_ptr<S>(f->slice_b, true);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_max, tk, dev::kThreads, 0) != hipSuccess ||
            per_cu_max < 1)
            rc = fail(EIGSOL_E_HIP, "triangular solve: occupancy query");
        f->grid = per_cu_max * f->ctx->num_cus;
    }
    int per_cu = 2;
    if (const char* env = std::getenv("EIGSOL_TRSV_BLOCKS_PER_CU")) per_cu = std::max(1, std::atoi(env));
    f->grid = std::min(f->grid, per_cu * f->ctx->num_cus);
    const int64_t units = f->tail_chunks ? (int64_t)f->nchunks - f->chunk0 : f->nslices;
    f->grid = (int)std::max<int64_t>(1, std::min<int64_t>(f->grid, (units + dev::kWaves - 1) / dev::kWaves));
    // multi-solve launches: chunk tail with the one-wave head (or none), K solves per launch
    // (EIGSOL_TRSV_MULTI=K, 1..4; 1 = one iteration per launch) on K copies of the grid at one
    // workgroup per CU per solve (EIGSOL_TRSV_MULTI_BLOCKS_PER_CU), when they are co-resident
    if (rc == EIGSOL_OK && f->tail_chunks && (f->hpos == 0 || f->wave_head)) {
        const char* e = std::getenv("EIGSOL_TRSV_MULTI");
        const int want = std::max(1, std::min(dev::kMaxMulti, e ? std::atoi(e) : kMultiDefault));
        int per_cu_role = 0;
        hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu_role, reinterpret_cast<const void*>(dev::sptrsv_chunk_role_kernel<S>), dev::kThreads, 0);
        int role_per_cu = 1;
        if (const char* env = std::getenv("EIGSOL_TRSV_MULTI_BLOCKS_PER_CU")) role_per_cu = std::max(1, std::atoi(env));
        const int gr = std::min(f->grid, role_per_cu * f->ctx->num_cus);
        int K = want;
        while (K > 1 && per_cu_role * f->ctx->num_cus < K * gr) --K;
        if (K > 1) {
            f->multi = K;
            f->grid_multi = K * gr;
            const char* hc = std::getenv("EIGSOL_TRSV_MULTI_HEAD");   // seq: the head solves one after another
            // the dynamic LDS of the concurrent head shares the CU's 160 KiB with the kernel's static
            // __shared__ state (its prologue record)
            hipFuncAttributes fa{};
            size_t static_lds = 256;
            if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(dev::sptrsv_whead_kernel<S, true, true>)) ==
                hipSuccess)
                static_lds = fa.sharedSizeBytes;
            f->hconc = (!(hc && !std::strcmp(hc, "seq")) &&
                        (size_t)K * (size_t)(f->hpos + 1) * sizeof(S) + 16 + static_lds <= (size_t)160 * 1024) ? 1 : 0;
        }
    }
    // EIGSOL_TRSV_PART_GRID: the partials kernels' grid.  Round 6 (tools/r06_c5_partgrid_ab.sh,
    // profiles/r06_c5_partgrid_ab.log, config 5 at K = 4): 2048 / 977 (n / 1024, the old cap) / 512 /
    // 256 / 192 / 128 / 64 blocks -> 0.4077 / 0.4076 / 0.4026 / 0.4010 / 0.4016 / 0.4049 / 0.4159 ms per
    // iteration: one block per CU, the last arriver sums fewer block partials per solve
    int64_t red_cap = 256;
    if (const char* e = std::getenv("EIGSOL_TRSV_PART_GRID")) red_cap = std::max<int64_t>(8, std::atoll(e));
    // never above grid * kWaves: wave_part (below) holds that many block partials
    f->red_grid = (int)std::max<int64_t>(1, std::min<int64_t>(f->grid * dev::kWaves,
                                                                  std::min<int64_t>(red_cap, (f->n + 1023) / 1024)));
    return rc;
}

// Solve state of a triangular factor: the two polled value buffers (every row unsolved: the
// sentinel; the zero slot z[n] stays 0 for good), the ticket / error words and the wave partials.
template <class S>
static int tri_state_alloc(ShiftFactor* f) {
    hipStream_t st = f->ctx->stream;
    const int64_t n = f->n;
    EIGSOL_TRY(dev_upload(st, &f->z[0], nullptr, (n + 1) * sizeof(S)));
    EIGSOL_TRY(dev_upload(st, &f->z[1], nullptr, (n + 1) * sizeof(S)));
    EIGSOL_TRY(dev_upload(st, (void**)&f->work, nullptr, 64));
    EIGSOL_TRY(dev_upload(st, (void**)&f->err, nullptr, 64));
    EIGSOL_TRY(dev_upload(st, &f->wave_part, nullptr, (size_t)f->grid * dev::kWaves * sizeof(dev::part4)));
    const uint32_t sent = (uint32_t)(dev::kSent & 0xffffffffu);
    for (void* zb : f->z) {
        hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(zb), (int)sent, n * sizeof(S) / 4, st);
        hipMemsetAsync(static_cast<char*>(zb) + n * sizeof(S), 0, sizeof(S), st);
    }
    hipMemsetAsync(f->work, 0, 64, st);
    hipMemsetAsync(f->err, 0, 64, st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail(EIGSOL_E_HIP, "factor upload");
    return EIGSOL_OK;
}

// Triangular CSR (host arrays, columns ascending per row) -> level-ordered factor of A - sigma I.
template <class S>
static int factor_tri_host(eigsol_ctx* ctx, int dtype, int64_t n, std::vector<int32_t>& rp,
                           std::vector<int32_t>& ci, std::vector<S>& v, bool up, double sre, double sim,
                           ShiftFactor** out) {
    hipStream_t st = ctx->stream;
    const int64_t nnz = rp[n];
    auto* f = new ShiftFactor();
    f->ctx = ctx;
    ctx_retain(f->ctx);
    f->dtype = dtype;
    f->n = n;
    f->sig_re = sre;
    f->sig_im = sim;
    f->nnz_total = nnz;
    int rc = EIGSOL_OK;
    f->upper = up ? 1 : 0;
    // split diagonal / off-diagonal; pivots d_i - sigma (missing diagonal: 0 - sigma)
    const S sig = make_sigma<S>(sre, sim);
    std::vector<int32_t> orp(n + 1, 0), oci;
    std::vector<S> ov, pv(n);
    oci.reserve(nnz);
    ov.reserve(nnz);
    for (int64_t i = 0; i < n; ++i) {
        S d = s_zero<S>();
        for (int32_t e = rp[i]; e < rp[i + 1]; ++e) {
            if (ci[e] == i) {
                d = h_add(d, v[e]);
            } else {
                oci.push_back(ci[e]);
                ov.push_back(v[e]);
            }
        }
        pv[i] = h_sub(d, sig);
        if (h_zero(pv[i])) {
            shift_free(f);
            return fail(EIGSOL_E_SOLVER, "solve_shifted: SparseLU factorization failed");
        }
        orp[i + 1] = (int32_t)oci.size();
    }
    f->nnz_off = (int64_t)oci.size();
    std::vector<int32_t> order;
    std::vector<int64_t> lstart, lcount;
    level_order(orp, oci, n, up, order, f->nlevels, lstart, lcount);
    f->npos = (int32_t)order.size();
    std::vector<int32_t> lmaxlen(f->nlevels, 0);   // longest row (off-diagonal entries) per level
    for (int32_t l = 0; l < f->nlevels; ++l)
        for (int64_t p = lstart[l]; p < lstart[l] + lcount[l]; ++p)
            lmaxlen[l] = std::max(lmaxlen[l], orp[order[p] + 1] - orp[order[p]]);
    if (const char* e = std::getenv("EIGSOL_TRSV_HEAD")) f->wave_head = std::strcmp(e, "block") ? 1 : 0;
    f->hlevels = head_levels<S>(lstart, lcount, lmaxlen, f->nlevels, f->wave_head != 0);
    if (const char* e = std::getenv("EIGSOL_TRSV_POLL_FAST"))
        f->poll_fast = (f->poll_fast & ~0xffff) | std::min(0xffff, std::max(0, std::atoi(e)));
    if (const char* e = std::getenv("EIGSOL_TRSV_POLL_SLOW"))
        f->poll_fast = (f->poll_fast & 0xffff) | (std::min(7, std::max(0, std::atoi(e))) << 16);
    if (const char* e = std::getenv("EIGSOL_TRSV_POLL_MODE")) f->poll_mode = std::atoi(e);
    f->hpos = (int32_t)lstart[f->hlevels];
    std::vector<int2> passes;
    for (int32_t l = 0; l < f->hlevels; ++l) {
        const int32_t p0 = (int32_t)lstart[l], p1 = (int32_t)(lstart[l] + lcount[l]);
        for (int32_t p = p0; p < p1; p += dev::kHeadRows) {
            const int32_t e = std::min(p1, p + dev::kHeadRows);
            passes.push_back(make_int2(p, e | (e == p1 ? dev::kPassBarrier : 0)));
        }
    }
    while (!passes.empty() && passes.size() % dev::kHeadDepth) passes.push_back(make_int2(0, 0));   // empty
    f->npass = (int32_t)passes.size();
    std::vector<int32_t> rowpos;
    if (f->hpos > 0) {
        rowpos.assign(n, -1);
        for (int32_t p = 0; p < f->hpos; ++p)
            if (order[p] >= 0) rowpos[order[p]] = p;
    }
    // head, pass-major (see sptrsv_head_kernel): columns are LDS positions of earlier head rows
    const size_t hslots = (size_t)f->npass * dev::kHeadThreads;
    std::vector<int32_t> hcol(hslots, f->hpos);   // padding: the zero slot
    std::vector<S> hval(hslots, s_zero<S>()), hpiv((size_t)f->npass * dev::kHeadRows, make_sigma<S>(1.0, 0.0));
    for (int32_t q = 0; q < f->npass; ++q) {
        const int32_t p0 = passes[q].x, p1 = passes[q].y & ~dev::kPassBarrier;
        for (int32_t p = p0; p < p1; ++p) {
            const size_t g = (size_t)q * dev::kHeadRows + (p - p0);
            const int32_t i = order[p];
            hpiv[g] = pv[i];
            for (int32_t e = orp[i]; e < orp[i + 1]; ++e) {
                hcol[g * dev::kRowLanes + (e - orp[i])] = rowpos[oci[e]];
                hval[g * dev::kRowLanes + (e - orp[i])] = ov[e];
            }
        }
    }
    // one-wave head (see sptrsv_whead_kernel): passes of <= 16 rows inside a level, 4 lanes per row,
    // entry idx of a row at lane 4 g + idx / 4, slot idx % 4; reciprocal pivots.
    // EIGSOL_TRSV_HEAD=block selects the one-workgroup head.
    std::vector<S> wval, wrp;
    std::vector<int32_t> wcol, wdst;
    if (f->hpos > 0) {
        auto recip = [](S p) -> S {
            if constexpr (is_real_v<S>) return (S)1 / p;
            else {
                const double d = (double)p.re * (double)p.re + (double)p.im * (double)p.im;
                S r;
                r.re = (decltype(p.re))((double)p.re / d);
                r.im = (decltype(p.im))(-(double)p.im / d);
                return r;
            }
        };
        int32_t q = 0;
        for (int32_t l = 0; l < f->hlevels; ++l) {
            const int32_t p0 = (int32_t)lstart[l], p1 = (int32_t)(lstart[l] + lcount[l]);
            for (int32_t p = p0; p < p1; p += dev::kWHeadRows, ++q) {
                wval.resize((size_t)(q + 1) * 256, s_zero<S>());
                wcol.resize((size_t)(q + 1) * 256, f->hpos);
                wrp.resize((size_t)(q + 1) * dev::kWHeadRows, make_sigma<S>(1.0, 0.0));
                wdst.resize((size_t)(q + 1) * dev::kWHeadRows, -1);
                for (int32_t u = 0; u < std::min(dev::kWHeadRows, p1 - p); ++u) {
                    const int32_t i = order[p + u];
                    wrp[(size_t)q * dev::kWHeadRows + u] = recip(pv[i]);
                    wdst[(size_t)q * dev::kWHeadRows + u] = p + u;
                    for (int32_t e = orp[i]; e < orp[i + 1]; ++e) {
                        const int32_t idx = e - orp[i];
                        const size_t slot = ((size_t)q * 4 + (size_t)(idx % 4)) * 64 + (size_t)(4 * u + idx / 4);
                        wcol[slot] = rowpos[oci[e]];
                        wval[slot] = ov[e];
                    }
                }
            }
        }
        while (q % dev::kWHeadDepth) {   // empty passes: the ring loop is straight-line code
            ++q;
            wval.resize((size_t)q * 256, s_zero<S>());
            wcol.resize((size_t)q * 256, f->hpos);
            wrp.resize((size_t)q * dev::kWHeadRows, make_sigma<S>(1.0, 0.0));
            wdst.resize((size_t)q * dev::kWHeadRows, -1);
        }
        f->nwpass = q;
    }
    // tail variant: slices (row per lane) for few, very wide levels; chunks (16 lanes per row)
    // otherwise.  EIGSOL_TRSV_TAIL=slice|chunk overrides.
    {
        // slices when most tail rows sit in levels of >= 64k rows (a wave's 64 rows then rarely
        // wait); measured: one 1M-row level 74 vs 195 us, config 5 (widest level 21k) 1.3 vs 0.86 ms
        int64_t trows = 0, wide = 0;
        for (int32_t l = f->hlevels; l < f->nlevels; ++l) {
            trows += lcount[l];
            if (lcount[l] >= 65536) wide += lcount[l];
        }
        f->tail_chunks = (trows > 0 && 2 * wide < trows) ? 1 : 0;
        if (const char* e = std::getenv("EIGSOL_TRSV_TAIL")) f->tail_chunks = std::strcmp(e, "slice") ? 1 : 0;
    }
    std::vector<int32_t> porder, pptr, pcol;
    std::vector<S> pval, ppiv;
    if (f->tail_chunks) {   // position-indexed copies: no dependent metadata loads in the kernel
        f->chunk0 = f->hpos / dev::kWaveRows;
        f->nchunks = f->npos / dev::kWaveRows;
        porder = order;
        pptr.assign((size_t)f->npos + 1, 0);
        ppiv.assign((size_t)f->npos, make_sigma<S>(1.0, 0.0));
        pcol.reserve(oci.size());
        pval.reserve(oci.size());
        int32_t longest = 0;
        for (int32_t p = 0; p < f->npos; ++p) {
            const int32_t i = order[p];
            if (i >= 0) {
                if (p >= f->hpos) longest = std::max(longest, orp[i + 1] - orp[i]);
                for (int32_t e = orp[i]; e < orp[i + 1]; ++e) {
                    pcol.push_back(oci[e]);
                    pval.push_back(ov[e]);
                }
                ppiv[p] = pv[i];
            }
            pptr[p + 1] = (int32_t)pcol.size();
        }
        // rows past 16 entries: the second entry of every lane is polled with the first
        // (EIGSOL_TRSV_TWO=0|1 overrides; round 4, the exact LU's U of config 5 made general)
        f->chunk_two = longest > dev::kRowLanes ? 1 : 0;
        if (const char* e = std::getenv("EIGSOL_TRSV_TWO")) f->chunk_two = std::atoi(e) != 0;
    }
    // tail slices (see sptrsv_slice_kernel): 64 rows of one level each; B = the smallest of
    // 4 / 8 / 16 that holds the entries of at least 95 % of the slices (longer slices loop)
    std::vector<int32_t> slen;   // longest row per slice
    std::vector<int64_t> sfirst;
    std::vector<int32_t> scount;
    for (int32_t l = f->tail_chunks ? f->nlevels : f->hlevels; l < f->nlevels; ++l)
        for (int64_t p = lstart[l]; p < lstart[l] + lcount[l]; p += 64) {
            const int32_t c = (int32_t)std::min<int64_t>(64, lstart[l] + lcount[l] - p);
            int32_t K = 0;
            for (int32_t u = 0; u < c; ++u) K = std::max(K, orp[order[p + u] + 1] - orp[order[p + u]]);
            sfirst.push_back(p);
            scount.push_back(c);
            slen.push_back(K);
        }
    f->nslices = (int32_t)slen.size();
    {
        std::vector<int32_t> sorted(slen);
        std::sort(sorted.begin(), sorted.end());
        const int32_t q95 = sorted.empty() ? 0 : sorted[(size_t)(0.95 * (double)(sorted.size() - 1))];
        f->slice_b = q95 <= 4 ? 4 : (q95 <= 8 ? 8 : 16);
        if (const char* e = std::getenv("EIGSOL_TRSV_SLICE_B")) {
            const int b = std::atoi(e);
            if (b == 4 || b == 8 || b == 16) f->slice_b = b;
        }
    }
    const int32_t Bs = f->slice_b;
    // the kernel prefetches "slice 0" for a wave past the last slice: slice 0 always exists (an
    // empty one when the head holds every level)
    std::vector<int2> smeta(std::max(1, f->nslices), make_int2(0, Bs));
    std::vector<int32_t> trow((size_t)std::max(1, f->nslices) * 64, -1);
    std::vector<S> tpiv((size_t)std::max(1, f->nslices) * 64, make_sigma<S>(1.0, 0.0));
    int64_t tent = 0;
    for (int32_t sl = 0; sl < f->nslices; ++sl) tent += 64 * (int64_t)std::max(slen[sl], Bs);
    tent += 64 * (int64_t)Bs;   // the prefetch of "slice ns" reads slice 0's range: keep it in bounds
    if (tent * (int64_t)sizeof(S) >= (int64_t)1 << 32) {
        shift_free(f);
        return fail(EIGSOL_E_UNSUPPORTED, "triangular solve: factor streams exceed 4 GiB");
    }
    std::vector<int32_t> tcol((size_t)tent, (int32_t)n);   // padding: the zero slot z[n]
    std::vector<S> tval((size_t)tent, s_zero<S>());
    {
        int64_t off = 0;
        for (int32_t sl = 0; sl < f->nslices; ++sl) {
            const int32_t Kp = std::max(slen[sl], Bs);
            smeta[sl] = make_int2((int32_t)off, Kp);
            for (int32_t u = 0; u < scount[sl]; ++u) {
                const int32_t i = order[sfirst[sl] + u];
                trow[(size_t)sl * 64 + u] = i;
                tpiv[(size_t)sl * 64 + u] = pv[i];
                for (int32_t e = orp[i]; e < orp[i + 1]; ++e) {
                    tcol[(size_t)(off + 64 * (e - orp[i]) + u)] = oci[e];
                    tval[(size_t)(off + 64 * (e - orp[i]) + u)] = ov[e];
                }
            }
            off += 64 * (int64_t)Kp;
        }
    }
    std::vector<int32_t>().swap(oci);
    std::vector<S>().swap(ov);
    auto up_ = [&](void** dst, const void* src, size_t bytes) -> int { return dev_upload(st, dst, src, bytes); };
    if (rc == EIGSOL_OK) rc = tri_launch_setup<S>(f);
    if (rc == EIGSOL_OK) rc = up_((void**)&f->order, order.data(), (size_t)f->hpos * 4);
    if (rc == EIGSOL_OK) rc = up_((void**)&f->hcol, hcol.data(), hcol.size() * 4);
    if (rc == EIGSOL_OK) rc = up_(&f->hval, hval.data(), hval.size() * sizeof(S));
    if (rc == EIGSOL_OK) rc = up_(&f->hpiv, hpiv.data(), hpiv.size() * sizeof(S));
    if (rc == EIGSOL_OK) rc = up_((void**)&f->passes, passes.data(), passes.size() * sizeof(int2));
    if (rc == EIGSOL_OK) rc = up_(&f->wval, wval.data(), wval.size() * sizeof(S));
    if (rc == EIGSOL_OK) rc = up_((void**)&f->wcol, wcol.data(), wcol.size() * 4);
    if (rc == EIGSOL_OK) rc = up_(&f->wrp, wrp.data(), wrp.size() * sizeof(S));
    if (rc == EIGSOL_OK) rc = up_((void**)&f->wdst, wdst.data(), wdst.size() * 4);
    if (rc == EIGSOL_OK) rc = up_((void**)&f->smeta, smeta.data(), smeta.size() * sizeof(int2));
    if (rc == EIGSOL_OK) rc = up_((void**)&f->trow, trow.data(), trow.size() * 4);
    if (rc == EIGSOL_OK) rc = up_(&f->tpiv, tpiv.data(), tpiv.size() * sizeof(S));
    if (rc == EIGSOL_OK) rc = up_((void**)&f->tcol, tcol.data(), tcol.size() * 4);
    if (rc == EIGSOL_OK) rc = up_(&f->tval, tval.data(), tval.size() * sizeof(S));
    if (rc == EIGSOL_OK) rc = up_((void**)&f->porder, porder.data(), porder.size() * 4);
    if (rc == EIGSOL_OK) rc = up_((void**)&f->pptr, pptr.data(), pptr.size() * 4);
    if (rc == EIGSOL_OK) rc = up_((void**)&f->pcol, pcol.data(), pcol.size() * 4);
    if (rc == EIGSOL_OK) rc = up_(&f->pval, pval.data(), pval.size() * sizeof(S));
    if (rc == EIGSOL_OK) rc = up_(&f->ppiv, ppiv.data(), ppiv.size() * sizeof(S));
    if (rc == EIGSOL_OK) rc = tri_state_alloc<S>(f);
    if (rc != EIGSOL_OK) { shift_free(f); return rc; }
    f->kind = 0;
    tri_dump<S>(f);
    *out = f;
    return EIGSOL_OK;
}

// EIGSOL_TRSV_DUMP=prefix (debugging): the built factor's position-indexed arrays, downloaded and
// written to prefix_<name>.bin (host and device builds compare byte for byte)
template <class S>
static void tri_dump(const ShiftFactor* f) {
    const char* pre = std::getenv("EIGSOL_TRSV_DUMP");
    if (!pre || f->kind != 0) return;
    hipStreamSynchronize(f->ctx->stream);
    auto put = [&](const char* name, const void* d, size_t bytes) {
        std::vector<unsigned char> h(bytes);
        if (bytes && hipMemcpy(h.data(), d, bytes, hipMemcpyDeviceToHost) != hipSuccess) return;
        const std::string path = std::string(pre) + "_" + name + ".bin";
        if (FILE* fp = std::fopen(path.c_str(), "wb")) {
            std::fwrite(h.data(), 1, bytes, fp);
            std::fclose(fp);
        }
    };
    const int32_t meta[12] = {f->nlevels, f->npos, f->hpos, f->hlevels, f->nwpass, f->chunk0, f->nchunks, f->chunk_two,
                              f->tail_chunks, f->grid, f->multi, (int32_t)f->nnz_off};
    if (FILE* fp = std::fopen((std::string(pre) + "_meta.bin").c_str(), "wb")) {
        std::fwrite(meta, sizeof(meta), 1, fp);
        std::fclose(fp);
    }
    put("porder", f->porder, (size_t)f->npos * 4);
    put("pptr", f->pptr, ((size_t)f->npos + 1) * 4);
    put("pcol", f->pcol, (size_t)f->nnz_off * 4);
    put("pval", f->pval, (size_t)f->nnz_off * sizeof(S));
    put("ppiv", f->ppiv, (size_t)f->npos * sizeof(S));
    put("order", f->order, (size_t)f->hpos * 4);
    put("wval", f->wval, (size_t)f->nwpass * 256 * sizeof(S));
    put("wcol", f->wcol, (size_t)f->nwpass * 256 * 4);
    put("wrp", f->wrp, (size_t)f->nwpass * 16 * sizeof(S));
    put("wdst", f->wdst, (size_t)f->nwpass * 16 * 4);
}

hipError_t tri_sort_rows_by_level(hipStream_t st, const int32_t* lev, int32_t* lev_out, int32_t* rows_out, int64_t n,
                                  int bits);
hipError_t tri_exclusive_scan(hipStream_t st, const int32_t* in, int32_t* out, int64_t n);

// Triangular CSR already on the device -> the level-ordered factor of A - sigma I, built on the device
// (round 5; the host build of config 5's 1M-row factor took 0.37 s, most of it moving 320 MB of
// matrix down and the layout back up).  The result is the host build's layout bit for bit: the
// same levels, positions sorted by level with ascending rows inside a level (stable radix sort),
// the same padding, the same position-indexed chunk CSR and the same one-wave head.  Only the small
// per-level tables (counts, longest rows) travel to the host, which takes the same head / tail
// decisions as factor_tri_host.  declined = true (nothing built) for a matrix that is not
// triangular or a layout this build does not produce (slice tail, one-workgroup head): the caller
// then takes the host path.
template <class S>
static int factor_tri_device(eigsol_csr* A, double sre, double sim, ShiftFactor** out, bool& declined) {
    declined = false;
    eigsol_ctx* ctx = A->ctx;
    hipStream_t st = ctx->stream;
    const int64_t n = A->nrows, nnz = A->nnz;
    const S* val = static_cast<const S*>(A->val);
    std::vector<void*> scratch;
    auto dalloc = [&](void** p, size_t bytes) -> int {
        EIGSOL_HIP(hipMalloc(p, std::max<size_t>(bytes, 16)));
        scratch.push_back(*p);
        return EIGSOL_OK;
    };
    int32_t* hostw = nullptr;   // pinned: flags[0..2], maxlev, err, nnz_off
    ShiftFactor* f = nullptr;
    auto finish = [&](int rc) {
        hipStreamSynchronize(st);
        for (void* p : scratch) hipFree(p);
        if (hostw) hipHostFree(hostw);
        if (rc != EIGSOL_OK || declined) {
            if (f) shift_free(f);
            return rc;
        }
        *out = f;
        return rc;
    };
    constexpr int64_t W = dev::kWaveRows;
    S* pv = nullptr;
    int32_t *offlen = nullptr, *lev = nullptr, *lcnt = nullptr, *lmax = nullptr, *words = nullptr;
    int rc = EIGSOL_OK;
    if ((rc = dalloc((void**)&pv, n * sizeof(S))) || (rc = dalloc((void**)&offlen, n * 4)) ||
        (rc = dalloc((void**)&lev, n * 4)) || (rc = dalloc((void**)&lcnt, (n + 1) * 4)) ||
        (rc = dalloc((void**)&lmax, (n + 1) * 4)) || (rc = dalloc((void**)&words, 64)))
        return finish(rc);
    if (hipHostMalloc(&hostw, 64, hipHostMallocDefault) != hipSuccess) return finish(fail(EIGSOL_E_HIP, "hipHostMalloc"));
    // words: [0..2] flags, [3] deepest level, [4] err, [5] ticket
    hipMemsetAsync(words, 0, 64, st);
    hipMemsetAsync(lev, 0xFF, n * 4, st);
    hipMemsetAsync(lcnt, 0, (n + 1) * 4, st);
    hipMemsetAsync(lmax, 0, (n + 1) * 4, st);
    const unsigned gb = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL((dev::tri_rows_kernel<S>), dim3(gb), dim3(256), 0, st, A->rowptr, A->col, val, n,
                       make_sigma<S>(sre, sim), pv, offlen, words);
    EIGSOL_HIP(hipMemcpyAsync(hostw, words, 64, hipMemcpyDeviceToHost, st));
    if (hipStreamSynchronize(st) != hipSuccess) return finish(fail(EIGSOL_E_HIP, "triangular analysis: row scan"));
    const bool up = !hostw[0], lo = !hostw[1];
    if (!up && !lo) {
        declined = true;
        return finish(EIGSOL_OK);
    }
    if (hostw[2]) return finish(fail(EIGSOL_E_SOLVER, "solve_shifted: SparseLU factorization failed"));
    hipLaunchKernelGGL(dev::tri_level_kernel, dim3(std::max(1, 4 * ctx->num_cus)), dim3(256), 0, st, A->rowptr, A->col,
                       offlen, n, up ? 1 : 0, lev, reinterpret_cast<uint32_t*>(words + 5), lcnt, lmax, words + 3,
                       words + 4);
    EIGSOL_HIP(hipMemcpyAsync(hostw, words, 64, hipMemcpyDeviceToHost, st));
    if (hipStreamSynchronize(st) != hipSuccess) return finish(fail(EIGSOL_E_HIP, "triangular analysis: levels"));
    if (hostw[4]) {   // a dependency wait ran out of time: build on the host instead
        declined = true;
        return finish(EIGSOL_OK);
    }
    const int32_t nlevels = hostw[3] + 1;
    std::vector<int32_t> hcnt(nlevels), hmax(nlevels);
    EIGSOL_HIP(hipMemcpyAsync(hcnt.data(), lcnt, nlevels * 4, hipMemcpyDeviceToHost, st));
    EIGSOL_HIP(hipMemcpyAsync(hmax.data(), lmax, nlevels * 4, hipMemcpyDeviceToHost, st));
    EIGSOL_HIP(hipStreamSynchronize(st));
    std::vector<int64_t> lstart(nlevels + 1, 0), lcount(hcnt.begin(), hcnt.end());
    for (int32_t l = 0; l < nlevels; ++l) lstart[l + 1] = lstart[l] + ((lcount[l] + W - 1) / W) * W;
    f = new ShiftFactor();
    f->ctx = ctx;
    ctx_retain(ctx);
    f->dtype = A->dtype;
    f->n = n;
    f->sig_re = sre;
    f->sig_im = sim;
    f->nnz_total = nnz;
    f->upper = up ? 1 : 0;
    f->nlevels = nlevels;
    f->npos = (int32_t)lstart[nlevels];
    if (const char* e = std::getenv("EIGSOL_TRSV_HEAD")) f->wave_head = std::strcmp(e, "block") ? 1 : 0;
    f->hlevels = head_levels<S>(lstart, lcount, hmax, f->nlevels, f->wave_head != 0);
    if (const char* e = std::getenv("EIGSOL_TRSV_POLL_FAST"))
        f->poll_fast = (f->poll_fast & ~0xffff) | std::min(0xffff, std::max(0, std::atoi(e)));
    if (const char* e = std::getenv("EIGSOL_TRSV_POLL_SLOW"))
        f->poll_fast = (f->poll_fast & 0xffff) | (std::min(7, std::max(0, std::atoi(e))) << 16);
    if (const char* e = std::getenv("EIGSOL_TRSV_POLL_MODE")) f->poll_mode = std::atoi(e);
    f->hpos = (int32_t)lstart[f->hlevels];
    {   // tail variant: the rule of factor_tri_host
        int64_t trows = 0, wide = 0;
        for (int32_t l = f->hlevels; l < f->nlevels; ++l) {
            trows += lcount[l];
            if (lcount[l] >= 65536) wide += lcount[l];
        }
        f->tail_chunks = (trows > 0 && 2 * wide < trows) ? 1 : 0;
        if (const char* e = std::getenv("EIGSOL_TRSV_TAIL")) f->tail_chunks = std::strcmp(e, "slice") ? 1 : 0;
    }
    if (!f->tail_chunks || (f->hpos > 0 && !f->wave_head)) {
        declined = true;
        return finish(EIGSOL_OK);
    }
    // positions: rows sorted by level, at each level's padded start
    int bits = 1;
    while (bits < 31 && (int64_t(1) << bits) <= (int64_t)(nlevels - 1)) ++bits;
    int32_t *lev_s = nullptr, *rows_s = nullptr, *ustart = nullptr, *pstart = nullptr, *plen = nullptr;
    if ((rc = dalloc((void**)&lev_s, n * 4)) || (rc = dalloc((void**)&rows_s, n * 4)) ||
        (rc = dalloc((void**)&ustart, (size_t)nlevels * 4)) || (rc = dalloc((void**)&pstart, (size_t)nlevels * 4)) ||
        (rc = dalloc((void**)&plen, ((size_t)f->npos + 1) * 4)))
        return finish(rc);
    if (tri_sort_rows_by_level(st, lev, lev_s, rows_s, n, bits) != hipSuccess)
        return finish(fail(EIGSOL_E_HIP, "triangular analysis: level sort"));
    std::vector<int32_t> hu(nlevels), hp(nlevels);
    {
        int64_t u = 0;
        for (int32_t l = 0; l < nlevels; ++l) {
            hu[l] = (int32_t)u;
            hp[l] = (int32_t)lstart[l];
            u += lcount[l];
        }
    }
    EIGSOL_HIP(hipMemcpyAsync(ustart, hu.data(), (size_t)nlevels * 4, hipMemcpyHostToDevice, st));
    EIGSOL_HIP(hipMemcpyAsync(pstart, hp.data(), (size_t)nlevels * 4, hipMemcpyHostToDevice, st));
    const int64_t npos = f->npos;
    EIGSOL_TRY(dev_upload(st, (void**)&f->porder, nullptr, (size_t)npos * 4));
    EIGSOL_HIP(hipMemsetAsync(f->porder, 0xFF, (size_t)npos * 4, st));
    hipLaunchKernelGGL(dev::tri_order_kernel, dim3(gb), dim3(256), 0, st, lev_s, rows_s, n, ustart, pstart, f->porder);
    EIGSOL_TRY(dev_upload(st, (void**)&f->order, nullptr, (size_t)f->hpos * 4));
    if (f->hpos > 0)
        EIGSOL_HIP(hipMemcpyAsync(f->order, f->porder, (size_t)f->hpos * 4, hipMemcpyDeviceToDevice, st));
    // position-indexed chunk CSR: pivots, row pointers (scan of the off-diagonal counts), entries
    const S one = make_sigma<S>(1.0, 0.0);
    EIGSOL_TRY(dev_upload(st, &f->ppiv, nullptr, (size_t)npos * sizeof(S)));
    EIGSOL_TRY(dev_upload(st, (void**)&f->pptr, nullptr, ((size_t)npos + 1) * 4));
    hipLaunchKernelGGL((dev::tri_poslen_kernel<S>), dim3((unsigned)((npos + 256) / 256)), dim3(256), 0, st, f->porder,
                       npos, offlen, pv, one, plen, static_cast<S*>(f->ppiv));
    if (tri_exclusive_scan(st, plen, f->pptr, npos) != hipSuccess)
        return finish(fail(EIGSOL_E_HIP, "triangular analysis: row pointer scan"));
    EIGSOL_HIP(hipMemcpyAsync(hostw + 5, f->pptr + npos, 4, hipMemcpyDeviceToHost, st));
    EIGSOL_HIP(hipStreamSynchronize(st));
    f->nnz_off = hostw[5];
    EIGSOL_TRY(dev_upload(st, (void**)&f->pcol, nullptr, (size_t)f->nnz_off * 4));
    EIGSOL_TRY(dev_upload(st, &f->pval, nullptr, (size_t)f->nnz_off * sizeof(S)));
    hipLaunchKernelGGL((dev::tri_gather_kernel<S>), dim3((unsigned)((npos * dev::kRowLanes + 255) / 256)), dim3(256), 0,
                       st, f->porder, npos, f->pptr, A->rowptr, A->col, val, offlen, f->pcol, static_cast<S*>(f->pval));
    f->chunk0 = f->hpos / dev::kWaveRows;
    f->nchunks = f->npos / dev::kWaveRows;
    {   // rows past 16 entries in the tail: the second entry of every lane is polled with the first
        int32_t longest = 0;
        for (int32_t l = f->hlevels; l < f->nlevels; ++l) longest = std::max(longest, hmax[l]);
        f->chunk_two = longest > dev::kRowLanes ? 1 : 0;
        if (const char* e = std::getenv("EIGSOL_TRSV_TWO")) f->chunk_two = std::atoi(e) != 0;
    }
    // one-wave head: passes of <= 16 rows inside a level, padded to the ring depth
    std::vector<int2> ptab;
    for (int32_t l = 0; l < f->hlevels; ++l) {
        const int32_t p0 = (int32_t)lstart[l], p1 = (int32_t)(lstart[l] + lcount[l]);
        for (int32_t p = p0; p < p1; p += dev::kWHeadRows) ptab.push_back(make_int2(p, std::min(dev::kWHeadRows, p1 - p)));
    }
    const int32_t nreal = (int32_t)ptab.size();
    int32_t nw = nreal;
    while (nw % dev::kWHeadDepth) ++nw;
    f->nwpass = f->hpos > 0 ? nw : 0;
    const size_t wslots = (size_t)f->nwpass * 256, wrows = (size_t)f->nwpass * dev::kWHeadRows;
    EIGSOL_TRY(dev_upload(st, &f->wval, nullptr, wslots * sizeof(S)));
    EIGSOL_TRY(dev_upload(st, (void**)&f->wcol, nullptr, wslots * 4));
    EIGSOL_TRY(dev_upload(st, &f->wrp, nullptr, wrows * sizeof(S)));
    EIGSOL_TRY(dev_upload(st, (void**)&f->wdst, nullptr, wrows * 4));
    if (f->nwpass > 0) {
        int32_t* rowpos = nullptr;
        int2* dtab = nullptr;
        if ((rc = dalloc((void**)&rowpos, n * 4)) || (rc = dalloc((void**)&dtab, (size_t)nreal * sizeof(int2))))
            return finish(rc);
        EIGSOL_HIP(hipMemcpyAsync(dtab, ptab.data(), (size_t)nreal * sizeof(int2), hipMemcpyHostToDevice, st));
        EIGSOL_HIP(hipMemsetAsync(rowpos, 0xFF, n * 4, st));
        EIGSOL_HIP(hipMemsetAsync(f->wval, 0, wslots * sizeof(S), st));
        EIGSOL_HIP(hipMemsetAsync(f->wdst, 0xFF, wrows * 4, st));
        hipLaunchKernelGGL((dev::fill_kernel<int32_t>), dim3(256), dim3(256), 0, st, f->wcol, (int64_t)wslots, f->hpos);
        hipLaunchKernelGGL((dev::fill_kernel<S>), dim3(64), dim3(256), 0, st, static_cast<S*>(f->wrp), (int64_t)wrows, one);
        hipLaunchKernelGGL(dev::tri_rowpos_kernel, dim3((unsigned)((f->hpos + 255) / 256)), dim3(256), 0, st, f->porder,
                           f->hpos, rowpos);
        hipLaunchKernelGGL((dev::tri_whead_kernel<S>), dim3((unsigned)((nreal * dev::kWHeadRows + 255) / 256)), dim3(256),
                           0, st, dtab, nreal, f->porder, A->rowptr, A->col, val, pv, rowpos, static_cast<S*>(f->wval),
                           f->wcol, static_cast<S*>(f->wrp), f->wdst);
    }
    // the one-workgroup head's tables stay empty (npass = 0: that head is not built here)
    EIGSOL_TRY(dev_upload(st, (void**)&f->hcol, nullptr, 0));
    EIGSOL_TRY(dev_upload(st, &f->hval, nullptr, 0));
    EIGSOL_TRY(dev_upload(st, &f->hpiv, nullptr, 0));
    EIGSOL_TRY(dev_upload(st, (void**)&f->passes, nullptr, 0));
    // slice tail: none (nslices = 0), but the empty slice 0 the slice kernels may prefetch exists
    {
        f->slice_b = 4;
        if (const char* e = std::getenv("EIGSOL_TRSV_SLICE_B")) {
            const int b = std::atoi(e);
            if (b == 4 || b == 8 || b == 16) f->slice_b = b;
        }
        const int32_t Bs = f->slice_b;
        f->nslices = 0;
        const std::vector<int2> smeta(1, make_int2(0, Bs));
        const std::vector<int32_t> trow(64, -1), tcol((size_t)64 * Bs, (int32_t)n);
        const std::vector<S> tpiv(64, one), tval((size_t)64 * Bs, s_zero<S>());
        EIGSOL_TRY(dev_upload(st, (void**)&f->smeta, smeta.data(), smeta.size() * sizeof(int2)));
        EIGSOL_TRY(dev_upload(st, (void**)&f->trow, trow.data(), trow.size() * 4));
        EIGSOL_TRY(dev_upload(st, &f->tpiv, tpiv.data(), tpiv.size() * sizeof(S)));
        EIGSOL_TRY(dev_upload(st, (void**)&f->tcol, tcol.data(), tcol.size() * 4));
        EIGSOL_TRY(dev_upload(st, &f->tval, tval.data(), tval.size() * sizeof(S)));
        EIGSOL_HIP(hipStreamSynchronize(st));   // the small host vectors above go out of scope
    }
    if (hipGetLastError() != hipSuccess) return finish(fail(EIGSOL_E_HIP, "triangular analysis: launch"));
    if ((rc = tri_launch_setup<S>(f)) != EIGSOL_OK) return finish(rc);
    if ((rc = tri_state_alloc<S>(f)) != EIGSOL_OK) return finish(rc);
    f->kind = 0;
    tri_dump<S>(f);
    return finish(EIGSOL_OK);
}

// triangular factor from host CSR arrays (the ILU(0) factors of the GMRES path, gmres.hip)
int shift_factor_tri(eigsol_ctx* ctx, int dtype, int64_t n, std::vector<int32_t>& rp, std::vector<int32_t>& ci,
                     const void* vals, bool up, ShiftFactor** out) {
    // the GMRES path's L / U (host arrays): uploaded once and analysed and laid out on the device
    // like a triangular A (round 5: the 1M general-sparse factor's two host layouts took ~0.8 s);
    // EIGSOL_TRSV_HOST=1 or a declined device analysis keeps the host build (the same bytes)
    auto run = [&](auto tag) {
        using S = decltype(tag);
        const char* host_env = std::getenv("EIGSOL_TRSV_HOST");
        if (n > 0 && !(host_env && std::atoi(host_env))) {
            // a bare device CSR (row pointers, columns, values): all the device analysis reads
            eigsol_csr A;
            A.ctx = ctx;
            A.dtype = dtype;
            A.nrows = A.ncols = n;
            A.nnz = rp[n];
            hipStream_t st = ctx->stream;
            int rc = EIGSOL_OK;
            if (hipMalloc(&A.rowptr, (n + 1) * 4) != hipSuccess || hipMalloc(&A.col, std::max<int64_t>(1, A.nnz) * 4) != hipSuccess ||
                hipMalloc(&A.val, std::max<int64_t>(1, A.nnz) * sizeof(S)) != hipSuccess)
                rc = fail(EIGSOL_E_HIP, "solve_shifted: triangular factor upload");
            if (rc == EIGSOL_OK) {
                hipMemcpyAsync(A.rowptr, rp.data(), (n + 1) * 4, hipMemcpyHostToDevice, st);
                hipMemcpyAsync(A.col, ci.data(), A.nnz * 4, hipMemcpyHostToDevice, st);
                hipMemcpyAsync(A.val, vals, A.nnz * sizeof(S), hipMemcpyHostToDevice, st);
            }
            bool declined = false;
            if (rc == EIGSOL_OK) rc = factor_tri_device<S>(&A, 0.0, 0.0, out, declined);
            hipStreamSynchronize(st);
            for (void* p : {(void*)A.rowptr, (void*)A.col, A.val})
                if (p) hipFree(p);
            A.rowptr = nullptr;
            A.col = nullptr;
            A.val = nullptr;
            if (!declined || rc != EIGSOL_OK) return rc;
        }
        std::vector<S> v(static_cast<const S*>(vals), static_cast<const S*>(vals) + rp[n]);
        return factor_tri_host<S>(ctx, dtype, n, rp, ci, v, up, 0.0, 0.0, out);
    };
    switch (dtype) {
        case EIGSOL_C128: return run(cplx{});
        case EIGSOL_F32: return run(0.0f);
        case EIGSOL_C64: return run(cplxf{});
        default: return run(0.0);
    }
}

// A triangular factor given as device CSR arrays (the GMRES path's L / U, split on the device):
// analysed and laid out on the device; a declined analysis or EIGSOL_TRSV_HOST=1 takes the host
// build on a downloaded copy (the same bytes).  The arrays stay the caller's.
int shift_factor_tri_dev(eigsol_ctx* ctx, int dtype, int64_t n, int32_t* rp, int32_t* ci, void* vals, int64_t nnz,
                         bool up, ShiftFactor** out) {
    auto run = [&](auto tag) -> int {
        using S = decltype(tag);
        hipStream_t st = ctx->stream;
        const char* host_env = std::getenv("EIGSOL_TRSV_HOST");
        if (n > 0 && !(host_env && std::atoi(host_env))) {
            eigsol_csr A;
            A.ctx = ctx;
            A.dtype = dtype;
            A.nrows = A.ncols = n;
            A.nnz = nnz;
            A.rowptr = rp;
            A.col = ci;
            A.val = vals;
            bool declined = false;
            const int rc = factor_tri_device<S>(&A, 0.0, 0.0, out, declined);
            A.rowptr = nullptr;
            A.col = nullptr;
            A.val = nullptr;
            if (!declined || rc != EIGSOL_OK) return rc;
        }
        std::vector<int32_t> hrp(n + 1), hci(nnz);
        std::vector<S> hv(nnz);
        EIGSOL_HIP(hipMemcpyAsync(hrp.data(), rp, (n + 1) * 4, hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(hipMemcpyAsync(hci.data(), ci, nnz * 4, hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(hipMemcpyAsync(hv.data(), vals, nnz * sizeof(S), hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(hipStreamSynchronize(st));
        return factor_tri_host<S>(ctx, dtype, n, hrp, hci, hv, up, 0.0, 0.0, out);
    };
    switch (dtype) {
        case EIGSOL_C128: return run(cplx{});
        case EIGSOL_F32: return run(0.0f);
        case EIGSOL_C64: return run(cplxf{});
        default: return run(0.0);
    }
}

int shift_factor_csr(eigsol_csr* A, const void* sigma, ShiftFactor** out) {
    if (A->dist) return fail(EIGSOL_E_UNSUPPORTED, "shifted inverse iteration: row-sharded matrices are not supported");
    double s[2] = {0.0, 0.0};
    load_scalar(sigma, A->dtype, s[0], s[1]);
    EIGSOL_HIP(hipSetDevice(A->ctx->device));
    switch (A->dtype) {
        case EIGSOL_C128: return factor_csr_t<cplx>(A, s[0], s[1], out);
        case EIGSOL_F32: return factor_csr_t<float>(A, s[0], 0.0, out);
        case EIGSOL_C64: return factor_csr_t<cplxf>(A, s[0], s[1], out);
        default: return factor_csr_t<double>(A, s[0], 0.0, out);
    }
}

int shift_grid(const ShiftFactor* f) { return (f->kind == 0 || f->dense_multi) ? f->grid : 1; }

// a new run of the iteration (session begin): no lagged check of the previous run is carried over
void shift_lag_reset(ShiftFactor* f) {
    f->lag_prev = false;
    if (f->gm) gmres_lag_reset(f->gm);
}

int shift_error(ShiftFactor* f) {
    if (f->kind != 0 && !f->dense_multi) return EIGSOL_OK;
    if (!f->hpin) EIGSOL_HIP(hipHostMalloc(&f->hpin, kPinBytes, hipHostMallocDefault));
    int32_t* he = static_cast<int32_t*>(f->hpin);
    EIGSOL_HIP(hipMemcpyAsync(he, f->err, 4, hipMemcpyDeviceToHost, f->ctx->stream));
    EIGSOL_HIP(stream_wait(f->ctx->stream));
    const int32_t e = *he;
    if (e) return fail(EIGSOL_E_SOLVER, "triangular solve: dependency wait exceeded its bound (internal error)");
    return EIGSOL_OK;
}

// buffers of the multi-solve launches, allocated by the first iteration launch (plain solves, e.g. the
// GMRES path's ILU(0) factors, never need them)
template <class S>
static int multi_alloc(ShiftFactor* f) {
    if (f->kpart) return EIGSOL_OK;
    hipStream_t st = f->ctx->stream;
    const int64_t n = f->n;
    const int K = f->multi;
    // buffer by buffer, so that a call after a failed allocation resumes instead of leaking
    for (int j = 0; j + 1 < K; ++j)
        if (!f->aux[j]) EIGSOL_HIP(hipMalloc(&f->aux[j], (size_t)std::max<int64_t>(n, 1) * sizeof(S)));
    for (int j = 1; j < K; ++j)
        for (void*& zb : f->zm[j]) {
            if (zb) continue;
            EIGSOL_HIP(hipMalloc(&zb, (size_t)(n + 1) * sizeof(S)));
            const uint32_t sent = (uint32_t)(dev::kSent & 0xffffffffu);
            EIGSOL_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(zb), (int)sent, n * sizeof(S) / 4, st));
            EIGSOL_HIP(hipMemsetAsync(static_cast<char*>(zb) + n * sizeof(S), 0, sizeof(S), st));
        }
    if (!f->kblk) EIGSOL_HIP(hipMalloc(&f->kblk, (size_t)(K - 1) * std::max(1, f->red_grid) * sizeof(dev::part4)));
    EIGSOL_HIP(hipMalloc(&f->kpart, (size_t)(K - 1) * sizeof(dev::part4)));   // last: marks the set complete
    EIGSOL_HIP(hipMemsetAsync(f->kpart, 0, (size_t)(K - 1) * sizeof(dev::part4), st));
    return EIGSOL_OK;
}

// the final iterate of a multi-solve launch that stopped on solve j < K - 1 (final_parity 2 + j)
void* shift_aux(const ShiftFactor* f, int j) { return (j >= 0 && j < dev::kMaxMulti - 1) ? f->aux[j] : nullptr; }

// x = M^-1 (b / bdiv) by the GMRES family; single precision through f->promo (widen, solve, narrow)
template <class S>
static int gm_solve_s(ShiftFactor* f, const void* b, double bdiv, void* y, const double* guess, bool lag = false) {
    if constexpr (kGmres<S>) {
        return lag ? gmres_solve_lag(f->gm, b, bdiv, y) : gmres_solve(f->gm, b, bdiv, y, guess);
    } else {
        using W = GmresScalar<S>;
        hipStream_t st = f->ctx->stream;
        W* wb = static_cast<W*>(f->promo);
        W* wy = wb + f->n;
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(4096, (f->n + 255) / 256));
        hipLaunchKernelGGL((dev::convert_kernel<S, W>), dim3(grid), dim3(256), 0, st, static_cast<const S*>(b), wb, f->n);
        EIGSOL_HIP(hipGetLastError());
        const int rc = lag ? gmres_solve_lag(f->gm, wb, bdiv, wy) : gmres_solve(f->gm, wb, bdiv, wy, guess);
        if (rc != EIGSOL_OK) return rc;
        hipLaunchKernelGGL((dev::convert_kernel<W, S>), dim3(grid), dim3(256), 0, st, wy, static_cast<S*>(y), f->n);
        EIGSOL_HIP(hipGetLastError());
        return EIGSOL_OK;
    }
}

template <class S>
static int shift_launch_t(ShiftFactor* f, bool iter, const void* b, void* y, void* buf0, void* buf1,
                          PowerCtl* ctl, const void* rank_part, void* my_part, void* trace, int parity,
                          bool first = false) {
    hipStream_t st = f->ctx->stream;
    if (f->kind == 2) {
        // ILU(0)-preconditioned GMRES: host-driven (one sync per Arnoldi step), so the iteration is
        // prologue launch -> host reads the stop decision -> solve -> partials launch
        if (!iter) {
            const int rc = gm_solve_s<S>(f, b, 0.0, y, nullptr);
            if (rc != EIGSOL_E_SOLVER) return rc;
            EIGSOL_TRY(gmres_dense_fallback<S>(f, rc));
            return shift_launch_t<S>(f, iter, b, y, buf0, buf1, ctl, rank_part, my_part, trace, parity);
        }
        dev::TriArgs<S> a{};
        a.n = f->n;
        a.work = f->work;
        a.wave_part = static_cast<dev::part4*>(f->wave_part);
        a.buf0 = static_cast<S*>(buf0);
        a.buf1 = static_cast<S*>(buf1);
        a.ctl = ctl;
        a.rank_part = static_cast<const dev::part4*>(rank_part);
        a.my_part = static_cast<dev::part4*>(my_part);
        a.trace = static_cast<S*>(trace);
        a.sig_re = f->sig_re;
        a.sig_im = f->sig_im;
        hipLaunchKernelGGL((dev::shift_decide_kernel<S>), dim3(1), dim3(64), 0, st, a, parity);
        struct Decision {
            PowerCarry cr;
            int32_t done;
        };
        static_assert(sizeof(Decision) <= kPinBytes, "pinned scratch");
        if (!f->hpin) EIGSOL_HIP(hipHostMalloc(&f->hpin, kPinBytes, hipHostMallocDefault));
        Decision* hd = static_cast<Decision*>(f->hpin);
        EIGSOL_HIP(hipMemcpyAsync(&hd->done, &ctl->done, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(hipMemcpyAsync(&hd->cr, &ctl->st[parity ^ 1], sizeof(PowerCarry), hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(stream_wait(st));
        if (f->lag_prev) {
            // the previous launch's direct solve was checked without a host wait (gmres_solve_lag): read
            // the check now; a miss redoes that iteration with the checked solve (and GMRES refinement),
            // its partials, and this launch's decision.  The previous launch read B[parity] and wrote
            // B[parity ^ 1]... in its own parity: it solved from buffer (parity ? buf1 : buf0) into
            // (parity ? buf0 : buf1), and neither has been touched since.
            f->lag_prev = false;
            const int v = gmres_lag_verdict(f->gm);
            if (v != EIGSOL_OK && v != EIGSOL_E_SOLVER) return v;
            if (v == EIGSOL_E_SOLVER) {
                const int pp = parity ^ 1;
                const int rc = gm_solve_s<S>(f, pp ? buf0 : buf1, f->lag_bdiv, pp ? buf1 : buf0, nullptr);
                if (rc == EIGSOL_E_SOLVER) {
                    // the checked solve failed too: the densified LU redoes the previous launch (its
                    // prologue re-takes that launch's decision from the same carry), then this one
                    EIGSOL_TRY(gmres_dense_fallback<S>(f, rc));
                    EIGSOL_HIP(hipMemsetAsync(&ctl->done, 0, sizeof(int32_t), st));
                    EIGSOL_TRY(shift_launch_t<S>(f, iter, b, y, buf0, buf1, ctl, rank_part, my_part, trace, pp));
                    return shift_launch_t<S>(f, iter, b, y, buf0, buf1, ctl, rank_part, my_part, trace, parity);
                }
                EIGSOL_TRY(rc);
                hipLaunchKernelGGL((dev::shift_part_kernel<S>), dim3(f->red_grid), dim3(dev::kThreads), 0, st, a, pp);
                EIGSOL_HIP(hipGetLastError());
                // this launch's decision again, from the corrected partials (the prologue writes the
                // same carry slot and trace entry; a stop it had decided is undone first)
                EIGSOL_HIP(hipMemsetAsync(&ctl->done, 0, sizeof(int32_t), st));
                hipLaunchKernelGGL((dev::shift_decide_kernel<S>), dim3(1), dim3(64), 0, st, a, parity);
                EIGSOL_HIP(hipMemcpyAsync(&hd->done, &ctl->done, sizeof(int32_t), hipMemcpyDeviceToHost, st));
                EIGSOL_HIP(hipMemcpyAsync(&hd->cr, &ctl->st[parity ^ 1], sizeof(PowerCarry), hipMemcpyDeviceToHost, st));
                EIGSOL_HIP(stream_wait(st));
            }
        }
        const int32_t done = hd->done;
        const PowerCarry cr = hd->cr;
        if (done) return EIGSOL_OK;
        // EIGSOL_GMRES_WARM=1: warm start from the latest eigenvalue estimate, y ~ x / (lambda - sigma)
        // (gmres.hip).  Off by default: round-4 A/B on config 5's matrix made general (tools/gmres_warm_ab.py)
        // gave 54 against 55 Arnoldi steps over the run and 9.1 against 8.9 ms per iteration - the
        // guess only beats x0 = 0 once the iterate's residual is below |lambda - sigma|, i.e. in the
        // last one or two iterations
        static const bool warm = [] {
            const char* e = std::getenv("EIGSOL_GMRES_WARM");
            return e && std::atoi(e) != 0;
        }();
        double guess[2] = {0.0, 0.0};
        bool use_guess = false;
        if (warm && cr.t >= 1) {
            const double dre = cr.rho_re - f->sig_re, dim = dtype_complex(f->dtype) ? cr.rho_im - f->sig_im : 0.0;
            const double d2 = dre * dre + dim * dim;
            if (d2 > 0.0 && std::isfinite(d2)) {
                guess[0] = dre / d2;
                guess[1] = -dim / d2;
                use_guess = true;
            }
        }
        // the direct solve's check is read at the next launch's decision wait (one host wait per
        // iteration instead of two) where the factor is complete and needs no refinement by design
        const bool lag = !use_guess && gmres_can_lag(f->gm);
        const int rc = gm_solve_s<S>(f, parity ? buf0 : buf1, cr.nrm, parity ? buf1 : buf0, use_guess ? guess : nullptr,
                                     lag);
        if (lag && rc == EIGSOL_OK) {
            f->lag_prev = true;
            f->lag_bdiv = cr.nrm;
        }
        if (rc == EIGSOL_E_SOLVER) {
            // switch to the densified LU and redo this launch on it: the dense kernel's prologue
            // re-evaluates the same decision from the same carry record (idempotent)
            EIGSOL_TRY(gmres_dense_fallback<S>(f, rc));
            return shift_launch_t<S>(f, iter, b, y, buf0, buf1, ctl, rank_part, my_part, trace, parity);
        }
        EIGSOL_TRY(rc);
        hipLaunchKernelGGL((dev::shift_part_kernel<S>), dim3(f->red_grid), dim3(dev::kThreads), 0, st, a, parity);
        EIGSOL_HIP(hipGetLastError());
        return EIGSOL_OK;
    }
    if (f->kind == 3)
        return band_launch(f->band, iter, b, y, buf0, buf1, ctl, rank_part, my_part, trace, parity);
    if (f->kind == 0) {
        dev::TriArgs<S> a{};
        a.order = f->order;
        a.n = f->n;
        const int e = ++f->epoch;
        a.zcur = static_cast<S*>(f->z[e & 1]);
        a.znext = static_cast<S*>(f->z[(e + 1) & 1]);
        a.work = f->work;
        a.err = f->err;
        a.wave_part = static_cast<dev::part4*>(f->wave_part);
        a.b_plain = static_cast<const S*>(b);
        a.y_plain = static_cast<S*>(y);
        a.buf0 = static_cast<S*>(buf0);
        a.buf1 = static_cast<S*>(buf1);
        a.ctl = ctl;
        a.rank_part = static_cast<const dev::part4*>(rank_part);
        a.my_part = static_cast<dev::part4*>(my_part);
        a.trace = static_cast<S*>(trace);
        a.sig_re = f->sig_re;
        a.sig_im = f->sig_im;
        a.hcol = f->hcol;
        a.hval = static_cast<const S*>(f->hval);
        a.hpiv = static_cast<const S*>(f->hpiv);
        a.passes = f->passes;
        a.npass = f->npass;
        a.hpos = f->hpos;
        a.poll_fast = f->poll_fast;
        a.poll_mode = f->poll_mode;
        a.wval = static_cast<const S*>(f->wval);
        a.wcol = f->wcol;
        a.wrp = static_cast<const S*>(f->wrp);
        a.wdst = f->wdst;
        a.nwpass = f->nwpass;
        // multi-solve launch; a session's launch 0 is a single solve (it measures the growth that
        // scales the chained solves of the later launches, shift_multi_prologue)
        const bool pair = iter && f->multi > 1 && !first;
        a.K = 1;
        a.zk[0] = a.zcur;
        a.zkn[0] = a.znext;
        if (pair) {
            EIGSOL_TRY(multi_alloc<S>(f));
            const int em = ++f->epoch_m;   // its own epoch: plain solves in between never skip a reset
            a.K = f->multi;
            for (int j = 1; j < f->multi; ++j) {
                a.zk[j] = static_cast<S*>(f->zm[j][em & 1]);
                a.zkn[j] = static_cast<S*>(f->zm[j][(em + 1) & 1]);
            }
            for (int j = 0; j + 1 < f->multi; ++j) a.aux[j] = static_cast<S*>(f->aux[j]);
            a.kpart = static_cast<dev::part4*>(f->kpart);
            a.kblk = static_cast<dev::part4*>(f->kblk);
        }
        if (f->hpos > 0 && f->wave_head && pair) {
            a.hconc = f->hconc;
            const size_t wl = (size_t)(f->hpos + 1) * sizeof(S) * (f->hconc ? f->multi : 1) + (f->hconc ? 16 : 0);
            const void* hk = reinterpret_cast<const void*>(dev::sptrsv_whead_kernel<S, true, true>);
            EIGSOL_HIP(hipFuncSetAttribute(hk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)wl));
            hipLaunchKernelGGL((dev::sptrsv_whead_kernel<S, true, true>), dim3(1), dim3(dev::kWHeadThreads), wl, st, a,
                               parity);
        } else if (f->hpos > 0 && f->wave_head) {
            const size_t wl = (size_t)(f->hpos + 1) * sizeof(S);
            const void* hk = iter ? reinterpret_cast<const void*>(dev::sptrsv_whead_kernel<S, true>)
                                  : reinterpret_cast<const void*>(dev::sptrsv_whead_kernel<S, false>);
            EIGSOL_HIP(hipFuncSetAttribute(hk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)wl));
            if (iter) hipLaunchKernelGGL((dev::sptrsv_whead_kernel<S, true>), dim3(1), dim3(dev::kWHeadThreads), wl, st, a, parity);
            else hipLaunchKernelGGL((dev::sptrsv_whead_kernel<S, false>), dim3(1), dim3(dev::kWHeadThreads), wl, st, a, parity);
        }
        const size_t hl = (size_t)(f->hpos + 1) * sizeof(S) + (size_t)f->npass * sizeof(int2);
        if (f->hpos > 0 && !f->wave_head) {
            const void* hk = iter ? reinterpret_cast<const void*>(dev::sptrsv_head_kernel<S, true>)
                                  : reinterpret_cast<const void*>(dev::sptrsv_head_kernel<S, false>);
            EIGSOL_HIP(hipFuncSetAttribute(hk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)hl));
            if (iter) hipLaunchKernelGGL((dev::sptrsv_head_kernel<S, true>), dim3(1), dim3(dev::kHeadThreads), hl, st, a, parity);
            else hipLaunchKernelGGL((dev::sptrsv_head_kernel<S, false>), dim3(1), dim3(dev::kHeadThreads), hl, st, a, parity);
        }
        // a head that failed to launch would leave the tail polling for values nobody writes
        EIGSOL_HIP(hipGetLastError());
        // cooperative: the static chunk schedule needs every wave of the grid resident
        void* kargs[] = {&a, &parity};
        a.smeta = f->smeta;
        a.trow = f->trow;
        a.tpiv = static_cast<const S*>(f->tpiv);
        a.tcol = f->tcol;
        a.tval = static_cast<const S*>(f->tval);
        a.nslices = f->nslices;
        a.porder = f->porder;
        a.pptr = f->pptr;
        a.pcol = f->pcol;
        a.pval = static_cast<const S*>(f->pval);
        a.ppiv = static_cast<const S*>(f->ppiv);
        a.chunk0 = f->chunk0;
        a.nchunks = f->nchunks;
        const void* tk = pair ? reinterpret_cast<const void*>(dev::sptrsv_chunk_role_kernel<S>)
                         : !f->tail_chunks ? slice_kernel_ptr<S>(f->slice_b, iter)
                         : f->chunk_two ? (iter ? reinterpret_cast<const void*>(dev::sptrsv_chunk_kernel<S, true, true>)
                                                : reinterpret_cast<const void*>(dev::sptrsv_chunk_kernel<S, false, true>))
                         : iter ? reinterpret_cast<const void*>(dev::sptrsv_chunk_kernel<S, true>)
                                : reinterpret_cast<const void*>(dev::sptrsv_chunk_kernel<S, false>);
        const int tgrid = pair ? f->grid_multi : f->grid;
        // EIGSOL_TRSV_NO_COOP=1: the same kernel through an ordinary launch, for profiling only
        // (rocprofv3 7.2 segfaults in its exit-time finaliser after any cooperative launch,
        // tools/coop_prof_repro.hip); the grid is one residency round, so on an otherwise idle
        // device every wave is resident anyway
        static const bool no_coop = std::getenv("EIGSOL_TRSV_NO_COOP") != nullptr;
        if (no_coop) EIGSOL_HIP(hipLaunchKernel(tk, dim3(tgrid), dim3(dev::kThreads), kargs, 0, st));
        else EIGSOL_HIP(hipLaunchCooperativeKernel(tk, dim3(tgrid), dim3(dev::kThreads), kargs, 0, st));
        if (pair)
            hipLaunchKernelGGL((dev::shift_multi_part_kernel<S>), dim3(f->red_grid), dim3(dev::kThreads), 0, st, a,
                               parity);
        else if (iter)   // every tail kernel publishes y in zcur (the chunk tail only there)
            hipLaunchKernelGGL((dev::shift_part_kernel<S, true>), dim3(f->red_grid), dim3(dev::kThreads), 0, st, a,
                               parity);
    } else if constexpr (!kDenseLU<S>) {
        return fail(EIGSOL_E_UNSUPPORTED, "single-precision dense factor");
    } else if (f->dense_multi) {
        dev::DenseTriArgs<S> a{};
        a.lu = static_cast<const S*>(f->lu);
        a.perm = f->perm;
        a.n = f->n;
        a.nblk = f->nchunks;
        a.epoch = ++f->epoch;
        a.flag_f = f->flag_f;
        a.flag_b = f->flag_b;
        a.tinv = static_cast<const S*>(f->tinv);
        a.tmul = static_cast<const S*>(f->tmul);
        a.z = static_cast<S*>(f->zf);
        a.b_plain = static_cast<const S*>(b);
        a.y_plain = static_cast<S*>(y);
        a.buf0 = static_cast<S*>(buf0);
        a.buf1 = static_cast<S*>(buf1);
        a.ctl = ctl;
        a.rank_part = static_cast<const dev::part4*>(rank_part);
        a.my_part = static_cast<dev::part4*>(my_part);
        a.wave_part = static_cast<dev::part4*>(f->wave_part);
        a.work = f->work;
        a.err = f->err;
        a.trace = static_cast<S*>(trace);
        a.sig_re = f->sig_re;
        a.sig_im = f->sig_im;
        // cooperative: the persistent block-row workgroups wait on each other's epoch flags
        void* kargs[] = {&a, &parity};
        const void* dk = f->dense_v == 2 ? dense_trsv2_ptr<S>(iter, dense_pf_mode<S>())
                                         : (iter ? reinterpret_cast<const void*>(dev::dense_trsv_kernel<S, true>)
                                                 : reinterpret_cast<const void*>(dev::dense_trsv_kernel<S, false>));
        EIGSOL_HIP(hipLaunchCooperativeKernel(dk, dim3(f->grid), dim3(256), kargs, 0, st));
    } else {
        dev::DenseSolveArgs<S> a{};
        a.lu = static_cast<const S*>(f->lu);
        a.perm = f->perm;
        a.n = f->n;
        a.b_plain = static_cast<const S*>(b);
        a.y_plain = static_cast<S*>(y);
        a.buf0 = static_cast<S*>(buf0);
        a.buf1 = static_cast<S*>(buf1);
        a.ctl = ctl;
        a.rank_part = static_cast<const dev::part4*>(rank_part);
        a.my_part = static_cast<dev::part4*>(my_part);
        a.trace = static_cast<S*>(trace);
        a.sig_re = f->sig_re;
        a.sig_im = f->sig_im;
        const void* k = iter ? reinterpret_cast<const void*>(dev::dense_lu_solve_kernel<S, true>)
                             : reinterpret_cast<const void*>(dev::dense_lu_solve_kernel<S, false>);
        EIGSOL_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)f->lds_bytes));
        if (iter) hipLaunchKernelGGL((dev::dense_lu_solve_kernel<S, true>), dim3(1), dim3(1024), f->lds_bytes, st, a, parity);
        else hipLaunchKernelGGL((dev::dense_lu_solve_kernel<S, false>), dim3(1), dim3(1024), f->lds_bytes, st, a, parity);
    }
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

template <class F>
static int by_dtype(int dtype, F&& fn) {
    switch (dtype) {
        case EIGSOL_C128: return fn(cplx{});
        case EIGSOL_F32: return fn(0.0f);
        case EIGSOL_C64: return fn(cplxf{});
        default: return fn(0.0);
    }
}

int shift_iter_launch(ShiftFactor* f, void* buf0, void* buf1, PowerCtl* ctl, const void* rank_part,
                      void* my_part, void* trace, int parity, int first) {
    return by_dtype(f->dtype, [&](auto tag) {
        return shift_launch_t<decltype(tag)>(f, true, nullptr, nullptr, buf0, buf1, ctl, rank_part, my_part, trace, parity,
                                             first != 0);
    });
}

int shift_solve_launch(ShiftFactor* f, const void* b_dev, void* y_dev) {
    return by_dtype(f->dtype, [&](auto tag) {
        return shift_launch_t<decltype(tag)>(f, false, b_dev, y_dev, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0);
    });
}

// algorithmic bytes of one solve (the SpTRSV counts like the SpMV) and variant
void shift_info(const ShiftFactor* f, double* bytes, int32_t* variant, int32_t* tiles) {
    const double sb = (double)scalar_bytes(f->dtype), n = (double)f->n;
    if (f->kind == 2) {
        gmres_info(f->gm, bytes, tiles);
        if (variant) {
            const int c = gmres_complete(f->gm);
            *variant = c == 2 ? 19 : c ? 18 : 7;   // 19: nested-dissection multifrontal LU
        }
    } else if (f->kind == 3) {
        band_info(f->band, bytes, tiles);
        if (variant) *variant = 8;
    } else if (f->kind == 0) {
        if (bytes) *bytes = (sb + 4.0) * (double)f->nnz_total + 4.0 * (n + 1.0) + 2.0 * sb * n;
        if (variant) *variant = f->multi > 1 ? 10 + f->multi : 3;   // 12/13/14: 2/3/4 iterations per launch
        if (tiles) *tiles = f->nlevels;
    } else {
        if (bytes) *bytes = sb * n * n + 2.0 * sb * n;
        if (variant) *variant = 4;
        if (tiles) *tiles = 0;
    }
}

}  // namespace eigsol

// Blocked Householder Hessenberg reduction (gfx950), the reference's reflector convention, for
// S = double and S = std::complex<double> (cplx).
//
// to_hessenberg_dense<S> (src/qr_method/to_hessenberg.hpp:38-77) applies H_j = I - 2 v_j v_j^H
// from both sides for every column j.  Here the reflectors of a panel of nb columns are
// accumulated in compact-WY form Q = H_k ... H_{k+nb-1} = I - V T V^H (T upper triangular,
// T(i,i) = 2) together with Y = A V T, and the trailing matrix is updated once per panel:
//     A <- Q^H (A Q) = (I - V T^H V^H)(A - Y V^H)
// (the dlahr2/dgehrd organisation; zlahr2/zgehrd for complex S).  Per panel column the only
// full-matrix pass is the GEMV y = A(:, j+1:n) v_j (BLAS-2, half the flops); everything else is
// GEMMs per panel.  Reflectors are generated exactly as the reference does (alpha =
// -phase(x0) ||x||, phase = x0 / |x0| (1 at x0 = 0), skipped when ||x(1:)|| == 0), so H matches the
// unblocked reduction to rounding.  For real S every conjugation below is the identity and the
// arithmetic is the real path's, operation for operation.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "kernels_common.hpp"
#include "mfma_rankk.hpp"

namespace eigsol {
namespace dev {

// Per-scalar configuration: panel width (complex panels are half as wide, so the rank-2 nb
// trailing update stays within rankk_mfma's K <= 32 for cplx), the largest order the per-column
// panel keeps in LDS, and the largest order of the cooperative panel (v staged in LDS).
template <class S> struct HessCfg;
template <> struct HessCfg<double> {
    static constexpr int NB = 32;
    static constexpr int kMaxLdsN = 16384;   // 128 KiB
    static constexpr int kCoopMaxN = 8192;   // v in LDS (64 KiB) and at most 2 rows per lane
};
template <> struct HessCfg<cplx> {
    static constexpr int NB = 16;
    static constexpr int kMaxLdsN = 8192;    // 128 KiB
    static constexpr int kCoopMaxN = 4096;   // v (64 KiB) + the partial / row buffers: < 160 KiB
};
// single precision (float / complex<float>): the same reductions in the scalar's own type; norms
// and the reflector's scalars are formed in double and rounded, like the power method's partials
template <> struct HessCfg<float> {
    static constexpr int NB = 32;
    static constexpr int kMaxLdsN = 16384;
    static constexpr int kCoopMaxN = 8192;
};
template <> struct HessCfg<cplxf> {
    static constexpr int NB = 16;
    static constexpr int kMaxLdsN = 16384;
    static constexpr int kCoopMaxN = 8192;
};
constexpr int kGemvCols = 128;      // columns per GEMV partial

__device__ __forceinline__ double cj(double a) { return a; }
__device__ __forceinline__ cplx cj(cplx a) { return cplx{a.re, -a.im}; }
__device__ __forceinline__ float cj(float a) { return a; }
__device__ __forceinline__ cplxf cj(cplxf a) { return cplxf{a.re, -a.im}; }
__device__ __forceinline__ double wsum(double v) { return wave_sum(v); }
__device__ __forceinline__ cplx wsum(cplx v) { return cplx{wave_sum(v.re), wave_sum(v.im)}; }
__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ cplxf wsum(cplxf v) { return cplxf{wsum(v.re), wsum(v.im)}; }
__device__ __forceinline__ void st_ag(double* p, double v) { st_agent(p, v); }
__device__ __forceinline__ void st_ag(cplx* p, cplx v) {
    st_agent(&p->re, v.re);
    st_agent(&p->im, v.im);
}
__device__ __forceinline__ void st_ag(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ag(cplxf* p, cplxf v) {
    st_ag(&p->re, v.re);
    st_ag(&p->im, v.im);
}
__device__ __forceinline__ double ld_ag(const double* p) { return ld_agent(p); }
__device__ __forceinline__ cplx ld_ag(const cplx* p) { return cplx{ld_agent(&p->re), ld_agent(&p->im)}; }
__device__ __forceinline__ float ld_ag(const float* p) {
    return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ cplxf ld_ag(const cplxf* p) { return cplxf{ld_ag(&p->re), ld_ag(&p->im)}; }
__device__ __forceinline__ double scal(double a, double s) { return a * s; }
__device__ __forceinline__ cplx scal(cplx a, double s) { return cplx{a.re * s, a.im * s}; }
__device__ __forceinline__ float scal(float a, double s) { return a * (float)s; }
__device__ __forceinline__ cplxf scal(cplxf a, double s) { return cplxf{a.re * (float)s, a.im * (float)s}; }
__device__ __forceinline__ double two_x(double a) { return 2.0 * a; }
__device__ __forceinline__ cplx two_x(cplx a) { return cplx{2.0 * a.re, 2.0 * a.im}; }
__device__ __forceinline__ float two_x(float a) { return 2.0f * a; }
__device__ __forceinline__ cplxf two_x(cplxf a) { return cplxf{2.0f * a.re, 2.0f * a.im}; }
__device__ __forceinline__ double neg2(double a) { return -2.0 * a; }
__device__ __forceinline__ cplx neg2(cplx a) { return cplx{-2.0 * a.re, -2.0 * a.im}; }
__device__ __forceinline__ float neg2(float a) { return -2.0f * a; }
__device__ __forceinline__ cplxf neg2(cplxf a) { return cplxf{-2.0f * a.re, -2.0f * a.im}; }

// The reference's reflector from x0 = a(j+1) and tail = ||a(j+2:)||^2 (to_hessenberg.hpp:45-65):
// alpha = -phase(x0) ||x||, v0 = x0 - alpha, rv = 1 / ||(v0, x(1:))||; sk when skipped.
__device__ __forceinline__ void hess_reflector(double x0, double tail, bool& sk, double& v0, double& rv, double& alpha) {
    sk = tail == 0.0;
    v0 = 0.0; rv = 0.0; alpha = 0.0;
    if (!sk) {
        const double nx = sqrt(tail + x0 * x0);
        const double sign = x0 == 0.0 ? 1.0 : (x0 > 0.0 ? 1.0 : -1.0);
        alpha = -sign * nx;
        v0 = x0 - alpha;
        const double vn = sqrt(tail + v0 * v0);
        if (vn == 0.0) sk = true;
        else rv = 1.0 / vn;
    }
}
__device__ __forceinline__ void hess_reflector(cplx x0, double tail, bool& sk, cplx& v0, double& rv, cplx& alpha) {
    sk = tail == 0.0;
    v0 = cplx{0.0, 0.0}; rv = 0.0; alpha = cplx{0.0, 0.0};
    if (!sk) {
        const double nx = sqrt(tail + sq_abs(x0));
        cplx ph{1.0, 0.0};
        if (x0.re != 0.0 || x0.im != 0.0) {
            const double ia = 1.0 / hypot(x0.re, x0.im);   // hh_make_kernel's phase (qr.hip)
            ph = cplx{x0.re * ia, x0.im * ia};
        }
        alpha = cplx{-ph.re * nx, -ph.im * nx};
        v0 = sub(x0, alpha);
        const double vn = sqrt(tail + sq_abs(v0));
        if (vn == 0.0) sk = true;
        else rv = 1.0 / vn;
    }
}

// single precision: the reflector's scalars in double (x0 exact in double), rounded to S
__device__ __forceinline__ void hess_reflector(float x0, double tail, bool& sk, float& v0, double& rv, float& alpha) {
    double v0d, ad;
    hess_reflector((double)x0, tail, sk, v0d, rv, ad);
    v0 = (float)v0d;
    alpha = (float)ad;
}
__device__ __forceinline__ void hess_reflector(cplxf x0, double tail, bool& sk, cplxf& v0, double& rv, cplxf& alpha) {
    cplx v0d, ad;
    hess_reflector(cplx{(double)x0.re, (double)x0.im}, tail, sk, v0d, rv, ad);
    v0 = cplxf{(float)v0d.re, (float)v0d.im};
    alpha = cplxf{(float)ad.re, (float)ad.im};
}

// block (1024 threads) sum of NB partials per thread -> sw[0..cnt)
template <class S, int NB>
__device__ __forceinline__ void block_sum_vec(S (&p)[NB], int cnt, S* red /*16*NB*/, S* sw) {
    const int w = threadIdx.x >> 6, ln = threadIdx.x & 63;
#pragma unroll
    for (int c = 0; c < NB; ++c) {
        if (c < cnt) {                      // static register index (no scratch)
            const S s = wsum(p[c]);
            if (ln == 0) red[w * NB + c] = s;
        }
    }
    __syncthreads();
    if ((int)threadIdx.x < cnt) {
        S s = s_zero<S>();
        for (int q = 0; q < (int)(blockDim.x >> 6); ++q) s = add(s, red[q * NB + threadIdx.x]);
        sw[threadIdx.x] = s;
    }
    __syncthreads();
}

// Panel column j (local index i): apply the panel's earlier reflectors from the right (via Y) and
// the left (via V, T), generate reflector i from rows j+1.., store the reduced column, and
// t = V(:, 0:i)^H v_i for the T / Y recursions.
template <class S>
__global__ __launch_bounds__(1024) void hess_panel_col(S* A, int n, int k, int j, int i, S* V, const S* Y,
                                                       const S* T, S* tvec, int* skip) {
    constexpr int NB = HessCfg<S>::NB;
    extern __shared__ double a_raw[];      // column j (n scalars)
    S* a = reinterpret_cast<S*>(a_raw);
    __shared__ S red[16 * NB];
    __shared__ S sw[NB];
    __shared__ S sw2[NB];
    __shared__ S vj[NB];
    __shared__ double rtl[17];   // block sum of the tail norm (its own scratch: red holds S)
    __shared__ double s_tail;
    const int tid = threadIdx.x, nt = blockDim.x;
    if (tid < i) vj[tid] = cj(V[j + (int64_t)tid * n]);   // conj of row j of V
    __syncthreads();
    // right: a -= Y(:, 0:i) V(j, 0:i)^H
    for (int r = tid; r < n; r += nt) {
        S x = A[r + (int64_t)j * n];
        for (int c = 0; c < i; ++c) x = sub(x, mul(Y[r + (int64_t)c * n], vj[c]));
        a[r] = x;
    }
    __syncthreads();
    // left: w = V^H a (rows k+1..), w = T^H w, a -= V w
    if (i > 0) {
        S p[NB];
#pragma unroll
        for (int c = 0; c < NB; ++c) p[c] = s_zero<S>();
        for (int r = k + 1 + tid; r < n; r += nt) {
            const S x = a[r];
#pragma unroll
            for (int c = 0; c < NB; ++c)
                if (c < i) p[c] = add(p[c], mul(cj(V[r + (int64_t)c * n]), x));
        }
        block_sum_vec<S, NB>(p, i, red, sw);
        if (tid < i) {
            S s = s_zero<S>();
            for (int c = 0; c <= tid; ++c) s = add(s, mul(cj(T[c + tid * NB]), sw[c]));   // (T^H w)_tid
            sw2[tid] = s;
        }
        __syncthreads();
        for (int r = k + 1 + tid; r < n; r += nt) {
            S x = a[r];
            for (int c = 0; c < i; ++c) x = sub(x, mul(V[r + (int64_t)c * n], sw2[c]));
            a[r] = x;
        }
        __syncthreads();
    }
    // reflector from a(j+1 : n)
    double tl = 0.0;
    for (int r = j + 2 + tid; r < n; r += nt) tl += sq_abs(a[r]);
    {
        double pp[1] = {tl};
        block_sum_vec<double, 1>(pp, 1, rtl, rtl + 16);
        if (tid == 0) s_tail = rtl[16];
        __syncthreads();
    }
    const double tail = s_tail;
    const S x0 = a[j + 1];
    bool sk;
    S v0, alpha;
    double rv;
    hess_reflector(x0, tail, sk, v0, rv, alpha);
    S* vcol = V + (int64_t)i * n;
    for (int r = tid; r < n; r += nt) {
        S v = s_zero<S>();
        if (!sk && r > j) v = scal(r == j + 1 ? v0 : a[r], rv);
        vcol[r] = v;
    }
    // store the reduced column (alpha on the subdiagonal, zeros below)
    for (int r = tid; r < n; r += nt) {
        S x = a[r];
        if (!sk && r == j + 1) x = alpha;
        if (!sk && r > j + 1) x = s_zero<S>();
        A[r + (int64_t)j * n] = x;
    }
    if (tid == 0) *skip = sk ? 1 : 0;
    __syncthreads();
    // t = V(:, 0:i)^H v (rows j+1..)
    if (i > 0) {
        S p[NB];
#pragma unroll
        for (int c = 0; c < NB; ++c) p[c] = s_zero<S>();
        if (!sk)
            for (int r = j + 1 + tid; r < n; r += nt) {
                const S v = vcol[r];
#pragma unroll
                for (int c = 0; c < NB; ++c)
                    if (c < i) p[c] = add(p[c], mul(cj(V[r + (int64_t)c * n]), v));
            }
        block_sum_vec<S, NB>(p, i, red, sw);
        if (tid < i) tvec[tid] = sw[tid];
    }
}

// y partials: ypart[ch * n + r] = sum_{c in chunk ch} A(r, c) v(c), columns j+1..n-1
template <class S>
__global__ __launch_bounds__(256) void hess_gemv(const S* A, int n, int c0, const S* v, S* ypart, const int* skip) {
    if (*skip) return;
    const int r = blockIdx.x * 256 + threadIdx.x;
    const int ch = blockIdx.y;
    const int cb = c0 + ch * kGemvCols;
    const int ce = min(n, cb + kGemvCols);
    if (r >= n) return;
    S s = s_zero<S>();
    for (int c = cb; c < ce; ++c) s = add(s, mul(A[r + (int64_t)c * n], v[c]));
    ypart[(int64_t)ch * n + r] = s;
}

// Y(:, i) = 2 (y - Y(:, 0:i) t);  T(0:i, i) = -2 T(0:i, 0:i) t, T(i, i) = 2
template <class S>
__global__ __launch_bounds__(256) void hess_y(int n, int i, int nch, const S* ypart, const S* tvec, S* Y, S* T,
                                              const int* skip) {
    constexpr int NB = HessCfg<S>::NB;
    const int r = blockIdx.x * 256 + threadIdx.x;
    const bool sk = *skip != 0;
    if (r < n) {
        S y = s_zero<S>();
        if (!sk) {
            for (int ch = 0; ch < nch; ++ch) y = add(y, ypart[(int64_t)ch * n + r]);
            for (int c = 0; c < i; ++c) y = sub(y, mul(Y[r + (int64_t)c * n], tvec[c]));
        }
        Y[r + (int64_t)i * n] = sk ? s_zero<S>() : two_x(y);
    }
    if (blockIdx.x == 0 && (int)threadIdx.x <= i) {
        const int c = threadIdx.x;
        S tc;
        set_re_im(tc, 2.0, 0.0);
        if (c < i) {
            S s = s_zero<S>();
            if (!sk)
                for (int q = c; q < i; ++q) s = add(s, mul(T[c + q * NB], tvec[q]));
            tc = neg2(s);
        }
        T[c + i * NB] = tc;
    }
}

// ------------------------------------------------------------------ blocked Householder QR
// qr_decompose_dense<S> (src/qr_method/qr_decompose.hpp:46-85) in compact-WY form: the panel's
// reflectors H_i = I - 2 v_i v_i^H (the reference's convention, reflector from the diagonal row
// down) give Q_p = H_k ... H_{k+nb-1} = I - V T V^H; per panel R(k:, c1:) <- Q_p^H R(k:, c1:)
// and Q(:, k:) <- Q(:, k:) Q_p are GEMMs.  Panel column j (local i), one workgroup with the column
// in LDS: apply the panel's earlier reflectors (a -= V T^H V^H a, rows k..), generate reflector i
// from rows j.., store R's column (alpha on the diagonal, exact zeros below), V(:, i) and the
// T column (T(0:i, i) = -2 T(0:i, 0:i) V(:, 0:i)^H v_i, T(i, i) = 2).
template <class S>
__global__ __launch_bounds__(1024) void qr_panel_col(S* R, int m, int k, int j, int i, S* V, S* T) {
    constexpr int NB = 32;
    extern __shared__ double qa_raw[];     // column j (m scalars)
    S* a = reinterpret_cast<S*>(qa_raw);
    __shared__ S red[16 * NB];
    __shared__ S sw[NB];
    __shared__ S sw2[NB];
    __shared__ double rtl[17];   // block sum of the tail norm (its own scratch: red holds S)
    __shared__ double s_tail;
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int r = tid; r < m; r += nt) a[r] = R[r + (int64_t)j * m];
    __syncthreads();
    if (i > 0) {   // a(k:) -= V T^H V^H a(k:)
        S p[NB];
#pragma unroll
        for (int c = 0; c < NB; ++c) p[c] = s_zero<S>();
        for (int r = k + tid; r < m; r += nt) {
            const S x = a[r];
#pragma unroll
            for (int c = 0; c < NB; ++c)
                if (c < i) p[c] = add(p[c], mul(cj(V[r + (int64_t)c * m]), x));
        }
        block_sum_vec<S, NB>(p, i, red, sw);
        if (tid < i) {
            S s = s_zero<S>();
            for (int c = 0; c <= tid; ++c) s = add(s, mul(cj(T[c + tid * NB]), sw[c]));
            sw2[tid] = s;
        }
        __syncthreads();
        for (int r = k + tid; r < m; r += nt) {
            S x = a[r];
            for (int c = 0; c < i; ++c) x = sub(x, mul(V[r + (int64_t)c * m], sw2[c]));
            a[r] = x;
        }
        __syncthreads();
    }
    double tl = 0.0;
    for (int r = j + 1 + tid; r < m; r += nt) tl += sq_abs(a[r]);
    {
        double pp[1] = {tl};
        block_sum_vec<double, 1>(pp, 1, rtl, rtl + 16);
        if (tid == 0) s_tail = rtl[16];
        __syncthreads();
    }
    const double tail = s_tail;
    bool sk;
    S v0, alpha;
    double rv;
    hess_reflector(a[j], tail, sk, v0, rv, alpha);
    S* vcol = V + (int64_t)i * m;
    for (int r = tid; r < m; r += nt) {
        S v = s_zero<S>();
        if (!sk && r >= j) v = scal(r == j ? v0 : a[r], rv);
        vcol[r] = v;
        S x = a[r];
        if (!sk && r == j) x = alpha;
        if (!sk && r > j) x = s_zero<S>();
        R[r + (int64_t)j * m] = x;
    }
    __syncthreads();
    // t = V(:, 0:i)^H v (rows j..), then the T column
    S p[NB];
#pragma unroll
    for (int c = 0; c < NB; ++c) p[c] = s_zero<S>();
    if (!sk && i > 0)
        for (int r = j + tid; r < m; r += nt) {
            const S v = vcol[r];
#pragma unroll
            for (int c = 0; c < NB; ++c)
                if (c < i) p[c] = add(p[c], mul(cj(V[r + (int64_t)c * m]), v));
        }
    if (i > 0) block_sum_vec<S, NB>(p, i, red, sw);
    if (tid <= i) {
        S tc;
        set_re_im(tc, 2.0, 0.0);
        if (tid < i) {
            S s2 = s_zero<S>();
            if (!sk)
                for (int q = tid; q < i; ++q) s2 = add(s2, mul(T[tid + q * NB], sw[q]));
            tc = neg2(s2);
        }
        T[tid + i * NB] = tc;
    }
}

// ------------------------------------------------------------------ cooperative panel (one launch)
// The whole panel (32 columns) in ONE cooperative launch of G co-resident blocks (host: ~32 rows each); block
// b owns rows [b R, (b+1) R).  Per column, three grid barriers separate
//   P1  right update of column j (own rows, kept in LDS) + partials of V^T a
//   P2  w = T^T (sum of partials); left update; partial of ||a(j+2:)||^2; x0 = a(j+1)
//   P3  reflector (every block, redundantly, from the reduced scalars); v and the reduced column
//       for own rows; partials of t = V^T v
//   P4  GEMV y = A(:, j+1:n) v for own rows (v staged in LDS), Y(:, i) and the T column
// (P4 -> the next P1 needs no barrier: P1 reads only own rows and V(j+1, 0:i), published in P3.
// The block partials are double-buffered for the same reason: a block that has finished P4 writes
// the next column's P1 partials while a slower block may still be gathering P3's, so P1/P2 and
// P3/P4 use separate halves of `part`.)
// Everything another block reads is written with agent-scope (sc1) stores and read with sc1 loads,
// so no L2 writeback/invalidate is needed; partial sums are combined in block order
// (deterministic).  The barrier spins are bounded: on expiry the kernel sets an error word and
// drains (the host then reports EIGSOL_E_HIP).
constexpr int kCoopThreads = 1024;
#ifndef EIGSOL_GEMV_BATCH
#define EIGSOL_GEMV_BATCH 16
#endif
#ifndef EIGSOL_HESS_SKIP_GEMV
#define EIGSOL_HESS_SKIP_GEMV 0   // timing experiments only
#endif
constexpr int kGemvBatch = EIGSOL_GEMV_BATCH;   // columns per GEMV step (loads in flight per lane)

template <class S>
struct CoopArgs {
    S* A;
    int n, k, nbp;
    S* V;
    S* Y;
    S* T;
    S* part;            // [2][G][NB]: P1 -> P2 partials in the first half, P3 -> P4 in the second
    double* tpart;      // [G]
    S* x0;              // a(j+1)
    unsigned* bar;      // barrier counters, 9 x 64 bytes (zeroed by the host before the launch)
    int* err;
    S* xu;              // kMerge: the column below row j + 1 before normalisation (n scalars)
    bool hier;          // two-level grid barrier (gridDim.x % 8 == 0)
};

__device__ __forceinline__ unsigned ld_agent_u32(const unsigned* p) {
    return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bar[0] counts arrivals of the whole grid; with hier (a grid that is a multiple of 8 blocks), block b
// first counts itself in its group's word bar[16 (1 + b % 8)] (the blocks one XCD holds, each group word on
// its own 64-byte line) and the group's last arriver adds the group to bar[0]: 8 + G / 8 serialised atomics
// per line instead of G on one
__device__ __forceinline__ void grid_barrier(unsigned* bar, unsigned& target, int* err, bool hier = false) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's sc1 stores are complete
    __syncthreads();
    target += gridDim.x;
    if (threadIdx.x == 0) {
        if (hier) {
            const unsigned gs = gridDim.x / 8;
            const unsigned old =
                __hip_atomic_fetch_add(bar + 16 * (1 + blockIdx.x % 8), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((old + 1) % gs == 0) __hip_atomic_fetch_add(bar, gs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        int spins = 0;
        while (ld_agent_u32(bar) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1 << 24)) { atomicOr(err, 1); break; }
        }
    }
    __syncthreads();
}

// kMerge (default; EIGSOL_HESS_MERGE=0: off): two grid barriers per column instead of three.  P2 also publishes
// the updated column below row j + 1 unnormalised (xu) with the partials of V^H over those rows;
// after its barrier every block forms the reflector from the reduced norm, scales xu into the GEMV's
// v on the fly, and t = V^H v = rv (conj(V(j+1, :)) v0 + the reduced partials) - no barrier between
// the reflector and the GEMV.  V(:, i) is then stored by each block for its own rows after that
// barrier, so the next column's P1 takes the one entry it reads from another block, V(j + 1, i),
// from the block's own copy (every block forms rv v0 itself).  The same reflectors; t and T round
// differently.
template <class S, int kCoopRowsPerLane, bool kMerge = false>
__global__ __launch_bounds__(kCoopThreads) void hess_panel_coop(CoopArgs<S> a) {
    constexpr int NB = HessCfg<S>::NB;
    extern __shared__ double vsh_raw[];      // v (n scalars) for the GEMV
    S* vsh = reinterpret_cast<S*>(vsh_raw);
    __shared__ S xs[kCoopRowsPerLane * 64];    // own rows of the current column
    __shared__ S ysum[16][kCoopRowsPerLane * 64];
    __shared__ S red[kCoopThreads];   // per-thread sums of block partials (and the norm partials as doubles)
    __shared__ S sv[NB], sw[NB], st[NB];
    __shared__ S Tl[NB * NB];   // this block's copy of T (every block forms each column from the same sums)
    __shared__ S s_scal[3];
    __shared__ double s_rv;
    __shared__ int s_sk;
    __shared__ S s_vrow;   // kMerge: V(j + 1, i) of the previous column (rv v0, or 0 when skipped)
    // Block partials of another phase: thread (s, c) loads blocks s, s + kSl, ... of column c at once
    // (independent sc1 loads) and sums them in that order; thread c then sums the kSl slices in order
    // (deterministic, the same in every block, for any grid size).
    constexpr int kSl = kCoopThreads / NB;
    auto gather = [&](const S* src, int cnt, S* dst) {
        const int nb = (int)gridDim.x;
        {
            const int c = threadIdx.x % NB, sl = threadIdx.x / NB;
            S acc = s_zero<S>();
            if (c < cnt) {
                constexpr int kU = 4;
                for (int b0 = sl; b0 < nb; b0 += kU * kSl) {
                    S t4[kU];
#pragma unroll
                    for (int u = 0; u < kU; ++u) {
                        const int b = b0 + u * kSl;
                        t4[u] = b < nb ? ld_ag(&src[b * NB + c]) : s_zero<S>();
                    }
#pragma unroll
                    for (int u = 0; u < kU; ++u) acc = add(acc, t4[u]);
                }
            }
            red[threadIdx.x] = acc;
        }
        __syncthreads();
        if ((int)threadIdx.x < cnt) {
            S acc = s_zero<S>();
            for (int sl = 0; sl < kSl; ++sl) acc = add(acc, red[sl * NB + threadIdx.x]);
            dst[threadIdx.x] = acc;
        }
        __syncthreads();
    };
    const int n = a.n, k = a.k;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int G = gridDim.x;
    const int R = (n + G - 1) / G;
    // row group: consecutive groups on one XCD (blocks are dealt to the 8 XCDs round-robin), so an
    // XCD's L2 sees 8 adjacent row stripes of every column; partials stay indexed by row group, so
    // every sum keeps its order
    // (4096^2: panels 151 -> 141 ms per reduction, rocprofv3 kernel trace, tools/hess_prof.sh)
    const int grp = (G % 8 == 0) ? ((int)blockIdx.x % 8) * (G / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
    const int r0 = grp * R, r1 = min(n, r0 + R);
    int rp = 64;   // lanes per column in the GEMV (a power of two >= R when R < 64; one row per lane)
    if (kCoopRowsPerLane == 1)
        while (rp > 8 && rp / 2 >= R) rp /= 2;
    unsigned target = 0;
    for (int e = tid; e < NB * NB; e += kCoopThreads) Tl[e] = s_zero<S>();
    for (int i = 0; i < a.nbp; ++i) {
        const int j = k + i;
        // ---------------- P1
        if (tid < i) sv[tid] = cj((kMerge && tid == i - 1) ? s_vrow : ld_ag(&a.V[j + (int64_t)tid * n]));
        __syncthreads();
        if (wv == 0)
            for (int q = 0; q < kCoopRowsPerLane; ++q) {
                const int r = r0 + lane + 64 * q;
                if (r < r1) {
                    S x = a.A[r + (int64_t)j * n];
                    for (int c = 0; c < i; ++c) x = sub(x, mul(a.Y[r + (int64_t)c * n], sv[c]));
                    xs[lane + 64 * q] = x;
                }
            }
        __syncthreads();
        // partials of w_c = sum_{r >= k+1} conj(V(r, c)) x(r): wave wv handles c = wv, wv + 16
        for (int c = wv; c < i; c += 16) {
            S p = s_zero<S>();
            for (int q = 0; q < kCoopRowsPerLane; ++q) {
                const int r = r0 + lane + 64 * q;
                if (r < r1 && r >= k + 1) p = add(p, mul(cj(a.V[r + (int64_t)c * n]), xs[lane + 64 * q]));
            }
            p = wsum(p);
            if (lane == 0) st_ag(&a.part[grp * NB + c], p);
        }
        grid_barrier(a.bar, target, a.err, a.hier);
        bool sk;
        if constexpr (kMerge) {
            // ---------------- P2 (merged): left update, norm partials, x0, xu, partials of V^H xu
            gather(a.part, i, sw);
            if (tid < i) {
                S s = s_zero<S>();
                for (int c = 0; c <= tid; ++c) s = add(s, mul(cj(Tl[c + tid * NB]), sw[c]));   // (T^H w)_tid
                st[tid] = s;
            }
            __syncthreads();
            double tl = 0.0;
            if (wv == 0)
                for (int q = 0; q < kCoopRowsPerLane; ++q) {
                    const int r = r0 + lane + 64 * q;
                    if (r < r1) {
                        S x = xs[lane + 64 * q];
                        if (r >= k + 1)
                            for (int c = 0; c < i; ++c) x = sub(x, mul(a.V[r + (int64_t)c * n], st[c]));
                        xs[lane + 64 * q] = x;
                        if (r >= j + 2) {
                            tl += sq_abs(x);
                            st_ag(&a.xu[r], x);
                        }
                        if (r == j + 1) st_ag(a.x0, x);
                    }
                }
            if (wv == 0) {
                tl = wave_sum(tl);
                if (lane == 0) st_agent(&a.tpart[grp], tl);
            }
            __syncthreads();
            for (int c = wv; c < i; c += 16) {
                S p = s_zero<S>();
                for (int q = 0; q < kCoopRowsPerLane; ++q) {
                    const int r = r0 + lane + 64 * q;
                    if (r < r1 && r >= j + 2) p = add(p, mul(cj(a.V[r + (int64_t)c * n]), xs[lane + 64 * q]));
                }
                p = wsum(p);
                if (lane == 0) st_ag(&a.part[(G + grp) * NB + c], p);
            }
            grid_barrier(a.bar, target, a.err, a.hier);
            // ---------------- P3 + P4: reflector (every block), own rows of V and the reduced column,
            // v for the GEMV from xu, t from the reduced partials
            double* redd = reinterpret_cast<double*>(red);
            if (tid < G) redd[tid] = ld_agent(&a.tpart[tid]);
            __syncthreads();
            if (tid == 0) {
                double tail = 0.0;
                for (int b = 0; b < G; ++b) tail += redd[b];
                const S x0 = ld_ag(a.x0);
                bool skr;
                S v0, alpha;
                double rv;
                hess_reflector(x0, tail, skr, v0, rv, alpha);
                s_sk = skr ? 1 : 0;
                s_scal[1] = v0;
                s_rv = rv;
                s_scal[2] = alpha;
                s_vrow = skr ? s_zero<S>() : scal(v0, rv);
            }
            __syncthreads();
            sk = s_sk != 0;
            const S v0 = s_scal[1], alpha = s_scal[2];
            const double rv = s_rv;
            if (wv == 0)
                for (int q = 0; q < kCoopRowsPerLane; ++q) {
                    const int r = r0 + lane + 64 * q;
                    if (r < r1) {
                        const S x = xs[lane + 64 * q];
                        S v = s_zero<S>();
                        if (!sk && r > j) v = scal(r == j + 1 ? v0 : x, rv);
                        st_ag(&a.V[r + (int64_t)i * n], v);
                        S red_col = x;
                        if (!sk && r == j + 1) red_col = alpha;
                        if (!sk && r > j + 1) red_col = s_zero<S>();
                        a.A[r + (int64_t)j * n] = red_col;
                    }
                }
            // v into LDS for every row: zero above row j + 1, rv v0 at j + 1, rv xu below
            for (int rb = tid; rb < n; rb += 4 * kCoopThreads) {
                S t4[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) t4[u] = ld_ag(&a.xu[min(max(rb + u * kCoopThreads, j + 2), n - 1)]);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int r = rb + u * kCoopThreads;
                    if (r < n) vsh[r] = (sk || r <= j) ? s_zero<S>() : scal(r == j + 1 ? v0 : t4[u], rv);
                }
            }
            __syncthreads();
            gather(a.part + (size_t)G * NB, i, sv);
            if (tid < i) {
                const S u = add(mul(cj(ld_ag(&a.V[(j + 1) + (int64_t)tid * n])), v0), sv[tid]);
                sv[tid] = sk ? s_zero<S>() : scal(u, rv);
            }
            __syncthreads();
        } else {
            // ---------------- P2
            gather(a.part, i, sw);
            if (tid < i) {
                S s = s_zero<S>();
                for (int c = 0; c <= tid; ++c) s = add(s, mul(cj(Tl[c + tid * NB]), sw[c]));   // (T^H w)_tid
                st[tid] = s;
            }
            __syncthreads();
            double tl = 0.0;
            if (wv == 0)
                for (int q = 0; q < kCoopRowsPerLane; ++q) {
                    const int r = r0 + lane + 64 * q;
                    if (r < r1) {
                        S x = xs[lane + 64 * q];
                        if (r >= k + 1)
                            for (int c = 0; c < i; ++c) x = sub(x, mul(a.V[r + (int64_t)c * n], st[c]));
                        xs[lane + 64 * q] = x;
                        if (r >= j + 2) tl += sq_abs(x);
                        if (r == j + 1) st_ag(a.x0, x);
                    }
                }
            if (wv == 0) {
                tl = wave_sum(tl);
                if (lane == 0) st_agent(&a.tpart[grp], tl);
            }
            grid_barrier(a.bar, target, a.err, a.hier);
            // ---------------- P3
            double* redd = reinterpret_cast<double*>(red);
            if (tid < G) redd[tid] = ld_agent(&a.tpart[tid]);
            __syncthreads();
            if (tid == 0) {
                double tail = 0.0;
                for (int b = 0; b < G; ++b) tail += redd[b];
                const S x0 = ld_ag(a.x0);
                bool sk;
                S v0, alpha;
                double rv;
                hess_reflector(x0, tail, sk, v0, rv, alpha);
                s_sk = sk ? 1 : 0;
                s_scal[1] = v0;
                s_rv = rv;
                s_scal[2] = alpha;
            }
            __syncthreads();
            sk = s_sk != 0;
            const S v0 = s_scal[1], alpha = s_scal[2];
            const double rv = s_rv;
            if (wv == 0)
                for (int q = 0; q < kCoopRowsPerLane; ++q) {
                    const int r = r0 + lane + 64 * q;
                    if (r < r1) {
                        const S x = xs[lane + 64 * q];
                        S v = s_zero<S>();
                        if (!sk && r > j) v = scal(r == j + 1 ? v0 : x, rv);
                        st_ag(&a.V[r + (int64_t)i * n], v);
                        xs[lane + 64 * q] = v;           // keep v for the t partials
                        S red_col = x;
                        if (!sk && r == j + 1) red_col = alpha;
                        if (!sk && r > j + 1) red_col = s_zero<S>();
                        a.A[r + (int64_t)j * n] = red_col;
                    }
                }
            __syncthreads();
            for (int c = wv; c < i; c += 16) {
                S p = s_zero<S>();
                for (int q = 0; q < kCoopRowsPerLane; ++q) {
                    const int r = r0 + lane + 64 * q;
                    if (r < r1) p = add(p, mul(cj(a.V[r + (int64_t)c * n]), xs[lane + 64 * q]));
                }
                p = wsum(p);
                if (lane == 0) st_ag(&a.part[(G + grp) * NB + c], p);
            }
            grid_barrier(a.bar, target, a.err, a.hier);
            // ---------------- P4
            // v into LDS: four independent coherent loads per thread in flight (clamped rows, so no
            // predicated load waits for the one before it)
            for (int rb = tid; rb < n; rb += 4 * kCoopThreads) {
                S t4[4];
    #pragma unroll
                for (int u = 0; u < 4; ++u) t4[u] = ld_ag(&a.V[min(rb + u * kCoopThreads, n - 1) + (int64_t)i * n]);
    #pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (rb + u * kCoopThreads < n) vsh[rb + u * kCoopThreads] = sk ? s_zero<S>() : t4[u];
            }
            __syncthreads();
            gather(a.part + (size_t)G * NB, i, sv);
            if (sk && tid < i) sv[tid] = s_zero<S>();
            __syncthreads();
        }
        S yacc[kCoopRowsPerLane];
#pragma unroll
        for (int q = 0; q < kCoopRowsPerLane; ++q) yacc[q] = s_zero<S>();
        if (!sk && !EIGSOL_HESS_SKIP_GEMV) {
            // kB columns per step with every load issued before the FMAs (bytes in flight: the
            // GEMV streams the trailing matrix once per column)
            // rp lanes per row group of a column, sub = 64 / rp columns per wave step: with fewer than
            // 64 rows per block (a larger grid) the wave's other lanes take the next columns
            const int nq = (r1 - r0 + 63) / 64;
            const int rl = lane & (rp - 1), sub = 64 / rp;
            const int cs = 16 * sub;
            int c = j + 1 + wv * sub + lane / rp;
            constexpr int kB = kGemvBatch * (int)sizeof(double) / (int)sizeof(S) / kCoopRowsPerLane;
            for (; c + cs * (kB - 1) < n; c += cs * kB) {
                S av[kB][kCoopRowsPerLane];
#pragma unroll
                for (int u = 0; u < kB; ++u)
#pragma unroll
                    for (int q = 0; q < kCoopRowsPerLane; ++q) {
                        const int r = min(r0 + rl + 64 * q, r1 - 1);
                        av[u][q] = q < nq ? a.A[r + (int64_t)(c + cs * u) * n] : s_zero<S>();
                    }
#pragma unroll
                for (int u = 0; u < kB; ++u) {
                    const S vc = vsh[c + cs * u];
#pragma unroll
                    for (int q = 0; q < kCoopRowsPerLane; ++q) yacc[q] = add(yacc[q], mul(av[u][q], vc));
                }
            }
            for (; c < n; c += cs) {
                const S vc = vsh[c];
#pragma unroll
                for (int q = 0; q < kCoopRowsPerLane; ++q) {
                    const int r = min(r0 + rl + 64 * q, r1 - 1);
                    if (q < nq) yacc[q] = add(yacc[q], mul(a.A[r + (int64_t)c * n], vc));
                }
            }
            // rows past r1 were clamped to r1 - 1: their sums are never stored
        }
#pragma unroll
        for (int q = 0; q < kCoopRowsPerLane; ++q) ysum[wv][lane + 64 * q] = yacc[q];
        __syncthreads();
        if (wv == 0)
            for (int q = 0; q < kCoopRowsPerLane; ++q) {
                const int r = r0 + lane + 64 * q;
                if (r < r1) {
                    S y = s_zero<S>();
                    for (int w = 0; w < 16; ++w)
                        for (int l = lane + 64 * q; l < 64 * (q + 1); l += rp) y = add(y, ysum[w][l]);
                    for (int c = 0; c < i; ++c) y = sub(y, mul(a.Y[r + (int64_t)c * n], sv[c]));
                    a.Y[r + (int64_t)i * n] = sk ? s_zero<S>() : two_x(y);
                }
            }
        // T column i in every block, from the LDS copy and the gathered sums (the same values and
        // order in every block); block 0 also publishes it for the trailing update
        if (tid <= i) {
            S tc;
            set_re_im(tc, 2.0, 0.0);
            if (tid < i) {
                S s = s_zero<S>();
                for (int q = tid; q < i; ++q) s = add(s, mul(Tl[tid + q * NB], sv[q]));
                tc = neg2(s);
            }
            Tl[tid + i * NB] = tc;
            if (blockIdx.x == 0) a.T[tid + i * NB] = tc;
        }
        __syncthreads();
    }
}

// The merged panel (two grid barriers per column) with fewer dependent round trips to memory: one row per
// lane (a grid of >= n / 64 blocks), the block's own rows of V(:, 0:i) and Y(:, 0:i) kept in LDS (the
// right and left updates and the partials of V^H a read no global memory), the own rows of A(:, j + 1)
// loaded before the second barrier, and everything the reflector and the GEMV need after that barrier
// (the norm partials, x0, xu, the partials of V^H xu and V(j + 1, 0:i)) loaded in one batch; V(j + 1, :)
// is also the next column's V(j, :).  The same operations in the same order as hess_panel_coop<S, 1, true>:
// bitwise its results (tests/test_gpu_qr.py::test_hessenberg_panel2_bitwise).
// kVG (orders past HessCfg<S>::kCoopMaxN, up to 64 rows per block x 256 blocks): v is not staged in LDS;
// the GEMV reads the published column xu and scales it on the fly (the same value as the staged v).
template <class S, bool kVG = false>
__global__ __launch_bounds__(kCoopThreads) void hess_panel_coop2(CoopArgs<S> a) {
    constexpr int NB = HessCfg<S>::NB;
    constexpr int kSl = kCoopThreads / NB;               // gather slices
    constexpr int kGU = 256 / kSl;                       // gather loads per thread (grid <= 256)
    constexpr int kXU = kVG ? 0 : HessCfg<S>::kCoopMaxN / kCoopThreads;   // xu loads per thread
    extern __shared__ double vsh_raw[];
    S* vsh = reinterpret_cast<S*>(vsh_raw);
    __shared__ S xs[64];
    __shared__ S ysum[16][64];
    __shared__ S red[kCoopThreads];
    __shared__ S vc[NB][64];     // own rows of V(:, c)
    __shared__ S yc[NB][64];     // own rows of Y(:, c)
    __shared__ double tps[256];
    __shared__ S sv[NB], sw[NB], st[NB], s_vj[NB];
    __shared__ S Tl[NB * NB];
    __shared__ S s_scal[3];
    __shared__ double s_rv;
    __shared__ int s_sk;
    auto gather2 = [&](const S* src, int cnt, S* dst) {   // hess_panel_coop's gather, the same order
        const int nb = (int)gridDim.x;
        {
            const int c = threadIdx.x % NB, sl = threadIdx.x / NB;
            S acc = s_zero<S>();
            if (c < cnt) {
                S t[kGU];
#pragma unroll
                for (int u = 0; u < kGU; ++u) {
                    const int b = sl + u * kSl;
                    t[u] = b < nb ? ld_ag(&src[b * NB + c]) : s_zero<S>();
                }
#pragma unroll
                for (int u = 0; u < kGU; ++u) acc = add(acc, t[u]);
            }
            red[threadIdx.x] = acc;
        }
        __syncthreads();
        if ((int)threadIdx.x < cnt) {
            S acc = s_zero<S>();
            for (int sl = 0; sl < kSl; ++sl) acc = add(acc, red[sl * NB + threadIdx.x]);
            dst[threadIdx.x] = acc;
        }
        __syncthreads();
    };
    const int n = a.n, k = a.k;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int G = gridDim.x;
    const int R = (n + G - 1) / G;
    const int grp = (G % 8 == 0) ? ((int)blockIdx.x % 8) * (G / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
    const int r0 = grp * R, r1 = min(n, r0 + R);
    int rp = 64;
    while (rp > 8 && rp / 2 >= R) rp /= 2;
    const int rown = r0 + lane;                 // wave 0: this lane's row
    const bool own = rown < r1;
    unsigned target = 0;
    for (int e = tid; e < NB * NB; e += kCoopThreads) Tl[e] = s_zero<S>();
    S acol = s_zero<S>();                       // wave 0: A(rown, j), loaded a column ahead
    if (wv == 0 && own) acol = a.A[rown + (int64_t)k * n];
    for (int i = 0; i < a.nbp; ++i) {
        const int j = k + i;
        // ---------------- P1 (no global loads)
        if (tid < i) sv[tid] = cj(s_vj[tid]);
        __syncthreads();
        if (wv == 0 && own) {
            S x = acol;
            for (int c = 0; c < i; ++c) x = sub(x, mul(yc[c][lane], sv[c]));
            xs[lane] = x;
        }
        __syncthreads();
        for (int c = wv; c < i; c += 16) {
            S p = s_zero<S>();
            if (own && rown >= k + 1) p = add(p, mul(cj(vc[c][lane]), xs[lane]));
            p = wsum(p);
            if (lane == 0) st_ag(&a.part[grp * NB + c], p);
        }
        grid_barrier(a.bar, target, a.err, a.hier);
        // ---------------- P2
        gather2(a.part, i, sw);
        if (tid < i) {
            S s = s_zero<S>();
            for (int c = 0; c <= tid; ++c) s = add(s, mul(cj(Tl[c + tid * NB]), sw[c]));
            st[tid] = s;
        }
        __syncthreads();
        if (wv == 0) {
            double tl = 0.0;
            if (own) {
                S x = xs[lane];
                if (rown >= k + 1)
                    for (int c = 0; c < i; ++c) x = sub(x, mul(vc[c][lane], st[c]));
                xs[lane] = x;
                if (rown >= j + 2) {
                    tl += sq_abs(x);
                    st_ag(&a.xu[rown], x);
                }
                if (rown == j + 1) st_ag(a.x0, x);
                if (i + 1 < a.nbp) acol = a.A[rown + (int64_t)(j + 1) * n];
            }
            tl = wave_sum(tl);
            if (lane == 0) st_agent(&a.tpart[grp], tl);
        }
        __syncthreads();
        for (int c = wv; c < i; c += 16) {
            S p = s_zero<S>();
            if (own && rown >= j + 2) p = add(p, mul(cj(vc[c][lane]), xs[lane]));
            p = wsum(p);
            if (lane == 0) st_ag(&a.part[(G + grp) * NB + c], p);
        }
        grid_barrier(a.bar, target, a.err, a.hier);
        // ---------------- P3 + P4: one batch of loads
        S xt[kXU > 0 ? kXU : 1];
#pragma unroll
        for (int u = 0; u < kXU; ++u) xt[u] = ld_ag(&a.xu[min(max(tid + u * kCoopThreads, j + 2), n - 1)]);
        S gt[kGU];
        const int gc = tid % NB, gsl = tid / NB;
#pragma unroll
        for (int u = 0; u < kGU; ++u) {
            const int b = gsl + u * kSl;
            gt[u] = (gc < i && b < G) ? ld_ag(&a.part[(G + b) * NB + gc]) : s_zero<S>();
        }
        const double tpv = tid < G ? ld_agent(&a.tpart[tid]) : 0.0;
        const S vrow = tid < i ? ld_ag(&a.V[(j + 1) + (int64_t)tid * n]) : s_zero<S>();
        const S x0 = ld_ag(a.x0);
        {
            S acc = s_zero<S>();
#pragma unroll
            for (int u = 0; u < kGU; ++u) acc = add(acc, gt[u]);
            red[tid] = acc;
        }
#pragma unroll
        for (int u = 0; u < kXU; ++u)
            if (tid + u * kCoopThreads < n) vsh[tid + u * kCoopThreads] = xt[u];   // scaled below
        if (tid < G) tps[tid] = tpv;
        __syncthreads();
        if (tid == 0) {
            double tail = 0.0;
            for (int b = 0; b < G; ++b) tail += tps[b];
            bool skr;
            S v0, alpha;
            double rv;
            hess_reflector(x0, tail, skr, v0, rv, alpha);
            s_sk = skr ? 1 : 0;
            s_scal[1] = v0;
            s_rv = rv;
            s_scal[2] = alpha;
        }
        if (tid < i) {
            S acc = s_zero<S>();
            for (int sl = 0; sl < kSl; ++sl) acc = add(acc, red[sl * NB + tid]);
            sw[tid] = acc;   // the reduced partials of V^H xu
        }
        __syncthreads();
        const bool sk = s_sk != 0;
        const S v0 = s_scal[1], alpha = s_scal[2];
        const double rv = s_rv;
        if (wv == 0 && own) {
            const S x = xs[lane];
            S v = s_zero<S>();
            if (!sk && rown > j) v = scal(rown == j + 1 ? v0 : x, rv);
            st_ag(&a.V[rown + (int64_t)i * n], v);
            vc[i][lane] = v;
            S red_col = x;
            if (!sk && rown == j + 1) red_col = alpha;
            if (!sk && rown > j + 1) red_col = s_zero<S>();
            a.A[rown + (int64_t)j * n] = red_col;
        }
#pragma unroll
        for (int u = 0; u < kXU; ++u) {
            const int r = tid + u * kCoopThreads;
            if (r < n) vsh[r] = (sk || r <= j) ? s_zero<S>() : scal(r == j + 1 ? v0 : vsh[r], rv);
        }
        if (tid < i) {
            const S u = add(mul(cj(vrow), v0), sw[tid]);
            sv[tid] = sk ? s_zero<S>() : scal(u, rv);
            s_vj[tid] = vrow;
        }
        if (tid == i) s_vj[i] = sk ? s_zero<S>() : scal(v0, rv);
        __syncthreads();
        S yacc = s_zero<S>();
        if (!sk && !EIGSOL_HESS_SKIP_GEMV) {
            const int rl = lane & (rp - 1), sub = 64 / rp;
            const int cs = 16 * sub;
            const int r = min(r0 + rl, r1 - 1);
            int c = j + 1 + wv * sub + lane / rp;
            if constexpr (kVG) {
                const S v0s = scal(v0, rv);
                constexpr int kB = kGemvBatch * (int)sizeof(double) / (int)sizeof(S) / 2;
                for (; c + cs * (kB - 1) < n; c += cs * kB) {
                    S av[kB], xv[kB];
#pragma unroll
                    for (int u = 0; u < kB; ++u) {
                        av[u] = a.A[r + (int64_t)(c + cs * u) * n];
                        xv[u] = ld_ag(&a.xu[max(c + cs * u, j + 2)]);
                    }
#pragma unroll
                    for (int u = 0; u < kB; ++u)
                        yacc = add(yacc, mul(av[u], c + cs * u == j + 1 ? v0s : scal(xv[u], rv)));
                }
                for (; c < n; c += cs)
                    yacc = add(yacc, mul(a.A[r + (int64_t)c * n], c == j + 1 ? v0s : scal(ld_ag(&a.xu[max(c, j + 2)]), rv)));
            } else {
                constexpr int kB = kGemvBatch * (int)sizeof(double) / (int)sizeof(S);
                for (; c + cs * (kB - 1) < n; c += cs * kB) {
                    S av[kB];
#pragma unroll
                    for (int u = 0; u < kB; ++u) av[u] = a.A[r + (int64_t)(c + cs * u) * n];
#pragma unroll
                    for (int u = 0; u < kB; ++u) yacc = add(yacc, mul(av[u], vsh[c + cs * u]));
                }
                for (; c < n; c += cs) yacc = add(yacc, mul(a.A[r + (int64_t)c * n], vsh[c]));
            }
        }
        ysum[wv][lane] = yacc;
        __syncthreads();
        if (wv == 0 && own) {
            S y = s_zero<S>();
            for (int w = 0; w < 16; ++w)
                for (int l = lane; l < 64; l += rp) y = add(y, ysum[w][l]);
            for (int c = 0; c < i; ++c) y = sub(y, mul(yc[c][lane], sv[c]));
            const S yv = sk ? s_zero<S>() : two_x(y);
            a.Y[rown + (int64_t)i * n] = yv;
            yc[i][lane] = yv;
        }
        if (tid <= i) {
            S tc;
            set_re_im(tc, 2.0, 0.0);
            if (tid < i) {
                S s = s_zero<S>();
                for (int q = tid; q < i; ++q) s = add(s, mul(Tl[tid + q * NB], sv[q]));
                tc = neg2(s);
            }
            Tl[tid + i * NB] = tc;
            if (blockIdx.x == 0) a.T[tid + i * NB] = tc;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ cooperative QR panel
// qr_blocked's panel (32 Householder columns of R, qr_decompose.hpp:46-85, with the compact-WY T of the
// panel) in ONE cooperative launch of G blocks, block b owning rows [b R, (b+1) R) (R <= 64: one row per
// lane of wave 0), instead of one single-workgroup launch per column that streams V three times through
// one CU.  Per column, two grid barriers:
//   P1  the column's own rows (kept in LDS) and the partials of V^H a over rows >= k
//   P2  p = sum of the partials, T's previous column from the previous column's t partials, w = T^H p,
//       a -= V w (own rows), partial of ||a(j+1:)||^2, x0 = a(j)
//   P3  the reflector (every block, from the same sums), V(:, i) and R(:, j) for own rows, partials of
//       t = V^H v (gathered after the next column's first barrier; the last column's after one more)
// The block's own rows of V are cached in LDS; partial sums are combined in block order (deterministic).
template <class S>
struct QrCoopArgs {
    S* R;
    int m, k, nbp;
    S* V;
    S* T;
    S* part;        // [2][G][32]: P1 partials, then the t partials
    double* tpart;  // [G]
    S* x0;
    unsigned* bar;
    int* err;
    bool hier;
};

template <class S>
__global__ __launch_bounds__(kCoopThreads) void qr_panel_coop(QrCoopArgs<S> a) {
    constexpr int NB = 32;
    constexpr int kSl = kCoopThreads / NB;
    constexpr int kGU = 256 / kSl;
    __shared__ S xs[64];
    __shared__ S vc[NB][64];
    __shared__ S red[kCoopThreads];
    __shared__ double tps[256];
    __shared__ S sp[NB], stt[NB], sw2[NB];
    __shared__ S Tl[NB * NB];
    __shared__ S s_scal[3];
    __shared__ double s_rv;
    __shared__ int s_sk, s_skprev;
    auto gather = [&](const S* src, int cnt, S* dst) {
        const int nb = (int)gridDim.x;
        {
            const int c = threadIdx.x % NB, sl = threadIdx.x / NB;
            S acc = s_zero<S>();
            if (c < cnt) {
                S t[kGU];
#pragma unroll
                for (int u = 0; u < kGU; ++u) {
                    const int b = sl + u * kSl;
                    t[u] = b < nb ? ld_ag(&src[b * NB + c]) : s_zero<S>();
                }
#pragma unroll
                for (int u = 0; u < kGU; ++u) acc = add(acc, t[u]);
            }
            red[threadIdx.x] = acc;
        }
        __syncthreads();
        if ((int)threadIdx.x < cnt) {
            S acc = s_zero<S>();
            for (int sl = 0; sl < kSl; ++sl) acc = add(acc, red[sl * NB + threadIdx.x]);
            dst[threadIdx.x] = acc;
        }
        __syncthreads();
    };
    // T column c from the gathered t = V(:, 0:c)^H v_c (stt), as qr_panel_col forms it
    auto t_column = [&](int c, bool skc) {
        if ((int)threadIdx.x <= c) {
            S tc;
            set_re_im(tc, 2.0, 0.0);
            if ((int)threadIdx.x < c) {
                S s2 = s_zero<S>();
                if (!skc)
                    for (int q = threadIdx.x; q < c; ++q) s2 = add(s2, mul(Tl[threadIdx.x + q * NB], stt[q]));
                tc = neg2(s2);
            }
            Tl[threadIdx.x + c * NB] = tc;
        }
        __syncthreads();
    };
    const int m = a.m, k = a.k;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int G = gridDim.x;
    const int R = (m + G - 1) / G;
    const int grp = (G % 8 == 0) ? ((int)blockIdx.x % 8) * (G / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
    const int r0 = grp * R, r1 = min(m, r0 + R);
    const int rown = r0 + lane;
    const bool own = rown < r1;
    unsigned target = 0;
    for (int e = tid; e < NB * NB; e += kCoopThreads) Tl[e] = s_zero<S>();
    if (tid == 0) s_skprev = 0;
    for (int i = 0; i < a.nbp; ++i) {
        const int j = k + i;
        // ---------------- P1
        if (wv == 0 && own) xs[lane] = a.R[rown + (int64_t)j * m];
        __syncthreads();
        for (int c = wv; c < i; c += 16) {
            S p = s_zero<S>();
            if (own && rown >= k) p = add(p, mul(cj(vc[c][lane]), xs[lane]));
            p = wsum(p);
            if (lane == 0) st_ag(&a.part[grp * NB + c], p);
        }
        grid_barrier(a.bar, target, a.err, a.hier);
        // ---------------- P2
        if (i > 0) {
            gather(a.part, i, sp);
            gather(a.part + (size_t)G * NB, i - 1, stt);
            t_column(i - 1, s_skprev != 0);
            if (tid < i) {
                S sacc = s_zero<S>();
                for (int c = 0; c <= tid; ++c) sacc = add(sacc, mul(cj(Tl[c + tid * NB]), sp[c]));
                sw2[tid] = sacc;
            }
            __syncthreads();
        }
        if (wv == 0) {
            double tl = 0.0;
            if (own) {
                S x = xs[lane];
                if (rown >= k)
                    for (int c = 0; c < i; ++c) x = sub(x, mul(vc[c][lane], sw2[c]));
                xs[lane] = x;
                if (rown >= j + 1) tl += sq_abs(x);
                if (rown == j) st_ag(a.x0, x);
            }
            tl = wave_sum(tl);
            if (lane == 0) st_agent(&a.tpart[grp], tl);
        }
        grid_barrier(a.bar, target, a.err, a.hier);
        // ---------------- P3
        {
            const double tpv = tid < G ? ld_agent(&a.tpart[tid]) : 0.0;
            const S x0 = ld_ag(a.x0);
            if (tid < G) tps[tid] = tpv;
            __syncthreads();
            if (tid == 0) {
                double tail = 0.0;
                for (int b = 0; b < G; ++b) tail += tps[b];
                bool skr;
                S v0, alpha;
                double rv;
                hess_reflector(x0, tail, skr, v0, rv, alpha);
                s_sk = skr ? 1 : 0;
                s_scal[1] = v0;
                s_rv = rv;
                s_scal[2] = alpha;
            }
            __syncthreads();
        }
        const bool sk = s_sk != 0;
        const S v0 = s_scal[1], alpha = s_scal[2];
        const double rv = s_rv;
        if (wv == 0 && own) {
            const S x = xs[lane];
            S v = s_zero<S>();
            if (!sk && rown >= j) v = scal(rown == j ? v0 : x, rv);
            st_ag(&a.V[rown + (int64_t)i * m], v);
            vc[i][lane] = v;
            S xr = x;
            if (!sk && rown == j) xr = alpha;
            if (!sk && rown > j) xr = s_zero<S>();
            a.R[rown + (int64_t)j * m] = xr;
        }
        __syncthreads();
        for (int c = wv; c < i; c += 16) {
            S p = s_zero<S>();
            if (!sk && own && rown >= j) p = add(p, mul(cj(vc[c][lane]), vc[i][lane]));
            p = wsum(p);
            if (lane == 0) st_ag(&a.part[(G + grp) * NB + c], p);
        }
        if (tid == 0) s_skprev = s_sk;
    }
    // the last column's T column, then block 0 publishes T
    grid_barrier(a.bar, target, a.err, a.hier);
    const int il = a.nbp - 1;
    if (il >= 0) {
        gather(a.part + (size_t)G * NB, il, stt);
        t_column(il, s_skprev != 0);
    }
    if (blockIdx.x == 0)
        for (int e = tid; e < NB * NB; e += kCoopThreads) a.T[e] = Tl[e];
}

// C (m x nn, ldc) += alpha * op(A) op(B); op = transpose when TA / TB.  64x64 tiles, 4x4/thread.
// Split-K: blockIdx.z takes rows [z kc, (z+1) kc) of the K range and, when gridDim.z > 1, writes its
// partial product to C + z * zstride (beta must be 0 then; gemm_reduce adds the partials in z order).
template <class S, bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_valu(int m, int nn, int kk, double alpha, const S* A, int64_t lda,
                                                 const S* B, int64_t ldb, double beta, S* C, int64_t ldc,
                                                 int kc, int64_t zstride) {
    constexpr int TM = 64, KT = 16;
    __shared__ S As[KT][TM + 1];
    __shared__ S Bs[KT][TM + 1];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int i0 = blockIdx.x * TM, j0 = blockIdx.y * TM;
    const int kb = blockIdx.z * kc;
    const int ke = min(kk, kb + kc);
    C += blockIdx.z * zstride;
    S acc[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int w = 0; w < 4; ++w) acc[u][w] = s_zero<S>();
    for (int k0 = kb; k0 < ke; k0 += KT) {
        for (int e = threadIdx.x; e < KT * TM; e += 256) {
            int r, q;
            // A tile: op(A)(i0 + r, k0 + q)
            if (!TA) { r = e % TM; q = e / TM; } else { q = e % KT; r = e / KT; }
            {
                const int gi = i0 + r, gk = k0 + q;
                S val = s_zero<S>();
                if (gi < m && gk < ke) val = TA ? cj(A[gk + (int64_t)gi * lda]) : A[gi + (int64_t)gk * lda];
                As[q][r] = val;
            }
            // B tile: op(B)(k0 + q, j0 + r)
            if (!TB) { q = e % KT; r = e / KT; } else { r = e % TM; q = e / TM; }
            {
                const int gk = k0 + q, gj = j0 + r;
                S val = s_zero<S>();
                if (gk < ke && gj < nn) val = TB ? cj(B[gj + (int64_t)gk * ldb]) : B[gk + (int64_t)gj * ldb];
                Bs[q][r] = val;
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < KT; ++q) {
            S av[4], bv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) { av[u] = As[q][tx + 16 * u]; bv[u] = Bs[q][ty + 16 * u]; }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int w = 0; w < 4; ++w) acc[u][w] = add(acc[u][w], mul(av[u], bv[w]));
        }
        __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int gi = i0 + tx + 16 * u, gj = j0 + ty + 16 * w;
            if (gi < m && gj < nn) {
                S* cp = C + gi + (int64_t)gj * ldc;
                *cp = add(beta == 0.0 ? s_zero<S>() : scal(*cp, beta), scal(acc[u][w], alpha));
            }
        }
}

// Same contract as gemm_f64, on the fp64 matrix cores: v_mfma_f64_16x16x4_f64.  A 64x64 block
// tile, four waves of 32x32 (2x2 MFMA tiles).  The product is formed transposed (A operand =
// B^T fragment, B operand = A^T fragment) so that the f64 C/D layout (col = lane & 15,
// row = (lane >> 4) + 4 reg, cdna_hip_programming.md) puts C's ROW on the lane: 16 lanes store
// 128 contiguous bytes of one column.
typedef double dbl4 __attribute__((ext_vector_type(4)));

template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_mfma_f64(int m, int nn, int kk, double alpha, const double* A,
                                                     int64_t lda, const double* B, int64_t ldb, double beta,
                                                     double* C, int64_t ldc, int kc, int64_t zstride) {
    constexpr int TM = 64, KT = 16;
    __shared__ double As[KT][TM + 1];   // As[k][row]
    __shared__ double Bs[KT][TM + 1];   // Bs[k][col]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wy = wave >> 1, wx = wave & 1;
    const int i0 = blockIdx.x * TM, j0 = blockIdx.y * TM;
    const int kb = blockIdx.z * kc;
    const int ke = min(kk, kb + kc);
    C += blockIdx.z * zstride;
    dbl4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
    for (int k0 = kb; k0 < ke; k0 += KT) {
        for (int e = threadIdx.x; e < KT * TM; e += 256) {
            int r, q;
            if (!TA) { r = e % TM; q = e / TM; } else { q = e % KT; r = e / KT; }
            {
                const int gi = i0 + r, gk = k0 + q;
                double val = 0.0;
                if (gi < m && gk < ke) val = TA ? A[gk + (int64_t)gi * lda] : A[gi + (int64_t)gk * lda];
                As[q][r] = val;
            }
            if (!TB) { q = e % KT; r = e / KT; } else { r = e % TM; q = e / TM; }
            {
                const int gk = k0 + q, gj = j0 + r;
                double val = 0.0;
                if (gk < ke && gj < nn) val = TB ? B[gj + (int64_t)gk * ldb] : B[gk + (int64_t)gj * ldb];
                Bs[q][r] = val;
            }
        }
        __syncthreads();
#pragma unroll
        for (int kq = 0; kq < KT; kq += 4) {
            const int k = kq + (lane >> 4);
            double bfrag[2], afrag[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                afrag[t] = Bs[k][32 * wx + 16 * t + (lane & 15)];   // B^T fragment (D rows = C columns)
                bfrag[t] = As[k][32 * wy + 16 * t + (lane & 15)];   // A^T fragment (D cols = C rows)
            }
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int tj = 0; tj < 2; ++tj)
                    acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(afrag[tj], bfrag[ti], acc[ti][tj], 0, 0, 0);
        }
        __syncthreads();
    }
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gi = i0 + 32 * wy + 16 * ti + (lane & 15);
                const int gj = j0 + 32 * wx + 16 * tj + (lane >> 4) + 4 * r;
                if (gi < m && gj < nn) {
                    double* cp = C + gi + (int64_t)gj * ldc;
                    *cp = (beta == 0.0 ? 0.0 : beta * *cp) + alpha * acc[ti][tj][r];
                }
            }
}

// Complex counterpart of gemm_mfma_f64: C = beta C + alpha op(A) op(B), op = conjugate transpose
// when TA / TB (alpha, beta real).  The tiles are staged as re / im planes and a complex tile
// product is four real MFMAs: re += Ar Br - Ai Bi, im += Ar Bi + Ai Br.
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_mfma_c128(int m, int nn, int kk, double alpha, const cplx* A,
                                                      int64_t lda, const cplx* B, int64_t ldb, double beta,
                                                      cplx* C, int64_t ldc, int kc, int64_t zstride) {
    constexpr int TM = 64, KT = 16;
    __shared__ double Ar[KT][TM + 1], Ai[KT][TM + 1];   // [k][row]
    __shared__ double Br[KT][TM + 1], Bi[KT][TM + 1];   // [k][col]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wy = wave >> 1, wx = wave & 1;
    const int i0 = blockIdx.x * TM, j0 = blockIdx.y * TM;
    const int kb = blockIdx.z * kc;
    const int ke = min(kk, kb + kc);
    C += blockIdx.z * zstride;
    dbl4 accR[2][2], accI[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) accR[a][b] = accI[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
    for (int k0 = kb; k0 < ke; k0 += KT) {
        for (int e = threadIdx.x; e < KT * TM; e += 256) {
            int r, q;
            if (!TA) { r = e % TM; q = e / TM; } else { q = e % KT; r = e / KT; }
            {
                const int gi = i0 + r, gk = k0 + q;
                cplx val{0.0, 0.0};
                if (gi < m && gk < ke) val = TA ? cj(A[gk + (int64_t)gi * lda]) : A[gi + (int64_t)gk * lda];
                Ar[q][r] = val.re;
                Ai[q][r] = val.im;
            }
            if (!TB) { q = e % KT; r = e / KT; } else { r = e % TM; q = e / TM; }
            {
                const int gk = k0 + q, gj = j0 + r;
                cplx val{0.0, 0.0};
                if (gk < ke && gj < nn) val = TB ? cj(B[gj + (int64_t)gk * ldb]) : B[gk + (int64_t)gj * ldb];
                Br[q][r] = val.re;
                Bi[q][r] = val.im;
            }
        }
        __syncthreads();
#pragma unroll
        for (int kq = 0; kq < KT; kq += 4) {
            const int k = kq + (lane >> 4);
            double bR[2], bI[2], aR[2], aI[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                bR[t] = Br[k][32 * wx + 16 * t + (lane & 15)];
                bI[t] = Bi[k][32 * wx + 16 * t + (lane & 15)];
                aR[t] = Ar[k][32 * wy + 16 * t + (lane & 15)];
                aI[t] = Ai[k][32 * wy + 16 * t + (lane & 15)];
            }
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int tj = 0; tj < 2; ++tj) {
                    accR[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(bR[tj], aR[ti], accR[ti][tj], 0, 0, 0);
                    accR[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(-bI[tj], aI[ti], accR[ti][tj], 0, 0, 0);
                    accI[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(bI[tj], aR[ti], accI[ti][tj], 0, 0, 0);
                    accI[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(bR[tj], aI[ti], accI[ti][tj], 0, 0, 0);
                }
        }
        __syncthreads();
    }
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gi = i0 + 32 * wy + 16 * ti + (lane & 15);
                const int gj = j0 + 32 * wx + 16 * tj + (lane >> 4) + 4 * r;
                if (gi < m && gj < nn) {
                    cplx* cp = C + gi + (int64_t)gj * ldc;
                    const cplx old = beta == 0.0 ? cplx{0.0, 0.0} : cplx{beta * cp->re, beta * cp->im};
                    *cp = cplx{old.re + alpha * accR[ti][tj][r], old.im + alpha * accI[ti][tj][r]};
                }
            }
}

// C = beta C + sum_z P[z] (m x nn, P packed with leading dimension m), partials added in z order
template <class S>
__global__ void gemm_reduce(int m, int nn, int nz, const S* P, double beta, S* C, int64_t ldc) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (int64_t)m * nn) return;
    const int i = (int)(idx % m);
    const int64_t j = idx / m;
    S s = s_zero<S>();
    for (int z = 0; z < nz; ++z) s = add(s, P[(int64_t)z * m * nn + idx]);
    S* c = C + i + j * ldc;
    *c = add(beta == 0.0 ? s_zero<S>() : scal(*c, beta), s);
}

// dst(0:rows, 0:cols) = conj(src(...)), column-major
template <class S>
__global__ void conj_copy2d(S* dst, int64_t ldd, const S* src, int64_t lds, int rows, int cols) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (int64_t)rows * cols) return;
    const int i = (int)(idx % rows);
    const int64_t j = idx / rows;
    dst[i + j * ldd] = cj(src[i + j * lds]);
}

}  // namespace dev

namespace {
template <class S, bool TA, bool TB>
void gemm(hipStream_t st, int m, int nn, int kk, double alpha, const S* A, int64_t lda, const S* B, int64_t ldb,
          double beta, S* C, int64_t ldc, S* work = nullptr, int64_t work_elems = 0) {
    if (m <= 0 || nn <= 0) return;
    const int bx = (m + 63) / 64, by = (nn + 63) / 64;
    // split K when the output has too few tiles to fill the chip (e.g. W = V^H A, nb rows)
    int nz = 1;
    if (work && bx * by < 512 && kk >= 512) {
        nz = std::min(16, std::max(1, 1024 / (bx * by)));
        nz = std::min<int64_t>(nz, work_elems / ((int64_t)m * nn));
        nz = std::max(1, std::min(nz, kk / 128));
    }
    auto launch = [&](dim3 g, double be, S* Cp, int64_t ldcp, int kc, int64_t zs) {
        if constexpr (std::is_same_v<S, double>) {
            static const bool valu = std::getenv("EIGSOL_GEMM_VALU") != nullptr;
            auto kern = valu ? dev::gemm_valu<double, TA, TB> : dev::gemm_mfma_f64<TA, TB>;
            hipLaunchKernelGGL(kern, g, dim3(256), 0, st, m, nn, kk, alpha, A, lda, B, ldb, be, Cp, ldcp, kc, zs);
        } else if constexpr (std::is_same_v<S, cplx>) {
            hipLaunchKernelGGL((dev::gemm_mfma_c128<TA, TB>), g, dim3(256), 0, st, m, nn, kk, alpha, A, lda, B, ldb,
                               be, Cp, ldcp, kc, zs);
        } else {   // single precision: the small panel GEMMs on the VALU
            hipLaunchKernelGGL((dev::gemm_valu<S, TA, TB>), g, dim3(256), 0, st, m, nn, kk, alpha, A, lda, B, ldb,
                               be, Cp, ldcp, kc, zs);
        }
    };
    if (nz <= 1) {
        launch(dim3(bx, by, 1), beta, C, ldc, kk, (int64_t)0);
        return;
    }
    const int kc = ((kk + nz - 1) / nz + 15) / 16 * 16;
    nz = (kk + kc - 1) / kc;
    launch(dim3(bx, by, nz), 0.0, work, (int64_t)m, kc, (int64_t)m * nn);
    const int64_t tot = (int64_t)m * nn;
    hipLaunchKernelGGL((dev::gemm_reduce<S>), dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, m, nn, nz, work,
                       beta, C, ldc);
}

// In place on the device matrix A (n x n, column-major, ld = n).
template <class S>
int hessenberg_blocked(hipStream_t st, S* A, int64_t n64) {
    constexpr bool kC = !is_real_v<S>;
    using Cfg = dev::HessCfg<S>;
    const int n = (int)n64;
    if (n < 3) return EIGSOL_OK;
    if (n > Cfg::kMaxLdsN) return fail(EIGSOL_E_UNSUPPORTED, "blocked Hessenberg: n above the LDS panel limit");
    constexpr int NB = Cfg::NB;
    const int maxch = (n + dev::kGemvCols - 1) / dev::kGemvCols;
    S *V = nullptr, *Y = nullptr, *T = nullptr, *tv = nullptr, *yp = nullptr, *W = nullptr;
    int* skip = nullptr;
    EIGSOL_HIP(hipMalloc(&V, (size_t)n * NB * sizeof(S)));
    S *L = nullptr, *R = nullptr, *M = nullptr;
    EIGSOL_HIP(hipMalloc(&L, (size_t)n * 2 * NB * sizeof(S)));   // [Y | V zero above the panel]
    EIGSOL_HIP(hipMalloc(&R, (size_t)n * 2 * NB * sizeof(S)));   // conj of [V(c1:, :) | W2^H]
    EIGSOL_HIP(hipMalloc(&M, (size_t)NB * NB * sizeof(S)));      // V^H Y
    Y = L;
    EIGSOL_HIP(hipMalloc(&T, NB * NB * sizeof(S)));
    EIGSOL_HIP(hipMalloc(&tv, NB * sizeof(S)));
    EIGSOL_HIP(hipMalloc(&yp, (size_t)maxch * n * sizeof(S)));
    EIGSOL_HIP(hipMalloc(&W, (size_t)NB * n * sizeof(S)));
    S* SK = nullptr;                      // split-K partials of W = V^H A (16 x NB x n)
    const int64_t sk_elems = (int64_t)16 * NB * n;
    EIGSOL_HIP(hipMalloc(&SK, sk_elems * sizeof(S)));
    EIGSOL_HIP(hipMalloc(&skip, 64));
    const size_t lds = (size_t)n * sizeof(S);
    // one cooperative launch per panel when the device supports it and n fits its LDS staging
    int coop_ok = 0, dev_id = 0;
    EIGSOL_HIP(hipGetDevice(&dev_id));
    EIGSOL_HIP(hipDeviceGetAttribute(&coop_ok, hipDeviceAttributeCooperativeLaunch, dev_id));
    // panel grid: about 32 rows per block, 16 .. 256 blocks (EIGSOL_HESS_G overrides: 8 .. 256, a multiple of
    // 8).  The panel's GEMV streams the trailing matrix once per column from the grid's CUs, its two grid
    // barriers per column grow with the grid; round 6 (tools/r06_hess_grid_ab.sh, profiles/r06_hess_grid_ab.log,
    // host in/out): 512^2 16 blocks 0.011 s (64: 0.014), 1024^2 32 0.024 (64: 0.026), 4096^2 128 0.167 (64:
    // 0.184, 256: 0.193), 8192^2 256 0.73 (64: 1.11)
    static const int g_env = [] {
        const char* e = std::getenv("EIGSOL_HESS_G");
        const int g = e ? std::atoi(e) : 0;
        return (g >= 8 && g <= 256 && g % 8 == 0) ? g : 0;
    }();
    const int G = g_env ? g_env : std::min(256, std::max(16, (n / 32 + 7) / 8 * 8));
    // two-level grid barrier from 64 blocks (EIGSOL_HESS_BAR=0: one counter).  Round 6
    // (tools/r06_hess_bar_ab.sh, profiles/r06_hess_bar_ab.log, host in/out): 4096^2 0.169 / 0.172 -> 0.161 /
    // 0.162 s, 8192^2 0.730 -> 0.689 s; at 32 blocks (1024^2) one counter stays (0.0240 against 0.0248 s)
    static const bool hier = [] {
        const char* e = std::getenv("EIGSOL_HESS_BAR");
        return !(e && std::atoi(e) == 0);
    }();
    constexpr size_t kBarBytes = 9 * 64;
    // past Cfg::kCoopMaxN (v no longer fits the panel's LDS) the merged panel reads v from the published
    // column (hess_panel_coop2<S, true>), up to 64 rows per block (n <= 16384); EIGSOL_HESS_VG=0 keeps such
    // orders on the per-column kernels
    // (EIGSOL_HESS_VG=2 also below the limit: the bitwise test of the global-v form)
    const char* vge = std::getenv("EIGSOL_HESS_VG");
    const bool vg = (n > Cfg::kCoopMaxN || (vge && std::atoi(vge) == 2)) && n <= 64 * G && !(vge && std::atoi(vge) == 0);
    bool coop = coop_ok && (n <= Cfg::kCoopMaxN || vg) && n <= 128 * G && std::getenv("EIGSOL_HESS_NO_COOP") == nullptr;
    const size_t coop_lds = vg ? 0 : (size_t)n * sizeof(S);
    // two grid barriers per panel column (hess_panel_coop kMerge; EIGSOL_HESS_MERGE=0: three).  Round 6
    // (tools/r06_hess_merge_ab.sh, profiles/r06_hess_merge_ab.log): to_hessenberg 4096^2 0.184 / 0.185 ->
    // 0.182 / 0.176 s; QR 4096^2 unchanged within noise (0.885 / 0.885 against 0.888 / 0.882 s), complex
    // 1.551 -> 1.545 s; eigenvalues one-to-one with the LAPACK fixtures
    static const bool merge = [] {
        const char* e = std::getenv("EIGSOL_HESS_MERGE");
        return !(e && std::atoi(e) == 0);
    }();
    // EIGSOL_HESS_PANEL2=0: the merged panel without the LDS caches and the batched loads
    const bool panel2 = [] {   // read per call (the bitwise test switches it)
        const char* e = std::getenv("EIGSOL_HESS_PANEL2");
        return !(e && std::atoi(e) == 0);
    }();
    if (vg && !(merge && panel2)) coop = false;   // only the merged LDS-cached panel has the global-v form
    const void* coop_kernel =
        n <= 64 * G
            ? (merge ? (panel2 ? (vg ? reinterpret_cast<const void*>(dev::hess_panel_coop2<S, true>)
                                     : reinterpret_cast<const void*>(dev::hess_panel_coop2<S>))
                               : reinterpret_cast<const void*>(dev::hess_panel_coop<S, 1, true>))
                     : reinterpret_cast<const void*>(dev::hess_panel_coop<S, 1>))
            : (merge ? reinterpret_cast<const void*>(dev::hess_panel_coop<S, 2, true>)
                     : reinterpret_cast<const void*>(dev::hess_panel_coop<S, 2>));
    S *part = nullptr, *x0s = nullptr, *xu = nullptr;
    double* tpart = nullptr;
    unsigned* bar = nullptr;
    int* err = nullptr;
    if (coop) {
        EIGSOL_HIP(hipMalloc(&part, 2 * G * NB * sizeof(S)));
        EIGSOL_HIP(hipMalloc(&tpart, G * sizeof(double)));
        EIGSOL_HIP(hipMalloc(&x0s, 64));
        EIGSOL_HIP(hipMalloc(&xu, (size_t)n * sizeof(S)));
        EIGSOL_HIP(hipMalloc(&bar, kBarBytes));
        EIGSOL_HIP(hipMalloc(&err, 64));
        EIGSOL_HIP(hipMemsetAsync(err, 0, 64, st));
        EIGSOL_HIP(hipFuncSetAttribute(coop_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)coop_lds));
    }
    EIGSOL_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(dev::hess_panel_col<S>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int last = n - 3;   // reflector columns 0 .. n-3 (to_hessenberg.hpp:38)
    for (int k = 0; k <= last; k += NB) {
        const int nbp = std::min(NB, last - k + 1);
        EIGSOL_HIP(hipMemsetAsync(T, 0, NB * NB * sizeof(S), st));
        if (coop) {
            EIGSOL_HIP(hipMemsetAsync(bar, 0, kBarBytes, st));
            dev::CoopArgs<S> ca{A, n, k, nbp, V, Y, T, part, tpart, x0s, bar, err, xu, hier && G % 8 == 0 && G >= 64};
            void* kargs[] = {&ca};
            // EIGSOL_HESS_COOP_PLAIN=1: the SAME panel kernel through an ordinary launch, for profiling
            // only (rocprofv3 7.2 crashes at exit after any cooperative launch, tools/coop_prof_repro.hip);
            // its G blocks are at most the CUs, so on an idle device all are resident,
            // and the grid barrier's bounded spin reports a failure instead of hanging otherwise
            static const bool plain = std::getenv("EIGSOL_HESS_COOP_PLAIN") != nullptr;
            if (plain)
                EIGSOL_HIP(hipLaunchKernel(coop_kernel, dim3(G), dim3(dev::kCoopThreads), kargs, coop_lds, st));
            else
                EIGSOL_HIP(hipLaunchCooperativeKernel(coop_kernel, dim3(G), dim3(dev::kCoopThreads), kargs,
                                                      coop_lds, st));
        }
        for (int i = 0; !coop && i < nbp; ++i) {
            const int j = k + i;
            hipLaunchKernelGGL(dev::hess_panel_col<S>, dim3(1), dim3(1024), lds, st, A, n, k, j, i, V, Y, T, tv, skip);
            const int c0 = j + 1;
            const int nch = (n - c0 + dev::kGemvCols - 1) / dev::kGemvCols;
            hipLaunchKernelGGL(dev::hess_gemv<S>, dim3((n + 255) / 256, nch), dim3(256), 0, st, A, n, c0,
                               V + (int64_t)i * n, yp, skip);
            hipLaunchKernelGGL(dev::hess_y<S>, dim3((n + 255) / 256), dim3(256), 0, st, n, i, nch, yp, tv, Y, T, skip);
        }
        const int c1 = k + nbp;           // first trailing column
        const int mt = n - c1;
        if (mt > 0) {
            // A <- Q^H A Q with Q = I - V T V^H, in one pass over the trailing columns:
            //   right: A Q = A - Y V^H (Y = A V T from the panel);
            //   left:  Q^H (A Q) = A Q - V W2, W2 = T^H V^H (A Q) = T^H (V^H A - (V^H Y) V^H);
            // so A(:, c1:) -= [Y | V] [V(c1:, :) | W2^H]^H, one rank-2nbp update (V is zero above
            // row k+1), with W0 = V^H A read from A before it.  The update kernel forms L Rc^T, so
            // R holds the conjugate of [V(c1:, :) | W2^H] = [conj V(c1:, :) | W2^T].
            const int rows = n - (k + 1);
            S* Vz = L + (int64_t)nbp * n;     // L = [Y | Vz], Y already in place
            S* R2 = R + (int64_t)nbp * n;
            gemm<S, true, false>(st, nbp, mt, rows, 1.0, V + (k + 1), n, A + (k + 1) + (int64_t)c1 * n, n, 0.0, W, NB,
                                 SK, sk_elems);
            gemm<S, true, false>(st, nbp, nbp, rows, 1.0, V + (k + 1), n, L + (k + 1), n, 0.0, M, NB, SK, sk_elems);
            if constexpr (kC) {
                gemm<S, false, true>(st, nbp, mt, nbp, -1.0, M, NB, V + c1, n, 1.0, W, NB);          // W = V^H (A Q)
                const int64_t cnt = (int64_t)mt * nbp;
                hipLaunchKernelGGL(dev::conj_copy2d<S>, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, R,
                                   (int64_t)n, V + c1, (int64_t)n, mt, nbp);                          // conj V(c1:, :)
                gemm<S, true, false>(st, mt, nbp, nbp, 1.0, W, NB, T, NB, 0.0, R2, n);               // W^H T
                hipLaunchKernelGGL(dev::conj_copy2d<S>, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, R2,
                                   (int64_t)n, R2, (int64_t)n, mt, nbp);                              // W2^T
            } else {
                EIGSOL_HIP(hipMemcpy2DAsync(R, n * sizeof(S), V + c1, n * sizeof(S), mt * sizeof(S), nbp,
                                            hipMemcpyDeviceToDevice, st));
                gemm<S, false, true>(st, nbp, mt, nbp, -1.0, M, NB, R, n, 1.0, W, NB);              // W = V^T (A Q)
                gemm<S, true, false>(st, mt, nbp, nbp, 1.0, W, NB, T, NB, 0.0, R2, n);              // W2^T = W^T T
            }
            EIGSOL_HIP(hipMemsetAsync(Vz, 0, (size_t)nbp * n * sizeof(S), st));
            EIGSOL_HIP(hipMemcpy2DAsync(Vz + (k + 1), n * sizeof(S), V + (k + 1), n * sizeof(S), rows * sizeof(S), nbp,
                                        hipMemcpyDeviceToDevice, st));
            rankk_update<S, false>(st, n, mt, 2 * nbp, -1.0, L, n, R, n, A + (int64_t)c1 * n, n);
        }
    }
    EIGSOL_HIP(hipGetLastError());
    int errh = 0;
    if (coop) {
        EIGSOL_HIP(hipMemcpyAsync(&errh, err, sizeof(int), hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(hipStreamSynchronize(st));
    }
    for (void* p : {(void*)V, (void*)L, (void*)R, (void*)M, (void*)T, (void*)tv, (void*)yp, (void*)W, (void*)skip,
                    (void*)part, (void*)tpart, (void*)x0s, (void*)xu, (void*)bar, (void*)err, (void*)SK})
        if (p) (void)hipFree(p);
    if (errh) return fail(EIGSOL_E_HIP, "blocked Hessenberg: grid barrier timed out (internal error)");
    return EIGSOL_OK;
}

// qr_decompose_dense (qr_decompose.hpp:46-85) blocked: R (m x n, in place) and Q (m x m, set here).
// Panels of 32 reflectors; m up to the LDS column limit (else the caller uses the per-reflector
// kernels).
template <class S>
int qr_blocked(hipStream_t st, S* R, int m, int n, S* Q) {
    constexpr bool kC = !is_real_v<S>;
    constexpr int NB = 32;
    if (m > dev::HessCfg<S>::kMaxLdsN) return fail(EIGSOL_E_UNSUPPORTED, "blocked QR: m above the LDS panel limit");
    const int kmax = std::min(m, n);
    S *V = nullptr, *Vc = nullptr, *T = nullptr, *W = nullptr, *W2 = nullptr, *Z = nullptr, *Z2 = nullptr, *SK = nullptr;
    const int64_t sk_elems = (int64_t)16 * NB * std::max(m, n);
    EIGSOL_HIP(hipMalloc(&V, (size_t)m * NB * sizeof(S)));
    if (kC) EIGSOL_HIP(hipMalloc(&Vc, (size_t)m * NB * sizeof(S)));
    EIGSOL_HIP(hipMalloc(&T, NB * NB * sizeof(S)));
    EIGSOL_HIP(hipMalloc(&W, (size_t)NB * std::max(n, 1) * sizeof(S)));
    EIGSOL_HIP(hipMalloc(&W2, (size_t)NB * std::max(n, 1) * sizeof(S)));
    EIGSOL_HIP(hipMalloc(&Z, (size_t)m * NB * sizeof(S)));
    EIGSOL_HIP(hipMalloc(&Z2, (size_t)m * NB * sizeof(S)));
    EIGSOL_HIP(hipMalloc(&SK, sk_elems * sizeof(S)));
    EIGSOL_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(dev::qr_panel_col<S>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)(m * sizeof(S))));
    // the panel as one cooperative launch (qr_panel_coop) from m >= 256 when the device supports it
    // (EIGSOL_QR_COOP=0: one qr_panel_col launch per column); its grid: about 32 rows per block, 16 .. 256
    // blocks, like the Hessenberg panel's
    int coop_ok = 0, dev_id = 0;
    EIGSOL_HIP(hipGetDevice(&dev_id));
    EIGSOL_HIP(hipDeviceGetAttribute(&coop_ok, hipDeviceAttributeCooperativeLaunch, dev_id));
    const char* qce = std::getenv("EIGSOL_QR_COOP");
    const int G = std::min(256, std::max(16, (m / 32 + 7) / 8 * 8));
    const bool coop = coop_ok && m >= 256 && m <= 64 * G && !(qce && std::atoi(qce) == 0);
    S *part = nullptr, *x0s = nullptr;
    double* tpart = nullptr;
    unsigned* bar = nullptr;
    int* err = nullptr;
    constexpr size_t kBarBytes = 9 * 64;
    if (coop) {
        EIGSOL_HIP(hipMalloc(&part, 2 * (size_t)G * NB * sizeof(S)));
        EIGSOL_HIP(hipMalloc(&tpart, G * sizeof(double)));
        EIGSOL_HIP(hipMalloc(&x0s, 64));
        EIGSOL_HIP(hipMalloc(&bar, kBarBytes));
        EIGSOL_HIP(hipMalloc(&err, 64));
        EIGSOL_HIP(hipMemsetAsync(err, 0, 64, st));
    }
    for (int k = 0; k < kmax; k += NB) {
        const int nbp = std::min(NB, kmax - k);
        EIGSOL_HIP(hipMemsetAsync(T, 0, NB * NB * sizeof(S), st));
        if (coop) {
            EIGSOL_HIP(hipMemsetAsync(bar, 0, kBarBytes, st));
            dev::QrCoopArgs<S> ca{R, m, k, nbp, V, T, part, tpart, x0s, bar, err, G >= 64};
            void* kargs[] = {&ca};
            static const bool plain = std::getenv("EIGSOL_HESS_COOP_PLAIN") != nullptr;   // profiling only
            if (plain)
                EIGSOL_HIP(hipLaunchKernel(reinterpret_cast<const void*>(dev::qr_panel_coop<S>), dim3(G),
                                           dim3(dev::kCoopThreads), kargs, 0, st));
            else
                EIGSOL_HIP(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(dev::qr_panel_coop<S>), dim3(G),
                                                      dim3(dev::kCoopThreads), kargs, 0, st));
        }
        for (int i = 0; !coop && i < nbp; ++i)
            hipLaunchKernelGGL(dev::qr_panel_col<S>, dim3(1), dim3(1024), m * sizeof(S), st, R, m, k, k + i, i, V, T);
        const int rows = m - k, c1 = k + nbp, mt = n - c1;
        if (mt > 0) {   // R(k:, c1:) <- (I - V T^H V^H) R(k:, c1:)
            gemm<S, true, false>(st, nbp, mt, rows, 1.0, V + k, m, R + k + (int64_t)c1 * m, m, 0.0, W, NB, SK, sk_elems);
            gemm<S, true, false>(st, nbp, mt, nbp, 1.0, T, NB, W, NB, 0.0, W2, NB);
            rankk_update<S, true>(st, rows, mt, nbp, -1.0, V + k, m, W2, NB, R + k + (int64_t)c1 * m, m);
        }
        // Q(:, k:) <- Q(:, k:) (I - V T V^H)
        gemm<S, false, false>(st, m, nbp, rows, 1.0, Q + (int64_t)k * m, m, V + k, m, 0.0, Z, m, SK, sk_elems);
        gemm<S, false, false>(st, m, nbp, nbp, 1.0, Z, m, T, NB, 0.0, Z2, m);
        const S* Vr = V;
        if constexpr (kC) {
            const int64_t cnt = (int64_t)m * nbp;
            hipLaunchKernelGGL(dev::conj_copy2d<S>, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, Vc, (int64_t)m, V,
                               (int64_t)m, m, nbp);
            Vr = Vc;
        }
        rankk_update<S, false>(st, m, rows, nbp, -1.0, Z2, m, Vr + k, m, Q + (int64_t)k * m, m);
    }
    EIGSOL_HIP(hipGetLastError());
    int errh = 0;
    if (coop) {
        EIGSOL_HIP(hipMemcpyAsync(&errh, err, sizeof(int), hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(hipStreamSynchronize(st));
    }
    for (void* p : {(void*)V, (void*)Vc, (void*)T, (void*)W, (void*)W2, (void*)Z, (void*)Z2, (void*)SK, (void*)part,
                    (void*)tpart, (void*)x0s, (void*)bar, (void*)err})
        if (p) (void)hipFree(p);
    if (errh) return fail(EIGSOL_E_HIP, "blocked QR: grid barrier timed out (internal error)");
    return EIGSOL_OK;
}
}  // namespace

int hessenberg_blocked_f64(hipStream_t st, double* A, int64_t n) { return hessenberg_blocked<double>(st, A, n); }
int hessenberg_blocked_c128(hipStream_t st, cplx* A, int64_t n) { return hessenberg_blocked<cplx>(st, A, n); }
int qr_blocked_f64(hipStream_t st, double* R, int64_t m, int64_t n, double* Q) { return qr_blocked<double>(st, R, (int)m, (int)n, Q); }
int qr_blocked_c128(hipStream_t st, cplx* R, int64_t m, int64_t n, cplx* Q) { return qr_blocked<cplx>(st, R, (int)m, (int)n, Q); }
int hessenberg_blocked_f32(hipStream_t st, float* A, int64_t n) { return hessenberg_blocked<float>(st, A, n); }
int hessenberg_blocked_c64(hipStream_t st, cplxf* A, int64_t n) { return hessenberg_blocked<cplxf>(st, A, n); }
int qr_blocked_f32(hipStream_t st, float* R, int64_t m, int64_t n, float* Q) { return qr_blocked<float>(st, R, (int)m, (int)n, Q); }
int qr_blocked_c64(hipStream_t st, cplxf* R, int64_t m, int64_t n, cplxf* Q) { return qr_blocked<cplxf>(st, R, (int)m, (int)n, Q); }

}  // namespace eigsol

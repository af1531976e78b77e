// Blocked Householder Hessenberg reduction (real, gfx950), the reference's reflector convention.
//
// to_hessenberg_dense<S> (src/qr_method/to_hessenberg.hpp:38-77) applies H_j = I - 2 v_j v_j^T
// from both sides for every column j.  Here the reflectors of a panel of nb columns are
// accumulated in compact-WY form Q = H_k ... H_{k+nb-1} = I - V T V^T (T upper triangular,
// T(i,i) = 2) together with Y = A V T, and the trailing matrix is updated once per panel:
//     A <- Q^T (A Q) = (I - V T^T V^T)(A - Y V^T)
// (the dlahr2/dgehrd organisation).  Per panel column the only full-matrix pass is the GEMV
// y = A(:, j+1:n) v_j (BLAS-2, half the flops); everything else is three GEMMs per panel.
// Reflectors are generated exactly as the reference does (alpha = -sign(x0) ||x||, skipped when
// ||x(1:)|| == 0), so H matches the unblocked reduction to rounding.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "kernels_common.hpp"
#include "mfma_rankk.hpp"

namespace eigsol {
namespace dev {

constexpr int kPanel = 32;          // reflectors per panel
constexpr int kGemvCols = 128;      // columns per GEMV partial
constexpr int kMaxLdsN = 16384;     // panel column kept in LDS (128 KiB)

// block (1024 threads) sum of kPanel partials per thread -> sw[0..cnt)
__device__ __forceinline__ void block_sum_vec(double (&p)[kPanel], int cnt, double* red /*16*kPanel*/,
                                              double* sw) {
    const int w = threadIdx.x >> 6, ln = threadIdx.x & 63;
#pragma unroll
    for (int c = 0; c < kPanel; ++c) {
        if (c < cnt) {                      // static register index (no scratch)
            const double s = wave_sum(p[c]);
            if (ln == 0) red[w * kPanel + c] = s;
        }
    }
    __syncthreads();
    if ((int)threadIdx.x < cnt) {
        double s = 0.0;
        for (int q = 0; q < (int)(blockDim.x >> 6); ++q) s += red[q * kPanel + threadIdx.x];
        sw[threadIdx.x] = s;
    }
    __syncthreads();
}

// Panel column j (local index i): apply the panel's earlier reflectors from the right (via Y) and
// the left (via V, T), generate reflector i from rows j+1.., store the reduced column, and
// t = V(:, 0:i)^T v_i for the T / Y recursions.
__global__ __launch_bounds__(1024) void hess_panel_col(double* A, int n, int k, int j, int i, double* V,
                                                       const double* Y, const double* T, double* tvec,
                                                       int* skip) {
    extern __shared__ double a[];          // column j (n doubles)
    __shared__ double red[16 * kPanel];
    __shared__ double sw[kPanel];
    __shared__ double sw2[kPanel];
    __shared__ double vj[kPanel];
    __shared__ double s_tail;
    const int tid = threadIdx.x, nt = blockDim.x;
    if (tid < i) vj[tid] = V[j + (int64_t)tid * n];   // row j of V
    __syncthreads();
    // right: a -= Y(:, 0:i) V(j, 0:i)^T
    for (int r = tid; r < n; r += nt) {
        double x = A[r + (int64_t)j * n];
        for (int c = 0; c < i; ++c) x -= Y[r + (int64_t)c * n] * vj[c];
        a[r] = x;
    }
    __syncthreads();
    // left: w = V^T a (rows k+1..), w = T^T w, a -= V w
    if (i > 0) {
        double p[kPanel];
#pragma unroll
        for (int c = 0; c < kPanel; ++c) p[c] = 0.0;
        for (int r = k + 1 + tid; r < n; r += nt) {
            const double x = a[r];
#pragma unroll
            for (int c = 0; c < kPanel; ++c)
                if (c < i) p[c] += V[r + (int64_t)c * n] * x;
        }
        block_sum_vec(p, i, red, sw);
        if (tid < i) {
            double s = 0.0;
            for (int c = 0; c <= tid; ++c) s += T[c + tid * kPanel] * sw[c];   // (T^T w)_tid
            sw2[tid] = s;
        }
        __syncthreads();
        for (int r = k + 1 + tid; r < n; r += nt) {
            double x = a[r];
            for (int c = 0; c < i; ++c) x -= V[r + (int64_t)c * n] * sw2[c];
            a[r] = x;
        }
        __syncthreads();
    }
    // reflector from a(j+1 : n)
    double tl = 0.0;
    for (int r = j + 2 + tid; r < n; r += nt) tl += a[r] * a[r];
    {
        double pp[kPanel];
        pp[0] = tl;
        block_sum_vec(pp, 1, red, sw);
        if (tid == 0) s_tail = sw[0];
        __syncthreads();
    }
    const double tail = s_tail;
    const double x0 = a[j + 1];
    bool sk = tail == 0.0;
    double v0 = 0.0, rv = 0.0, alpha = 0.0;
    if (!sk) {
        const double nx = sqrt(tail + x0 * x0);
        const double sign = x0 == 0.0 ? 1.0 : (x0 > 0.0 ? 1.0 : -1.0);
        alpha = -sign * nx;
        v0 = x0 - alpha;
        const double vn = sqrt(tail + v0 * v0);
        if (vn == 0.0) sk = true;
        else rv = 1.0 / vn;
    }
    double* vcol = V + (int64_t)i * n;
    for (int r = tid; r < n; r += nt) {
        double v = 0.0;
        if (!sk && r > j) v = (r == j + 1 ? v0 : a[r]) * rv;
        vcol[r] = v;
    }
    // store the reduced column (alpha on the subdiagonal, zeros below)
    for (int r = tid; r < n; r += nt) {
        double x = a[r];
        if (!sk && r == j + 1) x = alpha;
        if (!sk && r > j + 1) x = 0.0;
        A[r + (int64_t)j * n] = x;
    }
    if (tid == 0) *skip = sk ? 1 : 0;
    __syncthreads();
    // t = V(:, 0:i)^T v (rows j+1..)
    if (i > 0) {
        double p[kPanel];
#pragma unroll
        for (int c = 0; c < kPanel; ++c) p[c] = 0.0;
        if (!sk)
            for (int r = j + 1 + tid; r < n; r += nt) {
                const double v = vcol[r];
#pragma unroll
                for (int c = 0; c < kPanel; ++c)
                    if (c < i) p[c] += V[r + (int64_t)c * n] * v;
            }
        block_sum_vec(p, i, red, sw);
        if (tid < i) tvec[tid] = sw[tid];
    }
}

// y partials: ypart[ch * n + r] = sum_{c in chunk ch} A(r, c) v(c), columns j+1..n-1
__global__ __launch_bounds__(256) void hess_gemv(const double* A, int n, int c0, const double* v,
                                                 double* ypart, const int* skip) {
    if (*skip) return;
    const int r = blockIdx.x * 256 + threadIdx.x;
    const int ch = blockIdx.y;
    const int cb = c0 + ch * kGemvCols;
    const int ce = min(n, cb + kGemvCols);
    if (r >= n) return;
    double s = 0.0;
    for (int c = cb; c < ce; ++c) s += A[r + (int64_t)c * n] * v[c];
    ypart[(int64_t)ch * n + r] = s;
}

// Y(:, i) = 2 (y - Y(:, 0:i) t);  T(0:i, i) = -2 T(0:i, 0:i) t, T(i, i) = 2
__global__ __launch_bounds__(256) void hess_y(int n, int i, int nch, const double* ypart, const double* tvec,
                                              double* Y, double* T, const int* skip) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    const bool sk = *skip != 0;
    if (r < n) {
        double y = 0.0;
        if (!sk) {
            for (int ch = 0; ch < nch; ++ch) y += ypart[(int64_t)ch * n + r];
            for (int c = 0; c < i; ++c) y -= Y[r + (int64_t)c * n] * tvec[c];
        }
        Y[r + (int64_t)i * n] = sk ? 0.0 : 2.0 * y;
    }
    if (blockIdx.x == 0 && (int)threadIdx.x <= i) {
        const int c = threadIdx.x;
        double tc = 2.0;
        if (c < i) {
            double s = 0.0;
            if (!sk)
                for (int q = c; q < i; ++q) s += T[c + q * kPanel] * tvec[q];
            tc = -2.0 * s;
        }
        T[c + i * kPanel] = tc;
    }
}

// ------------------------------------------------------------------ cooperative panel (one launch)
// The whole panel (32 columns) in ONE cooperative launch of kCoopBlocks co-resident blocks; block
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
#ifndef EIGSOL_COOP_BLOCKS
#define EIGSOL_COOP_BLOCKS 64
#endif
constexpr int kCoopBlocks = EIGSOL_COOP_BLOCKS;
constexpr int kCoopThreads = 1024;
constexpr int kCoopMaxN = 8192;          // v in LDS (64 KiB) and at most 2 rows per lane
#ifndef EIGSOL_GEMV_BATCH
#define EIGSOL_GEMV_BATCH 16
#endif
#ifndef EIGSOL_HESS_SKIP_GEMV
#define EIGSOL_HESS_SKIP_GEMV 0   // timing experiments only
#endif
constexpr int kGemvBatch = EIGSOL_GEMV_BATCH;   // columns per GEMV step (loads in flight per lane)

struct CoopArgs {
    double* A;
    int n, k, nbp;
    double* V;
    double* Y;
    double* T;
    double* part;       // [2][G][kPanel]: P1 -> P2 partials in the first half, P3 -> P4 in the second
    double* tpart;      // [G]
    double* x0;         // a(j+1)
    unsigned* bar;      // barrier counter (zeroed by the host before the launch)
    int* err;
};

__device__ __forceinline__ unsigned ld_agent_u32(const unsigned* p) {
    return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void grid_barrier(unsigned* bar, unsigned& target, int* err) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's sc1 stores are complete
    __syncthreads();
    target += gridDim.x;
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int spins = 0;
        while (ld_agent_u32(bar) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1 << 24)) { atomicOr(err, 1); break; }
        }
    }
    __syncthreads();
}

template <int kCoopRowsPerLane>
__global__ __launch_bounds__(kCoopThreads) void hess_panel_coop(CoopArgs a) {
    extern __shared__ double vsh[];          // v (n doubles) for the GEMV
    __shared__ double xs[kCoopRowsPerLane * 64];    // own rows of the current column
    __shared__ double ysum[16][kCoopRowsPerLane * 64];
    __shared__ double red[kCoopBlocks * kPanel];   // gathered block partials
    __shared__ double sv[kPanel], sw[kPanel], st[kPanel];
    __shared__ double s_scal[4];
    // Block partials of another phase: all threads load them at once (independent sc1 loads),
    // then thread c sums column c in block order (deterministic).
    auto gather = [&](const double* src, int cnt, double* dst) {
        const int nb = (int)gridDim.x;
        for (int e = threadIdx.x; e < nb * kPanel; e += kCoopThreads) {
            const int b = e / kPanel, c = e % kPanel;
            red[e] = c < cnt ? ld_agent(&src[b * kPanel + c]) : 0.0;
        }
        __syncthreads();
        if ((int)threadIdx.x < cnt) {
            double acc = 0.0;
            for (int b = 0; b < nb; ++b) acc += red[b * kPanel + threadIdx.x];
            dst[threadIdx.x] = acc;
        }
        __syncthreads();
    };
    const int n = a.n, k = a.k;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int G = gridDim.x;
    const int R = (n + G - 1) / G;
    const int r0 = blockIdx.x * R, r1 = min(n, r0 + R);
    unsigned target = 0;
    for (int i = 0; i < a.nbp; ++i) {
        const int j = k + i;
        // ---------------- P1
        if (tid < i) sv[tid] = ld_agent(&a.V[j + (int64_t)tid * n]);
        __syncthreads();
        if (wv == 0)
            for (int q = 0; q < kCoopRowsPerLane; ++q) {
                const int r = r0 + lane + 64 * q;
                if (r < r1) {
                    double x = a.A[r + (int64_t)j * n];
                    for (int c = 0; c < i; ++c) x -= a.Y[r + (int64_t)c * n] * sv[c];
                    xs[lane + 64 * q] = x;
                }
            }
        __syncthreads();
        // partials of w_c = sum_{r >= k+1} V(r, c) x(r): wave wv handles c = wv, wv + 16
        for (int c = wv; c < i; c += 16) {
            double p = 0.0;
            for (int q = 0; q < kCoopRowsPerLane; ++q) {
                const int r = r0 + lane + 64 * q;
                if (r < r1 && r >= k + 1) p += a.V[r + (int64_t)c * n] * xs[lane + 64 * q];
            }
            p = wave_sum(p);
            if (lane == 0) st_agent(&a.part[blockIdx.x * kPanel + c], p);
        }
        grid_barrier(a.bar, target, a.err);
        // ---------------- P2
        gather(a.part, i, sw);
        if (tid < i) {
            double s = 0.0;
            for (int c = 0; c <= tid; ++c) s += ld_agent(&a.T[c + tid * kPanel]) * sw[c];   // (T^T w)_tid
            st[tid] = s;
        }
        __syncthreads();
        double tl = 0.0;
        if (wv == 0)
            for (int q = 0; q < kCoopRowsPerLane; ++q) {
                const int r = r0 + lane + 64 * q;
                if (r < r1) {
                    double x = xs[lane + 64 * q];
                    if (r >= k + 1)
                        for (int c = 0; c < i; ++c) x -= a.V[r + (int64_t)c * n] * st[c];
                    xs[lane + 64 * q] = x;
                    if (r >= j + 2) tl += x * x;
                    if (r == j + 1) st_agent(a.x0, x);
                }
            }
        if (wv == 0) {
            tl = wave_sum(tl);
            if (lane == 0) st_agent(&a.tpart[blockIdx.x], tl);
        }
        grid_barrier(a.bar, target, a.err);
        // ---------------- P3
        if (tid < G) red[tid] = ld_agent(&a.tpart[tid]);
        __syncthreads();
        if (tid == 0) {
            double tail = 0.0;
            for (int b = 0; b < G; ++b) tail += red[b];
            const double x0 = ld_agent(a.x0);
            double sk = tail == 0.0 ? 1.0 : 0.0, v0 = 0.0, rv = 0.0, alpha = 0.0;
            if (sk == 0.0) {
                const double nx = sqrt(tail + x0 * x0);
                const double sign = x0 == 0.0 ? 1.0 : (x0 > 0.0 ? 1.0 : -1.0);
                alpha = -sign * nx;
                v0 = x0 - alpha;
                const double vn = sqrt(tail + v0 * v0);
                if (vn == 0.0) sk = 1.0;
                else rv = 1.0 / vn;
            }
            s_scal[0] = sk; s_scal[1] = v0; s_scal[2] = rv; s_scal[3] = alpha;
        }
        __syncthreads();
        const bool sk = s_scal[0] != 0.0;
        const double v0 = s_scal[1], rv = s_scal[2], alpha = s_scal[3];
        if (wv == 0)
            for (int q = 0; q < kCoopRowsPerLane; ++q) {
                const int r = r0 + lane + 64 * q;
                if (r < r1) {
                    const double x = xs[lane + 64 * q];
                    double v = 0.0;
                    if (!sk && r > j) v = (r == j + 1 ? v0 : x) * rv;
                    st_agent(&a.V[r + (int64_t)i * n], v);
                    xs[lane + 64 * q] = v;           // keep v for the t partials
                    double red_col = x;
                    if (!sk && r == j + 1) red_col = alpha;
                    if (!sk && r > j + 1) red_col = 0.0;
                    a.A[r + (int64_t)j * n] = red_col;
                }
            }
        __syncthreads();
        for (int c = wv; c < i; c += 16) {
            double p = 0.0;
            for (int q = 0; q < kCoopRowsPerLane; ++q) {
                const int r = r0 + lane + 64 * q;
                if (r < r1) p += a.V[r + (int64_t)c * n] * xs[lane + 64 * q];
            }
            p = wave_sum(p);
            if (lane == 0) st_agent(&a.part[(G + blockIdx.x) * kPanel + c], p);
        }
        grid_barrier(a.bar, target, a.err);
        // ---------------- P4
        for (int r = tid; r < n; r += kCoopThreads) vsh[r] = sk ? 0.0 : ld_agent(&a.V[r + (int64_t)i * n]);
        __syncthreads();
        gather(a.part + (size_t)G * kPanel, i, sv);
        if (sk && tid < i) sv[tid] = 0.0;
        __syncthreads();
        double yacc[kCoopRowsPerLane];
#pragma unroll
        for (int q = 0; q < kCoopRowsPerLane; ++q) yacc[q] = 0.0;
        if (!sk && !EIGSOL_HESS_SKIP_GEMV) {
            // 8 columns per step with every load issued before the FMAs (bytes in flight: the
            // GEMV streams the trailing matrix once per column)
            const int nq = (r1 - r0 + 63) / 64;
            int c = j + 1 + wv;
            constexpr int kB = kGemvBatch / kCoopRowsPerLane;   // loads in flight per lane
            for (; c + 16 * (kB - 1) < n; c += 16 * kB) {
                double av[kB][kCoopRowsPerLane];
#pragma unroll
                for (int u = 0; u < kB; ++u)
#pragma unroll
                    for (int q = 0; q < kCoopRowsPerLane; ++q) {
                        const int r = min(r0 + lane + 64 * q, r1 - 1);
                        av[u][q] = q < nq ? a.A[r + (int64_t)(c + 16 * u) * n] : 0.0;
                    }
#pragma unroll
                for (int u = 0; u < kB; ++u) {
                    const double vc = vsh[c + 16 * u];
#pragma unroll
                    for (int q = 0; q < kCoopRowsPerLane; ++q) yacc[q] += av[u][q] * vc;
                }
            }
            for (; c < n; c += 16) {
                const double vc = vsh[c];
#pragma unroll
                for (int q = 0; q < kCoopRowsPerLane; ++q) {
                    const int r = min(r0 + lane + 64 * q, r1 - 1);
                    if (q < nq) yacc[q] += a.A[r + (int64_t)c * n] * vc;
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
                    double y = 0.0;
                    for (int w = 0; w < 16; ++w) y += ysum[w][lane + 64 * q];
                    for (int c = 0; c < i; ++c) y -= a.Y[r + (int64_t)c * n] * sv[c];
                    a.Y[r + (int64_t)i * n] = sk ? 0.0 : 2.0 * y;
                }
            }
        if (blockIdx.x == 0 && tid <= i) {
            double tc = 2.0;
            if (tid < i) {
                double s = 0.0;
                for (int q = tid; q < i; ++q) s += ld_agent(&a.T[tid + q * kPanel]) * sv[q];
                tc = -2.0 * s;
            }
            st_agent(&a.T[tid + i * kPanel], tc);
        }
        __syncthreads();
        (void)red;
    }
}

// C (m x nn, ldc) += alpha * op(A) op(B); op = transpose when TA / TB.  64x64 tiles, 4x4/thread.
// Split-K: blockIdx.z takes rows [z kc, (z+1) kc) of the K range and, when gridDim.z > 1, writes its
// partial product to C + z * zstride (beta must be 0 then; gemm_reduce adds the partials in z order).
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_f64(int m, int nn, int kk, double alpha, const double* A, int64_t lda,
                                                const double* B, int64_t ldb, double beta, double* C, int64_t ldc,
                                                int kc, int64_t zstride) {
    constexpr int TM = 64, KT = 16;
    __shared__ double As[KT][TM + 1];
    __shared__ double Bs[KT][TM + 1];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int i0 = blockIdx.x * TM, j0 = blockIdx.y * TM;
    const int kb = blockIdx.z * kc;
    const int ke = min(kk, kb + kc);
    C += blockIdx.z * zstride;
    double acc[4][4] = {};
    for (int k0 = kb; k0 < ke; k0 += KT) {
        for (int e = threadIdx.x; e < KT * TM; e += 256) {
            int r, q;
            // A tile: op(A)(i0 + r, k0 + q)
            if (!TA) { r = e % TM; q = e / TM; } else { q = e % KT; r = e / KT; }
            {
                const int gi = i0 + r, gk = k0 + q;
                double val = 0.0;
                if (gi < m && gk < ke) val = TA ? A[gk + (int64_t)gi * lda] : A[gi + (int64_t)gk * lda];
                As[q][r] = val;
            }
            // B tile: op(B)(k0 + q, j0 + r)
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
        for (int q = 0; q < KT; ++q) {
            double av[4], bv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) { av[u] = As[q][tx + 16 * u]; bv[u] = Bs[q][ty + 16 * u]; }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int w = 0; w < 4; ++w) acc[u][w] += av[u] * bv[w];
        }
        __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int gi = i0 + tx + 16 * u, gj = j0 + ty + 16 * w;
            if (gi < m && gj < nn) {
                double* cp = C + gi + (int64_t)gj * ldc;
                *cp = (beta == 0.0 ? 0.0 : beta * *cp) + alpha * acc[u][w];
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

// C = beta C + sum_z P[z] (m x nn, P packed with leading dimension m), partials added in z order
__global__ void gemm_reduce(int m, int nn, int nz, const double* P, double beta, double* C, int64_t ldc) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (int64_t)m * nn) return;
    const int i = (int)(idx % m);
    const int64_t j = idx / m;
    double s = 0.0;
    for (int z = 0; z < nz; ++z) s += P[(int64_t)z * m * nn + idx];
    double* c = C + i + j * ldc;
    *c = (beta == 0.0 ? 0.0 : beta * *c) + s;
}

}  // namespace dev

namespace {
template <bool TA, bool TB>
void gemm(hipStream_t st, int m, int nn, int kk, double alpha, const double* A, int64_t lda, const double* B,
          int64_t ldb, double beta, double* C, int64_t ldc, double* work = nullptr, int64_t work_elems = 0) {
    if (m <= 0 || nn <= 0) return;
    const int bx = (m + 63) / 64, by = (nn + 63) / 64;
    // split K when the output has too few tiles to fill the chip (e.g. W = V^T A, 32 rows)
    int nz = 1;
    if (work && bx * by < 512 && kk >= 512) {
        nz = std::min(16, std::max(1, 1024 / (bx * by)));
        nz = std::min<int64_t>(nz, work_elems / ((int64_t)m * nn));
        nz = std::max(1, std::min(nz, kk / 128));
    }
    static const bool valu = std::getenv("EIGSOL_GEMM_VALU") != nullptr;
    auto kern = valu ? dev::gemm_f64<TA, TB> : dev::gemm_mfma_f64<TA, TB>;
    if (nz <= 1) {
        hipLaunchKernelGGL(kern, dim3(bx, by, 1), dim3(256), 0, st, m, nn, kk, alpha, A, lda, B, ldb, beta, C, ldc,
                           kk, (int64_t)0);
        return;
    }
    const int kc = ((kk + nz - 1) / nz + 15) / 16 * 16;
    nz = (kk + kc - 1) / kc;
    hipLaunchKernelGGL(kern, dim3(bx, by, nz), dim3(256), 0, st, m, nn, kk, alpha, A, lda, B, ldb, 0.0, work,
                       (int64_t)m, kc, (int64_t)m * nn);
    const int64_t tot = (int64_t)m * nn;
    hipLaunchKernelGGL(dev::gemm_reduce, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, m, nn, nz, work, beta,
                       C, ldc);
}
}  // namespace

// In place on the device matrix A (n x n, column-major, ld = n).
int hessenberg_blocked_f64(hipStream_t st, double* A, int64_t n64) {
    const int n = (int)n64;
    if (n < 3) return EIGSOL_OK;
    if (n > dev::kMaxLdsN) return fail(EIGSOL_E_UNSUPPORTED, "blocked Hessenberg: n > 16384");
    constexpr int NB = dev::kPanel;
    const int maxch = (n + dev::kGemvCols - 1) / dev::kGemvCols;
    double *V = nullptr, *Y = nullptr, *T = nullptr, *tv = nullptr, *yp = nullptr, *W = nullptr, *W2 = nullptr;
    int* skip = nullptr;
    EIGSOL_HIP(hipMalloc(&V, (size_t)n * NB * sizeof(double)));
    double *L = nullptr, *R = nullptr, *M = nullptr;
    EIGSOL_HIP(hipMalloc(&L, (size_t)n * 2 * NB * sizeof(double)));   // [Y | V zero above the panel]
    EIGSOL_HIP(hipMalloc(&R, (size_t)n * 2 * NB * sizeof(double)));   // [V(c1:, :) | W2^T]
    EIGSOL_HIP(hipMalloc(&M, (size_t)NB * NB * sizeof(double)));      // V^T Y
    Y = L;
    EIGSOL_HIP(hipMalloc(&T, NB * NB * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&tv, NB * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&yp, (size_t)maxch * n * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&W, (size_t)NB * n * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&W2, (size_t)NB * n * sizeof(double)));
    double* SK = nullptr;                 // split-K partials of W = V^T A (16 x 32 x n)
    const int64_t sk_elems = (int64_t)16 * NB * n;
    EIGSOL_HIP(hipMalloc(&SK, sk_elems * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&skip, 64));
    const size_t lds = (size_t)n * sizeof(double);
    // one cooperative launch per panel when the device supports it and n fits its LDS staging
    int coop_ok = 0, dev_id = 0;
    EIGSOL_HIP(hipGetDevice(&dev_id));
    EIGSOL_HIP(hipDeviceGetAttribute(&coop_ok, hipDeviceAttributeCooperativeLaunch, dev_id));
    bool coop = coop_ok && n <= dev::kCoopMaxN && std::getenv("EIGSOL_HESS_NO_COOP") == nullptr;
    const size_t coop_lds = (size_t)n * sizeof(double);
    const void* coop_kernel = n <= 64 * dev::kCoopBlocks ? reinterpret_cast<const void*>(dev::hess_panel_coop<1>)
                                                         : reinterpret_cast<const void*>(dev::hess_panel_coop<2>);
    double *part = nullptr, *tpart = nullptr, *x0s = nullptr;
    unsigned* bar = nullptr;
    int* err = nullptr;
    if (coop) {
        EIGSOL_HIP(hipMalloc(&part, 2 * dev::kCoopBlocks * NB * sizeof(double)));
        EIGSOL_HIP(hipMalloc(&tpart, dev::kCoopBlocks * sizeof(double)));
        EIGSOL_HIP(hipMalloc(&x0s, 64));
        EIGSOL_HIP(hipMalloc(&bar, 64));
        EIGSOL_HIP(hipMalloc(&err, 64));
        EIGSOL_HIP(hipMemsetAsync(err, 0, 64, st));
        EIGSOL_HIP(hipFuncSetAttribute(coop_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)coop_lds));
    }
    EIGSOL_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(dev::hess_panel_col),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int last = n - 3;   // reflector columns 0 .. n-3 (to_hessenberg.hpp:38)
    for (int k = 0; k <= last; k += NB) {
        const int nbp = std::min(NB, last - k + 1);
        EIGSOL_HIP(hipMemsetAsync(T, 0, NB * NB * sizeof(double), st));
        if (coop) {
            EIGSOL_HIP(hipMemsetAsync(bar, 0, 64, st));
            dev::CoopArgs ca{A, n, k, nbp, V, Y, T, part, tpart, x0s, bar, err};
            void* kargs[] = {&ca};
            // EIGSOL_HESS_COOP_PLAIN=1: the SAME panel kernel through an ordinary launch, for profiling
            // only (rocprofv3 7.2 crashes at exit after any cooperative launch, tools/coop_prof_repro.hip);
            // its kCoopBlocks blocks are far fewer than the CUs, so on an idle device all are resident,
            // and the grid barrier's bounded spin reports a failure instead of hanging otherwise
            static const bool plain = std::getenv("EIGSOL_HESS_COOP_PLAIN") != nullptr;
            if (plain)
                EIGSOL_HIP(hipLaunchKernel(coop_kernel, dim3(dev::kCoopBlocks), dim3(dev::kCoopThreads), kargs, coop_lds, st));
            else
                EIGSOL_HIP(hipLaunchCooperativeKernel(coop_kernel, dim3(dev::kCoopBlocks), dim3(dev::kCoopThreads), kargs,
                                                      coop_lds, st));
        }
        for (int i = 0; !coop && i < nbp; ++i) {
            const int j = k + i;
            hipLaunchKernelGGL(dev::hess_panel_col, dim3(1), dim3(1024), lds, st, A, n, k, j, i, V, Y, T, tv, skip);
            const int c0 = j + 1;
            const int nch = (n - c0 + dev::kGemvCols - 1) / dev::kGemvCols;
            hipLaunchKernelGGL(dev::hess_gemv, dim3((n + 255) / 256, nch), dim3(256), 0, st, A, n, c0,
                               V + (int64_t)i * n, yp, skip);
            hipLaunchKernelGGL(dev::hess_y, dim3((n + 255) / 256), dim3(256), 0, st, n, i, nch, yp, tv, Y, T, skip);
        }
        const int c1 = k + nbp;           // first trailing column
        const int mt = n - c1;
        if (mt > 0) {
            // A <- Q^T A Q with Q = I - V T V^T, in one pass over the trailing columns:
            //   right: A Q = A - Y V^T (Y = A V T from the panel);
            //   left:  Q^T (A Q) = A Q - V W2, W2 = T^T V^T (A Q) = T^T (V^T A - (V^T Y) V^T);
            // so A(:, c1:) -= [Y | V] [V(c1:, :) | W2^T]^T, one rank-2nbp update (V is zero above
            // row k+1), with W0 = V^T A read from A before it.
            const int rows = n - (k + 1);
            double* Vz = L + (int64_t)nbp * n;     // L = [Y | Vz], Y already in place
            double* R2 = R + (int64_t)nbp * n;     // R = [V(c1:, :) | W2^T]
            gemm<true, false>(st, nbp, mt, rows, 1.0, V + (k + 1), n, A + (k + 1) + (int64_t)c1 * n, n, 0.0, W, NB,
                              SK, sk_elems);
            gemm<true, false>(st, nbp, nbp, rows, 1.0, V + (k + 1), n, L + (k + 1), n, 0.0, M, NB, SK, sk_elems);
            EIGSOL_HIP(hipMemcpy2DAsync(R, n * sizeof(double), V + c1, n * sizeof(double), mt * sizeof(double), nbp,
                                        hipMemcpyDeviceToDevice, st));
            gemm<false, true>(st, nbp, mt, nbp, -1.0, M, NB, R, n, 1.0, W, NB);              // W = V^T (A Q)
            gemm<true, false>(st, mt, nbp, nbp, 1.0, W, NB, T, NB, 0.0, R2, n);              // W2^T = W^T T
            EIGSOL_HIP(hipMemsetAsync(Vz, 0, (size_t)nbp * n * sizeof(double), st));
            EIGSOL_HIP(hipMemcpy2DAsync(Vz + (k + 1), n * sizeof(double), V + (k + 1), n * sizeof(double),
                                        rows * sizeof(double), nbp, hipMemcpyDeviceToDevice, st));
            rankk_update<double, false>(st, n, mt, 2 * nbp, -1.0, L, n, R, n, A + (int64_t)c1 * n, n);
        }
    }
    EIGSOL_HIP(hipGetLastError());
    int errh = 0;
    if (coop) {
        EIGSOL_HIP(hipMemcpyAsync(&errh, err, sizeof(int), hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(hipStreamSynchronize(st));
    }
    for (void* p : {(void*)V, (void*)L, (void*)R, (void*)M, (void*)T, (void*)tv, (void*)yp, (void*)W, (void*)W2, (void*)skip,
                    (void*)part, (void*)tpart, (void*)x0s, (void*)bar, (void*)err, (void*)SK})
        if (p) (void)hipFree(p);
    if (errh) return fail(EIGSOL_E_HIP, "blocked Hessenberg: grid barrier timed out (internal error)");
    return EIGSOL_OK;
}

}  // namespace eigsol

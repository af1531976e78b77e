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
#include <vector>

#include "kernels_common.hpp"

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

// C (m x nn, ldc) += alpha * op(A) op(B); op = transpose when TA / TB.  64x64 tiles, 4x4/thread.
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_f64(int m, int nn, int kk, double alpha, const double* A, int64_t lda,
                                                const double* B, int64_t ldb, double beta, double* C, int64_t ldc) {
    constexpr int TM = 64, KT = 16;
    __shared__ double As[KT][TM + 1];
    __shared__ double Bs[KT][TM + 1];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int i0 = blockIdx.x * TM, j0 = blockIdx.y * TM;
    double acc[4][4] = {};
    for (int k0 = 0; k0 < kk; k0 += KT) {
        for (int e = threadIdx.x; e < KT * TM; e += 256) {
            int r, q;
            // A tile: op(A)(i0 + r, k0 + q)
            if (!TA) { r = e % TM; q = e / TM; } else { q = e % KT; r = e / KT; }
            {
                const int gi = i0 + r, gk = k0 + q;
                double val = 0.0;
                if (gi < m && gk < kk) val = TA ? A[gk + (int64_t)gi * lda] : A[gi + (int64_t)gk * lda];
                As[q][r] = val;
            }
            // B tile: op(B)(k0 + q, j0 + r)
            if (!TB) { q = e % KT; r = e / KT; } else { r = e % TM; q = e / TM; }
            {
                const int gk = k0 + q, gj = j0 + r;
                double val = 0.0;
                if (gk < kk && gj < nn) val = TB ? B[gj + (int64_t)gk * ldb] : B[gk + (int64_t)gj * ldb];
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

}  // namespace dev

namespace {
template <bool TA, bool TB>
void gemm(hipStream_t st, int m, int nn, int kk, double alpha, const double* A, int64_t lda, const double* B,
          int64_t ldb, double beta, double* C, int64_t ldc) {
    if (m <= 0 || nn <= 0) return;
    hipLaunchKernelGGL((dev::gemm_f64<TA, TB>), dim3((m + 63) / 64, (nn + 63) / 64), dim3(256), 0, st, m, nn, kk,
                       alpha, A, lda, B, ldb, beta, C, ldc);
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
    EIGSOL_HIP(hipMalloc(&Y, (size_t)n * NB * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&T, NB * NB * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&tv, NB * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&yp, (size_t)maxch * n * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&W, (size_t)NB * n * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&W2, (size_t)NB * n * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&skip, 64));
    const size_t lds = (size_t)n * sizeof(double);
    EIGSOL_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(dev::hess_panel_col),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int last = n - 3;   // reflector columns 0 .. n-3 (to_hessenberg.hpp:38)
    for (int k = 0; k <= last; k += NB) {
        const int nbp = std::min(NB, last - k + 1);
        EIGSOL_HIP(hipMemsetAsync(T, 0, NB * NB * sizeof(double), st));
        for (int i = 0; i < nbp; ++i) {
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
            // right: A(:, c1:n) -= Y V(c1:n, :)^T
            gemm<false, true>(st, n, mt, nbp, -1.0, Y, n, V + c1, n, 1.0, A + (int64_t)c1 * n, n);
            // left: W = V(k+1:n, :)^T A(k+1:n, c1:n); W2 = T^T W; A(k+1:n, c1:n) -= V W2
            const int rows = n - (k + 1);
            gemm<true, false>(st, nbp, mt, rows, 1.0, V + (k + 1), n, A + (k + 1) + (int64_t)c1 * n, n, 0.0, W, NB);
            gemm<true, false>(st, nbp, mt, nbp, 1.0, T, NB, W, NB, 0.0, W2, NB);
            gemm<false, false>(st, rows, mt, nbp, -1.0, V + (k + 1), n, W2, NB, 1.0, A + (k + 1) + (int64_t)c1 * n, n);
        }
    }
    EIGSOL_HIP(hipGetLastError());
    for (void* p : {(void*)V, (void*)Y, (void*)T, (void*)tv, (void*)yp, (void*)W, (void*)W2, (void*)skip})
        (void)hipFree(p);
    return EIGSOL_OK;
}

}  // namespace eigsol

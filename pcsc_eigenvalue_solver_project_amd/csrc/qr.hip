// Dense QR-method kernels for gfx950: Householder Hessenberg reduction, Householder QR, the
// reference's unshifted QR iteration, and Francis implicit double-shift sweeps.
//
// Reference (numeric core replaced):
//   to_hessenberg_dense<S>   src/qr_method/to_hessenberg.hpp:23-80
//   qr_decompose_dense<S>    src/qr_method/qr_decompose.hpp:25-86
//   qr_eigenvalues_dense<S>  src/qr_method/qr_eigenvalues.hpp:40-108 (unshifted H <- RQ)
// Householder convention (both reductions): x = column segment, alpha = -phase(x0) ||x||
// (phase 1 when x0 == 0), v = (x - alpha e1) / ||x - alpha e1||, reflector I - 2 v v^H; a step is
// skipped when ||x(1:)|| == 0 or ||v|| == 0 (to_hessenberg.hpp:45-65, qr_decompose.hpp:53-73).
//
// Device structure: every reflector is three launches, none of which needs a grid-wide sync —
//   hh_make   (one block)   : v and the skip flag from the column segment;
//   hh_left   (block/column): w_j = v^H B(:, j); B(:, j) -= 2 v w_j        (column-local)
//   hh_right  (block/16 rows): w_i = B(i, :) v;  B(i, :) -= 2 w_i v^H      (row-local)
// The matrix stays in HBM (a 4096^2 fp64 matrix is 128 MiB, inside the 256 MiB Infinity Cache).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <vector>

#include "kernels_common.hpp"

namespace eigsol {
namespace dev {

__device__ __forceinline__ double conj_(double a) { return a; }
__device__ __forceinline__ cplx conj_(cplx a) { return cplx{a.re, -a.im}; }
__device__ __forceinline__ double scale_(double a, double s) { return a * s; }
__device__ __forceinline__ cplx scale_(cplx a, double s) { return cplx{a.re * s, a.im * s}; }
__device__ __forceinline__ double abs_(double a) { return fabs(a); }
__device__ __forceinline__ double abs_(cplx a) { return hypot(a.re, a.im); }
__device__ __forceinline__ bool is_zero(double a) { return a == 0.0; }
__device__ __forceinline__ bool is_zero(cplx a) { return a.re == 0.0 && a.im == 0.0; }
__device__ __forceinline__ float conj_(float a) { return a; }
__device__ __forceinline__ cplxf conj_(cplxf a) { return cplxf{a.re, -a.im}; }
__device__ __forceinline__ float scale_(float a, double s) { return a * (float)s; }
__device__ __forceinline__ cplxf scale_(cplxf a, double s) { return cplxf{a.re * (float)s, a.im * (float)s}; }
__device__ __forceinline__ double abs_(float a) { return fabs((double)a); }
__device__ __forceinline__ double abs_(cplxf a) { return hypot((double)a.re, (double)a.im); }
__device__ __forceinline__ bool is_zero(float a) { return a == 0.0f; }
__device__ __forceinline__ bool is_zero(cplxf a) { return a.re == 0.0f && a.im == 0.0f; }

template <class S>
__device__ __forceinline__ S at(const S* A, int64_t ld, int64_t i, int64_t j) { return A[i + j * ld]; }

// block-wide deterministic sum (1024 threads = 16 waves), result broadcast to all threads
__device__ __forceinline__ double block_sum_1024(double v, double* sm /*16*/) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sm[w] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += sm[i];
    return s;
}

// reflector from x = A(r0 : r0+m, col): v (m scalars) and skip flag
template <class S>
__global__ __launch_bounds__(1024) void hh_make_kernel(const S* A, int64_t ld, int64_t r0, int64_t col,
                                                       int64_t m, S* v, int* skip) {
    __shared__ double sm[16];
    const S* x = A + r0 + col * ld;
    double tail = 0.0;
    for (int64_t i = 1 + threadIdx.x; i < m; i += blockDim.x) tail += sq_abs(x[i]);
    tail = block_sum_1024(tail, sm);
    const S x0 = x[0];
    const double nx = sqrt(tail + sq_abs(x0));   // ||x||
    if (tail == 0.0) {                            // ||x(1:)|| == 0: nothing to annihilate
        if (threadIdx.x == 0) *skip = 1;
        return;
    }
    S sign;
    if (is_zero(x0)) set_re_im(sign, 1.0, 0.0);
    else sign = scale_(x0, 1.0 / abs_(x0));
    // alpha = -sign * ||x||;  v0 = x0 - alpha = x0 + sign * ||x||
    S v0 = add(x0, scale_(sign, nx));
    const double vn = sqrt(tail + sq_abs(v0));
    if (vn == 0.0) {
        if (threadIdx.x == 0) *skip = 1;
        return;
    }
    const double rv = 1.0 / vn;
    for (int64_t i = threadIdx.x; i < m; i += blockDim.x) v[i] = scale_(i == 0 ? v0 : x[i], rv);
    if (threadIdx.x == 0) *skip = 0;
}

// B = A(r0 : r0+m, c0 : c1):  B(:, j) -= 2 v (v^H B(:, j)), one block per column
template <class S>
__global__ __launch_bounds__(256) void hh_left_kernel(S* A, int64_t ld, int64_t r0, int64_t m, int64_t c0,
                                                      const S* v, const int* skip) {
    if (*skip) return;
    __shared__ double sm[3 * kWaves];
    S* b = A + r0 + (c0 + blockIdx.x) * ld;
    double wr = 0.0, wi = 0.0;
    for (int64_t i = threadIdx.x; i < m; i += 256) acc_dot(wr, wi, v[i], b[i]);
    double dummy = 0.0;
    block_sum3(wr, wi, dummy, sm);
    __shared__ double s_w[2];
    if (threadIdx.x == 0) { s_w[0] = wr; s_w[1] = wi; }
    __syncthreads();
    S w2;
    set_re_im(w2, 2.0 * s_w[0], 2.0 * s_w[1]);
    for (int64_t i = threadIdx.x; i < m; i += 256) b[i] = sub(b[i], mul(v[i], w2));
}

// B = A(0 : nr, c0 : c0+m):  B(i, :) -= 2 (B(i, :) v) v^H, 16 rows per block, 16 lanes per row
template <class S>
__global__ __launch_bounds__(256) void hh_right_kernel(S* A, int64_t ld, int64_t nr, int64_t c0, int64_t m,
                                                       const S* v, const int* skip) {
    if (*skip) return;
    const int lane = threadIdx.x & 15;
    const int64_t i = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
    const bool live = i < nr;
    S* row = A + (live ? i : 0) + c0 * ld;
    S w = s_zero<S>();
    if (live)
        for (int64_t j = lane; j < m; j += 16) w = add(w, mul(row[j * ld], v[j]));
    // sum over the 16 lanes of the row (xor butterfly stays inside the group)
    double re, im = 0.0;
    if constexpr (is_real_v<S>) re = w;
    else { re = w.re; im = w.im; }
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) {
        re += __shfl_xor(re, off, 64);
        im += __shfl_xor(im, off, 64);
    }
    S w2;
    set_re_im(w2, 2.0 * re, 2.0 * im);
    if (live)
        for (int64_t j = lane; j < m; j += 16) row[j * ld] = sub(row[j * ld], mul(w2, conj_(v[j])));
}

template <class S>
__global__ void set_identity_kernel(S* A, int64_t n) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= n * n) return;
    S z = s_zero<S>();
    if (idx % n == idx / n) set_re_im(z, 1.0, 0.0);
    A[idx] = z;
}

// C = A * B (n x n, column-major), 64x64 tiles, 256 threads, 4x4 per thread
template <class S>
__global__ __launch_bounds__(256) void gemm_nn_kernel(const S* A, const S* B, S* C, int64_t n) {
    constexpr int T = 64, KT = 16;
    __shared__ S As[KT][T + 1];
    __shared__ S Bs[KT][T + 1];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int64_t i0 = (int64_t)blockIdx.x * T, j0 = (int64_t)blockIdx.y * T;
    S acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = s_zero<S>();
    for (int64_t k0 = 0; k0 < n; k0 += KT) {
        for (int e = threadIdx.x; e < KT * T; e += 256) {
            const int r = e % T, kk = e / T;
            const int64_t gi = i0 + r, gk = k0 + kk;
            As[kk][r] = (gi < n && gk < n) ? A[gi + gk * n] : s_zero<S>();
            const int64_t gj = j0 + r;
            Bs[kk][r] = (gk < n && gj < n) ? B[gk + gj * n] : s_zero<S>();
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < KT; ++kk) {
            S a[4], b[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) { a[q] = As[kk][tx + 16 * q]; b[q] = Bs[kk][ty + 16 * q]; }
#pragma unroll
            for (int p = 0; p < 4; ++p)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[p][q] = add(acc[p][q], mul(a[p], b[q]));
        }
        __syncthreads();
    }
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t gi = i0 + tx + 16 * p, gj = j0 + ty + 16 * q;
            if (gi < n && gj < n) C[gi + gj * n] = acc[p][q];
        }
}

// max_i |H(i, i-1)| and ||H||_F (qr_eigenvalues.hpp:79-88), one block, deterministic order
template <class S>
__global__ __launch_bounds__(1024) void subdiag_frob_kernel(const S* H, int64_t n, double* out) {
    __shared__ double sm[16];
    __shared__ double smx[1024];
    double f = 0.0, mx = 0.0;
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = threadIdx.x; i < n; i += 1024) {
            const S h = H[i + j * n];
            f += sq_abs(h);
            if (i == j + 1) mx = fmax(mx, abs_(h));
        }
    f = block_sum_1024(f, sm);
    smx[threadIdx.x] = mx;
    __syncthreads();
    for (int off = 512; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) smx[threadIdx.x] = fmax(smx[threadIdx.x], smx[threadIdx.x + off]);
        __syncthreads();
    }
    if (threadIdx.x == 0) { out[0] = smx[0]; out[1] = sqrt(f); }
}

template <class S>
__global__ void diag_kernel(const S* H, int64_t n, S* d) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) d[i] = H[i + i * n];
}

// ------------------------------------------------------------ Francis double shift (real)
// Whole active problem in LDS, one workgroup: scalar control (deflation search, shifts, the
// reflector) by thread 0, row and column updates of every 3x3 reflector by all threads.  The
// algorithm is the textbook eigenvalue-only double-shift QR (the oracle's hqr_francis restates
// it): deflation when |h(l,l-1)| <= eps (|h(l-1,l-1)| + |h(l,l)|), exceptional shifts at 10 and
// 20 iterations, `maxits` sweeps per eigenvalue before giving up.
struct HqrCtl {
    int nn, l, m, its, stage, fail;
    int total;          // sweeps performed
    int maxits;         // most sweeps any single deflation needed
    double t;           // accumulated exceptional shift
    double p, q, r, xs, ys, zs;
};

constexpr int kHqrMaxN = 128;   // 128^2 fp64 = 128 KiB of LDS

__global__ __launch_bounds__(1024) void hqr_lds_kernel(const double* Hin, int64_t ld, int n, double* wr,
                                                       double* wi, int maxits, int* info) {
    __shared__ double a[kHqrMaxN * kHqrMaxN];
    __shared__ HqrCtl c;
    __shared__ double s_anorm;
    const int tid = threadIdx.x;
    auto A = [&](int i, int j) -> double& { return a[i + j * n]; };
    for (int e = tid; e < n * n; e += blockDim.x) {
        const int i = e % n, j = e / n;
        a[e] = Hin[i + (int64_t)j * ld];
    }
    __syncthreads();
    if (tid == 0) {
        double s = 0.0;
        for (int i = 0; i < n; ++i)
            for (int j = max(i - 1, 0); j < n; ++j) s += fabs(A(i, j));
        s_anorm = s;
        c.nn = n - 1;
        c.t = 0.0;
        c.fail = 0;
        c.total = 0;
        c.maxits = 0;
        c.its = 0;
    }
    __syncthreads();
    const double eps = 2.220446049250313e-16;
    __shared__ int s_l;
    while (true) {
        // ---- deflation scan in parallel: the largest l in [1, nn] with a negligible h(l, l-1)
        if (tid == 0) s_l = 0;
        __syncthreads();
        const int nn0 = c.nn;
        if (nn0 < 0) break;
        for (int l = 1 + tid; l <= nn0; l += blockDim.x) {
            const double s0 = fabs(A(l - 1, l - 1)) + fabs(A(l, l));
            const double sc = s0 == 0.0 ? s_anorm : s0;
            if (fabs(A(l, l - 1)) <= eps * sc) atomicMax(&s_l, l);
        }
        __syncthreads();
        // ---- thread 0: 1x1 / 2x2 deflation or the next sweep's shift (start row m = l)
        if (tid == 0) {
            c.stage = 0;   // 0: sweep, 1: stop, 3: deflated (scan again)
            const int nn = nn0;
            const int l = s_l;
            if (l > 0) A(l, l - 1) = 0.0;
            const double x = A(nn, nn);
            if (l == nn) {
                wr[nn] = x + c.t; wi[nn] = 0.0; c.nn = nn - 1;
                c.maxits = max(c.maxits, c.its);
                c.its = 0;
                c.stage = 3;
            } else {
                const double y = A(nn - 1, nn - 1);
                const double w = A(nn, nn - 1) * A(nn - 1, nn);
                if (l == nn - 1) {
                    const double p = 0.5 * (y - x);
                    const double q = p * p + w;
                    const double z = sqrt(fabs(q));
                    const double xx = x + c.t;
                    if (q >= 0.0) {
                        const double zz = p + (p >= 0 ? fabs(z) : -fabs(z));
                        wr[nn - 1] = wr[nn] = xx + zz;
                        if (zz != 0.0) wr[nn] = xx - w / zz;
                        wi[nn - 1] = wi[nn] = 0.0;
                    } else {
                        wr[nn - 1] = wr[nn] = xx + p;
                        wi[nn - 1] = -z;
                        wi[nn] = z;
                    }
                    c.nn = nn - 2;
                    c.maxits = max(c.maxits, c.its);
                    c.its = 0;
                    c.stage = 3;
                } else if (c.its >= maxits) {
                    c.fail = 1;
                    c.stage = 1;
                } else {
                    double xs = x, ys = y, ws = w;
                    if (c.its == 10 || c.its == 20) {   // exceptional shift
                        c.t += xs;
                        for (int i = 0; i <= nn; ++i) A(i, i) -= xs;
                        const double s = fabs(A(nn, nn - 1)) + fabs(A(nn - 1, nn - 2));
                        ys = xs = 0.75 * s;
                        ws = -0.4375 * s * s;
                    }
                    ++c.its;
                    ++c.total;
                    // the sweep starts at m = l (the textbook's search for two small consecutive
                    // subdiagonals is an O(n) scalar loop; starting at l is always valid)
                    const int m = l;
                    const double z = A(m, m);
                    const double r0 = xs - z, s1 = ys - z;
                    double p = (r0 * s1 - ws) / A(m + 1, m) + A(m, m + 1);
                    double q = A(m + 1, m + 1) - z - r0 - s1;
                    double r = A(m + 2, m + 1);
                    const double sc = fabs(p) + fabs(q) + fabs(r);
                    p /= sc; q /= sc; r /= sc;
                    c.l = l;
                    c.m = m;
                    c.p = p; c.q = q; c.r = r;
                }
            }
        }
        __syncthreads();
        if (c.stage == 1) break;
        if (c.stage == 3) continue;
        {
            // clear the sub-subdiagonals of the active block (textbook: before the sweep)
            const int m = c.m, nn = c.nn;
            for (int i = m + tid; i <= nn - 2; i += blockDim.x) {
                A(i + 2, i) = 0.0;
                if (i != m) A(i + 2, i - 1) = 0.0;
            }
            __syncthreads();
        }
        const int l = c.l, m = c.m, nn = c.nn;
        // ---- the sweep: one 3x3 reflector per k, updates in parallel
        for (int k = m; k <= nn - 1; ++k) {
            if (tid == 0) {
                double p = c.p, q = c.q, r = c.r, xs = 1.0;
                if (k != m) {
                    p = A(k, k - 1);
                    q = A(k + 1, k - 1);
                    r = (k != nn - 1) ? A(k + 2, k - 1) : 0.0;
                    xs = fabs(p) + fabs(q) + fabs(r);
                    if (xs != 0.0) { p /= xs; q /= xs; r /= xs; }
                }
                const double s = (p >= 0 ? 1.0 : -1.0) * sqrt(p * p + q * q + r * r);
                if (s != 0.0) {
                    if (k == m) {
                        if (l != m) A(k, k - 1) = -A(k, k - 1);
                    } else {
                        A(k, k - 1) = -s * xs;
                    }
                    p += s;
                    c.xs = p / s;
                    c.ys = q / s;
                    c.zs = r / s;
                    c.q = q / p;
                    c.r = r / p;
                    c.stage = 2;   // apply
                } else {
                    c.stage = 0;   // skip
                }
            }
            __syncthreads();
            if (c.stage == 2) {
                const double xs = c.xs, ys = c.ys, zs = c.zs, q = c.q, r = c.r;
                const bool three = k != nn - 1;
                for (int j = k + tid; j <= nn; j += blockDim.x) {
                    double p = A(k, j) + q * A(k + 1, j);
                    if (three) { p += r * A(k + 2, j); A(k + 2, j) -= p * zs; }
                    A(k + 1, j) -= p * ys;
                    A(k, j) -= p * xs;
                }
                __syncthreads();
                const int mmin = nn < k + 3 ? nn : k + 3;
                for (int i = l + tid; i <= mmin; i += blockDim.x) {
                    double p = xs * A(i, k) + ys * A(i, k + 1);
                    if (three) { p += zs * A(i, k + 2); A(i, k + 2) -= p * r; }
                    A(i, k + 1) -= p * q;
                    A(i, k) -= p;
                }
            }
            __syncthreads();
        }
    }
    if (tid == 0) { info[0] = c.fail; info[1] = max(c.maxits, c.its); info[2] = c.total; }
}

// max |a_ij| as the bit pattern of a non-negative double (ordered like the value), for the
// norm-range check before the Francis path
__global__ __launch_bounds__(256) void absmax_kernel(const double* A, int64_t cnt, unsigned long long* out) {
    double m = 0.0;
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * 256) m = fmax(m, fabs(A[i]));
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) atomicMax(out, (unsigned long long)__double_as_longlong(m));
}

__global__ __launch_bounds__(256) void scale_pow2_kernel(double* A, int64_t cnt, int e) {
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * 256)
        A[i] = __builtin_amdgcn_ldexp(A[i], e);
}
}  // namespace dev

// ============================================================================ host drivers
int hessenberg_blocked_f64(hipStream_t st, double* A, int64_t n);
int hessenberg_blocked_c128(hipStream_t st, cplx* A, int64_t n);
int qr_blocked_f64(hipStream_t st, double* R, int64_t m, int64_t n, double* Q);
int qr_blocked_c128(hipStream_t st, cplx* R, int64_t m, int64_t n, cplx* Q);
int hessenberg_blocked_f32(hipStream_t st, float* A, int64_t n);
int hessenberg_blocked_c64(hipStream_t st, cplxf* A, int64_t n);
int qr_blocked_f32(hipStream_t st, float* R, int64_t m, int64_t n, float* Q);
int qr_blocked_c64(hipStream_t st, cplxf* R, int64_t m, int64_t n, cplxf* Q);

namespace {

template <class S>
struct QrWork {
    S* v = nullptr;
    int* skip = nullptr;
    double* red = nullptr;
    double* hred = nullptr;   // pinned host copy of red (a pageable copy sleeps ~1 ms per iteration)
};

template <class S>
int work_alloc(QrWork<S>& w, int64_t n) {
    EIGSOL_HIP(hipMalloc(&w.v, std::max<int64_t>(n, 1) * sizeof(S)));
    EIGSOL_HIP(hipMalloc(&w.skip, 64));
    EIGSOL_HIP(hipMalloc(&w.red, 64));
    EIGSOL_HIP(hipHostMalloc(&w.hred, 64, hipHostMallocDefault));
    return EIGSOL_OK;
}
template <class S>
void work_free(QrWork<S>& w) {
    if (w.v) (void)hipFree(w.v);
    if (w.skip) (void)hipFree(w.skip);
    if (w.red) (void)hipFree(w.red);
    if (w.hred) (void)hipHostFree(w.hred);
}

// one reflector: x = A(r0 : r0+m, col); left on A(r0 : r0+m, lc0 : lc1); right on B(0 : nr, r0 : r0+m)
template <class S>
void reflect(hipStream_t st, S* A, int64_t lda, int64_t r0, int64_t col, int64_t m, int64_t lc0,
             int64_t lc1, S* B, int64_t ldb, int64_t nr, QrWork<S>& w) {
    hipLaunchKernelGGL((dev::hh_make_kernel<S>), dim3(1), dim3(1024), 0, st, A, lda, r0, col, m, w.v, w.skip);
    if (lc1 > lc0)
        hipLaunchKernelGGL((dev::hh_left_kernel<S>), dim3(lc1 - lc0), dim3(256), 0, st, A, lda, r0, m, lc0,
                           w.v, w.skip);
    if (nr > 0)
        hipLaunchKernelGGL((dev::hh_right_kernel<S>), dim3((nr + 15) / 16), dim3(256), 0, st, B, ldb, nr, r0,
                           m, w.v, w.skip);
}

// to_hessenberg_dense (to_hessenberg.hpp:38-77) on H (device, n x n, in place)
template <class S>
int hessenberg_t(hipStream_t st, S* H, int64_t n, QrWork<S>& w) {
    for (int64_t k = 0; k + 2 < n; ++k) {
        const int64_t m = n - k - 1;
        // left: rows k+1.., cols k..n-1; right: rows 0..n-1, cols k+1..n-1
        reflect<S>(st, H, n, k + 1, k, m, k, n, H, n, n, w);
    }
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

// Matrices of moderate size use the blocked (panel + GEMM) reduction (hessenberg.hip): real up to
// n = 16384, complex up to 8192 (the panel column in LDS); others the per-reflector kernels above
// (EIGSOL_HESS_UNBLOCKED=1 forces those, for A/B).
template <class S>
int hessenberg_dev(hipStream_t st, S* H, int64_t n, QrWork<S>& w) {
    static const bool unblocked = std::getenv("EIGSOL_HESS_UNBLOCKED") != nullptr;
    if (!unblocked) {
        if constexpr (std::is_same_v<S, double>) {
            if (n >= 64 && n <= 16384) return hessenberg_blocked_f64(st, H, n);
        } else if constexpr (std::is_same_v<S, cplx>) {
            if (n >= 64 && n <= 8192) return hessenberg_blocked_c128(st, H, n);
        } else if constexpr (std::is_same_v<S, float>) {
            if (n >= 64 && n <= 16384) return hessenberg_blocked_f32(st, H, n);
        } else {
            if (n >= 64 && n <= 16384) return hessenberg_blocked_c64(st, H, n);
        }
    }
    return hessenberg_t<S>(st, H, n, w);
}

// qr_decompose_dense (qr_decompose.hpp:46-85): R = A (m x n) in place, Q (m x m) = I then updated
// Blocked (compact WY, hessenberg.hip) from min(m, n) >= 64 while a column fits the panel
// kernel's LDS; EIGSOL_QR_UNBLOCKED=1 forces the per-reflector kernels (A/B).
template <class S>
int qr_decompose_t(hipStream_t st, S* R, int64_t m, int64_t n, S* Q, QrWork<S>& w) {
    hipLaunchKernelGGL((dev::set_identity_kernel<S>), dim3((m * m + 255) / 256), dim3(256), 0, st, Q, m);
    static const bool unblocked = std::getenv("EIGSOL_QR_UNBLOCKED") != nullptr;
    const int64_t lds_max = std::is_same_v<S, cplx> ? 8192 : 16384;
    if (!unblocked && std::min(m, n) >= 64 && m <= lds_max && n <= INT32_MAX / 2) {
        if constexpr (std::is_same_v<S, double>) return qr_blocked_f64(st, R, m, n, Q);
        else if constexpr (std::is_same_v<S, cplx>) return qr_blocked_c128(st, R, m, n, Q);
        else if constexpr (std::is_same_v<S, float>) return qr_blocked_f32(st, R, m, n, Q);
        else return qr_blocked_c64(st, R, m, n, Q);
    }
    const int64_t kmax = std::min(m, n);
    for (int64_t k = 0; k < kmax; ++k) {
        const int64_t rows = m - k;
        if (rows < 2) continue;   // x.tail(0).norm() == 0: skipped by the reference too
        reflect<S>(st, R, m, k, k, rows, k, n, Q, m, m, w);
    }
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

}  // namespace

// ---------------------------------------------------------------------------- C ABI entry points
template <class S>
static int hessenberg_host(eigsol_ctx* ctx, int64_t n, const void* A, void* Hout) {
    hipStream_t st = ctx->stream;
    S* H = nullptr;
    EIGSOL_HIP(hipMalloc(&H, std::max<int64_t>(n * n, 1) * sizeof(S)));
    QrWork<S> w;
    int rc = work_alloc(w, n);
    if (rc == EIGSOL_OK && hipMemcpyAsync(H, A, n * n * sizeof(S), hipMemcpyHostToDevice, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "to_hessenberg: upload");
    if (rc == EIGSOL_OK) rc = hessenberg_dev<S>(st, H, n, w);
    if (rc == EIGSOL_OK && hipMemcpyAsync(Hout, H, n * n * sizeof(S), hipMemcpyDeviceToHost, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "to_hessenberg: download");
    if (rc == EIGSOL_OK && stream_wait(st) != hipSuccess) rc = fail(EIGSOL_E_HIP, "to_hessenberg: sync");
    work_free(w);
    (void)hipFree(H);
    return rc;
}

template <class S>
static int qr_decompose_host(eigsol_ctx* ctx, int64_t m, int64_t n, const void* A, void* Qout, void* Rout) {
    hipStream_t st = ctx->stream;
    S *R = nullptr, *Q = nullptr;
    EIGSOL_HIP(hipMalloc(&R, m * n * sizeof(S)));
    EIGSOL_HIP(hipMalloc(&Q, m * m * sizeof(S)));
    QrWork<S> w;
    int rc = work_alloc(w, m);
    if (rc == EIGSOL_OK && hipMemcpyAsync(R, A, m * n * sizeof(S), hipMemcpyHostToDevice, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "qr_decompose: upload");
    if (rc == EIGSOL_OK) rc = qr_decompose_t<S>(st, R, m, n, Q, w);
    if (rc == EIGSOL_OK && Qout && hipMemcpyAsync(Qout, Q, m * m * sizeof(S), hipMemcpyDeviceToHost, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "qr_decompose: download Q");
    if (rc == EIGSOL_OK && Rout && hipMemcpyAsync(Rout, R, m * n * sizeof(S), hipMemcpyDeviceToHost, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "qr_decompose: download R");
    if (rc == EIGSOL_OK && stream_wait(st) != hipSuccess) rc = fail(EIGSOL_E_HIP, "qr_decompose: sync");
    work_free(w);
    (void)hipFree(R);
    (void)hipFree(Q);
    return rc;
}

// qr_eigenvalues_dense, reference algorithm (unshifted): Hessenberg, then H <- R Q until
// max |H(i,i-1)| <= tol (1 + ||H||_F); iterations = iter + 1 (qr_eigenvalues.hpp:61-104)
template <class S>
static int qr_unshifted_host(eigsol_ctx* ctx, int64_t n, const void* A, int max_iter, double tol,
                             void* eig, int32_t* iters, int32_t* conv) {
    hipStream_t st = ctx->stream;
    S *H = nullptr, *Q = nullptr, *R = nullptr, *d = nullptr;
    int rc = EIGSOL_OK;
    if (hipMalloc(&H, n * n * sizeof(S)) != hipSuccess || hipMalloc(&Q, n * n * sizeof(S)) != hipSuccess ||
        hipMalloc(&R, n * n * sizeof(S)) != hipSuccess || hipMalloc(&d, n * sizeof(S)) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: hipMalloc");
    QrWork<S> w;
    if (rc == EIGSOL_OK) rc = work_alloc(w, n);
    if (rc == EIGSOL_OK && hipMemcpyAsync(H, A, n * n * sizeof(S), hipMemcpyHostToDevice, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: upload");
    if (rc == EIGSOL_OK) rc = hessenberg_dev<S>(st, H, n, w);
    int iter = 0;
    bool converged = false;
    const dim3 g((n + 63) / 64, (n + 63) / 64);
    for (iter = 0; rc == EIGSOL_OK && iter < max_iter; ++iter) {
        if (hipMemcpyAsync(R, H, n * n * sizeof(S), hipMemcpyDeviceToDevice, st) != hipSuccess) {
            rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: copy");
            break;
        }
        rc = qr_decompose_t<S>(st, R, n, n, Q, w);
        if (rc != EIGSOL_OK) break;
        hipLaunchKernelGGL((dev::gemm_nn_kernel<S>), g, dim3(256), 0, st, R, Q, H, n);
        hipLaunchKernelGGL((dev::subdiag_frob_kernel<S>), dim3(1), dim3(1024), 0, st, H, n, w.red);
        const double* red = w.hred;
        if (hipMemcpyAsync(w.hred, w.red, 2 * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
            stream_wait(st) != hipSuccess) {
            rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: convergence check");
            break;
        }
        if (red[0] <= tol * (1.0 + red[1])) {
            converged = true;
            break;
        }
    }
    if (rc == EIGSOL_OK) {
        hipLaunchKernelGGL((dev::diag_kernel<S>), dim3((n + 255) / 256), dim3(256), 0, st, H, n, d);
        if (hipMemcpyAsync(eig, d, n * sizeof(S), hipMemcpyDeviceToHost, st) != hipSuccess ||
            stream_wait(st) != hipSuccess)
            rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: download");
    }
    if (iters) *iters = iter + 1;
    if (conv) *conv = converged ? 1 : 0;
    work_free(w);
    for (void* p : {(void*)H, (void*)Q, (void*)R, (void*)d}) (void)hipFree(p);
    return rc;
}

// Francis double shift on a real matrix (Hessenberg on the device, then the sweeps)
int francis_large_f64(eigsol_ctx* ctx, double* H, int64_t n, int maxits, double* wr, double* wi,
                      int32_t* sweeps, int32_t* fail_out);

static int qr_francis_host(eigsol_ctx* ctx, int64_t n, const double* A, int max_iter, double* wr,
                           double* wi, int32_t* iters, int32_t* conv) {
    hipStream_t st = ctx->stream;
    double* H = nullptr;
    int rc = EIGSOL_OK;
    if (hipMalloc(&H, n * n * sizeof(double)) != hipSuccess) rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: hipMalloc");
    QrWork<double> w;
    if (rc == EIGSOL_OK) rc = work_alloc(w, n);
    if (rc == EIGSOL_OK && hipMemcpyAsync(H, A, n * n * sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: upload");
    // LAPACK xGEEV's range guard: a matrix whose largest entry lies outside [smlnum, bignum]
    // (smlnum = sqrt(safe min) / eps) is scaled into range first, here by an exact power of two, and
    // the eigenvalues are scaled back; squared norms in the reflectors would under- or overflow
    // otherwise.  Matrices inside the range are untouched (bit-identical path).
    int escale = 0;
    unsigned long long bits = 0;   // max |a_ij| as its bit pattern (nonnegative doubles order as integers)
    if (rc == EIGSOL_OK) {
        unsigned long long* dmax = nullptr;
        if (hipMallocAsync(reinterpret_cast<void**>(&dmax), sizeof(bits), st) != hipSuccess) {
            rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: hipMallocAsync");
        } else {
            hipMemsetAsync(dmax, 0, sizeof(bits), st);
            hipLaunchKernelGGL(dev::absmax_kernel, dim3(1024), dim3(256), 0, st, H, n * n, dmax);
            hipMemcpyAsync(&bits, dmax, sizeof(bits), hipMemcpyDeviceToHost, st);
            (void)hipFreeAsync(dmax, st);
            if (stream_wait(st) != hipSuccess) rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: norm-range check");
        }
    }
    if (rc == EIGSOL_OK) {
        double amax;
        std::memcpy(&amax, &bits, sizeof(amax));
        const double smlnum = std::sqrt(std::numeric_limits<double>::min()) / std::numeric_limits<double>::epsilon();
        if (std::isfinite(amax) && amax > 0.0 && (amax < smlnum || amax > 1.0 / smlnum)) {
            escale = -std::ilogb(amax);
            hipLaunchKernelGGL(dev::scale_pow2_kernel, dim3(1024), dim3(256), 0, st, H, n * n, escale);
        }
    }
    if (rc == EIGSOL_OK) rc = hessenberg_dev<double>(st, H, n, w);
    int32_t sweeps = 0, failed = 0;
    if (rc == EIGSOL_OK) rc = francis_large_f64(ctx, H, n, max_iter, wr, wi, &sweeps, &failed);
    if (rc == EIGSOL_OK && escale != 0)
        for (int64_t i = 0; i < n; ++i) {
            wr[i] = std::ldexp(wr[i], -escale);
            wi[i] = std::ldexp(wi[i], -escale);
        }
    if (iters) *iters = sweeps;
    if (conv) *conv = failed ? 0 : 1;
    work_free(w);
    (void)hipFree(H);
    return rc;
}

// Complex multishift QR (zfrancis.hip): Hessenberg on the device, then complex sweeps; the same
// norm-range guard as the real path (max |Re|, |Im| of the entries outside [smlnum, 1/smlnum] ->
// exact power-of-two scaling, eigenvalues scaled back)
int francis_large_c128(eigsol_ctx* ctx, cplx* H, int64_t n, int maxits, cplx* w_host, int32_t* sweeps_out,
                       int32_t* fail_out);

static int qr_francis_c128_host(eigsol_ctx* ctx, int64_t n, const void* A, int max_iter, cplx* w,
                                int32_t* iters, int32_t* conv) {
    hipStream_t st = ctx->stream;
    cplx* H = nullptr;
    int rc = EIGSOL_OK;
    if (hipMalloc(&H, n * n * sizeof(cplx)) != hipSuccess) rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: hipMalloc");
    QrWork<cplx> wk;
    if (rc == EIGSOL_OK) rc = work_alloc(wk, n);
    if (rc == EIGSOL_OK && hipMemcpyAsync(H, A, n * n * sizeof(cplx), hipMemcpyHostToDevice, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: upload");
    int escale = 0;
    if (rc == EIGSOL_OK) {
        unsigned long long* dmax = nullptr;
        unsigned long long bits = 0;
        if (hipMallocAsync(reinterpret_cast<void**>(&dmax), sizeof(bits), st) != hipSuccess) {
            rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: hipMallocAsync");
        } else {
            double* Hd = reinterpret_cast<double*>(H);
            hipMemsetAsync(dmax, 0, sizeof(bits), st);
            hipLaunchKernelGGL(dev::absmax_kernel, dim3(1024), dim3(256), 0, st, Hd, 2 * n * n, dmax);
            hipMemcpyAsync(&bits, dmax, sizeof(bits), hipMemcpyDeviceToHost, st);
            (void)hipFreeAsync(dmax, st);
            if (stream_wait(st) != hipSuccess) rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: norm-range check");
            double amax;
            std::memcpy(&amax, &bits, sizeof(amax));
            const double smlnum = std::sqrt(std::numeric_limits<double>::min()) / std::numeric_limits<double>::epsilon();
            if (rc == EIGSOL_OK && std::isfinite(amax) && amax > 0.0 && (amax < smlnum || amax > 1.0 / smlnum)) {
                escale = -std::ilogb(amax);
                hipLaunchKernelGGL(dev::scale_pow2_kernel, dim3(1024), dim3(256), 0, st, Hd, 2 * n * n, escale);
            }
        }
    }
    if (rc == EIGSOL_OK) rc = hessenberg_dev<cplx>(st, H, n, wk);
    int32_t sweeps = 0, failed = 0;
    if (rc == EIGSOL_OK) rc = francis_large_c128(ctx, H, n, max_iter, w, &sweeps, &failed);
    if (rc == EIGSOL_OK && escale != 0)
        for (int64_t i = 0; i < n; ++i) {
            w[i].re = std::ldexp(w[i].re, -escale);
            w[i].im = std::ldexp(w[i].im, -escale);
        }
    if (iters) *iters = sweeps;
    if (conv) *conv = failed ? 0 : 1;
    work_free(wk);
    (void)hipFree(H);
    return rc;
}

// Small problems: the whole matrix in LDS (n <= kHqrMaxN).  Larger: see francis.hip.
int hqr_lds(hipStream_t st, const double* H, int64_t ld, int n, int maxits, double* wr_dev, double* wi_dev,
            int* info_dev) {
    if (n > dev::kHqrMaxN) return fail(EIGSOL_E_UNSUPPORTED, "hqr_lds: n > 128");
    // one wave for shift-sized problems (its barriers cost nothing), four waves otherwise
    const int threads = n <= 64 ? 64 : 256;
    hipLaunchKernelGGL(dev::hqr_lds_kernel, dim3(1), dim3(threads), 0, st, H, ld, n, wr_dev, wi_dev, maxits, info_dev);
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

int wide_hessenberg(eigsol_ctx* ctx, int dtype, int64_t n, const void* A, void* H);   // wide.hip
int wide_qr_decompose(eigsol_ctx* ctx, int dtype, int64_t m, int64_t n, const void* A, void* Q, void* R);
int wide_qr_eigenvalues(eigsol_ctx* ctx, int dtype, int64_t n, const void* A, const eigsol_solver_options* opts,
                        int variant, void* eig, double* eig_im, int32_t* iters, int32_t* conv);

}  // namespace eigsol

using namespace eigsol;

extern "C" {

int eigsol_hessenberg_dense(eigsol_ctx* ctx, int dtype, int64_t n, const void* A_colmajor, void* H_out) {
    if (!ctx || (!A_colmajor && n) || (!H_out && n)) return fail(EIGSOL_E_INVALID, "eigsol_hessenberg_dense: null pointer");
    if (n == 0) return EIGSOL_OK;
    EIGSOL_HIP(hipSetDevice(ctx->device));
    if (dtype_wide(dtype)) return wide_hessenberg(ctx, dtype, n, A_colmajor, H_out);
    if (!dtype_valid(dtype)) return fail(EIGSOL_E_INVALID, "eigsol_hessenberg_dense: unknown dtype");
    switch (dtype) {
        case EIGSOL_C128: return hessenberg_host<cplx>(ctx, n, A_colmajor, H_out);
        case EIGSOL_F32: return hessenberg_host<float>(ctx, n, A_colmajor, H_out);
        case EIGSOL_C64: return hessenberg_host<cplxf>(ctx, n, A_colmajor, H_out);
        default: return hessenberg_host<double>(ctx, n, A_colmajor, H_out);
    }
}

int eigsol_qr_decompose_dense(eigsol_ctx* ctx, int dtype, int64_t m, int64_t n, const void* A_colmajor,
                              void* Q_out, void* R_out) {
    if (!ctx) return fail(EIGSOL_E_INVALID, "eigsol_qr_decompose_dense: null ctx");
    if (m == 0 || n == 0) return fail(EIGSOL_E_EMPTY, "qr_decompose_dense: empty matrix");
    if (!A_colmajor) return fail(EIGSOL_E_INVALID, "eigsol_qr_decompose_dense: null A");
    EIGSOL_HIP(hipSetDevice(ctx->device));
    if (dtype_wide(dtype)) return wide_qr_decompose(ctx, dtype, m, n, A_colmajor, Q_out, R_out);
    if (!dtype_valid(dtype)) return fail(EIGSOL_E_INVALID, "eigsol_qr_decompose_dense: unknown dtype");
    switch (dtype) {
        case EIGSOL_C128: return qr_decompose_host<cplx>(ctx, m, n, A_colmajor, Q_out, R_out);
        case EIGSOL_F32: return qr_decompose_host<float>(ctx, m, n, A_colmajor, Q_out, R_out);
        case EIGSOL_C64: return qr_decompose_host<cplxf>(ctx, m, n, A_colmajor, Q_out, R_out);
        default: return qr_decompose_host<double>(ctx, m, n, A_colmajor, Q_out, R_out);
    }
}

int eigsol_qr_eigenvalues_dense(eigsol_ctx* ctx, int dtype, int64_t n, const void* A_colmajor,
                                const eigsol_solver_options* opts, int variant, void* eig_re_or_c,
                                double* eig_im, int32_t* iterations, int32_t* converged) {
    if (!ctx || !opts) return fail(EIGSOL_E_INVALID, "eigsol_qr_eigenvalues_dense: null pointer");
    if (n == 0) {   // qr_eigenvalues.hpp:55-57
        if (iterations) *iterations = 0;
        if (converged) *converged = 1;
        return EIGSOL_OK;
    }
    if (!A_colmajor || !eig_re_or_c) return fail(EIGSOL_E_INVALID, "eigsol_qr_eigenvalues_dense: null pointer");
    EIGSOL_HIP(hipSetDevice(ctx->device));
    if (dtype_wide(dtype))
        return wide_qr_eigenvalues(ctx, dtype, n, A_colmajor, opts, variant, eig_re_or_c, eig_im, iterations, converged);
    if (!dtype_valid(dtype)) return fail(EIGSOL_E_INVALID, "eigsol_qr_eigenvalues_dense: unknown dtype");
    if (dtype == EIGSOL_F32 || dtype == EIGSOL_C64) {
        // single precision: the reference's unshifted iteration natively (blocked QR decompositions
        // and products in float); the Francis sweeps are built in double (the facade promotes)
        if (variant != EIGSOL_QR_UNSHIFTED)
            return fail(EIGSOL_E_UNSUPPORTED, "qr_eigenvalues: the multishift sweeps run in double precision");
        return dtype == EIGSOL_F32
                   ? qr_unshifted_host<float>(ctx, n, A_colmajor, opts->max_iterations, opts->tolerance, eig_re_or_c,
                                              iterations, converged)
                   : qr_unshifted_host<cplxf>(ctx, n, A_colmajor, opts->max_iterations, opts->tolerance, eig_re_or_c,
                                              iterations, converged);
    }
    if (variant != EIGSOL_QR_UNSHIFTED && dtype == EIGSOL_C128)
        return qr_francis_c128_host(ctx, n, A_colmajor, opts->max_iterations, static_cast<cplx*>(eig_re_or_c),
                                    iterations, converged);
    if (variant == EIGSOL_QR_UNSHIFTED || dtype == EIGSOL_C128)
        return dtype == EIGSOL_C128
                   ? qr_unshifted_host<cplx>(ctx, n, A_colmajor, opts->max_iterations, opts->tolerance,
                                             eig_re_or_c, iterations, converged)
                   : qr_unshifted_host<double>(ctx, n, A_colmajor, opts->max_iterations, opts->tolerance,
                                               eig_re_or_c, iterations, converged);
    std::vector<double> wi(n);
    const int rc = qr_francis_host(ctx, n, static_cast<const double*>(A_colmajor), opts->max_iterations,
                                   static_cast<double*>(eig_re_or_c), wi.data(), iterations, converged);
    if (rc == EIGSOL_OK && eig_im) std::memcpy(eig_im, wi.data(), n * sizeof(double));
    return rc;
}

}  // extern "C"

// Extended precision on gfx950: long double / std::complex<long double> as double-double.
//
// The reference admits long double and std::complex<long double> (ScalarConcept,
// src/core/types.hpp:28-30) and computes every solver in them through Eigen (x87 80-bit, a 64-bit
// significand).  These kernels compute the same loops in double-double (wide.hpp, a 106-bit
// significand), so no input is rounded and no operation is narrower than the reference's:
//   * products A x (CSR: one row per lane, ascending columns, as Eigen's CSC scatter sums a row;
//     dense: row tiles x column chunks), norms and Rayleigh quotients in double-double;
//   * powerMethodImpl (power_method.hpp:47-99) with the reference's stopping rule
//     (tolerance.hpp:28-33), one product per iteration (the Rayleigh product A x_k is the next
//     iteration's y, power_method.hpp:69 / :81, computed once);
//   * shiftedInversePowerImpl (shifted_inverse_power_solver.hpp:21-79) and solve_shifted
//     (solve_shifted.hpp:48-118): A - sigma I is factored ONCE in fp64 (the library's triangular,
//     band, GMRES or dense factor of the matrix rounded to double) and every solve is refined to
//     double-double accuracy: y <- y + M64^-1 r with the residual r = b - (A - sigma I) y computed in
//     double-double (classical mixed-precision iterative refinement; it contracts by ~cond(M) 2^-53
//     per step, so a few steps reach the double-double floor); the Rayleigh quotient is x^H (A x)
//     on A itself (:62), a double-double product;
//   * to_hessenberg_dense (to_hessenberg.hpp:23-80), qr_decompose_dense (qr_decompose.hpp:25-86)
//     and the reference's unshifted qr_eigenvalues_dense (qr_eigenvalues.hpp:40-108): per-reflector
//     kernels (make / left / right) in double-double, H <- R Q by a double-double GEMM.
// The host runs the reference loops' scalar logic in double-double too (one synchronisation per
// iteration: this is the precision path, not the headline path).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <numeric>
#include <type_traits>
#include <vector>

#include "internal.hpp"
#include "wide.hpp"

namespace eigsol {

int csr_upload(eigsol_ctx* ctx, int dtype, int64_t nrows, int64_t ncols, int64_t nnz, const int32_t* rowptr,
               const int32_t* colidx, const void* values, eigsol_csr** out, int64_t xoff);
struct ShiftFactor;
int shift_factor_csr(eigsol_csr* A, const void* sigma, ShiftFactor** out);
int shift_factor_dense(eigsol_dense* A, const void* sigma, ShiftFactor** out);
void shift_factor_free(ShiftFactor* f);
int shift_solve_launch(ShiftFactor* f, const void* b_dev, void* y_dev);
int shift_error(ShiftFactor* f);
void shift_info(const ShiftFactor* f, double* bytes, int32_t* variant, int32_t* tiles);

namespace wdev {

constexpr int kT = 256;          // threads of the vector / product kernels
constexpr int kMaxBlocks = 1024; // blocks of a reduction (partials summed on the host, in order)

__device__ __forceinline__ dd shfl_dd(dd v, int off) {
    return dd{__shfl_xor(v.hi, off, 64), __shfl_xor(v.lo, off, 64)};
}
// dd_add is commutative bit for bit (two_sum is exact either way), so the butterfly leaves the same
// sum in every lane
__device__ __forceinline__ dd wave_sum(dd v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = dd_add(v, shfl_dd(v, off));
    return v;
}
// N double-double sums over the block, in wave order; every thread gets the totals
template <int N>
__device__ __forceinline__ void block_sum(dd (&v)[N], dd* sm /* N * 16 */) {
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] = wave_sum(v[q]);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int q = 0; q < N; ++q) sm[q * 16 + w] = v[q];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < N; ++q) {
        dd s = sm[q * 16];
        for (int i = 1; i < nw; ++i) s = dd_add(s, sm[q * 16 + i]);
        v[q] = s;
    }
    __syncthreads();
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// y = b + sgn (A x - sig x): one row per lane, the row's entries in ascending column order
// (sig != 0 only for square A: the refinement residual of A - sigma I)
template <class T>
__global__ __launch_bounds__(kT) void spmv_kernel(int64_t nrows, const int32_t* __restrict__ rp,
                                                  const int32_t* __restrict__ ci, const T* __restrict__ val,
                                                  const T* __restrict__ x, const T* __restrict__ b, T sig, int sgn,
                                                  T* __restrict__ y) {
    using O = wide_ops<T>;
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= nrows) return;
    T s = O::zero();
    const int32_t e1 = rp[i + 1];
    for (int32_t e = rp[i]; e < e1; ++e) s = O::add(s, O::mul(val[e], x[ci[e]]));
    if (!O::is_zero(sig)) s = O::sub(s, O::mul(sig, x[i]));
    if (sgn < 0) s = O::sub(O::zero(), s);
    if (b) s = O::add(b[i], s);
    y[i] = s;
}

__device__ __forceinline__ cdd shfl_cdd(cdd v, int off) { return cdd{shfl_dd(v.re, off), shfl_dd(v.im, off)}; }
template <class T> __device__ __forceinline__ T shfl_w(T v, int off);
template <> __device__ __forceinline__ dd shfl_w<dd>(dd v, int off) { return shfl_dd(v, off); }
template <> __device__ __forceinline__ cdd shfl_w<cdd>(cdd v, int off) { return shfl_cdd(v, off); }

// One power iteration of the CSR session in one pass (power_method.hpp:78-81): z = A x as (A y) /
// normY (two double-double divisions per row instead of one per entry: a 1e-32-relative rounding
// difference from A (y / normY), far inside the x87 reference's own), A y by G lanes per row
// (entries strided over the group, a butterfly in fixed order), x = y / normY and z written by the
// row's first lane,
// and the block partials of {|z|^2, Re x^H z, Im x^H z} (rows in a fixed order per block; the host
// sums the blocks in order).  Replaces scale + one-row-per-lane product + dot pass: the vectors are
// read once and the matrix stream is coalesced across a group.
template <class T, int G>
__global__ __launch_bounds__(kT) void power_fused_kernel(int64_t n, const int32_t* __restrict__ rp,
                                                         const int32_t* __restrict__ ci, const T* __restrict__ val,
                                                         const T* __restrict__ y, dd nrm, T* __restrict__ x,
                                                         T* __restrict__ z, dd* __restrict__ part) {
    using O = wide_ops<T>;
    __shared__ dd sm[3 * 16];
    constexpr int RB = kT / G;   // rows per block tile
    const int g = threadIdx.x % G;
    dd acc[3] = {dd{0.0, 0.0}, dd{0.0, 0.0}, dd{0.0, 0.0}};
    for (int64_t base = (int64_t)blockIdx.x * RB; base < n; base += (int64_t)gridDim.x * RB) {
        const int64_t i = base + threadIdx.x / G;
        T sum = O::zero();
        if (i < n) {
            const int32_t e1 = rp[i + 1];
            for (int32_t e = rp[i] + g; e < e1; e += G) sum = O::add(sum, O::mul(val[e], y[ci[e]]));
        }
#pragma unroll
        for (int off = G / 2; off > 0; off >>= 1) sum = O::add(sum, shfl_w<T>(sum, off));
        if (i < n && g == 0) {
            const T xi = O::div_r(y[i], nrm);
            sum = O::div_r(sum, nrm);
            x[i] = xi;
            z[i] = sum;
            acc[0] = dd_add(acc[0], O::abs2(sum));
            const T pr = O::mul(O::conj(xi), sum);
            acc[1] = dd_add(acc[1], O::real(pr));
            acc[2] = dd_add(acc[2], O::imag(pr));
        }
    }
    block_sum<3>(acc, sm);
    if (threadIdx.x == 0)
        for (int q = 0; q < 3; ++q) part[3 * blockIdx.x + q] = acc[q];
}

// Two-phase variant (EIGSOL_DD_FUSED2, default): the per-row epilogue (two double-double divisions,
// |z|^2 and conj(x) z: most of a row's instructions) ran on one lane of every group of G, i.e. at
// 1 / G of the wave.  Here a block first forms the row sums of kT rows (G passes of kT / G rows, G
// lanes per row, the same strided order and butterfly) into LDS, then every thread finishes one row:
// the same x and z values, the partials summed per thread over its rows (a different order).
template <class T, int G>
__global__ __launch_bounds__(kT) void power_fused2_kernel(int64_t n, const int32_t* __restrict__ rp,
                                                          const int32_t* __restrict__ ci, const T* __restrict__ val,
                                                          const T* __restrict__ y, dd nrm, T* __restrict__ x,
                                                          T* __restrict__ z, dd* __restrict__ part) {
    using O = wide_ops<T>;
    __shared__ dd sm[3 * 16];
    __shared__ T srow[kT];
    constexpr int RB = kT / G;   // rows per pass
    const int g = threadIdx.x % G, r = threadIdx.x / G;
    dd acc[3] = {dd{0.0, 0.0}, dd{0.0, 0.0}, dd{0.0, 0.0}};
    for (int64_t base = (int64_t)blockIdx.x * kT; base < n; base += (int64_t)gridDim.x * kT) {
#pragma unroll
        for (int p = 0; p < G; ++p) {
            const int64_t i = base + p * RB + r;
            T sum = O::zero();
            if (i < n) {
                const int32_t e1 = rp[i + 1];
                for (int32_t e = rp[i] + g; e < e1; e += G) sum = O::add(sum, O::mul(val[e], y[ci[e]]));
            }
#pragma unroll
            for (int off = G / 2; off > 0; off >>= 1) sum = O::add(sum, shfl_w<T>(sum, off));
            if (g == 0) srow[p * RB + r] = sum;
        }
        __syncthreads();
        const int64_t i = base + threadIdx.x;
        if (i < n) {
            const T xi = O::div_r(y[i], nrm);
            const T zi = O::div_r(srow[threadIdx.x], nrm);
            x[i] = xi;
            z[i] = zi;
            acc[0] = dd_add(acc[0], O::abs2(zi));
            const T pr = O::mul(O::conj(xi), zi);
            acc[1] = dd_add(acc[1], O::real(pr));
            acc[2] = dd_add(acc[2], O::imag(pr));
        }
        __syncthreads();
    }
    block_sum<3>(acc, sm);
    if (threadIdx.x == 0)
        for (int q = 0; q < 3; ++q) part[3 * blockIdx.x + q] = acc[q];
}

// out[q] = sum of the nb block partials part[3 b + q] (thread t: blocks t, t + kT, ... in order, then
// the block sum in wave order): deterministic for a given nb
__global__ __launch_bounds__(kT) void sum3_kernel(const dd* __restrict__ part, int nb, dd* __restrict__ out) {
    __shared__ dd sm[3 * 16];
    dd v[3] = {dd{0.0, 0.0}, dd{0.0, 0.0}, dd{0.0, 0.0}};
    for (int b = threadIdx.x; b < nb; b += kT)
#pragma unroll
        for (int q = 0; q < 3; ++q) v[q] = dd_add(v[q], part[3 * b + q]);
    block_sum<3>(v, sm);
    if (threadIdx.x == 0)
        for (int q = 0; q < 3; ++q) out[q] = v[q];
}

// dense, column-major m x n: part[c * m + i] = sum over the columns of chunk c of A(i, j) x_j
template <class T>
__global__ __launch_bounds__(kT) void gemv_part_kernel(int64_t m, int64_t n, const T* __restrict__ A,
                                                       const T* __restrict__ x, int64_t cw, T* __restrict__ part) {
    using O = wide_ops<T>;
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    const int64_t c = blockIdx.y;
    if (i >= m) return;
    const int64_t j0 = c * cw, j1 = std::min<int64_t>(n, j0 + cw);
    T s = O::zero();
    for (int64_t j = j0; j < j1; ++j) s = O::add(s, O::mul(A[i + j * m], x[j]));
    part[c * m + i] = s;
}
template <class T>
__global__ __launch_bounds__(kT) void gemv_combine_kernel(int64_t m, int nch, const T* __restrict__ part,
                                                          const T* __restrict__ x, const T* __restrict__ b, T sig,
                                                          int sgn, T* __restrict__ y) {
    using O = wide_ops<T>;
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= m) return;
    T s = part[i];
    for (int c = 1; c < nch; ++c) s = O::add(s, part[(int64_t)c * m + i]);
    if (!O::is_zero(sig)) s = O::sub(s, O::mul(sig, x[i]));
    if (sgn < 0) s = O::sub(O::zero(), s);
    if (b) s = O::add(b[i], s);
    y[i] = s;
}

// per block: {sum |a_i|^2, Re sum conj(w_i) a_i, Im ...} (w == nullptr: the norm only)
template <class T>
__global__ __launch_bounds__(kT) void dot_kernel(int64_t n, const T* __restrict__ a, const T* __restrict__ w,
                                                 dd* __restrict__ part) {
    using O = wide_ops<T>;
    __shared__ dd sm[3 * 16];
    dd v[3] = {dd{0.0, 0.0}, dd{0.0, 0.0}, dd{0.0, 0.0}};
    for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT) {
        const T ai = a[i];
        v[0] = dd_add(v[0], O::abs2(ai));
        if (w) {
            const T p = O::mul(O::conj(w[i]), ai);
            v[1] = dd_add(v[1], O::real(p));
            v[2] = dd_add(v[2], O::imag(p));
        }
    }
    block_sum<3>(v, sm);
    if (threadIdx.x == 0)
        for (int q = 0; q < 3; ++q) part[3 * blockIdx.x + q] = v[q];
}

// x = y / nrm (x.normalize(), power_method.hpp:62; x = y / normY, :78)
template <class T>
__global__ __launch_bounds__(kT) void scale_kernel(int64_t n, const T* y, dd nrm, T* x) {   // may run in place
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (i < n) x[i] = wide_ops<T>::div_r(y[i], nrm);
}

// the residual rounded to fp64 (hi parts: the nearest double of a normalised double-double)
template <class T>
__global__ __launch_bounds__(kT) void round_kernel(int64_t n, const T* __restrict__ r, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    if constexpr (wide_ops<T>::complex) {
        out[2 * i] = r[i].re.hi;
        out[2 * i + 1] = r[i].im.hi;
    } else {
        out[i] = r[i].hi;
    }
}
// matrix entries rounded to fp64 (the shadow matrix the fp64 factor is built from)
template <class T>
__global__ __launch_bounds__(kT) void hi_kernel(int64_t cnt, const T* __restrict__ a, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= cnt) return;
    if constexpr (wide_ops<T>::complex) {
        out[2 * i] = a[i].re.hi;
        out[2 * i + 1] = a[i].im.hi;
    } else {
        out[i] = a[i].hi;
    }
}

// y += sgn d (d an fp64 correction); per block {sum |d|^2, sum |y|^2} in double (magnitudes only)
template <class T>
__global__ __launch_bounds__(kT) void accum_kernel(int64_t n, T* __restrict__ y, const double* __restrict__ d,
                                                   double sgn, double* __restrict__ part) {
    __shared__ double sm[2 * 4];
    double nd = 0.0, ny = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT) {
        if constexpr (wide_ops<T>::complex) {
            const double dr = sgn * d[2 * i], di = sgn * d[2 * i + 1];
            cdd v = y[i];
            v.re = dd_add_d(v.re, dr);
            v.im = dd_add_d(v.im, di);
            y[i] = v;
            nd += dr * dr + di * di;
            ny += v.re.hi * v.re.hi + v.im.hi * v.im.hi;
        } else {
            const double di = sgn * d[i];
            const dd v = dd_add_d(y[i], di);
            y[i] = v;
            nd += di * di;
            ny += v.hi * v.hi;
        }
    }
    nd = wave_sum_d(nd);
    ny = wave_sum_d(ny);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sm[w] = nd; sm[4 + w] = ny; }
    __syncthreads();
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = sm[0] + sm[1] + sm[2] + sm[3];
        part[2 * blockIdx.x + 1] = sm[4] + sm[5] + sm[6] + sm[7];
    }
}

// ------------------------------------------------------------------ Householder (QR method)
// reflector of x = A(r0 : r0+m, col) (to_hessenberg.hpp:42-66, qr_decompose.hpp:51-74):
// skip when ||x(1:)|| == 0 or ||v|| == 0; alpha = -sign ||x||, sign = x0 / |x0| (1 for x0 == 0),
// v = (x - alpha e1) / ||x - alpha e1||.  The column is scaled by the power of two 2^-e that brings
// its largest entry to [1, 2) before any square is formed (exact, so inside the double range the
// reflector is bitwise the unscaled one); v is scale-free, so entries near 1e+-170, whose squares
// leave the double range but not the x87 long double's, still give the reference's reflector.
template <class T>
__global__ __launch_bounds__(1024) void hh_make_kernel(const T* A, int64_t ld, int64_t r0, int64_t col, int64_t m,
                                                       T* v, int* skip) {
    using O = wide_ops<T>;
    __shared__ dd sm[16];
    const T* x = A + r0 + col * ld;
    double mx = 0.0;
    for (int64_t i = threadIdx.x; i < m; i += blockDim.x) mx = fmax(mx, O::maxabs(x[i]));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off, 64));
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6].hi = mx;
    __syncthreads();
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) mx = fmax(mx, sm[w].hi);
    __syncthreads();
    const int e = (mx > 0.0 && mx <= 1.7976931348623157e308) ? ilogb(mx) : 0;
    dd t[1] = {dd{0.0, 0.0}};
    for (int64_t i = 1 + threadIdx.x; i < m; i += blockDim.x) t[0] = dd_add(t[0], O::abs2(O::ldexp(x[i], -e)));
    block_sum<1>(t, sm);
    const dd tail = t[0];
    if (tail.hi == 0.0) {
        if (threadIdx.x == 0) *skip = 1;
        return;
    }
    const T x0 = O::ldexp(x[0], -e);
    const dd nx = dd_sqrt(dd_add(tail, O::abs2(x0)));
    const T sign = O::is_zero(x0) ? O::one() : O::div_r(x0, O::abs(x0));
    const T v0 = O::add(x0, O::mul_r(sign, nx));   // x0 - alpha
    const dd vn = dd_sqrt(dd_add(tail, O::abs2(v0)));
    if (vn.hi == 0.0) {
        if (threadIdx.x == 0) *skip = 1;
        return;
    }
    for (int64_t i = threadIdx.x; i < m; i += blockDim.x) v[i] = O::div_r(i == 0 ? v0 : O::ldexp(x[i], -e), vn);
    if (threadIdx.x == 0) *skip = 0;
}

// B = A(r0 : r0+m, c0 : ...): B(:, j) -= 2 v (v^H B(:, j)), one block per column
template <class T>
__global__ __launch_bounds__(kT) void hh_left_kernel(T* A, int64_t ld, int64_t r0, int64_t m, int64_t c0, const T* v,
                                                     const int* skip) {
    using O = wide_ops<T>;
    if (*skip) return;
    __shared__ dd sm[2 * 16];
    T* b = A + r0 + (c0 + blockIdx.x) * ld;
    T w = O::zero();
    for (int64_t i = threadIdx.x; i < m; i += kT) w = O::add(w, O::mul(O::conj(v[i]), b[i]));
    dd s[2] = {O::real(w), O::imag(w)};
    block_sum<2>(s, sm);
    const T w2 = O::mul_r(O::make(s[0], s[1]), dd{2.0, 0.0});
    for (int64_t i = threadIdx.x; i < m; i += kT) b[i] = O::sub(b[i], O::mul(v[i], w2));
}

// B = A(0 : nr, c0 : c0+m): B(i, :) -= 2 (B(i, :) v) v^H, 16 rows per block, 16 lanes per row
template <class T>
__global__ __launch_bounds__(kT) void hh_right_kernel(T* A, int64_t ld, int64_t nr, int64_t c0, int64_t m, const T* v,
                                                      const int* skip) {
    using O = wide_ops<T>;
    if (*skip) return;
    const int lane = threadIdx.x & 15;
    const int64_t i = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
    const bool live = i < nr;
    T* row = A + (live ? i : 0) + c0 * ld;
    T w = O::zero();
    if (live)
        for (int64_t j = lane; j < m; j += 16) w = O::add(w, O::mul(row[j * ld], v[j]));
    dd re = O::real(w), im = O::imag(w);
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) {
        re = dd_add(re, shfl_dd(re, off));
        im = dd_add(im, shfl_dd(im, off));
    }
    const T w2 = O::mul_r(O::make(re, im), dd{2.0, 0.0});
    if (live)
        for (int64_t j = lane; j < m; j += 16) row[j * ld] = O::sub(row[j * ld], O::mul(w2, O::conj(v[j])));
}

template <class T>
__global__ void set_identity_kernel(T* A, int64_t n) {
    const int64_t idx = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (idx >= n * n) return;
    A[idx] = (idx % n == idx / n) ? wide_ops<T>::one() : wide_ops<T>::zero();
}

// C = A B (n x n, column-major), 16 x 16 output tile per block, k in steps of 16 through LDS
template <class T>
__global__ __launch_bounds__(kT) void gemm_nn_kernel(const T* A, const T* B, T* C, int64_t n) {
    using O = wide_ops<T>;
    __shared__ T As[16][17];
    __shared__ T Bs[16][17];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int64_t i = (int64_t)blockIdx.x * 16 + tx, j = (int64_t)blockIdx.y * 16 + ty;
    T acc = O::zero();
    for (int64_t k0 = 0; k0 < n; k0 += 16) {
        const int64_t ka = k0 + ty, kb = k0 + tx;
        As[ty][tx] = (i < n && ka < n) ? A[i + ka * n] : O::zero();          // As[k][i]
        Bs[ty][tx] = (kb < n && j < n) ? B[kb + j * n] : O::zero();          // Bs[j][k]
        __syncthreads();
#pragma unroll 4
        for (int kk = 0; kk < 16; ++kk) acc = O::add(acc, O::mul(As[kk][tx], Bs[ty][kk]));
        __syncthreads();
    }
    if (i < n && j < n) C[i + j * n] = acc;
}

// max_i |H(i, i-1)| and ||H||_F^2 (qr_eigenvalues.hpp:79-88), one block
template <class T>
__global__ __launch_bounds__(kT) void subdiag_frob_kernel(const T* H, int64_t n, dd* out) {
    using O = wide_ops<T>;
    __shared__ dd sm[16];
    __shared__ dd smx[kT];
    dd f[1] = {dd{0.0, 0.0}};
    dd mx{0.0, 0.0};
    for (int64_t idx = threadIdx.x; idx < n * n; idx += kT) {
        const T h = H[idx];
        f[0] = dd_add(f[0], O::abs2(h));
        const int64_t i = idx % n, j = idx / n;
        if (i == j + 1) {
            const dd a = O::abs(h);
            if (dd_le(mx, a)) mx = a;
        }
    }
    block_sum<1>(f, sm);
    smx[threadIdx.x] = mx;
    __syncthreads();
    for (int off = kT / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off && dd_le(smx[threadIdx.x], smx[threadIdx.x + off]))
            smx[threadIdx.x] = smx[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = smx[0];
        out[1] = f[0];
    }
}

template <class T>
__global__ void diag_kernel(const T* H, int64_t n, T* d) {
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (i < n) d[i] = H[i + i * n];
}

}  // namespace wdev

// ====================================================================================== host
namespace {

template <class T>
using W = wide_ops<T>;

inline unsigned nblk(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + wdev::kT - 1) / wdev::kT); }
inline unsigned rgrid(int64_t n) { return (unsigned)std::min<int64_t>(wdev::kMaxBlocks, nblk(n)); }

// host scalars are kept as cdd (real: im = 0); the device scalar of type T from one
template <class T> inline T from_c(const cdd& a);
template <> inline dd from_c<dd>(const cdd& a) { return a.re; }
template <> inline cdd from_c<cdd>(const cdd& a) { return a; }

template <class F>
int by_wide(int dtype, F&& fn) {
    if (dtype == EIGSOL_CDD) return fn(cdd{});
    return fn(dd{});
}

// tolerance.hpp:28-33 for the long double instantiation: |a - b| and 1 + |a| in extended
// precision, each converted to double, compared in double
inline bool close_rel(const cdd& a, const cdd& b, double tol) {
    const double diff = dd_to_d(cdd_abs(cdd_sub(a, b)));
    const double scale = dd_to_d(dd_add_d(cdd_abs(a), 1.0));
    return diff <= tol * scale;
}

}  // namespace

// ---------------------------------------------------------------- matrices
// Plain CSR of double-double values, columns ascending inside every row (the reference's CSC
// scatter sums a row in ascending column order, power_method.hpp:69)
int wide_csr_upload(eigsol_ctx* ctx, int dtype, int64_t nrows, int64_t ncols, int64_t nnz, const int32_t* rowptr,
                    const int32_t* colidx, const void* values, eigsol_csr** out) {
    const size_t sb = scalar_bytes(dtype);
    std::vector<int32_t> cs(colidx, colidx + nnz);
    std::vector<unsigned char> vs((const unsigned char*)values, (const unsigned char*)values + (size_t)nnz * sb);
    std::vector<int32_t> perm;
    for (int64_t i = 0; i < nrows; ++i) {
        const int32_t b = rowptr[i], e = rowptr[i + 1];
        bool sorted = true;
        for (int32_t k = b + 1; k < e && sorted; ++k) sorted = colidx[k] >= colidx[k - 1];
        if (sorted) continue;
        perm.resize(e - b);
        std::iota(perm.begin(), perm.end(), b);
        std::stable_sort(perm.begin(), perm.end(), [&](int32_t x, int32_t y) { return colidx[x] < colidx[y]; });
        for (int32_t k = b; k < e; ++k) {
            cs[k] = colidx[perm[k - b]];
            std::memcpy(&vs[(size_t)k * sb], (const unsigned char*)values + (size_t)perm[k - b] * sb, sb);
        }
    }
    auto* A = new eigsol_csr();
    A->ctx = ctx;
    ctx_retain(ctx);
    A->dtype = dtype;
    A->nrows = nrows;
    A->ncols = ncols;
    A->nnz = nnz;
    hipStream_t s = ctx->stream;
    hipError_t e;
    if ((e = hipMalloc(&A->rowptr, (nrows + 1) * sizeof(int32_t))) != hipSuccess ||
        (e = hipMalloc(&A->col, std::max<int64_t>(nnz, 1) * sizeof(int32_t))) != hipSuccess ||
        (e = hipMalloc(&A->val, std::max<int64_t>(nnz, 1) * sb)) != hipSuccess ||
        (e = hipMemcpyAsync(A->rowptr, rowptr, (nrows + 1) * sizeof(int32_t), hipMemcpyHostToDevice, s)) != hipSuccess ||
        (nnz && (e = hipMemcpyAsync(A->col, cs.data(), nnz * sizeof(int32_t), hipMemcpyHostToDevice, s)) != hipSuccess) ||
        (nnz && (e = hipMemcpyAsync(A->val, vs.data(), nnz * sb, hipMemcpyHostToDevice, s)) != hipSuccess) ||
        (e = hipStreamSynchronize(s)) != hipSuccess) {
        csr_release(A);
        return fail(EIGSOL_E_HIP, std::string("eigsol_csr_create (double-double): ") + hipGetErrorString(e));
    }
    *out = A;
    return EIGSOL_OK;
}

// y = b + sgn ((A - sig I) x) on device buffers
template <class T>
static int csr_apply(eigsol_csr* A, const void* x, void* y, const void* b, T sig, int sgn) {
    if (A->nrows == 0) return EIGSOL_OK;
    hipLaunchKernelGGL((wdev::spmv_kernel<T>), dim3(nblk(A->nrows)), dim3(wdev::kT), 0, A->ctx->stream, A->nrows,
                       A->rowptr, A->col, static_cast<const T*>(A->val), static_cast<const T*>(x),
                       static_cast<const T*>(b), sig, sgn, static_cast<T*>(y));
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

template <class T>
static int dense_apply(eigsol_dense* A, const void* x, void* y, const void* b, T sig, int sgn) {
    const int64_t m = A->nrows, n = A->ncols;
    if (m == 0) return EIGSOL_OK;
    if (!A->ypart) {
        // ~2048 blocks over row tiles x column chunks of >= 16 columns
        const int64_t rt = (m + wdev::kT - 1) / wdev::kT;
        int64_t nch = std::max<int64_t>(1, 2048 / rt);
        nch = std::min<int64_t>(nch, std::max<int64_t>(1, (n + 15) / 16));
        A->nchunk = (int)nch;
        A->cw = (int)std::max<int64_t>(1, (n + nch - 1) / nch);
        EIGSOL_HIP(hipMalloc(&A->ypart, (size_t)nch * (size_t)m * sizeof(T)));
    }
    hipStream_t st = A->ctx->stream;
    hipLaunchKernelGGL((wdev::gemv_part_kernel<T>), dim3(nblk(m), A->nchunk), dim3(wdev::kT), 0, st, m, n,
                       static_cast<const T*>(A->a), static_cast<const T*>(x), (int64_t)A->cw,
                       static_cast<T*>(A->ypart));
    hipLaunchKernelGGL((wdev::gemv_combine_kernel<T>), dim3(nblk(m)), dim3(wdev::kT), 0, st, m, A->nchunk,
                       static_cast<const T*>(A->ypart), static_cast<const T*>(x), static_cast<const T*>(b), sig, sgn,
                       static_cast<T*>(y));
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

int wide_csr_spmv(eigsol_csr* A, const void* x, void* y) {
    return by_wide(A->dtype, [&](auto tag) {
        using T = decltype(tag);
        return csr_apply<T>(A, x, y, nullptr, W<T>::zero(), 1);
    });
}
int wide_dense_gemv(eigsol_dense* A, const void* x, void* y) {
    return by_wide(A->dtype, [&](auto tag) {
        using T = decltype(tag);
        return dense_apply<T>(A, x, y, nullptr, W<T>::zero(), 1);
    });
}

// fp64 shadows (the matrix rounded to double) for the shifted solves' factor
static int csr_shadow(eigsol_csr* A) {
    if (A->shadow) return EIGSOL_OK;
    hipStream_t st = A->ctx->stream;
    const bool cx = A->dtype == EIGSOL_CDD;
    const int64_t n = A->nrows, nnz = A->nnz;
    std::vector<int32_t> rp(n + 1), ci(std::max<int64_t>(nnz, 1));
    std::vector<double> hv(std::max<int64_t>(nnz, 1) * (cx ? 2 : 1));
    double* dv = nullptr;
    EIGSOL_HIP(hipMalloc(&dv, hv.size() * sizeof(double)));
    int rc = EIGSOL_OK;
    if (nnz) {
        if (cx)
            hipLaunchKernelGGL((wdev::hi_kernel<cdd>), dim3(nblk(nnz)), dim3(wdev::kT), 0, st, nnz,
                               static_cast<const cdd*>(A->val), dv);
        else
            hipLaunchKernelGGL((wdev::hi_kernel<dd>), dim3(nblk(nnz)), dim3(wdev::kT), 0, st, nnz,
                               static_cast<const dd*>(A->val), dv);
    }
    if (hipMemcpyAsync(rp.data(), A->rowptr, (n + 1) * sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
        (nnz && hipMemcpyAsync(ci.data(), A->col, nnz * sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess) ||
        (nnz && hipMemcpyAsync(hv.data(), dv, hv.size() * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess) ||
        stream_wait(st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "double-double matrix: fp64 shadow download");
    (void)hipFree(dv);
    EIGSOL_TRY(rc);
    return csr_upload(A->ctx, cx ? EIGSOL_C128 : EIGSOL_F64, n, A->ncols, nnz, rp.data(), ci.data(), hv.data(),
                      &A->shadow, 0);
}

static int dense_shadow(eigsol_dense* A) {
    if (A->shadow) return EIGSOL_OK;
    const bool cx = A->dtype == EIGSOL_CDD;
    const int64_t cnt = A->nrows * A->ncols;
    auto* B = new eigsol_dense();
    B->ctx = A->ctx;
    ctx_retain(B->ctx);
    B->dtype = cx ? EIGSOL_C128 : EIGSOL_F64;
    B->nrows = A->nrows;
    B->ncols = A->ncols;
    if (hipMalloc(&B->a, (size_t)std::max<int64_t>(cnt, 1) * (cx ? 16 : 8) + 64) != hipSuccess) {
        dense_release(B);
        return fail(EIGSOL_E_HIP, "double-double matrix: fp64 shadow allocation");
    }
    hipStream_t st = A->ctx->stream;
    if (cnt) {
        if (cx)
            hipLaunchKernelGGL((wdev::hi_kernel<cdd>), dim3(nblk(cnt)), dim3(wdev::kT), 0, st, cnt,
                               static_cast<const cdd*>(A->a), static_cast<double*>(B->a));
        else
            hipLaunchKernelGGL((wdev::hi_kernel<dd>), dim3(nblk(cnt)), dim3(wdev::kT), 0, st, cnt,
                               static_cast<const dd*>(A->a), static_cast<double*>(B->a));
    }
    if (hipGetLastError() != hipSuccess || stream_wait(st) != hipSuccess) {
        dense_release(B);
        return fail(EIGSOL_E_HIP, "double-double matrix: fp64 shadow");
    }
    A->shadow = B;
    return EIGSOL_OK;
}

// ---------------------------------------------------------------- the iteration (power / shifted)
struct WideSession {
    eigsol_ctx* ctx = nullptr;
    eigsol_csr* csr = nullptr;
    eigsol_dense* dense = nullptr;
    int dtype = EIGSOL_DD;
    int64_t n = 0;
    size_t sb = 16;
    bool shifted = false;
    ShiftFactor* f = nullptr;
    cdd sig{};
    void* x = nullptr;      // current iterate x_k (normalised)
    void* y = nullptr;      // pending y = A x_k (power) / the solve (shifted)
    void* z = nullptr;      // A x for the Rayleigh quotient
    void* r = nullptr;      // refinement residual
    double* r64 = nullptr;  // residual rounded to fp64
    double* d64 = nullptr;  // fp64 correction
    dd* part = nullptr;     // reduction partials (3 per block)
    dd* fpart = nullptr;    // power_fused_kernel's block partials and their sum
    double* dpart = nullptr;
    dd* hpart = nullptr;       // pinned host copies of part / dpart (a pageable copy sleeps ~1 ms)
    double* hdpart = nullptr;
    // reference loop state (power_method.hpp:60-96 / shifted_inverse_power_solver.hpp:36-76)
    eigsol_solver_options opts{1000, 1e-10};
    bool begun = false, done = false, converged = false, initialized = false;
    int32_t k = 0, iters = 0;
    cdd lambda{};
    dd pend_n2{};           // ||y||^2 of the pending product (power)
    std::vector<cdd> trace;
    int32_t trace_cap = 0;
    // accounting of the last solve / iteration
    int32_t refine_steps = 0;
    double solve_bytes = 0.0;
};

void wide_session_free(WideSession* s) {
    if (!s) return;
    hipSetDevice(s->ctx->device);
    hipStreamSynchronize(s->ctx->stream);
    for (void* p : {s->x, s->y, s->z, s->r, (void*)s->r64, (void*)s->d64, (void*)s->part, (void*)s->dpart, (void*)s->fpart})
        if (p) hipFree(p);
    for (void* p : {(void*)s->hpart, (void*)s->hdpart})
        if (p) hipHostFree(p);
    if (s->f) shift_factor_free(s->f);
    if (s->csr) csr_release(s->csr);
    if (s->dense) dense_release(s->dense);
    ctx_release(s->ctx);
    delete s;
}

template <class T>
static int apply(WideSession* s, const void* x, void* y, const void* b, T sig, int sgn) {
    return s->csr ? csr_apply<T>(s->csr, x, y, b, sig, sgn) : dense_apply<T>(s->dense, x, y, b, sig, sgn);
}

// {||a||^2, w^H a} in double-double, partials of the blocks summed on the host in block order
template <class T>
static int reduce(WideSession* s, const void* a, const void* w, dd& n2, cdd& dot) {
    const unsigned g = rgrid(s->n);
    hipStream_t st = s->ctx->stream;
    hipLaunchKernelGGL((wdev::dot_kernel<T>), dim3(g), dim3(wdev::kT), 0, st, s->n, static_cast<const T*>(a),
                       static_cast<const T*>(w), s->part);
    EIGSOL_HIP(hipGetLastError());
    EIGSOL_HIP(hipMemcpyAsync(s->hpart, s->part, 3 * g * sizeof(dd), hipMemcpyDeviceToHost, st));
    EIGSOL_HIP(stream_wait(st));
    n2 = dd{0.0, 0.0};
    dot = cdd{};
    for (unsigned b = 0; b < g; ++b) {
        n2 = dd_add(n2, s->hpart[3 * b]);
        dot.re = dd_add(dot.re, s->hpart[3 * b + 1]);
        dot.im = dd_add(dot.im, s->hpart[3 * b + 2]);
    }
    return EIGSOL_OK;
}

// x = y / normY, z = A x, {||z||^2, x^H z}: one launch, lanes per row from the mean row length
// (one block per kT / G rows up to kFusedBlocks, so every CU keeps many rows' dependent loads in
// flight; the block partials are reduced on the device in a fixed order and three values come back)
constexpr int kFusedBlocks = 16384;   // cap of EIGSOL_DD_BLOCKS (default 2048: 1024 / 2048 / 4096 blocks 0.151 / 0.142 / 0.144 ms, band 1M)
template <class T>
static int power_fused(WideSession* s, dd nrm, dd& n2, cdd& dot) {
    hipStream_t st = s->ctx->stream;
    eigsol_csr* A = s->csr;
    const double avg = s->n ? (double)A->nnz / (double)s->n : 0.0;
    if (!s->fpart) EIGSOL_HIP(hipMalloc(&s->fpart, (3 * (size_t)kFusedBlocks + 3) * sizeof(dd)));
    static const bool two = [] {
        const char* e = std::getenv("EIGSOL_DD_FUSED2");
        return !(e && std::atoi(e) == 0);
    }();
    unsigned g = 1;
    auto go = [&](auto gtag) {
        constexpr int G = decltype(gtag)::value;
        static const int64_t cap = [] {
            const char* e = std::getenv("EIGSOL_DD_BLOCKS");
            return e ? std::max<int64_t>(1, std::min<int64_t>(kFusedBlocks, std::atoll(e))) : (int64_t)2048;
        }();
        // EIGSOL_DD_FUSED2=0: the one-phase kernel (the row epilogue on one lane of G)
        const int64_t rows = two ? wdev::kT : wdev::kT / G;   // rows per block tile
        g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cap, (s->n + rows - 1) / rows));
        if (two)
            hipLaunchKernelGGL((wdev::power_fused2_kernel<T, G>), dim3(g), dim3(wdev::kT), 0, st, s->n, A->rowptr,
                               A->col, static_cast<const T*>(A->val), static_cast<const T*>(s->y), nrm,
                               static_cast<T*>(s->x), static_cast<T*>(s->z), s->fpart);
        else
            hipLaunchKernelGGL((wdev::power_fused_kernel<T, G>), dim3(g), dim3(wdev::kT), 0, st, s->n, A->rowptr,
                               A->col, static_cast<const T*>(A->val), static_cast<const T*>(s->y), nrm,
                               static_cast<T*>(s->x), static_cast<T*>(s->z), s->fpart);
    };
    static const int force_g = [] {   // EIGSOL_DD_G: lanes per row (2 / 4 / 8 / 16 / 32), A/B only
        const char* e = std::getenv("EIGSOL_DD_G");
        return e ? std::atoi(e) : 0;
    }();
    // lanes per row from the mean row length.  Two-phase kernel (round 6, tools/r06_dd_power_prof.py,
    // band matrices of 1M rows): 4 entries per row G = 2 / 4: 0.057 / 0.059 ms; 10: G = 2 / 4 / 8
    // 0.137 / 0.080 / 0.091 ms; 32: G = 4 / 8 / 16 0.228 / 0.178 / 0.197 ms; 64: G = 8 / 16 / 32
    // 0.300 / 0.304 / 0.421 ms (profiles/r06_dd_power_ab.log)
    const double lim[4] = {two ? 5.0 : 0.0, two ? 20.0 : 6.0, two ? 48.0 : 12.0, two ? 96.0 : 24.0};
    if (force_g == 2 || (!force_g && avg <= lim[0])) go(std::integral_constant<int, 2>{});
    else if (force_g == 4 || (!force_g && avg <= lim[1])) go(std::integral_constant<int, 4>{});
    else if (force_g == 8 || (!force_g && avg <= lim[2])) go(std::integral_constant<int, 8>{});
    else if (force_g == 16 || (!force_g && avg <= lim[3])) go(std::integral_constant<int, 16>{});
    else go(std::integral_constant<int, 32>{});
    EIGSOL_HIP(hipGetLastError());
    hipLaunchKernelGGL(wdev::sum3_kernel, dim3(1), dim3(wdev::kT), 0, st, s->fpart, (int)g,
                       s->fpart + 3 * (size_t)kFusedBlocks);
    EIGSOL_HIP(hipGetLastError());
    EIGSOL_HIP(hipMemcpyAsync(s->hpart, s->fpart + 3 * (size_t)kFusedBlocks, 3 * sizeof(dd), hipMemcpyDeviceToHost, st));
    EIGSOL_HIP(stream_wait(st));
    n2 = s->hpart[0];
    dot = cdd{s->hpart[1], s->hpart[2]};
    return EIGSOL_OK;
}

// y = (A - sigma I)^{-1} b to double-double accuracy: fp64 solves of the rounded residual,
// corrections accumulated in double-double, residual b - (A - sigma I) y in double-double
template <class T>
static int refine_solve(WideSession* s, const void* b, void* y) {
    hipStream_t st = s->ctx->stream;
    const int64_t n = s->n;
    const T sig = from_c<T>(s->sig);
    EIGSOL_HIP(hipMemsetAsync(y, 0, n * sizeof(T), st));
    EIGSOL_HIP(hipMemcpyAsync(s->r, b, n * sizeof(T), hipMemcpyDeviceToDevice, st));
    constexpr int kMaxSteps = 30;
    const unsigned g = rgrid(n);
    double prev = std::numeric_limits<double>::infinity();
    double fbytes = 0.0;
    shift_info(s->f, &fbytes, nullptr, nullptr);
    const double nnz = s->csr ? (double)s->csr->nnz : (double)n * (double)n;
    const double rbytes = (sizeof(T) + (s->csr ? 4.0 : 0.0)) * nnz + 3.0 * sizeof(T) * n;
    s->refine_steps = 0;
    s->solve_bytes = 0.0;
    for (int it = 0; it < kMaxSteps; ++it) {
        hipLaunchKernelGGL((wdev::round_kernel<T>), dim3(nblk(n)), dim3(wdev::kT), 0, st, n,
                           static_cast<const T*>(s->r), s->r64);
        EIGSOL_HIP(hipGetLastError());
        EIGSOL_TRY(shift_solve_launch(s->f, s->r64, s->d64));
        hipLaunchKernelGGL((wdev::accum_kernel<T>), dim3(g), dim3(wdev::kT), 0, st, n, static_cast<T*>(y), s->d64,
                           1.0, s->dpart);
        EIGSOL_HIP(hipGetLastError());
        EIGSOL_HIP(hipMemcpyAsync(s->hdpart, s->dpart, 2 * g * sizeof(double), hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(stream_wait(st));
        ++s->refine_steps;
        s->solve_bytes += fbytes + rbytes;
        double nd = 0.0, ny = 0.0;
        for (unsigned q = 0; q < g; ++q) { nd += s->hdpart[2 * q]; ny += s->hdpart[2 * q + 1]; }
        nd = std::sqrt(nd);
        ny = std::sqrt(ny);
        if (!std::isfinite(nd) || !std::isfinite(ny))
            return fail(EIGSOL_E_SOLVER, "solve_shifted (double-double): the fp64 factor produced a non-finite correction");
        if (nd == 0.0 || nd <= std::ldexp(ny, -100)) break;   // at the double-double floor
        if (it >= 1 && nd >= prev) {
            // not contracting (A - sigma I singular to double precision): undo the step, keep the best iterate
            hipLaunchKernelGGL((wdev::accum_kernel<T>), dim3(g), dim3(wdev::kT), 0, st, n, static_cast<T*>(y), s->d64,
                               -1.0, s->dpart);
            EIGSOL_HIP(hipGetLastError());
            break;
        }
        if (it >= 1 && nd > 0.5 * prev) break;   // stagnating: the attainable accuracy is reached
        prev = nd;
        EIGSOL_TRY(apply<T>(s, y, s->r, b, sig, -1));   // r = b - (A - sigma I) y
    }
    return shift_error(s->f);
}

int wide_session_create(eigsol_ctx* ctx, eigsol_csr* csr, eigsol_dense* dense, const void* sigma, int32_t trace_cap,
                        WideSession** out) {
    auto* s = new WideSession();
    s->ctx = ctx;
    ctx_retain(ctx);
    s->dtype = csr ? csr->dtype : dense->dtype;
    s->n = csr ? csr->nrows : dense->nrows;
    s->sb = scalar_bytes(s->dtype);
    s->trace_cap = std::max(0, trace_cap);
    if (csr) { s->csr = csr; csr_retain(csr); }
    else { s->dense = dense; dense_retain(dense); }
    int rc = EIGSOL_OK;
    if (sigma) {
        s->shifted = true;
        std::memcpy(&s->sig, sigma, s->sb);   // dd: re only (the rest of s->sig stays zero)
        const double sh[2] = {s->sig.re.hi, s->dtype == EIGSOL_CDD ? s->sig.im.hi : 0.0};
        rc = csr ? csr_shadow(csr) : dense_shadow(dense);
        if (rc == EIGSOL_OK) rc = csr ? shift_factor_csr(csr->shadow, sh, &s->f) : shift_factor_dense(dense->shadow, sh, &s->f);
    }
    const size_t vb = (size_t)std::max<int64_t>(s->n, 1) * s->sb;
    const unsigned g = rgrid(s->n);
    if (rc == EIGSOL_OK &&
        (hipMalloc(&s->x, vb) != hipSuccess || hipMalloc(&s->y, vb) != hipSuccess || hipMalloc(&s->z, vb) != hipSuccess ||
         hipMalloc(&s->part, 3 * g * sizeof(dd)) != hipSuccess ||
         hipHostMalloc(&s->hpart, 3 * g * sizeof(dd), hipHostMallocDefault) != hipSuccess ||
         hipHostMalloc(&s->hdpart, 2 * g * sizeof(double), hipHostMallocDefault) != hipSuccess ||
         (s->shifted && (hipMalloc(&s->r, vb) != hipSuccess ||
                         hipMalloc(&s->r64, (size_t)std::max<int64_t>(s->n, 1) * (s->dtype == EIGSOL_CDD ? 16 : 8)) != hipSuccess ||
                         hipMalloc(&s->d64, (size_t)std::max<int64_t>(s->n, 1) * (s->dtype == EIGSOL_CDD ? 16 : 8)) != hipSuccess ||
                         hipMalloc(&s->dpart, 2 * g * sizeof(double)) != hipSuccess))))
        rc = fail(EIGSOL_E_HIP, "double-double session: hipMalloc");
    if (rc != EIGSOL_OK) { wide_session_free(s); return rc; }
    *out = s;
    return EIGSOL_OK;
}

template <class T>
static int begin_t(WideSession* s, const eigsol_solver_options* opts, const void* x0, int on_dev) {
    hipStream_t st = s->ctx->stream;
    s->opts = *opts;
    EIGSOL_HIP(hipMemcpyAsync(s->x, x0, s->n * sizeof(T), on_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
    dd n2;
    cdd dummy;
    EIGSOL_TRY(reduce<T>(s, s->x, nullptr, n2, dummy));
    const dd nx = dd_sqrt(n2);
    if (nx.hi > 0.0)   // x.normalize() (Eigen leaves a zero vector unchanged)
        hipLaunchKernelGGL((wdev::scale_kernel<T>), dim3(nblk(s->n)), dim3(wdev::kT), 0, st, s->n,
                           static_cast<const T*>(s->x), nx, static_cast<T*>(s->x));
    s->k = 0;
    s->iters = 0;
    s->lambda = cdd{};
    s->initialized = false;
    s->converged = false;
    s->trace.clear();
    s->done = opts->max_iterations <= 0;
    if (!s->done && !s->shifted) {   // the first product y = A x_0 (power_method.hpp:69)
        EIGSOL_TRY(apply<T>(s, s->x, s->y, nullptr, W<T>::zero(), 1));
        EIGSOL_TRY(reduce<T>(s, s->y, nullptr, s->pend_n2, dummy));
    }
    EIGSOL_HIP(stream_wait(st));
    s->begun = true;
    return EIGSOL_OK;
}

// one reference iteration k (power_method.hpp:68-96 / shifted_inverse_power_solver.hpp:48-76)
template <class T>
static int iterate_t(WideSession* s) {
    hipStream_t st = s->ctx->stream;
    dd n2;
    cdd dummy;
    if (s->shifted) {
        EIGSOL_TRY(refine_solve<T>(s, s->x, s->y));   // y = solve_shifted(A, shift, x)   :51
        EIGSOL_TRY(reduce<T>(s, s->y, nullptr, n2, dummy));
    } else {
        n2 = s->pend_n2;                               // y = A x                          :69
    }
    const dd normY = dd_sqrt(n2);
    if (normY.hi == 0.0) {                             // :73-76 / :54-57
        s->iters = s->k + 1;
        s->done = true;
        return EIGSOL_OK;
    }
    dd nz;
    cdd dot;
    if (s->csr && !s->shifted) {
        // x = y / normY, A x and x.dot(A x) in one pass (power_fused_kernel)
        EIGSOL_TRY(power_fused<T>(s, normY, nz, dot));
    } else {
        hipLaunchKernelGGL((wdev::scale_kernel<T>), dim3(nblk(s->n)), dim3(wdev::kT), 0, st, s->n,
                           static_cast<const T*>(s->y), normY, static_cast<T*>(s->x));   // x = y / normY
        EIGSOL_TRY(apply<T>(s, s->x, s->z, nullptr, W<T>::zero(), 1));                  // A x
        EIGSOL_TRY(reduce<T>(s, s->z, s->x, nz, dot));                                    // x.dot(A x)
    }
    const cdd lam = W<T>::complex ? dot : cdd{dot.re, dd{0.0, 0.0}};
    if ((int32_t)s->trace.size() < s->trace_cap) s->trace.push_back(lam);
    s->iters = s->k + 1;
    if (s->initialized && close_rel(lam, s->lambda, s->opts.tolerance)) {
        s->lambda = lam;
        s->converged = true;
        s->done = true;
        return EIGSOL_OK;
    }
    s->lambda = lam;
    s->initialized = true;
    ++s->k;
    if (s->k >= s->opts.max_iterations) s->done = true;
    if (!s->shifted) {   // A x_k is the next iteration's y
        std::swap(s->y, s->z);
        s->pend_n2 = nz;
    }
    return EIGSOL_OK;
}

int wide_begin(WideSession* s, const eigsol_solver_options* opts, const void* x0, int on_dev) {
    EIGSOL_HIP(hipSetDevice(s->ctx->device));
    return by_wide(s->dtype, [&](auto tag) { return begin_t<decltype(tag)>(s, opts, x0, on_dev); });
}

int wide_step(WideSession* s, int32_t nsteps) {
    if (!s->begun) return fail(EIGSOL_E_INVALID, "eigsol_power_step: session not begun");
    EIGSOL_HIP(hipSetDevice(s->ctx->device));
    for (int32_t i = 0; i < nsteps && !s->done; ++i)
        EIGSOL_TRY(by_wide(s->dtype, [&](auto tag) { return iterate_t<decltype(tag)>(s); }));
    return EIGSOL_OK;
}

int wide_query(WideSession* s, int32_t* done, int32_t* launches) {
    if (!s->begun) return fail(EIGSOL_E_INVALID, "eigsol_power_query: session not begun");
    if (done) *done = s->done ? 1 : 0;
    if (launches) *launches = s->iters;
    return EIGSOL_OK;
}

int wide_finish(WideSession* s, void* lambda_out, void* x_out, int x_on_dev, int32_t* iterations, int32_t* converged) {
    if (!s->begun) return fail(EIGSOL_E_INVALID, "eigsol_power_finish: session not begun");
    if (!s->done) return fail(EIGSOL_E_INVALID, "eigsol_power_finish: iteration has not terminated");
    EIGSOL_HIP(hipSetDevice(s->ctx->device));
    if (lambda_out) std::memcpy(lambda_out, &s->lambda, s->sb);   // dd: the real part's pair
    if (iterations) *iterations = s->iters;
    if (converged) *converged = s->converged ? 1 : 0;
    if (x_out) {
        EIGSOL_HIP(hipMemcpyAsync(x_out, s->x, s->n * s->sb, x_on_dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                                  s->ctx->stream));
        EIGSOL_HIP(hipStreamSynchronize(s->ctx->stream));
    }
    return EIGSOL_OK;
}

int wide_trace(WideSession* s, void* trace_host, int32_t capacity, int32_t* count) {
    if (!s->begun) return fail(EIGSOL_E_INVALID, "eigsol_power_trace: session not begun");
    const int32_t n = (int32_t)s->trace.size();
    if (trace_host)
        for (int32_t i = 0; i < std::min(n, capacity); ++i)
            std::memcpy(static_cast<char*>(trace_host) + (size_t)i * s->sb, &s->trace[i], s->sb);
    if (count) *count = n;
    return EIGSOL_OK;
}

void wide_info(const WideSession* s, double* bytes, int32_t* variant, int32_t* tiles, int32_t* grid) {
    const double sb = (double)s->sb, n = (double)s->n;
    if (s->shifted) {
        if (bytes) *bytes = s->solve_bytes;
        if (variant) *variant = 17;
        if (tiles) *tiles = s->refine_steps;
    } else if (s->csr) {
        if (bytes) *bytes = (sb + 4.0) * (double)s->csr->nnz + 4.0 * (n + 1.0) + 3.0 * sb * n;   // y read, x and z written
        if (variant) *variant = 15;
        if (tiles) *tiles = 0;
    } else {
        if (bytes) *bytes = sb * n * n + 2.0 * sb * n;
        if (variant) *variant = 16;
        if (tiles) *tiles = 0;
    }
    if (grid) *grid = (int32_t)nblk(s->n);
}

// solve_shifted<S> (solve_shifted.hpp:48-118) in double-double: factor, one refined solve
int wide_solve_shifted(eigsol_csr* csr, eigsol_dense* dense, const void* sigma, const void* b, int64_t nb, void* x) {
    eigsol_ctx* ctx = csr ? csr->ctx : dense->ctx;
    WideSession* s = nullptr;
    EIGSOL_TRY(wide_session_create(ctx, csr, dense, sigma, 0, &s));
    hipStream_t st = ctx->stream;
    int rc = EIGSOL_OK;
    if (hipMemcpyAsync(s->x, b, nb * s->sb, hipMemcpyHostToDevice, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "solve_shifted: upload");
    if (rc == EIGSOL_OK)
        rc = by_wide(s->dtype, [&](auto tag) { return refine_solve<decltype(tag)>(s, s->x, s->y); });
    if (rc == EIGSOL_OK && (hipMemcpyAsync(x, s->y, nb * s->sb, hipMemcpyDeviceToHost, st) != hipSuccess ||
                            stream_wait(st) != hipSuccess))
        rc = fail(EIGSOL_E_HIP, "solve_shifted: download");
    wide_session_free(s);
    return rc;
}

// ---------------------------------------------------------------- QR method in double-double
namespace {

template <class T>
struct WQr {
    T* v = nullptr;
    int* skip = nullptr;
    dd* red = nullptr;
};
template <class T>
int wqr_alloc(WQr<T>& w, int64_t n) {
    EIGSOL_HIP(hipMalloc(&w.v, std::max<int64_t>(n, 1) * sizeof(T)));
    EIGSOL_HIP(hipMalloc(&w.skip, 64));
    EIGSOL_HIP(hipMalloc(&w.red, 64));
    return EIGSOL_OK;
}
template <class T>
void wqr_free(WQr<T>& w) {
    for (void* p : {(void*)w.v, (void*)w.skip, (void*)w.red})
        if (p) (void)hipFree(p);
}

// one reflector: x = A(r0 : r0+m, col); left on A(r0 : r0+m, lc0 : lc1); right on B(0 : nr, r0 : r0+m)
template <class T>
void wreflect(hipStream_t st, T* A, int64_t lda, int64_t r0, int64_t col, int64_t m, int64_t lc0, int64_t lc1, T* B,
              int64_t ldb, int64_t nr, WQr<T>& w) {
    hipLaunchKernelGGL((wdev::hh_make_kernel<T>), dim3(1), dim3(1024), 0, st, A, lda, r0, col, m, w.v, w.skip);
    if (lc1 > lc0)
        hipLaunchKernelGGL((wdev::hh_left_kernel<T>), dim3(lc1 - lc0), dim3(wdev::kT), 0, st, A, lda, r0, m, lc0, w.v,
                           w.skip);
    if (nr > 0)
        hipLaunchKernelGGL((wdev::hh_right_kernel<T>), dim3((nr + 15) / 16), dim3(wdev::kT), 0, st, B, ldb, nr, r0, m,
                           w.v, w.skip);
}

// to_hessenberg_dense (to_hessenberg.hpp:38-77)
template <class T>
int whessenberg(hipStream_t st, T* H, int64_t n, WQr<T>& w) {
    for (int64_t k = 0; k + 2 < n; ++k) wreflect<T>(st, H, n, k + 1, k, n - k - 1, k, n, H, n, n, w);
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

// qr_decompose_dense (qr_decompose.hpp:46-85): R (m x n) in place, Q (m x m) from the identity
template <class T>
int wqr_decompose(hipStream_t st, T* R, int64_t m, int64_t n, T* Q, WQr<T>& w) {
    hipLaunchKernelGGL((wdev::set_identity_kernel<T>), dim3(nblk(m * m)), dim3(wdev::kT), 0, st, Q, m);
    for (int64_t k = 0; k < std::min(m, n); ++k) {
        const int64_t rows = m - k;
        if (rows < 2) continue;   // x.tail(0).norm() == 0: skipped by the reference too
        wreflect<T>(st, R, m, k, k, rows, k, n, Q, m, m, w);
    }
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

template <class T>
int whessenberg_host(eigsol_ctx* ctx, int64_t n, const void* A, void* Hout) {
    hipStream_t st = ctx->stream;
    T* H = nullptr;
    EIGSOL_HIP(hipMalloc(&H, std::max<int64_t>(n * n, 1) * sizeof(T)));
    WQr<T> w;
    int rc = wqr_alloc(w, n);
    if (rc == EIGSOL_OK && hipMemcpyAsync(H, A, n * n * sizeof(T), hipMemcpyHostToDevice, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "to_hessenberg: upload");
    if (rc == EIGSOL_OK) rc = whessenberg<T>(st, H, n, w);
    if (rc == EIGSOL_OK && (hipMemcpyAsync(Hout, H, n * n * sizeof(T), hipMemcpyDeviceToHost, st) != hipSuccess ||
                            stream_wait(st) != hipSuccess))
        rc = fail(EIGSOL_E_HIP, "to_hessenberg: download");
    wqr_free(w);
    (void)hipFree(H);
    return rc;
}

template <class T>
int wqr_decompose_host(eigsol_ctx* ctx, int64_t m, int64_t n, const void* A, void* Qout, void* Rout) {
    hipStream_t st = ctx->stream;
    T *R = nullptr, *Q = nullptr;
    EIGSOL_HIP(hipMalloc(&R, m * n * sizeof(T)));
    if (hipMalloc(&Q, m * m * sizeof(T)) != hipSuccess) {
        (void)hipFree(R);
        return fail(EIGSOL_E_HIP, "qr_decompose: hipMalloc");
    }
    WQr<T> w;
    int rc = wqr_alloc(w, m);
    if (rc == EIGSOL_OK && hipMemcpyAsync(R, A, m * n * sizeof(T), hipMemcpyHostToDevice, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "qr_decompose: upload");
    if (rc == EIGSOL_OK) rc = wqr_decompose<T>(st, R, m, n, Q, w);
    if (rc == EIGSOL_OK && Qout && hipMemcpyAsync(Qout, Q, m * m * sizeof(T), hipMemcpyDeviceToHost, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "qr_decompose: download Q");
    if (rc == EIGSOL_OK && Rout && hipMemcpyAsync(Rout, R, m * n * sizeof(T), hipMemcpyDeviceToHost, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "qr_decompose: download R");
    if (rc == EIGSOL_OK && stream_wait(st) != hipSuccess) rc = fail(EIGSOL_E_HIP, "qr_decompose: sync");
    wqr_free(w);
    (void)hipFree(R);
    (void)hipFree(Q);
    return rc;
}

// qr_eigenvalues_dense (qr_eigenvalues.hpp:61-104): Hessenberg, then H <- R Q until
// max |H(i, i-1)| <= tol (1 + ||H||_F), compared in extended precision; iterations = iter + 1
template <class T>
int wqr_unshifted_host(eigsol_ctx* ctx, int64_t n, const void* A, int max_iter, double tol, void* eig, int32_t* iters,
                       int32_t* conv) {
    hipStream_t st = ctx->stream;
    T *H = nullptr, *Q = nullptr, *R = nullptr, *d = nullptr;
    int rc = EIGSOL_OK;
    if (hipMalloc(&H, n * n * sizeof(T)) != hipSuccess || hipMalloc(&Q, n * n * sizeof(T)) != hipSuccess ||
        hipMalloc(&R, n * n * sizeof(T)) != hipSuccess || hipMalloc(&d, n * sizeof(T)) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: hipMalloc");
    WQr<T> w;
    if (rc == EIGSOL_OK) rc = wqr_alloc(w, n);
    if (rc == EIGSOL_OK && hipMemcpyAsync(H, A, n * n * sizeof(T), hipMemcpyHostToDevice, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: upload");
    if (rc == EIGSOL_OK) rc = whessenberg<T>(st, H, n, w);
    int iter = 0;
    bool converged = false;
    const dim3 g((unsigned)((n + 15) / 16), (unsigned)((n + 15) / 16));
    for (iter = 0; rc == EIGSOL_OK && iter < max_iter; ++iter) {
        if (hipMemcpyAsync(R, H, n * n * sizeof(T), hipMemcpyDeviceToDevice, st) != hipSuccess) {
            rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: copy");
            break;
        }
        rc = wqr_decompose<T>(st, R, n, n, Q, w);
        if (rc != EIGSOL_OK) break;
        hipLaunchKernelGGL((wdev::gemm_nn_kernel<T>), g, dim3(wdev::kT), 0, st, R, Q, H, n);
        hipLaunchKernelGGL((wdev::subdiag_frob_kernel<T>), dim3(1), dim3(wdev::kT), 0, st, H, n, w.red);
        dd red[2];
        if (hipMemcpyAsync(red, w.red, sizeof(red), hipMemcpyDeviceToHost, st) != hipSuccess ||
            stream_wait(st) != hipSuccess) {
            rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: convergence check");
            break;
        }
        const dd scale = dd_sqrt(red[1]);
        const dd thresh = dd_mul(dd_from(tol), dd_add_d(scale, 1.0));
        if (dd_le(red[0], thresh)) {
            converged = true;
            break;
        }
    }
    if (rc == EIGSOL_OK) {
        hipLaunchKernelGGL((wdev::diag_kernel<T>), dim3(nblk(n)), dim3(wdev::kT), 0, st, H, n, d);
        if (hipMemcpyAsync(eig, d, n * sizeof(T), hipMemcpyDeviceToHost, st) != hipSuccess ||
            stream_wait(st) != hipSuccess)
            rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: download");
    }
    if (iters) *iters = iter + 1;
    if (conv) *conv = converged ? 1 : 0;
    wqr_free(w);
    for (void* p : {(void*)H, (void*)Q, (void*)R, (void*)d})
        if (p) (void)hipFree(p);
    return rc;
}

// ---------------------------------------------------------------- long double Francis QR
// qr_eigenvalues<long double> with the implicit-shift variant (north_star's algorithm class; the
// reference's ScalarConcept admits long double, types.hpp:28-30): the double-double Hessenberg
// matrix H is rounded to fp64 and its eigenvalues found by the fp64 multishift sweeps
// (francis.hip / zfrancis.hip); then every eigenvalue is refined on H ITSELF, in double-double, by
// Newton's method on det(H - mu I).  For an unreduced Hessenberg matrix Hyman's recurrence gives
// det(H - mu I) = +-c(mu) prod h(i, i-1) from the vector x with x(n-1) = 1 solving rows 1 .. n-1 of
// (H - mu I) x = c e_0 (back substitution through the subdiagonal), c = row 0's residual; the
// same recurrence differentiated gives c'(mu), and mu <- mu - c / c' converges quadratically from
// the fp64 eigenvalue (error ~1e-16 cond) to the double-double floor in two or three steps.
// Exact zeros on the subdiagonal split H into blocks; each block has its own recurrence and the
// eigenvalue is refined on the block whose Newton step from the fp64 value is the smallest.  x and
// its derivative are rescaled by powers of two when they leave [2^-300, 2^300] (the ratio c / c'
// is scale-invariant).  A refinement that moves the eigenvalue by more than 1e-8 (1 + |lambda|)
// (a Newton step that left the fp64 eigenvalue's basin) is discarded and the fp64 value kept.
namespace wqdev {

template <class T> __device__ __forceinline__ cdd as_cdd(const T& a);
template <> __device__ __forceinline__ cdd as_cdd<dd>(const dd& a) { EIGSOL_EXACT return cdd{a, dd{0.0, 0.0}}; }
template <> __device__ __forceinline__ cdd as_cdd<cdd>(const cdd& a) { return a; }

__device__ __forceinline__ double cdd_maxhi(const cdd& a) { return fmax(fabs(a.re.hi), fabs(a.im.hi)); }

constexpr int kHyT = 1024;   // threads of the refinement (one workgroup per eigenvalue)

// One workgroup per eigenvalue; thread t owns rows t + kHyT k, k < R (n <= kHyT R).  Per column j
// (descending): every owned row i <= j adds (h(i, j) - mu [i = j]) x_j to r_i and the same with
// x'_j (minus x_j at i = j) to r'_i; the owner of row j then forms x_{j-1} = -r_j / h(j, j-1) (and
// x'_{j-1}), or closes the block at a zero subdiagonal.  One barrier per column, two LDS slots
// alternating by column parity.
template <class T, int R>
__global__ __launch_bounds__(kHyT) void hyman_newton_kernel(const T* __restrict__ H, int n, const cdd* __restrict__ lam0,
                                                            cdd* __restrict__ lam_out, int32_t* __restrict__ steps_out,
                                                            int max_newton) {
    EIGSOL_EXACT
    __shared__ cdd sx[2][2];      // [parity] {x_j, x'_j}
    __shared__ int sflag[2][2];   // [parity] {reset rows < j+1 (block closed), scale exponent}
    __shared__ cdd s_delta;       // Newton step of the selected block
    __shared__ double s_best;     // |step| of the best block (first pass)
    __shared__ int s_hi, s_cur_hi, s_done, s_upd;
    const int t = threadIdx.x;
    const int64_t ld = n;
    const cdd zero = cdd{dd{0.0, 0.0}, dd{0.0, 0.0}};
    const cdd one = cdd{dd{1.0, 0.0}, dd{0.0, 0.0}};
    const cdd l0 = lam0[blockIdx.x];
    cdd mu = l0;
    int steps = 0;
    if (t == 0) { s_hi = -1; s_done = 0; }
    for (int it = 0; it < max_newton; ++it) {
        cdd r[R], rp[R];
#pragma unroll
        for (int k = 0; k < R; ++k) { r[k] = zero; rp[k] = zero; }
        if (t == 0) {
            sx[(n - 1) & 1][0] = one;
            sx[(n - 1) & 1][1] = zero;
            sflag[(n - 1) & 1][0] = 0;
            sflag[(n - 1) & 1][1] = 0;
            s_cur_hi = n;
            s_best = -1.0;
        }
        __syncthreads();
        for (int j = n - 1; j >= 0; --j) {
            const int par = j & 1;
            const cdd xj = sx[par][0], xpj = sx[par][1];
            const int reset = sflag[par][0], esc = sflag[par][1];
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const int i = t + kHyT * k;
                if (i <= j) {
                    if (reset) { r[k] = zero; rp[k] = zero; }   // rows of the next block start afresh
                    else if (esc) { r[k] = cdd_ldexp(r[k], esc); rp[k] = cdd_ldexp(rp[k], esc); }
                    cdd a = as_cdd<T>(H[i + (int64_t)j * ld]);
                    if (i == j) a = cdd_sub(a, mu);
                    r[k] = cdd_add(r[k], cdd_mul(a, xj));
                    rp[k] = cdd_add(rp[k], cdd_mul(a, xpj));
                    if (i == j) rp[k] = cdd_sub(rp[k], xj);
                }
            }
            // the owner of row j: next x, or the block [j, cur_hi) closes
            if (t == (j % kHyT)) {
                const int k = j / kHyT;
                cdd rj = r[0], rpj = rp[0];
#pragma unroll
                for (int q = 1; q < R; ++q)
                    if (q == k) { rj = r[q]; rpj = rp[q]; }
                const cdd sub_h = j > 0 ? as_cdd<T>(H[j + (int64_t)(j - 1) * ld]) : zero;
                const int np = (j - 1) & 1;
                if (j == 0 || cdd_is_zero(sub_h)) {
                    // block [j, cur_hi): c = r_j, c' = r'_j, Newton step c / c'
                    const cdd d = cdd_div(rj, rpj);
                    const double ad = cdd_maxhi(d);
                    const bool ok = ad == ad && ad <= 1.7976931348623157e308;
                    if (it == 0) {
                        if (ok && (s_best < 0.0 || ad < s_best)) { s_best = ad; s_delta = d; s_hi = s_cur_hi; }
                    } else if (s_cur_hi == s_hi) {
                        s_delta = ok ? d : zero;
                        s_best = ok ? ad : -1.0;
                    }
                    if (j > 0) {
                        sx[np][0] = one;
                        sx[np][1] = zero;
                        sflag[np][0] = 1;
                        sflag[np][1] = 0;
                        s_cur_hi = j;
                    }
                } else {
                    cdd xn = cdd_neg(cdd_div(rj, sub_h));
                    cdd xpn = cdd_neg(cdd_div(rpj, sub_h));
                    const double m = fmax(cdd_maxhi(xn), cdd_maxhi(xpn));
                    int e = 0;
                    if (m > 0x1p300 || (m > 0.0 && m < 0x1p-300)) e = -ilogb(m);
                    if (e) { xn = cdd_ldexp(xn, e); xpn = cdd_ldexp(xpn, e); }
                    sx[np][0] = xn;
                    sx[np][1] = xpn;
                    sflag[np][0] = 0;
                    sflag[np][1] = e;
                }
            }
            __syncthreads();
        }
        // Newton update (thread 0 decides, everyone reads mu): mu <- mu - c / c' of the selected
        // block; stop after a step at the double-double floor, or without a usable step
        if (t == 0) {
            s_upd = 0;
            if (s_best < 0.0) {
                s_done = 1;
            } else {
                const cdd mn = cdd_sub(mu, s_delta);
                ++steps;
                const double am = fmax(cdd_maxhi(mn), 1e-300);
                if (s_best <= 0x1p-104 * am || it + 1 == max_newton) s_done = 1;
                sx[0][0] = mn;   // hand mu over through LDS (slot free until the next pass starts)
                s_upd = 1;
            }
        }
        __syncthreads();
        if (s_upd) mu = sx[0][0];
        const int done = s_done;
        __syncthreads();
        if (done) break;
    }
    if (t == 0) {
        // discard a refinement that left the fp64 eigenvalue's neighbourhood
        const cdd dm = cdd_sub(mu, l0);
        const double move = cdd_maxhi(dm), scale = 1.0 + cdd_maxhi(l0);
        const bool keep = move == move && move <= 1e-8 * scale;
        lam_out[blockIdx.x] = keep ? mu : l0;
        steps_out[blockIdx.x] = keep ? steps : -1;
    }
}

// hi parts of the double-double Hessenberg matrix (fp64 / complex fp64) and max |hi| (bits)
template <class T>
__global__ __launch_bounds__(wdev::kT) void hi_parts_kernel(const T* __restrict__ H, int64_t cnt, double* __restrict__ out,
                                                      unsigned long long* __restrict__ amax) {
    double m = 0.0;
    for (int64_t e = (int64_t)blockIdx.x * wdev::kT + threadIdx.x; e < cnt; e += (int64_t)gridDim.x * wdev::kT) {
        if constexpr (std::is_same_v<T, dd>) {
            out[e] = H[e].hi;
            m = fmax(m, fabs(H[e].hi));
        } else {
            out[2 * e] = H[e].re.hi;
            out[2 * e + 1] = H[e].im.hi;
            m = fmax(m, fmax(fabs(H[e].re.hi), fabs(H[e].im.hi)));
        }
    }
    for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off, 64));
    if ((threadIdx.x & 63) == 0 && m > 0.0) atomicMax(amax, (unsigned long long)__double_as_longlong(m));
}

__global__ __launch_bounds__(wdev::kT) void ldexp_kernel(double* __restrict__ a, int64_t cnt, int e) {
    for (int64_t i = (int64_t)blockIdx.x * wdev::kT + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * wdev::kT)
        a[i] = ldexp(a[i], e);
}

}  // namespace wqdev

}  // namespace

int francis_large_f64(eigsol_ctx* ctx, double* H, int64_t n, int maxits, double* wr, double* wi, int32_t* sweeps,
                      int32_t* fail_out);
int francis_large_c128(eigsol_ctx* ctx, cplx* H, int64_t n, int maxits, cplx* w_host, int32_t* sweeps_out,
                       int32_t* fail_out);

namespace {

constexpr int kHyMaxRows = 8;   // refinement: n <= kHyT * 8 = 8192

template <class T, int R>
static void hyman_launch(hipStream_t st, const T* H, int n, const cdd* l0, cdd* l1, int32_t* steps, int64_t count) {
    hipLaunchKernelGGL((wqdev::hyman_newton_kernel<T, R>), dim3((unsigned)count), dim3(wqdev::kHyT), 0, st, H, n, l0,
                       l1, steps, 4);
}

// eig: n scalars of T (DD: the real parts); eig_im (DD only, may be null): n dd imaginary parts
template <class T>
int wqr_francis_host(eigsol_ctx* ctx, int64_t n, const void* A, int max_iter, void* eig, double* eig_im,
                     int32_t* iters, int32_t* conv) {
    if (n > (int64_t)wqdev::kHyT * kHyMaxRows)
        return fail(EIGSOL_E_UNSUPPORTED, "qr_eigenvalues: the double-double Francis refinement handles n <= 8192");
    constexpr bool cx = std::is_same_v<T, cdd>;
    hipStream_t st = ctx->stream;
    T* H = nullptr;
    double* H64 = nullptr;
    cdd *dl0 = nullptr, *dl1 = nullptr;
    int32_t* dsteps = nullptr;
    unsigned long long* damax = nullptr;
    int rc = EIGSOL_OK;
    if (hipMalloc(&H, n * n * sizeof(T)) != hipSuccess || hipMalloc(&H64, n * n * (cx ? 16 : 8)) != hipSuccess ||
        hipMalloc(&dl0, n * sizeof(cdd)) != hipSuccess || hipMalloc(&dl1, n * sizeof(cdd)) != hipSuccess ||
        hipMalloc(&dsteps, n * sizeof(int32_t)) != hipSuccess || hipMalloc(&damax, 64) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: hipMalloc");
    WQr<T> w;
    if (rc == EIGSOL_OK) rc = wqr_alloc(w, n);
    if (rc == EIGSOL_OK && hipMemcpyAsync(H, A, n * n * sizeof(T), hipMemcpyHostToDevice, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: upload");
    if (rc == EIGSOL_OK) rc = whessenberg<T>(st, H, n, w);
    // fp64 rounding of H, with LAPACK xGEEV's range guard (max |h| outside [smlnum, 1 / smlnum]:
    // exact power-of-two scaling for the sweeps, eigenvalues scaled back)
    unsigned long long bits = 0;
    if (rc == EIGSOL_OK) {
        hipMemsetAsync(damax, 0, 8, st);
        hipLaunchKernelGGL((wqdev::hi_parts_kernel<T>), dim3(rgrid(n * n)), dim3(wdev::kT), 0, st, H, n * n, H64, damax);
        if (hipMemcpyAsync(&bits, damax, 8, hipMemcpyDeviceToHost, st) != hipSuccess || stream_wait(st) != hipSuccess)
            rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: fp64 rounding");
    }
    int escale = 0;
    if (rc == EIGSOL_OK) {
        double amax;
        std::memcpy(&amax, &bits, sizeof(amax));
        const double smlnum = std::sqrt(std::numeric_limits<double>::min()) / std::numeric_limits<double>::epsilon();
        if (std::isfinite(amax) && amax > 0.0 && (amax < smlnum || amax > 1.0 / smlnum)) {
            escale = -std::ilogb(amax);
            hipLaunchKernelGGL(wqdev::ldexp_kernel, dim3(rgrid(n * n * (cx ? 2 : 1))), dim3(wdev::kT), 0, st, H64,
                               n * n * (cx ? 2 : 1), escale);
        }
    }
    std::vector<cdd> l0(n);
    int32_t sweeps = 0, failed = 0;
    if (rc == EIGSOL_OK) {
        if constexpr (cx) {
            std::vector<cplx> wv(n);
            rc = francis_large_c128(ctx, reinterpret_cast<cplx*>(H64), n, max_iter, wv.data(), &sweeps, &failed);
            for (int64_t i = 0; i < n && rc == EIGSOL_OK; ++i)
                l0[i] = cdd{dd{std::ldexp(wv[i].re, -escale), 0.0}, dd{std::ldexp(wv[i].im, -escale), 0.0}};
        } else {
            std::vector<double> wr(n), wi(n);
            rc = francis_large_f64(ctx, H64, n, max_iter, wr.data(), wi.data(), &sweeps, &failed);
            for (int64_t i = 0; i < n && rc == EIGSOL_OK; ++i)
                l0[i] = cdd{dd{std::ldexp(wr[i], -escale), 0.0}, dd{std::ldexp(wi[i], -escale), 0.0}};
        }
    }
    std::vector<cdd> l1(n);
    std::vector<int32_t> steps(n, 0);
    if (rc == EIGSOL_OK && hipMemcpyAsync(dl0, l0.data(), n * sizeof(cdd), hipMemcpyHostToDevice, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: upload eigenvalues");
    if (rc == EIGSOL_OK) {
        const int R = (int)((n + wqdev::kHyT - 1) / wqdev::kHyT);
        const int ni = (int)n;
        if (R <= 1) hyman_launch<T, 1>(st, H, ni, dl0, dl1, dsteps, n);
        else if (R <= 2) hyman_launch<T, 2>(st, H, ni, dl0, dl1, dsteps, n);
        else if (R <= 4) hyman_launch<T, 4>(st, H, ni, dl0, dl1, dsteps, n);
        else hyman_launch<T, 8>(st, H, ni, dl0, dl1, dsteps, n);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(l1.data(), dl1, n * sizeof(cdd), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(steps.data(), dsteps, n * sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
            stream_wait(st) != hipSuccess)
            rc = fail(EIGSOL_E_HIP, "qr_eigenvalues: double-double refinement");
    }
    if (rc == EIGSOL_OK) {
        if (std::getenv("EIGSOL_WIDE_QR_DEBUG")) {
            int kept = 0, mx = 0;
            for (int32_t s : steps) { kept += s < 0; mx = std::max(mx, s); }
            std::fprintf(stderr, "[wide-qr] n %lld sweeps %d refinement: %d kept fp64, max Newton steps %d\n",
                         (long long)n, sweeps, kept, mx);
        }
        for (int64_t i = 0; i < n; ++i) {
            if constexpr (cx) {
                static_cast<cdd*>(eig)[i] = l1[i];
            } else {
                static_cast<dd*>(eig)[i] = l1[i].re;
                if (eig_im) {
                    eig_im[2 * i] = l1[i].im.hi;
                    eig_im[2 * i + 1] = l1[i].im.lo;
                }
            }
        }
    }
    if (iters) *iters = sweeps;
    if (conv) *conv = failed ? 0 : 1;
    wqr_free(w);
    for (void* p : {(void*)H, (void*)H64, (void*)dl0, (void*)dl1, (void*)dsteps, (void*)damax})
        if (p) (void)hipFree(p);
    return rc;
}

}  // namespace

int wide_hessenberg(eigsol_ctx* ctx, int dtype, int64_t n, const void* A, void* H) {
    return by_wide(dtype, [&](auto tag) { return whessenberg_host<decltype(tag)>(ctx, n, A, H); });
}
int wide_qr_decompose(eigsol_ctx* ctx, int dtype, int64_t m, int64_t n, const void* A, void* Q, void* R) {
    return by_wide(dtype, [&](auto tag) { return wqr_decompose_host<decltype(tag)>(ctx, m, n, A, Q, R); });
}
int wide_qr_eigenvalues(eigsol_ctx* ctx, int dtype, int64_t n, const void* A, const eigsol_solver_options* opts,
                        int variant, void* eig, double* eig_im, int32_t* iters, int32_t* conv) {
    if (variant != EIGSOL_QR_UNSHIFTED)
        return by_wide(dtype, [&](auto tag) {
            return wqr_francis_host<decltype(tag)>(ctx, n, A, opts->max_iterations, eig, eig_im, iters, conv);
        });
    return by_wide(dtype, [&](auto tag) {
        return wqr_unshifted_host<decltype(tag)>(ctx, n, A, opts->max_iterations, opts->tolerance, eig, iters, conv);
    });
}

}  // namespace eigsol

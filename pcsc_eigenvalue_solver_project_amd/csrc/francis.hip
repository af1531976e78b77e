// Francis multishift QR sweeps for large real Hessenberg matrices (gfx950).
//
// The north_star replaces the reference's unshifted QR iteration (qr_eigenvalues.hpp:69-94,
// which does not converge on general input) with implicit-shift sweeps.  A sweep
// on the active block [l, ihi] chases a CHAIN of nb double-shift bulges (3x3 Householder
// reflectors, the textbook eigenvalue-only algorithm of the oracle's hqr_francis) down the
// block.  Bulges are 3 rows apart, so one chase step moves every bulge by one row at once: their
// left updates touch disjoint rows and their right updates disjoint columns (associativity makes
// the simultaneous step an exact product of the reflectors).
//
// Locality: the chain is chased inside an LDS window [s, e) of at most kWin rows/columns with
// the window's orthogonal factor U accumulated alongside; the parts of the reflectors' updates
// outside the window are applied afterwards as two small GEMMs (one fused launch),
//     H(s:e, e:ihi]   <- U^T H(s:e, e:ihi]        H[l, s) x [s, e) <- H[l, s) x [s, e) U,
// so every HBM element of the active block is touched O(1) times per window instead of once per
// reflector.  Shifts: eigenvalues of the trailing 2nb x 2nb block (in-LDS Francis solver,
// hqr_lds_kernel); blocks of at most 128 rows are finished entirely in LDS.  Deflation: the
// conventional criterion |h(k,k-1)| <= eps (|h(k,k)| + |h(k-1,k-1)|).
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernels_common.hpp"

namespace eigsol {

int hqr_lds(hipStream_t st, const double* H, int64_t ld, int n, int maxits, double* wr_dev, double* wi_dev,
            int* info_dev);

namespace dev {

constexpr int kWin = 96;        // window rows/columns (H window + U: 2 x 72 KiB of LDS)
constexpr int kMaxBulges = 16;

// compiler-only ordering of LDS accesses (one wave's LDS operations execute in issue order)
#define EIGSOL_LDS_ORDER() asm volatile("" ::: "memory")

struct ChaseArgs {
    double* H;
    int64_t n;        // leading dimension
    int s, e;         // window [s, e)
    int l, ihi;       // active block
    int t0, t1;       // chase steps of this window
    int nb;           // bulges in the chain
    const double* shifts;   // per bulge: xs (= ys) and ws of the shift pair
    double* U;        // out: (e - s)^2 accumulated factor, column-major
};

__global__ __launch_bounds__(1024) void chase_kernel(ChaseArgs a) {
    // H window with an odd leading dimension: the left updates walk a row across columns, and a
    // stride of an even number of doubles would put every lane of a wave on the same LDS bank
    __shared__ double h[kWin * (kWin + 1)];
    __shared__ double u[kWin * kWin];
    __shared__ double rp[kMaxBulges][6];   // xs, ys, zs, q, r, active (as double)
    __shared__ int rk[kMaxBulges];
    const int W = a.e - a.s;
    const int ldh = W | 1;
    const int tid = threadIdx.x;
    const int nt = blockDim.x;
    auto Hw = [&](int i, int j) -> double& { return h[(i - a.s) + (j - a.s) * ldh]; };
    {
        // window load: all global loads first (9 per thread), then the LDS stores
        constexpr int kPer = (kWin * kWin + 1023) / 1024;
        double tmp[kPer];
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int idx = tid + q * 1024;
            const int i = idx % W, j = idx / W;
            tmp[q] = idx < W * W ? a.H[(a.s + i) + (int64_t)(a.s + j) * a.n] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int idx = tid + q * 1024;
            if (idx < W * W) {
                const int i = idx % W, j = idx / W;
                h[i + j * ldh] = tmp[q];
                u[idx] = (i == j) ? 1.0 : 0.0;
            }
        }
    }
    __syncthreads();
    const int l = a.l, ihi = a.ihi;
    for (int t = a.t0; t < a.t1; ++t) {
        // ---- reflectors of every active bulge (one thread per bulge)
        if (tid < a.nb) {
            const int b = tid;
            const int k = l + t - 3 * b;
            const bool live = k >= l && k <= ihi - 1;
            rk[b] = k;
            rp[b][5] = 0.0;
            if (live) {
                double p, q, r, xs = 1.0;
                if (k == l) {
                    // first column of (H - s1)(H - s2) e_l, shift pair given by (xs = ys, ws)
                    const double sx = a.shifts[2 * b], sw = a.shifts[2 * b + 1];
                    const double z = Hw(l, l);
                    const double rr = sx - z, ss = sx - z;
                    p = (rr * ss - sw) / Hw(l + 1, l) + Hw(l, l + 1);
                    q = Hw(l + 1, l + 1) - z - rr - ss;
                    r = (l + 2 <= ihi) ? Hw(l + 2, l + 1) : 0.0;
                    const double sc = fabs(p) + fabs(q) + fabs(r);
                    if (sc != 0.0) { const double is = 1.0 / sc; p *= is; q *= is; r *= is; }
                } else {
                    p = Hw(k, k - 1);
                    q = Hw(k + 1, k - 1);
                    r = (k != ihi - 1) ? Hw(k + 2, k - 1) : 0.0;
                    xs = fabs(p) + fabs(q) + fabs(r);
                    if (xs != 0.0) { const double is = 1.0 / xs; p *= is; q *= is; r *= is; }
                }
                // scaling by reciprocals: three divisions per reflector instead of eight (the
                // step's serial latency); the reflector stays orthogonal to rounding
                const double sg = (p >= 0 ? 1.0 : -1.0) * sqrt(p * p + q * q + r * r);
                if (sg != 0.0) {
                    if (k != l) {
                        Hw(k, k - 1) = -sg * xs;
                        Hw(k + 1, k - 1) = 0.0;
                        if (k != ihi - 1) Hw(k + 2, k - 1) = 0.0;
                    }
                    p += sg;
                    const double isg = 1.0 / sg, ip = 1.0 / p;
                    rp[b][0] = p * isg;
                    rp[b][1] = q * isg;
                    rp[b][2] = r * isg;
                    rp[b][3] = q * ip;
                    rp[b][4] = r * ip;
                    rp[b][5] = 1.0;
                }
            }
        }
        __syncthreads();
        // ---- left updates: wave b owns bulge b; rows k..k+2, window columns j in [k, e)
        const int wv = tid >> 6, ln = tid & 63;
        if (wv < a.nb && rp[wv][5] != 0.0) {
            const int k = rk[wv];
            const double xs = rp[wv][0], ys = rp[wv][1], zs = rp[wv][2], q = rp[wv][3], r = rp[wv][4];
            const bool three = k != ihi - 1;
            for (int j = k + ln; j < a.e; j += 64) {
                double p = Hw(k, j) + q * Hw(k + 1, j);
                if (three) { p += r * Hw(k + 2, j); Hw(k + 2, j) -= p * zs; }
                Hw(k + 1, j) -= p * ys;
                Hw(k, j) -= p * xs;
            }
        }
        __syncthreads();
        // ---- right updates: window rows i in [max(l, s), min(k+3, ihi)], then all rows of U
        if (wv < a.nb && rp[wv][5] != 0.0) {
            const int k = rk[wv];
            const double xs = rp[wv][0], ys = rp[wv][1], zs = rp[wv][2], q = rp[wv][3], r = rp[wv][4];
            const bool three = k != ihi - 1;
            const int ilast = min(k + 3, ihi);
            for (int i = max(l, a.s) + ln; i <= ilast; i += 64) {
                double p = xs * Hw(i, k) + ys * Hw(i, k + 1);
                if (three) { p += zs * Hw(i, k + 2); Hw(i, k + 2) -= p * r; }
                Hw(i, k + 1) -= p * q;
                Hw(i, k) -= p;
            }
            double* u0 = u + (k - a.s) * W;
            for (int i = ln; i < W; i += 64) {
                double p = xs * u0[i] + ys * u0[i + W];
                if (three) { p += zs * u0[i + 2 * W]; u0[i + 2 * W] -= p * r; }
                u0[i + W] -= p * q;
                u0[i] -= p;
            }
        }
        __syncthreads();
    }
    for (int idx = tid; idx < W * W; idx += nt) {
        const int i = idx % W, j = idx / W;
        a.H[(a.s + i) + (int64_t)(a.s + j) * a.n] = h[i + j * ldh];
        a.U[idx] = u[idx];
    }
}

// The same chase with two barriers per step and no serial section.  Wave b owns bulge b for the
// whole window: every lane computes the bulge's reflector redundantly from the same LDS words
// (column k-1 of the window is only ever written by bulge b's own updates), then
//   phase A: the left update of rows k..k+2 (columns [k, e)) and the U update (columns k..k+2);
//   phase B: the right update of columns k..k+2 (rows [max(l, s), min(k+3, ihi)]).
// Within a phase the bulges touch disjoint words: lefts own disjoint rows, rights disjoint
// columns, and a left (rows k..k+2, columns >= k) meets neither the reflector column k-1 of its
// own bulge nor the reflector columns of the others.  The barrier between the phases orders
// left(b+1) before right(b) on their shared 3 x 3 block; the barrier after phase B orders
// right(b) before the next step.  Each lane handles at most two columns / rows per phase, all
// LDS reads issued before the dependent arithmetic.
__global__ __launch_bounds__(1024) void chase_wave_kernel(ChaseArgs a) {
    __shared__ double h[kWin * (kWin + 1)];
    __shared__ double u[kWin * kWin];
    const int W = a.e - a.s;
    const int ldh = W | 1;
    const int tid = threadIdx.x;
    auto Hw = [&](int i, int j) -> double& { return h[(i - a.s) + (j - a.s) * ldh]; };
    {
        constexpr int kPer = (kWin * kWin + 1023) / 1024;
        double tmp[kPer];
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int idx = tid + q * 1024;
            const int i = idx % W, j = idx / W;
            tmp[q] = idx < W * W ? a.H[(a.s + i) + (int64_t)(a.s + j) * a.n] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int idx = tid + q * 1024;
            if (idx < W * W) {
                const int i = idx % W, j = idx / W;
                h[i + j * ldh] = tmp[q];
                u[idx] = (i == j) ? 1.0 : 0.0;
            }
        }
    }
    __syncthreads();
    const int l = a.l, ihi = a.ihi;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), ln = tid & 63;
    const int rlo = max(l, a.s);
    for (int t = a.t0; t < a.t1; ++t) {
        const int k = l + t - 3 * wv;
        bool act = wv < a.nb && k >= l && k <= ihi - 1;     // wave-uniform
        const bool three = k != ihi - 1;
        double ax = 0.0, ay = 0.0, az = 0.0, bq = 0.0, br = 0.0;
        if (act) {
            double p, q, r, xk = 1.0;
            if (k == l) {
                const double sx = a.shifts[2 * wv], sw = a.shifts[2 * wv + 1];
                const double z = Hw(l, l);
                const double rr = sx - z;
                p = (rr * rr - sw) / Hw(l + 1, l) + Hw(l, l + 1);
                q = Hw(l + 1, l + 1) - z - rr - rr;
                r = (l + 2 <= ihi) ? Hw(l + 2, l + 1) : 0.0;
                const double sc = fabs(p) + fabs(q) + fabs(r);
                if (sc != 0.0) { const double is = 1.0 / sc; p *= is; q *= is; r *= is; }
            } else {
                p = Hw(k, k - 1);
                q = Hw(k + 1, k - 1);
                r = three ? Hw(k + 2, k - 1) : 0.0;
                xk = fabs(p) + fabs(q) + fabs(r);
                if (xk != 0.0) { const double is = 1.0 / xk; p *= is; q *= is; r *= is; }
            }
            const double sg = (p >= 0 ? 1.0 : -1.0) * sqrt(p * p + q * q + r * r);
            act = sg != 0.0;
            if (act) {
                EIGSOL_LDS_ORDER();
                if (k != l && ln == 0) {
                    Hw(k, k - 1) = -sg * xk;
                    Hw(k + 1, k - 1) = 0.0;
                    if (three) Hw(k + 2, k - 1) = 0.0;
                }
                p += sg;
                const double isg = 1.0 / sg, ip = 1.0 / p;
                ax = p * isg; ay = q * isg; az = r * isg; bq = q * ip; br = r * ip;
                // ---- phase A: left update, columns k + ln and k + ln + 64 of rows k..k+2
                const int j0 = k + ln, j1 = j0 + 64;
                const bool c0 = j0 < a.e, c1 = j1 < a.e;
                double h00 = 0, h01 = 0, h02 = 0, h10 = 0, h11 = 0, h12 = 0;
                if (c0) { h00 = Hw(k, j0); h01 = Hw(k + 1, j0); if (three) h02 = Hw(k + 2, j0); }
                if (c1) { h10 = Hw(k, j1); h11 = Hw(k + 1, j1); if (three) h12 = Hw(k + 2, j1); }
                // U columns k..k+2 (window-relative), rows ln and ln + 64
                double* u0 = u + (k - a.s) * W;
                const int i0 = ln, i1 = ln + 64;
                const bool d0 = i0 < W, d1 = i1 < W;
                double u00 = 0, u01 = 0, u02 = 0, u10 = 0, u11 = 0, u12 = 0;
                if (d0) { u00 = u0[i0]; u01 = u0[i0 + W]; if (three) u02 = u0[i0 + 2 * W]; }
                if (d1) { u10 = u0[i1]; u11 = u0[i1 + W]; if (three) u12 = u0[i1 + 2 * W]; }
                {
                    const double p0 = h00 + bq * h01 + (three ? br * h02 : 0.0);
                    const double p1 = h10 + bq * h11 + (three ? br * h12 : 0.0);
                    if (c0) { Hw(k, j0) = h00 - p0 * ax; Hw(k + 1, j0) = h01 - p0 * ay; if (three) Hw(k + 2, j0) = h02 - p0 * az; }
                    if (c1) { Hw(k, j1) = h10 - p1 * ax; Hw(k + 1, j1) = h11 - p1 * ay; if (three) Hw(k + 2, j1) = h12 - p1 * az; }
                }
                {
                    const double p0 = ax * u00 + ay * u01 + (three ? az * u02 : 0.0);
                    const double p1 = ax * u10 + ay * u11 + (three ? az * u12 : 0.0);
                    if (d0) { u0[i0] = u00 - p0; u0[i0 + W] = u01 - p0 * bq; if (three) u0[i0 + 2 * W] = u02 - p0 * br; }
                    if (d1) { u0[i1] = u10 - p1; u0[i1 + W] = u11 - p1 * bq; if (three) u0[i1 + 2 * W] = u12 - p1 * br; }
                }
            }
        }
        __syncthreads();
        // ---- phase B: right update, rows rlo + ln and rlo + ln + 64 of columns k..k+2
        if (act) {
            const int ilast = min(k + 3, ihi);
            const int i0 = rlo + ln, i1 = i0 + 64;
            const bool c0 = i0 <= ilast, c1 = i1 <= ilast;
            double h00 = 0, h01 = 0, h02 = 0, h10 = 0, h11 = 0, h12 = 0;
            if (c0) { h00 = Hw(i0, k); h01 = Hw(i0, k + 1); if (three) h02 = Hw(i0, k + 2); }
            if (c1) { h10 = Hw(i1, k); h11 = Hw(i1, k + 1); if (three) h12 = Hw(i1, k + 2); }
            const double p0 = ax * h00 + ay * h01 + (three ? az * h02 : 0.0);
            const double p1 = ax * h10 + ay * h11 + (three ? az * h12 : 0.0);
            if (c0) { Hw(i0, k) = h00 - p0; Hw(i0, k + 1) = h01 - p0 * bq; if (three) Hw(i0, k + 2) = h02 - p0 * br; }
            if (c1) { Hw(i1, k) = h10 - p1; Hw(i1, k + 1) = h11 - p1 * bq; if (three) Hw(i1, k + 2) = h12 - p1 * br; }
        }
        __syncthreads();
    }
    for (int idx = tid; idx < W * W; idx += 1024) {
        const int i = idx % W, j = idx / W;
        a.H[(a.s + i) + (int64_t)(a.s + j) * a.n] = h[i + j * ldh];
        a.U[idx] = u[idx];
    }
}

// Both delayed updates of a window in ONE launch: blocks [0, nl) take 16-column panels of
//     H(s:e, c0:c1) <- U^T H(s:e, c0:c1)
// and blocks [nl, nl + nr) 16-row panels of
//     H(r0:r1, s:e) <- H(r0:r1, s:e) U.
// 256 threads = 16 columns (rows) x 16 groups of 6 outputs; U staged in LDS, the panel too.
__global__ __launch_bounds__(256) void win_gemm_fused(double* H, int64_t n, int s, int W, int64_t c0, int64_t c1,
                                                      int nl, int64_t r0, int64_t r1, const double* U) {
    __shared__ double um[kWin * kWin];     // left: um[i * kWin + r] = U(i, r); right: um[i * kWin + j] = U(i, j)
    __shared__ double x[kWin * 17];          // left: 16 x (kWin + 1) panel; right: kWin x 17
    const bool left = (int)blockIdx.x < nl;
    for (int idx = threadIdx.x; idx < kWin * kWin; idx += 256) {
        const int i = idx / kWin, r = idx % kWin;
        um[idx] = (i < W && r < W) ? U[i + r * W] : 0.0;
    }
    const int c = threadIdx.x & 15, g = threadIdx.x >> 4;
    double acc[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) acc[q] = 0.0;
    if (left) {
        const int64_t cb = c0 + (int64_t)blockIdx.x * 16;
        const int nc = (int)min<int64_t>(16, c1 - cb);
        for (int idx = threadIdx.x; idx < W * 16; idx += 256) {
            const int i = idx % W, cc = idx / W;
            x[cc * (kWin + 1) + i] = cc < nc ? H[(s + i) + (cb + cc) * n] : 0.0;   // column-major panel, odd stride
        }
        __syncthreads();
        for (int i = 0; i < W; ++i) {
            const double xv = x[c * (kWin + 1) + i];
            const double* ur = um + i * kWin + 6 * g;
#pragma unroll
            for (int q = 0; q < 6; ++q) acc[q] += ur[q] * xv;
        }
        if (c < nc)
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                const int r = 6 * g + q;
                if (r < W) H[(s + r) + (cb + c) * n] = acc[q];
            }
    } else {
        const int64_t rb = r0 + (int64_t)(blockIdx.x - nl) * 16;
        const int nr = (int)min<int64_t>(16, r1 - rb);
        for (int idx = threadIdx.x; idx < 16 * W; idx += 256) {
            const int rr = idx & 15, i = idx >> 4;
            x[i * 17 + rr] = rr < nr ? H[(rb + rr) + (int64_t)(s + i) * n] : 0.0;
        }
        __syncthreads();
        for (int i = 0; i < W; ++i) {
            const double xv = x[i * 17 + c];
            const double* ur = um + i * kWin + 6 * g;
#pragma unroll
            for (int q = 0; q < 6; ++q) acc[q] += xv * ur[q];
        }
        if (c < nr)
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                const int j = 6 * g + q;
                if (j < W) H[(rb + c) + (int64_t)(s + j) * n] = acc[q];
            }
    }
}

// ------------------------------------------------------------ one-wave Francis double shift
// The textbook double-shift QR (the oracle's hqr_francis) on an n x n Hessenberg matrix in LDS,
// run by ONE wave: every lane computes each 3x3 reflector redundantly from the same LDS words, so
// no step needs a workgroup barrier and scalar values never travel through LDS; a wave's LDS
// accesses execute in issue order, and compiler barriers keep them in program order.  kSchur:
// full-row/column updates and the orthogonal factor V accumulated (real Schur form T = V S V^T,
// block sizes in bs[]); otherwise the eigenvalue-only updates of the active block.  Exceptional
// shifts at 10 and 20 sweeps are given in unshifted form (no diagonal shifting), every reflector
// zeroes the bulge entries it consumes.  Eigenvalues go to wr/wi (complex pairs: -im, +im).

__device__ __forceinline__ int wave_max_int(int v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
    return v;
}

template <bool kSchur>
__device__ void wave_hqr(double* t, double* v, int n, int LD, int maxits, double* wr, double* wi, int* bs,
                         int& fail, int& total, int& maxsw) {
    const int lane = threadIdx.x & 63;
    auto T = [&](int i, int j) -> double& { return t[i + j * LD]; };
    auto V = [&](int i, int j) -> double& { return v[i + j * LD]; };
    const double eps = 2.220446049250313e-16;
    int nn = n - 1, its = 0;
    fail = 0;
    total = 0;
    maxsw = 0;
    EIGSOL_LDS_ORDER();
    while (nn >= 0) {
        int lm = 0;
        for (int l = 1 + lane; l <= nn; l += 64) {
            const double s0 = fabs(T(l - 1, l - 1)) + fabs(T(l, l));
            const double h = T(l, l - 1);
            if (h == 0.0 || fabs(h) <= eps * s0) lm = l;    // ascending per lane: the last is the max
        }
        const int l = __builtin_amdgcn_readfirstlane(wave_max_int(lm));
        EIGSOL_LDS_ORDER();
        if (l > 0 && lane == 0) T(l, l - 1) = 0.0;
        EIGSOL_LDS_ORDER();
        const double x = T(nn, nn);
        if (l == nn) {
            if (lane == 0) {
                wr[nn] = x;
                wi[nn] = 0.0;
                if (kSchur) bs[nn] = 1;
            }
            --nn;
            maxsw = max(maxsw, its);
            its = 0;
            EIGSOL_LDS_ORDER();
            continue;
        }
        const double y = T(nn - 1, nn - 1), w = T(nn, nn - 1) * T(nn - 1, nn);
        if (l == nn - 1) {
            if (lane == 0) {
                const double p = 0.5 * (y - x), q = p * p + w, z = sqrt(fabs(q));
                if (q >= 0.0) {
                    const double zz = p + (p >= 0 ? fabs(z) : -fabs(z));
                    wr[nn - 1] = wr[nn] = x + zz;
                    if (zz != 0.0) wr[nn] = x - w / zz;
                    wi[nn - 1] = wi[nn] = 0.0;
                } else {
                    wr[nn - 1] = wr[nn] = x + p;
                    wi[nn - 1] = -z;
                    wi[nn] = z;
                }
                if (kSchur) bs[nn] = bs[nn - 1] = 2;
            }
            nn -= 2;
            maxsw = max(maxsw, its);
            its = 0;
            EIGSOL_LDS_ORDER();
            continue;
        }
        if (its >= maxits) {
            fail = 1;
            break;
        }
        double xs = x, ys = y, ws = w;
        if (its == 10 || its == 20) {
            const double sc = fabs(T(nn, nn - 1)) + fabs(T(nn - 1, nn - 2));
            xs = ys = x + 0.75 * sc;
            ws = -0.4375 * sc * sc;
        }
        ++its;
        ++total;
        const int m = l;
        double p0, q0, r0;
        {
            const double z = T(m, m), rr = xs - z, ss = ys - z;
            p0 = (rr * ss - ws) / T(m + 1, m) + T(m, m + 1);
            q0 = T(m + 1, m + 1) - z - rr - ss;
            r0 = T(m + 2, m + 1);
            const double sc = fabs(p0) + fabs(q0) + fabs(r0);
            p0 /= sc; q0 /= sc; r0 /= sc;
        }
        for (int i = m + lane; i <= nn - 2; i += 64) {
            T(i + 2, i) = 0.0;
            if (i != m) T(i + 2, i - 1) = 0.0;
        }
        EIGSOL_LDS_ORDER();
        const int jend = kSchur ? n : nn + 1;      // left updates: to the matrix end (Schur) or the block end
        const int ibeg = kSchur ? 0 : l;           // right updates: from row 0 (Schur) or the block top
        for (int k = m; k <= nn - 1; ++k) {
            double p = p0, q = q0, r = r0, xk = 1.0;
            const bool three = k != nn - 1;
            if (k != m) {
                p = T(k, k - 1);
                q = T(k + 1, k - 1);
                r = three ? T(k + 2, k - 1) : 0.0;
                xk = fabs(p) + fabs(q) + fabs(r);
                if (xk != 0.0) { const double is = 1.0 / xk; p *= is; q *= is; r *= is; }
            }
            const double sg = (p >= 0 ? 1.0 : -1.0) * sqrt(p * p + q * q + r * r);
            if (sg == 0.0) continue;
            EIGSOL_LDS_ORDER();
            if (lane == 0) {
                if (k == m) {
                    if (l != m) T(k, k - 1) = -T(k, k - 1);
                } else {
                    T(k, k - 1) = -sg * xk;
                    T(k + 1, k - 1) = 0.0;
                    if (three) T(k + 2, k - 1) = 0.0;
                }
            }
            p += sg;
            const double isg = 1.0 / sg, ip = 1.0 / p;
            const double ax = p * isg, ay = q * isg, az = r * isg, bq = q * ip, br = r * ip;
            for (int j = k + lane; j < jend; j += 64) {
                double pp = T(k, j) + bq * T(k + 1, j);
                if (three) { pp += br * T(k + 2, j); T(k + 2, j) -= pp * az; }
                T(k + 1, j) -= pp * ay;
                T(k, j) -= pp * ax;
            }
            EIGSOL_LDS_ORDER();
            const int imax = nn < k + 3 ? nn : k + 3;
            for (int i = ibeg + lane; i <= imax; i += 64) {
                double pp = ax * T(i, k) + ay * T(i, k + 1);
                if (three) { pp += az * T(i, k + 2); T(i, k + 2) -= pp * br; }
                T(i, k + 1) -= pp * bq;
                T(i, k) -= pp;
            }
            if (kSchur)
                for (int i = lane; i < n; i += 64) {
                    double pp = ax * V(i, k) + ay * V(i, k + 1);
                    if (three) { pp += az * V(i, k + 2); V(i, k + 2) -= pp * br; }
                    V(i, k + 1) -= pp * bq;
                    V(i, k) -= pp;
                }
            EIGSOL_LDS_ORDER();
        }
    }
    maxsw = max(maxsw, its);
}

constexpr int kHqrWaveMax = 128;

// eigenvalues of an n x n (n <= 128) Hessenberg block: info = {fail, most sweeps per deflation, total}
__global__ __launch_bounds__(64) void hqr_wave_kernel(const double* Hin, int64_t ld, int n, double* wr, double* wi,
                                                      int maxits, int* info) {
    constexpr int LD = kHqrWaveMax + 1;
    __shared__ double t[kHqrWaveMax * LD];
    for (int e = threadIdx.x; e < n * n; e += 64) {
        const int i = e % n, j = e / n;
        t[i + j * LD] = Hin[i + (int64_t)j * ld];
    }
    __syncthreads();
    int fail, total, maxsw;
    wave_hqr<false>(t, nullptr, n, LD, maxits, wr, wi, nullptr, fail, total, maxsw);
    if (threadIdx.x == 0) {
        info[0] = fail;
        info[1] = maxsw;
        info[2] = total;
    }
}

// ------------------------------------------------------------ aggressive early deflation
// (Braman, Byers & Mathias, 2002; LAPACK xLAQR3's idea, restated for one wave.)
// The trailing nw x nw window T = H[kw:kw+nw, kw:kw+nw] of the active block is brought to real
// Schur form T = V S V^T (wave_hqr<true>).  Coupled to the rest of the block only through the
// spike s = H(kw, kw-1), the similarity turns that entry into the column s V(0, :)^T; trailing
// Schur blocks whose spike entries are negligible (|s v| <= ulp |lambda|, LAPACK's test) are
// deflated outright, scanning from the bottom up to the first block that is not.  When some
// deflate, the undeflated top part with its spike is reduced back to Hessenberg form (Householder,
// accumulated into V), the window and the new H(kw, kw-1) are written back and the caller applies
// V to the rows above the window (H[l:kw, kw:kw+nw] V, the only other part an eigenvalue-only
// iteration reads).  The undeflated eigenvalues are the next sweep's shifts.
constexpr int kAedMax = 96;

struct AedCtl {
    int nd;
    double beta, tau;
};

__global__ __launch_bounds__(64) void aed_kernel(double* H, int64_t n, int kw, int nw, int spike_valid, int maxits,
                                                 double* wr, double* wi, double* Vout, int* info) {
    constexpr int LD = kAedMax + 1;
    __shared__ double t[kAedMax * LD];
    __shared__ double v[kAedMax * LD];
    __shared__ double hv[kAedMax];        // Householder vector
    __shared__ double sp[kAedMax];
    __shared__ int bs[kAedMax];           // Schur block size ending at each row (1 or 2)
    __shared__ AedCtl c;
    const int tid = threadIdx.x, nt = 64;
    auto T = [&](int i, int j) -> double& { return t[i + j * LD]; };
    auto V = [&](int i, int j) -> double& { return v[i + j * LD]; };
    for (int e = tid; e < nw * nw; e += nt) {
        const int i = e % nw, j = e / nw;
        T(i, j) = H[(kw + i) + (int64_t)(kw + j) * n];
        V(i, j) = i == j ? 1.0 : 0.0;
    }
    const double spike = (spike_valid && kw > 0) ? H[kw + (int64_t)(kw - 1) * n] : 0.0;
    __syncthreads();
    const double eps = 2.220446049250313e-16;
    int fail, total, maxsw;
    // ---------------- phase A: real Schur form with V
    wave_hqr<true>(t, v, nw, LD, maxits, wr + kw, wi + kw, bs, fail, total, maxsw);
    __syncthreads();
    // ---------------- phase B: spike test from the bottom
    if (tid == 0) {
        int nd = 0;
        if (!fail) {
            const double smlnum = 2.2250738585072014e-308 * (nw / eps);
            int j = nw - 1;
            while (j >= 0) {
                const int b = bs[j];
                double foo, spk;
                if (b == 1) {
                    foo = fabs(T(j, j));
                    if (foo == 0.0) foo = fabs(spike);
                    spk = fabs(spike * V(0, j));
                } else {
                    foo = fabs(T(j, j)) + sqrt(fabs(T(j, j - 1))) * sqrt(fabs(T(j - 1, j)));
                    if (foo == 0.0) foo = fabs(spike);
                    spk = fmax(fabs(spike * V(0, j)), fabs(spike * V(0, j - 1)));
                }
                if (spk > fmax(smlnum, eps * foo)) break;
                nd += b;
                j -= b;
            }
        }
        c.nd = nd;
        c.beta = 0.0;
    }
    __syncthreads();
    const int nd = c.nd, m = nw - nd;
    // ---------------- phase C: undeflated part + spike back to Hessenberg form
    // apply P = I - tau hv hv^T (hv[0..len), hv[0] = 1) to rows/columns [o, o + len)
    auto reflect = [&](int o, int len, int jlo) {
        const double tau = c.tau;
        for (int j = jlo + tid; j < nw; j += nt) {                       // left: T[o:o+len, jlo:nw]
            double w = 0.0;
            for (int i = 0; i < len; ++i) w += hv[i] * T(o + i, j);
            w *= tau;
            for (int i = 0; i < len; ++i) T(o + i, j) -= w * hv[i];
        }
        __syncthreads();
        for (int i = tid; i < m; i += nt) {                              // right: T[0:m, o:o+len]
            double w = 0.0;
            for (int jj = 0; jj < len; ++jj) w += T(i, o + jj) * hv[jj];
            w *= tau;
            for (int jj = 0; jj < len; ++jj) T(i, o + jj) -= w * hv[jj];
        }
        for (int i = tid; i < nw; i += nt) {                             // V[:, o:o+len]
            double w = 0.0;
            for (int jj = 0; jj < len; ++jj) w += V(i, o + jj) * hv[jj];
            w *= tau;
            for (int jj = 0; jj < len; ++jj) V(i, o + jj) -= w * hv[jj];
        }
        __syncthreads();
    };
    // Householder vector of x[0..len) (thread 0): hv[0] = 1, c.tau, returns beta
    auto house = [&](const double* x, int len) -> double {
        const double alpha = x[0];
        double xn = 0.0;
        for (int i = 1; i < len; ++i) xn += x[i] * x[i];
        xn = sqrt(xn);
        hv[0] = 1.0;
        if (xn == 0.0) {
            c.tau = 0.0;
            for (int i = 1; i < len; ++i) hv[i] = 0.0;
            return alpha;
        }
        const double beta = -(alpha >= 0 ? 1.0 : -1.0) * sqrt(alpha * alpha + xn * xn);
        c.tau = (beta - alpha) / beta;
        const double sc = 1.0 / (alpha - beta);
        for (int i = 1; i < len; ++i) hv[i] = x[i] * sc;
        return beta;
    };
    if (nd > 0 && m > 0) {
        if (tid == 0) {
            for (int i = 0; i < m; ++i) sp[i] = spike * V(0, i);
            c.tau = 0.0;
            c.beta = m > 1 ? house(sp, m) : sp[0];
        }
        __syncthreads();
        if (m > 1 && c.tau != 0.0) reflect(0, m, 0);
        for (int col = 0; col + 2 < m; ++col) {
            if (tid == 0) {
                const double b = house(&T(col + 1, col), m - col - 1);
                T(col + 1, col) = b;
                for (int i = col + 2; i < m; ++i) T(i, col) = 0.0;
            }
            __syncthreads();
            if (c.tau != 0.0) reflect(col + 1, m - col - 1, col + 1);
        }
    }
    // ---------------- phase D: write back (only when something deflated)
    if (nd > 0) {
        for (int e = tid; e < nw * nw; e += nt) {
            const int i = e % nw, j = e / nw;
            H[(kw + i) + (int64_t)(kw + j) * n] = i > j + 1 ? 0.0 : T(i, j);
            Vout[e] = V(i, j);
        }
        if (tid == 0 && spike_valid && kw > 0) H[kw + (int64_t)(kw - 1) * n] = c.beta;
    }
    if (tid == 0) {
        info[0] = fail;
        info[1] = nd;
        info[2] = total;
        info[3] = m;
    }
}

// diagonal and subdiagonal of the block [0, ihi]: out[0..n) = h(i,i), out[n..2n) = h(i,i-1)
__global__ void diag_sub_kernel(const double* H, int64_t n, int ihi, double* out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i > ihi) return;
    out[i] = H[i + (int64_t)i * n];
    out[n + i] = i > 0 ? H[i + (int64_t)(i - 1) * n] : 0.0;
}

__global__ void zero_entry_kernel(double* H, int64_t n, int i, int j) { H[i + (int64_t)j * n] = 0.0; }

}  // namespace dev

// ---------------------------------------------------------------------------------- host loop
// eigenvalues of an n <= 128 Hessenberg block in LDS: the one-wave solver (EIGSOL_HQR_WAVE=0: the
// workgroup solver of qr.hip, for A/B)
static int hqr_small(hipStream_t st, const double* H, int64_t ld, int n, int maxits, double* wr, double* wi,
                     int* info) {
    static const bool wave = [] {
        const char* e = std::getenv("EIGSOL_HQR_WAVE");
        return !e || std::atoi(e) != 0;
    }();
    if (!wave) return hqr_lds(st, H, ld, n, maxits, wr, wi, info);
    hipLaunchKernelGGL(dev::hqr_wave_kernel, dim3(1), dim3(64), 0, st, H, ld, n, wr, wi, maxits, info);
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

static constexpr int kSmallDefault = 128;
// AED window: 40 measured best at 4096 (32: 2.63 s, 40: 2.58 s, 48: 2.60 s, 64: 2.92 s, 96: 4.28 s, off: 2.89 s);
// the window's one-wave Schur factorisation costs O(nw^3) latency-bound steps
static constexpr int kAedDefault = 40;   // blocks finished by the in-LDS solver (EIGSOL_QR_SMALL)

int francis_large_f64(eigsol_ctx* ctx, double* H, int64_t n, int maxits, double* wr, double* wi,
                      int32_t* sweeps_out, int32_t* fail_out) {
    hipStream_t st = ctx->stream;
    const double eps = 2.220446049250313e-16;
    double *dwr = nullptr, *dwi = nullptr, *dds = nullptr, *dU = nullptr, *dsh = nullptr;
    int* dinfo = nullptr;
    EIGSOL_HIP(hipMalloc(&dwr, n * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&dwi, n * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&dds, 2 * n * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&dU, dev::kWin * dev::kWin * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&dsh, 4 * dev::kMaxBulges * sizeof(double)));
    EIGSOL_HIP(hipMalloc(&dinfo, 64));
    std::vector<double> ds(2 * n), swr(2 * dev::kMaxBulges), swi(2 * dev::kMaxBulges);
    int rc = EIGSOL_OK;
    int sweeps = 0, failed = 0;
    int ihi = (int)n - 1;
    int stall = 0;               // sweeps on the current bottom block without a deflation
    // `sweeps` tracks the largest number of sweeps any single deflation needed
    const int max_stall = std::max(1, maxits);
    static const int kSmall = [] {
        const char* e = std::getenv("EIGSOL_QR_SMALL");
        return e ? std::max(16, std::min(128, std::atoi(e))) : kSmallDefault;
    }();
    static const bool stats = std::getenv("EIGSOL_QR_STATS") != nullptr;
    static const bool chase_v1 = std::getenv("EIGSOL_CHASE_V1") != nullptr;   // A/B: three-barrier chase
    static const int max_bulges = [] {                 // experiments: cap the bulges per chain
        const char* e = std::getenv("EIGSOL_QR_NB");
        return e ? std::max(1, std::min(dev::kMaxBulges, std::atoi(e))) : dev::kMaxBulges;
    }();
    long long st_steps = 0;
    static const int aed_win = [] {
        const char* e = std::getenv("EIGSOL_QR_AED");   // AED window (0: off)
        return e ? std::max(0, std::min(dev::kAedMax, std::atoi(e))) : kAedDefault;
    }();
    constexpr int kNibble = 14;   // % of the AED window deflated that skips the sweep (LAPACK's NIBBLE)
    int st_sweeps = 0, st_windows = 0, st_small = 0, st_small_rows = 0, st_aed = 0, st_aed_defl = 0;
    auto finish_small = [&](int l, int hi) -> int {
        const int m = hi - l + 1;
        EIGSOL_TRY(hqr_small(st, H + l + (int64_t)l * n, n, m, std::max(1, maxits), dwr + l, dwi + l, dinfo));
        int info[3];
        EIGSOL_HIP(hipMemcpyAsync(info, dinfo, sizeof(info), hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(hipStreamSynchronize(st));
        if (info[0]) failed = 1;
        sweeps = std::max(sweeps, info[1]);
        return EIGSOL_OK;
    };
    while (rc == EIGSOL_OK && ihi >= 0) {
        // deflation scan of [0, ihi]
        hipLaunchKernelGGL(dev::diag_sub_kernel, dim3((ihi + 256) / 256), dim3(256), 0, st, H, n, ihi, dds);
        if (hipMemcpyAsync(ds.data(), dds, 2 * n * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            rc = fail(EIGSOL_E_HIP, "francis: deflation scan");
            break;
        }
        int l = ihi;
        while (l > 0) {
            const double s0 = std::fabs(ds[l - 1]) + std::fabs(ds[l]);
            if (std::fabs(ds[n + l]) <= eps * s0 || ds[n + l] == 0.0) break;
            --l;
        }
        const int N = ihi - l + 1;
        if (N <= kSmall) {
            ++st_small;
            st_small_rows += N;
            rc = finish_small(l, ihi);
            ihi = l - 1;
            sweeps = std::max(sweeps, stall);
            stall = 0;
            continue;
        }
        if (++stall > max_stall) { failed = 1; sweeps = std::max(sweeps, stall); break; }
        // aggressive early deflation on the trailing window; its undeflated eigenvalues are the shifts
        int nb = std::min(max_bulges, std::max(1, N / 8));
        int ns = 2 * nb;
        bool have_shifts = false;
        if (aed_win > 0) {
            const int nw = std::min(aed_win, N);
            const int kw = ihi - nw + 1;
            hipLaunchKernelGGL(dev::aed_kernel, dim3(1), dim3(64), 0, st, H, n, kw, nw, kw > l ? 1 : 0, 60, dwr, dwi,
                               dU, dinfo);
            int info[4];
            std::vector<double> awr(nw), awi(nw);
            if (hipMemcpyAsync(info, dinfo, sizeof(info), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipMemcpyAsync(awr.data(), dwr + kw, nw * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipMemcpyAsync(awi.data(), dwi + kw, nw * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess) {
                rc = fail(EIGSOL_E_HIP, "francis: aed");
                break;
            }
            ++st_aed;
            if (!info[0]) {
                const int nd = info[1], m = info[3];
                if (nd > 0) {
                    st_aed_defl += nd;
                    const int nr = kw > l ? (kw - l + 15) / 16 : 0;
                    if (nr > 0)
                        hipLaunchKernelGGL(dev::win_gemm_fused, dim3(nr), dim3(256), 0, st, H, n, kw, nw, (int64_t)0,
                                           (int64_t)0, 0, (int64_t)l, (int64_t)kw, dU);
                    ihi = kw + m - 1;
                    sweeps = std::max(sweeps, stall);
                    stall = 0;
                    if (100 * nd >= kNibble * nw || m < 4) continue;   // enough deflated: look again first
                }
                // shifts: the bottom undeflated eigenvalues of the window
                const int N2 = ihi - l + 1;
                nb = std::min({max_bulges, std::max(1, N2 / 8), std::max(1, m / 2)});
                ns = 2 * nb;
                for (int i = 0; i < ns; ++i) {
                    swr[i] = awr[m - ns + i];
                    swi[i] = awi[m - ns + i];
                }
                have_shifts = true;
            }
        }
        if (!have_shifts) {
            // shifts: eigenvalues of the trailing 2nb x 2nb block
            rc = hqr_small(st, H + (ihi - ns + 1) + (int64_t)(ihi - ns + 1) * n, n, ns, 60, dwr + ihi - ns + 1,
                           dwi + ihi - ns + 1, dinfo);
            if (rc != EIGSOL_OK) break;
            if (hipMemcpyAsync(swr.data(), dwr + ihi - ns + 1, ns * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipMemcpyAsync(swi.data(), dwi + ihi - ns + 1, ns * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess) {
                rc = fail(EIGSOL_E_HIP, "francis: shifts");
                break;
            }
        }
        // pair the shifts: conjugate pairs stay together, reals are paired in order;
        // every 6th stalled sweep uses exceptional shifts from the bottom subdiagonal
        std::vector<double> sh(2 * nb);
        if (stall % 6 == 0) {
            for (int b = 0; b < nb; ++b) {
                const double sc = std::fabs(ds[n + ihi - b]) + std::fabs(ds[ihi - b]) + 1e-300;
                sh[2 * b] = ds[ihi - b] + 0.75 * sc;
                sh[2 * b + 1] = -0.4375 * sc * sc;
            }
        } else {
            std::vector<std::pair<double, double>> cplx_pairs, reals;
            for (int i = 0; i < ns; ++i) {
                if (swi[i] > 0.0) cplx_pairs.push_back({swr[i], swi[i]});
                else if (swi[i] == 0.0) reals.push_back({swr[i], 0.0});
            }
            int b = 0;
            for (auto& c : cplx_pairs) {
                if (b >= nb) break;
                sh[2 * b] = c.first;                    // xs = ys = a, ws = -b^2
                sh[2 * b + 1] = -c.second * c.second;
                ++b;
            }
            for (size_t i = 0; i + 1 < reals.size() && b < nb; i += 2) {
                const double s1 = reals[i].first, s2 = reals[i + 1].first;
                sh[2 * b] = 0.5 * (s1 + s2);            // xs = ys = (s1+s2)/2, ws = ((s1-s2)/2)^2
                sh[2 * b + 1] = 0.25 * (s1 - s2) * (s1 - s2);
                ++b;
            }
            for (; b < nb; ++b) {                       // odd leftovers: a real double shift
                const double s1 = reals.empty() ? ds[ihi] : reals.back().first;
                sh[2 * b] = s1;
                sh[2 * b + 1] = 0.0;
            }
        }
        if (hipMemcpyAsync(dsh, sh.data(), 2 * nb * sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess) {
            rc = fail(EIGSOL_E_HIP, "francis: shift upload");
            break;
        }
        ++st_sweeps;
        // chase the chain window by window
        const int T = (ihi - 1 - l) + 3 * (nb - 1) + 1;
        int t0 = 0;
        while (t0 < T) {
            int s;
            if (t0 <= 3 * (nb - 1)) s = std::max(0, l - 1);
            else s = std::max(0, l + t0 - 3 * (nb - 1) - 1);
            const int e = std::min(s + dev::kWin, ihi + 1);
            const int kmax = (e == ihi + 1) ? ihi - 1 : e - 4;
            int t1 = t0;
            while (t1 < T) {
                int blead = std::max(0, (l + t1 - (ihi - 1) + 2) / 3);   // first bulge not yet past ihi-1
                if (blead >= nb) { t1 = T; break; }
                const int k = l + t1 - 3 * blead;
                if (k > kmax) break;
                ++t1;
            }
            if (t1 == t0) { rc = fail(EIGSOL_E_SOLVER, "francis: window did not advance (internal error)"); break; }
            ++st_windows;
            st_steps += t1 - t0;
            dev::ChaseArgs ca{H, n, s, e, l, ihi, t0, t1, nb, dsh, dU};
            if (chase_v1) hipLaunchKernelGGL(dev::chase_kernel, dim3(1), dim3(1024), 0, st, ca);
            else hipLaunchKernelGGL(dev::chase_wave_kernel, dim3(1), dim3(1024), 0, st, ca);
            const int W = e - s;
            const int nlb = e <= ihi ? (ihi + 1 - e + 15) / 16 : 0;
            const int nrb = s > l ? (s - l + 15) / 16 : 0;
            if (nlb + nrb > 0)
                hipLaunchKernelGGL(dev::win_gemm_fused, dim3(nlb + nrb), dim3(256), 0, st, H, n, s, W, (int64_t)e,
                                   (int64_t)ihi + 1, nlb, (int64_t)l, (int64_t)s, dU);
            t0 = t1;
        }
        if (hipGetLastError() != hipSuccess) { rc = fail(EIGSOL_E_HIP, "francis: launch"); break; }
        // a deflation anywhere below resets the stall counter at the next scan
        hipLaunchKernelGGL(dev::diag_sub_kernel, dim3((ihi + 256) / 256), dim3(256), 0, st, H, n, ihi, dds);
        if (hipMemcpyAsync(ds.data(), dds, 2 * n * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            rc = fail(EIGSOL_E_HIP, "francis: deflation scan");
            break;
        }
        for (int k = ihi; k > l; --k)
            if (std::fabs(ds[n + k]) <= eps * (std::fabs(ds[k - 1]) + std::fabs(ds[k]))) {
                sweeps = std::max(sweeps, stall);
                stall = 0;
                break;
            }
    }
    if (rc == EIGSOL_OK) {
        if (hipMemcpyAsync(wr, dwr, n * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(wi, dwi, n * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            rc = fail(EIGSOL_E_HIP, "francis: download");
    }
    if (stats)
        std::fprintf(stderr, "francis: n=%lld sweeps=%d windows=%d steps=%lld small_blocks=%d small_rows=%d kSmall=%d "
                     "aed=%d aed_deflated=%d aed_win=%d\n",
                     (long long)n, st_sweeps, st_windows, st_steps, st_small, st_small_rows, kSmall, st_aed, st_aed_defl,
                     aed_win);
    for (void* p : {(void*)dwr, (void*)dwi, (void*)dds, (void*)dU, (void*)dsh, (void*)dinfo}) (void)hipFree(p);
    // iterations reported: sweeps spent on the slowest deflation (>= 1, the final check), so that
    // iterations <= maxIterations exactly when the iteration converged
    *sweeps_out = std::max(1, sweeps);
    *fail_out = failed;
    return rc;
}

}  // namespace eigsol

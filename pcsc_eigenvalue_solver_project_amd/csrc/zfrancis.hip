// Complex multishift QR sweeps (eigenvalues only) for std::complex<double> Hessenberg matrices.
//
// The reference's qr_eigenvalues_dense<std::complex<double>> (qr_eigenvalues.hpp:40-108) runs the
// unshifted iteration H <- R Q, which does not converge on general input (a complex N(0,1) matrix
// has eigenvalues of equal modulus).  This is the complex counterpart of francis.hip: the same
// small-bulge chase geometry, with complex arithmetic and shifts that need not come in conjugate
// pairs (LAPACK ZLAQR5's bulges):
//   * a bulge carries two shifts (s1, s2); its first column is (H - s1)(H - s2) e_l (scaled as in
//     ZLAQR1), and it is chased down by 3 x 3 complex Householder reflectors Q = I - tau v v^H
//     (ZLARFG's convention: Q^H (alpha, x) = (beta, 0) with beta real), the last step by a 2 x 2;
//   * bulges sit 3 rows apart and move together: every bulge's left update (Q^H on rows k..k+2)
//     runs before any right update (Q on columns k..k+2), which touch disjoint words within a
//     phase, and associativity makes the simultaneous step the product of the sequential ones;
//   * the chain is chased inside an LDS window [s, e) of at most 64 rows/columns (complex: H and
//     its accumulated unitary U take 2 x 64 KiB of LDS), one wave per bulge; the window's updates
//     outside it are applied afterwards as complex GEMMs over the columns right of the window
//     (U^H X) and the rows above it (X U);
//   * shifts: eigenvalues of the trailing 2 nb x 2 nb block; every 6th sweep without a deflation
//     uses exceptional shifts; active blocks of at most 64 rows are finished in LDS by a one-wave
//     single-shift QR (the ZLAHQR iteration: Wilkinson shift, exceptional shifts at iterations 10
//     and 20, Ahues-Tisseur deflation test).
// Deflation: |h(k,k-1)| <= eps (|h(k,k)| + |h(k-1,k-1)|) with |z| = |Re z| + |Im z| (ZLAHQR's cabs1).
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernels_common.hpp"

namespace eigsol {
namespace dev {

constexpr int kZWin = 64;         // window rows/columns
constexpr int kZSmall = 64;       // blocks finished by the one-wave solver
constexpr int kZMaxBulges = 32;   // per sweep (shifts from a <= 64 block); per window <= 16, one wave each
constexpr int kZMaxGroups = 4;    // bulge chains chased concurrently, one window (workgroup) each

__device__ __forceinline__ cplx cconj(cplx a) { return cplx{a.re, -a.im}; }
__device__ __forceinline__ double cabs1(cplx a) { return fabs(a.re) + fabs(a.im); }
__device__ __forceinline__ cplx cscale(cplx a, double s) { return cplx{a.re * s, a.im * s}; }
__device__ __forceinline__ cplx cmul_conj(cplx a, cplx b) {   // conj(a) * b
    return cplx{a.re * b.re + a.im * b.im, a.re * b.im - a.im * b.re};
}
__device__ __forceinline__ cplx csqrt_(cplx z) {
    const double r = hypot(z.re, z.im);
    if (r == 0.0) return cplx{0.0, 0.0};
    const double t = sqrt(0.5 * (r + fabs(z.re)));
    return z.re >= 0.0 ? cplx{t, z.im / (2.0 * t)} : cplx{fabs(z.im) / (2.0 * t), copysign(t, z.im)};
}
// robust quotient (Smith's algorithm)
__device__ __forceinline__ cplx cdiv_s(cplx a, cplx b) {
    if (fabs(b.re) >= fabs(b.im)) {
        const double r = b.im / b.re, d = b.re + b.im * r;
        return cplx{(a.re + a.im * r) / d, (a.im - a.re * r) / d};
    }
    const double r = b.re / b.im, d = b.re * r + b.im;
    return cplx{(a.re * r + a.im) / d, (a.im * r - a.re) / d};
}

__device__ __forceinline__ double rcp_nr(double x) {   // x != 0, finite, normal reciprocal
    double r = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-x, r, 1.0);
    return __builtin_fma(r, e, r);
}

// ZLARFG on (alpha, x1, x2) (x2 ignored when !three): Q = I - tau v v^H, v = (1, v1, v2),
// Q^H (alpha, x1, x2) = (beta, 0, 0).  tau = 0 (Q = I) when x = 0 and alpha is real.  The caller
// scales the input to O(1).
__device__ __forceinline__ void zhouse(cplx a, cplx x1, cplx x2, bool three, double& beta, cplx& tau, cplx& v1,
                                       cplx& v2) {
    const double xn2 = sq_abs(x1) + (three ? sq_abs(x2) : 0.0);
    if (xn2 == 0.0 && a.im == 0.0) {
        beta = a.re;
        tau = cplx{0.0, 0.0};
        v1 = v2 = cplx{0.0, 0.0};
        return;
    }
    const double an = sqrt(a.re * a.re + a.im * a.im + xn2);
    beta = a.re >= 0.0 ? -an : an;
    // the step's serial chain: reciprocals (v_rcp_f64 + two Newton steps, within an ulp or two)
    // instead of IEEE divisions; x / d by Smith's scaling with one reciprocal of the denominator
    const double ib = rcp_nr(beta);
    tau = cplx{(beta - a.re) * ib, -a.im * ib};
    const cplx d = cplx{a.re - beta, a.im};   // |d| >= |beta| > 0
    const bool re_big = fabs(d.re) >= fabs(d.im);
    const double r = re_big ? d.im * rcp_nr(d.re) : d.re * rcp_nr(d.im);
    const double id = rcp_nr(re_big ? __builtin_fma(d.im, r, d.re) : __builtin_fma(d.re, r, d.im));
    auto qt = [&](cplx x) -> cplx {
        return re_big ? cplx{__builtin_fma(x.im, r, x.re) * id, __builtin_fma(-x.re, r, x.im) * id}
                      : cplx{__builtin_fma(x.re, r, x.im) * id, __builtin_fma(x.im, r, -x.re) * id};
    };
    v1 = qt(x1);
    v2 = three ? qt(x2) : cplx{0.0, 0.0};
}

// sqrt of a in [2^-4, 2^4] (no range reduction): hardware reciprocal square root, then Goldschmidt /
// Newton corrections to full double precision (francis.hip's, restated for this translation unit)
__device__ __forceinline__ double sqrt_nr(double a) {
    const double y = __builtin_amdgcn_rsq(a);
    double s = a * y, h = 0.5 * y;
    const double r = __builtin_fma(-h, s, 0.5);
    s = __builtin_fma(s, r, s);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-s, s, a);
    s = __builtin_fma(d, h, s);
    d = __builtin_fma(-s, s, a);
    return __builtin_fma(d, h, s);
}

// zhouse for the 2 x 2 reflectors of the one-wave QR, on any scale: (alpha, x1) is scaled by a power
// of two (exact) so that its largest component lies in [1/2, 1), which puts the norm's square in
// [1/4, 4] and lets the hardware square root seed replace the IEEE sequence; tau and v are
// scale-free, beta is scaled back.  The same reflector as zhouse up to the rounding of the square
// root and reciprocals.
__device__ __forceinline__ void zhouse2_scaled(cplx a, cplx x1, double& beta, cplx& tau, cplx& v1) {
    const double m = fmax(fmax(fabs(a.re), fabs(a.im)), fmax(fabs(x1.re), fabs(x1.im)));
    const int ex = m > 0.0 ? __builtin_amdgcn_frexp_exp(m) : 0;
    const cplx as{__builtin_amdgcn_ldexp(a.re, -ex), __builtin_amdgcn_ldexp(a.im, -ex)};
    const cplx xs{__builtin_amdgcn_ldexp(x1.re, -ex), __builtin_amdgcn_ldexp(x1.im, -ex)};
    const double xn2 = sq_abs(xs);
    if (xn2 == 0.0 && as.im == 0.0) {
        beta = a.re;
        tau = cplx{0.0, 0.0};
        v1 = cplx{0.0, 0.0};
        return;
    }
    const double an = sqrt_nr(__builtin_fma(as.re, as.re, __builtin_fma(as.im, as.im, xn2)));
    const double bs = as.re >= 0.0 ? -an : an;
    const double ib = rcp_nr(bs);
    tau = cplx{(bs - as.re) * ib, -as.im * ib};
    const cplx d = cplx{as.re - bs, as.im};   // |d| >= |bs| > 0
    const bool re_big = fabs(d.re) >= fabs(d.im);
    const double r = re_big ? d.im * rcp_nr(d.re) : d.re * rcp_nr(d.im);
    const double id = rcp_nr(re_big ? __builtin_fma(d.im, r, d.re) : __builtin_fma(d.re, r, d.im));
    v1 = re_big ? cplx{__builtin_fma(xs.im, r, xs.re) * id, __builtin_fma(-xs.re, r, xs.im) * id}
                : cplx{__builtin_fma(xs.re, r, xs.im) * id, __builtin_fma(xs.im, r, -xs.re) * id};
    beta = __builtin_amdgcn_ldexp(bs, ex);
}

// ---------------------------------------------------------------- one-wave single-shift QR (n <= 64)
// Eigenvalues of an n x n Hessenberg block (ZLAHQR without Schur vectors; updates confined to the
// active block).  info[0] = 1 if some eigenvalue needed more than 30 max(10, n) iterations,
// info[1] = most iterations any eigenvalue took.
// One wave, so no barriers: a wave's LDS operations complete in program order, and the compiler
// fence keeps the program order.
#define EIGSOL_ZWAVE_ORDER() asm volatile("" ::: "memory")
// kSchur = false: eigenvalues only, updates confined to the active block (ZLAHQR with WANTT =
// WANTZ = false).  kSchur = true: the full Schur form T = V^H H V of the n x n block (left updates
// to column n-1, right updates from row 0, V accumulated: WANTT = WANTZ = true), for the AED.
// w[i] = the eigenvalue deflated at row i; failed / maxits / steps as for the kernel below.
// AED early stop (kSchur, spk >= 0 = cabs1 of the window's spike): when an eigenvalue deflates at
// the bottom row i its Schur vector column V(:, i) is final (later sweeps touch columns < i only),
// so the AED spike test is taken right there; the first eigenvalue that fails it ends the
// factorisation (stop = i; the rows above stay unreduced).  stop = -1: ran to completion.
// dtol: relative subdiagonal at which the block splits (ulp: ZLAHQR's test; the sweeps' shifts are
// computed with a looser one, EIGSOL_ZQR_SHIFT_TOL)
template <bool kSchur, bool kFast = true>
__device__ void zwave_hqr(cplx* h, cplx* v, int n, cplx* w, int& failed, int& maxits, int& steps,
                          double spk = -1.0, int* stop = nullptr, double dtol = 2.220446049250313e-16) {
    constexpr int lh = kZSmall + 1;
    const int ln = threadIdx.x;
    auto H = [&](int i, int j) -> cplx& { return h[i + j * lh]; };
    auto V = [&](int i, int j) -> cplx& { return v[i + j * lh]; };
    const double ulp = 2.220446049250313e-16, smlnum = 2.2250738585072014e-308 * ((double)n / ulp);
    const int itmax = 30 * max(10, n);
    int i = n - 1;
    failed = 0;
    maxits = 0;
    steps = 0;
    while (i >= 0) {
        int l = 0, its = 0;
        for (; its <= itmax; ++its) {
            // the largest k in (l, i] with a negligible subdiagonal (l if none): the serial downward
            // scan's answer, one k per lane, then a wave max
            int kf = l;
            for (int k = i - ln; k > l; k -= 64) {
                const cplx hk = H(k, k - 1);
                bool neg = cabs1(hk) <= smlnum;
                if (!neg) {
                    double tst = cabs1(H(k - 1, k - 1)) + cabs1(H(k, k));
                    if (tst == 0.0) {
                        if (k - 2 >= l) tst += fabs(H(k - 1, k - 2).re);
                        if (k + 1 <= i) tst += fabs(H(k + 1, k).re);
                    }
                    if (cabs1(hk) <= dtol * tst) {
                        const double ab = fmax(cabs1(hk), cabs1(H(k - 1, k))), ba = fmin(cabs1(hk), cabs1(H(k - 1, k)));
                        const cplx dd = sub(H(k - 1, k - 1), H(k, k));
                        const double aa = fmax(cabs1(H(k, k)), cabs1(dd)), bb = fmin(cabs1(H(k, k)), cabs1(dd));
                        const double s = aa + ab;
                        neg = ba * (ab / s) <= fmax(smlnum, dtol * (bb * (aa / s)));
                    }
                }
                if (neg) { kf = k; break; }
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) kf = max(kf, __shfl_xor(kf, off, 64));
            l = __builtin_amdgcn_readfirstlane(kf);
            EIGSOL_ZWAVE_ORDER();
            if (l > 0 && ln == 0) H(l, l - 1) = cplx{0.0, 0.0};
            EIGSOL_ZWAVE_ORDER();
            if (l >= i) break;
            // shift
            cplx t;
            if (its == 10) {
                t = add(cplx{0.75 * fabs(H(l + 1, l).re), 0.0}, H(l, l));
            } else if (its == 20) {
                t = add(cplx{0.75 * fabs(H(i, i - 1).re), 0.0}, H(i, i));
            } else {
                t = H(i, i);
                const cplx u = mul(csqrt_(H(i - 1, i)), csqrt_(H(i, i - 1)));
                double s = cabs1(u);
                if (s != 0.0) {
                    const cplx x = cscale(sub(H(i - 1, i - 1), t), 0.5);
                    const double sx = cabs1(x);
                    s = fmax(s, sx);
                    const cplx xs = cscale(x, 1.0 / s), us = cscale(u, 1.0 / s);
                    cplx y = cscale(csqrt_(add(mul(xs, xs), mul(us, us))), s);
                    if (sx > 0.0) {
                        const cplx xn = cscale(x, 1.0 / sx);
                        if (xn.re * y.re + xn.im * y.im < 0.0) y = cplx{-y.re, -y.im};
                    }
                    t = sub(t, mul(u, cdiv_s(u, add(x, y))));
                }
            }
            // single-shift sweep from l
            steps += i - l;
            for (int kk = l; kk < i; ++kk) {
                // kFast: the left update's rows kk, kk+1 (columns >= kk: this step's own stores go to
                // column kk-1) and V's columns kk, kk+1 are loaded first, so their LDS latency
                // overlaps the reflector's chain; the reflector is zhouse2_scaled's
                const int c = kk + ln;
                const bool cl = c <= (kSchur ? n - 1 : i);
                cplx a0{0.0, 0.0}, a1{0.0, 0.0}, w0{0.0, 0.0}, w1{0.0, 0.0};
                if (kFast) {
                    if (cl) { a0 = H(kk, c); a1 = H(kk + 1, c); }
                    if (kSchur && ln < n) { w0 = V(ln, kk); w1 = V(ln, kk + 1); }
                }
                cplx v0, v1;
                if (kk == l) {
                    const cplx h11s = sub(H(l, l), t);
                    const cplx h21 = H(l + 1, l);
                    const double s = cabs1(h11s) + cabs1(h21);
                    v0 = s > 0.0 ? cscale(h11s, 1.0 / s) : h11s;
                    v1 = s > 0.0 ? cscale(h21, 1.0 / s) : h21;
                } else {
                    v0 = H(kk, kk - 1);
                    v1 = H(kk + 1, kk - 1);
                }
                double beta;
                cplx tau, vv, unused;
                if (kFast) zhouse2_scaled(v0, v1, beta, tau, vv);
                else zhouse(v0, v1, cplx{0.0, 0.0}, false, beta, tau, vv, unused);
                EIGSOL_ZWAVE_ORDER();
                if (kk > l && ln == 0) {
                    H(kk, kk - 1) = cplx{beta, 0.0};
                    H(kk + 1, kk - 1) = cplx{0.0, 0.0};
                }
                const cplx ct = cconj(tau);
                {   // left: rows kk, kk+1, columns kk..i (Schur: ..n-1)
                    if (cl) {
                        if (!kFast) { a0 = H(kk, c); a1 = H(kk + 1, c); }
                        const cplx s = mul(ct, add(a0, cmul_conj(vv, a1)));
                        H(kk, c) = sub(a0, s);
                        H(kk + 1, c) = sub(a1, mul(s, vv));
                    }
                }
                EIGSOL_ZWAVE_ORDER();
                {   // right: columns kk, kk+1, rows l..min(kk+2, i) (Schur: from row 0; and V)
                    const int r = (kSchur ? 0 : l) + ln;
                    if (r <= min(kk + 2, i)) {
                        const cplx b0 = H(r, kk), b1 = H(r, kk + 1);
                        const cplx s = mul(tau, add(b0, mul(b1, vv)));
                        H(r, kk) = sub(b0, s);
                        H(r, kk + 1) = sub(b1, mul(s, cconj(vv)));
                    }
                    if (kSchur && ln < n) {
                        if (!kFast) { w0 = V(ln, kk); w1 = V(ln, kk + 1); }
                        const cplx s = mul(tau, add(w0, mul(w1, vv)));
                        V(ln, kk) = sub(w0, s);
                        V(ln, kk + 1) = sub(w1, mul(s, cconj(vv)));
                    }
                }
                EIGSOL_ZWAVE_ORDER();
            }
        }
        if (its > itmax) {
            failed = 1;
            break;
        }
        maxits = max(maxits, its);
        // H(l..i) has deflated to a single eigenvalue at i (l == i)
        if (ln == 0) w[i] = H(i, i);
        if (kSchur && spk >= 0.0) {
            double foo = cabs1(H(i, i));
            if (foo == 0.0) foo = spk;
            if (spk * cabs1(V(0, i)) > fmax(smlnum, ulp * foo)) {
                *stop = i;
                return;
            }
        }
        i = l - 1;
    }
    if (stop) *stop = -1;
    if (failed) {
        for (int r = ln; r <= i; r += 64) w[r] = H(r, r);   // best effort, flagged as failed
    }
}

// Eigenvalues of an n x n Hessenberg block (n <= 64) in LDS.  kFast: zwave_hqr's step (EIGSOL_ZQR_STEP)
template <bool kFast>
__global__ __launch_bounds__(64) void zhqr_wave_kernel(const cplx* Hin, int64_t ld, int n, cplx* w, int* info,
                                                       double dtol) {
    __shared__ cplx h[kZSmall * (kZSmall + 1)];
    constexpr int lh = kZSmall + 1;
    const int ln = threadIdx.x;
    for (int idx = ln; idx < n * n; idx += 64) h[(idx % n) + (idx / n) * lh] = Hin[(idx % n) + (int64_t)(idx / n) * ld];
    __syncthreads();
    int failed, maxits, steps;
    zwave_hqr<false, kFast>(h, nullptr, n, w, failed, maxits, steps, -1.0, nullptr, dtol);
    if (ln == 0) {
        info[0] = failed;
        info[1] = maxits;
    }
}

// ---------------------------------------------------------------- complex aggressive early deflation
// (ZLAQR3's idea, restated for one wave, as francis.hip's aed_kernel is for the real case.)  The
// trailing nw x nw window T = H[kw:kw+nw, kw:kw+nw] of the active block is brought to complex
// Schur form T = V S V^H (zwave_hqr<true>).  The window is coupled to the rest of the block only
// through the spike s = H(kw, kw-1), which the similarity turns into the column s conj(V(0, :))^T;
// trailing eigenvalues whose spike entry is negligible (cabs1(s) cabs1(V(0, j)) <=
// max(smlnum, ulp cabs1(S(j, j))), ZLAQR3's test; no reordering) deflate outright, scanning from
// the bottom to the first that does not.  When some deflate, the undeflated top part with its
// spike is reduced back to Hessenberg form by complex Householder reflectors (ZLARFG convention,
// accumulated into V), the window and the new spike are written back, and the caller applies V to
// the rows of the block above the window (H[l:kw, kw:kw+nw] V).  w[kw + i] = S(i, i): the
// deflated eigenvalues are final, the undeflated ones are the next sweep's shifts.
// info = {fail, deflated, iterations, undeflated, steps}.
struct ZAedCtl {
    cplx tau, spike;
    double beta;
    int fail, maxsw, steps, nd;
};
// 256 threads: wave 0 runs the one-wave Schur factorisation, the spike test and the Householder
// vectors; the reflector applications of the back-reduction take four lanes per row / column (each
// sums every fourth term, the four partial sums meet as (s0 + s1) + (s2 + s3)).  Round 4: the
// one-wave version summed each dot product in one chain.
constexpr int kZAedThreads = 256;
__device__ __forceinline__ cplx quad_sum(cplx sq, int q) {   // (s0 + s1) + (s2 + s3) over the 4-lane group
    const cplx o1{__shfl_xor(sq.re, 1, 64), __shfl_xor(sq.im, 1, 64)};
    const cplx pr = (q & 1) ? add(o1, sq) : add(sq, o1);
    const cplx o2{__shfl_xor(pr.re, 2, 64), __shfl_xor(pr.im, 2, 64)};
    return (q & 2) ? add(o2, pr) : add(pr, o2);
}
// Concurrent shifts (round 5, as francis.hip's ShiftJob): workgroup 1 of the launch copies the
// pre-AED trailing ns x ns block [kb, kb + ns) into its LDS, raises flag = epoch, and computes its
// eigenvalues on one wave while workgroup 0 runs the AED; workgroup 0 writes the window back only
// after the flag.
struct ZShiftJob {
    int kb, ns;
    double dtol;
    cplx* w;
    int* info;            // {fail, most sweeps per deflation, -, wait timed out}
    unsigned* flag;
    unsigned epoch;
};

template <bool kFast>
__global__ __launch_bounds__(kZAedThreads) void zaed_kernel(cplx* Hg, int64_t n, int kw, int nw, int spike_valid,
                                                            int early, cplx* w, cplx* Vout, int* info, ZShiftJob sj) {
    constexpr int lh = kZSmall + 1;
    constexpr int NT = kZAedThreads;
    __shared__ cplx t[kZSmall * lh];
    __shared__ cplx v[kZSmall * lh];
    __shared__ cplx hv[kZSmall];
    __shared__ cplx sp[kZSmall];
    __shared__ ZAedCtl c;
    const int tid = threadIdx.x, ln = tid & 63, wv0 = tid < 64;
    if (blockIdx.x == 1) {   // the concurrent shifts
        const int ns = sj.ns;
        for (int e = tid; e < ns * ns; e += NT) t[(e % ns) + (e / ns) * lh] = Hg[(sj.kb + e % ns) + (int64_t)(sj.kb + e / ns) * n];
        __syncthreads();
        if (tid == 0) __hip_atomic_store(sj.flag, sj.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        if (wv0) {
            int fail, maxsw, steps;
            zwave_hqr<false, kFast>(t, nullptr, ns, sj.w, fail, maxsw, steps, -1.0, nullptr, sj.dtol);
            if (ln == 0) {
                sj.info[0] = fail;
                sj.info[1] = maxsw;
            }
        }
        return;
    }
    const int grp = tid >> 2, q = tid & 3;   // 64 groups of four lanes
    auto T = [&](int i, int j) -> cplx& { return t[i + j * lh]; };
    auto V = [&](int i, int j) -> cplx& { return v[i + j * lh]; };
    for (int e = tid; e < nw * nw; e += NT) {
        const int i = e % nw, j = e / nw;
        T(i, j) = Hg[(kw + i) + (int64_t)(kw + j) * n];
        V(i, j) = i == j ? cplx{1.0, 0.0} : cplx{0.0, 0.0};
    }
    const cplx spike = (spike_valid && kw > 0) ? Hg[kw + (int64_t)(kw - 1) * n] : cplx{0.0, 0.0};
    __syncthreads();
    if (wv0) {
        int fail, maxsw, steps, stop = -1;
        zwave_hqr<true, kFast>(t, v, nw, w + kw, fail, maxsw, steps, early ? cabs1(spike) : -1.0, &stop);
        // spike test, one window row per lane; deflated = the trailing run of negligible entries
        const double ulp = 2.220446049250313e-16, smlnum = 2.2250738585072014e-308 * ((double)nw / ulp);
        int nd = 0;
        if (early) {
            nd = fail ? 0 : nw - 1 - stop;   // the spike test ran inside the factorisation
        } else if (!fail) {
            bool keep = false;
            if (ln < nw) {
                double foo = cabs1(T(ln, ln));
                if (foo == 0.0) foo = cabs1(spike);
                keep = cabs1(spike) * cabs1(V(0, ln)) > fmax(smlnum, ulp * foo);
            }
            const unsigned long long km = __ballot(keep);
            nd = km ? nw - 1 - (63 - __clzll(km)) : nw;
        }
        if (ln == 0) {
            c.fail = fail;
            c.maxsw = maxsw;
            c.steps = steps;
            c.nd = nd;
        }
    }
    __syncthreads();
    const int nd = c.nd;
    const int m = nw - nd;
    // undeflated part + spike back to Hessenberg form.  Q = I - tau hv hv^H (hv[0] = 1) applied
    // as Q^H T on rows [o, o + len) (columns [jlo, nw)), then T Q on T's rows [0, m) and V Q
    auto reflect = [&](int o, int len, int jlo) {
        const cplx tau = c.tau, ctau = cconj(tau);
        for (int j = jlo + grp; j < nw; j += NT / 4) {
            cplx sq{0.0, 0.0};
            for (int i = q; i < len; i += 4) sq = add(sq, cmul_conj(hv[i], T(o + i, j)));
            const cplx wv = mul(ctau, quad_sum(sq, q));
            for (int i = q; i < len; i += 4) T(o + i, j) = sub(T(o + i, j), mul(hv[i], wv));
        }
        __syncthreads();
        if (grp < nw) {
            cplx sq{0.0, 0.0};
            for (int jj = q; jj < len; jj += 4) sq = add(sq, mul(V(grp, o + jj), hv[jj]));
            const cplx wv = mul(tau, quad_sum(sq, q));
            for (int jj = q; jj < len; jj += 4) V(grp, o + jj) = sub(V(grp, o + jj), mul(wv, cconj(hv[jj])));
        }
        if (grp < m) {
            cplx sq{0.0, 0.0};
            for (int jj = q; jj < len; jj += 4) sq = add(sq, mul(T(grp, o + jj), hv[jj]));
            const cplx wv = mul(tau, quad_sum(sq, q));
            for (int jj = q; jj < len; jj += 4) T(grp, o + jj) = sub(T(grp, o + jj), mul(wv, cconj(hv[jj])));
        }
        __syncthreads();
    };
    // ZLARFG of x[0..len) by wave 0: hv, c.tau (0: Q = I), c.beta (real); every thread calls it
    auto house = [&](const cplx* x, int len) {
        cplx tau{0.0, 0.0}, sc{0.0, 0.0};
        double beta = 0.0;
        if (wv0) {
            const cplx alpha = x[0];
            double part = 0.0;
            for (int i = 1 + ln; i < len; i += 64) part += sq_abs(x[i]);
            const double xn2 = wave_sum(part);
            beta = alpha.re;
            if (xn2 != 0.0 || alpha.im != 0.0) {
                beta = -copysign(sqrt(sq_abs(alpha) + xn2), alpha.re);
                tau = cplx{(beta - alpha.re) / beta, -alpha.im / beta};
                sc = cdiv_s(cplx{1.0, 0.0}, cplx{alpha.re - beta, alpha.im});
            }
        }
        __syncthreads();   // x may alias a T column the stores below do not touch; order the reads
        if (wv0) {
            for (int i = 1 + ln; i < len; i += 64) hv[i] = mul(x[i], sc);
            if (ln == 0) {
                hv[0] = cplx{1.0, 0.0};
                c.tau = tau;
                c.beta = beta;
            }
        }
        __syncthreads();
    };
    if (nd > 0 && m > 0) {
        for (int i = tid; i < m; i += NT) sp[i] = mul(spike, cconj(V(0, i)));
        __syncthreads();
        if (m > 1) {
            house(sp, m);
            if (tid == 0) c.spike = cplx{c.beta, 0.0};
            __syncthreads();
            if (c.tau.re != 0.0 || c.tau.im != 0.0) reflect(0, m, 0);
        } else {
            if (tid == 0) c.spike = sp[0];
            __syncthreads();
        }
        for (int col = 0; col + 2 < m; ++col) {
            house(&T(col + 1, col), m - col - 1);
            if (tid == 0) T(col + 1, col) = cplx{c.beta, 0.0};
            for (int i = col + 2 + tid; i < m; i += NT) T(i, col) = cplx{0.0, 0.0};
            __syncthreads();
            if (c.tau.re != 0.0 || c.tau.im != 0.0) reflect(col + 1, m - col - 1, col + 1);
        }
    } else if (tid == 0) {
        c.spike = cplx{0.0, 0.0};
    }
    __syncthreads();
    if (gridDim.x > 1) {   // the concurrent shifts' copy is taken before the write-back (bounded wait)
        if (tid == 0) {
            int timed_out = 0;
            if (nd > 0) {
                const long long t0 = wall_clock64();
                while (__hip_atomic_load(sj.flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != sj.epoch) {
                    if (wall_clock64() - t0 > 100000000ll) { timed_out = 1; break; }
                    __builtin_amdgcn_s_sleep(2);
                }
            }
            sj.info[3] = timed_out;
        }
        __syncthreads();
    }
    if (nd > 0) {
        for (int e = tid; e < nw * nw; e += NT) {
            const int i = e % nw, j = e / nw;
            Hg[(kw + i) + (int64_t)(kw + j) * n] = i > j + 1 ? cplx{0.0, 0.0} : T(i, j);
            Vout[e] = V(i, j);
        }
        if (tid == 0 && spike_valid && kw > 0) Hg[kw + (int64_t)(kw - 1) * n] = c.spike;
    }
    if (tid == 0) {
        info[0] = c.fail;
        info[1] = nd;
        info[2] = c.maxsw;
        info[3] = m;
        info[4] = c.steps;
    }
}

// ---------------------------------------------------------------- windowed multishift chase
struct ZChaseWin {
    int s, e;          // window [s, e)
    int t0, t1;        // chase steps of this launch (chain-relative)
    int nb;            // bulges of the chain
    const cplx* shifts;   // 2 per bulge
    cplx* U;           // out: (e - s)^2, column-major
};
struct ZChaseBatch {   // one workgroup per window; the windows are disjoint
    cplx* H;
    int64_t n;
    int l, ihi;
    ZChaseWin w[kZMaxGroups];
};
struct ZChaseArgs {
    cplx* H;
    int64_t n;
    int l, ihi;
    int s, e, t0, t1, nb;
    const cplx* shifts;
    cplx* U;
};

__global__ __launch_bounds__(1024) void zchase_kernel(ZChaseBatch b) {
    const ZChaseWin wd = b.w[blockIdx.x];
    const ZChaseArgs a{b.H, b.n, b.l, b.ihi, wd.s, wd.e, wd.t0, wd.t1, wd.nb, wd.shifts, wd.U};
    __shared__ cplx h[kZWin * (kZWin + 1)];
    __shared__ cplx u[kZWin * kZWin];
    constexpr int lh = kZWin + 1, lu = kZWin;
    const int W = a.e - a.s;
    const int tid = threadIdx.x;
    auto Hw = [&](int i, int j) -> cplx& { return h[(i - a.s) + (j - a.s) * lh]; };
    for (int idx = tid; idx < W * W; idx += 1024) {
        const int i = idx % W, j = idx / W;
        h[i + j * lh] = a.H[(a.s + i) + (int64_t)(a.s + j) * a.n];
        u[i + j * lu] = (i == j) ? cplx{1.0, 0.0} : cplx{0.0, 0.0};
    }
    __syncthreads();
    const int l = a.l, ihi = a.ihi;
    const int wv = tid >> 6, ln = tid & 63;
    const int rlo = max(l, a.s);
    for (int t = a.t0; t < a.t1; ++t) {
        const int k = l + t - 3 * wv;
        const bool live = wv < a.nb && k >= l && k <= ihi - 1;
        const bool three = k != ihi - 1;
        double beta = 0.0;
        cplx tau{0.0, 0.0}, v1{0.0, 0.0}, v2{0.0, 0.0};
        bool act = false;
        if (live) {
            cplx p, q, r;
            int ex = 0;
            if (k == l) {
                const cplx s1 = a.shifts[2 * wv], s2 = a.shifts[2 * wv + 1];
                const cplx h11 = Hw(l, l), h21 = Hw(l + 1, l), h12 = Hw(l, l + 1), h22 = Hw(l + 1, l + 1);
                const double s = cabs1(sub(h11, s2)) + cabs1(h21);
                if (s == 0.0) {
                    p = q = r = cplx{0.0, 0.0};
                } else {
                    const cplx h21s = cscale(h21, 1.0 / s);
                    p = add(mul(h21s, h12), mul(sub(h11, s1), cscale(sub(h11, s2), 1.0 / s)));
                    q = mul(h21s, sub(add(h11, h22), add(s1, s2)));
                    r = three ? mul(h21s, Hw(l + 2, l + 1)) : cplx{0.0, 0.0};
                }
            } else {
                p = Hw(k, k - 1);
                q = Hw(k + 1, k - 1);
                r = three ? Hw(k + 2, k - 1) : cplx{0.0, 0.0};
            }
            const double mx = fmax(fmax(cabs1(p), cabs1(q)), cabs1(r));
            if (mx > 0.0) {
                ex = __builtin_amdgcn_frexp_exp(mx);   // exact power-of-two scaling into [1/2, 1)
                p = cplx{ldexp(p.re, -ex), ldexp(p.im, -ex)};
                q = cplx{ldexp(q.re, -ex), ldexp(q.im, -ex)};
                r = cplx{ldexp(r.re, -ex), ldexp(r.im, -ex)};
                zhouse(p, q, r, three, beta, tau, v1, v2);
                act = true;
                if (k != l && ln == 0) {
                    Hw(k, k - 1) = cplx{ldexp(beta, ex), 0.0};
                    Hw(k + 1, k - 1) = cplx{0.0, 0.0};
                    if (three) Hw(k + 2, k - 1) = cplx{0.0, 0.0};
                }
                const cplx ct = cconj(tau);
                // phase A: left update (Q^H on rows k..k+2), columns [k, e)
                const int c = k + ln;
                if (c < a.e) {
                    const cplx x0 = Hw(k, c), x1 = Hw(k + 1, c);
                    const cplx x2 = three ? Hw(k + 2, c) : cplx{0.0, 0.0};
                    cplx wsum = add(x0, cmul_conj(v1, x1));
                    if (three) wsum = add(wsum, cmul_conj(v2, x2));
                    const cplx s = mul(ct, wsum);
                    Hw(k, c) = sub(x0, s);
                    Hw(k + 1, c) = sub(x1, mul(s, v1));
                    if (three) Hw(k + 2, c) = sub(x2, mul(s, v2));
                }
                // U <- U Q on columns k..k+2 (window-relative), every row
                if (ln < W) {
                    const int kk = k - a.s;
                    const cplx y0 = u[ln + kk * lu], y1 = u[ln + (kk + 1) * lu];
                    const cplx y2 = three ? u[ln + (kk + 2) * lu] : cplx{0.0, 0.0};
                    cplx wsum = add(y0, mul(y1, v1));
                    if (three) wsum = add(wsum, mul(y2, v2));
                    const cplx s = mul(tau, wsum);
                    u[ln + kk * lu] = sub(y0, s);
                    u[ln + (kk + 1) * lu] = sub(y1, mul(s, cconj(v1)));
                    if (three) u[ln + (kk + 2) * lu] = sub(y2, mul(s, cconj(v2)));
                }
            }
        }
        __syncthreads();
        if (act) {   // phase B: right update (Q on columns k..k+2), rows [rlo, min(k + 3, ihi)]
            const int r = rlo + ln;
            if (r <= min(k + 3, ihi)) {
                const cplx y0 = Hw(r, k), y1 = Hw(r, k + 1);
                const cplx y2 = three ? Hw(r, k + 2) : cplx{0.0, 0.0};
                cplx wsum = add(y0, mul(y1, v1));
                if (three) wsum = add(wsum, mul(y2, v2));
                const cplx s = mul(tau, wsum);
                Hw(r, k) = sub(y0, s);
                Hw(r, k + 1) = sub(y1, mul(s, cconj(v1)));
                if (three) Hw(r, k + 2) = sub(y2, mul(s, cconj(v2)));
            }
        }
        __syncthreads();
    }
    for (int idx = tid; idx < W * W; idx += 1024) {
        const int i = idx % W, j = idx / W;
        a.H[(a.s + i) + (int64_t)(a.s + j) * a.n] = h[i + j * lh];
        a.U[idx] = u[i + j * lu];
    }
}

// Delayed window updates.  left: H(s:s+W, cols) <- U^H H(s:s+W, cols) for the columns [lo, hi);
// right: H(rows, s:s+W) <- H(rows, s:s+W) U for the rows [lo, hi).  8 output columns (rows) per
// workgroup of 128 threads; U and the panel staged in LDS, each thread a 4 x 1 register tile of
// the output (the LDS pitches keep a wave's 16-byte reads on distinct banks).  The regions are a
// few hundred columns, so narrow workgroups are what spreads a launch over the CUs: 32 columns per
// workgroup 0.436 s, 16: 0.39 s, 8: 0.37 s for the 1024^2 complex QR.
constexpr int kZG = 8;   // output columns (left) / rows (right) per workgroup
constexpr int kZB = kZG / 8;   // register-tile columns per thread
struct ZWinGemm {
    int s, W;          // window rows/columns [s, s + W)
    int64_t lo, hi;    // left: columns [lo, hi); right: rows [lo, hi)
    int blk0;          // first workgroup of this window
    const cplx* U;
};
struct ZWinGemmBatch {   // left regions of different windows own disjoint rows, right regions disjoint columns
    cplx* H;
    int64_t n;
    int nw;
    ZWinGemm w[kZMaxGroups];
};
template <bool kLeft>
__global__ __launch_bounds__(128) void zwin_gemm_kernel(ZWinGemmBatch bt) {
    int g = 0;
#pragma unroll
    for (int q = 1; q < kZMaxGroups; ++q)
        if (q < bt.nw && (int)blockIdx.x >= bt.w[q].blk0) g = q;
    cplx* H = bt.H;
    const int64_t n = bt.n;
    const int s = bt.w[g].s, W = bt.w[g].W;
    const int64_t lo = bt.w[g].lo, hi = bt.w[g].hi;
    const cplx* U = bt.w[g].U;
    constexpr int LU = kZWin + 1;    // U pitch
    constexpr int LX = kZWin + 1;    // panel pitch
    __shared__ cplx us[kZWin * LU];
    __shared__ cplx xs[kZG * LX];
    const int tid = threadIdx.x;
    const int64_t b0 = lo + (int64_t)(blockIdx.x - bt.w[g].blk0) * kZG;
    const int nb = (int)std::min<int64_t>(kZG, hi - b0);
    for (int idx = tid; idx < W * W; idx += 128) us[(idx % W) + (idx / W) * LU] = U[idx];
    if (kLeft) {   // xs[r + c LX] = H(s + r, b0 + c)
        for (int idx = tid; idx < W * kZG; idx += 128) {
            const int r = idx % W, c = idx / W;
            xs[r + c * LX] = c < nb ? H[(s + r) + (b0 + c) * n] : cplx{0.0, 0.0};
        }
    } else {       // xs[r + c LX] = H(b0 + c, s + r)  (row c of the block, transposed)
        for (int idx = tid; idx < W * kZG; idx += 128) {
            const int c = idx % kZG, r = idx / kZG;
            xs[r + c * LX] = c < nb ? H[(b0 + c) + (int64_t)(s + r) * n] : cplx{0.0, 0.0};
        }
    }
    __syncthreads();
    // output tile: 4 window indices (i0 + 16 a) x 4 block columns/rows (c0 + 8 b)
    const int i0 = tid & 15, c0 = tid >> 4;   // 16 x 8 threads
    cplx acc[4][kZB];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < kZB; ++b) acc[a][b] = cplx{0.0, 0.0};
    for (int r = 0; r < W; ++r) {
        cplx uu[4], xx[kZB];
#pragma unroll
        for (int a = 0; a < 4; ++a) uu[a] = kLeft ? us[r + (i0 + 16 * a) * LU] : us[r + (i0 + 16 * a) * LU];
#pragma unroll
        for (int b = 0; b < kZB; ++b) xx[b] = xs[r + (c0 + 8 * b) * LX];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < kZB; ++b)
                acc[a][b] = add(acc[a][b], kLeft ? cmul_conj(uu[a], xx[b]) : mul(xx[b], uu[a]));
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < kZB; ++b) {
            const int i = i0 + 16 * a, c = c0 + 8 * b;
            if (i < W && c < nb) {
                if (kLeft) H[(s + i) + (b0 + c) * n] = acc[a][b];          // (U^H X)(i, c)
                else H[(b0 + c) + (int64_t)(s + i) * n] = acc[a][b];       // (X U)(c, i)
            }
        }
}

// The same delayed updates on the fp64 matrix cores (v_mfma_f64_16x16x4_f64): a complex tile
// product is four real ones on split re/im planes.  64 output columns (left) / rows (right) per
// workgroup of 4 waves, each wave a 16-wide strip against the window's 4 row tiles; U (and the
// left panel) staged in LDS as re/im planes at a pitch of kZWin + 2 (the real kernel's
// conflict-free pitch).  D layout: lane L, register r holds D[(L >> 4) + 4 r][L & 15].
typedef double zdbl4 __attribute__((ext_vector_type(4)));
constexpr int kZUP = kZWin + 2;
constexpr int kZMG = 64;   // outputs per workgroup
constexpr int kZMT = 4 * kZMG;   // threads: one wave per 16 outputs
template <bool kLeft>
__global__ __launch_bounds__(kZMT) void zwin_gemm_mfma(ZWinGemmBatch bt) {
    __shared__ double ur[kZWin * kZUP], ui[kZWin * kZUP];
    __shared__ double xr_s[kLeft ? kZMG * kZUP : 1], xi_s[kLeft ? kZMG * kZUP : 1];
    int g = 0;
#pragma unroll
    for (int q = 1; q < kZMaxGroups; ++q)
        if (q < bt.nw && (int)blockIdx.x >= bt.w[q].blk0) g = q;
    const ZWinGemm w = bt.w[g];
    const int W = w.W;
    const int64_t n = bt.n;
    const int64_t base = w.lo + (int64_t)((int)blockIdx.x - w.blk0) * kZMG;
    const int cnt = (int)min<int64_t>(kZMG, w.hi - base);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int li = lane & 15, lk = lane >> 4;
    constexpr int kKs = kZWin / 4;
    // right: this lane's X(r_j, k), k = lk, lk + 4, ... (issued first, consumed last)
    cplx xv[kLeft ? 1 : kKs];
    const int rj = 16 * wave + li;
    const bool rv = rj < cnt;
    if constexpr (!kLeft) {
        const cplx* xrow = bt.H + (base + min(rj, max(cnt - 1, 0))) + (int64_t)w.s * n;
#pragma unroll
        for (int q = 0; q < kKs; ++q) xv[q] = xrow[(int64_t)min(4 * q + lk, W - 1) * n];
    }
    {
        constexpr int kPU = kZWin * kZWin / kZMT;
        cplx tu[kPU];
#pragma unroll
        for (int q = 0; q < kPU; ++q) {
            const int idx = threadIdx.x + kZMT * q;
            const int k = idx % kZWin, rho = idx / kZWin;
            tu[q] = w.U[min(k, W - 1) + min(rho, W - 1) * W];
        }
        if constexpr (kLeft) {
            constexpr int kPX = kZWin * kZMG / kZMT;
            cplx tx[kPX];
#pragma unroll
            for (int q = 0; q < kPX; ++q) {
                const int idx = threadIdx.x + kZMT * q;
                const int k = idx % kZWin, c = idx / kZWin;
                tx[q] = bt.H[(w.s + min(k, W - 1)) + (base + min(c, max(cnt - 1, 0))) * n];
            }
#pragma unroll
            for (int q = 0; q < kPX; ++q) {
                const int idx = threadIdx.x + kZMT * q;
                const int k = idx % kZWin, c = idx / kZWin;
                const bool ok = k < W && c < cnt;
                xr_s[k + c * kZUP] = ok ? tx[q].re : 0.0;
                xi_s[k + c * kZUP] = ok ? tx[q].im : 0.0;
            }
        }
#pragma unroll
        for (int q = 0; q < kPU; ++q) {
            const int idx = threadIdx.x + kZMT * q;
            const int k = idx % kZWin, rho = idx / kZWin;
            const bool ok = k < W && rho < W;
            ur[k + rho * kZUP] = ok ? tu[q].re : 0.0;
            ui[k + rho * kZUP] = ok ? tu[q].im : 0.0;
        }
    }
    __syncthreads();
    constexpr int kT = kZWin / 16;
    zdbl4 aR[kT], aI[kT];
#pragma unroll
    for (int t = 0; t < kT; ++t) aR[t] = aI[t] = zdbl4{0.0, 0.0, 0.0, 0.0};
    if constexpr (kLeft) {
        // D[i][j] = sum_k X(k, c_i) conj(U(k, rho_j)): re = Xr Ur + Xi Ui, im = Xi Ur - Xr Ui
        const int co = (16 * wave + li) * kZUP;
#pragma unroll
        for (int q = 0; q < kKs; ++q) {   // rows k >= W of both LDS images are zero
            const int k = 4 * q + lk;
            const double xr = xr_s[co + k], xi = xi_s[co + k];
            double br[kT], bi[kT];
#pragma unroll
            for (int t = 0; t < kT; ++t) {
                br[t] = ur[k + (16 * t + li) * kZUP];
                bi[t] = ui[k + (16 * t + li) * kZUP];
            }
#pragma unroll
            for (int t = 0; t < kT; ++t) {
                aR[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(xr, br[t], aR[t], 0, 0, 0);
                aR[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(xi, bi[t], aR[t], 0, 0, 0);
                aI[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(xi, br[t], aI[t], 0, 0, 0);
                aI[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(-xr, bi[t], aI[t], 0, 0, 0);
            }
        }
#pragma unroll
        for (int t = 0; t < kT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int c = 16 * wave + lk + 4 * r, rho = 16 * t + li;
                if (c < cnt && rho < W) bt.H[(w.s + rho) + (base + c) * n] = cplx{aR[t][r], aI[t][r]};
            }
    } else {
        // D[i][j] = sum_k U(k, rho_i) X(r_j, k): re = Ur Xr - Ui Xi, im = Ur Xi + Ui Xr
#pragma unroll
        for (int q = 0; q < kKs; ++q) {
            const int k = 4 * q + lk;
            const bool ok = rv && k < W;
            const double xr = ok ? xv[q].re : 0.0, xi = ok ? xv[q].im : 0.0;
            double ar[kT], ai[kT];
#pragma unroll
            for (int t = 0; t < kT; ++t) {
                ar[t] = ur[k + (16 * t + li) * kZUP];
                ai[t] = ui[k + (16 * t + li) * kZUP];
            }
#pragma unroll
            for (int t = 0; t < kT; ++t) {
                aR[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[t], xr, aR[t], 0, 0, 0);
                aR[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(-ai[t], xi, aR[t], 0, 0, 0);
                aI[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[t], xi, aI[t], 0, 0, 0);
                aI[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[t], xr, aI[t], 0, 0, 0);
            }
        }
#pragma unroll
        for (int t = 0; t < kT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int rho = 16 * t + lk + 4 * r;
                if (rv && rho < W) bt.H[(base + rj) + (int64_t)(w.s + rho) * n] = cplx{aR[t][r], aI[t][r]};
            }
    }
}

__global__ void zdiag_sub_kernel(const cplx* H, int64_t n, int ihi, cplx* out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i > ihi) return;
    out[i] = H[i + (int64_t)i * n];
    out[n + i] = i > 0 ? H[i + (int64_t)(i - 1) * n] : cplx{0.0, 0.0};
}

}  // namespace dev

static double cabs1_h(const cplx& a) { return std::fabs(a.re) + std::fabs(a.im); }

// AED window (EIGSOL_ZQR_AED overrides, 0: off).  Early-stop AED, 32 bulges in 4 chains: window
// 32 / 48 / 64 at 1024^2 0.292 / 0.287 / 0.320 s; 48 vs 64 at 4096^2 2.65 / 2.75 s.  Without the
// AED: 1024^2 0.37-0.42 s, 4096^2 4.4 s; the full-Schur AED (EIGSOL_ZQR_AED_FULL=1) 0.54 / 4.4 s.
static constexpr int kZAedDefault = 48;

// eigenvalues of the complex Hessenberg matrix H (device, n x n, leading dimension n; destroyed)
int francis_large_c128(eigsol_ctx* ctx, cplx* H, int64_t n, int maxits, cplx* w_host, int32_t* sweeps_out,
                       int32_t* fail_out) {
    hipStream_t st = ctx->stream;
    const double eps = 2.220446049250313e-16;
    cplx *dw = nullptr, *dds = nullptr, *dU = nullptr, *dsh = nullptr;
    int* dinfo = nullptr;
    int rc = EIGSOL_OK;
    if (hipMalloc(&dw, n * sizeof(cplx)) != hipSuccess || hipMalloc(&dds, 2 * n * sizeof(cplx)) != hipSuccess ||
        hipMalloc(&dU, (size_t)dev::kZMaxGroups * dev::kZWin * dev::kZWin * sizeof(cplx)) != hipSuccess ||
        hipMalloc(&dsh, 2 * dev::kZMaxBulges * sizeof(cplx)) != hipSuccess || hipMalloc(&dinfo, 64) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "complex QR: hipMalloc");
    cplx* dV = nullptr;   // the AED window's unitary factor
    if (rc == EIGSOL_OK && hipMalloc(&dV, (size_t)dev::kZSmall * dev::kZSmall * sizeof(cplx)) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "complex QR: hipMalloc");
    cplx* dsw = nullptr;       // concurrent shifts
    int* dsinfo = nullptr;
    unsigned* dflag = nullptr;
    unsigned flag_epoch = 0;
    if (rc == EIGSOL_OK && (hipMalloc(&dsw, dev::kZSmall * sizeof(cplx)) != hipSuccess || hipMalloc(&dsinfo, 64) != hipSuccess ||
                            hipMalloc(&dflag, 64) != hipSuccess || hipMemsetAsync(dflag, 0, 64, st) != hipSuccess))
        rc = fail(EIGSOL_E_HIP, "complex QR: hipMalloc");
    // every per-sweep transfer goes through pinned host memory: a pageable hipMemcpyAsync is staged
    // by the runtime and waited for with a sleeping wait, ~1 ms per copy (round-4 kernel trace of
    // 4096^2: 1.12 s of 2.8 s idle after such copies, tools/gap_analysis.py)
    struct Staging {
        int info[8];
        int cinfo[4];
        cplx aw[dev::kZSmall];
        cplx cw[dev::kZSmall];   // concurrent shifts
        cplx sh[2 * dev::kZMaxBulges];
    };
    Staging* hp = nullptr;
    cplx* ds = nullptr;   // deflation scans: diagonal [0, n), subdiagonal [n, 2n)
    if (rc == EIGSOL_OK && (hipHostMalloc(&hp, sizeof(Staging), hipHostMallocDefault) != hipSuccess ||
                            hipHostMalloc(&ds, 2 * n * sizeof(cplx), hipHostMallocDefault) != hipSuccess))
        rc = fail(EIGSOL_E_HIP, "complex QR: hipHostMalloc");
    cplx* const aw = hp ? hp->aw : nullptr;
    int sweeps = 0, failed = 0, stall = 0;
    int st_sweeps = 0, st_aed = 0, st_aed_defl = 0, st_small = 0, st_conc = 0;
    // concurrent shifts (EIGSOL_ZQR_CONC): 0 off (default), 1 when the AED deflates nothing (bitwise
    // the sequential sweeps), 2 also after a deflation (the pre-AED block's spectrum without the
    // deflated eigenvalues, LAPACK xLAQR0's undeflated shifts).  Measured and left off (round 5,
    // tools/zqr_conc_ab.sh, 4096^2): a launch ends with its slower workgroup, and the 64 x 64
    // complex shift QR (~2.5 ms) outlasts the AED (~1 ms), so every AED - also the 70 % after which
    // the sweep is skipped - waits for it: 1.569 s -> 2.285 s (mode 1, same 122 sweeps, bitwise the
    // same eigenvalues), 2.085 s (mode 2, 131 sweeps)
    static const int conc_mode = [] {
        const char* e = std::getenv("EIGSOL_ZQR_CONC");
        return e ? std::atoi(e) : 0;
    }();
    static const bool stats = std::getenv("EIGSOL_QR_STATS") != nullptr;
    // the one-wave QR's step (zwave_hqr kFast, EIGSOL_ZQR_STEP): 1 loads ahead and takes the scaled
    // reflector (default), 0 the round-5 step
    static const bool fast_step = [] {
        const char* e = std::getenv("EIGSOL_ZQR_STEP");
        return !(e && !std::strcmp(e, "0"));
    }();
    int ihi = (int)n - 1;
    const int max_stall = std::max(1, maxits);
    // the shifts' QR splits at a looser relative subdiagonal than the eigenvalues' (EIGSOL_ZQR_SHIFT_TOL;
    // the real path's round-4 grid, francis.hip, put its optimum at 1e-4)
    static const double shift_tol = [] {
        const char* e = std::getenv("EIGSOL_ZQR_SHIFT_TOL");
        return e ? std::max(2.220446049250313e-16, std::atof(e)) : 2.220446049250313e-16;
    }();
    auto small = [&](int l, int hi, cplx* wdst, int info[2], double dtol = 2.220446049250313e-16) -> int {
        hipLaunchKernelGGL(fast_step ? dev::zhqr_wave_kernel<true> : dev::zhqr_wave_kernel<false>, dim3(1), dim3(64), 0,
                           st, H + l + (int64_t)l * n, (int64_t)n, hi - l + 1, wdst, dinfo, dtol);
        EIGSOL_HIP(hipMemcpyAsync(hp->info, dinfo, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(stream_wait(st));
        info[0] = hp->info[0];
        info[1] = hp->info[1];
        return EIGSOL_OK;
    };
    auto scan = [&]() -> int {   // only the ihi + 1 leading entries of each half travel
        hipLaunchKernelGGL(dev::zdiag_sub_kernel, dim3((ihi + 256) / 256), dim3(256), 0, st, H, (int64_t)n, ihi, dds);
        EIGSOL_HIP(hipMemcpyAsync(ds, dds, (ihi + 1) * sizeof(cplx), hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(hipMemcpyAsync(ds + n, dds + n, (ihi + 1) * sizeof(cplx), hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(stream_wait(st));
        return EIGSOL_OK;
    };
    bool scanned = false;   // the previous sweep's closing scan is still current (nothing ran since)
    while (rc == EIGSOL_OK && ihi >= 0) {
        if (!scanned && (rc = scan()) != EIGSOL_OK) break;
        scanned = false;
        int l = ihi;
        while (l > 0) {
            const cplx sd = ds[n + l];
            if (cabs1_h(sd) <= eps * (cabs1_h(ds[l - 1]) + cabs1_h(ds[l])) || (sd.re == 0.0 && sd.im == 0.0)) break;
            --l;
        }
        const int N = ihi - l + 1;
        if (N <= dev::kZSmall) {
            int info[2];
            ++st_small;
            if ((rc = small(l, ihi, dw + l, info)) != EIGSOL_OK) break;
            if (info[0]) failed = 1;
            sweeps = std::max({sweeps, stall, info[1]});
            stall = 0;
            ihi = l - 1;
            continue;
        }
        if (++stall > max_stall) { failed = 1; sweeps = std::max(sweeps, stall); break; }
        // up to 32 bulges per sweep (64 shifts) in C chains of at most 8 (a chain's 3 nb rows must
        // leave its 64-row window room to advance), the chains chased concurrently in disjoint
        // windows.  With the AED (round 3) 32 bulges in 4 chains beat 16 in 2: 1024^2 0.31 -> 0.29 s,
        // 2048^2 0.93 -> 0.77 s, 4096^2 3.28 -> 2.65 s (tools/qr_ab_round3.sh)
        static const int max_nb = [] {
            const char* e = std::getenv("EIGSOL_ZQR_NB");
            return e ? std::max(1, std::min(dev::kZMaxBulges, std::atoi(e))) : 32;
        }();
        static const int max_groups = [] {
            const char* e = std::getenv("EIGSOL_ZQR_GROUPS");
            return e ? std::max(1, std::min(dev::kZMaxGroups, std::atoi(e))) : 4;
        }();
        // aggressive early deflation on the trailing window; its undeflated eigenvalues are the shifts
        static const int aed_win = [] {
            const char* e = std::getenv("EIGSOL_ZQR_AED");   // AED window (0: off)
            return e ? std::max(0, std::min(dev::kZSmall, std::atoi(e))) : kZAedDefault;
        }();
        static const int nibble = [] {   // % of the window deflated that skips the sweep (LAPACK's NIBBLE)
            const char* e = std::getenv("EIGSOL_ZQR_NIBBLE");
            return e ? std::max(1, std::atoi(e)) : 14;
        }();
        // EIGSOL_ZQR_AED_FULL=1: the window's whole Schur form (LAPACK's AED, the undeflated
        // eigenvalues become the shifts); default: early stop at the first undeflatable eigenvalue,
        // shifts from the trailing block afterwards
        static const bool aed_full = [] {
            const char* e = std::getenv("EIGSOL_ZQR_AED_FULL");
            return e && std::atoi(e) != 0;
        }();
        // bulges of a sweep on an active block of Nact rows (C chains of nbg): the shift count 2 nb
        auto plan = [&](int Nact, int cap, int& C, int& nbg) {
            int nb = std::min(max_nb, std::max(1, Nact / 16));
            if (cap >= 2) nb = std::min(nb, cap / 2);
            C = std::max(1, std::min({max_groups, (nb + 7) / 8, 1 + Nact / (4 * (dev::kZWin + 12))}));
            nbg = std::max(1, std::min(8, nb / C));
            return nbg * C;
        };
        int m_aed = 0;
        int conc_n = 0;            // candidate shifts from the concurrent workgroup (in hp->cw)
        if (aed_win >= 4) {
            const int nw = std::min(aed_win, N);
            const int kw = ihi - nw + 1;
            int C0, nbg0;
            const int ns0 = 2 * plan(N, 0, C0, nbg0);   // the shift block if the AED deflates nothing
            const bool conc = conc_mode > 0 && !aed_full && ns0 >= 2 && ns0 <= dev::kZSmall;
            dev::ZShiftJob sj{ihi - ns0 + 1, ns0, shift_tol, dsw, dsinfo, dflag, ++flag_epoch};
            hipLaunchKernelGGL(fast_step ? dev::zaed_kernel<true> : dev::zaed_kernel<false>, dim3(conc ? 2 : 1),
                               dim3(dev::kZAedThreads), 0, st, H, (int64_t)n, kw, nw,
                               kw > l ? 1 : 0, aed_full ? 0 : 1, dw, dV, dinfo, sj);
            int* info = hp->info;
            if (hipMemcpyAsync(info, dinfo, 5 * sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipMemcpyAsync(aw, dw + kw, nw * sizeof(cplx), hipMemcpyDeviceToHost, st) != hipSuccess ||
                (conc && (hipMemcpyAsync(hp->cinfo, dsinfo, 4 * sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
                          hipMemcpyAsync(hp->cw, dsw, ns0 * sizeof(cplx), hipMemcpyDeviceToHost, st) != hipSuccess)) ||
                stream_wait(st) != hipSuccess) {
                rc = fail(EIGSOL_E_HIP, "complex QR: aed");
                break;
            }
            ++st_aed;
            const bool conc_ok = conc && !hp->cinfo[0] && !hp->cinfo[3];
            if (conc_ok && !info[0] && info[1] == 0) conc_n = ns0;   // pre-AED block = post-AED block
            if (conc_ok && conc_mode > 1 && !info[0] && info[1] > 0 && ns0 >= nw) {
                // the deflated eigenvalues (bottom of the window) removed from the block's spectrum by
                // nearest match; the rest keep their order
                const int nd = info[1];
                std::vector<int> used(ns0, 0);
                for (int j = nw - nd; j < nw; ++j) {
                    int best = -1;
                    double bd = 0.0;
                    for (int i = 0; i < ns0; ++i) {
                        if (used[i]) continue;
                        const double d = std::hypot(hp->cw[i].re - aw[j].re, hp->cw[i].im - aw[j].im);
                        if (best < 0 || d < bd) { best = i; bd = d; }
                    }
                    if (best >= 0) used[best] = 1;
                }
                int k = 0;
                for (int i = 0; i < ns0; ++i)
                    if (!used[i]) hp->cw[k++] = hp->cw[i];
                conc_n = k;
            }
            if (!info[0]) {
                const int nd = info[1];
                m_aed = aed_full ? info[3] : 0;   // early-stopped windows carry no shifts
                if (nd > 0) {
                    st_aed_defl += nd;
                    if (kw > l) {   // rows of the block above the window: H[l, kw) x [kw, kw + nw) V
                        dev::ZWinGemmBatch rb{H, (int64_t)n, 1, {}};
                        rb.w[0] = dev::ZWinGemm{kw, nw, (int64_t)l, (int64_t)kw, 0, dV};
                        hipLaunchKernelGGL(dev::zwin_gemm_mfma<false>, dim3((kw - l + dev::kZMG - 1) / dev::kZMG),
                                           dim3(dev::kZMT), 0, st, rb);
                    }
                    const int m = info[3];
                    ihi = kw + m - 1;
                    sweeps = std::max(sweeps, stall);
                    stall = 0;
                    if (100 * nd >= nibble * nw || m < 2 || ihi - l + 1 <= dev::kZSmall) continue;
                }
            }
        }
        const int Nact = ihi - l + 1;   // after the AED's deflations
        int C, nbg;
        int nb = plan(Nact, m_aed >= 2 ? m_aed : (conc_n >= 2 ? conc_n : 0), C, nbg);
        const int ns = 2 * nb;
        cplx* const sh = hp->sh;   // ns values; the chase reads them from dsh
        // every 6th sweep without a deflation: exceptional shifts (LAPACK's KEXSH; stall is 0 right
        // after the AED deflated, and such a sweep takes the regular shifts).  EIGSOL_ZQR_EXC_LEGACY=1:
        // round 3's test, which also took stall == 0 (ad hoc shifts after every partial deflation)
        static const bool exc_legacy = [] {
            const char* e = std::getenv("EIGSOL_ZQR_EXC_LEGACY");
            return e && std::atoi(e) != 0;
        }();
        bool exceptional = exc_legacy ? stall % 6 == 0 : (stall > 0 && stall % 6 == 0);
        if (!exceptional && m_aed >= 2) {   // the bottom undeflated eigenvalues of the AED window
            for (int i = 0; i < ns; ++i) sh[i] = aw[m_aed - ns + i];
            if (hipMemcpyAsync(dsh, sh, ns * sizeof(cplx), hipMemcpyHostToDevice, st) != hipSuccess) {
                rc = fail(EIGSOL_E_HIP, "complex QR: shift upload");
                break;
            }
        } else if (!exceptional && conc_n >= ns) {   // the concurrent workgroup's (bottom ns of them)
            for (int i = 0; i < ns; ++i) sh[i] = hp->cw[conc_n - ns + i];
            ++st_conc;
            if (hipMemcpyAsync(dsh, sh, ns * sizeof(cplx), hipMemcpyHostToDevice, st) != hipSuccess) {
                rc = fail(EIGSOL_E_HIP, "complex QR: shift upload");
                break;
            }
        } else if (!exceptional) {
            int info[2];
            if ((rc = small(ihi - ns + 1, ihi, dsh, info, shift_tol)) != EIGSOL_OK) break;   // shifts written to dsh
            if (info[0]) exceptional = true;
        }
        if (exceptional) {
            for (int b = 0; b < nb; ++b) {
                const cplx d = ds[ihi - b];
                const double sc = cabs1_h(ds[n + ihi - b]) + cabs1_h(d) * 1e-3 + 1e-300;
                sh[2 * b] = cplx{d.re + 0.75 * sc, d.im};
                sh[2 * b + 1] = cplx{d.re - 0.75 * sc, d.im};
            }
            if (hipMemcpyAsync(dsh, sh, ns * sizeof(cplx), hipMemcpyHostToDevice, st) != hipSuccess) {
                rc = fail(EIGSOL_E_HIP, "complex QR: shift upload");
                break;
            }
        }
        ++st_sweeps;
        // chase: chain g starts G steps after chain g-1 (windows stay disjoint); a round advances
        // every started chain's window by the same number of steps
        const int G = dev::kZWin + 3 * nbg;
        const int Tg = (ihi - 1 - l) + 3 * (nbg - 1) + 1;   // steps of one chain
        const int T = (C - 1) * G + Tg;
        int t0 = 0;
        while (t0 < T && rc == EIGSOL_OK) {
            dev::ZChaseBatch cb{H, (int64_t)n, l, ihi, {}};
            int t1 = T, nwin = 0;
            int g_act[dev::kZMaxGroups];
            for (int g = 0; g < C; ++g) {
                const int tl = t0 - g * G;
                if (tl < 0) { t1 = std::min(t1, g * G); break; }    // later chains start at a round boundary
                if (tl >= Tg) continue;                              // chain done
                const int s = tl <= 3 * (nbg - 1) ? std::max(0, l - 1) : std::max(0, l + tl - 3 * (nbg - 1) - 1);
                const int e = std::min(s + dev::kZWin, ihi + 1);
                const int kmax = (e == ihi + 1) ? ihi - 1 : e - 4;
                int tl1 = tl;
                while (tl1 < Tg) {
                    const int blead = std::max(0, (l + tl1 - (ihi - 1) + 2) / 3);   // first bulge not past ihi-1
                    if (blead >= nbg) { tl1 = Tg; break; }
                    if (l + tl1 - 3 * blead > kmax) break;
                    ++tl1;
                }
                t1 = std::min(t1, tl1 + g * G);
                cb.w[nwin] = dev::ZChaseWin{s, e, tl, 0, nbg, dsh + 2 * g * nbg, dU + (size_t)nwin * dev::kZWin * dev::kZWin};
                g_act[nwin++] = g;
            }
            if (nwin == 0 && t1 > t0) { t0 = t1; continue; }   // every started chain done, the next not yet due
            if (t1 <= t0 || nwin == 0) { rc = fail(EIGSOL_E_SOLVER, "complex QR: window did not advance (internal error)"); break; }
            for (int q = 0; q < nwin; ++q) {
                cb.w[q].t1 = t1 - g_act[q] * G;
                if (q > 0 && cb.w[q].e > cb.w[q - 1].s) { rc = fail(EIGSOL_E_SOLVER, "complex QR: windows overlap (internal error)"); break; }
            }
            if (rc != EIGSOL_OK) break;
            hipLaunchKernelGGL(dev::zchase_kernel, dim3(nwin), dim3(1024), 0, st, cb);
            // delayed updates: every left region, then every right region (U_a^H X U_b = (U_a^H X) U_b)
            // on the matrix cores by default; EIGSOL_ZGEMM_VALU=1: the VALU kernel (8-column workgroups)
            static const bool valu = [] {
                const char* e = std::getenv("EIGSOL_ZGEMM_VALU");
                return e && std::atoi(e) != 0;
            }();
            const int per = valu ? dev::kZG : dev::kZMG;
            dev::ZWinGemmBatch lb{H, (int64_t)n, 0, {}}, rb{H, (int64_t)n, 0, {}};
            int nlb = 0, nrb = 0;
            for (int q = 0; q < nwin; ++q) {
                const dev::ZChaseWin& w = cb.w[q];
                const int W = w.e - w.s;
                if (w.e <= ihi) {
                    lb.w[lb.nw++] = dev::ZWinGemm{w.s, W, (int64_t)w.e, (int64_t)ihi + 1, nlb, w.U};
                    nlb += (ihi + 1 - w.e + per - 1) / per;
                }
                if (w.s > l) {
                    rb.w[rb.nw++] = dev::ZWinGemm{w.s, W, (int64_t)l, (int64_t)w.s, nrb, w.U};
                    nrb += (w.s - l + per - 1) / per;
                }
            }
            if (valu) {
                if (nlb > 0) hipLaunchKernelGGL(dev::zwin_gemm_kernel<true>, dim3(nlb), dim3(128), 0, st, lb);
                if (nrb > 0) hipLaunchKernelGGL(dev::zwin_gemm_kernel<false>, dim3(nrb), dim3(128), 0, st, rb);
            } else {
                if (nlb > 0) hipLaunchKernelGGL(dev::zwin_gemm_mfma<true>, dim3(nlb), dim3(dev::kZMT), 0, st, lb);
                if (nrb > 0) hipLaunchKernelGGL(dev::zwin_gemm_mfma<false>, dim3(nrb), dim3(dev::kZMT), 0, st, rb);
            }
            t0 = t1;
        }
        if (hipGetLastError() != hipSuccess) { rc = fail(EIGSOL_E_HIP, "complex QR: launch"); break; }
        if ((rc = scan()) != EIGSOL_OK) break;
        scanned = true;
        for (int k = ihi; k > l; --k)
            if (cabs1_h(ds[n + k]) <= eps * (cabs1_h(ds[k - 1]) + cabs1_h(ds[k]))) {
                sweeps = std::max(sweeps, stall);
                stall = 0;
                break;
            }
    }
    if (rc == EIGSOL_OK) {
        if (hipMemcpyAsync(w_host, dw, n * sizeof(cplx), hipMemcpyDeviceToHost, st) != hipSuccess ||
            stream_wait(st) != hipSuccess)
            rc = fail(EIGSOL_E_HIP, "complex QR: download");
    }
    if (stats)
        std::fprintf(stderr, "complex francis: n=%lld sweeps=%d small_blocks=%d aed=%d aed_deflated=%d conc_shifts=%d\n",
                     (long long)n, st_sweeps, st_small, st_aed, st_aed_defl, st_conc);
    for (void* p : {(void*)dw, (void*)dds, (void*)dU, (void*)dsh, (void*)dinfo, (void*)dV, (void*)dsw, (void*)dsinfo,
                    (void*)dflag})
        if (p) (void)hipFree(p);
    if (ds) (void)hipHostFree(ds);
    if (hp) (void)hipHostFree(hp);
    *sweeps_out = std::max(1, sweeps);
    *fail_out = failed;
    return rc;
}

}  // namespace eigsol

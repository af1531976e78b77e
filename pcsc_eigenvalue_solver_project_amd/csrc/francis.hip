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
// outside the window are applied afterwards as small GEMMs on the fp64 matrix cores,
//     H(s:e, e:ihi]   <- U^T H(s:e, e:ihi]        H[l, s) x [s, e) <- H[l, s) x [s, e) U,
// so every HBM element of the active block is touched O(1) times per window instead of once per
// reflector.  Concurrency: the chain is split into C groups of 4+ bulges spaced kWin + 3 nbg
// rows apart, each chased in its own window by its own workgroup (one CU each) in the same
// launch; windows never overlap, and their delayed updates commute (left regions own disjoint
// rows, right regions disjoint columns; a left region of a trailing window meets the right
// region of a leading one, so all lefts run before all rights).  A chase step costs ~1.15 us
// with 4 bulges and ~2.05 us with 16 (instruction issue of 16 waves on 4 SIMDs), so 4-bulge
// groups move 1.8x more bulges per microsecond.  Shifts: the undeflated eigenvalues of the
// aggressive-early-deflation window (aed_kernel), else the trailing block's; blocks of at most
// 128 rows are finished entirely in LDS.  Deflation: |h(k,k-1)| <= eps (|h(k,k)| + |h(k-1,k-1)|).
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
constexpr int kMaxBulges = 48;   // shifts per sweep / 2 (at most 16 per window: one wave each; the
                                 // shifts' block of 2 nb <= 96 rows fits the one-wave solver)

// compiler-only ordering of LDS accesses (one wave's LDS operations execute in issue order)
#define EIGSOL_LDS_ORDER() asm volatile("" ::: "memory")

typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int kMaxGroups = 8;   // bulge groups chased concurrently, one window (workgroup) each

// One window of a chase round: group g's bulges j = 0..nb-1 sit at rows k = l + t - 3 j for the
// group-local steps t in [t0, t1); the window [s, e) holds them for the whole round.
struct ChaseWin {
    int s, e;         // window [s, e)
    int t0, t1;       // group-local chase steps of this round
    int nb;           // bulges of the group
    const double* shifts;   // per bulge: xs (= ys) and ws of the shift pair
    double* U;        // out: (e - s)^2 accumulated factor, column-major
};
struct ChaseArgs {
    double* H;
    int64_t n;        // leading dimension
    int l, ihi;       // active block
    ChaseWin w[kMaxGroups];   // window of workgroup blockIdx.x
};

// Reciprocal without the IEEE division sequence: v_rcp_f64 and two Newton steps (within an ulp
// or two; a Householder reflector built from it is orthogonal to the same order).  x != 0, finite.
// sqrt of a in [2^-4, 2^4] (no range reduction): hardware reciprocal square root, then Goldschmidt /
// Newton corrections to full double precision (v_sqrt_f64 alone is far from it)
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

__device__ __forceinline__ double rcp_nr(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-x, r, 1.0);
    return __builtin_fma(r, e, r);
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
// U is only ever right-multiplied, and bulge b touches U's columns k..k+2 for three consecutive
// steps before bulge b+1 takes them over, so wave b keeps its three columns in registers: per
// step it loads the new column k+2 (stored by bulge b-1 at the end of its previous phase A) and
// stores the column it drops, instead of reading and writing all three.
__global__ __launch_bounds__(1024) void chase_wave_kernel(ChaseArgs ca) {
    const ChaseWin a = ca.w[blockIdx.x];
    __shared__ double h[kWin * (kWin + 1)];
    __shared__ double u[kWin * kWin];
    __shared__ double trash[4];   // target of the stores of lanes past a row / column range (branch-free)
    const int W = a.e - a.s;
    // compile-time LDS pitches (odd for H): every LDS address is shifts and adds of wave-uniform
    // and per-lane terms, no integer multiplies on a step's path
    constexpr int ldh = kWin + 1, ldu = kWin;
    const int tid = threadIdx.x;
    auto Hw = [&](int i, int j) -> double& { return h[(i - a.s) + (j - a.s) * ldh]; };
    {
        constexpr int kPer = (kWin * kWin + 1023) / 1024;
        double tmp[kPer];
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int idx = tid + q * 1024;
            const int i = idx % W, j = idx / W;
            tmp[q] = idx < W * W ? ca.H[(a.s + i) + (int64_t)(a.s + j) * ca.n] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int idx = tid + q * 1024;
            if (idx < W * W) {
                const int i = idx % W, j = idx / W;
                h[i + j * ldh] = tmp[q];
                u[i + j * ldu] = (i == j) ? 1.0 : 0.0;
            }
        }
    }
    __syncthreads();
    const int l = ca.l, ihi = ca.ihi;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), ln = tid & 63;
    const int rlo = max(l, a.s);
    const int i0 = ln, i1 = ln + 64;            // U rows of this lane
    const bool d0 = i0 < W, d1 = i1 < W;
    auto live = [&](int t) { const int k = l + t - 3 * wv; return wv < a.nb && k >= l && k <= ihi - 1 && t < a.t1; };
    // U columns k, k+1, k+2 (window-relative), rows i0 and i1
    double uc0[2] = {0, 0}, uc1[2] = {0, 0}, uc2[2] = {0, 0};
    // U rows past W: clamped loads, stores into `trash`
    const int i0c = min(i0, W - 1), i1c = min(i1, W - 1);
    auto uload = [&](double* c, int col) {
        c[0] = u[i0c + col * ldu];
        c[1] = u[i1c + col * ldu];
    };
    auto ustore = [&](const double* c, int col) {
        *(d0 ? &u[i0 + col * ldu] : &trash[0]) = c[0];
        *(d1 ? &u[i1 + col * ldu] : &trash[1]) = c[1];
    };
    double ax = 0.0, ay = 0.0, az = 0.0, bq = 0.0, br = 0.0;
    // phase A of bulge wv at row k (reflector, left update, U columns); `three` compile-time
    auto phase_a = [&](const int t, const int k, auto three_c) -> bool {
        constexpr bool three = decltype(three_c)::value;
        const int kk = k - a.s;
        if (t == a.t0 || !live(t - 1)) {
            uload(uc0, kk);
            uload(uc1, kk + 1);
            if (three) uload(uc2, kk + 2);
        } else {
            uc0[0] = uc1[0]; uc0[1] = uc1[1];
            uc1[0] = uc2[0]; uc1[1] = uc2[1];
            if (three) uload(uc2, kk + 2);
        }
        // the left update's rows k..k+2 (columns >= k: no other bulge writes them in this phase, and
        // this step's own stores go to column k-1) are loaded first, so their LDS latency overlaps
        // the reflector's chain
        double l0[2], l1[2], l2[2];
#pragma unroll
        for (int x = 0; x < 2; ++x) {
            const int j = k + ln + 64 * x;
            const int jc = min(j, a.e - 1);    // clamped: lanes past the window read a valid word
            l0[x] = Hw(k, jc);
            l1[x] = Hw(k + 1, jc);
            l2[x] = three ? Hw(k + 2, jc) : 0.0;
        }
        double p, q, r;
        int ex = 0;
        if (k == l) {
            const double sx = a.shifts[2 * wv], sw = a.shifts[2 * wv + 1];
            const double z = Hw(l, l);
            const double rr = sx - z;
            p = (rr * rr - sw) / Hw(l + 1, l) + Hw(l, l + 1);
            q = Hw(l + 1, l + 1) - z - rr - rr;
            r = (three && l + 2 <= ihi) ? Hw(l + 2, l + 1) : 0.0;
            const double sc = fabs(p) + fabs(q) + fabs(r);
            if (sc != 0.0) { const double is = rcp_nr(sc); p *= is; q *= is; r *= is; }
        } else {
            // scaled by a power of two (exact) into [1/2, 1): the norm's square root needs no range
            // reduction
            p = Hw(k, k - 1);
            q = Hw(k + 1, k - 1);
            r = three ? Hw(k + 2, k - 1) : 0.0;
            ex = __builtin_amdgcn_frexp_exp(fmax(fmax(fabs(p), fabs(q)), fabs(r)));
            p = __builtin_amdgcn_ldexp(p, -ex);
            q = __builtin_amdgcn_ldexp(q, -ex);
            r = __builtin_amdgcn_ldexp(r, -ex);
        }
        const double nrm2 = __builtin_fma(p, p, __builtin_fma(q, q, r * r));
        const bool act = nrm2 != 0.0;
        if (act) {
            const double sg = (p >= 0 ? 1.0 : -1.0) * sqrt_nr(nrm2);
            EIGSOL_LDS_ORDER();
            if (k != l && ln == 0) {
                Hw(k, k - 1) = -__builtin_amdgcn_ldexp(sg, ex);
                Hw(k + 1, k - 1) = 0.0;
                if (three) Hw(k + 2, k - 1) = 0.0;
            }
            p += sg;
            const double isg = rcp_nr(sg), ip = rcp_nr(p);
            ax = p * isg; ay = q * isg; az = r * isg; bq = q * ip; br = r * ip;
            // left update, columns k + ln and k + ln + 64 of rows k..k+2
#pragma unroll
            for (int x = 0; x < 2; ++x) {
                const int j = k + ln + 64 * x;
                const bool ok = j < a.e;
                double pp = __builtin_fma(bq, l1[x], l0[x]);
                if (three) {
                    pp = __builtin_fma(br, l2[x], pp);
                    *(ok ? &Hw(k + 2, j) : &trash[2]) = __builtin_fma(-pp, az, l2[x]);
                }
                *(ok ? &Hw(k + 1, j) : &trash[1]) = __builtin_fma(-pp, ay, l1[x]);
                *(ok ? &Hw(k, j) : &trash[0]) = __builtin_fma(-pp, ax, l0[x]);
            }
#pragma unroll
            for (int x = 0; x < 2; ++x) {   // U columns k..k+2 in registers
                double pu = __builtin_fma(ay, uc1[x], ax * uc0[x]);
                if (three) pu = __builtin_fma(az, uc2[x], pu);
                uc0[x] -= pu;
                uc1[x] = __builtin_fma(-pu, bq, uc1[x]);
                if (three) uc2[x] = __builtin_fma(-pu, br, uc2[x]);
            }
        }
        // drop column k (bulge b+1 loads it next step); at the bulge's last step here, all three
        ustore(uc0, kk);
        if (!live(t + 1)) {
            ustore(uc1, kk + 1);
            if (three) ustore(uc2, kk + 2);
        }
        return act;
    };
    // phase B: right update, rows rlo + ln and rlo + ln + 64 of columns k..k+2
    auto phase_b = [&](const int k, auto three_c) {
        constexpr bool three = decltype(three_c)::value;
        const int ilast = min(k + 3, ihi);
#pragma unroll
        for (int x = 0; x < 2; ++x) {
            const int i = rlo + ln + 64 * x;
            const bool ok = i <= ilast;
            const int ic = min(i, ilast);
            const double h0 = Hw(ic, k), h1 = Hw(ic, k + 1);
            double pp = __builtin_fma(ay, h1, ax * h0);
            double h2 = 0.0;
            if (three) { h2 = Hw(ic, k + 2); pp = __builtin_fma(az, h2, pp); }
            *(ok ? &Hw(i, k) : &trash[0]) = h0 - pp;
            *(ok ? &Hw(i, k + 1) : &trash[1]) = __builtin_fma(-pp, bq, h1);
            if (three) *(ok ? &Hw(i, k + 2) : &trash[2]) = __builtin_fma(-pp, br, h2);
        }
    };
    for (int t = a.t0; t < a.t1; ++t) {
        const int k = __builtin_amdgcn_readfirstlane(l + t - 3 * wv);
        const bool lv = live(t);                           // wave-uniform
        const bool three = k != ihi - 1;
        bool act = false;
        if (lv) act = three ? phase_a(t, k, std::true_type{}) : phase_a(t, k, std::false_type{});
        __syncthreads();
        if (act) {
            if (three) phase_b(k, std::true_type{});
            else phase_b(k, std::false_type{});
        }
        __syncthreads();
    }
    for (int idx = tid; idx < W * W; idx += 1024) {
        const int i = idx % W, j = idx / W;
        ca.H[(a.s + i) + (int64_t)(a.s + j) * ca.n] = h[i + j * ldh];
        a.U[idx] = u[i + j * ldu];
    }
}

// The delayed updates of up to kMaxGroups windows on the fp64 matrix cores
// (v_mfma_f64_16x16x4_f64).  One launch applies one side for every window:
//   left : H(s:s+W, lo:hi) <- U^T H(s:s+W, lo:hi)      64 columns per workgroup
//   right: H(lo:hi, s:s+W) <- H(lo:hi, s:s+W) U        64 rows per workgroup
// Left regions of different windows own disjoint rows and right regions disjoint columns, so a
// launch is race-free; a left region of a window meets the right region of a window further down
// the chain, hence lefts and rights are two launches (U_g^T X U_h = (U_g^T X) U_h).
// U is staged in LDS (odd pitch, zero-padded to kWin), the left panel too; each wave computes a
// kWin x 16 strip as six 16 x 16 tiles.  D layout of the f64 MFMA: lane L, register r holds
// D[(L >> 4) + 4 r][L & 15] (cdna_hip_programming.md); D's column index is put on the output's
// row, so 16 lanes store 128 contiguous bytes of one column.
struct WinGemm {
    int s, W;          // window rows/columns [s, s + W)
    int64_t lo, hi;    // left: columns [lo, hi); right: rows [lo, hi)
    int blk0;          // first workgroup of this window
    const double* U;   // W x W, column-major
};
struct WinGemmBatch {
    double* H;
    int64_t n;
    int nw;
    WinGemm w[kMaxGroups + 1];
};
constexpr int kUP = kWin + 2;   // LDS pitch of U and of the left panel: (k + 2 i) mod 32 distinct for 32 lanes

// kTile columns (left) / rows (right) of the off-window region per workgroup.  64: each wave owns
// 16 of them and all six 16-row tiles of U; 32: waves (w & 1) own 16 of them and (w >> 1) three of
// the six U tiles, so twice as many workgroups share a launch's MFMA work (a launch covers only a
// few thousand columns, fewer workgroups than CUs at 64).  The k order of every output element is
// the same for both tilings (bitwise the same updates).
template <bool kLeft, int kTile = 64>
__global__ __launch_bounds__(256) void win_gemm_mfma(WinGemmBatch b) {
    constexpr int kT = kTile == 64 ? 6 : 3;                // U row tiles per wave
    __shared__ double us[kWin * kUP];                    // us[k + rho * kUP] = U(k, rho)
    __shared__ double xs[kLeft ? kTile * kUP : 1];       // left: xs[k + c * kUP] = H(s + k, c0 + c)
    int g = 0;
#pragma unroll
    for (int q = 1; q < kMaxGroups + 1; ++q)
        if (q < b.nw && (int)blockIdx.x >= b.w[q].blk0) g = q;
    const WinGemm w = b.w[g];
    const int W = w.W;
    const int64_t base = w.lo + (int64_t)((int)blockIdx.x - w.blk0) * kTile;
    const int cnt = (int)min<int64_t>(kTile, w.hi - base);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int ct = kTile == 64 ? wave : (wave & 1);      // this wave's 16 columns / rows of the tile
    const int t0 = kTile == 64 ? 0 : 3 * (wave >> 1);    // ... and its first U row tile
    // right: this lane's X(r_j, k) for k = lk, lk + 4, ... (issued first, consumed last)
    constexpr int kKs = kWin / 4;
    double xv[kLeft ? 1 : kKs];
    const int rj = 16 * ct + li;
    const bool rv = rj < cnt;
    if constexpr (!kLeft) {
        const double* xr = b.H + (base + min(rj, max(cnt - 1, 0))) + (int64_t)w.s * b.n;
#pragma unroll
        for (int q = 0; q < kKs; ++q) {
            const int k = 4 * q + lk;
            xv[q] = xr[(int64_t)min(k, W - 1) * b.n];
        }
    }
    {
        // U (and the left panel) into LDS: every global load of the thread issued before any store
        constexpr int kPU = kWin * kWin / 256;
        double tu[kPU];
#pragma unroll
        for (int q = 0; q < kPU; ++q) {
            const int idx = threadIdx.x + 256 * q;
            const int k = idx % kWin, rho = idx / kWin;
            tu[q] = w.U[min(k, W - 1) + min(rho, W - 1) * W];
        }
        if constexpr (kLeft) {
            constexpr int kPX = kWin * kTile / 256;
            double tx[kPX];
#pragma unroll
            for (int q = 0; q < kPX; ++q) {
                const int idx = threadIdx.x + 256 * q;
                const int k = idx % kWin, c = idx / kWin;
                tx[q] = b.H[(w.s + min(k, W - 1)) + (base + min(c, max(cnt - 1, 0))) * b.n];
            }
#pragma unroll
            for (int q = 0; q < kPX; ++q) {
                const int idx = threadIdx.x + 256 * q;
                const int k = idx % kWin, c = idx / kWin;
                xs[k + c * kUP] = (k < W && c < cnt) ? tx[q] : 0.0;
            }
        }
#pragma unroll
        for (int q = 0; q < kPU; ++q) {
            const int idx = threadIdx.x + 256 * q;
            const int k = idx % kWin, rho = idx / kWin;
            us[k + rho * kUP] = (k < W && rho < W) ? tu[q] : 0.0;
        }
    }
    __syncthreads();
    dbl4 acc[kT];
#pragma unroll
    for (int t = 0; t < kT; ++t) acc[t] = dbl4{0.0, 0.0, 0.0, 0.0};
    if constexpr (kLeft) {
        // D[i][j] = sum_k X(k, c_i) U(k, rho_j): i = column 16 ct + i, j = row 16 (t0 + t) + j
        const double* xc = xs + (16 * ct + li) * kUP;
#pragma unroll
        for (int q = 0; q < kKs; ++q) {     // rows k >= W of both LDS images are zero
            const int k = 4 * q + lk;
            const double av = xc[k];
            double bv[kT];
#pragma unroll
            for (int t = 0; t < kT; ++t) bv[t] = us[k + (16 * (t0 + t) + li) * kUP];
#pragma unroll
            for (int t = 0; t < kT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv[t], acc[t], 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < kT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int c = 16 * ct + lk + 4 * r, rho = 16 * (t0 + t) + li;
                if (c < cnt && rho < W) b.H[(w.s + rho) + (base + c) * b.n] = acc[t][r];
            }
    } else {
        // D[i][j] = sum_k U(k, rho_i) X(r_j, k): i = output column rho, j = row 16 ct + j
#pragma unroll
        for (int q = 0; q < kKs; ++q) {
            const int k = 4 * q + lk;
            const double bv = (rv && k < W) ? xv[q] : 0.0;
            double av[kT];
#pragma unroll
            for (int t = 0; t < kT; ++t) av[t] = us[k + (16 * (t0 + t) + li) * kUP];
#pragma unroll
            for (int t = 0; t < kT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[t], bv, acc[t], 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < kT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int rho = 16 * (t0 + t) + lk + 4 * r;
                if (rv && rho < W) b.H[(base + rj) + (int64_t)(w.s + rho) * b.n] = acc[t][r];
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

// AED early stop (kSchur, spk >= 0 = |spike|): a block deflating at the bottom has final Schur
// vector columns (later sweeps touch only the columns of the rows above), so the AED spike test is
// taken when it deflates; the first block that fails it ends the factorisation (*stop = its last
// row; the rows above stay unreduced).  *stop = -1: ran to completion.
template <bool kSchur, int NX>
__device__ void wave_hqr(double* t, double* v, int n, int LD, int maxits, double* wr, double* wi, int* bs,
                         int& fail, int& total, int& maxsw, int* steps_out = nullptr, double spk = -1.0,
                         int* stop = nullptr, double dtol = 2.220446049250313e-16) {
    const int lane = threadIdx.x & 63;
    auto T = [&](int i, int j) -> double& { return t[i + j * LD]; };
    auto V = [&](int i, int j) -> double& { return v[i + j * LD]; };
    const double eps = 2.220446049250313e-16;
    const double aed_sml = 2.2250738585072014e-308 * (n / eps);
    if (stop) *stop = -1;
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
            if (h == 0.0 || fabs(h) <= dtol * s0) lm = l;   // ascending per lane: the last is the max
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
            if (kSchur && spk >= 0.0) {
                const double foo = x == 0.0 ? spk : fabs(x);
                if (fabs(spk * V(0, nn)) > fmax(aed_sml, eps * foo)) {
                    *stop = nn;
                    return;
                }
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
            if (kSchur && spk >= 0.0) {
                double foo = fabs(x) + sqrt(fabs(T(nn, nn - 1))) * sqrt(fabs(T(nn - 1, nn)));
                if (foo == 0.0) foo = spk;
                if (fmax(fabs(spk * V(0, nn)), fabs(spk * V(0, nn - 1))) > fmax(aed_sml, eps * foo)) {
                    *stop = nn;
                    return;
                }
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
        if (steps_out) *steps_out += nn - m;
        // one reflector step; `three` is a compile-time constant (only the sweep's last step is a
        // 2-row reflector), k is wave-uniform, and the updates are explicit FMAs, so the step is
        // straight-line code on a single wave (its cost is instruction issue)
        auto step = [&](const int k, auto three_c) {
            constexpr bool three = decltype(three_c)::value;
            // every load that does not depend on this step's reflector is issued first, so its LDS
            // latency overlaps the reflector's sqrt / reciprocal chain: the left update's rows
            // k..k+2 and (Schur) V's columns k..k+2 (neither is written before they are used)
            double l0[NX], l1[NX], l2[NX], w0[NX], w1[NX], w2[NX];
#pragma unroll
            for (int x = 0; x < NX; ++x) {
                const int j = k + lane + 64 * x, i = lane + 64 * x;
                l0[x] = l1[x] = l2[x] = w0[x] = w1[x] = w2[x] = 0.0;
                if (j < jend) {
                    l0[x] = T(k, j);
                    l1[x] = T(k + 1, j);
                    if (three) l2[x] = T(k + 2, j);
                }
                if (kSchur && i < n) {
                    w0[x] = V(i, k);
                    w1[x] = V(i, k + 1);
                    if (three) w2[x] = V(i, k + 2);
                }
            }
            // the bulge column is scaled by a power of two (exact, two instructions instead of a
            // reciprocal) into [1/2, 1), so the norm's square root needs no range reduction: the
            // step's serial chain is its latency
            double p = p0, q = q0, r = three ? r0 : 0.0;
            int ex = 0;
            if (k != m) {
                p = T(k, k - 1);
                q = T(k + 1, k - 1);
                r = three ? T(k + 2, k - 1) : 0.0;
                ex = __builtin_amdgcn_frexp_exp(fmax(fmax(fabs(p), fabs(q)), fabs(r)));
                p = __builtin_amdgcn_ldexp(p, -ex);
                q = __builtin_amdgcn_ldexp(q, -ex);
                r = __builtin_amdgcn_ldexp(r, -ex);
            }
            const double nrm2 = __builtin_fma(p, p, __builtin_fma(q, q, r * r));
            if (nrm2 == 0.0) return;
            const double sg = (p >= 0 ? 1.0 : -1.0) * sqrt_nr(nrm2);
            if (sg == 0.0) return;
            EIGSOL_LDS_ORDER();
            if (lane == 0 && k != m) {
                T(k, k - 1) = -__builtin_amdgcn_ldexp(sg, ex);
                T(k + 1, k - 1) = 0.0;
                if (three) T(k + 2, k - 1) = 0.0;
            }
            p += sg;
            const double isg = rcp_nr(sg), ip = rcp_nr(p);
            const double ax = p * isg, ay = q * isg, az = r * isg, bq = q * ip, br = r * ip;
#pragma unroll
            for (int x = 0; x < NX; ++x) {        // NX = ceil(n / 64): no loop control on the step's path
                const int j = k + lane + 64 * x;
                if (j < jend) {
                    double pp = __builtin_fma(bq, l1[x], l0[x]);
                    if (three) {
                        pp = __builtin_fma(br, l2[x], pp);
                        T(k + 2, j) = __builtin_fma(-pp, az, l2[x]);
                    }
                    T(k + 1, j) = __builtin_fma(-pp, ay, l1[x]);
                    T(k, j) = __builtin_fma(-pp, ax, l0[x]);
                }
            }
            EIGSOL_LDS_ORDER();
            const int imax = nn < k + 3 ? nn : k + 3;
            // right update of T (rows through k+3 read after the left update's stores) and of V
#pragma unroll
            for (int x = 0; x < NX; ++x) {
                const int i = lane + 64 * x;
                const int it = ibeg + i;
                const bool ct = it <= imax, cv = kSchur && i < n;
                double t0 = 0, t1 = 0, t2 = 0;
                if (ct) { t0 = T(it, k); t1 = T(it, k + 1); if (three) t2 = T(it, k + 2); }
                const double pt = three ? __builtin_fma(az, t2, __builtin_fma(ay, t1, ax * t0)) : __builtin_fma(ay, t1, ax * t0);
                const double pv = three ? __builtin_fma(az, w2[x], __builtin_fma(ay, w1[x], ax * w0[x])) : __builtin_fma(ay, w1[x], ax * w0[x]);
                if (ct) {
                    T(it, k) = t0 - pt;
                    T(it, k + 1) = __builtin_fma(-pt, bq, t1);
                    if (three) T(it, k + 2) = __builtin_fma(-pt, br, t2);
                }
                if (cv) {
                    V(i, k) = w0[x] - pv;
                    V(i, k + 1) = __builtin_fma(-pv, bq, w1[x]);
                    if (three) V(i, k + 2) = __builtin_fma(-pv, br, w2[x]);
                }
            }
            EIGSOL_LDS_ORDER();
        };
        for (int k = m; k <= nn - 2; ++k) step(__builtin_amdgcn_readfirstlane(k), std::true_type{});
        step(nn - 1, std::false_type{});
    }
    maxsw = max(maxsw, its);
}

constexpr int kHqrWaveMax = 128;

// eigenvalues of an n x n (n <= 128) Hessenberg block: info = {fail, most sweeps per deflation, total}
// dtol: relative subdiagonal below which the block splits (eps: LAPACK's test; the sweeps' shifts
// are computed with a looser one, EIGSOL_QR_SHIFT_TOL)
__global__ __launch_bounds__(64) void hqr_wave_kernel(const double* Hin, int64_t ld, int n, double* wr, double* wi,
                                                      int maxits, int* info, double dtol) {
    constexpr int LD = kHqrWaveMax + 1;
    __shared__ double t[kHqrWaveMax * LD];
    for (int e = threadIdx.x; e < n * n; e += 64) {
        const int i = e % n, j = e / n;
        t[i + j * LD] = Hin[i + (int64_t)j * ld];
    }
    __syncthreads();
    int fail, total, maxsw;
    if (n <= 64) wave_hqr<false, 1>(t, nullptr, n, LD, maxits, wr, wi, nullptr, fail, total, maxsw, nullptr, -1.0, nullptr, dtol);
    else wave_hqr<false, 2>(t, nullptr, n, LD, maxits, wr, wi, nullptr, fail, total, maxsw, nullptr, -1.0, nullptr, dtol);
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
    double beta, tau, hbeta;
};

// 256 threads: wave 0 runs the one-wave Schur factorisation (phase A) and the Householder vectors;
// the reflector applications of phase C take four lanes per row / column, each one of the
// original four FMA chains of the dot products, combined in the same order (round 4: bitwise the
// one-wave kernel's results, phase C ~3x shorter)
constexpr int kAedThreads = 256;
// Concurrent shifts (ShiftJob, round 5): a second workgroup of the same launch computes the
// eigenvalues of the trailing ns x ns block of the active block as it stands BEFORE the AED -- the
// block the next sweep's shift QR would read when the AED deflates nothing -- on its own wave while
// workgroup 0 runs the AED.  It copies the block into its LDS first and raises flag = epoch;
// workgroup 0 writes the window back only after seeing the flag, so the copy is the pre-AED state.
struct ShiftJob {
    int kb, ns;                // block [kb, kb + ns) of H
    double dtol;               // split tolerance of the shifts' QR (EIGSOL_QR_SHIFT_TOL)
    double *wr, *wi;           // ns eigenvalues
    int* info;                 // {fail, most sweeps per deflation, total, wait timed out}
    unsigned* flag;
    unsigned epoch;
};

__device__ __forceinline__ unsigned ld_flag(const unsigned* p) {
    return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kAedThreads) void aed_kernel(double* H, int64_t n, int kw, int nw, int spike_valid, int maxits,
                                                 int early, double* wr, double* wi, double* Vout, int* info,
                                                 ShiftJob sj) {
    constexpr int LD = kAedMax + 1;
    __shared__ double t[kAedMax * LD];
    __shared__ double v[kAedMax * LD];
    __shared__ double hv[kAedMax];        // Householder vector
    __shared__ double sp[kAedMax];
    __shared__ int bs[kAedMax];           // Schur block size ending at each row (1 or 2)
    __shared__ AedCtl c;
    const int tid = threadIdx.x, nt = kAedThreads;
    if (blockIdx.x == 1) {   // the concurrent shifts (ShiftJob)
        const int ns = sj.ns;
        for (int e = tid; e < ns * ns; e += nt) {
            const int i = e % ns, j = e / ns;
            t[i + j * LD] = H[(sj.kb + i) + (int64_t)(sj.kb + j) * n];
        }
        __syncthreads();
        if (tid == 0) __hip_atomic_store(sj.flag, sj.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        if (tid < 64) {
            int fail = 0, total = 0, maxsw = 0;
            if (ns <= 64) wave_hqr<false, 1>(t, nullptr, ns, LD, maxits, sj.wr, sj.wi, nullptr, fail, total, maxsw, nullptr, -1.0, nullptr, sj.dtol);
            else wave_hqr<false, 2>(t, nullptr, ns, LD, maxits, sj.wr, sj.wi, nullptr, fail, total, maxsw, nullptr, -1.0, nullptr, sj.dtol);
            if (tid == 0) {
                sj.info[0] = fail;
                sj.info[1] = maxsw;
                sj.info[2] = total;
            }
        }
        return;
    }
    const int grp = tid >> 2, q = tid & 3;   // phase C: 64 groups of four lanes (one wave holds 16 groups)
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
    int fail = 0, total = 0, maxsw = 0;
    const long long tA = wall_clock64();
    // ---------------- phase A: real Schur form with V
    int steps = 0, stop = -1;
    const double spk = early ? fabs(spike) : -1.0;
    if (tid < 64) {
        if (nw <= 64) wave_hqr<true, 1>(t, v, nw, LD, maxits, wr + kw, wi + kw, bs, fail, total, maxsw, &steps, spk, &stop);
        else wave_hqr<true, 2>(t, v, nw, LD, maxits, wr + kw, wi + kw, bs, fail, total, maxsw, &steps, spk, &stop);
    }
    __syncthreads();
    const long long tB = wall_clock64();
    // ---------------- phase B: spike test from the bottom
    if (tid == 0 && early) {
        c.nd = fail ? 0 : nw - 1 - stop;   // the spike test ran inside the factorisation
        c.beta = 0.0;
    } else if (tid == 0) {
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
    const long long tC = wall_clock64();
    // ---------------- phase C: undeflated part + spike back to Hessenberg form
    // apply P = I - tau hv hv^T (hv[0..len), hv[0] = 1) to rows/columns [o, o + len); the dot
    // products run four independent FMA chains so that their LDS reads overlap (one wave: the
    // step's cost is latency)
    auto dot4 = [&](auto elem, int len) -> double {
        double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
        int i = 0;
        for (; i + 4 <= len; i += 4) {
            s0 = __builtin_fma(hv[i], elem(i), s0);
            s1 = __builtin_fma(hv[i + 1], elem(i + 1), s1);
            s2 = __builtin_fma(hv[i + 2], elem(i + 2), s2);
            s3 = __builtin_fma(hv[i + 3], elem(i + 3), s3);
        }
        for (; i < len; ++i) s0 = __builtin_fma(hv[i], elem(i), s0);
        return (s0 + s1) + (s2 + s3);
    };
    (void)dot4;
    // lane q of a group runs chain q of dot4 (chain 0 also takes the tail), the four chains meet
    // as (s0 + s1) + (s2 + s3): dot4's value, bit for bit
    auto dotq = [&](auto elem, int len) -> double {
        const int full = len & ~3;
        double sq = 0.0;
        for (int i = q; i < full; i += 4) sq = __builtin_fma(hv[i], elem(i), sq);
        if (q == 0)
            for (int i = full; i < len; ++i) sq = __builtin_fma(hv[i], elem(i), sq);
        const double o1 = __shfl_xor(sq, 1, 64);
        const double pr = (q & 1) ? o1 + sq : sq + o1;
        const double o2 = __shfl_xor(pr, 2, 64);
        return (q & 2) ? o2 + pr : pr + o2;
    };
    auto reflect = [&](int o, int len, int jlo) {
        const double tau = c.tau;
        for (int j = jlo + grp; j < nw; j += nt / 4) {                   // left: T[o:o+len, jlo:nw]
            const double w = tau * dotq([&](int i) { return T(o + i, j); }, len);
            for (int i = q; i < len; i += 4) T(o + i, j) = __builtin_fma(-w, hv[i], T(o + i, j));
        }
        __syncthreads();
        for (int i = grp; i < nw; i += nt / 4) {                         // right: T[0:m, o:o+len], V[:, o:o+len]
            const double wv = tau * dotq([&](int jj) { return V(i, o + jj); }, len);
            if (i < m) {
                const double w = tau * dotq([&](int jj) { return T(i, o + jj); }, len);
                for (int jj = q; jj < len; jj += 4) T(i, o + jj) = __builtin_fma(-w, hv[jj], T(i, o + jj));
            }
            for (int jj = q; jj < len; jj += 4) V(i, o + jj) = __builtin_fma(-wv, hv[jj], V(i, o + jj));
        }
        __syncthreads();
    };
    // Householder vector of x[0..len) by the whole wave: hv[0] = 1, c.tau; returns beta (every lane)
    auto house = [&](const double* x, int len) -> double {
        if (tid < 64) {
            const double alpha = x[0];
            double part = 0.0;
            for (int i = 1 + tid; i < len; i += 64) part = __builtin_fma(x[i], x[i], part);
            const double xn = sqrt(wave_sum(part));
            double beta = alpha, sc = 0.0, tau = 0.0;
            if (xn != 0.0) {
                beta = -(alpha >= 0 ? 1.0 : -1.0) * sqrt(alpha * alpha + xn * xn);
                tau = (beta - alpha) / beta;
                sc = 1.0 / (alpha - beta);
            }
            EIGSOL_LDS_ORDER();
            for (int i = 1 + tid; i < len; i += 64) hv[i] = x[i] * sc;
            if (tid == 0) {
                hv[0] = 1.0;
                c.tau = tau;
                c.hbeta = beta;
            }
        }
        __syncthreads();
        return c.hbeta;
    };
    if (nd > 0 && m > 0) {
        for (int i = tid; i < m; i += nt) sp[i] = spike * V(0, i);
        if (tid == 0) c.tau = 0.0;
        __syncthreads();
        const double b0 = m > 1 ? house(sp, m) : sp[0];
        if (tid == 0) c.beta = b0;
        __syncthreads();
        if (m > 1 && c.tau != 0.0) reflect(0, m, 0);
        for (int col = 0; col + 2 < m; ++col) {
            const double b = house(&T(col + 1, col), m - col - 1);
            __syncthreads();   // every wave has read beta before the next house overwrites it
            if (tid == 0) T(col + 1, col) = b;
            for (int i = col + 2 + tid; i < m; i += nt) T(i, col) = 0.0;
            __syncthreads();
            if (c.tau != 0.0) reflect(col + 1, m - col - 1, col + 1);
        }
    }
    const long long tD = wall_clock64();
    // ---------------- phase D: write back (only when something deflated), after the concurrent
    // shifts' workgroup has copied its pre-AED block (a bounded wait: ~1 s of the constant clock)
    if (gridDim.x > 1) {
        if (tid == 0) {
            int timed_out = 0;
            if (nd > 0) {
                const long long t0 = wall_clock64();
                while (ld_flag(sj.flag) != sj.epoch) {
                    if (wall_clock64() - t0 > 100000000ll) { timed_out = 1; break; }
                    __builtin_amdgcn_s_sleep(2);
                }
            }
            sj.info[3] = timed_out;
        }
        __syncthreads();
    }
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
        info[4] = steps;
        info[5] = (int)(tB - tA);   // wall-clock ticks (100 MHz) of phases A, B, C
        info[6] = (int)(tC - tB);
        info[7] = (int)(tD - tC);
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
                     int* info, double dtol = 2.220446049250313e-16) {
    static const bool wave = [] {
        const char* e = std::getenv("EIGSOL_HQR_WAVE");
        return !e || std::atoi(e) != 0;
    }();
    if (!wave) return hqr_lds(st, H, ld, n, maxits, wr, wi, info);
    hipLaunchKernelGGL(dev::hqr_wave_kernel, dim3(1), dim3(64), 0, st, H, ld, n, wr, wi, maxits, info, dtol);
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

static constexpr int kSmallDefault = 128;
// AED window at 4096 with 4-bulge groups (up to 24 bulges per sweep): 40 -> 1.90 s, 48 -> 1.82 s, 56 -> 1.87 s
// (one chain of 16 bulges: 40 was best); the window's one-wave Schur factorisation costs O(nw^3) latency-bound steps
static constexpr int kAedDefault = 64;   // EIGSOL_QR_AED overrides (0: off)

int francis_large_f64(eigsol_ctx* ctx, double* H, int64_t n, int maxits, double* wr, double* wi,
                      int32_t* sweeps_out, int32_t* fail_out) {
    hipStream_t st = ctx->stream;
    const double eps = 2.220446049250313e-16;
    double *dwr = nullptr, *dwi = nullptr, *dds = nullptr, *dU = nullptr, *dsh = nullptr;
    int* dinfo = nullptr;
    double* dsw = nullptr;      // concurrent shifts (ShiftJob): re, im
    int* dsinfo = nullptr;
    unsigned* dflag = nullptr;
    unsigned flag_epoch = 0;
    int rc = EIGSOL_OK;
    if (hipMalloc(&dsw, 2 * dev::kAedMax * sizeof(double)) != hipSuccess || hipMalloc(&dsinfo, 64) != hipSuccess ||
        hipMalloc(&dflag, 64) != hipSuccess || hipMemsetAsync(dflag, 0, 64, st) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "francis: device workspace");
    if (rc == EIGSOL_OK && (hipMalloc(&dwr, n * sizeof(double)) != hipSuccess || hipMalloc(&dwi, n * sizeof(double)) != hipSuccess ||
        hipMalloc(&dds, 2 * n * sizeof(double)) != hipSuccess ||
        hipMalloc(&dU, dev::kMaxGroups * dev::kWin * dev::kWin * sizeof(double)) != hipSuccess ||
        hipMalloc(&dsh, 4 * dev::kMaxBulges * sizeof(double)) != hipSuccess || hipMalloc(&dinfo, 64) != hipSuccess))
        rc = fail(EIGSOL_E_HIP, "francis: device workspace");
    // every per-sweep transfer goes through pinned host memory: a pageable hipMemcpyAsync is staged
    // by the runtime and waited for with a sleeping wait, ~1 ms per copy (round-4 kernel trace,
    // tools/gap_analysis.py), more than a sweep's kernels at the end of the iteration
    struct Staging {
        int info[8];
        int cinfo[4];
        double awr[dev::kAedMax], awi[dev::kAedMax];
        double cwr[2 * dev::kAedMax];   // concurrent shifts: re [0, kAedMax), im [kAedMax, 2 kAedMax)
        double swr[2 * dev::kMaxBulges], swi[2 * dev::kMaxBulges], sh[2 * dev::kMaxBulges];
    };
    Staging* hp = nullptr;
    double* ds = nullptr;   // deflation scans: diagonal [0, n), subdiagonal [n, 2n)
    // on any allocation failure rc is set, the loop below never runs and the common cleanup at the
    // end frees whatever was allocated
    if (rc == EIGSOL_OK && (hipHostMalloc(&hp, sizeof(Staging), hipHostMallocDefault) != hipSuccess ||
                            hipHostMalloc(&ds, 2 * n * sizeof(double), hipHostMallocDefault) != hipSuccess))
        rc = fail(EIGSOL_E_HIP, "francis: pinned staging");
    double* const swr = hp ? hp->swr : nullptr;
    double* const swi = hp ? hp->swi : nullptr;
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
    static const int max_groups = [] {                 // bulge groups chased concurrently (EIGSOL_QR_GROUPS)
        const char* e = std::getenv("EIGSOL_QR_GROUPS");
        return e ? std::max(1, std::min(dev::kMaxGroups, std::atoi(e))) : dev::kMaxGroups;
    }();
    static const int max_bulges = [] {                 // experiments: cap the bulges per chain
        const char* e = std::getenv("EIGSOL_QR_NB");
        return e ? std::max(1, std::min(dev::kMaxBulges, std::atoi(e))) : 32;
    }();
    long long st_steps = 0, st_aed_steps = 0, st_aed_ph[3] = {0, 0, 0};
    static const int aed_win = [] {
        const char* e = std::getenv("EIGSOL_QR_AED");   // AED window (0: off)
        return e ? std::max(0, std::min(dev::kAedMax, std::atoi(e))) : kAedDefault;
    }();
    // AED early stop (default; EIGSOL_QR_AED_EARLY=0: the whole window Schur form, whose undeflated
    // eigenvalues are the shifts).  4096^2: 1.33 -> 1.23 s (the window's factorisation stops at the
    // first undeflatable block: 378 -> 192 ms of one-wave steps; the shifts then come from the
    // trailing block, and the sweeps drop from 146 to 128); grid over window 48/56/64, nibble 30/50,
    // bulges 28/36: window 64, nibble 30, 28 bulges is the optimum (tools/qr_ab_round3.sh)
    static const bool aed_early = [] {
        const char* e = std::getenv("EIGSOL_QR_AED_EARLY");
        return !e || std::atoi(e) != 0;
    }();
    // the shifts' QR splits at a looser relative subdiagonal than the eigenvalues' (shifts need no
    // full accuracy; EIGSOL_QR_SHIFT_TOL).  Round 4 (tools/shift_tol_ab.sh, 4096^2, three seeds):
    // eps / 1e-6 / 1e-5 / 1e-4 / 1e-3 -> 1.181-1.192 / 1.147-1.158 / 1.143-1.161 / 1.109-1.130 /
    // 1.109-1.126 s, the eigenvalues one-to-one with LAPACK's at every setting (2.9e-12 at 1e-4)
    static const double shift_tol = [] {
        const char* e = std::getenv("EIGSOL_QR_SHIFT_TOL");
        return e ? std::max(2.220446049250313e-16, std::atof(e)) : 1e-4;
    }();
    // window-GEMM tile (EIGSOL_QR_GEMM_TILE = 32 | 64; default: 32 when a launch's 64-wide tiles
    // would not cover the CUs)
    static const int gemm_tile = [] {
        const char* e = std::getenv("EIGSOL_QR_GEMM_TILE");
        const int v = e ? std::atoi(e) : 0;
        return (v == 32 || v == 64) ? v : 0;
    }();
    // % of the AED window deflated that skips the sweep (LAPACK's NIBBLE).  Round 5, after the
    // concurrent shifts (tools/qr_nibble_r5.sh, 4096^2, seeds 42 / 7 / 20251226): 30 / 25 / 20 / 15 / 10
    // -> 0.941 / 0.920 / 0.904 / 0.889 / 0.911 s (seed 42), 0.931 / 0.895 / 0.909 / 0.889 / 0.900,
    // 0.927 / 0.913 / 0.904 / 0.884 / 0.919: 15
    static const int kNibble = [] {
        const char* e = std::getenv("EIGSOL_QR_NIBBLE");
        return e ? std::max(1, std::atoi(e)) : 15;
    }();
    int st_sweeps = 0, st_windows = 0, st_small = 0, st_small_rows = 0, st_aed = 0, st_aed_defl = 0, st_conc = 0;
    // concurrent shifts (EIGSOL_QR_CONC): 0 off (the shift QR after the AED, one wave), 1 when the AED
    // deflates nothing (bitwise the sequential sweeps), 2 (default) also after a small deflation
    // (LAPACK xLAQR0's undeflated window eigenvalues).  Round 5 (tools/qr_conc_ab.sh, 4096^2, two
    // seeds): only 2 of 115 sweeps follow an AED that deflated nothing, so mode 1 is mode 0 (0.946 /
    // 0.949 s); mode 2 runs 141 sweeps instead of 115 but skips their 0.79 ms shift QRs, whose
    // eigenvalue QR of the window hides under the AED (~1.1 ms): 0.946 -> 0.928 s and 0.948 ->
    // 0.930 s (seed 7), one-to-one with LAPACK (3.3e-12)
    static const int conc_mode = [] {
        const char* e = std::getenv("EIGSOL_QR_CONC");
        return e ? std::atoi(e) : 2;
    }();
    auto finish_small = [&](int l, int hi) -> int {
        const int m = hi - l + 1;
        EIGSOL_TRY(hqr_small(st, H + l + (int64_t)l * n, n, m, std::max(1, maxits), dwr + l, dwi + l, dinfo));
        int* info = hp->info;
        EIGSOL_HIP(hipMemcpyAsync(info, dinfo, 3 * sizeof(int), hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(stream_wait(st));
        if (info[0]) failed = 1;
        sweeps = std::max(sweeps, info[1]);
        return EIGSOL_OK;
    };
    // deflation scan of [0, ihi]: diagonal and subdiagonal into pinned host memory (only the
    // ihi + 1 leading entries of each half travel)
    auto scan = [&]() -> int {
        hipLaunchKernelGGL(dev::diag_sub_kernel, dim3((ihi + 256) / 256), dim3(256), 0, st, H, n, ihi, dds);
        if (hipMemcpyAsync(ds, dds, (ihi + 1) * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(ds + n, dds + n, (ihi + 1) * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
            stream_wait(st) != hipSuccess)
            return fail(EIGSOL_E_HIP, "francis: deflation scan");
        return EIGSOL_OK;
    };
    bool scanned = false;   // the previous sweep's closing scan is still current (nothing ran since)
    while (rc == EIGSOL_OK && ihi >= 0) {
        if (!scanned && (rc = scan()) != EIGSOL_OK) break;
        scanned = false;
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
            // concurrent shifts: the pre-AED trailing ns block's eigenvalues on a second workgroup
            // (ShiftJob); used when the AED deflates nothing (the very block the sequential shift QR
            // would read, so the sweep is bitwise the same) and, LAPACK xLAQR0-style, when it
            // deflated a few and the block is the window itself (the undeflated window eigenvalues)
            const bool conc = conc_mode > 0 && ns <= dev::kAedMax && ns >= 2;
            dev::ShiftJob sj{ihi - ns + 1, ns, shift_tol, dsw, dsw + dev::kAedMax, dsinfo, dflag, ++flag_epoch};
            hipLaunchKernelGGL(dev::aed_kernel, dim3(conc ? 2 : 1), dim3(dev::kAedThreads), 0, st, H, n, kw, nw,
                               kw > l ? 1 : 0, 60, aed_early ? 1 : 0, dwr, dwi, dU, dinfo, sj);
            int* info = hp->info;
            double* const awr = hp->awr;
            double* const awi = hp->awi;
            if (hipMemcpyAsync(info, dinfo, 8 * sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipMemcpyAsync(awr, dwr + kw, nw * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipMemcpyAsync(awi, dwi + kw, nw * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
                (conc && (hipMemcpyAsync(hp->cinfo, dsinfo, 4 * sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
                          hipMemcpyAsync(hp->cwr, dsw, 2 * dev::kAedMax * sizeof(double), hipMemcpyDeviceToHost, st) !=
                              hipSuccess)) ||
                stream_wait(st) != hipSuccess) {
                rc = fail(EIGSOL_E_HIP, "francis: aed");
                break;
            }
            const bool conc_ok = conc && !hp->cinfo[0] && !hp->cinfo[3];
            ++st_aed;
            st_aed_steps += info[4];
            st_aed_ph[0] += info[5]; st_aed_ph[1] += info[6]; st_aed_ph[2] += info[7];
            if (!info[0]) {
                const int nd = info[1], m = info[3];
                if (nd > 0) {
                    st_aed_defl += nd;
                    if (kw > l) {   // rows above the window: H[l, kw) x [kw, kw + nw) V
                        dev::WinGemmBatch gb{H, n, 1, {}};
                        gb.w[0] = dev::WinGemm{kw, nw, (int64_t)l, (int64_t)kw, 0, dU};
                        hipLaunchKernelGGL(dev::win_gemm_mfma<false>, dim3((kw - l + 63) / 64), dim3(256), 0, st, gb);
                    }
                    ihi = kw + m - 1;
                    sweeps = std::max(sweeps, stall);
                    stall = 0;
                    if (100 * nd >= kNibble * nw || m < 4) continue;   // enough deflated: look again first
                }
                if (conc_ok && nd == 0) {   // the block the shift QR below would solve, already solved
                    for (int i = 0; i < ns; ++i) {
                        swr[i] = hp->cwr[i];
                        swi[i] = hp->cwr[dev::kAedMax + i];
                    }
                    have_shifts = true;
                    ++st_conc;
                } else if (conc_ok && conc_mode > 1 && nd > 0 && ns == nw && m >= ns / 2) {
                    // the window's undeflated eigenvalues (LAPACK xLAQR0): the window's spectrum with
                    // each deflated eigenvalue's nearest match removed; the last (ns - nd) rounded to
                    // an even count
                    std::vector<int> used(ns, 0);
                    for (int j = m; j < nw; ++j) {
                        int best = -1;
                        double bd = 0.0;
                        for (int i = 0; i < ns; ++i) {
                            if (used[i]) continue;
                            const double d = std::hypot(hp->cwr[i] - awr[j], hp->cwr[dev::kAedMax + i] - awi[j]);
                            if (best < 0 || d < bd) { best = i; bd = d; }
                        }
                        if (best >= 0) used[best] = 1;
                    }
                    int k = 0;
                    for (int i = 0; i < ns; ++i)
                        if (!used[i]) {
                            swr[k] = hp->cwr[i];
                            swi[k] = hp->cwr[dev::kAedMax + i];
                            ++k;
                        }
                    const int N2 = ihi - l + 1;
                    nb = std::min({max_bulges, std::max(1, N2 / 8), std::max(1, k / 2)});
                    ns = 2 * nb;
                    for (int i = 0; i < ns; ++i) {   // the bottom ns of the undeflated ones
                        swr[i] = swr[k - ns + i];
                        swi[i] = swi[k - ns + i];
                    }
                    have_shifts = true;
                    ++st_conc;
                }
                // shifts: the bottom undeflated eigenvalues of the window (early-stopped windows
                // have none: the trailing block's, below)
                if (!aed_early) {
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
        }
        // every 6th sweep without a deflation uses exceptional shifts (LAPACK xLAQR0's KEXSH, NDFL
        // counted from 1 after a deflation): stall counts those sweeps, 0 right after the AED deflated.
        // Round 3 took stall == 0 as exceptional too, so every sweep after a partial AED deflation ran
        // on ad hoc shifts (and its shift QR went unused); EIGSOL_QR_EXC_LEGACY=1 restores that for A/B
        static const bool exc_legacy = [] {
            const char* e = std::getenv("EIGSOL_QR_EXC_LEGACY");
            return e && std::atoi(e) != 0;
        }();
        const bool exceptional = exc_legacy ? stall % 6 == 0 : (stall > 0 && stall % 6 == 0);
        if (!have_shifts && !exceptional) {
            nb = std::min(max_bulges, std::max(1, (ihi - l + 1) / 8));
            ns = 2 * nb;
            // shifts: eigenvalues of the trailing 2nb x 2nb block
            rc = hqr_small(st, H + (ihi - ns + 1) + (int64_t)(ihi - ns + 1) * n, n, ns, 60, dwr + ihi - ns + 1,
                           dwi + ihi - ns + 1, dinfo, shift_tol);
            if (rc != EIGSOL_OK) break;
            if (hipMemcpyAsync(swr, dwr + ihi - ns + 1, ns * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipMemcpyAsync(swi, dwi + ihi - ns + 1, ns * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
                stream_wait(st) != hipSuccess) {
                rc = fail(EIGSOL_E_HIP, "francis: shifts");
                break;
            }
        }
        // pair the shifts: conjugate pairs stay together, reals are paired in order;
        // every 6th stalled sweep uses exceptional shifts from the bottom subdiagonal
        double* const sh = hp->sh;   // 2 nb values; the chase reads them from dsh
        if (exceptional) {
            nb = std::min(max_bulges, std::max(1, (ihi - l + 1) / 8));
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
        if (hipMemcpyAsync(dsh, sh, 2 * nb * sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess) {
            rc = fail(EIGSOL_E_HIP, "francis: shift upload");
            break;
        }
        ++st_sweeps;
        // chase: C groups of nbg bulges, group g starting G steps after group g-1, each group in its
        // own LDS window; a round advances every group's window by the same number of steps
        // groups of >= 4 bulges; the spacing costs (C - 1) G extra steps, kept below N / 4
        const int Nact = ihi - l + 1;   // after the AED's deflations
        const int C = std::max(1, std::min({max_groups, nb / 4, 1 + Nact / (4 * (dev::kWin + 12))}));
        const int nbg = std::min(nb / C, 16);   // one wave per bulge: at most 16 per window
        const int G = dev::kWin + 3 * nbg;   // group spacing: windows stay disjoint
        const int Tg = (ihi - 1 - l) + 3 * (nbg - 1) + 1;     // steps of one group
        const int T = (C - 1) * G + Tg;
        int t0 = 0;
        while (t0 < T && rc == EIGSOL_OK) {
            dev::ChaseArgs ca{H, n, l, ihi, {}};
            int t1 = T, nwin = 0;
            int g_act[dev::kMaxGroups];
            for (int g = 0; g < C; ++g) {
                const int tl = t0 - g * G;
                if (tl < 0) { t1 = std::min(t1, g * G); break; }    // later groups start at a round boundary
                if (tl >= Tg) continue;                              // group done
                int s;
                if (tl <= 3 * (nbg - 1)) s = std::max(0, l - 1);
                else s = std::max(0, l + tl - 3 * (nbg - 1) - 1);
                const int e = std::min(s + dev::kWin, ihi + 1);
                const int kmax = (e == ihi + 1) ? ihi - 1 : e - 4;
                int tl1 = tl;
                while (tl1 < Tg) {
                    const int blead = std::max(0, (l + tl1 - (ihi - 1) + 2) / 3);   // first bulge not past ihi-1
                    if (blead >= nbg) { tl1 = Tg; break; }
                    if (l + tl1 - 3 * blead > kmax) break;
                    ++tl1;
                }
                t1 = std::min(t1, tl1 + g * G);
                ca.w[nwin] = dev::ChaseWin{s, e, tl, 0, nbg, dsh + 2 * g * nbg, dU + (size_t)nwin * dev::kWin * dev::kWin};
                g_act[nwin++] = g;
            }
            if (nwin == 0 && t1 > t0) { t0 = t1; continue; }   // every started group done, the next not yet due
            if (t1 <= t0 || nwin == 0) { rc = fail(EIGSOL_E_SOLVER, "francis: window did not advance (internal error)"); break; }
            for (int q = 0; q < nwin; ++q) {
                ca.w[q].t1 = t1 - g_act[q] * G;
                if (q > 0 && ca.w[q].e > ca.w[q - 1].s) { rc = fail(EIGSOL_E_SOLVER, "francis: windows overlap (internal error)"); break; }
            }
            if (rc != EIGSOL_OK) break;
            st_windows += nwin;
            st_steps += t1 - t0;
            hipLaunchKernelGGL(dev::chase_wave_kernel, dim3(nwin), dim3(1024), 0, st, ca);
            // delayed updates: every left region, then every right region; tiles of gemm_tile
            // columns / rows per workgroup (32 when 64-wide tiles would leave CUs idle)
            dev::WinGemmBatch lb{H, n, 0, {}}, rb{H, n, 0, {}};
            int nlb = 0, nrb = 0, span = 0;
            for (int q = 0; q < nwin; ++q) {
                const dev::ChaseWin& w = ca.w[q];
                if (w.e <= ihi) span += ihi + 1 - w.e;
                if (w.s > l) span += w.s - l;
            }
            const int tile = gemm_tile > 0 ? gemm_tile : (span / 64 < ctx->num_cus ? 32 : 64);
            for (int q = 0; q < nwin; ++q) {
                const dev::ChaseWin& w = ca.w[q];
                const int W = w.e - w.s;
                if (w.e <= ihi) {
                    lb.w[lb.nw++] = dev::WinGemm{w.s, W, (int64_t)w.e, (int64_t)ihi + 1, nlb, w.U};
                    nlb += (ihi + 1 - w.e + tile - 1) / tile;
                }
                if (w.s > l) {
                    rb.w[rb.nw++] = dev::WinGemm{w.s, W, (int64_t)l, (int64_t)w.s, nrb, w.U};
                    nrb += (w.s - l + tile - 1) / tile;
                }
            }
            if (tile == 32) {
                if (nlb > 0) hipLaunchKernelGGL((dev::win_gemm_mfma<true, 32>), dim3(nlb), dim3(256), 0, st, lb);
                if (nrb > 0) hipLaunchKernelGGL((dev::win_gemm_mfma<false, 32>), dim3(nrb), dim3(256), 0, st, rb);
            } else {
                if (nlb > 0) hipLaunchKernelGGL(dev::win_gemm_mfma<true>, dim3(nlb), dim3(256), 0, st, lb);
                if (nrb > 0) hipLaunchKernelGGL(dev::win_gemm_mfma<false>, dim3(nrb), dim3(256), 0, st, rb);
            }
            t0 = t1;
        }
        if (hipGetLastError() != hipSuccess) { rc = fail(EIGSOL_E_HIP, "francis: launch"); break; }
        // a deflation anywhere below resets the stall counter; the scan also serves the next pass
        if ((rc = scan()) != EIGSOL_OK) break;
        scanned = true;
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
            stream_wait(st) != hipSuccess)
            rc = fail(EIGSOL_E_HIP, "francis: download");
    }
    if (stats)
        std::fprintf(stderr, "francis: n=%lld sweeps=%d windows=%d steps=%lld small_blocks=%d small_rows=%d kSmall=%d "
                     "aed=%d aed_deflated=%d aed_win=%d aed_steps=%lld aed_phase_ms=%.1f/%.1f/%.1f conc_shifts=%d\n",
                     (long long)n, st_sweeps, st_windows, st_steps, st_small, st_small_rows, kSmall, st_aed, st_aed_defl,
                     aed_win, st_aed_steps, st_aed_ph[0] * 1e-5, st_aed_ph[1] * 1e-5, st_aed_ph[2] * 1e-5, st_conc);
    for (void* p : {(void*)dwr, (void*)dwi, (void*)dds, (void*)dU, (void*)dsh, (void*)dinfo, (void*)dsw, (void*)dsinfo,
                    (void*)dflag})
        (void)hipFree(p);
    if (ds) (void)hipHostFree(ds);
    if (hp) (void)hipHostFree(hp);
    // iterations reported: sweeps spent on the slowest deflation (>= 1, the final check), so that
    // iterations <= maxIterations exactly when the iteration converged
    *sweeps_out = std::max(1, sweeps);
    *fail_out = failed;
    return rc;
}

}  // namespace eigsol

// Nested-dissection multifrontal LU of M = A - sigma I on gfx950, for general sparse patterns whose
// LU has real fill (a 2-D or 3-D mesh under any numbering).
//
// Replaces the SparseLU branch of solve_shifted<S> (src/matrix/solve_shifted.hpp:85-117: M = A,
// M(i, i) -= sigma with coeffRef inserting a missing diagonal :96-102, analyzePattern + factorize
// :104-106, solve :112-115).  SparseLU orders columns with COLAMD and factors supernodes on one
// core; here the order is a nested dissection of the pattern of M + M^T and the factorization is
// multifrontal, so that the work is dense blocks on the matrix cores and independent fronts run
// side by side:
//   * ordering (host): recursive bisection of the graph by breadth-first level structures from a
//     pseudo-peripheral vertex; the median level, thinned to the vertices that touch the next
//     level, is the separator; pieces of at most EIGSOL_MF_LEAF (64) vertices are leaves;
//     disconnected pieces are split into components and the small ones packed together.  The
//     tree is numbered in postorder, so every supernode (a leaf or a separator) owns a contiguous
//     range of columns and its descendants come before it;
//   * symbolic (host): struct(s) = the indices past s's columns that s's rows reach in M + M^T or
//     through a child's struct; the front of s is the dense (ns + ms)^2 matrix on the index list
//     [s's columns, struct(s)], column-major, resident in HBM for the factor's lifetime;
//   * numeric (device, by tree height, all fronts of a height in the same launches): M's entries
//     scattered into their fronts once; per height the children's Schur blocks extend-added into
//     their parents (one launch per child rank, so the sum order is fixed); then panels of NB
//     pivots: one workgroup per front factors its panel with partial pivoting restricted to the
//     front's own pivot rows (no delayed pivots; a zero pivot fails the factor), swaps whole rows
//     (LAPACK getrf style) and solves U12 = L11^-1 A12; one batched launch runs every front's
//     trailing update A22 -= L21 U12 on the fp64 matrix cores (rankk_tile, 64 x 64 tiles, all
//     fronts of the height in one grid).  The trailing block left after the last panel is the
//     Schur complement the parent receives;
//   * solve: gather b into the new numbering; forward by height (one workgroup per front: the
//     children's contribution vectors extend-added in a fixed order, the pivot permutation, the
//     unit-lower L11 solve by 64-row blocks - the block's triangle on one wave by lane broadcasts,
//     the rows below as a GEMV by the workgroup - and the front's own contribution L21 y); then
//     backward from the root (x of struct(s) gathered from the ancestors, y - U12 x, the U11
//     solve by blocks from the bottom); scatter back.  Every sum has a fixed order: the solve is
//     deterministic.
// The pivoting is restricted to each front, so the factor is the exact LU of a row-permuted M
// only when no pivot is tiny; gmres.hip therefore treats it like the no-pivot exact LU: the solve
// is checked by its true residual and refined by GMRES cycles on the same factor when it misses.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <numeric>
#include <thread>
#include <vector>

#include "kernels_common.hpp"
#include "mfma_rankk.hpp"
#include "multifrontal.hpp"

namespace eigsol {

namespace dev {

struct MfFront {
    int64_t off;    // front at F + off: d x d, column-major, leading dimension d
    int64_t uoff;   // forward contribution vector (ms entries) at u + uoff
    int64_t sof;    // struct indices (new numbering) at sidx + sof; their positions in the parent's list at cmap + sof
    int32_t d, ns, c0, ms;
    int32_t ch0, ch1;   // children chl[ch0 .. ch1) (fixed order)
    int32_t parent;
    int32_t flag0;  // large fronts: first of the front's pivot-block flags; -1: solved by one workgroup
    int64_t zoff;   // large fronts: assembled right-hand side (d entries) at z + zoff
    int64_t goff;   // inverse form (ns <= 64, d <= 256; -1: none) at F + goff: [inv(L11); L21 inv(L11)]
                    // (d x ns, ld d), then [inv(U11), -inv(U11) U12] (ns x d, ld ns)
};

__device__ __forceinline__ double mf_rl(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), src);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ cplx mf_rl(cplx v, int src) { return cplx{mf_rl(v.re, src), mf_rl(v.im, src)}; }
// write-through stores / agent-scope loads of values handed between workgroups of one launch
__device__ __forceinline__ void mf_st(double* p, double v) { st_agent(p, v); }
__device__ __forceinline__ void mf_st(cplx* p, cplx v) {
    st_agent(&p->re, v.re);
    st_agent(&p->im, v.im);
}
__device__ __forceinline__ double mf_ld(const double* p) { return ld_agent(p); }
__device__ __forceinline__ cplx mf_ld(const cplx* p) { return cplx{ld_agent(&p->re), ld_agent(&p->im)}; }

// value flags of the row-block solve (EIGSOL_MF_VALFLAG): an unsolved pivot value holds this NaN in
// every 8-byte word, a solved one never does (a NaN result is stored as the default quiet NaN), so a
// waiting block polls the values themselves instead of a flag and then the values
#ifndef EIGSOL_MF_UNROLL
#define EIGSOL_MF_UNROLL 8   // loads in flight per thread in the small fronts' inverse-form products
#endif
constexpr unsigned long long kMfSent = 0x7FF4DEAD7FF4DEADull;
__device__ __forceinline__ bool mf_unready(double v) { return (unsigned long long)__double_as_longlong(v) == kMfSent; }
__device__ __forceinline__ bool mf_unready(cplx v) { return mf_unready(v.re) || mf_unready(v.im); }
__device__ __forceinline__ double mf_sent(double) { return __longlong_as_double((long long)kMfSent); }
__device__ __forceinline__ cplx mf_sent(cplx) { return cplx{mf_sent(0.0), mf_sent(0.0)}; }
__device__ __forceinline__ double mf_clean(double v) { return v != v ? __longlong_as_double(0x7FF8000000000000ll) : v; }
__device__ __forceinline__ cplx mf_clean(cplx v) { return cplx{mf_clean(v.re), mf_clean(v.im)}; }
template <class S>
__device__ __forceinline__ S mf_poll(const S* p, int32_t* err, int bo) {
    S v = mf_ld(p);
    int spins = 0;
    while (mf_unready(v)) {
        if (!(bo & 1)) __builtin_amdgcn_s_sleep(1);
        else if (spins < 4) __builtin_amdgcn_s_sleep(2);
        else __builtin_amdgcn_s_sleep(8);
        v = mf_ld(p);
        if (++spins > (1 << 22)) {
            atomicOr(err, 4);
            break;
        }
    }
    return v;
}

// M's entries into their fronts: F[dst[e]] = v[e] (every destination distinct)
template <class S>
__global__ __launch_bounds__(256) void mf_scatter_kernel(const int64_t* dst, const S* v, int64_t nnz, S* F) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e < nnz) F[dst[e]] = v[e];
}

// extend-add of one child's Schur block into its parent: tab = (child, first column) pairs, 64
// columns per workgroup; children of one parent are in different launches (fixed order)
template <class S>
__global__ __launch_bounds__(256) void mf_extend_kernel(const MfFront* fr, const int32_t* tab, const int32_t* cmap,
                                                        S* F) {
    const int32_t c = tab[2 * blockIdx.x], col0 = tab[2 * blockIdx.x + 1];
    const MfFront fc = fr[c];
    const MfFront fp = fr[fc.parent];
    const int32_t* map = cmap + fc.sof;
    const S* src = F + fc.off + (int64_t)fc.ns * (fc.d + 1);
    S* dst = F + fp.off;
    const int cend = min(fc.ms, col0 + 64);
    for (int cc = col0; cc < cend; ++cc) {
        const int64_t pc = (int64_t)map[cc] * fp.d;
        const S* sc = src + (int64_t)cc * fc.d;
        for (int r = threadIdx.x; r < fc.ms; r += 256) {
            const int64_t o = pc + map[r];
            dst[o] = add(dst[o], sc[r]);
        }
    }
}

// a / b for a pivot b whose squared modulus underflows (exact power-of-two scaling of b)
__device__ inline double sdiv_tiny(double a, double b) { return a / b; }
__device__ inline cplx sdiv_tiny(cplx a, cplx b) {
    const cplx q = cdiv(a, cplx{ldexp(b.re, 600), ldexp(b.im, 600)});
    return cplx{ldexp(q.re, 600), ldexp(q.im, 600)};
}

// Panel q of every front in list[0 .. gridDim.x): pivots k0 .. k0 + kb - 1 (k0 = q NB), each the
// first row of largest modulus among the front's remaining pivot rows [k, ns); the whole row
// swapped (all d columns), the column below the diagonal scaled, the panel's other columns
// rank-1 updated; then U12 = L11^-1 A12 on the columns right of the panel (one column per thread).
// tau > 0 (static pivoting, the retry after a zero pivot): a pivot column whose remaining front
// rows are all exactly zero gets the pivot tau on its diagonal (counted in *nstat) instead of
// failing - a perturbation of M that the checked solve's GMRES refinement then removes.
template <class S, int NB>
__global__ __launch_bounds__(256) void mf_panel_kernel(const MfFront* fr, const int32_t* list, int q, S* F,
                                                       int32_t* piv, int32_t* zpiv, double tau, int32_t* nstat) {
    __shared__ double sv[4];
    __shared__ int si[4];
    __shared__ int s_p, s_fix;
    __shared__ S l11[NB * NB];
    const MfFront f = fr[list[blockIdx.x]];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int d = f.d, ns = f.ns;
    const int k0 = q * NB, kb = min(NB, ns - k0), c1 = k0 + kb;
    S* A = F + f.off;
    for (int k = k0; k < c1; ++k) {
        double best = -1.0;
        int bi = k;
        for (int i = k + tid; i < ns; i += 256) {
            const double s = mod_abs(A[i + (int64_t)k * d]);   // no underflow below |a| ~ 1e-162
            if (s > best) { best = s; bi = i; }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const double ob = __shfl_xor(best, off, 64);
            const int oi = __shfl_xor(bi, off, 64);
            if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
        }
        if (lane == 0) { sv[wv] = best; si[wv] = bi; }
        __syncthreads();
        if (tid == 0) {
            double b = sv[0];
            int p = si[0];
            for (int w = 1; w < 4; ++w)
                if (sv[w] > b || (sv[w] == b && si[w] < p)) { b = sv[w]; p = si[w]; }
            s_p = p;
            piv[f.c0 + k] = p;
            s_fix = 0;
            if (!(b > 0.0)) {
                if (tau > 0.0) {
                    s_fix = 1;
                    atomicAdd(nstat, 1);
                } else {
                    atomicOr(zpiv, 1);
                }
            }
        }
        __syncthreads();
        const int p = s_p;
        if (s_fix) {   // the whole column is zero in the front's rows: p == k, no interchange
            if (tid == 0) set_re_im(A[k + (int64_t)k * d], tau, 0.0);
            __syncthreads();
        }
        if (p != k)
            for (int j = tid; j < d; j += 256) {
                const S t = A[k + (int64_t)j * d];
                A[k + (int64_t)j * d] = A[p + (int64_t)j * d];
                A[p + (int64_t)j * d] = t;
            }
        __syncthreads();
        const S dk = A[k + (int64_t)k * d];
        if (sq_abs(dk) >= 1e-280) {
            for (int i = k + 1 + tid; i < d; i += 256) A[i + (int64_t)k * d] = sdiv(A[i + (int64_t)k * d], dk);
        } else if (mod_abs(dk) > 0.0) {
            // |pivot| below ~1e-140: its squared modulus (the textbook complex quotient's
            // denominator) would underflow; divide by the pivot scaled by 2^600, then rescale
            for (int i = k + 1 + tid; i < d; i += 256) A[i + (int64_t)k * d] = sdiv_tiny(A[i + (int64_t)k * d], dk);
        }
        __syncthreads();
        const int m = d - k - 1, w = c1 - k - 1;
        for (int e = tid; e < m * w; e += 256) {
            const int i = k + 1 + e % m, j = k + 1 + e / m;
            A[i + (int64_t)j * d] = sub(A[i + (int64_t)j * d], mul(A[i + (int64_t)k * d], A[k + (int64_t)j * d]));
        }
        __syncthreads();
    }
    for (int e = tid; e < kb * kb; e += 256) {
        const int i = e % kb, j = e / kb;
        l11[i + j * NB] = A[(k0 + i) + (int64_t)(k0 + j) * d];
    }
    __syncthreads();
    for (int c = c1 + tid; c < d; c += 256) {
        S* col = A + (int64_t)c * d + k0;
        S x[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) x[i] = i < kb ? col[i] : s_zero<S>();
#pragma unroll
        for (int j = 0; j < NB - 1; ++j) {
            if (j < kb) {
#pragma unroll
                for (int i = j + 1; i < NB; ++i) x[i] = sub(x[i], mul(l11[i + j * NB], x[j]));
            }
        }
#pragma unroll
        for (int i = 0; i < NB; ++i)
            if (i < kb) col[i] = x[i];
    }
}

// trailing update of panel q, every front of the launch: tab = (front, tile row, tile column)
template <class S, int NB>
__global__ __launch_bounds__(256) void mf_gemm_kernel(const MfFront* fr, const int32_t* tab, int q, S* F) {
    const int32_t s = tab[3 * blockIdx.x], tr = tab[3 * blockIdx.x + 1], tc = tab[3 * blockIdx.x + 2];
    const MfFront f = fr[s];
    const int d = f.d, k0 = q * NB, kb = min(NB, f.ns - k0), c1 = k0 + kb, m = d - c1;
    S* A = F + f.off;
    rankk_tile<S, true>(tr, tc, m, m, kb, -1.0, A + c1 + (int64_t)k0 * d, d, A + k0 + (int64_t)c1 * d, d,
                        A + c1 + (int64_t)c1 * d, d);
}

// ---------------------------------------------------------------- solve
// w = b in the new numbering
template <class S>
__global__ __launch_bounds__(256) void mf_gather_kernel(const int32_t* perm, const S* b, S* w, int64_t n,
                                                        const uint8_t* bigm) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) w[i] = (bigm && bigm[i]) ? mf_sent(s_zero<S>()) : b[perm[i]];   // bigm: large fronts' pivot rows
}
template <class S>
__global__ __launch_bounds__(256) void mf_scatter_out_kernel(const int32_t* perm, const S* x, S* out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[perm[i]] = x[i];
}

// forward: fronts list[0 .. gridDim.x) of one height.  LDS: r (ns), y (ns), acc (ms).
template <class S>
__device__ __forceinline__ void mf_fwd_front(const MfFront f, unsigned char* lds_raw, const MfFront* fr,
                                             const int32_t* chl, const S* F, const int32_t* cmap, const int32_t* pinv,
                                             S* w, S* u) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int d = f.d, ns = f.ns, ms = f.ms;
    S* r = reinterpret_cast<S*>(lds_raw);
    S* y = r + ns;
    S* acc = y + ns;
    // up to KC children: every child's header, its first 256 (position, value) pairs and this
    // thread's pivot index are loaded before anything waits on them (one chain of dependent loads
    // instead of one per child); the contributions are then applied child by child in the fixed
    // order, as before
    constexpr int KC = 4;
    const int nch = f.ch1 - f.ch0;
    const bool pre = nch <= KC;
    int cms[KC], cpos[KC];
    const int32_t* cmp[KC];
    const S* cup[KC];
    S cval[KC];
    if (pre) {
#pragma unroll
        for (int q = 0; q < KC; ++q)
            if (q < nch) {
                const MfFront c = fr[chl[f.ch0 + q]];
                cms[q] = c.ms;
                cmp[q] = cmap + c.sof;
                cup[q] = u + c.uoff;
            }
#pragma unroll
        for (int q = 0; q < KC; ++q)
            if (q < nch && tid < cms[q]) {
                cpos[q] = cmp[q][tid];
                cval[q] = cup[q][tid];
            }
    }
    const int pv = tid < ns ? pinv[f.c0 + tid] : 0;
    for (int t = tid; t < ns; t += 256) r[t] = w[f.c0 + t];
    for (int t = tid; t < ms; t += 256) acc[t] = s_zero<S>();
    __syncthreads();
    auto apply = [&](int pos, S v) {
        if (pos < ns) r[pos] = sub(r[pos], v);
        else acc[pos - ns] = add(acc[pos - ns], v);
    };
    if (pre) {
#pragma unroll
        for (int q = 0; q < KC; ++q)
            if (q < nch) {
                if (tid < cms[q]) apply(cpos[q], cval[q]);
                for (int t = tid + 256; t < cms[q]; t += 256) apply(cmp[q][t], cup[q][t]);
                __syncthreads();
            }
    } else {
        for (int k = f.ch0; k < f.ch1; ++k) {
            const MfFront c = fr[chl[k]];
            const int32_t* map = cmap + c.sof;
            const S* uc = u + c.uoff;
            for (int t = tid; t < c.ms; t += 256) apply(map[t], uc[t]);
            __syncthreads();
        }
    }
    if (tid < ns) y[tid] = r[pv];
    for (int t = tid + 256; t < ns; t += 256) y[t] = r[pinv[f.c0 + t]];
    __syncthreads();
    if (f.goff >= 0) {
        // one product over the d rows, tpr threads per row (columns interleaved), partials summed
        // in a fixed order
        const S* G = F + f.goff;
        if (d > 128) {   // one thread per row
            for (int i = tid; i < d; i += 256) {
                S v = s_zero<S>();
                const S* Gi = G + i;
                const int jn = i < ns ? i + 1 : ns;   // inv(L11) is lower triangular: skip its zeros
#pragma unroll EIGSOL_MF_UNROLL
                for (int j = 0; j < jn; ++j) v = add(v, mul(Gi[(int64_t)j * d], y[j]));
                if (i < ns) w[f.c0 + i] = v;
                else u[f.uoff + i - ns] = add(acc[i - ns], v);
            }
            return;
        }
        S* part = acc + ms;
        const int R = d <= 64 ? 64 : 128, tpr = 256 / R;
        const int i = tid % R, p = tid / R;
        S sacc = s_zero<S>();
        if (i < d) {
            const S* Gi = G + i;
            const int jn = i < ns ? i + 1 : ns;   // inv(L11) is lower triangular: skip its zeros
#pragma unroll EIGSOL_MF_UNROLL
            for (int j = p; j < jn; j += tpr) sacc = add(sacc, mul(Gi[(int64_t)j * d], y[j]));
        }
        part[p * R + i] = sacc;
        __syncthreads();
        if (tid < d) {
            S v = part[tid];
            for (int q = 1; q < tpr; ++q) v = add(v, part[q * R + tid]);
            if (tid < ns) w[f.c0 + tid] = v;
            else u[f.uoff + tid - ns] = add(acc[tid - ns], v);
        }
        return;
    }
    const S* A = F + f.off;
    for (int jb = 0; jb < ns; jb += 64) {
        const int bw = min(64, ns - jb);
        if (wv == 0) {
            S v = lane < bw ? y[jb + lane] : s_zero<S>();
            const int row = jb + min(lane, bw - 1);
            for (int j0 = 0; j0 < bw; j0 += 16) {
                S lv[16];
#pragma unroll
                for (int t = 0; t < 16; ++t) lv[t] = A[row + (int64_t)(jb + min(j0 + t, bw - 1)) * d];
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    const int j = j0 + t;
                    if (j < bw) {
                        const S yj = mf_rl(v, j);
                        if (lane > j) v = sub(v, mul(lv[t], yj));
                    }
                }
            }
            if (lane < bw) y[jb + lane] = v;
        }
        __syncthreads();
        for (int i = jb + bw + tid; i < d; i += 256) {
            S s = s_zero<S>();
            const S* Ai = A + i + (int64_t)jb * d;
            for (int j0 = 0; j0 < bw; j0 += 16) {
                S lv[16];
#pragma unroll
                for (int t = 0; t < 16; ++t) lv[t] = Ai[(int64_t)min(j0 + t, bw - 1) * d];
#pragma unroll
                for (int t = 0; t < 16; ++t)
                    if (j0 + t < bw) s = add(s, mul(lv[t], y[jb + j0 + t]));
            }
            if (i < ns) y[i] = sub(y[i], s);
            else acc[i - ns] = add(acc[i - ns], s);
        }
        __syncthreads();
    }
    for (int t = tid; t < ns; t += 256) w[f.c0 + t] = y[t];
    for (int t = tid; t < ms; t += 256) u[f.uoff + t] = acc[t];
}

template <class S>
__global__ __launch_bounds__(256) void mf_fwd_kernel(const MfFront* fr, const int32_t* list, const int32_t* chl,
                                                     const S* F, const int32_t* cmap, const int32_t* pinv, S* w,
                                                     S* u) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    mf_fwd_front<S>(fr[list[blockIdx.x]], lds_raw, fr, chl, F, cmap, pinv, w, u);
}

// a whole small subtree per workgroup: its fronts are the postorder range [lo, hi], children
// before parents, so the forward pass walks it upward without any other workgroup (the children's
// contributions were written by this workgroup, visible after its barrier)
template <class S>
__global__ __launch_bounds__(256) void mf_fwd_sub_kernel(const MfFront* fr, const int32_t* ranges, const int32_t* chl,
                                                         const S* F, const int32_t* cmap, const int32_t* pinv, S* w,
                                                         S* u) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const int32_t lo = ranges[2 * blockIdx.x], hi = ranges[2 * blockIdx.x + 1];
    for (int32_t s = lo; s <= hi; ++s) {
        mf_fwd_front<S>(fr[s], lds_raw, fr, chl, F, cmap, pinv, w, u);
        __syncthreads();
    }
}

// backward: fronts list[0 .. gridDim.x) of one height (their ancestors solved).  LDS: t (ns), xs (ms).
template <class S>
__device__ __forceinline__ void mf_bwd_front(const MfFront f, unsigned char* lds_raw, const S* F,
                                             const int32_t* sidx, const S* w, S* x) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int d = f.d, ns = f.ns, ms = f.ms;
    S* t = reinterpret_cast<S*>(lds_raw);
    S* xs = t + ns;
    const S w0 = tid < ns ? w[f.c0 + tid] : s_zero<S>();   // issued before the struct gather waits
    for (int q = tid; q < ms; q += 256) xs[q] = x[sidx[f.sof + q]];
    if (f.goff >= 0) {
        // x(pivots) = [inv(U11), -inv(U11) U12] [w(pivots); x(struct)]: wave p takes columns p, p + 4, ...
        if (tid < ns) t[tid] = w0;
        for (int q = tid + 256; q < ns; q += 256) t[q] = w[f.c0 + q];
        __syncthreads();
        const S* G = F + f.goff + (int64_t)d * ns;
        S* part = xs + ms;
        const int k = lane, p = wv;
        S sacc = s_zero<S>();
        if (k < ns) {
            const S* Gk = G + k;
            // inv(U11) is upper triangular: columns from k on (the first of them congruent to p mod 4)
            const int c0 = k > p ? p + ((k - p + 3) / 4) * 4 : p;
#pragma unroll EIGSOL_MF_UNROLL
            for (int c = c0; c < d; c += 4) sacc = add(sacc, mul(Gk[(int64_t)c * ns], c < ns ? t[c] : xs[c - ns]));
        }
        part[p * 64 + k] = sacc;
        __syncthreads();
        if (tid < ns) x[f.c0 + tid] = add(add(add(part[tid], part[64 + tid]), part[128 + tid]), part[192 + tid]);
        return;
    }
    __syncthreads();
    const S* A = F + f.off;
    for (int k = tid; k < ns; k += 256) {
        S s = s_zero<S>();
        const S* Ak = A + k + (int64_t)ns * d;
        int q0 = 0;
        for (; q0 + 8 <= ms; q0 += 8) {
            S uv[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) uv[e] = Ak[(int64_t)(q0 + e) * d];
#pragma unroll
            for (int e = 0; e < 8; ++e) s = add(s, mul(uv[e], xs[q0 + e]));
        }
        for (; q0 < ms; ++q0) s = add(s, mul(Ak[(int64_t)q0 * d], xs[q0]));
        t[k] = sub(w[f.c0 + k], s);
    }
    __syncthreads();
    for (int jb = ((ns - 1) / 64) * 64; jb >= 0; jb -= 64) {
        const int bw = min(64, ns - jb);
        if (wv == 0) {
            S v = lane < bw ? t[jb + lane] : s_zero<S>();
            const int row = jb + min(lane, bw - 1);
            for (int j1 = bw; j1 > 0; j1 -= 16) {
                S uv[16];
#pragma unroll
                for (int e = 0; e < 16; ++e) uv[e] = A[row + (int64_t)(jb + max(j1 - 1 - e, 0)) * d];
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int j = j1 - 1 - e;
                    if (j >= 0) {
                        if (lane == j) v = sdiv(v, uv[e]);
                        const S xj = mf_rl(v, j);
                        if (lane < j) v = sub(v, mul(uv[e], xj));
                    }
                }
            }
            if (lane < bw) t[jb + lane] = v;
        }
        __syncthreads();
        for (int i = tid; i < jb; i += 256) {
            S s = s_zero<S>();
            const S* Ai = A + i + (int64_t)jb * d;
            for (int j0 = 0; j0 < bw; j0 += 16) {
                S uv[16];
#pragma unroll
                for (int e = 0; e < 16; ++e) uv[e] = Ai[(int64_t)min(j0 + e, bw - 1) * d];
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    if (j0 + e < bw) s = add(s, mul(uv[e], t[jb + j0 + e]));
            }
            t[i] = sub(t[i], s);
        }
        __syncthreads();
    }
    for (int k = tid; k < ns; k += 256) x[f.c0 + k] = t[k];
}

template <class S>
__global__ __launch_bounds__(256) void mf_bwd_kernel(const MfFront* fr, const int32_t* list, const S* F,
                                                     const int32_t* sidx, const S* w, S* x) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    mf_bwd_front<S>(fr[list[blockIdx.x]], lds_raw, F, sidx, w, x);
}

// the backward pass over a small subtree: parents before children (the subtree root's ancestors
// were solved by earlier launches)
template <class S>
__global__ __launch_bounds__(256) void mf_bwd_sub_kernel(const MfFront* fr, const int32_t* ranges, const S* F,
                                                         const int32_t* sidx, const S* w, S* x) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const int32_t lo = ranges[2 * blockIdx.x], hi = ranges[2 * blockIdx.x + 1];
    for (int32_t s = hi; s >= lo; --s) {
        mf_bwd_front<S>(fr[s], lds_raw, F, sidx, w, x);
        __syncthreads();
    }
}

// ---- small fronts (ns <= 64 pivots, ms <= 192 struct rows): one wave per front, four fronts per
// workgroup, no workgroup barrier (each wave's LDS slice is its own), so a CU keeps up to 32
// fronts in flight.  Same arithmetic order as mf_fwd_kernel / mf_bwd_kernel's single block.
constexpr int kWaveNs = 64, kWaveMs = 192;

__device__ __forceinline__ void mf_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <class S>
__global__ __launch_bounds__(256) void mf_fwd_wave_kernel(const MfFront* fr, const int32_t* list, int32_t cnt,
                                                          const int32_t* chl, const S* F, const int32_t* cmap,
                                                          const int32_t* pinv, S* w, S* u) {
    __shared__ S sh[4][2 * kWaveNs + kWaveMs];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int t = blockIdx.x * 4 + wv;
    if (t >= cnt) return;
    const MfFront f = fr[list[t]];
    const int d = f.d, ns = f.ns, ms = f.ms;
    S* r = sh[wv];
    S* y = r + kWaveNs;
    S* acc = y + kWaveNs;
    if (lane < ns) r[lane] = w[f.c0 + lane];
    for (int k = lane; k < ms; k += 64) acc[k] = s_zero<S>();
    mf_wave_sync();
    for (int k = f.ch0; k < f.ch1; ++k) {
        const MfFront c = fr[chl[k]];
        const int32_t* map = cmap + c.sof;
        const S* uc = u + c.uoff;
        for (int q = lane; q < c.ms; q += 64) {
            const int pos = map[q];
            const S v = uc[q];
            if (pos < ns) r[pos] = sub(r[pos], v);
            else acc[pos - ns] = add(acc[pos - ns], v);
        }
        mf_wave_sync();
    }
    const S* A = F + f.off;
    S v = lane < ns ? r[pinv[f.c0 + lane]] : s_zero<S>();
    const int row = min(lane, ns - 1);
    for (int j0 = 0; j0 < ns; j0 += 16) {
        S lv[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) lv[q] = A[row + (int64_t)min(j0 + q, ns - 1) * d];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int j = j0 + q;
            if (j < ns) {
                const S yj = mf_rl(v, j);
                if (lane > j) v = sub(v, mul(lv[q], yj));
            }
        }
    }
    if (lane < ns) {
        y[lane] = v;
        w[f.c0 + lane] = v;
    }
    mf_wave_sync();
    for (int i = ns + lane; i < d; i += 64) {
        S sacc = s_zero<S>();
        const S* Ai = A + i;
        for (int j0 = 0; j0 < ns; j0 += 16) {
            S lv[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) lv[q] = Ai[(int64_t)min(j0 + q, ns - 1) * d];
#pragma unroll
            for (int q = 0; q < 16; ++q)
                if (j0 + q < ns) sacc = add(sacc, mul(lv[q], y[j0 + q]));
        }
        u[f.uoff + (i - ns)] = add(acc[i - ns], sacc);
    }
}

template <class S>
__global__ __launch_bounds__(256) void mf_bwd_wave_kernel(const MfFront* fr, const int32_t* list, int32_t cnt,
                                                          const S* F, const int32_t* sidx, const S* w, S* x) {
    __shared__ S sh[4][kWaveMs];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int t = blockIdx.x * 4 + wv;
    if (t >= cnt) return;
    const MfFront f = fr[list[t]];
    const int d = f.d, ns = f.ns, ms = f.ms;
    S* xs = sh[wv];
    for (int q = lane; q < ms; q += 64) xs[q] = x[sidx[f.sof + q]];
    mf_wave_sync();
    const S* A = F + f.off;
    const int row = min(lane, ns - 1);
    S s = s_zero<S>();
    {
        const S* Ak = A + row + (int64_t)ns * d;
        for (int q0 = 0; q0 < ms; q0 += 16) {
            S uv[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) uv[e] = Ak[(int64_t)min(q0 + e, ms - 1) * d];
#pragma unroll
            for (int e = 0; e < 16; ++e)
                if (q0 + e < ms) s = add(s, mul(uv[e], xs[q0 + e]));
        }
    }
    S v = lane < ns ? sub(w[f.c0 + lane], s) : s_zero<S>();
    for (int j1 = ns; j1 > 0; j1 -= 16) {
        S uv[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) uv[e] = A[row + (int64_t)max(j1 - 1 - e, 0) * d];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int j = j1 - 1 - e;
            if (j >= 0) {
                if (lane == j) v = sdiv(v, uv[e]);
                const S xj = mf_rl(v, j);
                if (lane < j) v = sub(v, mul(uv[e], xj));
            }
        }
    }
    if (lane < ns) x[f.c0 + lane] = v;
}

// ---- the lower heights in one launch each way (dataflow, opt-in EIGSOL_MF_FLOW=1): one workgroup
// per front in height order (forward ascending, backward descending), waiting for the fronts it
// reads - the children's contributions (forward) or the parent's solution (backward) - through
// per-front epoch flags; a front only waits for fronts of lower workgroup index (in-order
// dispatch), values are handed over write-through and loaded at agent scope.  Same arithmetic, in
// the same order, as mf_fwd_kernel / mf_bwd_kernel.  Measured and rejected as the default: 2.01 ->
// 4.5 ms per 1M iteration (waiting workgroups hold the CU slots the producers need, and the
// acquire polls invalidate L2).  A ticket-ordered persistent variant hung in a way that device
// printf made disappear; not kept.
__device__ __forceinline__ void mf_wait_flag(const int32_t* f, int32_t epoch, int32_t* err, int who = -1) {
    (void)who;
    int spins = 0;
    while (__hip_atomic_load(const_cast<int32_t*>(f), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1 << 22)) {
            atomicOr(err, 2);
            break;
        }
    }
}

template <class S>
__global__ __launch_bounds__(256) void mf_fwd_flow_kernel(const MfFront* fr, const int32_t* order, int32_t cnt,
                                                          int32_t* done, int32_t epoch, const int32_t* chl,
                                                          const S* F, const int32_t* cmap, const int32_t* pinv, S* w,
                                                          S* u, int32_t* err) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    {
        const int32_t t = (int32_t)blockIdx.x;
        if (t >= cnt) return;
        const int32_t sidx_f = order[t];
        const MfFront f = fr[sidx_f];
        const int d = f.d, ns = f.ns, ms = f.ms;
        S* r = reinterpret_cast<S*>(lds_raw);
        S* y = r + ns;
        S* acc = y + ns;
        for (int k = f.ch0 + tid; k < f.ch1; k += 256) mf_wait_flag(done + chl[k], epoch, err, sidx_f);
        for (int q = tid; q < ns; q += 256) r[q] = w[f.c0 + q];
        for (int q = tid; q < ms; q += 256) acc[q] = s_zero<S>();
        __syncthreads();
        for (int k = f.ch0; k < f.ch1; ++k) {
            const MfFront c = fr[chl[k]];
            const int32_t* map = cmap + c.sof;
            const S* uc = u + c.uoff;
            for (int q = tid; q < c.ms; q += 256) {
                const int pos = map[q];
                const S v = mf_ld(uc + q);
                if (pos < ns) r[pos] = sub(r[pos], v);
                else acc[pos - ns] = add(acc[pos - ns], v);
            }
            __syncthreads();
        }
        for (int q = tid; q < ns; q += 256) y[q] = r[pinv[f.c0 + q]];
        __syncthreads();
        const S* A = F + f.off;
        for (int jb = 0; jb < ns; jb += 64) {
            const int bw = min(64, ns - jb);
            if (wv == 0) {
                S v = lane < bw ? y[jb + lane] : s_zero<S>();
                const int row = jb + min(lane, bw - 1);
                for (int j0 = 0; j0 < bw; j0 += 16) {
                    S lv[16];
#pragma unroll
                    for (int q = 0; q < 16; ++q) lv[q] = A[row + (int64_t)(jb + min(j0 + q, bw - 1)) * d];
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const int j = j0 + q;
                        if (j < bw) {
                            const S yj = mf_rl(v, j);
                            if (lane > j) v = sub(v, mul(lv[q], yj));
                        }
                    }
                }
                if (lane < bw) y[jb + lane] = v;
            }
            __syncthreads();
            for (int i = jb + bw + tid; i < d; i += 256) {
                S sacc = s_zero<S>();
                const S* Ai = A + i + (int64_t)jb * d;
                for (int j0 = 0; j0 < bw; j0 += 16) {
                    S lv[16];
#pragma unroll
                    for (int q = 0; q < 16; ++q) lv[q] = Ai[(int64_t)min(j0 + q, bw - 1) * d];
#pragma unroll
                    for (int q = 0; q < 16; ++q)
                        if (j0 + q < bw) sacc = add(sacc, mul(lv[q], y[jb + j0 + q]));
                }
                if (i < ns) y[i] = sub(y[i], sacc);
                else acc[i - ns] = add(acc[i - ns], sacc);
            }
            __syncthreads();
        }
        for (int q = tid; q < ns; q += 256) w[f.c0 + q] = y[q];
        for (int q = tid; q < ms; q += 256) mf_st(u + f.uoff + q, acc[q]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // release: writes the XCD's L2 back, so pollers on other XCDs see the flag and the values
        // (a relaxed agent-scope store was measured never to reach them)
        if (tid == 0) __hip_atomic_store(done + sidx_f, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <class S>
__global__ __launch_bounds__(256) void mf_bwd_flow_kernel(const MfFront* fr, const int32_t* order, int32_t cnt,
                                                          int32_t* done, int32_t epoch, int32_t hflow,
                                                          const int32_t* height, const S* F, const int32_t* sidx,
                                                          const S* w, S* x, int32_t* err) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    {
        const int32_t t = (int32_t)blockIdx.x;
        if (t >= cnt) return;
        const int32_t sf = order[t];
        const MfFront f = fr[sf];
        const int d = f.d, ns = f.ns, ms = f.ms;
        S* tv_ = reinterpret_cast<S*>(lds_raw);
        S* xs = tv_ + ns;
        if (tid == 0 && f.parent >= 0 && height[f.parent] < hflow) mf_wait_flag(done + f.parent, epoch, err, sf);
        __syncthreads();
        for (int q = tid; q < ms; q += 256) xs[q] = mf_ld(x + sidx[f.sof + q]);
        __syncthreads();
        const S* A = F + f.off;
        for (int k = tid; k < ns; k += 256) {
            S sacc = s_zero<S>();
            const S* Ak = A + k + (int64_t)ns * d;
            int q0 = 0;
            for (; q0 + 8 <= ms; q0 += 8) {
                S uv[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) uv[e] = Ak[(int64_t)(q0 + e) * d];
#pragma unroll
                for (int e = 0; e < 8; ++e) sacc = add(sacc, mul(uv[e], xs[q0 + e]));
            }
            for (; q0 < ms; ++q0) sacc = add(sacc, mul(Ak[(int64_t)q0 * d], xs[q0]));
            tv_[k] = sub(w[f.c0 + k], sacc);
        }
        __syncthreads();
        for (int jb = ((ns - 1) / 64) * 64; jb >= 0; jb -= 64) {
            const int bw = min(64, ns - jb);
            if (wv == 0) {
                S v = lane < bw ? tv_[jb + lane] : s_zero<S>();
                const int row = jb + min(lane, bw - 1);
                for (int j1 = bw; j1 > 0; j1 -= 16) {
                    S uv[16];
#pragma unroll
                    for (int e = 0; e < 16; ++e) uv[e] = A[row + (int64_t)(jb + max(j1 - 1 - e, 0)) * d];
#pragma unroll
                    for (int e = 0; e < 16; ++e) {
                        const int j = j1 - 1 - e;
                        if (j >= 0) {
                            if (lane == j) v = sdiv(v, uv[e]);
                            const S xj = mf_rl(v, j);
                            if (lane < j) v = sub(v, mul(uv[e], xj));
                        }
                    }
                }
                if (lane < bw) tv_[jb + lane] = v;
            }
            __syncthreads();
            for (int i = tid; i < jb; i += 256) {
                S sacc = s_zero<S>();
                const S* Ai = A + i + (int64_t)jb * d;
                for (int j0 = 0; j0 < bw; j0 += 16) {
                    S uv[16];
#pragma unroll
                    for (int e = 0; e < 16; ++e) uv[e] = Ai[(int64_t)min(j0 + e, bw - 1) * d];
#pragma unroll
                    for (int e = 0; e < 16; ++e)
                        if (j0 + e < bw) sacc = add(sacc, mul(uv[e], tv_[jb + j0 + e]));
                }
                tv_[i] = sub(tv_[i], sacc);
            }
            __syncthreads();
        }
        for (int k = tid; k < ns; k += 256) mf_st(x + f.c0 + k, tv_[k]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(done + sf, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---- large fronts: one workgroup per 64-row block, sync-free (the dense path's blocked TRSV,
// shifted.hip dense_trsv_kernel, on a front).  Pivot block k of a front publishes its solved 64
// values with write-through stores and raises flag[flag0 + k] to the solve's epoch; a row block
// waits for the flags of the blocks it multiplies.  Blocks a row block waits for have lower
// workgroup indices (forward: ascending pivot blocks, then the struct rows; backward: descending),
// and the launches are small (hundreds of workgroups, all resident), so every wait ends.
// back-off: short sleeps (the chain's hand-off latency is what a solve waits on; the pollers are
// a few hundred workgroups), or the dense TRSV's growing sleeps (EIGSOL_MF_BACKOFF=1)
__device__ __forceinline__ void mf_wait(const int32_t* f, int32_t epoch, int32_t* err, int bo) {
    int spins = 0;
    for (;;) {
        const int32_t v = (bo & 2) ? __hip_atomic_load(const_cast<int32_t*>(f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : __hip_atomic_load(const_cast<int32_t*>(f), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (v == epoch) break;
        if (!(bo & 1)) __builtin_amdgcn_s_sleep(1);
        else if (spins < 4) __builtin_amdgcn_s_sleep(2);
        else if (spins < 16) __builtin_amdgcn_s_sleep(8);
        else __builtin_amdgcn_s_sleep(32);
        if (++spins > (1 << 24)) { atomicOr(err, 1); break; }
    }
}

// z (d entries per large front) = the permuted pivot right-hand side, then the children's
// contributions to the struct rows; one workgroup per front.  LDS: r (ns)
template <class S>
__device__ __forceinline__ void mf_big_asm_front(const MfFront& f, unsigned char* lds_raw, const MfFront* fr,
                                                 const int32_t* chl, const int32_t* cmap, const int32_t* pinv, S* w,
                                                 const S* u, S* z, int bo) {
    const int tid = threadIdx.x, ns = f.ns, ms = f.ms;
    S* r = reinterpret_cast<S*>(lds_raw);
    S* zs = z + f.zoff;
    for (int t = tid; t < ns; t += 256) r[t] = w[f.c0 + t];
    for (int t = tid; t < ms; t += 256) zs[ns + t] = s_zero<S>();
    __syncthreads();
    for (int k = f.ch0; k < f.ch1; ++k) {
        const MfFront c = fr[chl[k]];
        const int32_t* map = cmap + c.sof;
        const S* uc = u + c.uoff;
        for (int t = tid; t < c.ms; t += 256) {
            const int pos = map[t];
            const S v = uc[t];
            if (pos < ns) r[pos] = sub(r[pos], v);
            else zs[pos] = add(zs[pos], v);   // each position once per child: no race
        }
        __syncthreads();
    }
    for (int t = tid; t < ns; t += 256) zs[t] = r[pinv[f.c0 + t]];
    // value flags: the pivot rows' w (read above, before the barrier) becomes "unsolved" for
    // mf_big_fwd_kernel, the next launch
    if (bo & 4)
        for (int t = tid; t < ns; t += 256) mf_st(w + f.c0 + t, mf_sent(s_zero<S>()));
}

template <class S>
__global__ __launch_bounds__(256) void mf_big_asm_kernel(const MfFront* fr, const int32_t* list, const int32_t* chl,
                                                         const int32_t* cmap, const int32_t* pinv, S* w,
                                                         const S* u, S* z, int bo) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    mf_big_asm_front<S>(fr[list[blockIdx.x]], lds_raw, fr, chl, cmap, pinv, w, u, z, bo);
}

// mf_big_asm_front for mf_fwd_height_kernel: the pivot right-hand side read from b through perm (the
// gather left these rows of w unsolved), the struct rows summed in LDS too, and every z entry stored
// once with its value as its flag.  The same sums in the same order.  LDS: r (d)
template <class S>
__device__ __forceinline__ void mf_big_asm_front2(const MfFront& f, unsigned char* lds_raw, const MfFront* fr,
                                                  const int32_t* chl, const int32_t* cmap, const int32_t* pinv,
                                                  const int32_t* perm, const S* bin, const S* u, S* z) {
    const int tid = threadIdx.x, ns = f.ns, ms = f.ms;
    S* r = reinterpret_cast<S*>(lds_raw);
    for (int t = tid; t < ns; t += 256) r[t] = bin[perm[f.c0 + t]];
    for (int t = tid; t < ms; t += 256) r[ns + t] = s_zero<S>();
    __syncthreads();
    for (int k = f.ch0; k < f.ch1; ++k) {
        const MfFront c = fr[chl[k]];
        const int32_t* map = cmap + c.sof;
        const S* uc = u + c.uoff;
        for (int t = tid; t < c.ms; t += 256) {
            const int pos = map[t];
            const S v = uc[t];
            if (pos < ns) r[pos] = sub(r[pos], v);
            else r[pos] = add(r[pos], v);   // each position once per child: no race
        }
        __syncthreads();
    }
    S* zs = z + f.zoff;
    for (int t = tid; t < ns; t += 256) mf_st(zs + t, mf_clean(r[pinv[f.c0 + t]]));
    for (int t = tid; t < ms; t += 256) mf_st(zs + ns + t, mf_clean(r[ns + t]));
}

// one launch for a height's small fronts (workgroups [0, nsmall): mf_fwd_kernel) and its large fronts'
// assembly (the rest: mf_big_asm_kernel); list = the small fronts, then the large ones.  They touch
// disjoint rows of w and read only lower heights' contributions, so they need no order between them.
template <class S>
__global__ __launch_bounds__(256) void mf_fwd_asm_kernel(const MfFront* fr, const int32_t* list, int32_t nsmall,
                                                         const int32_t* chl, const S* F, const int32_t* cmap,
                                                         const int32_t* pinv, S* w, S* u, S* z, int bo) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const MfFront f = fr[list[blockIdx.x]];
    if ((int32_t)blockIdx.x < nsmall) mf_fwd_front<S>(f, lds_raw, fr, chl, F, cmap, pinv, w, u);
    else mf_big_asm_front<S>(f, lds_raw, fr, chl, cmap, pinv, w, u, z, bo);
}

template <class S>
__device__ __forceinline__ S mf_rls(S v, int j) { return mf_rl(v, j); }

// scalars per pivot block of the large fronts in Tinv: inv(L_kk), inv(U_kk) (mf_inv_kernel), then the
// premultiplied next-to-diagonal tiles inv(L_kk) L_{k,k-1}, inv(U_kk) U_{k,k+1} (mf_premul_kernel)
constexpr int kMfTinv = 16384;

// Inverted diagonal blocks of the large fronts (one workgroup per pivot block, after the
// factorization): Tinv + kMfTinv k holds inv(L_kk) (unit lower), then inv(U_kk), 64 x 64 column-major,
// the identity past a partial block's rn rows.  The solves then apply a diagonal block as a
// 64 x 64 product split over the four waves instead of a 64-step dependent chain on one wave.
template <class S>
__global__ __launch_bounds__(256) void mf_inv_kernel(const MfFront* fr, const int32_t* tab, const S* F, S* Tinv) {
    __shared__ S T[64 * 65];
    __shared__ S X[64 * 65];
    const int s = tab[2 * blockIdx.x], k = tab[2 * blockIdx.x + 1];
    const MfFront f = fr[s];
    const int tid = threadIdx.x, d = f.d;
    const int r0 = 64 * k, rn = min(64, f.ns - r0);
    const S* A = F + f.off;
    S one;
    set_re_im(one, 1.0, 0.0);
    for (int e = tid; e < 64 * 64; e += 256) {
        const int i = e & 63, j = e >> 6;
        T[i + j * 65] = (i < rn && j < rn) ? A[(r0 + i) + (int64_t)(r0 + j) * d] : (i == j ? one : s_zero<S>());
    }
    __syncthreads();
    S* out = Tinv + (int64_t)(f.flag0 + k) * kMfTinv;
    // inv(L): thread t < 64 solves column t by forward substitution (unit diagonal)
    if (tid < 64) {
        const int t = tid;
        for (int i = 0; i < 64; ++i) {
            S v = i == t ? one : s_zero<S>();
            for (int j = t; j < i; ++j) v = sub(v, mul(T[i + j * 65], X[j + t * 65]));
            X[i + t * 65] = i < t ? s_zero<S>() : v;
        }
    }
    __syncthreads();
    for (int e = tid; e < 64 * 64; e += 256) out[e] = X[(e & 63) + (e >> 6) * 65];
    __syncthreads();
    // inv(U): back substitution, column t
    if (tid < 64) {
        const int t = tid;
        for (int i = 63; i >= 0; --i) {
            S v = i == t ? one : s_zero<S>();
            for (int j = i + 1; j <= t; ++j) v = sub(v, mul(T[i + j * 65], X[j + t * 65]));
            X[i + t * 65] = i > t ? s_zero<S>() : sdiv(v, T[i + i * 65]);
        }
    }
    __syncthreads();
    for (int e = tid; e < 64 * 64; e += 256) out[4096 + e] = X[(e & 63) + (e >> 6) * 65];
}

// Inverse form of a one-workgroup front with at most 64 pivots (after the factorization;
// EIGSOL_MF_INVFORM=0: off, EIGSOL_MF_INV_D: most rows, default 256): the
// forward solve of the front becomes one product [inv(L11); L21 inv(L11)] (P r) and the backward one
// [inv(U11), -inv(U11) U12] [t; x(struct)], every load independent, instead of a dependent chain
// over the pivot columns on one wave followed by the struct rows (the diagonal blocks of the large
// fronts are inverted the same way, mf_inv_kernel).
template <class S>
__global__ __launch_bounds__(256) void mf_invform_kernel(const MfFront* fr, const int32_t* list, S* F) {
    __shared__ S T[64 * 65];
    __shared__ S X[64 * 65];
    const MfFront f = fr[list[blockIdx.x]];
    const int tid = threadIdx.x, d = f.d, ns = f.ns;
    const S* A = F + f.off;
    S* Gf = F + f.goff;
    S* Gb = Gf + (int64_t)d * ns;
    S one;
    set_re_im(one, 1.0, 0.0);
    for (int e = tid; e < 64 * 64; e += 256) {
        const int i = e & 63, j = e >> 6;
        T[i + j * 65] = (i < ns && j < ns) ? A[i + (int64_t)j * d] : (i == j ? one : s_zero<S>());
    }
    __syncthreads();
    if (tid < 64) {   // inv(L11), column t (unit lower)
        const int t = tid;
        for (int i = 0; i < 64; ++i) {
            S v = i == t ? one : s_zero<S>();
            for (int j = t; j < i; ++j) v = sub(v, mul(T[i + j * 65], X[j + t * 65]));
            X[i + t * 65] = i < t ? s_zero<S>() : v;
        }
    }
    __syncthreads();
    // rows < ns: inv(L11); rows ns .. d: W = L21 inv(L11), W(i, j) = sum_{k >= j} L21(i, k) inv(L11)(k, j)
    for (int e = tid; e < d * ns; e += 256) {
        const int i = e % d, j = e / d;
        S v;
        if (i < ns) {
            v = X[i + j * 65];
        } else {
            v = s_zero<S>();
            for (int k = j; k < ns; ++k) v = add(v, mul(A[i + (int64_t)k * d], X[k + j * 65]));
        }
        Gf[i + (int64_t)j * d] = v;
    }
    __syncthreads();
    if (tid < 64) {   // inv(U11), column t
        const int t = tid;
        for (int i = 63; i >= 0; --i) {
            S v = i == t ? one : s_zero<S>();
            for (int j = i + 1; j <= t; ++j) v = sub(v, mul(T[i + j * 65], X[j + t * 65]));
            X[i + t * 65] = i > t ? s_zero<S>() : sdiv(v, T[i + i * 65]);
        }
    }
    __syncthreads();
    // columns < ns: inv(U11); columns ns + q: -inv(U11) U12(:, q), U12(k, q) = A(k, ns + q)
    for (int e = tid; e < ns * d; e += 256) {
        const int i = e % ns, c = e / ns;
        S v;
        if (c < ns) {
            v = X[i + c * 65];
        } else {
            v = s_zero<S>();
            for (int k = i; k < ns; ++k) v = sub(v, mul(X[i + k * 65], A[k + (int64_t)c * d]));
        }
        Gb[i + (int64_t)c * ns] = v;
    }
}
template <class S>
__global__ __launch_bounds__(256) void mf_invform2_kernel(const MfFront* fr, const int32_t* list, S* F) {
    // mf_invform_kernel's forms with the same operations in the same order, restructured for latency:
    // inv(L11) (wave 0) and inv(U11) (wave 1) concurrently into one LDS array X (strictly below the
    // diagonal inv(L11), whose unit diagonal is implicit; on and above it inv(U11)), and L21 / U12 read
    // from HBM once, 64-row / 64-column tiles staged in T (free after the inversions), instead of one
    // HBM load per multiply-add.
    __shared__ S T[64 * 65];
    __shared__ S X[64 * 65];
    const MfFront f = fr[list[blockIdx.x]];
    const int tid = threadIdx.x, d = f.d, ns = f.ns, wv = tid >> 6, lane = tid & 63;
    const S* A = F + f.off;
    S* Gf = F + f.goff;
    S* Gb = Gf + (int64_t)d * ns;
    S one;
    set_re_im(one, 1.0, 0.0);
    for (int e = tid; e < 64 * 64; e += 256) {
        const int i = e & 63, j = e >> 6;
        T[i + j * 65] = (i < ns && j < ns) ? A[i + (int64_t)j * d] : (i == j ? one : s_zero<S>());
    }
    __syncthreads();
    // XL(k, j) / XU(i, k) as the old kernel's X held them
    auto xl = [&](int k, int j) { return k == j ? one : (k < j ? s_zero<S>() : X[k + j * 65]); };
    if (wv == 0) {   // inv(L11), column t (unit lower)
        const int t = lane;
        for (int i = t + 1; i < 64; ++i) {
            S v = s_zero<S>();
            for (int j = t; j < i; ++j) v = sub(v, mul(T[i + j * 65], xl(j, t)));
            X[i + t * 65] = v;
        }
    } else if (wv == 1) {   // inv(U11), column t
        const int t = lane;
        for (int i = t; i >= 0; --i) {
            S v = i == t ? one : s_zero<S>();
            for (int j = i + 1; j <= t; ++j) v = sub(v, mul(T[i + j * 65], X[j + t * 65]));
            X[i + t * 65] = sdiv(v, T[i + i * 65]);
        }
    }
    __syncthreads();
    // rows < ns of the forward form: inv(L11)
    for (int e = tid; e < ns * ns; e += 256) {
        const int i = e % ns, j = e / ns;
        Gf[i + (int64_t)j * d] = xl(i, j);
    }
    // columns < ns of the backward form: inv(U11)
    for (int e = tid; e < ns * ns; e += 256) {
        const int i = e % ns, c = e / ns;
        Gb[i + (int64_t)c * ns] = i <= c ? X[i + c * 65] : s_zero<S>();
    }
    // W = L21 inv(L11), 64 rows of L21 at a time through T
    for (int i0 = ns; i0 < d; i0 += 64) {
        const int rn = min(64, d - i0);
        __syncthreads();
        for (int e = tid; e < 64 * ns; e += 256) {
            const int i = e & 63, k = e >> 6;
            if (i < rn) T[i + k * 65] = A[(i0 + i) + (int64_t)k * d];
        }
        __syncthreads();
        for (int e = tid; e < rn * ns; e += 256) {
            const int i = e % rn, j = e / rn;
            S v = s_zero<S>();
            for (int k = j; k < ns; ++k) v = add(v, mul(T[i + k * 65], xl(k, j)));
            Gf[(i0 + i) + (int64_t)j * d] = v;
        }
    }
    // -inv(U11) U12, 64 columns of U12 at a time through T
    for (int c0 = ns; c0 < d; c0 += 64) {
        const int cn = min(64, d - c0);
        __syncthreads();
        for (int e = tid; e < ns * 64; e += 256) {
            const int k = e % ns, c = e / ns;
            if (c < cn) T[k + c * 65] = A[k + (int64_t)(c0 + c) * d];
        }
        __syncthreads();
        for (int e = tid; e < ns * cn; e += 256) {
            const int i = e % ns, c = e / ns;
            S v = s_zero<S>();
            for (int k = i; k < ns; ++k) v = sub(v, mul(X[i + k * 65], T[k + c * 65]));
            Gb[i + (int64_t)(c0 + c) * ns] = v;
        }
    }
}


// The premultiplied next-to-diagonal tiles of the large fronts' row-block solves (bo & 8), one
// workgroup per pivot block after mf_inv_kernel: Tinv + kMfTinv k + 8192 = inv(L_kk) L_{k,k-1} (k >= 1;
// rows past a partial block zero), + 12288 = inv(U_kk) U_{k,k+1} (k <= nblk - 2; columns past a partial
// next block zero), 64 x 64 column-major.  Thread = one column, 16 rows.
template <class S>
__global__ __launch_bounds__(256) void mf_premul_kernel(const MfFront* fr, const int32_t* tab, const S* F, S* Tinv) {
    __shared__ S ti[64 * 65];
    __shared__ S tl[64 * 65];
    const int s = tab[2 * blockIdx.x], k = tab[2 * blockIdx.x + 1];
    const MfFront f = fr[s];
    const int tid = threadIdx.x, d = f.d, ns = f.ns;
    const int nblk = (ns + 63) / 64;
    const int r0 = 64 * k, rn = min(64, ns - r0);
    const S* A = F + f.off;
    S* base = Tinv + (int64_t)(f.flag0 + k) * kMfTinv;
    for (int up = 0; up < 2; ++up) {
        S* out = base + 8192 + 4096 * up;
        const int c = up ? k + 1 : k - 1;
        if (c < 0 || c >= nblk) {
            for (int e = tid; e < 4096; e += 256) out[e] = s_zero<S>();
            continue;
        }
        const int c0 = 64 * c, cn = min(64, ns - c0);
        __syncthreads();
        for (int e = tid; e < 4096; e += 256) {
            const int i = e & 63, j = e >> 6;
            ti[i + j * 65] = base[4096 * up + e];
            tl[i + j * 65] = (i < rn && j < cn) ? A[(r0 + i) + (int64_t)(c0 + j) * d] : s_zero<S>();
        }
        __syncthreads();
        const int j = tid & 63, i0 = (tid >> 6) * 16;
        S o[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) o[t] = s_zero<S>();
        for (int q = 0; q < 64; ++q) {
            const S b = tl[q + j * 65];
#pragma unroll
            for (int t = 0; t < 16; ++t) o[t] = add(o[t], mul(ti[(i0 + t) + q * 65], b));
        }
#pragma unroll
        for (int t = 0; t < 16; ++t) out[(i0 + t) + j * 64] = o[t];
    }
}

// acc += tile(row, c0 .. c0 + 16) * yv over the columns below lim (tile values already loaded)
template <class S>
__device__ __forceinline__ void mf_acc16(S& acc, const S (&tv)[16], const S* yv, int c0, int lim) {
#pragma unroll
    for (int t = 0; t < 16; ++t)
        if (c0 + t < lim) acc = add(acc, mul(tv[t], yv[t]));
}

// forward, large fronts: tab = (front, row block) pairs; row block k < nblk: pivot rows
// [64 k, 64 k + 64) (applies inv(L_kk), publishes, raises the flag); k >= nblk: struct rows (their
// contribution u = children's part + L21 y).  Every wave takes 16 columns of each column block:
// its tile values are loaded before the block's flag is awaited.
template <class S>
__device__ __forceinline__ void mf_big_fwd_block(const int bid, const MfFront* fr, const int32_t* tab, const S* F,
                                                 const S* Tinv, S* z, S* w, S* u, int32_t* flag, int32_t epoch,
                                                 int32_t* err, int bo, S* x, const bool zpoll) {
    __shared__ S part[4][64];
    __shared__ S ysh[4][16];
    __shared__ S vsh[64];
    const int s = tab[2 * bid], rb = tab[2 * bid + 1];
    const MfFront f = fr[s];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int d = f.d, ns = f.ns;
    const int nblk = (ns + 63) / 64;
    const bool piv = rb < nblk;
    const int r0 = piv ? 64 * rb : ns + 64 * (rb - nblk);
    const int rn = min(64, (piv ? ns : d) - r0);
    const S* A = F + f.off;
    const int row = r0 + min(lane, rn - 1);
    S iv[16];
    if (piv) {
        const S* ti = Tinv + (int64_t)(f.flag0 + rb) * kMfTinv + lane + (16 * wv) * 64;
#pragma unroll
        for (int t = 0; t < 16; ++t) iv[t] = ti[t * 64];
    }
    S acc = s_zero<S>();
    // the assembled right-hand side of these rows, loaded before the chain of waits (it was a
    // dependent round trip after the last one, on every hand-off's critical path)
    // zpoll (mf_fwd_height_kernel): z is assembled in this launch and value-flagged; wave 0 polls it after
    // the chain and hands the slot back to the sentinel (this workgroup is its only reader)
    S zr = (!zpoll && lane < rn) ? z[f.zoff + r0 + lane] : s_zero<S>();
    // bo & 8 (value flags only): block rb - 1 enters last, as a product with the premultiplied tile
    // inv(L_rr) L_{r,r-1} after y' = inv(L_rr) (z - the other blocks), so a hand-off is followed by one
    // 64 x 64 product instead of two
    const bool premul = (bo & 12) == 12 && piv && rb >= 1;
    const int cend = piv ? (premul ? rb - 1 : rb) : nblk;
    for (int c = 0; c < cend; ++c) {
        const int c0 = 64 * c + 16 * wv;
        S tv[16];
        const S* tile = A + row;
#pragma unroll
        for (int t = 0; t < 16; ++t) tv[t] = tile[(int64_t)min(c0 + t, ns - 1) * d];
        if (bo & 4) {
            if (lane < 16) ysh[wv][lane] = c0 + lane < ns ? mf_poll(w + f.c0 + c0 + lane, err, bo) : s_zero<S>();
        } else {
            if (lane == 0) mf_wait(flag + f.flag0 + c, epoch, err, bo);
            __builtin_amdgcn_wave_barrier();
            if (!(bo & 2)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            if (lane < 16) ysh[wv][lane] = c0 + lane < ns ? mf_ld(w + f.c0 + c0 + lane) : s_zero<S>();
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        mf_acc16(acc, tv, ysh[wv], c0, ns);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    S tm[16];
    S yl = s_zero<S>();
    const int lc0 = 64 * (rb - 1) + 16 * wv;
    if (premul) {
        if (lane < 16) yl = mf_ld(w + f.c0 + lc0 + lane);   // first poll, under the reductions
        const S* tp = Tinv + (int64_t)(f.flag0 + rb) * kMfTinv + 8192 + lane + (16 * wv) * 64;
#pragma unroll
        for (int t = 0; t < 16; ++t) tm[t] = tp[t * 64];
    }
    if (zpoll && wv == 0 && lane < rn) {
        zr = mf_poll(z + f.zoff + r0 + lane, err, bo);
        mf_st(z + f.zoff + r0 + lane, mf_sent(s_zero<S>()));
    }
    part[wv][lane] = acc;
    __syncthreads();
    const S sum = add(add(part[0][lane], part[1][lane]), add(part[2][lane], part[3][lane]));
    if (!piv) {
        if (wv == 0 && lane < rn) u[f.uoff + (r0 - ns) + lane] = add(zr, sum);
        return;
    }
    if (wv == 0) vsh[lane] = lane < rn ? sub(zr, sum) : s_zero<S>();
    __syncthreads();
    S p = s_zero<S>();
#pragma unroll
    for (int t = 0; t < 16; ++t) p = add(p, mul(iv[t], vsh[16 * wv + t]));
    part[wv][lane] = p;
    __syncthreads();
    S y = s_zero<S>();
    if (wv == 0) y = add(add(part[0][lane], part[1][lane]), add(part[2][lane], part[3][lane]));
    if (premul) {
        __shared__ S part2[4][64];
        if (lane < 16) {
            if (mf_unready(yl)) yl = mf_poll(w + f.c0 + lc0 + lane, err, bo);
            ysh[wv][lane] = yl;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        S q = s_zero<S>();
#pragma unroll
        for (int t = 0; t < 16; ++t) q = add(q, mul(tm[t], ysh[wv][t]));
        part2[wv][lane] = q;
        __syncthreads();
        if (wv == 0) y = sub(y, add(add(part2[0][lane], part2[1][lane]), add(part2[2][lane], part2[3][lane])));
    }
    if (wv != 0) return;
    if (bo & 4) {
        // publish (the value is its own flag); x of these rows becomes "unsolved" for the backward pass
        if (lane < rn) {
            mf_st(w + f.c0 + r0 + lane, mf_clean(y));
            mf_st(x + f.c0 + r0 + lane, mf_sent(y));
        }
        return;
    }
    if (lane < rn) mf_st(w + f.c0 + r0 + lane, y);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(flag + f.flag0 + rb, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

template <class S>
__global__ __launch_bounds__(256) void mf_big_fwd_kernel(const MfFront* fr, const int32_t* tab, const S* F,
                                                         const S* Tinv, S* z, S* w, S* u, int32_t* flag,
                                                         int32_t epoch, int32_t* err, int bo, S* x) {
    mf_big_fwd_block<S>((int)blockIdx.x, fr, tab, F, Tinv, z, w, u, flag, epoch, err, bo, x, false);
}

// One forward launch per height with large fronts (value flags): workgroups [0, nsmall) the small fronts,
// [nsmall, nsmall + nbig) the large fronts' assembly (mf_big_asm_front2: z written once per entry,
// value-flagged), the rest the large fronts' row blocks (mf_big_fwd_block, polling z after their chain).
// Every workgroup waits only on lower-indexed ones; the large fronts' pivot rows of w were set to the
// sentinel by mf_gather_kernel.
template <class S>
__global__ __launch_bounds__(256) void mf_fwd_height_kernel(const MfFront* fr, const int32_t* list, int32_t nsmall,
                                                            int32_t nbig, const int32_t* tab, const int32_t* chl,
                                                            const S* F, const S* Tinv, const int32_t* cmap,
                                                            const int32_t* pinv, const int32_t* perm, const S* bin,
                                                            S* w, S* u, S* z, int32_t* err, int bo, S* x) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const int32_t b = (int32_t)blockIdx.x;
    if (b < nsmall) mf_fwd_front<S>(fr[list[b]], lds_raw, fr, chl, F, cmap, pinv, w, u);
    else if (b < nsmall + nbig) mf_big_asm_front2<S>(fr[list[b]], lds_raw, fr, chl, cmap, pinv, perm, bin, u, z);
    else mf_big_fwd_block<S>((int)(b - nsmall - nbig), fr, tab, F, Tinv, z, w, u, nullptr, 0, err, bo, x, true);
}

// backward, large fronts: tab = (front, pivot block) pairs, blocks descending within a front:
// t = y - U12 x(struct) - U[rows, later blocks] x, then inv(U_kk) t (publish, flag)
template <class S>
__device__ __forceinline__ void mf_big_bwd_block(const int bid, const MfFront* fr, const int32_t* tab, const S* F,
                                                 const S* Tinv, const int32_t* sidx, const S* w, S* x,
                                                 int32_t* flag, int32_t epoch, int32_t* err, int bo) {
    __shared__ S part[4][64];
    __shared__ S ysh[4][16];
    __shared__ S vsh[64];
    extern __shared__ __align__(16) unsigned char xs_raw[];
    S* xsh = reinterpret_cast<S*>(xs_raw);   // x(struct), ms entries
    const int s = tab[2 * bid], rb = tab[2 * bid + 1];
    const MfFront f = fr[s];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int d = f.d, ns = f.ns, ms = f.ms;
    const int nblk = (ns + 63) / 64;
    const int r0 = 64 * rb, rn = min(64, ns - r0);
    const S* A = F + f.off;
    const int row = r0 + min(lane, rn - 1);
    S iv[16];
    {
        const S* ti = Tinv + (int64_t)(f.flag0 + rb) * kMfTinv + 4096 + lane + (16 * wv) * 64;
#pragma unroll
        for (int t = 0; t < 16; ++t) iv[t] = ti[t * 64];
    }
    S acc = s_zero<S>();
    const S wr = lane < rn ? w[f.c0 + r0 + lane] : s_zero<S>();   // loaded before the waits (see forward)
    // U12 x(struct): x(struct) (the ancestors' x: earlier launches) gathered into LDS once, then
    // 16-column chunks, wave wv every 4th, two chunks' tiles in flight (the gather and the tile
    // loads used to chain one round trip per chunk: ms = 1000 took ~50 us of a 68 us launch)
    for (int q = tid; q < ms; q += 256) xsh[q] = x[sidx[f.sof + q]];
    __syncthreads();
    {
        const S* tile = A + row + (int64_t)ns * d;
        int q0 = 16 * wv;
        for (; q0 + 64 < ms; q0 += 128) {
            S ta[16], tb[16];
#pragma unroll
            for (int t = 0; t < 16; ++t) ta[t] = tile[(int64_t)(q0 + t) * d];
#pragma unroll
            for (int t = 0; t < 16; ++t) tb[t] = tile[(int64_t)min(q0 + 64 + t, ms - 1) * d];
            mf_acc16(acc, ta, xsh + q0, q0, ms);
            mf_acc16(acc, tb, xsh + q0 + 64, q0 + 64, ms);
        }
        if (q0 < ms) {
            S ta[16];
#pragma unroll
            for (int t = 0; t < 16; ++t) ta[t] = tile[(int64_t)min(q0 + t, ms - 1) * d];
            mf_acc16(acc, ta, xsh + q0, q0, ms);
        }
    }
    // later pivot blocks of this front as their flags rise (the last block first); bo & 8: block rb + 1
    // last, as a product with the premultiplied inv(U_rr) U_{r,r+1} (see the forward block)
    const bool premul = (bo & 12) == 12 && rb + 1 < nblk;
    for (int c = nblk - 1; c > (premul ? rb + 1 : rb); --c) {
        const int c0 = 64 * c + 16 * wv;
        S tv[16];
        const S* tile = A + row;
#pragma unroll
        for (int t = 0; t < 16; ++t) tv[t] = tile[(int64_t)min(c0 + t, ns - 1) * d];
        if (bo & 4) {
            if (lane < 16) ysh[wv][lane] = c0 + lane < ns ? mf_poll(x + f.c0 + c0 + lane, err, bo) : s_zero<S>();
        } else {
            if (lane == 0) mf_wait(flag + f.flag0 + c, epoch, err, bo);
            __builtin_amdgcn_wave_barrier();
            if (!(bo & 2)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            if (lane < 16) ysh[wv][lane] = c0 + lane < ns ? mf_ld(x + f.c0 + c0 + lane) : s_zero<S>();
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        mf_acc16(acc, tv, ysh[wv], c0, ns);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    S tm[16];
    S xl = s_zero<S>();
    const int lc0 = 64 * (rb + 1) + 16 * wv;
    if (premul) {
        if (lane < 16 && lc0 + lane < ns) xl = mf_ld(x + f.c0 + lc0 + lane);
        const S* tp = Tinv + (int64_t)(f.flag0 + rb) * kMfTinv + 12288 + lane + (16 * wv) * 64;
#pragma unroll
        for (int t = 0; t < 16; ++t) tm[t] = tp[t * 64];
    }
    part[wv][lane] = acc;
    __syncthreads();
    if (wv == 0) {
        const S sum = add(add(part[0][lane], part[1][lane]), add(part[2][lane], part[3][lane]));
        vsh[lane] = lane < rn ? sub(wr, sum) : s_zero<S>();
    }
    __syncthreads();
    S p = s_zero<S>();
#pragma unroll
    for (int t = 0; t < 16; ++t) p = add(p, mul(iv[t], vsh[16 * wv + t]));
    part[wv][lane] = p;
    __syncthreads();
    S xv = s_zero<S>();
    if (wv == 0) xv = add(add(part[0][lane], part[1][lane]), add(part[2][lane], part[3][lane]));
    if (premul) {
        __shared__ S part2[4][64];
        if (lane < 16) {
            if (lc0 + lane < ns) {
                if (mf_unready(xl)) xl = mf_poll(x + f.c0 + lc0 + lane, err, bo);
            } else {
                xl = s_zero<S>();
            }
            ysh[wv][lane] = xl;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        S q = s_zero<S>();
#pragma unroll
        for (int t = 0; t < 16; ++t) q = add(q, mul(tm[t], ysh[wv][t]));
        part2[wv][lane] = q;
        __syncthreads();
        if (wv == 0) xv = sub(xv, add(add(part2[0][lane], part2[1][lane]), add(part2[2][lane], part2[3][lane])));
    }
    if (wv != 0) return;
    if (bo & 4) {
        if (lane < rn) mf_st(x + f.c0 + r0 + lane, mf_clean(xv));
        return;
    }
    if (lane < rn) mf_st(x + f.c0 + r0 + lane, xv);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(flag + f.flag0 + rb, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

template <class S>
__global__ __launch_bounds__(256) void mf_big_bwd_kernel(const MfFront* fr, const int32_t* tab, const S* F,
                                                         const S* Tinv, const int32_t* sidx, const S* w, S* x,
                                                         int32_t* flag, int32_t epoch, int32_t* err, int bo) {
    mf_big_bwd_block<S>((int)blockIdx.x, fr, tab, F, Tinv, sidx, w, x, flag, epoch, err, bo);
}

// one launch for a height's large-front row blocks (workgroups [0, nbb), waiting on each other's values;
// dispatched first) and its small fronts (the rest, mf_bwd_kernel's; they read only their ancestors' x)
template <class S>
__global__ __launch_bounds__(256) void mf_bwd_big_small_kernel(const MfFront* fr, const int32_t* tab, int32_t nbb,
                                                               const int32_t* list, const S* F, const S* Tinv,
                                                               const int32_t* sidx, const S* w, S* x,
                                                               int32_t* flag, int32_t epoch, int32_t* err, int bo) {
    if ((int32_t)blockIdx.x < nbb) {
        mf_big_bwd_block<S>((int)blockIdx.x, fr, tab, F, Tinv, sidx, w, x, flag, epoch, err, bo);
    } else {
        extern __shared__ __align__(16) unsigned char lds_raw[];
        mf_bwd_front<S>(fr[list[blockIdx.x - nbb]], lds_raw, F, sidx, w, x);
    }
}

// ---- large fronts, two pivot blocks per workgroup (EIGSOL_MF_PAIR=1, value flags only; off by
// default: measured slower, see MfFactor::pair).  A chain of
// 64-row blocks pays one cross-CU hand-off per block (the producer's write-through store, the
// consumer's poll: ~2-3 us with the chip busy).  Here a workgroup owns pivot blocks 2u and 2u + 1:
// it awaits the dependencies the two share once, solves block 2u, and hands its values to block
// 2u + 1 in LDS, so a front's chain crosses CUs once per pair.  Every row's sum keeps
// mf_big_fwd_kernel's / mf_big_bwd_kernel's order (the column blocks in the same sequence, the
// handed-over block last), so the solution is bitwise the same.
// Reduction of the four waves' partial row sums, then the inverted diagonal block: returns the
// block's solution in wave 0 (lane = row); part / vsh are the caller's LDS, synchronised here.
template <class S>
__device__ __forceinline__ S mf_pair_finish(S acc, S rhs, int rn, const S (&iv)[16], S (&part)[4][64], S* vsh) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    part[wv][lane] = acc;
    __syncthreads();
    if (wv == 0) {
        const S sum = add(add(part[0][lane], part[1][lane]), add(part[2][lane], part[3][lane]));
        vsh[lane] = lane < rn ? sub(rhs, sum) : s_zero<S>();
    }
    __syncthreads();
    S p = s_zero<S>();
#pragma unroll
    for (int t = 0; t < 16; ++t) p = add(p, mul(iv[t], vsh[16 * wv + t]));
    part[wv][lane] = p;
    __syncthreads();
    return add(add(part[0][lane], part[1][lane]), add(part[2][lane], part[3][lane]));
}

// forward: tab = (front, unit); unit < npair = ceil(nblk / 2) covers pivot blocks 2 unit and
// 2 unit + 1, the others are struct row blocks (nblk + unit - npair, as mf_big_fwd_kernel)
template <class S>
__global__ __launch_bounds__(256) void mf_big_fwd2_kernel(const MfFront* fr, const int32_t* tab, const S* F,
                                                          const S* Tinv, const S* z, S* w, S* u, int32_t* err, int bo,
                                                          S* x) {
    __shared__ S part[4][64];
    __shared__ S ysh[4][16];
    __shared__ S vsh[64];
    __shared__ S ya[64];
    const int s = tab[2 * blockIdx.x], un = tab[2 * blockIdx.x + 1];
    const MfFront f = fr[s];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int d = f.d, ns = f.ns;
    const int nblk = (ns + 63) / 64, npair = (nblk + 1) / 2;
    const bool piv = un < npair;
    const int ba = piv ? 2 * un : nblk + (un - npair);   // the (first) row block
    const bool hasb = piv && ba + 1 < nblk;
    const int ra0 = piv ? 64 * ba : ns + 64 * (ba - nblk);
    const int rna = min(64, (piv ? ns : d) - ra0);
    const int rnb = hasb ? min(64, ns - (ra0 + 64)) : 0;
    const S* A = F + f.off;
    const int rowa = ra0 + min(lane, rna - 1);
    const int rowb = hasb ? ra0 + 64 + min(lane, rnb - 1) : rowa;
    S iva[16], ivb[16];
    if (piv) {
        const S* ti = Tinv + (int64_t)(f.flag0 + ba) * kMfTinv + lane + (16 * wv) * 64;
#pragma unroll
        for (int t = 0; t < 16; ++t) iva[t] = ti[t * 64];
    }
    if (hasb) {
        const S* ti = Tinv + (int64_t)(f.flag0 + ba + 1) * kMfTinv + lane + (16 * wv) * 64;
#pragma unroll
        for (int t = 0; t < 16; ++t) ivb[t] = ti[t * 64];
    }
    const S zra = lane < rna ? z[f.zoff + ra0 + lane] : s_zero<S>();
    const S zrb = (hasb && lane < rnb) ? z[f.zoff + ra0 + 64 + lane] : s_zero<S>();
    // block 2u + 1's tile over block 2u's columns: loaded before the chain of waits
    S th[16];
    if (hasb) {
        const int c0 = 64 * ba + 16 * wv;
#pragma unroll
        for (int t = 0; t < 16; ++t) th[t] = A[rowb + (int64_t)min(c0 + t, ns - 1) * d];
    }
    S acca = s_zero<S>(), accb = s_zero<S>();
    const int cend = piv ? ba : nblk;
    for (int c = 0; c < cend; ++c) {
        const int c0 = 64 * c + 16 * wv;
        S tva[16], tvb[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) tva[t] = A[rowa + (int64_t)min(c0 + t, ns - 1) * d];
        if (hasb) {
#pragma unroll
            for (int t = 0; t < 16; ++t) tvb[t] = A[rowb + (int64_t)min(c0 + t, ns - 1) * d];
        }
        if (lane < 16) ysh[wv][lane] = c0 + lane < ns ? mf_poll(w + f.c0 + c0 + lane, err, bo) : s_zero<S>();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        mf_acc16(acca, tva, ysh[wv], c0, ns);
        if (hasb) mf_acc16(accb, tvb, ysh[wv], c0, ns);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    if (!piv) {
        part[wv][lane] = acca;
        __syncthreads();
        const S sum = add(add(part[0][lane], part[1][lane]), add(part[2][lane], part[3][lane]));
        if (wv == 0 && lane < rna) u[f.uoff + (ra0 - ns) + lane] = add(zra, sum);
        return;
    }
    const S y = mf_pair_finish(acca, zra, rna, iva, part, vsh);
    if (wv == 0) {
        // publish (the value is its own flag); x of these rows becomes "unsolved" for the backward pass
        const S yc = mf_clean(y);
        if (lane < rna) {
            mf_st(w + f.c0 + ra0 + lane, yc);
            mf_st(x + f.c0 + ra0 + lane, mf_sent(y));
        }
        ya[lane] = yc;   // what block 2u + 1 would have polled
    }
    if (!hasb) return;
    __syncthreads();
    mf_acc16(accb, th, ya + 16 * wv, 64 * ba + 16 * wv, ns);
    const S yb = mf_pair_finish(accb, zrb, rnb, ivb, part, vsh);
    if (wv == 0 && lane < rnb) {
        mf_st(w + f.c0 + ra0 + 64 + lane, mf_clean(yb));
        mf_st(x + f.c0 + ra0 + 64 + lane, mf_sent(yb));
    }
}

// backward: tab = (front, unit), units descending; unit u covers pivot blocks 2u + 1 (when it
// exists, solved first) and 2u
template <class S>
__global__ __launch_bounds__(256) void mf_big_bwd2_kernel(const MfFront* fr, const int32_t* tab, const S* F,
                                                          const S* Tinv, const int32_t* sidx, const S* w, S* x,
                                                          int32_t* err, int bo) {
    __shared__ S part[4][64];
    __shared__ S ysh[4][16];
    __shared__ S vsh[64];
    __shared__ S xa[64];
    extern __shared__ __align__(16) unsigned char xs_raw[];
    S* xsh = reinterpret_cast<S*>(xs_raw);   // x(struct), ms entries
    const int s = tab[2 * blockIdx.x], un = tab[2 * blockIdx.x + 1];
    const MfFront f = fr[s];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int d = f.d, ns = f.ns, ms = f.ms;
    const int nblk = (ns + 63) / 64;
    const int bl = 2 * un;                   // the lower block (always present)
    const bool hash = bl + 1 < nblk;         // the higher block, solved first
    const int rl0 = 64 * bl, rnl = min(64, ns - rl0);
    const int rh0 = rl0 + 64, rnh = hash ? min(64, ns - rh0) : 0;
    const S* A = F + f.off;
    const int rowl = rl0 + min(lane, rnl - 1);
    const int rowh = hash ? rh0 + min(lane, rnh - 1) : rowl;
    S ivl[16], ivh[16];
    {
        const S* ti = Tinv + (int64_t)(f.flag0 + bl) * kMfTinv + 4096 + lane + (16 * wv) * 64;
#pragma unroll
        for (int t = 0; t < 16; ++t) ivl[t] = ti[t * 64];
    }
    if (hash) {
        const S* ti = Tinv + (int64_t)(f.flag0 + bl + 1) * kMfTinv + 4096 + lane + (16 * wv) * 64;
#pragma unroll
        for (int t = 0; t < 16; ++t) ivh[t] = ti[t * 64];
    }
    const S wl = lane < rnl ? w[f.c0 + rl0 + lane] : s_zero<S>();
    const S wh = (hash && lane < rnh) ? w[f.c0 + rh0 + lane] : s_zero<S>();
    // the lower block's tile over the higher block's columns (used after the higher block is solved)
    S tl[16];
    if (hash) {
        const int c0 = rh0 + 16 * wv;
#pragma unroll
        for (int t = 0; t < 16; ++t) tl[t] = A[rowl + (int64_t)min(c0 + t, ns - 1) * d];
    }
    S accl = s_zero<S>(), acch = s_zero<S>();
    // U12 x(struct) for both blocks' rows (x(struct) gathered into LDS once)
    for (int q = tid; q < ms; q += 256) xsh[q] = x[sidx[f.sof + q]];
    __syncthreads();
    {
        const S* tile_l = A + rowl + (int64_t)ns * d;
        const S* tile_h = A + rowh + (int64_t)ns * d;
        int q0 = 16 * wv;
        for (; q0 + 64 < ms; q0 += 128) {
            S ta[16], tb[16];
#pragma unroll
            for (int t = 0; t < 16; ++t) ta[t] = tile_l[(int64_t)(q0 + t) * d];
#pragma unroll
            for (int t = 0; t < 16; ++t) tb[t] = tile_l[(int64_t)min(q0 + 64 + t, ms - 1) * d];
            mf_acc16(accl, ta, xsh + q0, q0, ms);
            mf_acc16(accl, tb, xsh + q0 + 64, q0 + 64, ms);
            if (hash) {
#pragma unroll
                for (int t = 0; t < 16; ++t) ta[t] = tile_h[(int64_t)(q0 + t) * d];
#pragma unroll
                for (int t = 0; t < 16; ++t) tb[t] = tile_h[(int64_t)min(q0 + 64 + t, ms - 1) * d];
                mf_acc16(acch, ta, xsh + q0, q0, ms);
                mf_acc16(acch, tb, xsh + q0 + 64, q0 + 64, ms);
            }
        }
        if (q0 < ms) {
            S ta[16];
#pragma unroll
            for (int t = 0; t < 16; ++t) ta[t] = tile_l[(int64_t)min(q0 + t, ms - 1) * d];
            mf_acc16(accl, ta, xsh + q0, q0, ms);
            if (hash) {
#pragma unroll
                for (int t = 0; t < 16; ++t) ta[t] = tile_h[(int64_t)min(q0 + t, ms - 1) * d];
                mf_acc16(acch, ta, xsh + q0, q0, ms);
            }
        }
    }
    // later pivot blocks (the last first) as their values arrive
    const int clow = hash ? bl + 1 : bl;
    for (int c = nblk - 1; c > clow; --c) {
        const int c0 = 64 * c + 16 * wv;
        S tvl[16], tvh[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) tvl[t] = A[rowl + (int64_t)min(c0 + t, ns - 1) * d];
        if (hash) {
#pragma unroll
            for (int t = 0; t < 16; ++t) tvh[t] = A[rowh + (int64_t)min(c0 + t, ns - 1) * d];
        }
        if (lane < 16) ysh[wv][lane] = c0 + lane < ns ? mf_poll(x + f.c0 + c0 + lane, err, bo) : s_zero<S>();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        mf_acc16(accl, tvl, ysh[wv], c0, ns);
        if (hash) mf_acc16(acch, tvh, ysh[wv], c0, ns);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    if (hash) {
        const S xh = mf_pair_finish(acch, wh, rnh, ivh, part, vsh);
        if (wv == 0) {
            const S xc = mf_clean(xh);
            if (lane < rnh) mf_st(x + f.c0 + rh0 + lane, xc);
            xa[lane] = xc;
        }
        __syncthreads();
        mf_acc16(accl, tl, xa + 16 * wv, rh0 + 16 * wv, ns);
    }
    const S xl = mf_pair_finish(accl, wl, rnl, ivl, part, vsh);
    if (wv == 0 && lane < rnl) mf_st(x + f.c0 + rl0 + lane, mf_clean(xl));
}

}  // namespace dev

// ================================================================== host side
struct MfFactor {
    eigsol_ctx* ctx = nullptr;
    int dtype = EIGSOL_F64;
    int64_t n = 0;
    int nb = 32;
    int64_t nfront = 0;
    dev::MfFront* fronts = nullptr;
    int32_t* chl = nullptr;
    int32_t* sidx = nullptr;
    int32_t* cmap = nullptr;
    int32_t* perm = nullptr;   // new -> old
    int32_t* pinv = nullptr;   // composite pivot permutation, per front local
    int32_t* lists = nullptr;  // fronts by height, each height's list by descending ns
    void* F = nullptr;
    void* u = nullptr;
    void* w = nullptr;
    void* x = nullptr;
    std::vector<int64_t> hstart;      // lists[hstart[h] .. hstart[h + 1])
    std::vector<int32_t> lds_fwd, lds_bwd;   // dynamic LDS bytes per height (one-workgroup fronts)
    std::vector<int32_t> lds_bbig;           // per height: x(struct) of the large fronts (mf_big_bwd_kernel)
    // solve: per height the one-workgroup fronts (slists[sstart[h] .. + nsmall[h])), then the
    // large fronts (the next nbig[h] entries: their assembly launch); the large fronts' row-block
    // tables (front, block) for the forward / backward launches at tabf / tabb + off[h], cnt[h] pairs
    int32_t* slists = nullptr;
    int32_t* tabf = nullptr;
    int32_t* tabb = nullptr;
    int32_t* tabf2 = nullptr;         // the same with two pivot blocks per entry (mf_big_fwd2 / bwd2_kernel)
    int32_t* tabb2 = nullptr;
    // EIGSOL_MF_PAIR=1 (value flags only; measured and left off, round 6, tools/r06_mf_pair_ab.sh):
    // 1M convection-diffusion 1.495 / 1.509 -> 1.776 / 1.793 ms per iteration, bitwise the same
    // solution - a workgroup holding two blocks' tiles (256 VGPRs + AGPRs, one wave per SIMD) loads
    // them at half the rate, and that, not the hand-off count, is what the chain waits on
    bool pair = false;
    int32_t* flags = nullptr;         // one per pivot block of the large fronts (epoch words)
    int32_t* err = nullptr;           // a flag wait that timed out
    void* z = nullptr;                // large fronts' assembled right-hand sides
    void* tinv = nullptr;             // inverted diagonal blocks of the large fronts and premultiplied tiles (kMfTinv scalars each)
    int32_t epoch = 0;
    int32_t hflow = 0;
    int32_t* flow_f = nullptr;
    int32_t* flow_b = nullptr;
    int32_t* fheight = nullptr;
    int32_t* done = nullptr;
    int32_t nflow = 0, lds_flow_f = 0, lds_flow_b = 0;
    int flow_mode = 3;
    int32_t* sub_ranges = nullptr;
    int32_t nsub = 0, lds_sub_f = 0, lds_sub_b = 0;                // bit 0 forward, bit 1 backward (EIGSOL_MF_FLOW_MODE, debugging)
    int backoff = 2;                  // EIGSOL_MF_BACKOFF: 1 growing sleeps, 2 relaxed polls (flag stores: release)
    bool fuse_asm = true;             // EIGSOL_MF_FUSE_ASM=0: small fronts and large-front assembly as two launches
    bool fuse_big = true;             // EIGSOL_MF_FUSE_BIG=0: no mf_fwd_height_kernel
    uint8_t* bigm = nullptr;          // [n] 1 on the large fronts' pivot rows (mf_fwd_height_kernel's gather)
    std::vector<int64_t> sstart, nwave, nsmall, nbig, foff, fcnt, boff, bcnt, foff2, fcnt2, boff2, bcnt2;
    std::vector<int32_t> lds_asm;
    std::vector<int32_t> lds_asm2;    // mf_fwd_height_kernel's assembly: d entries per large front
    MfStats st;
    // solves replayed as a hipGraph per (b, out) pair seen twice (value flags, no flow kernels:
    // the launches' arguments are then the same for every solve of that pair)
    struct Graph {
        const void* b;
        void* out;
        int uses;
        hipGraphExec_t exec;
    };
    std::vector<Graph> graphs;
    int64_t nstatic = 0;   // static pivots of the factorization (0 unless the retry set them)
};

void mf_free(MfFactor* f) {
    if (!f) return;
    hipSetDevice(f->ctx->device);
    hipStreamSynchronize(f->ctx->stream);
    for (void* p : {(void*)f->fronts, (void*)f->chl, (void*)f->sidx, (void*)f->cmap, (void*)f->perm, (void*)f->pinv,
                    (void*)f->lists, f->F, f->u, f->w, f->x, (void*)f->slists, (void*)f->tabf, (void*)f->tabb,
                    (void*)f->tabf2, (void*)f->tabb2, (void*)f->flags, (void*)f->err, f->z, f->tinv, (void*)f->flow_f, (void*)f->flow_b,
                    (void*)f->fheight, (void*)f->done, (void*)f->sub_ranges, (void*)f->bigm})
        if (p) hipFree(p);
    for (auto& g : f->graphs)
        if (g.exec) hipGraphExecDestroy(g.exec);
    ctx_release(f->ctx);
    delete f;
}

const MfStats& mf_stats(const MfFactor* f) { return f->st; }

namespace {

struct SymGraph {
    std::vector<int64_t> ptr;
    std::vector<int32_t> adj;
};

// pattern of M + M^T without the diagonal, each list sorted and unique
// fn(begin, end) over [0, n) in contiguous chunks on up to nth host threads
template <class Fn>
void par_for(int64_t n, int nth, Fn fn) {
    if (nth <= 1 || n < 4096) { fn((int64_t)0, n); return; }
    std::vector<std::thread> th;
    const int64_t chunk = (n + nth - 1) / nth;
    try {
        for (int t = 1; t < nth; ++t) {
            const int64_t b = t * chunk, e = std::min(n, b + chunk);
            if (b < e) th.emplace_back(fn, b, e);
        }
    } catch (const std::exception&) {
        for (auto& x : th) x.join();
        fn(chunk, n);   // no more threads: the rest on this one
        fn((int64_t)0, std::min(n, chunk));
        return;
    }
    fn((int64_t)0, std::min(n, chunk));
    for (auto& x : th) x.join();
}

int host_threads() {
    int nth = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (const char* e = std::getenv("EIGSOL_MF_THREADS")) nth = std::max(1, std::atoi(e));
    return nth;
}

// pattern of M + M^T without the diagonal, each list sorted and unique: M's rows merged with the
// rows of its transpose (a counting-sort transpose keeps them sorted)
bool sym_graph(int64_t n, const std::vector<int32_t>& rp, const std::vector<int32_t>& ci, SymGraph& g,
               const std::atomic<bool>* stop = nullptr) {
    const int nth = host_threads();
    auto stopped = [&]() { return stop && stop->load(std::memory_order_relaxed); };
    std::vector<int64_t> tp(n + 1, 0);
    for (int64_t e = 0; e < (int64_t)rp[n]; ++e) ++tp[ci[e] + 1];
    for (int64_t i = 0; i < n; ++i) tp[i + 1] += tp[i];
    if (stopped()) return false;
    std::vector<int32_t> tc(rp[n]);
    {
        std::vector<int64_t> fill(tp.begin(), tp.end() - 1);
        for (int64_t i = 0; i < n; ++i) {
            if ((i & 65535) == 0 && stopped()) return false;
            for (int32_t e = rp[i]; e < rp[i + 1]; ++e) tc[fill[ci[e]]++] = (int32_t)i;
        }
    }
    // merge row i of M and of M^T (both ascending), without i and repeats; count, then fill
    auto merge = [&](int64_t i, int32_t* out) -> int64_t {
        int64_t a = rp[i], ae = rp[i + 1], b = tp[i], be = tp[i + 1], k = 0;
        int32_t last = -1;
        while (a < ae || b < be) {
            int32_t c;
            if (b >= be || (a < ae && ci[a] <= tc[b])) c = ci[a++];
            else c = tc[b++];
            if (c == i || c == last) continue;
            last = c;
            if (out) out[k] = c;
            ++k;
        }
        return k;
    };
    g.ptr.assign(n + 1, 0);
    par_for(n, nth, [&](int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) {
            if ((i & 65535) == 0 && stopped()) return;
            g.ptr[i + 1] = merge(i, nullptr);
        }
    });
    if (stopped()) return false;
    for (int64_t i = 0; i < n; ++i) g.ptr[i + 1] += g.ptr[i];
    if (stopped()) return false;
    g.adj.resize(g.ptr[n]);
    par_for(n, nth, [&](int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) {
            if ((i & 65535) == 0 && stopped()) return;
            merge(i, g.adj.data() + g.ptr[i]);
        }
    });
    return !stopped();
}

struct NdNode {
    std::vector<int32_t> members;
    int32_t parent;
    std::vector<int32_t> key;   // position in the dissection (independent of thread timing)
};

// Nested dissection of the vertices of g: tree nodes (leaves and separators) with parents, in a
// canonical order (sorted by key: the path of choices from the whole graph to the node's piece).
// Pieces are dissected by a pool of host threads (they touch disjoint vertex sets; a piece's BFS
// reads its neighbours' set tags with relaxed atomics); the tree does not depend on the timing.
bool nested_dissection(int64_t n, const SymGraph& g, int leaf, std::vector<NdNode>& tree,
                       const std::atomic<bool>* stop) {
    struct Task {
        std::vector<int32_t> nodes;
        int32_t parent;
        std::vector<int32_t> key;
    };
    std::vector<Task> stack;
    {
        Task t;
        t.nodes.resize(n);
        std::iota(t.nodes.begin(), t.nodes.end(), 0);
        t.parent = -1;
        stack.push_back(std::move(t));
    }
    // per-vertex state in one record, so a neighbour test touches one cache line: the piece tag
    // (written by the piece's owner, read by the neighbouring pieces' BFS), the BFS stamp and level
    struct Vs {
        int64_t tag, seen;
        int32_t level;
    };
    std::vector<Vs> vs(n, Vs{-1, -1, 0});
    // pseudo-peripheral restarts per piece (EIGSOL_MF_PP_ROUNDS).  1M convection-diffusion: 2 / 1 / 0
    // rounds -> 1.374e8 / 1.368e8 / 1.47e8 factor entries, 1.13e11 / 1.12e11 / 1.83e11 flops; on the box
    // the set-up is the same for 1 and 2 (0.63-0.67 s) and the solve 1.55 against 1.57 ms: 2 stays
    static const int pp_rounds = [] {
        const char* e = std::getenv("EIGSOL_MF_PP_ROUNDS");
        return e ? std::max(0, std::atoi(e)) : 2;
    }();
    std::atomic<int64_t> stamp{0}, bstamp{0};
    std::mutex mu;
    std::condition_variable cv;
    int active = 0;
    bool aborted = false;
    auto tag_of = [&](int32_t v) { return __atomic_load_n(&vs[v].tag, __ATOMIC_RELAXED); };
    auto add_node = [&](std::vector<int32_t>&& members, int32_t parent, std::vector<int32_t> key) -> int32_t {
        std::lock_guard<std::mutex> lk(mu);
        tree.push_back(NdNode{std::move(members), parent, std::move(key)});
        return (int32_t)tree.size() - 1;
    };
    auto push_task = [&](Task&& t) {
        std::lock_guard<std::mutex> lk(mu);
        stack.push_back(std::move(t));
        cv.notify_one();
    };
    auto work = [&]() {
        std::vector<int32_t> q;
        // raised inside a BFS once *stop is seen (checked every 64K visits: a whole-graph BFS of the
        // top piece takes tens of ms), the task then abandons the dissection
        bool cut = false;
        // BFS inside the piece tagged `tag` from root: q holds the visit order, vs[].level the levels
        auto bfs = [&](int32_t root, int64_t tag) -> int32_t {
            const int64_t b = ++bstamp;
            q.clear();
            q.push_back(root);
            vs[root].seen = b;
            vs[root].level = 0;
            int32_t depth = 0;
            for (size_t h = 0; h < q.size(); ++h) {
                const int32_t v = q[h];
                if ((h & 65535) == 65535 && stop && stop->load(std::memory_order_relaxed)) {
                    cut = true;
                    return depth;
                }
                const int32_t lw = vs[v].level + 1;
                for (int64_t e = g.ptr[v]; e < g.ptr[v + 1]; ++e) {
                    const int32_t w = g.adj[e];
                    if (tag_of(w) != tag || vs[w].seen == b) continue;
                    vs[w].seen = b;
                    vs[w].level = lw;
                    depth = std::max(depth, lw);
                    q.push_back(w);
                }
            }
            return depth;
        };
        auto sub_degree = [&](int32_t v, int64_t tag) {
            int32_t dgr = 0;
            for (int64_t e = g.ptr[v]; e < g.ptr[v + 1]; ++e) dgr += tag_of(g.adj[e]) == tag;
            return dgr;
        };
        for (;;) {
            Task t;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return aborted || !stack.empty() || active == 0; });
                if (aborted || stack.empty()) { cv.notify_all(); return; }
                t = std::move(stack.back());
                stack.pop_back();
                ++active;
            }
            auto done = [&]() {
                std::lock_guard<std::mutex> lk(mu);
                --active;
                if (active == 0 && stack.empty()) cv.notify_all();
            };
            auto abort_task = [&]() {
                std::lock_guard<std::mutex> lk(mu);
                aborted = true;
                --active;
                cv.notify_all();
            };
            if (cut || (stop && stop->load(std::memory_order_relaxed))) {
                abort_task();
                return;
            }
            const int64_t sz = (int64_t)t.nodes.size();
            if (sz == 0) { done(); continue; }
            if (sz <= leaf) {
                add_node(std::move(t.nodes), t.parent, std::move(t.key));
                done();
                continue;
            }
            const int64_t tag = ++stamp;
            for (int32_t v : t.nodes) __atomic_store_n(&vs[v].tag, tag, __ATOMIC_RELAXED);
            // from the piece's first vertex: connectivity, and the first pseudo-peripheral level set
            const int32_t depth0 = bfs(t.nodes[0], tag);
            if (cut) {
                abort_task();
                return;
            }
            if ((int64_t)q.size() < sz) {
                // disconnected: components (in the order of their first vertex in the piece); the
                // small ones packed into leaves, the others new pieces
                std::vector<std::vector<int32_t>> comps;
                const int64_t b0 = vs[t.nodes[0]].seen;   // this piece's first BFS; later ones are larger
                comps.push_back(q);
                for (int32_t v : t.nodes) {
                    if (vs[v].seen >= b0) continue;
                    bfs(v, tag);
                    if (cut) break;
                    comps.push_back(q);
                }
                if (cut) {
                    abort_task();
                    return;
                }
                std::vector<int32_t> pack;
                int32_t slot = 0;
                auto key_at = [&](int32_t k) {
                    std::vector<int32_t> kk = t.key;
                    kk.push_back(k);
                    return kk;
                };
                for (auto& c : comps) {
                    if ((int64_t)c.size() > leaf) {
                        push_task(Task{std::move(c), t.parent, key_at(slot++)});
                        continue;
                    }
                    if ((int64_t)(pack.size() + c.size()) > leaf) {
                        add_node(std::move(pack), t.parent, key_at(slot++));
                        pack.clear();
                    }
                    pack.insert(pack.end(), c.begin(), c.end());
                }
                if (!pack.empty()) add_node(std::move(pack), t.parent, key_at(slot++));
                done();
                continue;
            }
            // pseudo-peripheral root (George-Liu): restart from a minimum-degree vertex of the last
            // level while the eccentricity grows
            int32_t root = t.nodes[0];
            int32_t ecc = depth0;   // q and the levels are still those of the BFS from root
            for (int round = 0; round < pp_rounds; ++round) {
                int32_t best = -1, bd = INT32_MAX;
                for (size_t h = q.size(); h-- > 0;) {
                    const int32_t v = q[h];
                    if (vs[v].level != ecc) break;
                    const int32_t dv = sub_degree(v, tag);
                    if (dv < bd || (dv == bd && v < best)) { bd = dv; best = v; }
                }
                const int32_t e2 = bfs(best, tag);
                if (e2 <= ecc) {
                    if (e2 < ecc) ecc = bfs(root, tag);   // restore the levels of the better root
                    break;
                }
                root = best;
                ecc = e2;
            }
            if (cut) {
                abort_task();
                return;
            }
            const int32_t nlev = ecc + 1;
            if (nlev < 3) {   // no level structure to cut: one dense front
                add_node(std::move(t.nodes), t.parent, std::move(t.key));
                done();
                continue;
            }
            std::vector<int64_t> cnt(nlev, 0);
            for (int32_t v : t.nodes) ++cnt[vs[v].level];
            int32_t m = 1;
            {
                int64_t cum = 0;
                for (int32_t l = 0; l < nlev; ++l) {
                    if (2 * (cum + cnt[l] / 2) >= sz) { m = l; break; }
                    cum += cnt[l];
                }
                m = std::max(1, std::min(nlev - 2, m));
            }
            // separator: the vertices of level m that touch level m + 1; the rest of level m joins A
            std::vector<int32_t> A, B, Sep;
            for (int32_t v : t.nodes) {
                const int32_t l = vs[v].level;
                if (l < m) A.push_back(v);
                else if (l > m) B.push_back(v);
                else {
                    bool touch = false;
                    for (int64_t e = g.ptr[v]; e < g.ptr[v + 1] && !touch; ++e)
                        touch = tag_of(g.adj[e]) == tag && vs[g.adj[e]].level == m + 1;
                    (touch ? Sep : A).push_back(v);
                }
            }
            std::vector<int32_t>().swap(t.nodes);
            std::vector<int32_t> ka = t.key, kb = t.key;
            ka.push_back(0);
            kb.push_back(1);
            const int32_t id = add_node(std::move(Sep), t.parent, std::move(t.key));
            push_task(Task{std::move(A), id, std::move(ka)});
            push_task(Task{std::move(B), id, std::move(kb)});
            done();
        }
    };
    int nth = host_threads();
    if (n < 20000) nth = 1;
    std::vector<std::thread> pool;
    try {
        for (int i = 1; i < nth; ++i) pool.emplace_back(work);
    } catch (const std::exception&) {   // fewer threads: the others do the work
    }
    work();
    for (auto& th : pool) th.join();
    if (aborted) return false;
    // canonical order: by key; parents renumbered
    std::vector<int32_t> ord(tree.size());
    std::iota(ord.begin(), ord.end(), 0);
    std::sort(ord.begin(), ord.end(), [&](int32_t x, int32_t y) { return tree[x].key < tree[y].key; });
    std::vector<int32_t> newid(tree.size());
    for (size_t i = 0; i < ord.size(); ++i) newid[ord[i]] = (int32_t)i;
    std::vector<NdNode> sorted;
    sorted.reserve(tree.size());
    for (int32_t o : ord) {
        NdNode nd = std::move(tree[o]);
        if (nd.parent >= 0) nd.parent = newid[nd.parent];
        std::vector<int32_t>().swap(nd.key);
        sorted.push_back(std::move(nd));
    }
    tree.swap(sorted);
    return true;
}

}  // namespace

// The ordering and symbolic structure (host only): fronts in postorder with their columns,
// structs, children, parent maps; per-height lists; work and size figures.
struct MfPlan {
    int64_t nt = 0;
    std::vector<int32_t> perm, iperm, snode, chl, sidx, cmap, height, lists;
    std::vector<int64_t> sof, hstart;
    std::vector<dev::MfFront> fr;
    int32_t H = 0;
    int64_t maxd = 0, maxns = 0, uo = 0;
    double fe = 0.0, fac = 0.0, flops = 0.0;
};

// returns false on an internal inconsistency (a struct entry outside the ancestors)
// max_front_entries: the plan is abandoned once the fronts' sum of d^2 passes it (a pattern
// without small separators, e.g. a random graph); stop: abandoned when raised (another thread's
// factor won)
bool mf_plan(int64_t n, const std::vector<int32_t>& rp, const std::vector<int32_t>& ci, int leaf, bool cplx_flops,
             MfPlan& P, double max_front_entries = 1e300, const std::atomic<bool>* stop = nullptr) {
    static const bool dbg = std::getenv("EIGSOL_MF_DEBUG") != nullptr;
    auto tp = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!dbg) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[mf] %s %.3f s\n", what, std::chrono::duration<double>(t - tp).count());
        tp = t;
    };
    // the graph relabelled in breadth-first order (neighbours get nearby labels: the many BFS
    // passes of the dissection then walk memory locally whatever the caller's numbering)
    SymGraph g;
    std::vector<int32_t> ord(n);   // label -> caller's index
    auto stopped = [&]() { return stop && stop->load(std::memory_order_relaxed); };
    {
        SymGraph g0;
        if (!sym_graph(n, rp, ci, g0, stop)) return false;
        lap("graph: symmetric pattern");
        std::vector<char> done(n, 0);
        int64_t head = 0, tail = 0;
        for (int64_t s0 = 0; s0 < n; ++s0) {
            if (done[s0]) continue;
            done[s0] = 1;
            ord[tail++] = (int32_t)s0;
            while (head < tail) {
                if ((head & 65535) == 0 && stopped()) return false;
                const int32_t v = ord[head++];
                for (int64_t e = g0.ptr[v]; e < g0.ptr[v + 1]; ++e)
                    if (!done[g0.adj[e]]) { done[g0.adj[e]] = 1; ord[tail++] = g0.adj[e]; }
            }
        }
        if (stopped()) return false;
        lap("graph: breadth-first labels");
        std::vector<int32_t> lab(n);
        for (int64_t k = 0; k < n; ++k) lab[ord[k]] = (int32_t)k;
        g.ptr.assign(n + 1, 0);
        for (int64_t k = 0; k < n; ++k) g.ptr[k + 1] = g.ptr[k] + (g0.ptr[ord[k] + 1] - g0.ptr[ord[k]]);
        g.adj.resize(g0.adj.size());
        par_for(n, host_threads(), [&](int64_t b, int64_t e) {
            for (int64_t k = b; k < e; ++k) {
                const int32_t v = ord[k];
                int64_t o = g.ptr[k];
                for (int64_t x = g0.ptr[v]; x < g0.ptr[v + 1]; ++x) g.adj[o++] = lab[g0.adj[x]];
                std::sort(g.adj.begin() + g.ptr[k], g.adj.begin() + o);
            }
        });
    }
    lap("graph");
    std::vector<NdNode> tree;
    if (!nested_dissection(n, g, leaf, tree, stop)) return false;
    lap("dissection");
    // postorder numbering: children before parents, each tree node one contiguous column range
    const int64_t nt = (int64_t)tree.size();
    P.nt = nt;
    std::vector<int32_t> post;   // tree node of each front (postorder)
    post.reserve(nt);
    {
        std::vector<std::vector<int32_t>> kids(nt);
        std::vector<int32_t> roots;
        for (int64_t i = 0; i < nt; ++i) {
            if (tree[i].parent < 0) roots.push_back((int32_t)i);
            else kids[tree[i].parent].push_back((int32_t)i);
        }
        std::vector<std::pair<int32_t, size_t>> st;
        for (int32_t r : roots) {
            st.push_back({r, 0});
            while (!st.empty()) {
                auto& top = st.back();
                if (top.second < kids[top.first].size()) {
                    const int32_t c = kids[top.first][top.second++];
                    st.push_back({c, 0});
                } else {
                    post.push_back(top.first);
                    st.pop_back();
                }
            }
        }
    }
    std::vector<int32_t> front_of_node(nt);
    for (int64_t s = 0; s < nt; ++s) front_of_node[post[s]] = (int32_t)s;
    P.perm.assign(n, 0);
    P.iperm.assign(n, 0);
    P.snode.assign(n, 0);
    P.fr.assign(nt, dev::MfFront{});
    auto& fr = P.fr;
    {
        int32_t c = 0;
        for (int64_t s = 0; s < nt; ++s) {
            const NdNode& nd = tree[post[s]];
            fr[s].c0 = c;
            fr[s].ns = (int32_t)nd.members.size();
            fr[s].parent = nd.parent < 0 ? -1 : front_of_node[nd.parent];
            for (int32_t v : nd.members) {
                P.perm[c] = v;
                P.iperm[v] = c;
                P.snode[c] = (int32_t)s;
                ++c;
            }
        }
    }
    std::vector<NdNode>().swap(tree);
    // children lists (postorder, i.e. the fixed extend-add order)
    auto& chl = P.chl;
    {
        std::vector<std::vector<int32_t>> ch(nt);
        for (int64_t s = 0; s < nt; ++s)
            if (fr[s].parent >= 0) ch[fr[s].parent].push_back((int32_t)s);
        for (int64_t s = 0; s < nt; ++s) {
            fr[s].ch0 = (int32_t)chl.size();
            chl.insert(chl.end(), ch[s].begin(), ch[s].end());
            fr[s].ch1 = (int32_t)chl.size();
        }
    }
    // heights (a leaf 0, a parent one above its highest child) and the per-height front lists
    // (descending ns: each panel's fronts are a prefix)
    P.height.assign(nt, 0);
    P.H = 0;
    for (int64_t s = 0; s < nt; ++s) {
        for (int32_t k = fr[s].ch0; k < fr[s].ch1; ++k) P.height[s] = std::max(P.height[s], P.height[chl[k]] + 1);
        P.H = std::max(P.H, P.height[s]);
    }
    P.hstart.assign(P.H + 2, 0);
    {
        std::vector<std::vector<int32_t>> byh(P.H + 1);
        for (int64_t s = 0; s < nt; ++s) byh[P.height[s]].push_back((int32_t)s);
        for (int32_t h = 0; h <= P.H; ++h) {
            std::stable_sort(byh[h].begin(), byh[h].end(), [&](int32_t a, int32_t b) { return fr[a].ns > fr[b].ns; });
            P.lists.insert(P.lists.end(), byh[h].begin(), byh[h].end());
            P.hstart[h + 1] = (int64_t)P.lists.size();
        }
    }
    // symbolic: struct(s) = indices >= c1 reached from s's rows in M + M^T or through a child's
    // struct (each list ascending).  A front needs only its children's lists, so the fronts of one
    // height are independent: they run on the host threads (a mark array per thread), height after
    // height, and the lists are concatenated in front order -- the same arrays as a serial pass.
    auto& sidx = P.sidx;
    auto& sof = P.sof;
    sof.assign(nt + 1, 0);
    {
        std::vector<std::vector<int32_t>> lists(nt);
        std::atomic<bool> over{false};
        std::atomic<double> fe_run{0.0};
        const int nth = host_threads();
        std::vector<std::vector<int32_t>> marks(std::max(1, nth));
        auto one = [&](int32_t s, std::vector<int32_t>& mark) {
            const int32_t c0 = fr[s].c0, c1 = c0 + fr[s].ns;
            std::vector<int32_t>& lst = lists[s];
            for (int32_t i = c0; i < c1; ++i) {
                const int32_t v = P.perm[i];
                for (int64_t e = g.ptr[v]; e < g.ptr[v + 1]; ++e) {
                    const int32_t j = P.iperm[g.adj[e]];
                    if (j >= c1 && mark[j] != s) { mark[j] = s; lst.push_back(j); }
                }
            }
            for (int32_t k = fr[s].ch0; k < fr[s].ch1; ++k)
                for (int32_t j : lists[chl[k]])
                    if (j >= c1 && mark[j] != s) { mark[j] = s; lst.push_back(j); }
            std::sort(lst.begin(), lst.end());
            const double d = (double)fr[s].ns + (double)lst.size();
            double cur = fe_run.load(std::memory_order_relaxed);
            while (!fe_run.compare_exchange_weak(cur, cur + d * d, std::memory_order_relaxed)) {}
            if (cur + d * d > max_front_entries) over.store(true, std::memory_order_relaxed);
        };
        for (int32_t h = 0; h <= P.H; ++h) {
            const int64_t b = P.hstart[h], m = P.hstart[h + 1] - b;
            const int use = m < 8 ? 1 : (int)std::min<int64_t>(std::max(1, nth), m);
            auto run = [&](int t) {
                std::vector<int32_t>& mark = marks[t];
                if (mark.empty()) mark.assign(n, -1);
                for (int64_t k = t; k < m; k += use) {   // fronts dealt round-robin: sizes vary by position
                    if (over.load(std::memory_order_relaxed) || stopped()) return;
                    one(P.lists[b + k], mark);
                }
            };
            if (use <= 1) {
                run(0);
            } else {
                std::vector<std::thread> th;
                try {
                    for (int t = 1; t < use; ++t) th.emplace_back(run, t);
                } catch (const std::exception&) {
                    for (auto& x : th) x.join();
                    th.clear();
                    for (int t = 1; t < use; ++t) run(t);   // no more threads: this one does the rest
                }
                run(0);
                for (auto& x : th) x.join();
            }
            if (over.load() || stopped()) return false;
        }
        int64_t tot = 0;
        for (int64_t s = 0; s < nt; ++s) tot += (int64_t)lists[s].size();
        sidx.reserve(tot);
        for (int64_t s = 0; s < nt; ++s) {
            sidx.insert(sidx.end(), lists[s].begin(), lists[s].end());
            std::vector<int32_t>().swap(lists[s]);
            sof[s + 1] = (int64_t)sidx.size();
            fr[s].ms = (int32_t)(sof[s + 1] - sof[s]);
            fr[s].sof = sof[s];
            fr[s].d = fr[s].ns + fr[s].ms;
        }
    }
    std::vector<int64_t>().swap(g.ptr);
    std::vector<int32_t>().swap(g.adj);
    // labels -> the caller's indices
    for (int64_t c = 0; c < n; ++c) {
        P.perm[c] = ord[P.perm[c]];
        P.iperm[P.perm[c]] = (int32_t)c;
    }
    lap("symbolic");
    // sizes and work
    for (int64_t s = 0; s < nt; ++s) {
        const double d = fr[s].d, ns = fr[s].ns;
        fr[s].off = (int64_t)P.fe;
        fr[s].uoff = P.uo;
        P.uo += fr[s].ms;
        P.fe += d * d;
        P.fac += ns * (2.0 * d - ns);
        // sum_{k < ns} 2 (d - k - 1)^2 multiply-adds ~ 2 (ns d^2 - ns^2 d + ns^3 / 3)
        P.flops += 2.0 * (ns * d * d - ns * ns * d + ns * ns * ns / 3.0);
        P.maxd = std::max<int64_t>(P.maxd, fr[s].d);
        P.maxns = std::max<int64_t>(P.maxns, fr[s].ns);
    }
    if (cplx_flops) P.flops *= 4.0;
    lap("sizes");
    // parent positions of every child's struct entries
    P.cmap.assign(sidx.size(), 0);
    for (int64_t s = 0; s < nt; ++s) {
        const int32_t p = fr[s].parent;
        if (p < 0) {
            if (fr[s].ms) return false;   // a root reaches nothing past itself
            continue;
        }
        const int32_t pc0 = fr[p].c0, pc1 = pc0 + fr[p].ns;
        const int32_t* ps = sidx.data() + sof[p];
        const int32_t pm = fr[p].ms;
        int32_t cur = 0;
        for (int64_t e = sof[s]; e < sof[s + 1]; ++e) {
            const int32_t j = sidx[e];
            if (j < pc0) return false;   // struct(s) must lie in the ancestors
            if (j < pc1) P.cmap[e] = j - pc0;
            else {
                while (cur < pm && ps[cur] < j) ++cur;   // both ascending
                if (cur == pm || ps[cur] != j) return false;
                P.cmap[e] = fr[p].ns + cur;
            }
        }
    }
    lap("parent maps");
    return true;
}

struct MfLaunch {
    int kind;   // 0 extend, 1 panel, 2 gemm
    int32_t h, q;
    int64_t off, cnt;
};

struct MfHost {
    MfPlan P;
    int64_t n = 0, nnz = 0;
    int nb = 32;
    int64_t sb = 16;
    std::vector<int64_t> dst;              // M's entries -> front offsets
    std::vector<MfLaunch> plan;            // factorization launches
    std::vector<int32_t> tab, slists, tabf, tabb, tabf2, tabb2, lds_asm, lds_asm2;
    std::vector<int64_t> sstart, nwave, nsmall, nbig, foff, fcnt, boff, bcnt, foff2, fcnt2, boff2, bcnt2;
    int32_t nflag = 0;
    int64_t zsz = 0;
    int32_t hflow = 0;                     // heights below it: the dataflow launches (0: off)
    std::vector<int32_t> flow_f, flow_b;   // their fronts, ascending / descending height
    int32_t lds_flow_f = 0, lds_flow_b = 0;
    std::vector<int32_t> sub_ranges;       // small subtrees solved by one workgroup each: (lo, hi) fronts
    int32_t lds_sub_f = 0, lds_sub_b = 0;
    std::vector<int32_t> inv_list;         // fronts with an inverse form (MfFront::goff)
    int64_t gsz = 0;                       // its scalars, stored after the fronts in F
    MfStats stt;
};

// The host half of the factor: plan, bounds, entry destinations, launch and solve tables.  Needs
// no device (free_bytes: the device memory the fronts may take), so gmres.hip runs it on a second
// host thread beside the natural-order fill attempt.
int mf_prepare_host(int64_t n, const std::vector<int32_t>& rp, const std::vector<int32_t>& ci, bool cplx_s,
                    double free_bytes, MfHost& X, const std::atomic<bool>* stop) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const int NB = cplx_s ? dev::RankKMax<cplx>::value : dev::RankKMax<double>::value;
    const int64_t sb = cplx_s ? 16 : 8;
    X.n = n;
    X.nb = NB;
    X.sb = sb;
    int leaf = 64;
    if (const char* e = std::getenv("EIGSOL_MF_LEAF")) leaf = std::max(4, std::atoi(e));
    MfPlan& P = X.P;
    double cap = 0.45 * free_bytes;
    if (const char* e = std::getenv("EIGSOL_MF_MAX_GB")) cap = std::min(cap, std::atof(e) * 1073741824.0);
    if (!mf_plan(n, rp, ci, leaf, cplx_s, P, cap / (double)sb, stop)) return EIGSOL_E_UNSUPPORTED;
    const int64_t nt = P.nt;
    auto& fr = P.fr;
    const auto& chl = P.chl;
    const auto& sidx = P.sidx;
    const auto& sof = P.sof;
    const auto& lists = P.lists;
    const auto& hstart = P.hstart;
    const int32_t H = P.H;
    const double fe = P.fe, fac = P.fac;
    MfStats& stt = X.stt;
    stt.fronts = nt;
    stt.heights = H + 1;
    stt.max_front = P.maxd;
    stt.max_pivots = P.maxns;
    stt.front_entries = fe;
    stt.factor_entries = fac;
    stt.flops = P.flops;
    // bounds: device memory for the fronts, the solve kernels' LDS, the work
    const double lds_max = 120.0 * 1024.0;
    if (fe * (double)sb > cap || (double)(P.maxns + P.maxd) * (double)sb > lds_max || P.flops > 4e13)
        return EIGSOL_E_UNSUPPORTED;
    // destinations of M's entries (the caller's numbering) in the fronts
    const int64_t nnz = rp[n];
    X.nnz = nnz;
    auto& dst = X.dst;
    dst.assign(nnz, 0);
    auto pos_in = [&](int32_t s, int32_t j) -> int64_t {
        const int32_t c0 = fr[s].c0;
        if (j < c0 + fr[s].ns) return j - c0;
        const int32_t* b = sidx.data() + sof[s];
        const int64_t k = std::lower_bound(b, b + fr[s].ms, j) - b;
        return (k < fr[s].ms && b[k] == j) ? fr[s].ns + k : -1;
    };
    std::atomic<bool> bad{false};
    par_for(n, host_threads(), [&](int64_t rb, int64_t re) {
        for (int64_t r = rb; r < re; ++r)
            for (int32_t e = rp[r]; e < rp[r + 1]; ++e) {
                const int32_t i = P.iperm[r], j = P.iperm[ci[e]];
                const int32_t s = P.snode[std::min(i, j)];
                const int64_t pi = pos_in(s, i), pj = pos_in(s, j);
                if (pi < 0 || pj < 0) { bad.store(true); return; }   // not in the front: an inconsistent plan
                dst[e] = fr[s].off + pi + pj * (int64_t)fr[s].d;
            }
    });
    if (bad.load()) return EIGSOL_E_UNSUPPORTED;
    // launch tables: extend-add (child, first column) per (height, child rank); trailing-update
    // tiles (front, tile row, tile column) per (height, panel)
    using Launch = MfLaunch;
    auto& plan = X.plan;
    auto& tab = X.tab;
    for (int32_t h = 0; h <= H; ++h) {
        const int32_t* L = lists.data() + hstart[h];
        const int64_t cnt = hstart[h + 1] - hstart[h];
        int32_t maxch = 0, maxq = 0;
        for (int64_t t = 0; t < cnt; ++t) {
            maxch = std::max(maxch, fr[L[t]].ch1 - fr[L[t]].ch0);
            maxq = std::max(maxq, (fr[L[t]].ns + NB - 1) / NB);
        }
        for (int32_t j = 0; j < maxch; ++j) {
            const int64_t o = (int64_t)tab.size();
            for (int64_t t = 0; t < cnt; ++t) {
                const dev::MfFront& p = fr[L[t]];
                if (p.ch1 - p.ch0 <= j) continue;
                const int32_t c = chl[p.ch0 + j];
                for (int32_t c0 = 0; c0 < fr[c].ms; c0 += 64) { tab.push_back(c); tab.push_back(c0); }
            }
            const int64_t k = ((int64_t)tab.size() - o) / 2;
            if (k) plan.push_back(Launch{0, h, j, o, k});
        }
        for (int32_t q = 0; q < maxq; ++q) {
            int64_t np = 0;
            while (np < cnt && fr[L[np]].ns > q * NB) ++np;
            plan.push_back(Launch{1, h, q, hstart[h], np});
            const int64_t o = (int64_t)tab.size();
            for (int64_t t = 0; t < np; ++t) {
                const dev::MfFront& f = fr[L[t]];
                const int32_t c1 = std::min(f.ns, (q + 1) * NB), m = f.d - c1;
                const int32_t nt64 = (m + 63) / 64;
                for (int32_t a = 0; a < nt64; ++a)
                    for (int32_t b = 0; b < nt64; ++b) { tab.push_back(L[t]); tab.push_back(a); tab.push_back(b); }
            }
            const int64_t k = ((int64_t)tab.size() - o) / 3;
            if (k) plan.push_back(Launch{2, h, q, o, k});
        }
    }
    // solve plan: fronts with many pivots or rows are solved by one workgroup per 64-row block
    // (mf_big_*), the others by one workgroup each (mf_fwd / mf_bwd)
    int big_ns = 96, big_d = 256;
    if (const char* e = std::getenv("EIGSOL_MF_BIG_NS")) big_ns = std::atoi(e);
    if (const char* e = std::getenv("EIGSOL_MF_BIG_D")) big_d = std::atoi(e);
    auto &slists = X.slists, &tabf = X.tabf, &tabb = X.tabb, &tabf2 = X.tabf2, &tabb2 = X.tabb2, &lds_asm = X.lds_asm;
    auto& lds_asm2 = X.lds_asm2;
    auto &sstart = X.sstart, &nwave = X.nwave, &nsmall = X.nsmall, &nbig = X.nbig, &foff = X.foff, &fcnt = X.fcnt,
         &boff = X.boff, &bcnt = X.bcnt, &foff2 = X.foff2, &fcnt2 = X.fcnt2, &boff2 = X.boff2, &bcnt2 = X.bcnt2;
    sstart.assign(H + 2, 0);
    for (auto* v : {&nwave, &nsmall, &nbig, &foff, &fcnt, &boff, &bcnt, &foff2, &fcnt2, &boff2, &bcnt2}) v->assign(H + 1, 0);
    // one wave per small front (EIGSOL_MF_WAVE=1): measured 2.21 against 2.01 ms per 1M iteration
    // with one workgroup per front - the same loads in flight per CU, and the struct rows' GEMV on
    // one wave instead of four
    bool wave_ok = false;
    if (const char* e = std::getenv("EIGSOL_MF_WAVE")) wave_ok = std::atoi(e) != 0;
    // small subtrees (at most sub_cap pivots, EIGSOL_MF_SUB; 0: off) solved whole by one workgroup
    // each: their fronts are a contiguous postorder range, so a workgroup walks it up (forward) and
    // down (backward) with no hand-off between workgroups and no per-height launch.  Measured and
    // left off (1M convection-diffusion, tools/mf_grid.sh): caps 256 / 512 / 1024 / 2048 pivots
    // 2.21 / 2.33 / 2.63 / 2.70 ms per iteration against 2.00 - the per-height launches keep every
    // front of a height in flight, a subtree's fronts run one after the other
    int sub_cap = 0;
    if (const char* e = std::getenv("EIGSOL_MF_SUB")) sub_cap = std::atoi(e);
    if (const char* e = std::getenv("EIGSOL_MF_FLOW"))
        if (std::atoi(e) != 0) sub_cap = 0;   // the dataflow experiment takes the lower heights itself
    std::vector<char> insub(nt, 0);
    X.sub_ranges.clear();
    if (sub_cap > 0) {
        std::vector<int64_t> subp(nt, 0);
        std::vector<int32_t> lo(nt);
        for (int64_t s2 = 0; s2 < nt; ++s2) {   // postorder: children first
            subp[s2] += fr[s2].ns;
            if (fr[s2].ch0 == fr[s2].ch1) lo[s2] = (int32_t)s2;
            else {
                int32_t m = (int32_t)s2;
                for (int32_t k = fr[s2].ch0; k < fr[s2].ch1; ++k) m = std::min(m, lo[chl[k]]);
                lo[s2] = m;
            }
            if (fr[s2].parent >= 0) subp[fr[s2].parent] += subp[s2];
            insub[s2] = subp[s2] <= sub_cap;
        }
        for (int64_t s2 = 0; s2 < nt; ++s2)
            if (insub[s2] && (fr[s2].parent < 0 || !insub[fr[s2].parent])) {
                X.sub_ranges.push_back(lo[s2]);
                X.sub_ranges.push_back((int32_t)s2);
            }
        for (int64_t s2 = 0; s2 < nt; ++s2)
            if (insub[s2]) {
                X.lds_sub_f = std::max<int32_t>(X.lds_sub_f, (int32_t)((2 * fr[s2].ns + fr[s2].ms) * sb));
                X.lds_sub_b = std::max<int32_t>(X.lds_sub_b, (int32_t)((fr[s2].ns + fr[s2].ms) * sb));
            }
    }
    lds_asm.assign(H + 1, 0);
    lds_asm2.assign(H + 1, 0);
    bool inv_on = true;
    int inv_d = 256;   // 256 / 384 / 512: 1.71 / 1.72 / 1.72 ms per 1M iteration (tools/mf_grid.sh)
    if (const char* e = std::getenv("EIGSOL_MF_INVFORM")) inv_on = std::atoi(e) != 0;
    if (const char* e = std::getenv("EIGSOL_MF_INV_D")) inv_d = std::max(1, std::atoi(e));
    int32_t& nflag = X.nflag;
    int64_t& zsz = X.zsz;
    for (int32_t h = 0; h <= H; ++h) {
        std::vector<int32_t> big, wg;
        for (int64_t t = hstart[h]; t < hstart[h + 1]; ++t) {
            dev::MfFront& q = fr[lists[t]];
            q.flag0 = -1;
            q.zoff = 0;
            if (insub[lists[t]]) continue;
            // fronts of at most 64 pivots and inv_d rows stay one-workgroup fronts (inverse form)
            const bool inv_ok = inv_on && q.ns <= 64 && q.d <= inv_d;
            const bool is_big = big_ns > 0 && (q.ns >= big_ns || (q.d >= big_d && !inv_ok));
            if (is_big) big.push_back(lists[t]);
            else if (wave_ok && q.ns <= dev::kWaveNs && q.ms <= dev::kWaveMs) slists.push_back(lists[t]);
            else wg.push_back(lists[t]);
        }
        nwave[h] = (int64_t)slists.size() - sstart[h];
        slists.insert(slists.end(), wg.begin(), wg.end());
        nsmall[h] = (int64_t)wg.size();
        nbig[h] = (int64_t)big.size();
        slists.insert(slists.end(), big.begin(), big.end());
        sstart[h + 1] = (int64_t)slists.size();
        foff[h] = (int64_t)tabf.size() / 2;
        boff[h] = (int64_t)tabb.size() / 2;
        foff2[h] = (int64_t)tabf2.size() / 2;
        boff2[h] = (int64_t)tabb2.size() / 2;
        for (int32_t b : big) {
            dev::MfFront& q = fr[b];
            const int32_t nblk = (q.ns + 63) / 64, nsb = (q.ms + 63) / 64;
            q.flag0 = nflag;
            q.zoff = zsz;
            nflag += nblk;
            zsz += q.d;
            for (int32_t k = 0; k < nblk + nsb; ++k) { tabf.push_back(b); tabf.push_back(k); }
            for (int32_t k = nblk - 1; k >= 0; --k) { tabb.push_back(b); tabb.push_back(k); }
            const int32_t npair = (nblk + 1) / 2;
            for (int32_t k = 0; k < npair + nsb; ++k) { tabf2.push_back(b); tabf2.push_back(k); }
            for (int32_t k = npair - 1; k >= 0; --k) { tabb2.push_back(b); tabb2.push_back(k); }
            lds_asm[h] = std::max<int32_t>(lds_asm[h], (int32_t)(q.ns * sb));
            lds_asm2[h] = std::max<int32_t>(lds_asm2[h], (int32_t)((q.ns + q.ms) * sb));   // d: mf_big_asm_front2
        }
        fcnt[h] = (int64_t)tabf.size() / 2 - foff[h];
        bcnt[h] = (int64_t)tabb.size() / 2 - boff[h];
        fcnt2[h] = (int64_t)tabf2.size() / 2 - foff2[h];
        bcnt2[h] = (int64_t)tabb2.size() / 2 - boff2[h];
    }
    // inverse forms of the one-workgroup fronts with at most 64 pivots and inv_d rows
    // (mf_invform_kernel), kept only while the fronts and the forms fit 0.6 of the device memory
    X.inv_list.clear();
    X.gsz = 0;
    {
        const bool on = inv_on;
        for (int64_t s2 = 0; s2 < nt; ++s2) {
            dev::MfFront& q = fr[s2];
            q.goff = -1;
            if (on && q.flag0 < 0 && q.ns <= 64 && q.d <= inv_d) {
                q.goff = (int64_t)fe + X.gsz;
                X.gsz += 2 * (int64_t)q.d * q.ns;
                X.inv_list.push_back((int32_t)s2);
            }
        }
        if (((double)fe + (double)X.gsz) * (double)sb > 0.6 * free_bytes) {
            for (int32_t s2 : X.inv_list) fr[s2].goff = -1;
            X.inv_list.clear();
            X.gsz = 0;
        }
    }
    // dataflow launches for the heights below the first one with a large front (EIGSOL_MF_FLOW=0: off)
    {
        bool flow = false;
        if (const char* e = std::getenv("EIGSOL_MF_FLOW")) flow = std::atoi(e) != 0;
        int32_t hf = H + 1;
        for (int32_t h = 0; h <= H; ++h)
            if (nbig[h]) { hf = h; break; }
        X.hflow = flow ? hf : 0;
        X.flow_f.clear();
        X.flow_b.clear();
        for (int32_t h = 0; h < X.hflow; ++h)
            for (int64_t t = hstart[h]; t < hstart[h + 1]; ++t) {
                const dev::MfFront& q = fr[lists[t]];
                X.flow_f.push_back(lists[t]);
                X.lds_flow_f = std::max<int32_t>(X.lds_flow_f, (int32_t)((2 * q.ns + q.ms) * sb));
                X.lds_flow_b = std::max<int32_t>(X.lds_flow_b, (int32_t)((q.ns + q.ms) * sb));
            }
        for (int32_t h = X.hflow - 1; h >= 0; --h)
            for (int64_t t = hstart[h]; t < hstart[h + 1]; ++t) X.flow_b.push_back(lists[t]);
    }
    stt.order_seconds = std::chrono::duration<double>(clk::now() - t0).count();
    if (std::getenv("EIGSOL_MF_DEBUG"))
        std::fprintf(stderr, "[mf] plan + maps + tables %.3f s; fronts %lld, heights %d, factor entries %.3g, flops %.3g\n",
                     stt.order_seconds, (long long)nt, H + 1, fac, P.flops);
    return EIGSOL_OK;
}

template <class S>
int mf_create_t(eigsol_ctx* ctx, int dtype, MfHost& X, const S* vals, MfFactor** out, double tau, int64_t* nstatic) {
    *out = nullptr;
    using clk = std::chrono::steady_clock;
    constexpr int NB = dev::RankKMax<S>::value;
    const int64_t sb = (int64_t)sizeof(S);
    if (X.nb != NB || X.sb != sb) return fail(EIGSOL_E_INVALID, "solve_shifted: multifrontal plan of another scalar type");
    const int64_t n = X.n, nnz = X.nnz;
    MfPlan& P = X.P;
    const int64_t nt = P.nt;
    auto& fr = P.fr;
    const auto& chl = P.chl;
    const auto& sidx = P.sidx;
    const auto& lists = P.lists;
    const auto& hstart = P.hstart;
    const int32_t H = P.H;
    const double fe = P.fe, fac = P.fac;
    const int64_t uo = P.uo;
    MfStats& stt = X.stt;
    using Launch = MfLaunch;
    const auto& dst = X.dst;
    const auto& plan = X.plan;
    const auto& tab = X.tab;
    const auto &slists = X.slists, &tabf = X.tabf, &tabb = X.tabb, &tabf2 = X.tabf2, &tabb2 = X.tabb2,
               &lds_asm = X.lds_asm;
    auto& lds_asm2 = X.lds_asm2;
    const auto &sstart = X.sstart, &nwave = X.nwave, &nsmall = X.nsmall, &nbig = X.nbig, &foff = X.foff,
               &fcnt = X.fcnt, &boff = X.boff, &bcnt = X.bcnt;
    const int32_t nflag = X.nflag;
    const int64_t zsz = X.zsz;
    (void)plan;
    // ---- device
    auto* f = new MfFactor();
    f->ctx = ctx;
    ctx_retain(ctx);
    f->dtype = dtype;
    f->n = n;
    f->nb = NB;
    f->nfront = nt;
    f->hstart = hstart;
    f->sstart = sstart;
    f->nwave = nwave;
    f->nsmall = nsmall;
    f->nbig = nbig;
    f->foff = foff;
    f->fcnt = fcnt;
    f->boff = boff;
    f->bcnt = bcnt;
    f->foff2 = X.foff2;
    f->fcnt2 = X.fcnt2;
    f->boff2 = X.boff2;
    f->bcnt2 = X.bcnt2;
    f->lds_asm = lds_asm;
    f->lds_asm2 = lds_asm2;
    // the fused forward launch's assembly holds a whole front's right-hand side in LDS
    for (int32_t b : lds_asm2)
        if (b > 120 * 1024) f->fuse_big = false;
    if (const char* e = std::getenv("EIGSOL_MF_PAIR")) f->pair = std::atoi(e) != 0;
    if (const char* e = std::getenv("EIGSOL_MF_BACKOFF")) f->backoff = std::atoi(e) & 3;
    if (const char* e = std::getenv("EIGSOL_MF_FUSE_ASM")) f->fuse_asm = std::atoi(e) != 0;
    if (const char* e = std::getenv("EIGSOL_MF_FUSE_BIG"))
        if (std::atoi(e) == 0) f->fuse_big = false;
    // value flags (bit 4; EIGSOL_MF_VALFLAG=0: epoch flags): 1M convection-diffusion 1.657 -> 1.567 ms
    {
        const char* e = std::getenv("EIGSOL_MF_VALFLAG");
        if (!(e && std::atoi(e) == 0)) f->backoff |= 4;
    }
    // the large fronts' row-block solves take their next-to-diagonal block premultiplied (bit 8, with
    // value flags; EIGSOL_MF_PREMUL=0: off)
    {
        const char* e = std::getenv("EIGSOL_MF_PREMUL");
        if (!(e && std::atoi(e) == 0)) f->backoff |= 8;
    }
    f->lds_fwd.assign(H + 1, 0);
    f->lds_bwd.assign(H + 1, 0);
    // the inverse-form branch keeps 256 partial sums after the front's vectors
    const int32_t inv_lds = X.gsz ? (int32_t)(256 * sb) : 0;
    for (int32_t h = 0; h <= H; ++h)
        for (int64_t t = sstart[h] + nwave[h]; t < sstart[h] + nwave[h] + nsmall[h]; ++t) {
            const dev::MfFront& q = fr[slists[t]];
            f->lds_fwd[h] = std::max<int32_t>(f->lds_fwd[h], (int32_t)((2 * q.ns + q.ms) * sb) + inv_lds);
            f->lds_bwd[h] = std::max<int32_t>(f->lds_bwd[h], (int32_t)((q.ns + q.ms) * sb) + inv_lds);
        }
    hipStream_t st = ctx->stream;
    int rc = EIGSOL_OK;
    int32_t *d_tab = nullptr, *d_piv = nullptr, *d_z = nullptr;
    int64_t* d_dst = nullptr;
    S* d_v = nullptr;
    // an allocation that fails after the plan's free-memory estimate declines the factor
    // (EIGSOL_E_UNSUPPORTED: the caller goes on with ILU(0)); the out-of-memory status is cleared
    auto dm = [&](void** p, size_t bytes) {
        if (rc == EIGSOL_OK && hipMalloc(p, std::max<size_t>(bytes, 16)) != hipSuccess) {
            (void)hipGetLastError();
            *p = nullptr;
            rc = fail(EIGSOL_E_UNSUPPORTED,
                      "solve_shifted: multifrontal buffers (" + std::to_string(bytes >> 20) + " MiB) declined");
        }
    };
    dm((void**)&f->fronts, nt * sizeof(dev::MfFront));
    dm((void**)&f->chl, chl.size() * 4);
    dm((void**)&f->sidx, sidx.size() * 4);
    dm((void**)&f->cmap, P.cmap.size() * 4);
    dm((void**)&f->perm, n * 4);
    dm((void**)&f->pinv, n * 4);
    dm((void**)&f->lists, lists.size() * 4);
    dm((void**)&f->slists, slists.size() * 4);
    dm((void**)&f->tabf, tabf.size() * 4);
    dm((void**)&f->tabb, tabb.size() * 4);
    dm((void**)&f->tabf2, tabf2.size() * 4);
    dm((void**)&f->tabb2, tabb2.size() * 4);
    dm((void**)&f->flags, (size_t)nflag * 4);
    dm((void**)&f->err, 4);
    dm(&f->z, (size_t)zsz * sb);
    dm((void**)&f->bigm, (size_t)n);
    dm(&f->tinv, (size_t)nflag * dev::kMfTinv * sb);
    f->hflow = X.hflow;
    f->nflow = (int32_t)X.flow_f.size();
    f->lds_flow_f = X.lds_flow_f;
    f->lds_flow_b = X.lds_flow_b;
    if (const char* e = std::getenv("EIGSOL_MF_FLOW_MODE")) f->flow_mode = std::atoi(e) & 3;
    dm((void**)&f->flow_f, X.flow_f.size() * 4);
    dm((void**)&f->flow_b, X.flow_b.size() * 4);
    dm((void**)&f->fheight, nt * 4);
    dm((void**)&f->done, nt * 4);
    f->nsub = (int32_t)(X.sub_ranges.size() / 2);
    f->lds_bbig.assign(H + 1, 0);
    for (int32_t h = 0; h <= H; ++h)
        for (int64_t t = sstart[h] + nwave[h] + nsmall[h]; t < sstart[h] + nwave[h] + nsmall[h] + nbig[h]; ++t)
            f->lds_bbig[h] = std::max<int32_t>(f->lds_bbig[h], (int32_t)(fr[slists[t]].ms * sb));
    f->lds_sub_f = X.lds_sub_f ? X.lds_sub_f + inv_lds : 0;
    f->lds_sub_b = X.lds_sub_b ? X.lds_sub_b + inv_lds : 0;
    dm((void**)&f->sub_ranges, X.sub_ranges.size() * 4);
    dm(&f->F, ((size_t)fe + (size_t)X.gsz) * sb);
    int32_t* d_inv = nullptr;
    if (!X.inv_list.empty()) dm((void**)&d_inv, X.inv_list.size() * 4);
    dm(&f->u, (size_t)uo * sb);
    dm(&f->w, n * sb);
    dm(&f->x, n * sb);
    dm((void**)&d_tab, tab.size() * 4);
    dm((void**)&d_piv, n * 4);
    dm((void**)&d_z, 8);   // [0] zero-pivot flag, [1] static pivots
    dm((void**)&d_dst, nnz * 8);
    dm((void**)&d_v, nnz * sb);
    std::vector<int32_t> hpiv(n);
    int32_t hz2[2] = {0, 0};
    const int32_t& hz = hz2[0];
    if (rc == EIGSOL_OK) {
        const auto t1 = clk::now();
        auto up = [&](void* d, const void* h, size_t b) {
            if (b) hipMemcpyAsync(d, h, b, hipMemcpyHostToDevice, st);
        };
        up(f->fronts, fr.data(), nt * sizeof(dev::MfFront));
        up(f->chl, chl.data(), chl.size() * 4);
        up(f->sidx, sidx.data(), sidx.size() * 4);
        up(f->cmap, P.cmap.data(), P.cmap.size() * 4);
        up(f->perm, P.perm.data(), n * 4);
        up(f->lists, lists.data(), lists.size() * 4);
        up(f->slists, slists.data(), slists.size() * 4);
        up(f->tabf, tabf.data(), tabf.size() * 4);
        up(f->tabb, tabb.data(), tabb.size() * 4);
        up(f->tabf2, tabf2.data(), tabf2.size() * 4);
        up(f->tabb2, tabb2.data(), tabb2.size() * 4);
        hipMemsetAsync(f->flags, 0, std::max<size_t>((size_t)nflag * 4, 4), st);
        up(f->flow_f, X.flow_f.data(), X.flow_f.size() * 4);
        up(f->flow_b, X.flow_b.data(), X.flow_b.size() * 4);
        up(f->fheight, P.height.data(), nt * 4);
        up(f->sub_ranges, X.sub_ranges.data(), X.sub_ranges.size() * 4);
        {
            // the large fronts' pivot rows (mf_fwd_height_kernel's gather) and an all-unsolved z
            std::vector<uint8_t> bm((size_t)n, 0);
            for (int32_t h = 0; h <= H; ++h)
                for (int64_t t = sstart[h] + nwave[h] + nsmall[h]; t < sstart[h] + nwave[h] + nsmall[h] + nbig[h]; ++t) {
                    const dev::MfFront& q = fr[slists[t]];
                    for (int32_t r = 0; r < q.ns; ++r) bm[(size_t)q.c0 + r] = 1;
                }
            up(f->bigm, bm.data(), (size_t)n);
            hipMemsetD32Async(static_cast<hipDeviceptr_t>(f->z), 0x7FF4DEADu, std::max<size_t>((size_t)zsz * sb / 4, 1), st);
        }
        hipMemsetAsync(f->done, 0, nt * 4, st);
        hipMemsetAsync(f->err, 0, 4, st);
        up(d_tab, tab.data(), tab.size() * 4);
        if (d_inv) up(d_inv, X.inv_list.data(), X.inv_list.size() * 4);
        up(d_dst, dst.data(), nnz * 8);
        up(d_v, vals, nnz * sb);
        hipMemsetAsync(f->F, 0, (size_t)fe * sb, st);
        hipMemsetAsync(d_z, 0, 8, st);
        S* F = static_cast<S*>(f->F);
        if (nnz)
            hipLaunchKernelGGL((dev::mf_scatter_kernel<S>), dim3((nnz + 255) / 256), dim3(256), 0, st, d_dst, d_v, nnz, F);
        for (const Launch& l : plan) {
            if (l.kind == 0)
                hipLaunchKernelGGL((dev::mf_extend_kernel<S>), dim3(l.cnt), dim3(256), 0, st, f->fronts, d_tab + l.off,
                                   f->cmap, F);
            else if (l.kind == 1)
                hipLaunchKernelGGL((dev::mf_panel_kernel<S, NB>), dim3(l.cnt), dim3(256), 0, st, f->fronts,
                                   f->lists + l.off, l.q, F, d_piv, d_z, tau, d_z + 1);
            else
                hipLaunchKernelGGL((dev::mf_gemm_kernel<S, NB>), dim3(l.cnt), dim3(256), 0, st, f->fronts, d_tab + l.off,
                                   l.q, F);
        }
        if (!tabb.empty()) {
            hipLaunchKernelGGL((dev::mf_inv_kernel<S>), dim3(tabb.size() / 2), dim3(256), 0, st, f->fronts, f->tabb, F,
                               static_cast<S*>(f->tinv));
            if ((f->backoff & 12) == 12)
                hipLaunchKernelGGL((dev::mf_premul_kernel<S>), dim3(tabb.size() / 2), dim3(256), 0, st, f->fronts,
                                   f->tabb, F, static_cast<S*>(f->tinv));
        }
        if (d_inv)
        {
            // EIGSOL_MF_INVFORM=1: round 5's kernel (one HBM load per multiply-add of L21 inv(L11) and inv(U11) U12)
            const char* ie = std::getenv("EIGSOL_MF_INVFORM");
            if (ie && std::atoi(ie) == 1)
                hipLaunchKernelGGL((dev::mf_invform_kernel<S>), dim3(X.inv_list.size()), dim3(256), 0, st, f->fronts, d_inv, F);
            else
                hipLaunchKernelGGL((dev::mf_invform2_kernel<S>), dim3(X.inv_list.size()), dim3(256), 0, st, f->fronts, d_inv, F);
        }
        hipMemcpyAsync(hpiv.data(), d_piv, n * 4, hipMemcpyDeviceToHost, st);
        hipMemcpyAsync(hz2, d_z, 8, hipMemcpyDeviceToHost, st);
        if (hipStreamSynchronize(st) != hipSuccess || hipGetLastError() != hipSuccess)
            rc = fail(EIGSOL_E_HIP, "solve_shifted: multifrontal factorization");
        stt.numeric_seconds = std::chrono::duration<double>(clk::now() - t1).count();
        if (std::getenv("EIGSOL_MF_DEBUG")) std::fprintf(stderr, "[mf] upload + numeric %.3f s\n", stt.numeric_seconds);
    }
    for (void* p : {(void*)d_tab, (void*)d_piv, (void*)d_z, (void*)d_dst, (void*)d_v, (void*)d_inv})
        if (p) hipFree(p);
    if (rc == EIGSOL_OK && hz) rc = fail(EIGSOL_E_SOLVER, "solve_shifted: multifrontal LU met a zero pivot");
    if (nstatic) *nstatic = hz2[1];
    f->nstatic = hz2[1];
    if (rc == EIGSOL_OK) {
        // composite interchange of every front: row t of the factored front is row q[t] of the assembled one
        std::vector<int32_t> pinv(n);
        for (int64_t s = 0; s < nt; ++s) {
            const int32_t c0 = fr[s].c0, ns = fr[s].ns;
            int32_t* qv = pinv.data() + c0;
            for (int32_t t = 0; t < ns; ++t) qv[t] = t;
            for (int32_t k = 0; k < ns; ++k) std::swap(qv[k], qv[hpiv[c0 + k]]);
        }
        if (hipMemcpyAsync(f->pinv, pinv.data(), n * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            rc = fail(EIGSOL_E_HIP, "solve_shifted: multifrontal pivots");
    }
    if (rc == EIGSOL_OK) {
        int32_t mx = 0;
        for (int32_t b : f->lds_fwd) mx = std::max(mx, b);
        for (int32_t b : f->lds_bwd) mx = std::max(mx, b);
        for (int32_t b : f->lds_asm) mx = std::max(mx, b);
        if (f->fuse_big)
            for (int32_t b : f->lds_asm2) mx = std::max(mx, b);
        mx = std::max(mx, std::max(f->lds_flow_f, f->lds_flow_b));
        mx = std::max(mx, std::max(f->lds_sub_f, f->lds_sub_b));
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(dev::mf_fwd_kernel<S>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, mx) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(dev::mf_bwd_kernel<S>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, mx) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(dev::mf_big_asm_kernel<S>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, mx) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(dev::mf_fwd_asm_kernel<S>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, mx) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(dev::mf_fwd_height_kernel<S>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, mx) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(dev::mf_fwd_flow_kernel<S>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, mx) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(dev::mf_bwd_flow_kernel<S>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, mx) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(dev::mf_fwd_sub_kernel<S>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, mx) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(dev::mf_bwd_sub_kernel<S>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, mx) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(dev::mf_big_bwd_kernel<S>),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                *std::max_element(f->lds_bbig.begin(), f->lds_bbig.end())) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(dev::mf_big_bwd2_kernel<S>),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                *std::max_element(f->lds_bbig.begin(), f->lds_bbig.end())) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(dev::mf_bwd_big_small_kernel<S>),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                std::max(mx, *std::max_element(f->lds_bbig.begin(), f->lds_bbig.end()))) != hipSuccess)
            rc = fail(EIGSOL_E_HIP, "solve_shifted: multifrontal solve LDS");
    }
    if (rc != EIGSOL_OK) {
        mf_free(f);
        return rc;
    }
    stt.solve_bytes = fac * (double)sb + 2.0 * (double)uo * (double)sb + 6.0 * (double)n * (double)sb;
    f->st = stt;
    *out = f;
    return EIGSOL_OK;
}

// Every launch of one solve, enqueued on st (direct, or inside a stream capture)
template <class S>
static void mf_solve_enqueue(MfFactor* f, hipStream_t st, const S* b, S* out, int32_t ef, int32_t eb) {
    const int64_t n = f->n;
    S* w = static_cast<S*>(f->w);
    S* x = static_cast<S*>(f->x);
    const S* F = static_cast<const S*>(f->F);
    // one forward launch per height with large fronts (mf_fwd_height_kernel; value flags, no pairs,
    // EIGSOL_MF_FUSE_BIG=0 off): the gather leaves those fronts' pivot rows of w unsolved
    const bool hfuse = f->bigm && f->fuse_big && (f->backoff & 4) && !f->pair;
    hipLaunchKernelGGL((dev::mf_gather_kernel<S>), dim3((n + 255) / 256), dim3(256), 0, st, f->perm, b, w, n,
                       hfuse ? f->bigm : (const uint8_t*)nullptr);
    const int32_t H = (int32_t)f->hstart.size() - 2;
    S* u = static_cast<S*>(f->u);
    S* z = static_cast<S*>(f->z);
    const int flow_grid = (int)std::max<int64_t>(1, f->nflow);   // one workgroup per front, in order
    const bool ff = f->nflow && (f->flow_mode & 1), fb = f->nflow && (f->flow_mode & 2);
    // two pivot blocks per workgroup (mf_big_fwd2 / bwd2_kernel): value flags only
    const bool pair = f->pair && (f->backoff & 4);
    if (f->nsub)
        hipLaunchKernelGGL((dev::mf_fwd_sub_kernel<S>), dim3(f->nsub), dim3(256), f->lds_sub_f, st, f->fronts,
                           f->sub_ranges, f->chl, F, f->cmap, f->pinv, w, u);
    if (ff) {
        hipLaunchKernelGGL((dev::mf_fwd_flow_kernel<S>), dim3(flow_grid), dim3(256), f->lds_flow_f, st, f->fronts,
                           f->flow_f, f->nflow, f->done, ef, f->chl, F, f->cmap, f->pinv, w, u, f->err);
    }
    for (int32_t h = ff ? f->hflow : 0; h <= H; ++h) {
        const int32_t* L = f->slists + f->sstart[h];
        const int64_t nw = f->nwave[h];
        if (nw)
            hipLaunchKernelGGL((dev::mf_fwd_wave_kernel<S>), dim3((nw + 3) / 4), dim3(256), 0, st, f->fronts, L,
                               (int32_t)nw, f->chl, F, f->cmap, f->pinv, w, u);
        if (hfuse && f->nbig[h]) {
            hipLaunchKernelGGL((dev::mf_fwd_height_kernel<S>), dim3(f->nsmall[h] + f->nbig[h] + f->fcnt[h]), dim3(256),
                               std::max(f->lds_fwd[h], f->lds_asm2[h]), st, f->fronts, L + nw, (int32_t)f->nsmall[h],
                               (int32_t)f->nbig[h], f->tabf + 2 * f->foff[h], f->chl, F, (const S*)f->tinv, f->cmap,
                               f->pinv, f->perm, b, w, u, z, f->err, f->backoff, x);
            continue;
        }
        // EIGSOL_MF_FUSE_ASM=0: the small fronts and the large fronts' assembly as two launches
        const bool fuse = f->fuse_asm && f->nsmall[h] && f->nbig[h];
        if (fuse)
            hipLaunchKernelGGL((dev::mf_fwd_asm_kernel<S>), dim3(f->nsmall[h] + f->nbig[h]), dim3(256),
                               std::max(f->lds_fwd[h], f->lds_asm[h]), st, f->fronts, L + nw, f->nsmall[h], f->chl, F,
                               f->cmap, f->pinv, w, u, z, f->backoff);
        else if (f->nsmall[h])
            hipLaunchKernelGGL((dev::mf_fwd_kernel<S>), dim3(f->nsmall[h]), dim3(256), f->lds_fwd[h], st, f->fronts,
                               L + nw, f->chl, F, f->cmap, f->pinv, w, u);
        if (f->nbig[h]) {
            if (!fuse)
                hipLaunchKernelGGL((dev::mf_big_asm_kernel<S>), dim3(f->nbig[h]), dim3(256), f->lds_asm[h], st,
                                   f->fronts, L + nw + f->nsmall[h], f->chl, f->cmap, f->pinv, w, (const S*)u, z,
                                   f->backoff);
            if (pair)
                hipLaunchKernelGGL((dev::mf_big_fwd2_kernel<S>), dim3(f->fcnt2[h]), dim3(256), 0, st, f->fronts,
                                   f->tabf2 + 2 * f->foff2[h], F, (const S*)f->tinv, (const S*)z, w, u, f->err,
                                   f->backoff, x);
            else
                hipLaunchKernelGGL((dev::mf_big_fwd_kernel<S>), dim3(f->fcnt[h]), dim3(256), 0, st, f->fronts,
                                   f->tabf + 2 * f->foff[h], F, (const S*)f->tinv, z, w, u, f->flags, ef,
                                   f->err, f->backoff, x);
        }
    }
    for (int32_t h = H; h >= (fb ? f->hflow : 0); --h) {
        const int32_t* L = f->slists + f->sstart[h];
        if (f->nbig[h] && pair)
            hipLaunchKernelGGL((dev::mf_big_bwd2_kernel<S>), dim3(f->bcnt2[h]), dim3(256), f->lds_bbig[h], st,
                               f->fronts, f->tabb2 + 2 * f->boff2[h], F, (const S*)f->tinv, f->sidx, (const S*)w, x,
                               f->err, f->backoff);
        const bool fuse = f->fuse_asm && !pair && f->nbig[h] && f->nsmall[h];
        if (fuse)
            hipLaunchKernelGGL((dev::mf_bwd_big_small_kernel<S>), dim3(f->bcnt[h] + f->nsmall[h]), dim3(256),
                               std::max(f->lds_bbig[h], f->lds_bwd[h]), st, f->fronts, f->tabb + 2 * f->boff[h],
                               f->bcnt[h], L + f->nwave[h], F, (const S*)f->tinv, f->sidx, (const S*)w, x, f->flags, eb,
                               f->err, f->backoff);
        else if (f->nbig[h] && !pair)
            hipLaunchKernelGGL((dev::mf_big_bwd_kernel<S>), dim3(f->bcnt[h]), dim3(256), f->lds_bbig[h], st, f->fronts,
                               f->tabb + 2 * f->boff[h], F, (const S*)f->tinv, f->sidx, (const S*)w, x, f->flags, eb,
                               f->err, f->backoff);
        const int64_t nw = f->nwave[h];
        if (f->nsmall[h] && !fuse)
            hipLaunchKernelGGL((dev::mf_bwd_kernel<S>), dim3(f->nsmall[h]), dim3(256), f->lds_bwd[h], st, f->fronts,
                               L + nw, F, f->sidx, w, x);
        if (nw)
            hipLaunchKernelGGL((dev::mf_bwd_wave_kernel<S>), dim3((nw + 3) / 4), dim3(256), 0, st, f->fronts, L,
                               (int32_t)nw, F, f->sidx, w, x);
    }
    if (f->nsub)
        hipLaunchKernelGGL((dev::mf_bwd_sub_kernel<S>), dim3(f->nsub), dim3(256), f->lds_sub_b, st, f->fronts,
                           f->sub_ranges, F, f->sidx, (const S*)w, x);
    if (fb)
        hipLaunchKernelGGL((dev::mf_bwd_flow_kernel<S>), dim3(flow_grid), dim3(256), f->lds_flow_b, st, f->fronts,
                           f->flow_b, f->nflow, f->done, eb, f->hflow, f->fheight, F, f->sidx, (const S*)w, x, f->err);
    hipLaunchKernelGGL((dev::mf_scatter_out_kernel<S>), dim3((n + 255) / 256), dim3(256), 0, st, f->perm, x, out, n);
}

template <class S>
int mf_solve_t(MfFactor* f, const S* b, S* out) {
    hipStream_t st = f->ctx->stream;
    const int64_t n = f->n;
    if (n == 0) return EIGSOL_OK;
    const int32_t ef = ++f->epoch, eb = ++f->epoch;   // flag words: forward, then backward values
    // EIGSOL_MF_GRAPH=1 (opt-in): the ~50 dependent launches of a solve replayed as one hipGraph
    // once a (b, out) pair repeats.  Only where no launch argument changes between solves: value
    // flags (the epoch words are unused) and no flow kernels.  Measured and rejected (round 6,
    // tools/r06_mf_graph_ab.sh, 1M convection-diffusion, two A/B pairs): 1.51 ms per iteration with
    // direct launches, 2.82 / 2.86 ms replayed - the replay serialises the nodes behind more than the
    // stream's own launch gaps
    static const bool graph_on = [] {
        const char* e = std::getenv("EIGSOL_MF_GRAPH");
        return e && std::atoi(e) != 0;
    }();
    const bool ff = f->nflow && (f->flow_mode & 1), fb = f->nflow && (f->flow_mode & 2);
    bool done = false;
    if (graph_on && (f->backoff & 4) && !ff && !fb && st != nullptr) {
        MfFactor::Graph* gr = nullptr;
        for (auto& g : f->graphs)
            if (g.b == b && g.out == out) gr = &g;
        if (!gr) {
            if (f->graphs.size() >= 8) {   // keep the most recent pairs
                if (f->graphs.front().exec) (void)hipGraphExecDestroy(f->graphs.front().exec);
                f->graphs.erase(f->graphs.begin());
            }
            f->graphs.push_back({b, out, 1, nullptr});
        } else if (!gr->exec && ++gr->uses >= 2) {
            hipGraph_t g = nullptr;
            if (hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) == hipSuccess) {
                mf_solve_enqueue<S>(f, st, b, out, ef, eb);
                if (hipStreamEndCapture(st, &g) != hipSuccess || !g ||
                    hipGraphInstantiate(&gr->exec, g, nullptr, nullptr, 0) != hipSuccess)
                    gr->exec = nullptr;
                if (g) (void)hipGraphDestroy(g);
            }
            (void)hipGetLastError();   // a failed capture leaves the direct launches below
        }
        if (gr && gr->exec) {
            EIGSOL_HIP(hipGraphLaunch(gr->exec, st));
            done = true;
        }
    }
    if (!done) mf_solve_enqueue<S>(f, st, b, out, ef, eb);
    EIGSOL_HIP(hipGetLastError());
    static const bool dbg = std::getenv("EIGSOL_MF_DEBUG") != nullptr;
    if (dbg) {
        int32_t e = 0;
        EIGSOL_HIP(hipMemcpyAsync(&e, f->err, 4, hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(hipStreamSynchronize(st));
        std::fprintf(stderr, "[mf] solve epoch %d err %d nflow %d hflow %d\n", f->epoch, e, f->nflow, f->hflow);
    }
    return EIGSOL_OK;
}

const int32_t* mf_err_word(const MfFactor* f) { return f->err; }

MfHost* mf_host_new() { return new MfHost(); }
const MfStats& mf_host_stats(const MfHost* X) { return X->stt; }
void mf_host_free(MfHost* X) { delete X; }

int mf_prepare(int64_t n, const std::vector<int32_t>& rp, const std::vector<int32_t>& ci, int dtype, double free_bytes,
               MfHost* X, const std::atomic<bool>* stop) {
    if (dtype != EIGSOL_C128 && dtype != EIGSOL_F64) return EIGSOL_E_UNSUPPORTED;
    try {
        return mf_prepare_host(n, rp, ci, dtype == EIGSOL_C128, free_bytes, *X, stop);
    } catch (const std::exception&) {   // host allocation of the plan: decline
        return EIGSOL_E_UNSUPPORTED;
    }
}

int mf_create(eigsol_ctx* ctx, int dtype, MfHost* X, const void* v, MfFactor** out, double static_pivot,
              int64_t* nstatic) {
    *out = nullptr;
    if (nstatic) *nstatic = 0;
    try {
        if (dtype == EIGSOL_C128)
            return mf_create_t<cplx>(ctx, dtype, *X, static_cast<const cplx*>(v), out, static_pivot, nstatic);
        if (dtype == EIGSOL_F64)
            return mf_create_t<double>(ctx, dtype, *X, static_cast<const double*>(v), out, static_pivot, nstatic);
    } catch (const std::exception& ex) {
        return fail(EIGSOL_E_UNSUPPORTED, std::string("solve_shifted: multifrontal factor: ") + ex.what());
    }
    return EIGSOL_E_UNSUPPORTED;
}

int mf_solve(MfFactor* f, const void* b, void* x) {
    if (f->dtype == EIGSOL_C128) return mf_solve_t<cplx>(f, static_cast<const cplx*>(b), static_cast<cplx*>(x));
    return mf_solve_t<double>(f, static_cast<const double*>(b), static_cast<double*>(x));
}

}  // namespace eigsol

// Host-only analysis of the multifrontal plan (ordering + symbolic), for tests and tools: perm_out
// (n entries, new -> old) and fronts_out (4 per front: first column, pivots, struct size, parent)
// may be null; stats_out[8] = fronts, heights, max front, max pivots, factor entries, front
// entries, flops (complex scalars if is_complex), 1 if the plan is consistent.
extern "C" int eigsol_mf_analyze(int64_t n, const int32_t* rowptr, const int32_t* colidx, int32_t leaf,
                                 int32_t is_complex, int32_t* perm_out, int32_t* fronts_out, int64_t fronts_cap,
                                 double* stats_out) {
    using namespace eigsol;
    if (n < 0 || n > INT32_MAX - 1 || (n > 0 && (!rowptr || !colidx)) || !stats_out || leaf < 1 ||
        (rowptr && rowptr[0] != 0))
        return fail(EIGSOL_E_INVALID, "eigsol_mf_analyze: bad arguments");
    for (int64_t i = 0; i < n; ++i) {
        if (rowptr[i + 1] < rowptr[i]) return fail(EIGSOL_E_INVALID, "eigsol_mf_analyze: row pointers not monotone");
        for (int32_t e = rowptr[i]; e < rowptr[i + 1]; ++e)
            if (colidx[e] < 0 || colidx[e] >= n) return fail(EIGSOL_E_INVALID, "eigsol_mf_analyze: column index out of range");
    }
    try {
        std::vector<int32_t> rp(rowptr, rowptr + n + 1), ci(colidx, colidx + (n ? rowptr[n] : 0));
        MfPlan P;
        const bool ok = mf_plan(n, rp, ci, leaf, is_complex != 0, P);
        stats_out[0] = (double)P.nt;
        stats_out[1] = (double)(P.H + 1);
        stats_out[2] = (double)P.maxd;
        stats_out[3] = (double)P.maxns;
        stats_out[4] = P.fac;
        stats_out[5] = P.fe;
        stats_out[6] = P.flops;
        stats_out[7] = ok ? 1.0 : 0.0;
        if (perm_out && n) std::copy(P.perm.begin(), P.perm.end(), perm_out);
        if (fronts_out) {
            if (fronts_cap < P.nt) return fail(EIGSOL_E_INVALID, "eigsol_mf_analyze: fronts_out too small");
            for (int64_t s = 0; s < P.nt; ++s) {
                fronts_out[4 * s] = P.fr[s].c0;
                fronts_out[4 * s + 1] = P.fr[s].ns;
                fronts_out[4 * s + 2] = P.fr[s].ms;
                fronts_out[4 * s + 3] = P.fr[s].parent;
            }
        }
        return EIGSOL_OK;
    } catch (const std::exception& ex) {
        return fail(EIGSOL_E_INVALID, std::string("eigsol_mf_analyze: ") + ex.what());
    }
}

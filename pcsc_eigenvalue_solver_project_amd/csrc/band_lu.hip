// Direct sparse LU of A - sigma I for general (non-triangular) sparse matrices: reverse
// Cuthill-McKee ordering + banded partial-pivot LU on gfx950.
//
// Replaces the SparseLU branch of solve_shifted<S> (src/matrix/solve_shifted.hpp:85-117): M = A,
// M(i, i) -= sigma with a missing diagonal inserted (:96-102), a direct factorisation
// (analyzePattern + factorize, :104-106) that fails only on a zero pivot (:108-110), then a solve
// (:112-115).  SparseLU orders columns with COLAMD and factors supernodes; this path orders rows
// and columns symmetrically with RCM, which confines the LU of a PDE-like pattern to a band:
//   * B = P M P^T, kl / ku its lower / upper bandwidths; with row interchanges confined to the
//     band (LAPACK xGBTRF), L keeps kl subdiagonals and U grows to kl + ku superdiagonals;
//   * storage: every column j keeps rows [j - TOP, j + BOT], TOP = kl + ku + NB - 1,
//     BOT = kl + NB - 1 (NB = panel width; the padding lets whole panel rectangles be addressed),
//     in a "skewed" column-major array of leading dimension ldab - 1: element (i, j) lives at
//     ab0 + i + j (ldab - 1).  Every rectangle inside the window is therefore an ordinary
//     column-major block, and the blocked dense-LU building blocks (panel, interchanges, TRSM,
//     rank-NB update on the fp64 matrix cores) run on it unchanged apart from their extents;
//   * panels of NB columns: one single-workgroup kernel pivots, interchanges (inside the panel)
//     and rank-1-updates the panel's NB columns; then the panel's interchanges on the columns to
//     its right, U12 = L11^-1 A12, and A22 -= L21 U12 (rankk_mfma).  Interchanges are NOT applied
//     to earlier panels' L columns (they would leave the band), so the forward solve interleaves
//     them panel by panel, as xGBTRS does;
//   * the solve (per iteration): one workgroup, the active window of the right-hand side in an
//     LDS ring: per panel the composite interchange (precomputed on the host as (dst, src) pairs),
//     the unit-lower NB x NB triangle on one wave (solved values broadcast by v_readlane), and the
//     L21 update of the next kl rows; then per block row from the bottom the upper triangle and the
//     U12 update of the kl + ku rows above.  In iteration mode it carries the fused
//     shifted-inverse prologue/epilogue of the dense path (shift_prologue, kernels_common.hpp).
// Chosen when the RCM band fits the device and the LDS ring (kl + ku + 2 NB <= 8192 complex /
// 16384 real entries); other general patterns go to the densified LU or ILU(0) + GMRES.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "band_lu.hpp"
#include "kernels_common.hpp"
#include "mfma_rankk.hpp"

namespace eigsol {

namespace dev {

__device__ __forceinline__ double bscore(double v) { return fabs(v); }
__device__ __forceinline__ double bscore(cplx v) { return hypot(v.re, v.im); }
__device__ __forceinline__ double bscore(float v) { return fabs((double)v); }
__device__ __forceinline__ double bscore(cplxf v) { return hypot((double)v.re, (double)v.im); }

__device__ __forceinline__ double b_readlane(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), src);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ cplx b_readlane(cplx v, int src) { return cplx{b_readlane(v.re, src), b_readlane(v.im, src)}; }
__device__ __forceinline__ float b_readlane(float v, int src) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src));
}
__device__ __forceinline__ cplxf b_readlane(cplxf v, int src) { return cplxf{b_readlane(v.re, src), b_readlane(v.im, src)}; }

// Scatter of M = A - sigma I (host-built CSR, diagonal present) into the band, rows and columns
// renumbered by iperm (old -> new).
template <class S>
__global__ __launch_bounds__(256) void band_scatter_kernel(const int32_t* rp, const int32_t* ci, const S* v,
                                                           const int32_t* iperm, int64_t n, S* ab0, int64_t ld) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    const int64_t i = iperm[r];
    for (int32_t e = rp[r]; e < rp[r + 1]; ++e) {
        const int64_t j = iperm[ci[e]];
        ab0[i + j * ld] = v[e];
    }
}

// Panel [k0, k0 + kb): for each column k, pivot = first row of largest modulus in rows
// [k, min(n, k + kl + 1)) (the band holds no entry of column k below k + kl), the row interchange
// across the panel's columns, the column scaled by the pivot (skipped for a zero pivot, as Eigen's
// partial_lu_impl does; the first zero pivot is recorded), and the rank-1 update of the panel's
// remaining columns.  One workgroup; the panel lives in L2.
template <class S>
__global__ __launch_bounds__(1024) void band_panel_kernel(S* ab0, int64_t ld, int64_t n, int64_t k0, int kb,
                                                          int64_t kl, int32_t* piv, int32_t* zero_pivot) {
    __shared__ double sv[16];
    __shared__ int si[16];
    __shared__ int s_p;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t c1 = k0 + kb;
    for (int64_t k = k0; k < c1; ++k) {
        const int64_t rend = min(n, k + kl + 1);
        double best = -1.0;
        int bi = (int)k;
        for (int64_t i = k + tid; i < rend; i += 1024) {
            const double s = bscore(ab0[i + k * ld]);
            if (s > best) { best = s; bi = (int)i; }
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
            for (int w = 1; w < 16; ++w)
                if (sv[w] > b || (sv[w] == b && si[w] < p)) { b = sv[w]; p = si[w]; }
            s_p = p;
            piv[k] = p;
            if (b == 0.0 && *zero_pivot < 0) *zero_pivot = (int)k;
        }
        __syncthreads();
        const int64_t p = s_p;
        if (p != k)
            for (int64_t j = k0 + tid; j < c1; j += 1024) {
                const S t = ab0[k + j * ld];
                ab0[k + j * ld] = ab0[p + j * ld];
                ab0[p + j * ld] = t;
            }
        __syncthreads();
        const S d = ab0[k + k * ld];
        if (bscore(d) != 0.0)
            for (int64_t i = k + 1 + tid; i < rend; i += 1024) ab0[i + k * ld] = sdiv(ab0[i + k * ld], d);
        __syncthreads();
        const int64_t m = rend - k - 1, w = c1 - k - 1;
        for (int64_t e = tid; e < m * w; e += 1024) {
            const int64_t i = k + 1 + e % m, j = k + 1 + e / m;
            ab0[i + j * ld] = sub(ab0[i + j * ld], mul(ab0[i + k * ld], ab0[k + j * ld]));
        }
        __syncthreads();
    }
}

// the panel's interchanges (rows r <-> piv[r], r = k0 .. k0 + kb - 1, in order) on columns [c1, cend)
template <class S>
__global__ __launch_bounds__(256) void band_laswp_kernel(S* ab0, int64_t ld, int64_t k0, int kb, int64_t c1,
                                                         int64_t cend, const int32_t* piv) {
    const int64_t c = c1 + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= cend) return;
    S* col = ab0 + c * ld;
    for (int j = 0; j < kb; ++j) {
        const int64_t r = k0 + j, p = piv[r];
        if (p != r) {
            const S t = col[r];
            col[r] = col[p];
            col[p] = t;
        }
    }
}

// U12 = L11^-1 A12 on columns [c1, cend): L11 (unit lower kb x kb) in LDS, one thread per column
template <class S, int NB>
__global__ __launch_bounds__(256) void band_trsm_kernel(S* ab0, int64_t ld, int64_t k0, int kb, int64_t c1,
                                                        int64_t cend) {
    __shared__ S l11[NB * NB];
    for (int e = threadIdx.x; e < kb * kb; e += 256) {
        const int i = e % kb, j = e / kb;
        l11[i + j * NB] = ab0[(k0 + i) + (k0 + j) * ld];
    }
    __syncthreads();
    const int64_t c = c1 + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= cend) return;
    S* col = ab0 + c * ld + k0;
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

template <class S>
struct BandSolveArgs {
    const S* ab0;            // element (i, j) at ab0[i + j * ld]
    int64_t ld;
    int64_t n, kl, ku;       // ku: U's superdiagonals after fill (kl + ku of B)
    int32_t nb;
    int32_t ring;            // LDS ring entries (power of two)
    const int32_t* perm;     // new -> old
    const int32_t* pstart;   // per panel: [pstart[c], pstart[c + 1]) composite interchange pairs
    const int32_t* pdst;
    const int32_t* psrc;
    S* zf;                   // forward results (new numbering)
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

template <class S>
__device__ __forceinline__ S ab0_at(const BandSolveArgs<S>& a, int64_t i, int64_t j) {
    return a.ab0[i + j * a.ld];
}

// One workgroup of 1024 threads: L z = P_panels (Pb) (interleaved), U w = z, y = P^T w.
template <class S, bool kIter>
__global__ __launch_bounds__(1024) void band_solve_kernel(BandSolveArgs<S> a, int parity) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    S* ring = reinterpret_cast<S*>(lds_raw);
    __shared__ Prologue pro;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const S* xin;
    S* yout;
    double nrm = 0.0;
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
    const int64_t n = a.n, kl = a.kl, ub = a.ku, ld = a.ld;
    const int NB = a.nb;
    const int64_t mask = a.ring - 1;
    auto rhs = [&](int64_t i) -> S {
        S v = xin[a.perm[i]];
        if constexpr (kIter) v = scale_in(v, nrm);
        return v;
    };
    // ---- forward: rows [k0, k0 + 2 NB + kl) live in the ring while panel k0 is processed
    for (int64_t i = tid; i < min(n, (int64_t)NB + kl); i += 1024) ring[i & mask] = rhs(i);
    __syncthreads();
    int c = 0;
    for (int64_t k0 = 0; k0 < n; k0 += NB, ++c) {
        const int kb = (int)min<int64_t>(NB, n - k0);
        const int64_t c1 = k0 + kb;
        const int p0 = a.pstart[c], m = a.pstart[c + 1] - p0;
        S sv = s_zero<S>();
        int dst = 0;
        if (tid < m) {
            dst = a.pdst[p0 + tid];
            sv = ring[a.psrc[p0 + tid] & mask];
        }
        __syncthreads();
        if (tid < m) ring[dst & mask] = sv;
        __syncthreads();
        if (wv == 0) {
            S v = lane < kb ? ring[(k0 + lane) & mask] : s_zero<S>();
            const int64_t row = k0 + min(lane, kb - 1);
            for (int j0 = 0; j0 < kb; j0 += 16) {
                S lv[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) lv[u] = ab0_at(a, row, k0 + min(j0 + u, kb - 1));
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int j = j0 + u;
                    if (j < kb) {
                        const S zj = b_readlane(v, j);
                        if (lane > j) v = sub(v, mul(lv[u], zj));
                    }
                }
            }
            if (lane < kb) {
                ring[(k0 + lane) & mask] = v;
                a.zf[k0 + lane] = v;
            }
        }
        __syncthreads();
        const int64_t rend = min(n, c1 + kl);
        for (int64_t r = c1 + tid; r < rend; r += 1024) {
            S acc = s_zero<S>();
            const S* lrow = a.ab0 + r + k0 * ld;
            for (int j0 = 0; j0 < kb; j0 += 16) {
                S lv[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) lv[u] = lrow[(int64_t)min(j0 + u, kb - 1) * ld];
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (j0 + u < kb) acc = add(acc, mul(lv[u], ring[(k0 + j0 + u) & mask]));
            }
            ring[r & mask] = sub(ring[r & mask], acc);
        }
        for (int64_t i = k0 + NB + kl + tid; i < min(n, k0 + 2 * NB + kl); i += 1024) ring[i & mask] = rhs(i);
        __syncthreads();
    }
    // ---- backward: block rows from the bottom; rows [r0 - NB - ub, r1) live in the ring
    const int64_t nblk = (n + NB - 1) / NB;
    {
        const int64_t r0 = (nblk - 1) * NB;
        for (int64_t i = max<int64_t>(0, r0 - ub) + tid; i < n; i += 1024) ring[i & mask] = a.zf[i];
    }
    __syncthreads();
    double n2 = 0.0, pr = 0.0, pi = 0.0;
    for (int64_t b = nblk - 1; b >= 0; --b) {
        const int64_t r0 = b * NB;
        const int rb = (int)min<int64_t>(NB, n - r0);
        if (wv == 0) {
            S v = lane < rb ? ring[(r0 + lane) & mask] : s_zero<S>();
            const int64_t row = r0 + min(lane, rb - 1);
            for (int j1 = rb; j1 > 0; j1 -= 16) {
                S uv[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) uv[u] = ab0_at(a, row, r0 + max(j1 - 1 - u, 0));
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int j = j1 - 1 - u;
                    if (j >= 0) {
                        if (lane == j) v = sdiv(v, uv[u]);
                        const S wj = b_readlane(v, j);
                        if (lane < j) v = sub(v, mul(uv[u], wj));
                    }
                }
            }
            if (lane < rb) {
                ring[(r0 + lane) & mask] = v;
                const int32_t o = a.perm[r0 + lane];
                yout[o] = v;
                if constexpr (kIter) {
                    const S xi = scale_in(xin[o], nrm);
                    n2 += sq_abs(v);
                    acc_dot(pr, pi, xi, v);
                }
            }
        }
        __syncthreads();
        const int64_t rbeg = max<int64_t>(0, r0 - ub);
        for (int64_t r = rbeg + tid; r < r0; r += 1024) {
            S acc = s_zero<S>();
            const S* urow = a.ab0 + r + r0 * ld;
            for (int j0 = 0; j0 < rb; j0 += 16) {
                S lv[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) lv[u] = urow[(int64_t)min(j0 + u, rb - 1) * ld];
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (j0 + u < rb) acc = add(acc, mul(lv[u], ring[(r0 + j0 + u) & mask]));
            }
            ring[r & mask] = sub(ring[r & mask], acc);
        }
        for (int64_t i = max<int64_t>(0, r0 - NB - ub) + tid; i < rbeg; i += 1024) ring[i & mask] = a.zf[i];
        __syncthreads();
    }
    if constexpr (kIter) {
        if (wv == 0) {
            n2 = wave_sum(n2);
            pr = wave_sum(pr);
            pi = wave_sum(pi);
            if (lane == 0) {
                a.my_part->a = n2;
                a.my_part->b = pr;
                a.my_part->c = pi;
                a.my_part->d = 0.0;
            }
        }
    }
}

}  // namespace dev

// ================================================================== host side
struct BandFactor {
    eigsol_ctx* ctx = nullptr;
    int dtype = EIGSOL_F64;
    int64_t n = 0, kl = 0, ku = 0;
    int nb = 64;
    int64_t ldab = 0, top = 0;
    void* ab = nullptr;
    int32_t* perm = nullptr;
    int32_t* pstart = nullptr;
    int32_t* pdst = nullptr;
    int32_t* psrc = nullptr;
    void* zf = nullptr;
    int32_t ring = 0;
    double sig_re = 0.0, sig_im = 0.0;
};

void band_free(BandFactor* f) {
    if (!f) return;
    hipSetDevice(f->ctx->device);
    hipStreamSynchronize(f->ctx->stream);
    for (void* p : {f->ab, (void*)f->perm, (void*)f->pstart, (void*)f->pdst, (void*)f->psrc, f->zf})
        if (p) hipFree(p);
    ctx_release(f->ctx);
    delete f;
}

// Reverse Cuthill-McKee on the pattern of M + M^T (diagonal ignored): per connected component a
// pseudo-peripheral root (George-Liu: repeated BFS from a minimum-degree node of the last level
// while the eccentricity grows), breadth-first numbering with each node's unnumbered neighbours
// in increasing degree, and the whole order reversed.
static void rcm_order(int64_t n, const int32_t* rp, const int32_t* ci, std::vector<int32_t>& order) {
    std::vector<int64_t> deg(n + 1, 0);
    for (int64_t i = 0; i < n; ++i)
        for (int32_t e = rp[i]; e < rp[i + 1]; ++e)
            if (ci[e] != i) { ++deg[i + 1]; ++deg[ci[e] + 1]; }
    std::vector<int64_t> arp(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) arp[i + 1] = arp[i] + deg[i + 1];
    std::vector<int32_t> adj(arp[n]);
    {
        std::vector<int64_t> fill(arp.begin(), arp.end() - 1);
        for (int64_t i = 0; i < n; ++i)
            for (int32_t e = rp[i]; e < rp[i + 1]; ++e)
                if (ci[e] != i) { adj[fill[i]++] = ci[e]; adj[fill[ci[e]]++] = (int32_t)i; }
    }
    std::vector<int32_t> dg(n);
    std::vector<int64_t> arp2(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) {   // sort + unique each list in place, compacted
        auto b = adj.begin() + arp[i], e = adj.begin() + arp[i + 1];
        std::sort(b, e);
        const int64_t u = std::unique(b, e) - b;
        std::copy(b, b + u, adj.begin() + arp2[i]);
        arp2[i + 1] = arp2[i] + u;
        dg[i] = (int32_t)u;
    }
    // nodes by ascending degree (counting sort, stable)
    int32_t maxd = 0;
    for (int64_t i = 0; i < n; ++i) maxd = std::max(maxd, dg[i]);
    std::vector<int64_t> cnt(maxd + 2, 0);
    for (int64_t i = 0; i < n; ++i) ++cnt[dg[i] + 1];
    for (int32_t d = 0; d <= maxd; ++d) cnt[d + 1] += cnt[d];
    std::vector<int32_t> bydeg(n);
    for (int64_t i = 0; i < n; ++i) bydeg[cnt[dg[i]]++] = (int32_t)i;
    std::vector<char> done(n, 0);
    std::vector<int64_t> mark(n, -1);
    int64_t stamp = 0;
    std::vector<int32_t> q;
    q.reserve(n);
    order.clear();
    order.reserve(n);
    std::vector<int32_t> nb;
    for (int64_t s_ = 0; s_ < n; ++s_) {
        const int32_t s = bydeg[s_];
        if (done[s]) continue;
        int32_t root = s;
        int64_t ecc = -1;
        for (int round = 0; round < 8; ++round) {
            ++stamp;
            q.clear();
            q.push_back(root);
            mark[root] = stamp;
            size_t head = 0, lvl_begin = 0;
            int64_t depth = 0;
            while (head < q.size()) {
                const size_t lvl_end = q.size();
                lvl_begin = head;
                for (; head < lvl_end; ++head) {
                    const int32_t u = q[head];
                    for (int64_t e = arp2[u]; e < arp2[u + 1]; ++e)
                        if (mark[adj[e]] != stamp) { mark[adj[e]] = stamp; q.push_back(adj[e]); }
                }
                if (q.size() > lvl_end) ++depth;
            }
            if (depth <= ecc) break;
            ecc = depth;
            int32_t best = q[lvl_begin];
            for (size_t t = lvl_begin; t < q.size(); ++t)
                if (dg[q[t]] < dg[best]) best = q[t];
            root = best;
        }
        size_t head = order.size();
        order.push_back(root);
        done[root] = 1;
        while (head < order.size()) {
            const int32_t u = order[head++];
            nb.clear();
            for (int64_t e = arp2[u]; e < arp2[u + 1]; ++e)
                if (!done[adj[e]]) { done[adj[e]] = 1; nb.push_back(adj[e]); }
            std::sort(nb.begin(), nb.end(), [&](int32_t x, int32_t y) { return dg[x] != dg[y] ? dg[x] < dg[y] : x < y; });
            order.insert(order.end(), nb.begin(), nb.end());
        }
    }
    std::reverse(order.begin(), order.end());
}

static void bandwidths(int64_t n, const int32_t* rp, const int32_t* ci, const int32_t* iperm, int64_t& kl,
                       int64_t& ku) {
    kl = ku = 0;
    for (int64_t r = 0; r < n; ++r) {
        const int64_t i = iperm ? iperm[r] : r;
        for (int32_t e = rp[r]; e < rp[r + 1]; ++e) {
            const int64_t j = iperm ? iperm[ci[e]] : ci[e];
            kl = std::max(kl, i - j);
            ku = std::max(ku, j - i);
        }
    }
}

// Ordering and band geometry for A (host CSR, n x n).  plan.ok: the band solve's LDS ring holds
// the kl + ku + 2 NB window.
void band_plan(int dtype, int64_t n, const int32_t* rp, const int32_t* ci, BandPlan& plan) {
    const bool cx = dtype_complex(dtype);
    plan.nb = cx ? dev::RankKMax<cplx>::value : dev::RankKMax<double>::value;
    std::vector<int32_t> order;
    rcm_order(n, rp, ci, order);
    std::vector<int32_t> iperm(n);
    for (int64_t i = 0; i < n; ++i) iperm[order[i]] = (int32_t)i;
    int64_t kl = 0, ku = 0, kl0 = 0, ku0 = 0;
    bandwidths(n, rp, ci, iperm.data(), kl, ku);
    bandwidths(n, rp, ci, nullptr, kl0, ku0);
    if (2 * kl0 + ku0 <= 2 * kl + ku) {   // the given order is as narrow: keep it
        for (int64_t i = 0; i < n; ++i) order[i] = (int32_t)i;
        kl = kl0;
        ku = ku0;
    }
    plan.perm = std::move(order);
    plan.kl = kl;
    plan.ku = ku;
    const int64_t nb = plan.nb;
    plan.ldab = (kl + ku + nb - 1) + (kl + nb - 1) + 1;
    const size_t sb = scalar_bytes(dtype);
    plan.bytes = (double)n * (double)plan.ldab * (double)sb;
    const int64_t need = kl + (kl + ku) + 2 * nb;   // backward window: rows [r0 - NB - (kl + ku), r0 + NB)
    int64_t ring = 1;
    while (ring < need) ring <<= 1;
    plan.ring = (int32_t)std::min<int64_t>(ring, INT32_MAX);
    plan.ok = (double)ring * (double)sb <= 128.0 * 1024.0;
}

template <class S>
static S bh_sub(S a, S b) {
    if constexpr (is_real_v<S>) return a - b;
    else return S{a.re - b.re, a.im - b.im};
}

template <class S>
static int band_create_t(eigsol_ctx* ctx, int dtype, int64_t n, const int32_t* rp, const int32_t* ci, const S* v,
                         double sre, double sim, BandPlan& plan, BandFactor** out) {
    // M = A - sigma I gains up to n inserted diagonal entries; its row pointers are int32
    if ((int64_t)rp[n] + n > (int64_t)INT32_MAX)
        return fail(EIGSOL_E_UNSUPPORTED, "solve_shifted: A - sigma I has more than 2^31 - 1 entries (int32 storage "
                                          "index) for the band factor");
    hipStream_t st = ctx->stream;
    auto* f = new BandFactor();
    f->ctx = ctx;
    ctx_retain(ctx);
    f->dtype = dtype;
    f->n = n;
    f->kl = plan.kl;
    f->ku = plan.ku;
    f->nb = plan.nb;
    f->ldab = plan.ldab;
    f->top = plan.kl + plan.ku + plan.nb - 1;
    f->ring = plan.ring;
    f->sig_re = sre;
    f->sig_im = sim;
    constexpr int NB = dev::RankKMax<S>::value;
    const int64_t ld = f->ldab - 1;
    // M = A - sigma I (solve_shifted.hpp:96-102: coeffRef inserts a missing diagonal), host CSR
    S sig;
    if constexpr (is_real_v<S>) { (void)sim; sig = (S)sre; }
    else sig = S{(decltype(S::re))sre, (decltype(S::re))sim};
    std::vector<int32_t> mrp(n + 1, 0), mci;
    std::vector<S> mv;
    mci.reserve(rp[n] + n);
    mv.reserve(rp[n] + n);
    for (int64_t i = 0; i < n; ++i) {
        bool have = false;
        for (int32_t e = rp[i]; e < rp[i + 1]; ++e) {
            if (ci[e] == i) {
                have = true;
                mci.push_back((int32_t)i);
                mv.push_back(bh_sub(v[e], sig));
            } else {
                mci.push_back(ci[e]);
                mv.push_back(v[e]);
            }
        }
        if (!have) { mci.push_back((int32_t)i); mv.push_back(bh_sub(s_zero<S>(), sig)); }
        mrp[i + 1] = (int32_t)mci.size();
    }
    std::vector<int32_t> iperm(n);
    for (int64_t i = 0; i < n; ++i) iperm[plan.perm[i]] = (int32_t)i;
    const int64_t nnzm = (int64_t)mci.size();
    int32_t *d_rp = nullptr, *d_ci = nullptr, *d_ip = nullptr, *piv = nullptr, *zp = nullptr;
    S* d_v = nullptr;
    int rc = EIGSOL_OK;
    const size_t abytes = (size_t)n * (size_t)f->ldab * sizeof(S);
    if (hipMalloc(&f->ab, abytes) != hipSuccess || hipMalloc(&f->zf, n * sizeof(S)) != hipSuccess ||
        hipMalloc(&f->perm, n * 4) != hipSuccess || hipMalloc(&d_rp, (n + 1) * 4) != hipSuccess ||
        hipMalloc(&d_ci, nnzm * 4) != hipSuccess || hipMalloc(&d_v, nnzm * sizeof(S)) != hipSuccess ||
        hipMalloc(&d_ip, n * 4) != hipSuccess || hipMalloc(&piv, n * 4) != hipSuccess || hipMalloc(&zp, 4) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "solve_shifted: band factor buffers (" + std::to_string(abytes >> 20) + " MiB)");
    S* ab0 = rc == EIGSOL_OK ? static_cast<S*>(f->ab) + f->top : nullptr;
    std::vector<int32_t> hpiv(n);
    int32_t hzp = -1;
    if (rc == EIGSOL_OK) {
        hipMemsetAsync(f->ab, 0, abytes, st);
        hipMemsetAsync(zp, 0xff, 4, st);
        hipMemcpyAsync(d_rp, mrp.data(), (n + 1) * 4, hipMemcpyHostToDevice, st);
        hipMemcpyAsync(d_ci, mci.data(), nnzm * 4, hipMemcpyHostToDevice, st);
        hipMemcpyAsync(d_v, mv.data(), nnzm * sizeof(S), hipMemcpyHostToDevice, st);
        hipMemcpyAsync(d_ip, iperm.data(), n * 4, hipMemcpyHostToDevice, st);
        hipMemcpyAsync(f->perm, plan.perm.data(), n * 4, hipMemcpyHostToDevice, st);
        hipLaunchKernelGGL((dev::band_scatter_kernel<S>), dim3((n + 255) / 256), dim3(256), 0, st, d_rp, d_ci, d_v, d_ip,
                           n, ab0, ld);
        const int64_t kl = f->kl, ub = f->kl + f->ku;
        for (int64_t k0 = 0; k0 < n; k0 += NB) {
            const int kb = (int)std::min<int64_t>(NB, n - k0);
            const int64_t c1 = k0 + kb;
            hipLaunchKernelGGL((dev::band_panel_kernel<S>), dim3(1), dim3(1024), 0, st, ab0, ld, n, k0, kb, kl, piv, zp);
            const int64_t cend = std::min<int64_t>(n, c1 + ub);   // row c1 - 1 holds columns < c1 + kl + ku
            if (cend > c1) {
                const int64_t w = cend - c1;
                hipLaunchKernelGGL((dev::band_laswp_kernel<S>), dim3((w + 255) / 256), dim3(256), 0, st, ab0, ld, k0, kb,
                                   c1, cend, piv);
                hipLaunchKernelGGL((dev::band_trsm_kernel<S, NB>), dim3((w + 255) / 256), dim3(256), 0, st, ab0, ld, k0,
                                   kb, c1, cend);
                const int64_t m = std::min<int64_t>(n, c1 + kl) - c1;   // L21: rows <= c1 - 1 + kl
                rankk_update<S, true>(st, (int)m, (int)w, kb, -1.0, ab0 + c1 + k0 * ld, ld, ab0 + k0 + c1 * ld, ld,
                                      ab0 + c1 + c1 * ld, ld);
            }
        }
        hipMemcpyAsync(hpiv.data(), piv, n * 4, hipMemcpyDeviceToHost, st);
        hipMemcpyAsync(&hzp, zp, 4, hipMemcpyDeviceToHost, st);
        if (hipStreamSynchronize(st) != hipSuccess) rc = fail(EIGSOL_E_HIP, "solve_shifted: band factorization");
    }
    for (void* p : {(void*)d_rp, (void*)d_ci, (void*)d_v, (void*)d_ip, (void*)piv, (void*)zp})
        if (p) hipFree(p);
    // a zero pivot is SparseLU's failed factorization (solve_shifted.hpp:108-110)
    if (rc == EIGSOL_OK && hzp >= 0) rc = fail(EIGSOL_E_SOLVER, "solve_shifted: SparseLU factorization failed");
    if (rc == EIGSOL_OK) {
        // composite interchange of each panel: new[dst] = old[src] over the rows it touches
        const int64_t np = (n + NB - 1) / NB;
        std::vector<int32_t> pstart(np + 1, 0), pdst, psrc, pos, cont;
        for (int64_t c = 0; c < np; ++c) {
            const int64_t k0 = c * NB, c1 = std::min<int64_t>(n, k0 + NB);
            pos.clear();
            cont.clear();
            auto slot = [&](int32_t r) -> size_t {
                for (size_t t = 0; t < pos.size(); ++t)
                    if (pos[t] == r) return t;
                pos.push_back(r);
                cont.push_back(r);
                return pos.size() - 1;
            };
            for (int64_t k = k0; k < c1; ++k) {
                if (hpiv[k] == k) continue;
                const size_t a = slot((int32_t)k), b = slot(hpiv[k]);
                std::swap(cont[a], cont[b]);
            }
            for (size_t t = 0; t < pos.size(); ++t)
                if (cont[t] != pos[t]) { pdst.push_back(pos[t]); psrc.push_back(cont[t]); }
            pstart[c + 1] = (int32_t)pdst.size();
        }
        if (pdst.empty()) { pdst.push_back(0); psrc.push_back(0); }
        if (hipMalloc(&f->pstart, (np + 1) * 4) != hipSuccess || hipMalloc(&f->pdst, pdst.size() * 4) != hipSuccess ||
            hipMalloc(&f->psrc, psrc.size() * 4) != hipSuccess)
            rc = fail(EIGSOL_E_HIP, "solve_shifted: band interchange tables");
        if (rc == EIGSOL_OK) {
            hipMemcpyAsync(f->pstart, pstart.data(), (np + 1) * 4, hipMemcpyHostToDevice, st);
            hipMemcpyAsync(f->pdst, pdst.data(), pdst.size() * 4, hipMemcpyHostToDevice, st);
            hipMemcpyAsync(f->psrc, psrc.data(), psrc.size() * 4, hipMemcpyHostToDevice, st);
            if (hipStreamSynchronize(st) != hipSuccess) rc = fail(EIGSOL_E_HIP, "solve_shifted: band upload");
        }
    }
    if (rc != EIGSOL_OK) {
        band_free(f);
        return rc;
    }
    *out = f;
    return EIGSOL_OK;
}

int band_create(eigsol_ctx* ctx, int dtype, int64_t n, const int32_t* rp, const int32_t* ci, const void* v,
                double sre, double sim, BandPlan& plan, BandFactor** out) {
    if (dtype == EIGSOL_C128)
        return band_create_t<cplx>(ctx, dtype, n, rp, ci, static_cast<const cplx*>(v), sre, sim, plan, out);
    if (dtype == EIGSOL_F64)
        return band_create_t<double>(ctx, dtype, n, rp, ci, static_cast<const double*>(v), sre, sim, plan, out);
    if (dtype == EIGSOL_F32)   // single precision: factored and solved in float (native)
        return band_create_t<float>(ctx, dtype, n, rp, ci, static_cast<const float*>(v), sre, sim, plan, out);
    return band_create_t<cplxf>(ctx, dtype, n, rp, ci, static_cast<const cplxf*>(v), sre, sim, plan, out);
}

template <class S>
static int band_launch_t(BandFactor* f, bool iter, const void* b, void* y, void* buf0, void* buf1, PowerCtl* ctl,
                         const void* rank_part, void* my_part, void* trace, int parity) {
    dev::BandSolveArgs<S> a{};
    a.ab0 = static_cast<const S*>(f->ab) + f->top;
    a.ld = f->ldab - 1;
    a.n = f->n;
    a.kl = f->kl;
    a.ku = f->kl + f->ku;
    a.nb = f->nb;
    a.ring = f->ring;
    a.perm = f->perm;
    a.pstart = f->pstart;
    a.pdst = f->pdst;
    a.psrc = f->psrc;
    a.zf = static_cast<S*>(f->zf);
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
    const size_t lds = (size_t)f->ring * sizeof(S);
    hipStream_t st = f->ctx->stream;
    const void* k = iter ? reinterpret_cast<const void*>(dev::band_solve_kernel<S, true>)
                         : reinterpret_cast<const void*>(dev::band_solve_kernel<S, false>);
    EIGSOL_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    if (iter) hipLaunchKernelGGL((dev::band_solve_kernel<S, true>), dim3(1), dim3(1024), lds, st, a, parity);
    else hipLaunchKernelGGL((dev::band_solve_kernel<S, false>), dim3(1), dim3(1024), lds, st, a, parity);
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

int band_launch(BandFactor* f, bool iter, const void* b, void* y, void* buf0, void* buf1, PowerCtl* ctl,
                const void* rank_part, void* my_part, void* trace, int parity) {
    if (f->dtype == EIGSOL_C128)
        return band_launch_t<cplx>(f, iter, b, y, buf0, buf1, ctl, rank_part, my_part, trace, parity);
    if (f->dtype == EIGSOL_F32)
        return band_launch_t<float>(f, iter, b, y, buf0, buf1, ctl, rank_part, my_part, trace, parity);
    if (f->dtype == EIGSOL_C64)
        return band_launch_t<cplxf>(f, iter, b, y, buf0, buf1, ctl, rank_part, my_part, trace, parity);
    return band_launch_t<double>(f, iter, b, y, buf0, buf1, ctl, rank_part, my_part, trace, parity);
}

// algorithmic bytes of one solve: the stored band of L and U (kl + 1 + kl + ku entries a column)
// once, the right-hand side and the solution once
void band_info(const BandFactor* f, double* bytes, int32_t* tiles) {
    const double sb = (double)scalar_bytes(f->dtype), n = (double)f->n;
    if (bytes) *bytes = sb * n * (double)(2 * f->kl + f->ku + 1) + 2.0 * sb * n;
    if (tiles) *tiles = (int32_t)(f->kl + f->ku);
}

}  // namespace eigsol

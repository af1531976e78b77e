// General (non-triangular) sparse shifted solve without densifying: ILU(0)-preconditioned
// restarted GMRES on gfx950.
//
// Replaces the SparseLU branch of solve_shifted<S> (src/matrix/solve_shifted.hpp:85-117: copy A,
// subtract sigma on the diagonal with coeffRef inserting a missing diagonal :100-102, factor,
// solve) for matrices too large to densify.  The reference factors exactly (COLAMD + SparseLU);
// here the solve is iterative to a stated residual, with memory O(nnz + n m):
//   * M = A - sigma I is built once (diagonal inserted where missing) and uploaded as a CSR; its
//     SpMV is the library's sliced kernel;
//   * the preconditioner K is an incomplete or a complete LU of M on the device: rows in dependency
//     levels of the strict lower pattern (a level's rows only read earlier levels), one thread per
//     row in IKJ order, one launch per level.  The pattern it factors on is M's closed under fill
//     (the symbolic LU without pivoting, so the factors are M's exact LU and GMRES converges in one
//     step) when that pattern holds at most EIGSOL_LU_FILL_CAP (default 3) x nnz(M) entries;
//     otherwise M's own pattern (ILU(0)).  Over the exact LU a solve is x = U^-1 L^-1 b and its
//     true residual; GMRES cycles run only if that misses the tolerance (refinement);
//   * the factors L (unit lower) and U are solved with the sync-free level-ordered triangular
//     solve of the config-5 path (shifted.hip), i.e. K^-1 v = U^-1 (L^-1 v);
//   * GMRES(m) with right preconditioning, x0 = 0, classical Gram-Schmidt with one
//     re-orthogonalisation pass (CGS2: two multi-column dot launches and two updates per step,
//     deterministic fixed-order reductions), Givens rotations and the small least-squares solve on
//     the host (one device->host copy of the new Hessenberg column per step).
// Stopping: the Arnoldi residual estimate below rtol ||b||, confirmed by the true residual
// ||b - M x|| <= rtol_true ||b|| (1e-12) at the end of a cycle (restart otherwise).  A solve stops
// early when two cycles in a row fail to halve the true residual (stagnation).  A solve that ends
// above rtol_accept = 1e-10 (the shifted-inverse parity tolerance on lambda) reports
// EIGSOL_E_SOLVER as SparseLU's failed solve (solve_shifted.hpp:112-114); shifted.hip then falls
// back to the densified LU wherever it fits the device.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <exception>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "kernels_common.hpp"
#include "multifrontal.hpp"

namespace eigsol {

struct ShiftFactor;
int shift_factor_tri(eigsol_ctx* ctx, int dtype, int64_t n, std::vector<int32_t>& rp, std::vector<int32_t>& ci,
                     const void* vals, bool up, ShiftFactor** out);
int shift_factor_tri_dev(eigsol_ctx* ctx, int dtype, int64_t n, int32_t* rp, int32_t* ci, void* vals, int64_t nnz,
                         bool up, ShiftFactor** out);
hipError_t tri_exclusive_scan(hipStream_t st, const int32_t* in, int32_t* out, int64_t n);
int shift_solve_launch(ShiftFactor* f, const void* b_dev, void* y_dev);
int shift_error(ShiftFactor* f);
void shift_factor_free(ShiftFactor* f);
void shift_info(const ShiftFactor* f, double* bytes, int32_t* variant, int32_t* tiles);
int csr_upload(eigsol_ctx* ctx, int dtype, int64_t nrows, int64_t ncols, int64_t nnz, const int32_t* rowptr,
               const int32_t* colidx, const void* values, eigsol_csr** out, int64_t xoff);

namespace dev {

// ILU(0), IKJ form, one thread per row of one level: for each stored k < i (ascending),
// l_ik = a_ik / u_kk, then a_ij -= l_ik u_kj for every stored j > k of row i that row k also stores
// (merge of the two ascending column lists).  Rows of a level only read rows of earlier levels.
template <class S>
__global__ __launch_bounds__(256) void ilu0_level_kernel(const int32_t* rp, const int32_t* ci, const int32_t* dpos,
                                                         S* val, const int32_t* rows, int32_t nrows, int32_t* zpiv) {
    const int32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= nrows) return;
    const int32_t i = rows[t];
    const int32_t e1 = rp[i + 1], di = dpos[i];
    for (int32_t e = rp[i]; e < di; ++e) {
        const int32_t k = ci[e];
        const S lik = sdiv(val[e], val[dpos[k]]);
        val[e] = lik;
        int32_t p = dpos[k] + 1;
        const int32_t pk = rp[k + 1];
        for (int32_t e2 = e + 1; e2 < e1; ++e2) {
            const int32_t j = ci[e2];
            while (p < pk && ci[p] < j) ++p;
            if (p < pk && ci[p] == j) val[e2] = sub(val[e2], mul(lik, val[p]));
        }
    }
    const S d = val[di];
    bool z;
    if constexpr (std::is_same_v<S, double>) z = d == 0.0;
    else z = d.re == 0.0 && d.im == 0.0;
    if (z) atomicOr(zpiv, 1);
}

// L / U split of the factored pattern: row counts (lcnt[n] = ucnt[n] = 0 for the exclusive scan)
__global__ __launch_bounds__(256) void gm_split_count_kernel(const int32_t* rp, const int32_t* dpos, int64_t n,
                                                             int32_t* lcnt, int32_t* ucnt) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        lcnt[i] = dpos[i] - rp[i] + 1;
        ucnt[i] = rp[i + 1] - dpos[i];
    } else if (i == n) {
        lcnt[n] = 0;
        ucnt[n] = 0;
    }
}

template <class S>
__global__ __launch_bounds__(256) void gm_split_fill_kernel(const int32_t* rp, const int32_t* ci, const S* v,
                                                            const int32_t* dpos, int64_t n, const int32_t* lrp,
                                                            const int32_t* urp, int32_t* lci, S* lv, int32_t* uci,
                                                            S* uv) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    int32_t o = lrp[i];
    for (int32_t e = rp[i]; e < dpos[i]; ++e, ++o) {
        lci[o] = ci[e];
        lv[o] = v[e];
    }
    lci[o] = (int32_t)i;
    S one;
    set_re_im(one, 1.0, 0.0);
    lv[o] = one;
    o = urp[i];
    for (int32_t e = dpos[i]; e < rp[i + 1]; ++e, ++o) {
        uci[o] = ci[e];
        uv[o] = v[e];
    }
}

// part[(blk * k + c) * 2 + {0, 1}] = block partial of sum_i conj(V(i, c)) w(i)
template <class S>
__global__ __launch_bounds__(kThreads) void gm_dots_kernel(const S* V, int64_t ldv, int k, const S* w, int64_t n,
                                                           double* part) {
    __shared__ double sm[3 * kWaves];
    const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
    const int64_t i0 = (int64_t)blockIdx.x * chunk, i1 = std::min<int64_t>(n, i0 + chunk);
    for (int c = 0; c < k; ++c) {
        const S* v = V + (int64_t)c * ldv;
        double rr = 0.0, ri = 0.0, dummy = 0.0;
        for (int64_t i = i0 + threadIdx.x; i < i1; i += kThreads) acc_dot(rr, ri, v[i], w[i]);
        block_sum3(rr, ri, dummy, sm);
        if (threadIdx.x == 0) {
            part[((int64_t)blockIdx.x * k + c) * 2] = rr;
            part[((int64_t)blockIdx.x * k + c) * 2 + 1] = ri;
        }
    }
}

// out[c] = sum of the G block partials (one workgroup per column c; thread t sums blocks t, t + 256,
// ... in order, then a fixed-order block reduction: deterministic for a given G).  Round 2's
// one-wave version summed the G = 489 partials of a 1M vector one after another per lane:
// 64 us per call, 14 % of a GMRES iteration.
__global__ __launch_bounds__(kThreads) void gm_reduce_kernel(const double* part, int G, int k, double* out) {
    __shared__ double sm[3 * kWaves];
    const int c = blockIdx.x;
    double rr = 0.0, ri = 0.0, dummy = 0.0;
    for (int b = threadIdx.x; b < G; b += kThreads) {
        rr += part[((int64_t)b * k + c) * 2];
        ri += part[((int64_t)b * k + c) * 2 + 1];
    }
    block_sum3(rr, ri, dummy, sm);
    if (threadIdx.x == 0) {
        out[2 * c] = rr;
        out[2 * c + 1] = ri;
    }
}

template <class S>
__device__ __forceinline__ S from_re_im(double re, double im) {
    if constexpr (std::is_same_v<S, double>) { (void)im; return re; }
    else return S{re, im};
}

// The checked direct solve's epilogue in one pass: r = b / bdiv - M x with M x = t (M uploaded) or
// t - sigma x (t = A x on the caller's matrix), and the block partials of ||r||^2 and ||x||^2 in
// gm_dots_kernel's layout for k = 2 (the same chunks and per-thread order: the sums are bitwise
// those of the separate shift / residual / two dot passes it replaces)
template <class S>
__global__ __launch_bounds__(kThreads) void gm_resid_norms_kernel(const S* b, double bdiv, const S* t, const S* x,
                                                                  double sre, double sim, int shift, S* r, int64_t n,
                                                                  double* part) {
    __shared__ double sm[3 * kWaves];
    const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
    const int64_t i0 = (int64_t)blockIdx.x * chunk, i1 = std::min<int64_t>(n, i0 + chunk);
    const S sig = from_re_im<S>(sre, sim);
    double rr = 0.0, ri = 0.0, xr = 0.0, xi = 0.0, dummy = 0.0;
    for (int64_t i = i0 + threadIdx.x; i < i1; i += kThreads) {
        const S xv = x[i];
        const S mx = shift ? sub(t[i], mul(sig, xv)) : t[i];
        const S rv = sub(scale_in(b[i], bdiv), mx);
        r[i] = rv;
        acc_dot(rr, ri, rv, rv);
        acc_dot(xr, xi, xv, xv);
    }
    block_sum3(rr, ri, dummy, sm);
    if (threadIdx.x == 0) {
        part[((int64_t)blockIdx.x * 2) * 2] = rr;
        part[((int64_t)blockIdx.x * 2) * 2 + 1] = ri;
    }
    dummy = 0.0;
    block_sum3(xr, xi, dummy, sm);
    if (threadIdx.x == 0) {
        part[((int64_t)blockIdx.x * 2 + 1) * 2] = xr;
        part[((int64_t)blockIdx.x * 2 + 1) * 2 + 1] = xi;
    }
}

// mode 0: w -= V(:, 0:k) h;  mode 1: w = V(:, 0:k) h   (h: k (re, im) pairs on the device)
template <class S>
__global__ __launch_bounds__(kThreads) void gm_combine_kernel(const S* V, int64_t ldv, int k, const double* h, S* w,
                                                              int64_t n, int mode) {
    __shared__ double hs[2 * 64];
    for (int c = threadIdx.x; c < 2 * k; c += kThreads) hs[c] = h[c];
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
        S acc = s_zero<S>();
        for (int c = 0; c < k; ++c) acc = add(acc, mul(V[(int64_t)c * ldv + i], from_re_im<S>(hs[2 * c], hs[2 * c + 1])));
        w[i] = mode ? acc : sub(w[i], acc);
    }
}

// dst = src / d  (d > 0)
template <class S>
__global__ __launch_bounds__(kThreads) void gm_div_kernel(const S* src, double d, S* dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads)
        dst[i] = divr(src[i], d);
}

// r = b / bdiv - Mx   (bdiv == 0: b unscaled; Mx == nullptr: zero)
template <class S>
__global__ __launch_bounds__(kThreads) void gm_resid_kernel(const S* b, double bdiv, const S* Mx, S* r, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
        const S bi = scale_in(b[i], bdiv);
        r[i] = Mx ? sub(bi, Mx[i]) : bi;
    }
}

// dst = src * (g_re + i g_im)   (real S: g_im ignored)
template <class S>
__global__ __launch_bounds__(kThreads) void gm_cscale_kernel(const S* src, double gre, double gim, S* dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads)
        dst[i] = mul(src[i], from_re_im<S>(gre, gim));
}

// y -= sigma x: M x = A x - sigma x on the caller's matrix A
template <class S>
__global__ __launch_bounds__(kThreads) void gm_shift_sub_kernel(const S* x, double sre, double sim, S* y, int64_t n) {
    const S sig = from_re_im<S>(sre, sim);
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads)
        y[i] = sub(y[i], mul(sig, x[i]));
}

template <class S>
__global__ __launch_bounds__(kThreads) void gm_axpy_kernel(S* x, const S* t, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads)
        x[i] = add(x[i], t[i]);
}

}  // namespace dev

struct GmresSolver {
    eigsol_ctx* ctx = nullptr;
    int dtype = EIGSOL_F64;
    int64_t n = 0;
    int m = 40;                 // Krylov dimension per cycle (EIGSOL_GMRES_M)
    int max_cycles = 30;
    double rtol = 1e-13;        // Arnoldi estimate target (EIGSOL_GMRES_RTOL)
    double rtol_true = 1e-12;   // true residual accepted at the end of a cycle
    double rtol_accept = 1e-10; // worst final residual reported as a success (EIGSOL_GMRES_ACCEPT)
    double normM = 0.0;         // max(||M||_1, ||M||_inf): the backward-error scale of a direct solve
    double be_accept = 1e-14;   // a direct solve whose normwise backward error is below this is accepted
    int64_t mf_static = 0;      // static pivots of the multifrontal factor (its zero-pivot retry)
    eigsol_csr* M = nullptr;    // M = A - sigma I uploaded (single-precision A only), else
    eigsol_csr* A = nullptr;    // the caller's device matrix: M x = A x - sigma x (no second copy of M)
    double sre = 0.0, sim = 0.0;
    ShiftFactor* L = nullptr;
    ShiftFactor* U = nullptr;
    void* V = nullptr;          // n x (m + 1), column-major
    void* Z = nullptr;          // n x m: K^-1 v_j of every Arnoldi step (flexible GMRES: no final preconditioner)
    void* t1 = nullptr;
    void* w = nullptr;
    void* x = nullptr;
    double* part = nullptr;
    double* hdev = nullptr;
    double* hpin = nullptr;     // pinned host mirror of hdev: a pageable copy costs a sleeping wait (~1 ms)
    int G = 1;
    int64_t nnzM = 0;
    int last_steps = 0;
    int complete = 0;           // 1: K is M's exact LU (complete fill), 2: the multifrontal LU, 0: ILU(0)
    MfFactor* mf = nullptr;     // complete == 2 (multifrontal.hip)
    int64_t nnzK = 0;           // entries of the factored pattern
    double last_bytes = 0.0;
    double last_relres = 0.0;
    bool lag_pending = false;   // a lagged direct solve whose check (lagpin) is still to be read
    int64_t lag_off() const { return 4 * (int64_t)m + 6; }   // its slot in hpin, past the cycles' use
};

void gmres_free(GmresSolver* g) {
    if (!g) return;
    hipSetDevice(g->ctx->device);
    hipStreamSynchronize(g->ctx->stream);
    if (g->L) shift_factor_free(g->L);
    if (g->U) shift_factor_free(g->U);
    if (g->mf) mf_free(g->mf);
    if (g->M) csr_release(g->M);
    if (g->A) csr_release(g->A);
    for (void* p : {g->V, g->Z, g->t1, g->w, g->x, (void*)g->part, (void*)g->hdev})
        if (p) hipFree(p);
    if (g->hpin) hipHostFree(g->hpin);
    ctx_release(g->ctx);
    delete g;
}

template <class S>
static S h_sub(S a, S b) {
    if constexpr (std::is_same_v<S, double>) return a - b;
    else return S{a.re - b.re, a.im - b.im};
}

// Symbolic LU of the pattern (rp, ci) without pivoting, up-looking: row i's pattern is its own
// columns plus, for every k < i in it (ascending, fill included), row k's columns past k.  Rows are
// sorted, the diagonal present.  Returns false (and stops early) once the pattern would exceed cap
// entries.
static bool lu_fill_pattern(int64_t n, const std::vector<int32_t>& rp, const std::vector<int32_t>& ci, int64_t cap,
                            std::vector<int32_t>& frp, std::vector<int32_t>& fci, std::vector<int32_t>& fdpos,
                            const std::atomic<bool>* stop = nullptr) {
    frp.assign(n + 1, 0);
    fci.clear();
    fdpos.assign(n, 0);
    std::vector<int32_t> mark(n, -1), lcols, ucols, heap;
    auto cmp = [](int32_t a, int32_t b) { return a > b; };   // min-heap
    for (int64_t i = 0; i < n; ++i) {
        if (stop && (i & 1023) == 0 && stop->load(std::memory_order_relaxed)) return false;
        lcols.clear();
        ucols.clear();
        heap.clear();
        for (int32_t e = rp[i]; e < rp[i + 1]; ++e) {
            const int32_t c = ci[e];
            mark[c] = (int32_t)i;
            if (c < i) heap.push_back(c);
            else ucols.push_back(c);
        }
        std::make_heap(heap.begin(), heap.end(), cmp);
        while (!heap.empty()) {
            std::pop_heap(heap.begin(), heap.end(), cmp);
            const int32_t k = heap.back();
            heap.pop_back();
            lcols.push_back(k);
            for (int32_t e = fdpos[k] + 1; e < frp[k + 1]; ++e) {
                const int32_t j = fci[e];
                if (mark[j] == (int32_t)i) continue;
                mark[j] = (int32_t)i;
                if (j < i) {
                    heap.push_back(j);
                    std::push_heap(heap.begin(), heap.end(), cmp);
                } else {
                    ucols.push_back(j);
                }
            }
            if ((int64_t)fci.size() + (int64_t)lcols.size() + (int64_t)ucols.size() + (int64_t)heap.size() > cap)
                return false;
        }
        std::sort(ucols.begin(), ucols.end());
        fdpos[i] = (int32_t)(fci.size() + lcols.size());
        fci.insert(fci.end(), lcols.begin(), lcols.end());
        fci.insert(fci.end(), ucols.begin(), ucols.end());
        if ((int64_t)fci.size() > cap) return false;
        frp[i + 1] = (int32_t)fci.size();
    }
    return true;
}

template <class S>
static int gmres_create_t(eigsol_ctx* ctx, int dtype, int64_t n, const int32_t* rp, const int32_t* ci, const S* v,
                          double sre, double sim, eigsol_csr* Adev, GmresSolver** out) {
    hipStream_t st = ctx->stream;
    static const bool dbg = std::getenv("EIGSOL_MF_DEBUG") != nullptr;
    auto tp = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!dbg) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[gmres] %s %.3f s\n", what, std::chrono::duration<double>(t - tp).count());
        tp = t;
    };
    auto* g = new GmresSolver();
    g->ctx = ctx;
    ctx_retain(ctx);
    g->dtype = dtype;
    g->n = n;
    if (const char* e = std::getenv("EIGSOL_GMRES_M")) g->m = std::max(2, std::min(60, std::atoi(e)));
    if (const char* e = std::getenv("EIGSOL_GMRES_RTOL")) g->rtol = std::atof(e);
    if (const char* e = std::getenv("EIGSOL_GMRES_ACCEPT")) g->rtol_accept = std::atof(e);
    if (const char* e = std::getenv("EIGSOL_DIRECT_BE_ACCEPT")) g->be_accept = std::atof(e);
    // M = A - sigma I, diagonal inserted where A stores none (solve_shifted.hpp:100-102)
    S sig;
    if constexpr (std::is_same_v<S, double>) { (void)sim; sig = sre; }
    else sig = S{sre, sim};
    // built on the host threads (rows in contiguous chunks): the same arrays and row sums as a serial
    // pass; the column sums are formed per row chunk and then added chunk by chunk, so ||M||_1 can
    // differ from a serial sum in its last bits (it only scales the direct solve's acceptance test).
    // 1M general-sparse matrix: 0.28 -> 0.10 s (round 6, tools/r06_buildM_ab.py: solutions bitwise
    // the serial build's)
    std::vector<int32_t> mrp(n + 1, 0), mci, dpos(n);
    std::vector<S> mv;
    const int nth = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    auto par = [&](int64_t cnt, auto fn) {   // fn(t, begin, end) over nth contiguous chunks
        const int T = cnt < 65536 ? 1 : nth;
        const int64_t ch = (cnt + T - 1) / T;
        std::vector<std::thread> th;
        int t = 1;
        try {
            for (; t < T; ++t) th.emplace_back(fn, t, std::min(cnt, t * ch), std::min(cnt, (t + 1) * ch));
        } catch (const std::exception&) {
        }
        for (int r = t; r < T; ++r) fn(r, std::min(cnt, r * ch), std::min(cnt, (r + 1) * ch));
        fn(0, (int64_t)0, std::min(cnt, ch));
        for (auto& x : th) x.join();
        return T;
    };
    par(n, [&](int, int64_t b, int64_t e) {   // row lengths of M: a missing diagonal is inserted
        for (int64_t r = b; r < e; ++r) {
            bool has = false;
            for (int32_t q = rp[r]; q < rp[r + 1]; ++q) has = has || ci[q] == r;
            mrp[r + 1] = rp[r + 1] - rp[r] + (has ? 0 : 1);
        }
    });
    for (int64_t r = 0; r < n; ++r) mrp[r + 1] += mrp[r];
    g->nnzM = mrp[n];
    mci.resize(g->nnzM);
    mv.resize(g->nnzM);
    std::unique_ptr<double[]> am(new double[g->nnzM]);    // |m_e|
    std::vector<double> rmaxs(nth, 0.0);
    par(n, [&](int t, int64_t b, int64_t e) {
        double rmax = 0.0;
        for (int64_t i = b; i < e; ++i) {
            int32_t o = mrp[i];
            bool have = false;
            auto put = [&](int32_t c, S val) {
                mci[o] = c;
                mv[o] = val;
                if constexpr (std::is_same_v<S, double>) am[o] = std::fabs(val);
                else am[o] = std::hypot(val.re, val.im);
                ++o;
            };
            for (int32_t q = rp[i]; q <= rp[i + 1]; ++q) {
                const bool end = q == rp[i + 1];
                if (!have && (end || ci[q] > i)) {   // diagonal slot before the first column past i
                    dpos[i] = o;
                    put((int32_t)i, h_sub(s_zero<S>(), sig));
                    have = true;
                }
                if (end) break;
                if (ci[q] == i) {
                    dpos[i] = o;
                    put((int32_t)i, h_sub(v[q], sig));
                    have = true;
                } else {
                    put(ci[q], v[q]);
                }
            }
            double rs = 0.0;
            for (int32_t q = mrp[i]; q < mrp[i + 1]; ++q) rs += am[q];
            rmax = std::max(rmax, rs);
        }
        rmaxs[t] = rmax;
    });
    {
        // column sums: each thread sums its row chunk into its own column array, the arrays are then
        // added column by column in thread order (at most 512 MB of them)
        const int T = (int)std::max<int64_t>(1, std::min<int64_t>(n < 65536 ? 1 : nth, ((int64_t)1 << 29) / (8 * std::max<int64_t>(n, 1))));
        std::vector<std::vector<double>> cs(T);
        const int64_t rch = (n + T - 1) / T;
        auto rows = [&](int t) {
            cs[t].assign(n, 0.0);
            const int64_t b = std::min<int64_t>(n, t * rch), e = std::min<int64_t>(n, (t + 1) * rch);
            for (int64_t q = mrp[b]; q < mrp[e]; ++q) cs[t][mci[q]] += am[q];
        };
        std::vector<double> cmaxs(T, 0.0);
        const int64_t cw = (n + T - 1) / T;
        auto cols = [&](int t) {
            const int64_t lo = std::min<int64_t>(n, t * cw), hi = std::min<int64_t>(n, (t + 1) * cw);
            double m = 0.0;
            for (int64_t c = lo; c < hi; ++c) {
                double sum = 0.0;
                for (int u = 0; u < T; ++u) sum += cs[u][c];
                m = std::max(m, sum);
            }
            cmaxs[t] = m;
        };
        auto run = [&](auto& fn) {
            std::vector<std::thread> th;
            int t = 1;
            try {
                for (; t < T; ++t) th.emplace_back([&fn, t] { fn(t); });
            } catch (const std::exception&) {
            }
            for (int r = t; r < T; ++r) fn(r);
            fn(0);
            for (auto& x : th) x.join();
        };
        run(rows);
        run(cols);
        g->normM = 0.0;
        for (double r : rmaxs) g->normM = std::max(g->normM, r);
        for (double c : cmaxs) g->normM = std::max(g->normM, c);
    }
    lap("build M");
    // products with M: on the caller's device matrix A when it is given (M x = A x - sigma x; round
    // 5: the host layout build and pageable upload of a second copy took 0.19 s of the 1M set-up)
    int rc = EIGSOL_OK;
    g->sre = sre;
    g->sim = sim;
    if (Adev) {
        g->A = Adev;
        csr_retain(Adev);
    } else {
        rc = csr_upload(ctx, dtype, n, n, g->nnzM, mrp.data(), mci.data(), mv.data(), &g->M, 0);
    }
    lap("upload M");
    // complete fill where affordable: M's values on the closed pattern, zeros at the fill
    // positions; the factorization below then produces the exact LU (round 4: the 1M config-5
    // matrix made general fills 16.5M -> ~24M entries and GMRES needs one step per solve instead of
    // 7-10 over ILU(0)).  M's own pattern is kept aside: the exact LU without pivoting meets a zero
    // pivot whenever a leading minor of M is singular, where ILU(0)'s (dropped-fill) pivots may all
    // be nonzero, so that case retries ILU(0) before reporting SparseLU's failure
    //
    // The multifrontal plan (host only: nested dissection, symbolic structure, tables) runs on a
    // second host thread beside the fill attempt; it is used where the fill passes the cap and is
    // abandoned (stop flag) where the exact LU wins.  EIGSOL_MF=0 skips it; a fill cap below 1
    // (ILU(0) forced) skips both.
    std::vector<int32_t> orp, oci, odpos;
    std::vector<S> ov;
    double ratio = 3.0;
    if (const char* e = std::getenv("EIGSOL_LU_FILL_CAP")) ratio = std::atof(e);
    MfHost* mfh = nullptr;
    int mf_prc = EIGSOL_E_UNSUPPORTED;
    std::atomic<bool> mf_stop{false}, fill_stop{false};
    std::thread mft;
    // joins the plan thread on every way out of this scope (an exception from the fill attempt
    // included: a joinable std::thread must never be destroyed)
    struct PlanJoin {
        std::thread& t;
        std::atomic<bool>& stop;
        ~PlanJoin() {
            if (t.joinable()) {
                stop.store(true);
                t.join();
            }
        }
    } plan_join{mft, mf_stop};
    size_t fb = 0;
    {
        const char* me = std::getenv("EIGSOL_MF");
        size_t tb = 0;
        if (rc == EIGSOL_OK && ratio >= 1.0 && !(me && !std::strcmp(me, "0"))) {
            if (hipMemGetInfo(&fb, &tb) == hipSuccess) {
                mfh = mf_host_new();
                try {
                    // a plan whose fronts store more than 6 x nnz(M) is a mesh-like pattern: the
                    // natural-order fill (capped at 3 x nnz) is then all but certain to pass its cap,
                    // so the attempt is cut short
                    mft = std::thread([&] {
                        mf_prc = mf_prepare(n, mrp, mci, dtype, (double)fb, mfh, &mf_stop);
                        if (mf_prc == EIGSOL_OK && mf_host_stats(mfh).factor_entries > 6.0 * (double)g->nnzM)
                            fill_stop.store(true);
                    });
                } catch (const std::exception&) {   // no thread: plan on this one after the fill attempt
                    mf_prc = -1;
                }
            }
        }
    }
    {
        std::vector<int32_t> frp, fci, fdpos;
        const bool filled = ratio >= 1.0 && lu_fill_pattern(n, mrp, mci,
                                                            std::min<int64_t>(INT32_MAX - 1, (int64_t)(ratio * (double)g->nnzM)),
                                                            frp, fci, fdpos, &fill_stop);
        lap("exact-LU fill attempt");
        if (filled) mf_stop.store(true);
        if (mft.joinable()) mft.join();
        if (mf_prc == -1 && !filled) mf_prc = mf_prepare(n, mrp, mci, dtype, (double)fb, mfh);
        lap("multifrontal plan (joined)");
        if (filled) {
            std::vector<S> fv(fci.size(), s_zero<S>());
            for (int64_t i = 0; i < n; ++i) {   // both rows sorted: merge M's entries into the pattern
                int32_t p = frp[i];
                for (int32_t e = mrp[i]; e < mrp[i + 1]; ++e) {
                    while (fci[p] < mci[e]) ++p;
                    fv[p] = mv[e];
                }
            }
            mrp.swap(frp);
            mci.swap(fci);
            mv.swap(fv);
            dpos.swap(fdpos);
            orp.swap(frp);
            oci.swap(fci);
            ov.swap(fv);
            odpos.swap(fdpos);
            g->complete = 1;
        }
    }
    // the exact LU's fill passes the cap: the nested-dissection multifrontal LU (its own ordering,
    // dense fronts on the matrix cores) where its plan fits the device; ILU(0) otherwise
    // mf_create: EIGSOL_E_SOLVER = a zero pivot inside a front, EIGSOL_E_UNSUPPORTED = declined (a
    // front buffer allocation failed after the plan's estimate): both continue with ILU(0) below;
    // EIGSOL_E_HIP = a device fault, reported
    // a front whose pivot column is zero in all of its rows (the pivot would have to come from a
    // later front: SparseLU's pivoting would take it, the front-restricted one cannot) is retried with
    // static pivots tau = sqrt(eps) max |m_ij| on such columns (SuperLU_DIST's remedy): K is then
    // the LU of a perturbation of M, and the checked direct solve's GMRES cycles refine it away
    auto static_tau = [&]() {
        double mx = 0.0;
        for (const S& e : mv) mx = std::max(mx, sq_abs(e));
        return std::sqrt(mx) * 1.4901161193847656e-08;
    };
    auto mf_try = [&](MfHost* h, const S* vals, const char* what) -> int {
        int mrc = mf_create(ctx, dtype, h, vals, &g->mf);
        lap(what);
        if (mrc == EIGSOL_E_SOLVER) {
            const char* se = std::getenv("EIGSOL_MF_STATIC");
            if (!(se && !std::strcmp(se, "0"))) {
                int64_t ns = 0;
                mrc = mf_create(ctx, dtype, h, vals, &g->mf, static_tau(), &ns);
                g->mf_static = ns;
                lap("multifrontal factor, static pivots");
            }
        }
        return mrc;
    };
    if (rc == EIGSOL_OK && !g->complete && mfh && mf_prc == EIGSOL_OK) {
        const int mrc = mf_try(mfh, mv.data(), "multifrontal factor");
        if (mrc == EIGSOL_OK) g->complete = 2;
        else if (mrc == EIGSOL_E_HIP) rc = mrc;
    }
    if (mfh) mf_host_free(mfh);
    int32_t zpiv = 0;
    // the factored pattern stays on the device: L and U are split from it there (round 5: the host
    // split of the 1M general-sparse factor took 0.26 s plus a 0.4 GB round trip)
    int32_t *k_rp = nullptr, *k_ci = nullptr, *k_dpos = nullptr;
    S* k_v = nullptr;
    auto free_k = [&]() {
        hipStreamSynchronize(st);
        for (void* p : {(void*)k_rp, (void*)k_ci, (void*)k_v, (void*)k_dpos})
            if (p) hipFree(p);
        k_rp = k_ci = k_dpos = nullptr;
        k_v = nullptr;
    };
    // IKJ factorization on the current pattern (mrp/mci/mv/dpos), level by level on the device
    auto factor = [&]() -> int {
        free_k();
        g->nnzK = (int64_t)mci.size();
        // ILU(0) levels: level(i) = 1 + max level of the rows its strict lower part reads
        std::vector<int32_t> lev(n, 0), lcount;
        for (int64_t i = 0; i < n; ++i) {
            int32_t l = 0;
            for (int32_t e = mrp[i]; e < dpos[i]; ++e) l = std::max(l, lev[mci[e]] + 1);
            lev[i] = l;
            if ((int32_t)lcount.size() <= l) lcount.resize(l + 1, 0);
            ++lcount[l];
        }
        std::vector<int32_t> lstart(lcount.size() + 1, 0), rows(n);
        for (size_t l = 0; l < lcount.size(); ++l) lstart[l + 1] = lstart[l] + lcount[l];
        {
            std::vector<int32_t> fill(lstart.begin(), lstart.end() - 1);
            for (int64_t i = 0; i < n; ++i) rows[fill[lev[i]]++] = (int32_t)i;
        }
        int frc = EIGSOL_OK;
        int32_t *d_rows = nullptr, *d_z = nullptr;
        if (hipMalloc(&k_rp, (n + 1) * 4) != hipSuccess || hipMalloc(&k_ci, std::max<int64_t>(1, g->nnzK) * 4) != hipSuccess ||
            hipMalloc(&k_v, std::max<int64_t>(1, g->nnzK) * sizeof(S)) != hipSuccess ||
            hipMalloc(&k_dpos, n * 4) != hipSuccess || hipMalloc(&d_rows, n * 4) != hipSuccess ||
            hipMalloc(&d_z, 4) != hipSuccess)
            frc = fail(EIGSOL_E_HIP, "solve_shifted: ILU(0) buffers");
        zpiv = 0;
        if (frc == EIGSOL_OK) {
            hipMemcpyAsync(k_rp, mrp.data(), (n + 1) * 4, hipMemcpyHostToDevice, st);
            hipMemcpyAsync(k_ci, mci.data(), g->nnzK * 4, hipMemcpyHostToDevice, st);
            hipMemcpyAsync(k_v, mv.data(), g->nnzK * sizeof(S), hipMemcpyHostToDevice, st);
            hipMemcpyAsync(k_dpos, dpos.data(), n * 4, hipMemcpyHostToDevice, st);
            hipMemcpyAsync(d_rows, rows.data(), n * 4, hipMemcpyHostToDevice, st);
            hipMemsetAsync(d_z, 0, 4, st);
            for (size_t l = 0; l < lcount.size(); ++l) {
                const int32_t cnt = lcount[l];
                hipLaunchKernelGGL((dev::ilu0_level_kernel<S>), dim3((cnt + 255) / 256), dim3(256), 0, st, k_rp, k_ci,
                                   k_dpos, k_v, d_rows + lstart[l], cnt, d_z);
            }
            hipMemcpyAsync(&zpiv, d_z, 4, hipMemcpyDeviceToHost, st);
            if (stream_wait(st) != hipSuccess) frc = fail(EIGSOL_E_HIP, "solve_shifted: ILU(0) factorization");
        }
        for (void* p : {(void*)d_rows, (void*)d_z})
            if (p) hipFree(p);
        return frc;
    };
    if (rc == EIGSOL_OK && !g->mf) rc = factor();
    lap("numeric factor (IKJ levels)");
    if (rc == EIGSOL_OK && zpiv && g->complete == 1) {
        // the exact LU without pivoting met a zero pivot (a singular leading minor of M): the
        // multifrontal LU, whose nested-dissection order and partial pivoting inside each front
        // avoid it where M itself is regular (the reference's SparseLU pivots, solve_shifted.hpp:
        // 104-106); its plan was abandoned when the fill fitted, so it is made now on M's own pattern
        const char* me = std::getenv("EIGSOL_MF");
        size_t fb2 = 0, tb2 = 0;
        if (!(me && !std::strcmp(me, "0")) && hipMemGetInfo(&fb2, &tb2) == hipSuccess) {
            free_k();
            MfHost* h2 = mf_host_new();
            if (mf_prepare(n, orp, oci, dtype, (double)fb2, h2) == EIGSOL_OK) {
                const int mrc = mf_try(h2, ov.data(), "multifrontal factor (after the exact LU's zero pivot)");
                if (mrc == EIGSOL_OK) {
                    g->complete = 2;
                    zpiv = 0;
                } else if (mrc == EIGSOL_E_HIP) {
                    rc = mrc;
                }
            }
            mf_host_free(h2);
        }
    }
    if (rc == EIGSOL_OK && zpiv && g->complete == 1) {
        // the exact LU met a zero pivot (and the multifrontal LU did not help): ILU(0) on M's own
        // pattern (GMRES then iterates over it)
        mrp.swap(orp);
        mci.swap(oci);
        mv.swap(ov);
        dpos.swap(odpos);
        g->complete = 0;
        rc = factor();
    }
    std::vector<int32_t>().swap(orp);
    std::vector<int32_t>().swap(oci);
    std::vector<int32_t>().swap(odpos);
    std::vector<S>().swap(ov);
    if (rc == EIGSOL_OK && zpiv)
        rc = fail(EIGSOL_E_SOLVER, g->complete ? "solve_shifted: sparse LU (complete fill, no pivoting) met a zero pivot"
                                               : "solve_shifted: ILU(0) factorization met a zero pivot");
    if (rc == EIGSOL_OK && !g->mf) {
        // split on the device: L = strict lower + unit diagonal (columns ascending: the lower part,
        // then i), U = diagonal + strict upper
        int32_t *lrp = nullptr, *urp = nullptr, *lci = nullptr, *uci = nullptr, *lcnt = nullptr, *ucnt = nullptr;
        S *lv = nullptr, *uv = nullptr;
        int32_t tot[2] = {0, 0};
        if (hipMalloc(&lrp, (n + 1) * 4) != hipSuccess || hipMalloc(&urp, (n + 1) * 4) != hipSuccess ||
            hipMalloc(&lcnt, (n + 1) * 4) != hipSuccess || hipMalloc(&ucnt, (n + 1) * 4) != hipSuccess)
            rc = fail(EIGSOL_E_HIP, "solve_shifted: L / U split");
        if (rc == EIGSOL_OK) {
            hipLaunchKernelGGL(dev::gm_split_count_kernel, dim3((n + 256) / 256), dim3(256), 0, st, k_rp, k_dpos, n,
                               lcnt, ucnt);
            if (tri_exclusive_scan(st, lcnt, lrp, n) != hipSuccess || tri_exclusive_scan(st, ucnt, urp, n) != hipSuccess)
                rc = fail(EIGSOL_E_HIP, "solve_shifted: L / U split scan");
        }
        if (rc == EIGSOL_OK) {
            hipMemcpyAsync(&tot[0], lrp + n, 4, hipMemcpyDeviceToHost, st);
            hipMemcpyAsync(&tot[1], urp + n, 4, hipMemcpyDeviceToHost, st);
            if (hipStreamSynchronize(st) != hipSuccess || hipMalloc(&lci, std::max(1, tot[0]) * 4) != hipSuccess ||
                hipMalloc(&lv, std::max(1, tot[0]) * sizeof(S)) != hipSuccess ||
                hipMalloc(&uci, std::max(1, tot[1]) * 4) != hipSuccess ||
                hipMalloc(&uv, std::max(1, tot[1]) * sizeof(S)) != hipSuccess)
                rc = fail(EIGSOL_E_HIP, "solve_shifted: L / U split buffers");
        }
        if (rc == EIGSOL_OK)
            hipLaunchKernelGGL((dev::gm_split_fill_kernel<S>), dim3((n + 255) / 256), dim3(256), 0, st, k_rp, k_ci, k_v,
                               k_dpos, n, lrp, urp, lci, lv, uci, uv);
        free_k();
        lap("split L / U");
        if (rc == EIGSOL_OK) rc = shift_factor_tri_dev(ctx, dtype, n, lrp, lci, lv, tot[0], false, &g->L);
        lap("triangular layout L");
        if (rc == EIGSOL_OK) rc = shift_factor_tri_dev(ctx, dtype, n, urp, uci, uv, tot[1], true, &g->U);
        lap("triangular layout U");
        hipStreamSynchronize(st);
        for (void* p : {(void*)lrp, (void*)urp, (void*)lci, (void*)uci, (void*)lv, (void*)uv, (void*)lcnt, (void*)ucnt})
            if (p) hipFree(p);
    }
    free_k();
    const size_t sb = sizeof(S);
    g->G = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n + 2047) / 2048));
    if (rc == EIGSOL_OK &&
        (hipMalloc(&g->V, (size_t)n * (g->m + 1) * sb) != hipSuccess || hipMalloc(&g->Z, (size_t)n * g->m * sb) != hipSuccess ||
         hipMalloc(&g->t1, n * sb) != hipSuccess ||
         hipMalloc(&g->w, n * sb) != hipSuccess ||
         hipMalloc(&g->x, n * sb) != hipSuccess ||
         hipMalloc(&g->part, (size_t)g->G * (g->m + 1) * 2 * sizeof(double)) != hipSuccess ||
         hipMalloc(&g->hdev, (size_t)(g->m + 2) * 6 * sizeof(double)) != hipSuccess ||
         hipHostMalloc(&g->hpin, (size_t)(g->m + 2) * 6 * sizeof(double), hipHostMallocDefault) != hipSuccess))
        rc = fail(EIGSOL_E_HIP, "solve_shifted: GMRES workspace");
    if (rc != EIGSOL_OK) {
        gmres_free(g);
        return rc;
    }
    *out = g;
    return EIGSOL_OK;
}

int gmres_create(eigsol_ctx* ctx, int dtype, int64_t n, const int32_t* rp, const int32_t* ci, const void* v,
                 double sre, double sim, GmresSolver** out, eigsol_csr* Adev) {
    if (Adev && (Adev->dtype != dtype || Adev->nrows != n || Adev->ncols != n || Adev->xoff != 0)) Adev = nullptr;
    if (dtype == EIGSOL_C128)
        return gmres_create_t<cplx>(ctx, dtype, n, rp, ci, static_cast<const cplx*>(v), sre, sim, Adev, out);
    if (dtype == EIGSOL_F64)
        return gmres_create_t<double>(ctx, dtype, n, rp, ci, static_cast<const double*>(v), sre, sim, Adev, out);
    return fail(EIGSOL_E_UNSUPPORTED, "solve_shifted: the GMRES path is built for double and complex<double>");
}

using hc = std::complex<double>;

// one Arnoldi orthogonalisation: h = V(:, 0:k)^H w, w -= V h, twice (CGS2); the coefficients of
// both passes and ||w|| after the second come back in one device->host copy (one sync per step)
template <class S>
static int cgs2(GmresSolver* g, S* V, int k, S* w, std::vector<hc>& h, double& wnorm) {
    hipStream_t st = g->ctx->stream;
    const int64_t n = g->n;
    const int gb = (int)std::min<int64_t>(2048, (n + dev::kThreads - 1) / dev::kThreads);
    const int64_t stride = 2 * (g->m + 1);   // hdev: [pass 0 | pass 1 | norm]
    for (int pass = 0; pass < 2; ++pass) {
        double* hp = g->hdev + pass * stride;
        hipLaunchKernelGGL((dev::gm_dots_kernel<S>), dim3(g->G), dim3(dev::kThreads), 0, st, V, n, k, w, n, g->part);
        hipLaunchKernelGGL(dev::gm_reduce_kernel, dim3(k), dim3(dev::kThreads), 0, st, g->part, g->G, k, hp);
        hipLaunchKernelGGL((dev::gm_combine_kernel<S>), dim3(gb), dim3(dev::kThreads), 0, st, V, n, k, hp, w, n, 0);
    }
    hipLaunchKernelGGL((dev::gm_dots_kernel<S>), dim3(g->G), dim3(dev::kThreads), 0, st, w, n, 1, w, n, g->part);
    hipLaunchKernelGGL(dev::gm_reduce_kernel, dim3(1), dim3(dev::kThreads), 0, st, g->part, g->G, 1, g->hdev + 2 * stride);
    const double* hb = g->hpin;
    EIGSOL_HIP(hipMemcpyAsync(g->hpin, g->hdev, (2 * stride + 2) * sizeof(double), hipMemcpyDeviceToHost, st));
    EIGSOL_HIP(stream_wait(st));
    h.assign(k, hc(0.0, 0.0));
    for (int c = 0; c < k; ++c)
        h[c] = hc(hb[2 * c], hb[2 * c + 1]) + hc(hb[stride + 2 * c], hb[stride + 2 * c + 1]);
    wnorm = std::sqrt(hb[2 * stride]);
    return EIGSOL_OK;
}

// y = M x
template <class S>
static int apply_M(GmresSolver* g, const S* x, S* y) {
    if (g->M) return eigsol_csr_spmv(g->M, x, y);
    EIGSOL_TRY(eigsol_csr_spmv(g->A, x, y));
    const int gb = (int)std::min<int64_t>(2048, (g->n + dev::kThreads - 1) / dev::kThreads);
    hipLaunchKernelGGL((dev::gm_shift_sub_kernel<S>), dim3(gb), dim3(dev::kThreads), 0, g->ctx->stream, x, g->sre,
                       g->sim, y, g->n);
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

template <class S>
static int gmres_solve_t(GmresSolver* g, const S* b, double bdiv, S* y, const double* guess) {
    hipStream_t st = g->ctx->stream;
    const int64_t n = g->n;
    const int m = g->m;
    const int gb = (int)std::min<int64_t>(2048, (n + dev::kThreads - 1) / dev::kThreads);
    S* V = static_cast<S*>(g->V);
    S* Z = static_cast<S*>(g->Z);
    S* w = static_cast<S*>(g->w);
    S* x = static_cast<S*>(g->x);
    S* t1 = static_cast<S*>(g->t1);
    double lb = 0.0, ub = 0.0, mb = 0.0;
    if (g->mf) lb = mf_stats(g->mf).solve_bytes;
    else {
        shift_info(g->L, &lb, nullptr, nullptr);
        shift_info(g->U, &ub, nullptr, nullptr);
    }
    const double sb = (double)sizeof(S);
    mb = (sb + 4.0) * (double)(g->A ? g->A->nnz : g->nnzM) + 4.0 * (double)(n + 1) + (g->A ? 5.0 : 2.0) * sb * (double)n;
    double bytes = 0.0;
    int steps = 0;
    auto norm_of = [&](S* v, double& out) -> int {
        hipLaunchKernelGGL((dev::gm_dots_kernel<S>), dim3(g->G), dim3(dev::kThreads), 0, st, v, n, 1, v, n, g->part);
        hipLaunchKernelGGL(dev::gm_reduce_kernel, dim3(1), dim3(dev::kThreads), 0, st, g->part, g->G, 1, g->hdev);
        EIGSOL_HIP(hipMemcpyAsync(g->hpin, g->hdev, 2 * sizeof(double), hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(stream_wait(st));
        out = std::sqrt(g->hpin[0]);
        return EIGSOL_OK;
    };
    auto precond = [&](const S* in, S* out) -> int {   // out = U^-1 L^-1 in
        if (g->mf) return mf_solve(g->mf, in, out);
        EIGSOL_TRY(shift_solve_launch(g->L, in, t1));
        return shift_solve_launch(g->U, t1, out);
    };
    // r0 = b / bdiv (x0 = 0)
    hipLaunchKernelGGL((dev::gm_resid_kernel<S>), dim3(gb), dim3(dev::kThreads), 0, st, b, bdiv, (const S*)nullptr, w, n);
    double beta = 0.0;
    bool direct_done = false;
    if (g->complete && !guess) {
        // exact factor: ||r0||, x = K^-1 r0, r = r0 - M x and ||r|| with one host wait
        hipLaunchKernelGGL((dev::gm_dots_kernel<S>), dim3(g->G), dim3(dev::kThreads), 0, st, w, n, 1, w, n, g->part);
        hipLaunchKernelGGL(dev::gm_reduce_kernel, dim3(1), dim3(dev::kThreads), 0, st, g->part, g->G, 1, g->hdev);
        EIGSOL_TRY(precond(w, x));
        // t1 = M x (or A x), then r, ||r||^2 and ||x||^2 in one pass and one reduction launch
        EIGSOL_TRY(eigsol_csr_spmv(g->M ? g->M : g->A, x, t1));
        hipLaunchKernelGGL((dev::gm_resid_norms_kernel<S>), dim3(g->G), dim3(dev::kThreads), 0, st, b, bdiv, t1, x,
                           g->sre, g->sim, g->M ? 0 : 1, w, n, g->part);
        hipLaunchKernelGGL(dev::gm_reduce_kernel, dim3(2), dim3(dev::kThreads), 0, st, g->part, g->G, 2, g->hdev + 2);
        EIGSOL_HIP(hipMemcpyAsync(g->hpin, g->hdev, 6 * sizeof(double), hipMemcpyDeviceToHost, st));
        int32_t* mf_err = reinterpret_cast<int32_t*>(g->hpin + 6);   // the multifrontal solve's wait-error word
        if (g->mf) EIGSOL_HIP(hipMemcpyAsync(mf_err, mf_err_word(g->mf), sizeof(int32_t), hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(stream_wait(st));
        if (g->mf && *mf_err) return fail(EIGSOL_E_HIP, "solve_shifted: a multifrontal solve wait did not complete");
        beta = std::sqrt(g->hpin[0]);
        direct_done = true;
    } else {
        EIGSOL_TRY(norm_of(w, beta));
    }
    const double bnorm = beta;
    // A direct solve next to an eigenvalue (||x|| >> ||b||) cannot reach a small relative residual in
    // double precision, and neither can refinement or the densified LU; it is accepted like the
    // reference's SparseLU solve when its normwise backward error ||r|| / (||M|| ||x|| + ||b||) is
    // at rounding level (be_accept), instead of running GMRES cycles to stagnation
    bool backward_ok = false;
    if (direct_done) {
        beta = bnorm > 0.0 ? std::sqrt(g->hpin[2]) : 0.0;
        const double xnorm = std::sqrt(g->hpin[4]);
        backward_ok = bnorm > 0.0 && beta <= g->be_accept * (g->normM * xnorm + bnorm);
        bytes += lb + ub + mb + 4.0 * sb * (double)n;
    } else {
        EIGSOL_HIP(hipMemsetAsync(x, 0, n * sizeof(S), st));
    }
    // Warm start for the shifted inverse iteration: once x_t is close to the eigenvector v
    // ((A - sigma I) v = (lambda - sigma) v), y_t = (A - sigma I)^{-1} x_t is close to
    // x_t / (lambda_{t-1} - sigma): x0 = guess * b / bdiv leaves a residual that shrinks with the
    // iterate's error, so later solves need fewer Arnoldi steps to the same 1e-12 relative residual
    // (kept only when it beats x0 = 0).
    if (guess && bnorm > 0.0) {
        hipLaunchKernelGGL((dev::gm_cscale_kernel<S>), dim3(gb), dim3(dev::kThreads), 0, st, w, guess[0], guess[1], x, n);
        EIGSOL_TRY(apply_M<S>(g, x, t1));
        hipLaunchKernelGGL((dev::gm_resid_kernel<S>), dim3(gb), dim3(dev::kThreads), 0, st, b, bdiv, t1, w, n);
        EIGSOL_TRY(norm_of(w, beta));
        bytes += mb + 4.0 * sb * (double)n;
        if (!(beta < bnorm)) {   // no better than zero: start from zero
            EIGSOL_HIP(hipMemsetAsync(x, 0, n * sizeof(S), st));
            hipLaunchKernelGGL((dev::gm_resid_kernel<S>), dim3(gb), dim3(dev::kThreads), 0, st, b, bdiv,
                               (const S*)nullptr, w, n);
            beta = bnorm;
        }
    }
    // exact LU (complete fill): x = U^-1 L^-1 r0 directly; GMRES cycles below only if its true
    // residual misses rtol_true (iterative refinement on the same factors)
    // (exact LU: done above, before the first host wait)
    double relres = beta / (bnorm > 0.0 ? bnorm : 1.0);
    int cycles = 0;
    if (bnorm > 0.0 && beta > 0.0 && relres > g->rtol_true && !backward_ok) {
        std::vector<double> hist;
        std::vector<hc> H((size_t)(m + 1) * m), cs(m), sn(m), gv(m + 1), h;
        for (int cycle = 0; cycle < g->max_cycles; ++cycle) {
            hipLaunchKernelGGL((dev::gm_div_kernel<S>), dim3(gb), dim3(dev::kThreads), 0, st, w, beta, V, n);
            std::fill(gv.begin(), gv.end(), hc(0.0, 0.0));
            gv[0] = beta;
            int k = 0;
            for (int j = 0; j < m; ++j) {
                S* vj = V + (int64_t)j * n;
                S* zj = Z + (int64_t)j * n;
                EIGSOL_TRY(precond(vj, zj));   // kept: x += Z y at the cycle's end needs no preconditioner
                EIGSOL_TRY(apply_M<S>(g, zj, w));
                double hn = 0.0;
                EIGSOL_TRY(cgs2<S>(g, V, j + 1, w, h, hn));
                bytes += lb + ub + mb + 2.0 * (3.0 * (j + 1) + 2.0) * sb * (double)n;
                ++steps;
                for (int i = 0; i <= j; ++i) H[(size_t)j * (m + 1) + i] = h[i];
                H[(size_t)j * (m + 1) + j + 1] = hn;
                // previous rotations, then a new one zeroing H(j+1, j)
                hc* col = &H[(size_t)j * (m + 1)];
                for (int i = 0; i < j; ++i) {
                    const hc a = col[i], c = col[i + 1];
                    col[i] = std::conj(cs[i]) * a + std::conj(sn[i]) * c;
                    col[i + 1] = -sn[i] * a + cs[i] * c;
                }
                const double na = std::abs(col[j]), nb = std::abs(col[j + 1]);
                const double r = std::hypot(na, nb);
                if (r == 0.0) {
                    cs[j] = 1.0;
                    sn[j] = 0.0;
                } else {
                    cs[j] = col[j] / r;
                    sn[j] = col[j + 1] / r;
                }
                col[j] = r;
                col[j + 1] = 0.0;
                const hc gj = gv[j];
                gv[j] = std::conj(cs[j]) * gj;
                gv[j + 1] = -sn[j] * gj;
                k = j + 1;
                const double est = std::abs(gv[j + 1]);
                if (hn > 0.0 && j + 1 < m)
                    hipLaunchKernelGGL((dev::gm_div_kernel<S>), dim3(gb), dim3(dev::kThreads), 0, st, w, hn,
                                       V + (int64_t)(j + 1) * n, n);
                if (est <= g->rtol * bnorm || hn == 0.0) break;
            }
            // y_k = R^-1 g (upper triangular, k x k), x += Z_k y_k (= K^-1 V_k y_k: the preconditioner is
            // fixed, so flexible GMRES's update is right-preconditioned GMRES's, one application fewer)
            std::vector<hc> yk(k);
            for (int i = k - 1; i >= 0; --i) {
                hc s = gv[i];
                for (int c = i + 1; c < k; ++c) s -= H[(size_t)c * (m + 1) + i] * yk[c];
                yk[i] = s / H[(size_t)i * (m + 1) + i];
            }
            double* yb = g->hpin;   // read by the copy before the next host write (norm_of syncs below)
            for (int i = 0; i < k; ++i) { yb[2 * i] = yk[i].real(); yb[2 * i + 1] = yk[i].imag(); }
            EIGSOL_HIP(hipMemcpyAsync(g->hdev, yb, 2 * k * sizeof(double), hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL((dev::gm_combine_kernel<S>), dim3(gb), dim3(dev::kThreads), 0, st, Z, n, k, g->hdev, w, n, 1);
            hipLaunchKernelGGL((dev::gm_axpy_kernel<S>), dim3(gb), dim3(dev::kThreads), 0, st, x, w, n);
            // true residual r = b - M x (the next cycle's start)
            EIGSOL_TRY(apply_M<S>(g, x, t1));
            hipLaunchKernelGGL((dev::gm_resid_kernel<S>), dim3(gb), dim3(dev::kThreads), 0, st, b, bdiv, t1, w, n);
            EIGSOL_TRY(norm_of(w, beta));
            bytes += mb + 2.0 * (double)k * sb * (double)n;
            relres = beta / bnorm;
            ++cycles;
            hist.push_back(relres);
            if (relres <= g->rtol_true || beta == 0.0) break;
            // stagnation: the last two cycles together did not halve the residual
            if (hist.size() >= 3 && relres > 0.5 * hist[hist.size() - 3]) break;
        }
    }
    EIGSOL_HIP(hipMemcpyAsync(y, x, n * sizeof(S), hipMemcpyDeviceToDevice, st));
    if (g->mf && (!direct_done || cycles > 0 || guess)) {
        // multifrontal solves after the first pass (refinement cycles, a warm-start guess): their
        // wait-error word, read once in one host wait
        int32_t* mf_err = reinterpret_cast<int32_t*>(g->hpin + 6);
        EIGSOL_HIP(hipMemcpyAsync(mf_err, mf_err_word(g->mf), sizeof(int32_t), hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(stream_wait(st));
        if (*mf_err) return fail(EIGSOL_E_HIP, "solve_shifted: a multifrontal solve wait did not complete");
    }
    if (g->L) EIGSOL_TRY(shift_error(g->L));
    if (g->U) EIGSOL_TRY(shift_error(g->U));
    g->last_steps = steps;
    g->last_bytes = bytes;
    g->last_relres = relres;
    if (!(relres <= g->rtol_accept) && !backward_ok) {
        char msg[160];
        std::snprintf(msg, sizeof msg,
                      "solve_shifted: SparseLU solve failed (ILU(0)-GMRES stopped at relative residual %.3g after %d "
                      "cycles)", relres, cycles);
        return fail(EIGSOL_E_SOLVER, msg);
    }
    return EIGSOL_OK;
}

// The shifted inverse iteration's direct solve with its check lagged (gmres_solve_lag): y = K^-1 (b /
// bdiv), then the true residual r = b / bdiv - M y and ||b / bdiv||, ||r||, ||y|| reduced and copied to
// the pinned slot without a host wait; the session reads them at its next decision wait
// (gmres_lag_verdict) and redoes the iteration with the checked solve if they miss the test.  Only
// for a complete factor without static pivots (the solve itself is then the reference's).
template <class S>
static int gmres_solve_lag_t(GmresSolver* g, const S* b, double bdiv, S* y) {
    hipStream_t st = g->ctx->stream;
    const int64_t n = g->n;
    const int gb = (int)std::min<int64_t>(2048, (n + dev::kThreads - 1) / dev::kThreads);
    S* w = static_cast<S*>(g->w);
    S* t1 = static_cast<S*>(g->t1);
    hipLaunchKernelGGL((dev::gm_resid_kernel<S>), dim3(gb), dim3(dev::kThreads), 0, st, b, bdiv, (const S*)nullptr, w, n);
    hipLaunchKernelGGL((dev::gm_dots_kernel<S>), dim3(g->G), dim3(dev::kThreads), 0, st, w, n, 1, w, n, g->part);
    hipLaunchKernelGGL(dev::gm_reduce_kernel, dim3(1), dim3(dev::kThreads), 0, st, g->part, g->G, 1, g->hdev);
    if (g->mf) EIGSOL_TRY(mf_solve(g->mf, w, y));
    else {
        EIGSOL_TRY(shift_solve_launch(g->L, w, t1));
        EIGSOL_TRY(shift_solve_launch(g->U, t1, y));
    }
    EIGSOL_TRY(eigsol_csr_spmv(g->M ? g->M : g->A, y, t1));
    hipLaunchKernelGGL((dev::gm_resid_norms_kernel<S>), dim3(g->G), dim3(dev::kThreads), 0, st, b, bdiv, t1, y,
                       g->sre, g->sim, g->M ? 0 : 1, w, n, g->part);
    hipLaunchKernelGGL(dev::gm_reduce_kernel, dim3(2), dim3(dev::kThreads), 0, st, g->part, g->G, 2, g->hdev + 2);
    double* slot = g->hpin + g->lag_off();
    EIGSOL_HIP(hipMemcpyAsync(slot, g->hdev, 6 * sizeof(double), hipMemcpyDeviceToHost, st));
    int32_t* err = reinterpret_cast<int32_t*>(slot + 6);
    *err = 0;
    if (g->mf) EIGSOL_HIP(hipMemcpyAsync(err, mf_err_word(g->mf), sizeof(int32_t), hipMemcpyDeviceToHost, st));
    g->lag_pending = true;
    double lb = 0.0, ub = 0.0;
    if (g->mf) lb = mf_stats(g->mf).solve_bytes;
    else {
        shift_info(g->L, &lb, nullptr, nullptr);
        shift_info(g->U, &ub, nullptr, nullptr);
    }
    const double sb = (double)sizeof(S);
    g->last_steps = 0;
    g->last_bytes = lb + ub + (sb + 4.0) * (double)(g->A ? g->A->nnz : g->nnzM) + 4.0 * (double)(n + 1) +
                    (g->A ? 5.0 : 2.0) * sb * (double)n + 4.0 * sb * (double)n;
    return EIGSOL_OK;
}

int gmres_can_lag(const GmresSolver* g) {
    const char* e = std::getenv("EIGSOL_GMRES_LAG");   // read per call: tests switch it inside one process
    const bool off = e && std::atoi(e) == 0;
    return !off && g->complete && g->mf_static == 0 && g->hpin ? 1 : 0;
}

void gmres_lag_reset(GmresSolver* g) { g->lag_pending = false; }

int gmres_solve_lag(GmresSolver* g, const void* b_dev, double bdiv, void* y_dev) {
    if (g->dtype == EIGSOL_C128)
        return gmres_solve_lag_t<cplx>(g, static_cast<const cplx*>(b_dev), bdiv, static_cast<cplx*>(y_dev));
    return gmres_solve_lag_t<double>(g, static_cast<const double*>(b_dev), bdiv, static_cast<double*>(y_dev));
}

// the pending lagged check (its copy done: the caller has waited on the stream since): EIGSOL_OK,
// EIGSOL_E_SOLVER (redo the iteration with the checked solve) or EIGSOL_E_HIP (a multifrontal solve
// wait timed out).  EIGSOL_GMRES_LAG_REDO=1 (tests) reports every check as missed.
int gmres_lag_verdict(GmresSolver* g) {
    if (!g->lag_pending) return EIGSOL_OK;
    g->lag_pending = false;
    const double* l = g->hpin + g->lag_off();
    if (*reinterpret_cast<const int32_t*>(l + 6))
        return fail(EIGSOL_E_HIP, "solve_shifted: a multifrontal solve wait did not complete");
    for (ShiftFactor* t : {g->L, g->U})   // the triangular solves' wait-error words
        if (t && shift_error(t) != EIGSOL_OK) return EIGSOL_E_HIP;
    const char* fe = std::getenv("EIGSOL_GMRES_LAG_REDO");
    const bool force = fe && std::atoi(fe) != 0;
    const double bnorm = std::sqrt(l[0]), beta = std::sqrt(l[2]), xnorm = std::sqrt(l[4]);
    const double relres = bnorm > 0.0 ? beta / bnorm : 0.0;
    g->last_relres = relres;
    const bool ok = bnorm == 0.0 || beta == 0.0 || relres <= g->rtol_true ||
                    beta <= g->be_accept * (g->normM * xnorm + bnorm);
    return (ok && !force) ? EIGSOL_OK : EIGSOL_E_SOLVER;
}

int gmres_solve(GmresSolver* g, const void* b_dev, double bdiv, void* y_dev, const double* guess) {
    if (g->dtype == EIGSOL_C128)
        return gmres_solve_t<cplx>(g, static_cast<const cplx*>(b_dev), bdiv, static_cast<cplx*>(y_dev), guess);
    return gmres_solve_t<double>(g, static_cast<const double*>(b_dev), bdiv, static_cast<double*>(y_dev), guess);
}

int gmres_complete(const GmresSolver* g) { return g->complete; }

void gmres_info(const GmresSolver* g, double* bytes, int32_t* steps) {
    if (bytes) *bytes = g->last_bytes;
    if (steps) *steps = g->last_steps;
}

}  // namespace eigsol

extern "C" int eigsol_sparse_lu_fill(int64_t n, const int32_t* rowptr, const int32_t* colidx, int64_t cap,
                                     int64_t* nnz_out, int32_t* lower_levels_out) {
    using namespace eigsol;
    if (n < 0 || (n > 0 && (!rowptr || !colidx)) || !nnz_out || n > INT32_MAX - 1 || (rowptr && rowptr[0] != 0))
        return fail(EIGSOL_E_INVALID, "eigsol_sparse_lu_fill: bad arguments");
    for (int64_t i = 0; i < n; ++i)
        if (rowptr[i + 1] < rowptr[i]) return fail(EIGSOL_E_INVALID, "eigsol_sparse_lu_fill: row pointers not monotone");
    try {
    // A's pattern with the diagonal inserted (the shifted matrix A - sigma I always stores it)
    std::vector<int32_t> mrp(n + 1, 0), mci;
    mci.reserve((size_t)rowptr[n] + n);
    for (int64_t i = 0; i < n; ++i) {
        bool have = false;
        for (int32_t e = rowptr[i]; e <= rowptr[i + 1]; ++e) {
            const bool end = e == rowptr[i + 1];
            if (!have && (end || colidx[e] >= i)) {
                mci.push_back((int32_t)i);
                have = true;
                if (!end && colidx[e] == i) continue;
            }
            if (end) break;
            if (colidx[e] < 0 || colidx[e] >= n)
                return fail(EIGSOL_E_INVALID, "eigsol_sparse_lu_fill: column index out of range");
            if (e > rowptr[i] && colidx[e] <= colidx[e - 1])
                return fail(EIGSOL_E_INVALID, "eigsol_sparse_lu_fill: rows must be sorted without repeats");
            mci.push_back(colidx[e]);
        }
        mrp[i + 1] = (int32_t)mci.size();
    }
    std::vector<int32_t> frp, fci, fdpos;
    if (!lu_fill_pattern(n, mrp, mci, std::min<int64_t>(cap, INT32_MAX - 1), frp, fci, fdpos)) {
        *nnz_out = -1;
        if (lower_levels_out) *lower_levels_out = 0;
        return EIGSOL_OK;
    }
    *nnz_out = (int64_t)fci.size();
    if (lower_levels_out) {
        std::vector<int32_t> lev(n, 0);
        int32_t top = n ? 1 : 0;
        for (int64_t i = 0; i < n; ++i) {
            int32_t l = 0;
            for (int32_t e = frp[i]; e < fdpos[i]; ++e) l = std::max(l, lev[fci[e]] + 1);
            lev[i] = l;
            top = std::max(top, l + 1);
        }
        *lower_levels_out = top;
    }
    return EIGSOL_OK;
    } catch (const std::exception& ex) {   // host allocation: no exception crosses the C ABI
        return fail(EIGSOL_E_INVALID, std::string("eigsol_sparse_lu_fill: ") + ex.what());
    }
}

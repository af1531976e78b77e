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
#include <cstring>
#include <vector>

#include "kernels_common.hpp"

namespace eigsol {

int hqr_lds(hipStream_t st, const double* H, int64_t ld, int n, int maxits, double* wr_dev, double* wi_dev,
            int* info_dev);

namespace dev {

constexpr int kWin = 96;        // window rows/columns (H window + U: 2 x 72 KiB of LDS)
constexpr int kMaxBulges = 16;

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
                    if (sc != 0.0) { p /= sc; q /= sc; r /= sc; }
                } else {
                    p = Hw(k, k - 1);
                    q = Hw(k + 1, k - 1);
                    r = (k != ihi - 1) ? Hw(k + 2, k - 1) : 0.0;
                    xs = fabs(p) + fabs(q) + fabs(r);
                    if (xs != 0.0) { p /= xs; q /= xs; r /= xs; }
                }
                const double sg = (p >= 0 ? 1.0 : -1.0) * sqrt(p * p + q * q + r * r);
                if (sg != 0.0) {
                    if (k != l) {
                        Hw(k, k - 1) = -sg * xs;
                        Hw(k + 1, k - 1) = 0.0;
                        if (k != ihi - 1) Hw(k + 2, k - 1) = 0.0;
                    }
                    p += sg;
                    rp[b][0] = p / sg;
                    rp[b][1] = q / sg;
                    rp[b][2] = r / sg;
                    rp[b][3] = q / p;
                    rp[b][4] = r / p;
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
static constexpr int kSmall = 128;   // blocks finished by the in-LDS solver

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
    auto finish_small = [&](int l, int hi) -> int {
        const int m = hi - l + 1;
        EIGSOL_TRY(hqr_lds(st, H + l + (int64_t)l * n, n, m, std::max(1, maxits), dwr + l, dwi + l, dinfo));
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
            rc = finish_small(l, ihi);
            ihi = l - 1;
            sweeps = std::max(sweeps, stall);
            stall = 0;
            continue;
        }
        if (++stall > max_stall) { failed = 1; sweeps = std::max(sweeps, stall); break; }
        // shifts: eigenvalues of the trailing 2nb x 2nb block
        const int nb = std::min(dev::kMaxBulges, std::max(1, N / 8));
        const int ns = 2 * nb;
        rc = hqr_lds(st, H + (ihi - ns + 1) + (int64_t)(ihi - ns + 1) * n, n, ns, 60, dwr + ihi - ns + 1,
                     dwi + ihi - ns + 1, dinfo);
        if (rc != EIGSOL_OK) break;
        if (hipMemcpyAsync(swr.data(), dwr + ihi - ns + 1, ns * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(swi.data(), dwi + ihi - ns + 1, ns * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            rc = fail(EIGSOL_E_HIP, "francis: shifts");
            break;
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
            dev::ChaseArgs ca{H, n, s, e, l, ihi, t0, t1, nb, dsh, dU};
            hipLaunchKernelGGL(dev::chase_kernel, dim3(1), dim3(1024), 0, st, ca);
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
    for (void* p : {(void*)dwr, (void*)dwi, (void*)dds, (void*)dU, (void*)dsh, (void*)dinfo}) (void)hipFree(p);
    // iterations reported: sweeps spent on the slowest deflation (>= 1, the final check), so that
    // iterations <= maxIterations exactly when the iteration converged
    *sweeps_out = std::max(1, sweeps);
    *fail_out = failed;
    return rc;
}

}  // namespace eigsol

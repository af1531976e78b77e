// Rank-K update on the fp64 matrix cores (gfx950, v_mfma_f64_16x16x4_f64), shared by the blocked
// Hessenberg reduction (hessenberg.hip) and the blocked LU of the shifted solve (shifted.hip).
//
//   C(m x nn) += alpha * L(m x K) * R^T          R stored nn x K      (kRT = false)
//   C(m x nn) += alpha * L(m x K) * Rt           Rt stored K x nn     (kRT = true)
//
// all column-major; S = double, cplx, float or cplxf (interleaved re, im; alpha real).  K <= KMAX, any K
// (the k-steps past K are masked).  Every operand fragment is loaded straight from global memory
// into registers — no LDS, no barrier: each wave owns a 32 x 32 tile of C, loads its 32 x K
// slices of L and R and its C tile, all before the first MFMA.
//
// Fragment layout of the f64 MFMA (cdna_hip_programming.md): A operand lane l holds A[l & 15][l >> 4],
// B operand lane l holds B[l >> 4][l & 15], D lane l register r holds D[(l >> 4) + 4 r][l & 15].
// The A operand carries R (its row index i = a column of C) and the B operand carries L (its
// column index j = a row of C), so D's column index lies on C's row: 16 lanes load and store 128
// contiguous bytes of one column of C.  A complex product takes four real MFMAs:
//   re += Rre Lre - Rim Lim,   im += Rre Lim + Rim Lre.
#pragma once

#include "kernels_common.hpp"

namespace eigsol {
namespace dev {

typedef double mfma_d4 __attribute__((ext_vector_type(4)));

typedef float mfma_f4 __attribute__((ext_vector_type(4)));

template <class S> struct RankKMax;
template <> struct RankKMax<double> { static constexpr int value = 64; };
template <> struct RankKMax<cplx> { static constexpr int value = 32; };
template <> struct RankKMax<float> { static constexpr int value = 64; };
template <> struct RankKMax<cplxf> { static constexpr int value = 32; };

__device__ __forceinline__ double re_of(double v) { return v; }
__device__ __forceinline__ double im_of(double) { return 0.0; }
__device__ __forceinline__ double re_of(cplx v) { return v.re; }
__device__ __forceinline__ double im_of(cplx v) { return v.im; }
__device__ __forceinline__ float re_of(float v) { return v; }
__device__ __forceinline__ float im_of(float) { return 0.0f; }
__device__ __forceinline__ float re_of(cplxf v) { return v.re; }
__device__ __forceinline__ float im_of(cplxf v) { return v.im; }

// Single precision (float, complex<float>) runs on v_mfma_f32_16x16x4_f32: the same operand
// layout as the f64 instruction, but the standard C/D map (lane l register r holds
// D[4 (l >> 4) + r][l & 15]) instead of the f64 one (D[(l >> 4) + 4 r][l & 15]).
template <class S> struct MfmaOf {
    using real = double;
    using acc = mfma_d4;
    static constexpr int kRowStride = 4;   // D row of (lk, r) = lk + 4 r
    static constexpr int kLkStride = 1;
    __device__ static acc step(real a, real b, acc c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
};
template <> struct MfmaOf<float> {
    using real = float;
    using acc = mfma_f4;
    static constexpr int kRowStride = 1;   // D row of (lk, r) = 4 lk + r
    static constexpr int kLkStride = 4;
    __device__ static acc step(real a, real b, acc c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
};
template <> struct MfmaOf<cplx> : MfmaOf<double> {};
template <> struct MfmaOf<cplxf> : MfmaOf<float> {};

// One 64 x 64 tile (tile row bx, tile column by) of the update, by a 256-thread workgroup; shared by
// rankk_mfma (one launch per update) and batched callers (multifrontal.hip: many fronts per launch).
template <class S, bool kRT>
__device__ __forceinline__ void rankk_tile(int bx, int by, int m, int nn, int K, double alpha, const S* L, int64_t ldl,
                                           const S* R, int64_t ldr, S* C, int64_t ldc) {
    constexpr bool kC = std::is_same_v<S, cplx> || std::is_same_v<S, cplxf>;
    using M = MfmaOf<S>;
    using Real = typename M::real;
    using Acc = typename M::acc;
    constexpr int KQ = RankKMax<S>::value / 4;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int r0 = bx * 64 + 32 * (wave & 1);
    const int c0 = by * 64 + 32 * (wave >> 1);
    S ra[2][KQ], lb[2][KQ];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int col = min(c0 + 16 * t + li, nn - 1), row = min(r0 + 16 * t + li, m - 1);
#pragma unroll
        for (int q = 0; q < KQ; ++q) {
            const int k = min(4 * q + lk, K - 1);
            ra[t][q] = kRT ? R[k + (int64_t)col * ldr] : R[col + (int64_t)k * ldr];
            lb[t][q] = L[row + (int64_t)k * ldl];
        }
    }
    // D row index of (lk, r): C's column offset inside the 16-column tile
    auto dcol = [&](int r) { return M::kLkStride * lk + M::kRowStride * r; };
    S c[2][2][4];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = min(r0 + 16 * ti + li, m - 1), col = min(c0 + 16 * tj + dcol(r), nn - 1);
                c[ti][tj][r] = C[row + (int64_t)col * ldc];
            }
    Acc are[2][2], aim[2][2];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) are[ti][tj] = aim[ti][tj] = Acc{0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
        if (4 * q >= K) break;
        const bool kv = 4 * q + lk < K;
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj) {
                const Real rr = kv ? re_of(ra[tj][q]) : Real(0), lr = kv ? re_of(lb[ti][q]) : Real(0);
                are[ti][tj] = M::step(rr, lr, are[ti][tj]);
                if constexpr (kC) {
                    const Real ri = kv ? im_of(ra[tj][q]) : Real(0), li_ = kv ? im_of(lb[ti][q]) : Real(0);
                    are[ti][tj] = M::step(-ri, li_, are[ti][tj]);
                    aim[ti][tj] = M::step(rr, li_, aim[ti][tj]);
                    aim[ti][tj] = M::step(ri, lr, aim[ti][tj]);
                }
            }
    }
    const Real al = (Real)alpha;
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = r0 + 16 * ti + li, col = c0 + 16 * tj + dcol(r);
                if (row < m && col < nn) {
                    if constexpr (kC)
                        C[row + (int64_t)col * ldc] = S{c[ti][tj][r].re + al * are[ti][tj][r],
                                                        c[ti][tj][r].im + al * aim[ti][tj][r]};
                    else
                        C[row + (int64_t)col * ldc] = c[ti][tj][r] + al * are[ti][tj][r];
                }
            }
}

template <class S, bool kRT>
__global__ __launch_bounds__(256) void rankk_mfma(int m, int nn, int K, double alpha, const S* L, int64_t ldl,
                                                  const S* R, int64_t ldr, S* C, int64_t ldc) {
    rankk_tile<S, kRT>(blockIdx.x, blockIdx.y, m, nn, K, alpha, L, ldl, R, ldr, C, ldc);
}

}  // namespace dev

// C += alpha L R^T (or L Rt), stream-ordered; K <= RankKMax<S>::value.
template <class S, bool kRT>
inline void rankk_update(hipStream_t st, int m, int nn, int K, double alpha, const S* L, int64_t ldl, const S* R,
                         int64_t ldr, S* C, int64_t ldc) {
    if (m <= 0 || nn <= 0 || K <= 0) return;
    hipLaunchKernelGGL((dev::rankk_mfma<S, kRT>), dim3((m + 63) / 64, (nn + 63) / 64), dim3(256), 0, st, m, nn, K,
                       alpha, L, ldl, R, ldr, C, ldc);
}

}  // namespace eigsol

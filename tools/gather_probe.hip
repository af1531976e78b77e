// Random-gather ceiling probe (MI355X): what a uniform-column SpMV can reach at best.
//
// Streams (value, column) pairs exactly like the sliced gather layout (lane-consecutive 16-byte
// value pairs and int32 columns, 16 entries per lane issued before any is used, non-temporal
// stream loads) and gathers x[col] for uniformly random columns over an x of n doubles; no row
// sums are stored except one per lane (8 bytes per 16 entries, like y).  Reported: ns per entry
// and the SpMV-equivalent algorithmic GB/s (12 bytes per entry + 24 bytes per row of 16 entries),
// for the config-3 (1M) and config-4-uniform (10M) x sizes.  Build:
//   hipcc -O3 --offload-arch=gfx950 tools/gather_probe.hip -o gpurun_out/gather_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>

template <int K>
__global__ __launch_bounds__(256) void gather_k(const double* __restrict__ val, const int* __restrict__ col,
                                                const double* __restrict__ x, double* __restrict__ y, long rows) {
    const long lanes = (long)gridDim.x * 256;
    for (long r = (long)blockIdx.x * 256 + threadIdx.x; r < rows; r += lanes) {
        const long base = (r / 64) * 64 * K + (r % 64);
        double v[K];
        int c[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            v[k] = __builtin_nontemporal_load(val + base + 64L * k);
            c[k] = __builtin_nontemporal_load(col + base + 64L * k);
        }
        double xv[K];
#pragma unroll
        for (int k = 0; k < K; ++k) xv[k] = x[c[k]];
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) s += v[k] * xv[k];
        y[r] = s;
    }
}

int main() {
    for (long n : {1000000L, 10000000L}) {
        constexpr int K = 16;
        const long nnz = n * K;
        std::vector<int> hc(nnz);
        std::mt19937_64 g(42);
        for (long i = 0; i < nnz; ++i) hc[i] = (int)(g() % (unsigned long)n);
        double *val, *x, *y;
        int* col;
        hipMalloc(&val, nnz * 8);
        hipMalloc(&col, nnz * 4);
        hipMalloc(&x, n * 8);
        hipMalloc(&y, n * 8);
        hipMemset(val, 0, nnz * 8);
        hipMemset(x, 0, n * 8);
        hipMemcpy(col, hc.data(), nnz * 4, hipMemcpyHostToDevice);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        for (int grid : {512, 1024, 2048, 4096}) {
            for (int w = 0; w < 3; ++w) gather_k<K><<<grid, 256>>>(val, col, x, y, n);
            hipEventRecord(e0);
            const int reps = 20;
            for (int r = 0; r < reps; ++r) gather_k<K><<<grid, 256>>>(val, col, x, y, n);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1e3 / reps;
            const double alg = 12.0 * nnz + 24.0 * n;   // SURVEY 8d bytes of the equivalent SpMV (K = 16)
            printf("n=%ld K=%d grid=%d: %.1f us  %.3f ns/entry  SpMV-equivalent %.1f GB/s\n", n, K, grid, us,
                   us * 1e3 / nnz, alg / (us * 1e-6) / 1e9);
        }
        hipFree(val);
        hipFree(col);
        hipFree(x);
        hipFree(y);
    }
    return 0;
}

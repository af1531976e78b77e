// HBM calibration probe (MI355X): streaming read+write copy and read-only reduction with 16-byte
// lane accesses, timed with hipEvents.  Gives the achievable ceiling the SpMV is compared to.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void copy_k(const double4* __restrict__ a, double4* __restrict__ b, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}
__global__ __launch_bounds__(256) void read_k(const double2* __restrict__ a, size_t n, double* out) {
    double s = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) { double2 v = a[i]; s += v.x + v.y; }
    if (s == 12345.678) out[0] = s;
}

int main(int argc, char** argv) {
    size_t bytes = (argc > 1 ? atoll(argv[1]) : 2048) * (size_t)1 << 20;
    double4 *a, *b; double* o;
    hipMalloc(&a, bytes); hipMalloc(&b, bytes); hipMalloc(&o, 64);
    hipMemset(a, 0, bytes); hipMemset(b, 0, bytes);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int grid : {1024, 2048, 4096, 8192}) {
        size_t n4 = bytes / sizeof(double4);
        for (int w = 0; w < 3; ++w) copy_k<<<grid, 256>>>(a, b, n4);
        hipEventRecord(e0);
        for (int r = 0; r < 20; ++r) copy_k<<<grid, 256>>>(a, b, n4);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        double cgbs = 2.0 * bytes * 20 / (ms / 1e3) / 1e9;
        size_t n2 = bytes / sizeof(double2);
        for (int w = 0; w < 3; ++w) read_k<<<grid, 256>>>((const double2*)a, n2, o);
        hipEventRecord(e0);
        for (int r = 0; r < 20; ++r) read_k<<<grid, 256>>>((const double2*)a, n2, o);
        hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        double rgbs = 1.0 * bytes * 20 / (ms / 1e3) / 1e9;
        printf("{\"bytes\": %zu, \"grid\": %d, \"copy_GBps\": %.1f, \"read_GBps\": %.1f}\n", bytes, grid, cgbs, rgbs);
    }
    return 0;
}

// Probe: does splitting a tile's bytes over 2-3 separate streams cost HBM bandwidth versus one
// contiguous stream of the same size?  Each block walks "tiles" of 24 KiB with 256 threads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

// one contiguous stream: 24 KiB per tile = 6 x 16 B per lane
__global__ __launch_bounds__(256) void one_stream(const double2* __restrict__ a, size_t ntiles, double* out) {
    double s = 0;
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const double2* p = a + t * 1536;
#pragma unroll
        for (int k = 0; k < 6; ++k) { double2 v = p[threadIdx.x + 256 * k]; s += v.x + v.y; }
    }
    if (s == 1.2345) out[0] = s;
}
// three streams: values 16 KiB (4 x 16 B/lane), columns 8 KiB (4 x 8 B/lane), rowptr 1 KiB (4 B/lane)
__global__ __launch_bounds__(256) void three_streams(const double2* __restrict__ v, const int2* __restrict__ c,
                                                    const int* __restrict__ r, size_t ntiles, double* out) {
    double s = 0;
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            double2 x = v[t * 1024 + threadIdx.x + 256 * k];
            int2 y = c[t * 1024 + threadIdx.x + 256 * k];
            s += x.x + x.y + y.x + y.y;
        }
        s += r[t * 256 + threadIdx.x];
    }
    if (s == 1.2345) out[0] = s;
}

int main() {
    const size_t ntiles = 56000;   // ~1.37 GB
    double2 *a, *v; int2* c; int* r; double* o;
    hipMalloc(&a, ntiles * 24576); hipMalloc(&v, ntiles * 16384); hipMalloc(&c, ntiles * 8192);
    hipMalloc(&r, ntiles * 1024); hipMalloc(&o, 64);
    hipMemset(a, 0, ntiles * 24576); hipMemset(v, 0, ntiles * 16384); hipMemset(c, 0, ntiles * 8192); hipMemset(r, 0, ntiles * 1024);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int grid : {1024, 1280, 2048, 4096}) {
        float ms1, ms3;
        for (int w = 0; w < 3; ++w) one_stream<<<grid, 256>>>(a, ntiles, o);
        hipEventRecord(e0); for (int i = 0; i < 20; ++i) one_stream<<<grid, 256>>>(a, ntiles, o);
        hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms1, e0, e1);
        for (int w = 0; w < 3; ++w) three_streams<<<grid, 256>>>(v, c, r, ntiles, o);
        hipEventRecord(e0); for (int i = 0; i < 20; ++i) three_streams<<<grid, 256>>>(v, c, r, ntiles, o);
        hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms3, e0, e1);
        printf("{\"grid\": %d, \"one_stream_GBps\": %.1f, \"three_streams_GBps\": %.1f}\n", grid,
               ntiles * 24576.0 * 20 / (ms1 / 1e3) / 1e9, ntiles * 25600.0 * 20 / (ms3 / 1e3) / 1e9);
    }
    return 0;
}

// Standalone check: does rocprofv3 --kernel-trace survive process exit after a cooperative launch?
// hipcc --offload-arch=gfx950 -o tools/coop_prof_repro tools/coop_prof_repro.hip
// rocprofv3 --kernel-trace --stats -d gpurun_out/coop -- ./tools/coop_prof_repro [plain]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
__global__ void touch(int* p) { if (threadIdx.x == 0) atomicAdd(p, 1); }
int main(int argc, char** argv) {
    const bool plain = argc > 1 && !std::strcmp(argv[1], "plain");
    int* d = nullptr;
    if (hipMalloc(&d, 4) != hipSuccess) return 2;
    (void)hipMemset(d, 0, 4);
    void* args[] = {&d};
    for (int i = 0; i < 10; ++i) {
        hipError_t e;
        if (plain) { touch<<<64, 256>>>(d); e = hipGetLastError(); }
        else e = hipLaunchCooperativeKernel((const void*)touch, dim3(64), dim3(256), args, 0, 0);
        if (e != hipSuccess) { std::printf("launch: %s\n", hipGetErrorString(e)); return 3; }
    }
    int h = 0;
    (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    std::printf("%s launches done: %d\n", plain ? "plain" : "cooperative", h);
    return h == 640 ? 0 : 1;
}

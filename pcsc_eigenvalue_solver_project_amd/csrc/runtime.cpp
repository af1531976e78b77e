// Context, error reporting and device-memory helpers of the C ABI (include/eigsol_hip.h).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>

#include "internal.hpp"

namespace eigsol {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int status, const std::string& msg) {
    g_last_error = msg;
    return status;
}

void dist_release_comm(eigsol_ctx* ctx);   // dist.hip

hipError_t stream_wait(hipStream_t st) {
    static const bool spin = [] {
        const char* e = std::getenv("EIGSOL_SYNC_SPIN");
        return e && std::atoi(e) != 0;
    }();
    if (!spin) return hipStreamSynchronize(st);
    hipError_t e;
    while ((e = hipStreamQuery(st)) == hipErrorNotReady) {
    }
    return e;
}

void ctx_retain(eigsol_ctx* c) { c->refs.fetch_add(1); }

void ctx_release(eigsol_ctx* ctx) {
    if (!ctx || ctx->refs.fetch_sub(1) != 1) return;
    (void)hipSetDevice(ctx->device);
    dist_release_comm(ctx);
    if (ctx->own_stream) {
        (void)hipStreamSynchronize(ctx->own_stream);
        (void)hipStreamDestroy(ctx->own_stream);
    }
    delete ctx;
}

// Blocks of `threads` threads resident at once over the whole chip, from the kernel's own VGPR
// and LDS usage (MI355X_MICROARCH.md § Register files: waves per SIMD = floor(512 / VGPR
// allocation), at most 8; 160 KiB LDS per CU).
int resident_blocks(eigsol_ctx* ctx, const void* kernel, int threads, size_t dyn_lds, int* grid) {
    hipFuncAttributes fa;
    EIGSOL_HIP(hipFuncGetAttributes(&fa, kernel));
    const int waves = std::max(1, threads / 64);
    const int vgpr_alloc = std::max(8, ((fa.numRegs + 7) / 8) * 8);
    const int by_vgpr = std::max(1, std::min(8, 512 / vgpr_alloc) * 4 / waves);
    const size_t lds = fa.sharedSizeBytes + dyn_lds;
    const int by_lds = lds ? (int)std::max<size_t>(1, 160 * 1024 / lds) : 32;
    *grid = std::max(1, std::min(by_vgpr, by_lds)) * ctx->num_cus;
    return EIGSOL_OK;
}

}  // namespace eigsol

using namespace eigsol;

extern "C" {

int eigsol_abi_version(void) { return EIGSOL_ABI_VERSION; }

const char* eigsol_status_string(int status) {
    switch (status) {
        case EIGSOL_OK: return "ok";
        case EIGSOL_E_NOT_SQUARE: return "matrix must be square";
        case EIGSOL_E_ZERO_SIZE: return "matrix has zero size";
        case EIGSOL_E_SCALAR_MISMATCH: return "scalar type mismatch";
        case EIGSOL_E_SIZE_MISMATCH: return "size mismatch";
        case EIGSOL_E_NOT_DENSE: return "only dense matrices are supported";
        case EIGSOL_E_SOLVER: return "solver failure";
        case EIGSOL_E_HIP: return "HIP error";
        case EIGSOL_E_RCCL: return "RCCL error";
        case EIGSOL_E_INVALID: return "invalid argument";
        case EIGSOL_E_NO_DEVICE: return "no gfx950 device";
        case EIGSOL_E_EMPTY: return "empty matrix";
        case EIGSOL_E_UNSUPPORTED: return "unsupported";
        default: return "unknown status";
    }
}

const char* eigsol_last_error(void) { return g_last_error.c_str(); }

int eigsol_device_count(int* count) {
    if (!count) return fail(EIGSOL_E_INVALID, "eigsol_device_count: null pointer");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return fail(EIGSOL_E_NO_DEVICE, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    }
    *count = n;
    return EIGSOL_OK;
}

int eigsol_ctx_create(int device, eigsol_ctx** out) {
    if (!out) return fail(EIGSOL_E_INVALID, "eigsol_ctx_create: null out");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return fail(EIGSOL_E_NO_DEVICE, "eigsol_ctx_create: no HIP device visible (" +
                                            std::string(hipGetErrorString(e)) + ")");
    if (device < 0 || device >= n)
        return fail(EIGSOL_E_INVALID, "eigsol_ctx_create: device index out of range");
    EIGSOL_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    EIGSOL_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(EIGSOL_E_NO_DEVICE, std::string("eigsol_ctx_create: device is ") +
                                            prop.gcnArchName + ", this build targets gfx950");
    auto* c = new eigsol_ctx();
    c->device = device;
    c->num_cus = prop.multiProcessorCount;
    hipError_t se = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    if (se != hipSuccess) {
        delete c;
        return fail(EIGSOL_E_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(se));
    }
    c->stream = c->own_stream;
    *out = c;
    return EIGSOL_OK;
}

int eigsol_ctx_destroy(eigsol_ctx* ctx) {
    ctx_release(ctx);
    return EIGSOL_OK;
}

int eigsol_ctx_set_stream(eigsol_ctx* ctx, void* s) {
    if (!ctx) return fail(EIGSOL_E_INVALID, "eigsol_ctx_set_stream: null ctx");
    ctx->stream = s ? static_cast<hipStream_t>(s) : ctx->own_stream;
    return EIGSOL_OK;
}

int eigsol_ctx_get_stream(eigsol_ctx* ctx, void** s) {
    if (!ctx || !s) return fail(EIGSOL_E_INVALID, "eigsol_ctx_get_stream: null pointer");
    *s = ctx->stream;
    return EIGSOL_OK;
}

int eigsol_ctx_synchronize(eigsol_ctx* ctx) {
    if (!ctx) return fail(EIGSOL_E_INVALID, "eigsol_ctx_synchronize: null ctx");
    EIGSOL_HIP(hipSetDevice(ctx->device));
    EIGSOL_HIP(hipStreamSynchronize(ctx->stream));
    return EIGSOL_OK;
}

int eigsol_malloc(eigsol_ctx* ctx, size_t bytes, void** dptr) {
    if (!ctx || !dptr) return fail(EIGSOL_E_INVALID, "eigsol_malloc: null pointer");
    EIGSOL_HIP(hipSetDevice(ctx->device));
    EIGSOL_HIP(hipMalloc(dptr, bytes ? bytes : 16));
    return EIGSOL_OK;
}

int eigsol_free(eigsol_ctx* ctx, void* dptr) {
    if (!ctx) return fail(EIGSOL_E_INVALID, "eigsol_free: null ctx");
    if (!dptr) return EIGSOL_OK;
    EIGSOL_HIP(hipSetDevice(ctx->device));
    EIGSOL_HIP(hipStreamSynchronize(ctx->stream));
    EIGSOL_HIP(hipFree(dptr));
    return EIGSOL_OK;
}

int eigsol_memcpy_h2d(eigsol_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!ctx || (!dst && bytes) || (!src && bytes))
        return fail(EIGSOL_E_INVALID, "eigsol_memcpy_h2d: null pointer");
    if (!bytes) return EIGSOL_OK;
    EIGSOL_HIP(hipSetDevice(ctx->device));
    EIGSOL_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    EIGSOL_HIP(hipStreamSynchronize(ctx->stream));
    return EIGSOL_OK;
}

int eigsol_memcpy_d2h(eigsol_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!ctx || (!dst && bytes) || (!src && bytes))
        return fail(EIGSOL_E_INVALID, "eigsol_memcpy_d2h: null pointer");
    if (!bytes) return EIGSOL_OK;
    EIGSOL_HIP(hipSetDevice(ctx->device));
    EIGSOL_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    EIGSOL_HIP(hipStreamSynchronize(ctx->stream));
    return EIGSOL_OK;
}

}  // extern "C"

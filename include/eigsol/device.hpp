// EigSol drop-in façade — binding to the C ABI of libeigsol_hip.so (include/eigsol_hip.h).
//
// One process-wide device context (device index from EIGSOL_DEVICE, default 0), created on first
// use.  Status codes from the library become the reference's exception types: every error the
// reference reports is a std::runtime_error carrying the reference's message (the library builds
// those messages, see eigsol_status in eigsol_hip.h); device/runtime failures are
// std::runtime_error too, with the library's detail.  There is no host fallback: without a
// gfx950 device the first solver call throws.
#pragma once

#include <complex>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <type_traits>

#include "../eigsol_hip.h"

namespace EigSol {
namespace detail {

inline void check(int status, const char* what) {
    if (status == EIGSOL_OK) return;
    std::string msg = eigsol_last_error();
    if (msg.empty()) msg = std::string(what) + ": " + eigsol_status_string(status);
    throw std::runtime_error(msg);
}

template <typename S>
constexpr eigsol_dtype dtype_of() {
    static_assert(std::is_same_v<S, double> || std::is_same_v<S, std::complex<double>> ||
                      std::is_same_v<S, float> || std::is_same_v<S, std::complex<float>> ||
                      std::is_same_v<S, long double> || std::is_same_v<S, std::complex<long double>>,
                  "the device path supports double, float, long double and their complex types");
    if constexpr (std::is_same_v<S, double>) return EIGSOL_F64;
    else if constexpr (std::is_same_v<S, std::complex<double>>) return EIGSOL_C128;
    else if constexpr (std::is_same_v<S, float>) return EIGSOL_F32;
    else if constexpr (std::is_same_v<S, std::complex<float>>) return EIGSOL_C64;
    else if constexpr (std::is_same_v<S, long double>) return EIGSOL_DD;   // double-double on the wire
    else return EIGSOL_CDD;
}

class Context {
public:
    static Context& get() {
        static Context c;
        return c;
    }
    eigsol_ctx* handle() {
        std::call_once(once_, [this] {
            int dev = 0;
            if (const char* e = std::getenv("EIGSOL_DEVICE")) dev = std::atoi(e);
            check(eigsol_ctx_create(dev, &ctx_), "eigsol_ctx_create");
        });
        return ctx_;
    }
    ~Context() {
        if (ctx_) eigsol_ctx_destroy(ctx_);
    }

private:
    Context() = default;
    std::once_flag once_;
    eigsol_ctx* ctx_ = nullptr;
};

inline eigsol_ctx* ctx() { return Context::get().handle(); }

// RAII owner of a device matrix handle.
class DeviceMatrix {
public:
    static std::shared_ptr<DeviceMatrix> dense(eigsol_dtype dt, std::int64_t r, std::int64_t c, const void* colmajor) {
        auto m = std::shared_ptr<DeviceMatrix>(new DeviceMatrix());
        check(eigsol_dense_create(ctx(), dt, r, c, colmajor, &m->dense_), "eigsol_dense_create");
        return m;
    }
    static std::shared_ptr<DeviceMatrix> csc(eigsol_dtype dt, std::int64_t r, std::int64_t c, std::int64_t nnz,
                                             const std::int32_t* colptr, const std::int32_t* rowidx, const void* v) {
        auto m = std::shared_ptr<DeviceMatrix>(new DeviceMatrix());
        check(eigsol_csr_create_from_csc(ctx(), dt, r, c, nnz, colptr, rowidx, v, &m->csr_), "eigsol_csr_create_from_csc");
        return m;
    }
    static std::shared_ptr<DeviceMatrix> coo(eigsol_dtype dt, std::int64_t r, std::int64_t c, std::int64_t nnz,
                                             const std::int32_t* row, const std::int32_t* col, const void* v) {
        auto m = std::shared_ptr<DeviceMatrix>(new DeviceMatrix());
        check(eigsol_csr_create_from_coo(ctx(), dt, r, c, nnz, row, col, v, &m->csr_), "eigsol_csr_create_from_coo");
        return m;
    }
    ~DeviceMatrix() {
        if (csr_) eigsol_csr_destroy(csr_);
        if (dense_) eigsol_dense_destroy(dense_);
    }
    eigsol_csr* csr() const { return csr_; }
    eigsol_dense* dense() const { return dense_; }

private:
    DeviceMatrix() = default;
    eigsol_csr* csr_ = nullptr;
    eigsol_dense* dense_ = nullptr;
};

}  // namespace detail
}  // namespace EigSol

// Power-iteration session: the host side of the fused device loop (include/eigsol_hip.h).
//
// Mirrors powerMethodImpl (src/power_method/power_method.hpp:47-99): begin() plays :60-66
// (x0 normalisation, lambda = 0, counters), each step() enqueues fused iterations of :68-96,
// finish() returns the EigenResult fields of :98.  The termination logic runs on the device
// (power_decide in internal.hpp), so the host only polls a done word between chunks.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "internal.hpp"

namespace eigsol {
int csr_grid(eigsol_csr* A, int* grid);
int csr_power_launch(eigsol_csr* A, int64_t xlen, void* buf0, void* buf1, PowerCtl* ctl,
                     const void* rank_part, int nranks, void* my_part, void* blk_part, void* trace,
                     int parity, int grid);
int dense_grid(eigsol_dense* A, int* grid);
int dense_power_launch(eigsol_dense* A, void* buf0, void* buf1, PowerCtl* ctl,
                       const void* rank_part, int nranks, void* my_part, void* blk_part,
                       void* trace, int parity, int grid);
int norm_partial_launch(eigsol_ctx* ctx, int dtype, const void* x, int64_t n, PowerCtl* ctl,
                        void* blk_part, void* out, int grid);
int scale_out_launch(eigsol_ctx* ctx, int dtype, const void* src, double nrm, void* dst, int64_t n);
int dist_exchange(eigsol_csr* A, void* y, void* rank_part);
struct ShiftFactor;
int shift_factor_csr(eigsol_csr* A, const void* sigma, ShiftFactor** out);
int shift_factor_dense(eigsol_dense* A, const void* sigma, ShiftFactor** out);
void shift_factor_free(ShiftFactor* f);
int shift_grid(const ShiftFactor* f);
int shift_error(ShiftFactor* f);
int shift_iter_launch(ShiftFactor* f, void* buf0, void* buf1, PowerCtl* ctl, const void* rank_part,
                      void* my_part, void* trace, int parity);
int shift_solve_launch(ShiftFactor* f, const void* b_dev, void* y_dev);
void shift_info(const ShiftFactor* f, double* bytes, int32_t* variant, int32_t* tiles);
}  // namespace eigsol

using namespace eigsol;

struct eigsol_power {
    eigsol_ctx* ctx = nullptr;
    eigsol_csr* csr = nullptr;
    eigsol_dense* dense = nullptr;
    ShiftFactor* shift = nullptr;   // shifted inverse iteration: factor of A - sigma I
    int dtype = EIGSOL_F64;
    int64_t n = 0;            // rows owned (= vector length on one GPU)
    int64_t nbuf = 0;         // own + ghost entries (x-space)
    int64_t xoff = 0;         // x-space index of own row 0 (row-sharded: lower ghosts first)
    bool dist = false;
    void* buf[2] = {nullptr, nullptr};
    PowerCtl* ctl = nullptr;
    void* rank_part = nullptr;   // part4[nranks]
    void* my_part = nullptr;     // part4 (== rank_part on one GPU)
    void* blk_part = nullptr;    // part4[grid]
    void* trace = nullptr;
    int32_t trace_cap = 0;
    int grid = 8;
    int parity = 0;
    int launches = 0;
    bool begun = false;
    bool trivial = false;     // maxIterations <= 0
    PowerCtl* host_ctl = nullptr;   // pinned mirror for polling
    eigsol_solver_options opts{1000, 1e-10};
};

static constexpr size_t kPart = 32;

static int session_alloc(eigsol_power* s, int32_t trace_cap) {
    const size_t sb = scalar_bytes(s->dtype);
    EIGSOL_HIP(hipSetDevice(s->ctx->device));
    for (int i = 0; i < 2; ++i) EIGSOL_HIP(hipMalloc(&s->buf[i], std::max<int64_t>(s->nbuf, 1) * sb + 64));
    EIGSOL_HIP(hipMalloc(&s->ctl, sizeof(PowerCtl)));
    EIGSOL_HIP(hipMalloc(&s->rank_part, kPart * std::max(1, s->ctx->nranks)));
    // rank partials are all-gathered in place: this rank's slot is rank_part[rank]
    s->my_part = static_cast<char*>(s->rank_part) + kPart * (s->dist ? s->ctx->rank : 0);
    EIGSOL_HIP(hipMalloc(&s->blk_part, kPart * std::max(8, s->grid)));
    if (trace_cap > 0) EIGSOL_HIP(hipMalloc(&s->trace, (size_t)trace_cap * sb));
    s->trace_cap = std::max(0, trace_cap);
    EIGSOL_HIP(hipHostMalloc(&s->host_ctl, sizeof(PowerCtl), hipHostMallocDefault));
    std::memset(s->host_ctl, 0, sizeof(PowerCtl));
    EIGSOL_HIP(hipMemsetAsync(s->ctl, 0, sizeof(PowerCtl), s->ctx->stream));
    EIGSOL_HIP(hipMemsetAsync(s->blk_part, 0, kPart * std::max(8, s->grid), s->ctx->stream));
    return EIGSOL_OK;
}

static void session_free(eigsol_power* s) {
    if (!s) return;
    hipSetDevice(s->ctx->device);
    hipStreamSynchronize(s->ctx->stream);
    hipFree(s->buf[0]);
    hipFree(s->buf[1]);
    hipFree(s->ctl);
    hipFree(s->rank_part);
    hipFree(s->blk_part);
    if (s->trace) hipFree(s->trace);
    if (s->host_ctl) hipHostFree(s->host_ctl);
    if (s->shift) shift_factor_free(s->shift);
    if (s->csr) csr_release(s->csr);
    if (s->dense) dense_release(s->dense);
    delete s;
}

static int launch_iteration(eigsol_power* s) {
    if (s->shift)
        return shift_iter_launch(s->shift, s->buf[0], s->buf[1], s->ctl, s->rank_part, s->my_part,
                                 s->trace, s->parity);
    if (s->csr && s->dist) {
        EIGSOL_TRY(csr_power_launch(s->csr, s->nbuf, s->buf[0], s->buf[1], s->ctl, s->rank_part,
                                    s->ctx->nranks, s->my_part, s->blk_part, s->trace, s->parity, s->grid));
        // launch t wrote y_t into buf[t & 1]: halo exchange + all-gather of the rank partials
        return dist_exchange(s->csr, s->buf[s->parity], s->rank_part);
    }
    if (s->csr)
        return csr_power_launch(s->csr, s->nbuf, s->buf[0], s->buf[1], s->ctl, s->rank_part,
                                s->ctx->nranks, s->my_part, s->blk_part, s->trace, s->parity, s->grid);
    return dense_power_launch(s->dense, s->buf[0], s->buf[1], s->ctl, s->rank_part, s->ctx->nranks,
                              s->my_part, s->blk_part, s->trace, s->parity, s->grid);
}

static int pull_ctl(eigsol_power* s) {
    EIGSOL_HIP(hipMemcpyAsync(s->host_ctl, s->ctl, sizeof(PowerCtl), hipMemcpyDeviceToHost, s->ctx->stream));
    EIGSOL_HIP(hipStreamSynchronize(s->ctx->stream));
    return EIGSOL_OK;
}

extern "C" {

int eigsol_power_create_csr(eigsol_csr* A, int32_t trace_capacity, eigsol_power** out) {
    if (!A || !out) return fail(EIGSOL_E_INVALID, "eigsol_power_create_csr: null pointer");
    *out = nullptr;
    if (!A->dist && A->nrows != A->ncols) return fail(EIGSOL_E_NOT_SQUARE, "powerMethod: matrix must be square");
    if (A->dist ? A->n_global == 0 : A->nrows == 0) return fail(EIGSOL_E_ZERO_SIZE, "powerMethod: matrix has zero size");
    auto* s = new eigsol_power();
    s->ctx = A->ctx;
    s->csr = A;
    s->dist = A->dist != 0;
    s->xoff = A->xoff;
    csr_retain(A);
    s->dtype = A->dtype;
    s->n = A->nrows;
    s->nbuf = A->ncols;
    int rc = csr_grid(A, &s->grid);
    if (rc == EIGSOL_OK) rc = session_alloc(s, trace_capacity);
    if (rc != EIGSOL_OK) { session_free(s); return rc; }
    *out = s;
    return EIGSOL_OK;
}

int eigsol_power_create_dense(eigsol_dense* A, int32_t trace_capacity, eigsol_power** out) {
    if (!A || !out) return fail(EIGSOL_E_INVALID, "eigsol_power_create_dense: null pointer");
    *out = nullptr;
    if (A->nrows != A->ncols) return fail(EIGSOL_E_NOT_SQUARE, "powerMethod: matrix must be square");
    if (A->nrows == 0) return fail(EIGSOL_E_ZERO_SIZE, "powerMethod: matrix has zero size");
    auto* s = new eigsol_power();
    s->ctx = A->ctx;
    s->dense = A;
    dense_retain(A);
    s->dtype = A->dtype;
    s->n = A->nrows;
    s->nbuf = A->ncols;
    int rc = dense_grid(A, &s->grid);
    if (rc == EIGSOL_OK) rc = session_alloc(s, trace_capacity);
    if (rc != EIGSOL_OK) { session_free(s); return rc; }
    *out = s;
    return EIGSOL_OK;
}

int eigsol_power_destroy(eigsol_power* s) {
    session_free(s);
    return EIGSOL_OK;
}

int eigsol_power_begin(eigsol_power* s, const eigsol_solver_options* opts, const void* x0,
                       int x0_on_device) {
    if (!s || !opts || !x0) return fail(EIGSOL_E_INVALID, "eigsol_power_begin: null pointer");
    EIGSOL_HIP(hipSetDevice(s->ctx->device));
    hipStream_t st = s->ctx->stream;
    const size_t sb = scalar_bytes(s->dtype);
    s->opts = *opts;
    s->trivial = opts->max_iterations <= 0;
    // y_{-1} = x0 lives in buf[1] (launch t reads buf[(t-1)&1]); own rows at x-space offset xoff
    char* x0dst = static_cast<char*>(s->buf[1]) + (size_t)s->xoff * sb;
    EIGSOL_HIP(hipMemcpyAsync(x0dst, x0, s->n * sb,
                              x0_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
    PowerCtl init;
    std::memset(&init, 0, sizeof(init));
    init.max_iter = opts->max_iterations;
    init.tol = opts->tolerance;
    init.trace_cap = s->trace_cap;
    init.nranks = s->ctx->nranks;
    init.st[0].t = -1;
    init.st[1].t = -1;
    std::memcpy(s->host_ctl, &init, sizeof(init));
    EIGSOL_HIP(hipMemcpyAsync(s->ctl, s->host_ctl, sizeof(PowerCtl), hipMemcpyHostToDevice, st));
    // ||x0||^2 partials -> the input norm of launch 0 (x.normalize(), power_method.hpp:62)
    EIGSOL_TRY(norm_partial_launch(s->ctx, s->dtype, x0dst, s->n, s->ctl, s->blk_part, s->my_part, s->grid));
    if (s->dist) EIGSOL_TRY(dist_exchange(s->csr, s->buf[1], s->rank_part));   // x0 ghosts + partials
    EIGSOL_HIP(hipStreamSynchronize(st));   // host_ctl is reused by query()
    s->parity = 0;
    s->launches = 0;
    s->begun = true;
    return EIGSOL_OK;
}

int eigsol_power_step(eigsol_power* s, int32_t nsteps) {
    if (!s || !s->begun) return fail(EIGSOL_E_INVALID, "eigsol_power_step: session not begun");
    if (s->trivial) return EIGSOL_OK;
    EIGSOL_HIP(hipSetDevice(s->ctx->device));
    for (int32_t i = 0; i < nsteps; ++i) {
        EIGSOL_TRY(launch_iteration(s));
        s->parity ^= 1;
        ++s->launches;
    }
    return EIGSOL_OK;
}

int eigsol_power_query(eigsol_power* s, int32_t* done, int32_t* launches) {
    if (!s || !s->begun) return fail(EIGSOL_E_INVALID, "eigsol_power_query: session not begun");
    if (s->trivial) {
        if (done) *done = 1;
        if (launches) *launches = 0;
        return EIGSOL_OK;
    }
    EIGSOL_HIP(hipSetDevice(s->ctx->device));
    EIGSOL_TRY(pull_ctl(s));
    if (s->shift) EIGSOL_TRY(shift_error(s->shift));
    if (done) *done = s->host_ctl->done;
    if (launches) *launches = s->host_ctl->launches;
    return EIGSOL_OK;
}

int eigsol_power_finish(eigsol_power* s, void* lambda_out, void* x_out, int x_out_on_device,
                        int32_t* iterations, int32_t* converged) {
    if (!s || !s->begun) return fail(EIGSOL_E_INVALID, "eigsol_power_finish: session not begun");
    EIGSOL_HIP(hipSetDevice(s->ctx->device));
    hipStream_t st = s->ctx->stream;
    const size_t sb = scalar_bytes(s->dtype);
    double lam[2] = {0.0, 0.0};
    int parity = 1;
    double fnorm = 0.0;
    int32_t it = 0, conv = 0;
    if (s->trivial) {
        // maxIterations <= 0: lambda = 0, x = normalised x0, 0 iterations (power_method.hpp:61-68)
        const int P = s->dist ? s->ctx->nranks : 1;
        std::vector<double> part(4 * P);
        EIGSOL_HIP(hipMemcpyAsync(part.data(), s->rank_part, sizeof(double) * 4 * P, hipMemcpyDeviceToHost, st));
        EIGSOL_HIP(hipStreamSynchronize(st));
        double n2 = 0.0;
        for (int r = 0; r < P; ++r) n2 += part[4 * r];   // rank order, as on the device
        fnorm = std::sqrt(n2);
        parity = 1;
    } else {
        EIGSOL_TRY(pull_ctl(s));
        if (!s->host_ctl->done)
            return fail(EIGSOL_E_INVALID, "eigsol_power_finish: iteration has not terminated");
        lam[0] = s->host_ctl->lam_re;
        lam[1] = s->host_ctl->lam_im;
        parity = s->host_ctl->final_parity;
        fnorm = s->host_ctl->final_norm;
        it = s->host_ctl->iters;
        conv = s->host_ctl->converged;
    }
    if (lambda_out) std::memcpy(lambda_out, lam, sb);
    if (iterations) *iterations = it;
    if (converged) *converged = conv;
    if (x_out) {
        void* src = static_cast<char*>(s->buf[parity]) + (size_t)s->xoff * sb;
        if (x_out_on_device) {
            EIGSOL_TRY(scale_out_launch(s->ctx, s->dtype, src, fnorm, x_out, s->n));
            EIGSOL_HIP(hipStreamSynchronize(st));
        } else {
            void* tmp = s->buf[parity ^ 1];
            EIGSOL_TRY(scale_out_launch(s->ctx, s->dtype, src, fnorm, tmp, s->n));
            EIGSOL_HIP(hipMemcpyAsync(x_out, tmp, s->n * sb, hipMemcpyDeviceToHost, st));
            EIGSOL_HIP(hipStreamSynchronize(st));
        }
    }
    return EIGSOL_OK;
}

int eigsol_power_trace(eigsol_power* s, void* trace_host, int32_t capacity, int32_t* count) {
    if (!s || !s->begun) return fail(EIGSOL_E_INVALID, "eigsol_power_trace: session not begun");
    int32_t n = 0;
    if (!s->trivial && s->trace) {
        EIGSOL_TRY(pull_ctl(s));
        n = s->host_ctl->ntrace;
        n = std::min(n, s->trace_cap);
        if (trace_host && capacity > 0) {
            const int32_t m = std::min(n, capacity);
            EIGSOL_HIP(hipMemcpy(trace_host, s->trace, (size_t)m * scalar_bytes(s->dtype), hipMemcpyDeviceToHost));
        }
    }
    if (count) *count = n;
    return EIGSOL_OK;
}

int eigsol_power_kernel_info(eigsol_power* s, double* bytes, int32_t* grid, int32_t* tiles,
                             int32_t* variant) {
    if (!s) return fail(EIGSOL_E_INVALID, "eigsol_power_kernel_info: null session");
    const double sb = (double)scalar_bytes(s->dtype);
    if (s->shift) {
        shift_info(s->shift, bytes, variant, tiles);
    } else if (s->csr) {
        // values + int32 columns + int32 row pointers + x read once + y written once
        const double nnz = (double)s->csr->nnz, n = (double)s->csr->nrows;
        if (bytes) *bytes = (sb + 4.0) * nnz + 4.0 * (n + 1.0) + 2.0 * sb * n;
        if (tiles) *tiles = s->csr->sliced ? s->csr->nslices : s->csr->ntiles;
        if (variant) *variant = s->csr->sliced ? 5 : (s->csr->windowed ? 1 : 0);
    } else {
        const double n = (double)s->dense->nrows;
        if (bytes) *bytes = sb * n * n + 2.0 * sb * n;
        if (tiles) *tiles = 0;
        if (variant) *variant = 2;
    }
    if (grid) *grid = s->grid;
    return EIGSOL_OK;
}

// One-shot solves: begin / step in doubling chunks until the device reports termination / finish.
static int run_to_completion(eigsol_power* s, const eigsol_solver_options* opts, const void* x0,
                             void* lambda_out, void* x_out, int32_t* iterations, int32_t* converged) {
    EIGSOL_TRY(eigsol_power_begin(s, opts, x0, 0));
    if (!s->trivial) {
        // Upper bound on launches: maxIterations + 2 (launch maxIter+1 only decides).
        const int64_t cap = (int64_t)opts->max_iterations + 2;
        int64_t issued = 0;
        int32_t chunk = 4;
        int32_t done = 0;
        while (!done) {
            const int32_t k = (int32_t)std::min<int64_t>(chunk, std::max<int64_t>(1, cap - issued));
            EIGSOL_TRY(eigsol_power_step(s, k));
            issued += k;
            EIGSOL_TRY(eigsol_power_query(s, &done, nullptr));
            chunk = std::min(chunk * 2, 64);
            if (!done && issued >= cap + 4)
                return fail(EIGSOL_E_SOLVER, "power iteration did not terminate (internal error)");
        }
    }
    return eigsol_power_finish(s, lambda_out, x_out, 0, iterations, converged);
}

int eigsol_power_csr(eigsol_csr* A, const eigsol_solver_options* opts, const void* x0,
                     void* lambda_out, void* x_out, int32_t* iterations, int32_t* converged) {
    if (!opts || !x0) return fail(EIGSOL_E_INVALID, "eigsol_power_csr: null opts/x0");
    eigsol_power* s = nullptr;
    EIGSOL_TRY(eigsol_power_create_csr(A, 0, &s));
    const int rc = run_to_completion(s, opts, x0, lambda_out, x_out, iterations, converged);
    session_free(s);
    return rc;
}

int eigsol_power_dense(eigsol_dense* A, const eigsol_solver_options* opts, const void* x0,
                       void* lambda_out, void* x_out, int32_t* iterations, int32_t* converged) {
    if (!opts || !x0) return fail(EIGSOL_E_INVALID, "eigsol_power_dense: null opts/x0");
    eigsol_power* s = nullptr;
    EIGSOL_TRY(eigsol_power_create_dense(A, 0, &s));
    const int rc = run_to_completion(s, opts, x0, lambda_out, x_out, iterations, converged);
    session_free(s);
    return rc;
}


// ---------------------------------------------------------------- shifted inverse iteration
// shiftedInversePowerMethod<S> (shifted_inverse_power_solver.hpp:112-125): the session factors
// A - sigma I once at creation and runs one fused solve launch per iteration.
static int shifted_create(eigsol_ctx* ctx, eigsol_csr* csr, eigsol_dense* dense, int dtype,
                          int64_t n, const void* sigma, int32_t trace_capacity, eigsol_power** out) {
    auto* s = new eigsol_power();
    s->ctx = ctx;
    s->dtype = dtype;
    s->n = n;
    s->nbuf = n;
    int rc = csr ? shift_factor_csr(csr, sigma, &s->shift) : shift_factor_dense(dense, sigma, &s->shift);
    if (rc == EIGSOL_OK) {
        if (csr) { s->csr = csr; csr_retain(csr); }
        else { s->dense = dense; dense_retain(dense); }
        s->grid = std::max(64, shift_grid(s->shift));
        rc = session_alloc(s, trace_capacity);
    }
    if (rc != EIGSOL_OK) { session_free(s); return rc; }
    *out = s;
    return EIGSOL_OK;
}

int eigsol_shifted_create_csr(eigsol_csr* A, const void* sigma, int32_t trace_capacity, eigsol_power** out) {
    if (!A || !sigma || !out) return fail(EIGSOL_E_INVALID, "eigsol_shifted_create_csr: null pointer");
    *out = nullptr;
    if (A->dist || A->nrows != A->ncols)
        return fail(EIGSOL_E_NOT_SQUARE, "shiftedInversePowerMethod: matrix must be square");
    if (A->nrows == 0) return fail(EIGSOL_E_ZERO_SIZE, "shiftedInversePowerMethod: matrix has zero size");
    return shifted_create(A->ctx, A, nullptr, A->dtype, A->nrows, sigma, trace_capacity, out);
}

int eigsol_shifted_create_dense(eigsol_dense* A, const void* sigma, int32_t trace_capacity, eigsol_power** out) {
    if (!A || !sigma || !out) return fail(EIGSOL_E_INVALID, "eigsol_shifted_create_dense: null pointer");
    *out = nullptr;
    if (A->nrows != A->ncols) return fail(EIGSOL_E_NOT_SQUARE, "shiftedInversePowerMethod: matrix must be square");
    if (A->nrows == 0) return fail(EIGSOL_E_ZERO_SIZE, "shiftedInversePowerMethod: matrix has zero size");
    return shifted_create(A->ctx, nullptr, A, A->dtype, A->nrows, sigma, trace_capacity, out);
}

int eigsol_shifted_inverse_csr(eigsol_csr* A, const void* sigma, const eigsol_solver_options* opts,
                               const void* x0, void* lambda_out, void* x_out, int32_t* iterations,
                               int32_t* converged) {
    if (!opts || !x0) return fail(EIGSOL_E_INVALID, "eigsol_shifted_inverse_csr: null opts/x0");
    eigsol_power* s = nullptr;
    EIGSOL_TRY(eigsol_shifted_create_csr(A, sigma, 0, &s));
    const int rc = run_to_completion(s, opts, x0, lambda_out, x_out, iterations, converged);
    session_free(s);
    return rc;
}

int eigsol_shifted_inverse_dense(eigsol_dense* A, const void* sigma, const eigsol_solver_options* opts,
                                 const void* x0, void* lambda_out, void* x_out, int32_t* iterations,
                                 int32_t* converged) {
    if (!opts || !x0) return fail(EIGSOL_E_INVALID, "eigsol_shifted_inverse_dense: null opts/x0");
    eigsol_power* s = nullptr;
    EIGSOL_TRY(eigsol_shifted_create_dense(A, sigma, 0, &s));
    const int rc = run_to_completion(s, opts, x0, lambda_out, x_out, iterations, converged);
    session_free(s);
    return rc;
}

// solve_shifted<S> (solve_shifted.hpp:48-118): x = (A - sigma I)^{-1} b, host buffers.
static int solve_once(ShiftFactor* f, eigsol_ctx* ctx, size_t sb, int64_t n, const void* b, void* x) {
    void* d = nullptr;
    EIGSOL_HIP(hipMalloc(&d, 2 * n * sb));
    char* bd = static_cast<char*>(d);
    char* yd = bd + n * sb;
    int rc = EIGSOL_OK;
    if (hipMemcpyAsync(bd, b, n * sb, hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "solve_shifted: upload");
    if (rc == EIGSOL_OK) rc = shift_solve_launch(f, bd, yd);
    if (rc == EIGSOL_OK && hipMemcpyAsync(x, yd, n * sb, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "solve_shifted: download");
    if (rc == EIGSOL_OK && hipStreamSynchronize(ctx->stream) != hipSuccess)
        rc = fail(EIGSOL_E_HIP, "solve_shifted: synchronize");
    if (rc == EIGSOL_OK) rc = shift_error(f);
    hipFree(d);
    return rc;
}

int eigsol_solve_shifted_csr(eigsol_csr* A, const void* sigma, const void* b, int64_t nb, void* x) {
    if (!A || !sigma || !b || !x) return fail(EIGSOL_E_INVALID, "eigsol_solve_shifted_csr: null pointer");
    if (A->dist || A->nrows != A->ncols)
        return fail(EIGSOL_E_NOT_SQUARE, "solve_shifted: A must be square (sparse case)");
    if (A->nrows != nb)
        return fail(EIGSOL_E_SIZE_MISMATCH, "solve_shifted: size mismatch between A and b (sparse case)");
    if (nb == 0) return EIGSOL_OK;
    EIGSOL_HIP(hipSetDevice(A->ctx->device));
    ShiftFactor* f = nullptr;
    EIGSOL_TRY(shift_factor_csr(A, sigma, &f));
    const int rc = solve_once(f, A->ctx, scalar_bytes(A->dtype), nb, b, x);
    shift_factor_free(f);
    return rc;
}

int eigsol_solve_shifted_dense(eigsol_dense* A, const void* sigma, const void* b, int64_t nb, void* x) {
    if (!A || !sigma || !b || !x) return fail(EIGSOL_E_INVALID, "eigsol_solve_shifted_dense: null pointer");
    if (A->nrows != A->ncols) return fail(EIGSOL_E_NOT_SQUARE, "solve_shifted: A must be square (dense case)");
    if (A->nrows != nb)
        return fail(EIGSOL_E_SIZE_MISMATCH, "solve_shifted: size mismatch between A and b (dense case)");
    if (nb == 0) return EIGSOL_OK;
    EIGSOL_HIP(hipSetDevice(A->ctx->device));
    ShiftFactor* f = nullptr;
    EIGSOL_TRY(shift_factor_dense(A, sigma, &f));
    const int rc = solve_once(f, A->ctx, scalar_bytes(A->dtype), nb, b, x);
    shift_factor_free(f);
    return rc;
}

}  // extern "C"

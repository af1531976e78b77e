// Nested-dissection multifrontal LU of the general-sparse shifted solve (multifrontal.hip): host
// interface.  Used by gmres.hip as the exact factor K of M = A - sigma I where the natural-order
// symbolic LU passes its fill cap (round 5: the permuted 1M convection-diffusion matrix).
#pragma once

#include <atomic>
#include <vector>

#include "internal.hpp"

namespace eigsol {

struct MfFactor;

struct MfStats {
    int64_t fronts = 0, heights = 0, max_front = 0, max_pivots = 0;
    double factor_entries = 0.0;   // stored L and U entries (the fronts' pivot rows and columns)
    double front_entries = 0.0;    // sum of d^2 over the fronts (device workspace)
    double flops = 0.0;            // real flops of the numeric factorization (estimate)
    double order_seconds = 0.0;    // host: nested dissection + symbolic structure
    double numeric_seconds = 0.0;  // device: assembly + partial factorizations (synchronised)
    double solve_bytes = 0.0;      // algorithmic bytes of one solve (factor entries + vectors)
};

struct MfHost;   // the host half of a factor (ordering, symbolic structure, launch tables)
MfHost* mf_host_new();
void mf_host_free(MfHost* X);
const MfStats& mf_host_stats(const MfHost* X);   // after a successful mf_prepare
// Host only (thread-safe, no device call): the plan for the pattern of M (n x n, CSR with sorted
// rows and every diagonal stored), dtype EIGSOL_F64 or EIGSOL_C128, its fronts bounded by
// free_bytes of device memory.  EIGSOL_OK, or EIGSOL_E_UNSUPPORTED when the plan exceeds its
// bounds (memory, LDS, work; no error text is kept) or *stop was raised while it ran.
int mf_prepare(int64_t n, const std::vector<int32_t>& rp, const std::vector<int32_t>& ci, int dtype, double free_bytes,
               MfHost* X, const std::atomic<bool>* stop = nullptr);
// The device half on a prepared plan with M's values: EIGSOL_OK with *out, EIGSOL_E_SOLVER on a
// zero pivot, EIGSOL_E_UNSUPPORTED when a front buffer cannot be allocated, or EIGSOL_E_HIP.
// static_pivot > 0: a pivot column that is exactly zero in every remaining row of its front (its
// pivot would have to come from outside the front) gets static_pivot on the diagonal instead - a
// perturbation of M (*nstatic counts them) that the caller's checked solve refines away.
int mf_create(eigsol_ctx* ctx, int dtype, MfHost* X, const void* v, MfFactor** out, double static_pivot = 0.0,
              int64_t* nstatic = nullptr);
// x = M^-1 b (device vectors, the caller's numbering), stream-ordered on ctx's stream
int mf_solve(MfFactor* f, const void* b, void* x);
void mf_free(MfFactor* f);
// device word a solve's flag / value waits set when one gives up (bounded spin): non-zero = broken solve
const int32_t* mf_err_word(const MfFactor* f);
const MfStats& mf_stats(const MfFactor* f);

}  // namespace eigsol

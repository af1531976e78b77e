// Nested-dissection multifrontal LU of the general-sparse shifted solve (multifrontal.hip): host
// interface.  Used by gmres.hip as the exact factor K of M = A - sigma I where the natural-order
// symbolic LU passes its fill cap (round 5: the permuted 1M convection-diffusion matrix).
#pragma once

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

// M (n x n, CSR with sorted rows and every diagonal stored; values S = double or cplx per dtype).
// Returns EIGSOL_OK with *out, EIGSOL_E_UNSUPPORTED when the plan exceeds its bounds (memory,
// LDS, work; the caller keeps another path; no error text is kept), EIGSOL_E_SOLVER on a zero
// pivot, or EIGSOL_E_HIP.
int mf_create(eigsol_ctx* ctx, int dtype, int64_t n, const std::vector<int32_t>& rp, const std::vector<int32_t>& ci,
              const void* v, MfFactor** out);
// x = M^-1 b (device vectors, the caller's numbering), stream-ordered on ctx's stream
int mf_solve(MfFactor* f, const void* b, void* x);
void mf_free(MfFactor* f);
const MfStats& mf_stats(const MfFactor* f);

}  // namespace eigsol

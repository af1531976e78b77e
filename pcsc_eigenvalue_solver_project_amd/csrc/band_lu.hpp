// Banded direct LU of the general-sparse shifted solve (band_lu.hip): host interface.
#pragma once

#include <vector>

#include "internal.hpp"

namespace eigsol {

struct BandPlan {
    std::vector<int32_t> perm;   // new -> old (reverse Cuthill-McKee, or the given order if as narrow)
    int64_t kl = 0, ku = 0;      // bandwidths of P M P^T (M = A with its diagonal)
    int nb = 64;                 // panel width (the rank-NB update's K)
    int64_t ldab = 0;            // stored rows per column (band + fill + panel padding)
    int32_t ring = 0;            // LDS ring entries of the solve kernel (power of two)
    double bytes = 0.0;          // device bytes of the band factor
    bool ok = false;             // the solve kernel's LDS ring holds the kl + (kl + ku) + 2 NB window
};

struct BandFactor;
void band_plan(int dtype, int64_t n, const int32_t* rp, const int32_t* ci, BandPlan& plan);
int band_create(eigsol_ctx* ctx, int dtype, int64_t n, const int32_t* rp, const int32_t* ci, const void* v,
                double sre, double sim, BandPlan& plan, BandFactor** out);
void band_free(BandFactor* f);
int band_launch(BandFactor* f, bool iter, const void* b, void* y, void* buf0, void* buf1, PowerCtl* ctl,
                const void* rank_part, void* my_part, void* trace, int parity);
void band_info(const BandFactor* f, double* bytes, int32_t* tiles);

}  // namespace eigsol

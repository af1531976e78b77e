// Device primitives of the triangular factor's on-device analysis (shifted.hip, factor_tri_device):
// a stable sort of the rows by dependency level and an exclusive scan of the per-position entry
// counts.  rocPRIM's device-wide radix sort and decoupled-lookback scan, kept in their own
// translation unit (heavy templates).
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <cstdint>

namespace eigsol {

// rows_out = the rows 0..n-1 ordered by level ascending, ascending row index inside a level (LSD
// radix sort is stable, and the values enter in row order); lev_out = their levels.  Levels lie in
// [0, 2^bits).
hipError_t tri_sort_rows_by_level(hipStream_t st, const int32_t* lev, int32_t* lev_out, int32_t* rows_out, int64_t n,
                                  int bits) {
    if (n <= 0) return hipSuccess;
    rocprim::counting_iterator<int32_t> rows(0);
    size_t bytes = 0;
    hipError_t e = rocprim::radix_sort_pairs(nullptr, bytes, lev, lev_out, rows, rows_out, (size_t)n, 0u,
                                             (unsigned)bits, st);
    if (e != hipSuccess) return e;
    void* tmp = nullptr;
    if ((e = hipMallocAsync(&tmp, bytes, st)) != hipSuccess) return e;
    e = rocprim::radix_sort_pairs(tmp, bytes, lev, lev_out, rows, rows_out, (size_t)n, 0u, (unsigned)bits, st);
    const hipError_t e2 = hipFreeAsync(tmp, st);
    return e != hipSuccess ? e : e2;
}

// out[0..n] = exclusive prefix sums of in[0..n) with out[n] = the total (in[n] must be 0: the scan
// runs over n + 1 entries)
hipError_t tri_exclusive_scan(hipStream_t st, const int32_t* in, int32_t* out, int64_t n) {
    size_t bytes = 0;
    hipError_t e = rocprim::exclusive_scan(nullptr, bytes, in, out, int32_t(0), (size_t)n + 1, rocprim::plus<int32_t>(),
                                           st);
    if (e != hipSuccess) return e;
    void* tmp = nullptr;
    if ((e = hipMallocAsync(&tmp, bytes, st)) != hipSuccess) return e;
    e = rocprim::exclusive_scan(tmp, bytes, in, out, int32_t(0), (size_t)n + 1, rocprim::plus<int32_t>(), st);
    const hipError_t e2 = hipFreeAsync(tmp, st);
    return e != hipSuccess ? e : e2;
}

}  // namespace eigsol

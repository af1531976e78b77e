/*
 * eigsol_hip.h — C ABI of the MI355X (gfx950) eigenvalue-solver hot path.
 *
 * This is the drop-in boundary for hugoheziyang/PCSC_Eigenvalue_Solver_Project.  The reference has
 * no FFI: its boundary is the header-only C++ template API, and the seam is the dense/sparse
 * dispatch inside each entry point.  Every function below replaces the numeric core behind one of
 * those seams (file:line in the reference):
 *
 *   powerMethod<S>                 src/power_method/power_method.hpp:135-148 (impl :47-99)
 *   shiftedInversePowerMethod<S>   src/power_method/shifted_inverse_power_solver.hpp:112-125 (impl :21-79)
 *   solve_shifted<S>               src/matrix/solve_shifted.hpp:48-118
 *   to_hessenberg<S>               src/qr_method/to_hessenberg.hpp:99-119 (impl :23-80)
 *   qr_eigenvalues<S>              src/qr_method/qr_eigenvalues.hpp:126-147 (impl :40-108)
 *   Matrix (dense / sparse store)  src/matrix/matrix.hpp:36-246
 *
 * The C++ drop-in façade (include/eigsol/...) keeps the reference's names, signatures and
 * exception messages and calls only this ABI.  Plain pointers and sizes; no torch / HIP types in
 * the signatures (streams are passed as void*).  Every call returns an eigsol_status; the
 * detail string of the last failure on the calling thread is eigsol_last_error().
 *
 * Scalars: EIGSOL_F64 = double, EIGSOL_C128 = std::complex<double> / double _Complex
 * (interleaved re, im), EIGSOL_F32 = float, EIGSOL_C64 = std::complex<float> (single-precision
 * paths listed at eigsol_dtype), EIGSOL_DD / EIGSOL_CDD = long double / std::complex<long double>
 * carried as double-double (see eigsol_dtype).  Dense storage is column-major (Matrix::Dense is an Eigen col-major
 * matrix, matrix.hpp:39-40).  Sparse storage is CSR with int32 indices on the device; the CSC
 * constructor accepts the reference's canonical Eigen::SparseMatrix<S> (ColMajor, int) layout
 * (matrix.hpp:43-44).
 */
#ifndef EIGSOL_HIP_H
#define EIGSOL_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EIGSOL_ABI_VERSION 1

typedef enum eigsol_status {
    EIGSOL_OK = 0,
    EIGSOL_E_NOT_SQUARE = 1,      /* "...: matrix must be square"   power_method.hpp:54 */
    EIGSOL_E_ZERO_SIZE = 2,       /* "...: matrix has zero size"    power_method.hpp:57 */
    EIGSOL_E_SCALAR_MISMATCH = 3, /* "...: scalar type mismatch"    power_method.hpp:138 */
    EIGSOL_E_SIZE_MISMATCH = 4,   /* size mismatch between A and b  solve_shifted.hpp:71 */
    EIGSOL_E_NOT_DENSE = 5,       /* "only dense matrices"          qr_eigenvalues.hpp:132 */
    EIGSOL_E_SOLVER = 6,          /* factorisation failed           solve_shifted.hpp:109 */
    EIGSOL_E_HIP = 7,             /* HIP runtime error */
    EIGSOL_E_RCCL = 8,            /* RCCL error */
    EIGSOL_E_INVALID = 9,         /* invalid argument (null pointer, malformed CSR, ...) */
    EIGSOL_E_NO_DEVICE = 10,      /* no usable gfx950 device */
    EIGSOL_E_EMPTY = 11,          /* "empty matrix"                 qr_decompose.hpp:39 */
    EIGSOL_E_UNSUPPORTED = 12     /* structure not supported by the device path */
} eigsol_status;

/* EIGSOL_F32 / EIGSOL_C64: float and std::complex<float> (ScalarConcept, types.hpp:28-30), stored
 * and multiplied in single precision on the device (CSR / dense power iteration, plain SpMV/GEMV,
 * triangular-CSR shifted inverse).  Other solvers accept only F64 / C128 (the C++ façade promotes
 * float input for those).
 * EIGSOL_DD / EIGSOL_CDD: long double and std::complex<long double> (types.hpp:28-30; the x87
 * 80-bit format, 64-bit significand, under g++ on x86-64).  A value is a double-double: two doubles
 * {hi, lo} whose unevaluated sum is the value, |lo| <= ulp(hi)/2 (106-bit significand); complex
 * values are {re.hi, re.lo, im.hi, im.lo}.  Every finite long double inside the double exponent
 * range converts exactly (hi = (double)v, lo = (double)(v - hi)).  Computed in double-double on the
 * device: CSR / dense products, the power method, the shifted inverse and solve_shifted (the fp64
 * factor of A - sigma I refined to double-double accuracy by residuals computed in double-double),
 * to_hessenberg, qr_decompose and the reference's unshifted qr_eigenvalues; the Francis variant
 * runs the fp64 sweeps and refines every eigenvalue in double-double (eigsol_qr_eigenvalues_dense);
 * the row-sharded path returns EIGSOL_E_UNSUPPORTED. */
typedef enum eigsol_dtype {
    EIGSOL_F64 = 0,
    EIGSOL_C128 = 1,
    EIGSOL_F32 = 2,
    EIGSOL_C64 = 3,
    EIGSOL_DD = 4,
    EIGSOL_CDD = 5
} eigsol_dtype;

/* SolverOptions (src/option/solver_option.hpp:14-20). */
typedef struct eigsol_solver_options {
    int32_t max_iterations; /* default 1000 */
    double tolerance;       /* default 1e-10; |a-b| <= tol*(1+|a|), tolerance.hpp:28-33 */
} eigsol_solver_options;

typedef struct eigsol_ctx eigsol_ctx;     /* one device + one stream (+ optional RCCL communicator) */
typedef struct eigsol_csr eigsol_csr;     /* device-resident CSR matrix (rows of one rank)          */
typedef struct eigsol_dense eigsol_dense; /* device-resident column-major dense matrix             */
typedef struct eigsol_power eigsol_power; /* device-resident power-iteration session               */

/* ---------------------------------------------------------------- library / context */
int eigsol_abi_version(void);
const char* eigsol_status_string(int status);
const char* eigsol_last_error(void);
int eigsol_device_count(int* count);
int eigsol_ctx_create(int device, eigsol_ctx** out);
int eigsol_ctx_destroy(eigsol_ctx* ctx);
/* Use the caller's hipStream_t (NULL = the context's own stream).  All work is stream-ordered. */
int eigsol_ctx_set_stream(eigsol_ctx* ctx, void* hip_stream);
int eigsol_ctx_get_stream(eigsol_ctx* ctx, void** hip_stream);
int eigsol_ctx_synchronize(eigsol_ctx* ctx);

/* ---------------------------------------------------------------- device memory helpers */
int eigsol_malloc(eigsol_ctx* ctx, size_t bytes, void** dptr);
int eigsol_free(eigsol_ctx* ctx, void* dptr);
int eigsol_memcpy_h2d(eigsol_ctx* ctx, void* dst, const void* src, size_t bytes);
int eigsol_memcpy_d2h(eigsol_ctx* ctx, void* dst, const void* src, size_t bytes);

/* ---------------------------------------------------------------- matrices (host in, HBM resident) */
/* CSR: rowptr[nrows+1], colidx[nnz] (0-based, < ncols), values[nnz].  Columns inside a row are
 * sorted ascending on upload (the reference's CSC product sums each row in ascending column
 * order, power_method.hpp:69).  Requires nnz < 2^31 (Eigen StorageIndex = int). */
int eigsol_csr_create(eigsol_ctx* ctx, eigsol_dtype dtype, int64_t nrows, int64_t ncols,
                      int64_t nnz, const int32_t* rowptr, const int32_t* colidx,
                      const void* values, eigsol_csr** out);
/* CSC (Eigen::SparseMatrix<S> compressed storage: outer = column pointers). */
int eigsol_csr_create_from_csc(eigsol_ctx* ctx, eigsol_dtype dtype, int64_t nrows, int64_t ncols,
                               int64_t nnz, const int32_t* colptr, const int32_t* rowidx,
                               const void* values, eigsol_csr** out);
/* COO triplets (row[k], col[k], values[k]) in any order, the text reader's sparse entries
 * (file_matrix_reader.hpp:84-132, "row col value" lines): ordered by (row, column) into CSR
 * directly, with no CSC step; repeated positions are summed in input order (what Matrix::Sparse's
 * compression does with repeated insert()s). */
int eigsol_csr_create_from_coo(eigsol_ctx* ctx, eigsol_dtype dtype, int64_t nrows, int64_t ncols,
                               int64_t nnz, const int32_t* rowidx, const int32_t* colidx,
                               const void* values, eigsol_csr** out);
/* Copy the device CSR back (rowptr[nrows+1], colidx[nnz], values[nnz]; columns ascending within
 * each row, duplicates already summed).  Single-device matrices only. */
int eigsol_csr_download(eigsol_csr* A, int32_t* rowptr, int32_t* colidx, void* values);
int eigsol_csr_destroy(eigsol_csr* A);
int eigsol_csr_info(eigsol_csr* A, int64_t* nrows, int64_t* ncols, int64_t* nnz, int* dtype);
/* y = A*x on device buffers (x: ncols scalars, y: nrows scalars), stream-ordered.  Each row is an
 * ascending-column sequential sum of products: bitwise equal to the reference's CSC scatter. */
int eigsol_csr_spmv(eigsol_csr* A, const void* x_dev, void* y_dev);

/* Dense, column-major nrows x ncols (Matrix::Dense<S>). */
int eigsol_dense_create(eigsol_ctx* ctx, eigsol_dtype dtype, int64_t nrows, int64_t ncols,
                        const void* colmajor, eigsol_dense** out);
int eigsol_dense_destroy(eigsol_dense* A);
int eigsol_dense_gemv(eigsol_dense* A, const void* x_dev, void* y_dev);

/* ---------------------------------------------------------------- power method
 * powerMethod<S>(M, opts) (power_method.hpp:135-148) with an explicit start vector x0 in place
 * of Vector<S>::Random (power_method.hpp:62; x0 is normalised by the library exactly as
 * x.normalize()).  The device runs ONE fused product per iteration: the reference's second
 * product x.dot(A*x) (:81) is the next iteration's y (:69), so the eigenvalue sequence is the
 * reference's.  Outputs mirror EigenResult<S> (eigen_result.hpp:22-52).
 * One-shot form: host buffers; lambda_out = 1 scalar, x_out = n scalars (either may be NULL). */
int eigsol_power_csr(eigsol_csr* A, const eigsol_solver_options* opts, const void* x0,
                     void* lambda_out, void* x_out, int32_t* iterations, int32_t* converged);
int eigsol_power_dense(eigsol_dense* A, const eigsol_solver_options* opts, const void* x0,
                       void* lambda_out, void* x_out, int32_t* iterations, int32_t* converged);

/* Session form (device-resident; what a caller with data already in HBM uses, and what the
 * benchmark times).  begin() normalises x0 and resets the state; step(k) enqueues k fused
 * iterations (launches after convergence exit immediately); query() synchronises and reports
 * whether the reference loop has terminated; finish() writes EigenResult fields.
 * trace_capacity > 0 records the Rayleigh quotient of every completed iteration on the device. */
int eigsol_power_create_csr(eigsol_csr* A, int32_t trace_capacity, eigsol_power** out);
int eigsol_power_create_dense(eigsol_dense* A, int32_t trace_capacity, eigsol_power** out);
int eigsol_power_destroy(eigsol_power* s);
int eigsol_power_begin(eigsol_power* s, const eigsol_solver_options* opts, const void* x0,
                       int x0_on_device);
int eigsol_power_step(eigsol_power* s, int32_t nsteps);
int eigsol_power_query(eigsol_power* s, int32_t* done, int32_t* launches);
int eigsol_power_finish(eigsol_power* s, void* lambda_out, void* x_out, int x_out_on_device,
                        int32_t* iterations, int32_t* converged);
int eigsol_power_trace(eigsol_power* s, void* trace_host, int32_t capacity, int32_t* count);
/* Device-side description of the hot kernel for roofline accounting: algorithmic bytes moved by
 * one fused iteration and the grid used. */
int eigsol_power_kernel_info(eigsol_power* s, double* bytes_per_iteration, int32_t* grid_blocks,
                             int32_t* tiles, int32_t* variant);
/* Demangled name of the kernel a CSR power session launches per iteration (e.g.
 * "void eigsol::dev::csr_slice_kernel<double, true, 12, false, false>(...)"), the string rocprofv3
 * reports; empty for other sessions. */
int eigsol_power_kernel_name(eigsol_power* s, char* buf, size_t capacity);
/* variant: 0 = CSR, x gathered from HBM; 1 = CSR, x window staged in LDS; 2 = dense GEMV;
 *          3 = shifted inverse, sync-free triangular solve (tiles = dependency levels);
 *          4 = shifted inverse, dense LU substitution;
 *          5 = CSR in 64-row slices, one row per lane (tiles = slices);
 *          6 = CSR one row per lane (single-precision fallback layout);
 *          7 = shifted inverse, ILU(0)-preconditioned GMRES (general sparse; bytes and tiles of the
 *              last solve: algorithmic bytes of all its steps, Arnoldi steps);
 *          8 = shifted inverse, RCM-banded direct LU (general sparse; tiles = kl + ku);
 *          15 = double-double CSR product (EIGSOL_DD / EIGSOL_CDD power method, one row per lane);
 *          16 = double-double dense GEMV (row tiles x column chunks);
 *          17 = double-double shifted inverse: fp64 factor + residual refinement in double-double
 *               (tiles = refinement steps of the last solve, bytes = all of its passes);
 *          18 = shifted inverse, general sparse: GMRES preconditioned by the exact sparse LU of
 *               A - sigma I (symbolic fill without pivoting, used when the filled pattern holds at most
 *               EIGSOL_LU_FILL_CAP x nnz entries; tiles and bytes as for 7) */

/* ---------------------------------------------------------------- shifted inverse iteration
 * shiftedInversePowerMethod<S>(M, ShiftedSolverOptions<S>{sigma, maxIter, tol})
 * (shifted_inverse_power_solver.hpp:112-125, impl :21-79).  A - sigma I is factored ONCE at
 * session creation (the reference refactors every iteration, solve_shifted.hpp:75-79,96-106):
 *   - triangular CSR (upper or lower; a missing diagonal counts as 0, solve_shifted.hpp:100-102):
 *     the matrix is its own factor; one sync-free level-ordered triangular solve per iteration;
 *   - non-triangular CSR: reverse Cuthill-McKee + banded partial-pivot LU on the device (a direct
 *     factor, like SparseLU) when the band fits; otherwise the densified partial-pivot LU up to
 *     n = 16384, and ILU(0) + restarted GMRES (1e-12 relative residual) above it.  A GMRES solve
 *     that stalls above 1e-10 falls back to the densified LU where it fits the device, else fails
 *     with EIGSOL_E_SOLVER ("solve_shifted: SparseLU solve failed (...)", solve_shifted.hpp:112-114).
 *     EIGSOL_SPARSE_SOLVER=band|lu|gmres forces a path, EIGSOL_GMRES_FALLBACK=0 disables the fallback;
 *   - dense: partial-pivot LU on the device.
 * sigma points at ONE scalar of the matrix dtype.  A zero pivot of a sparse matrix fails with
 * EIGSOL_E_SOLVER ("solve_shifted: SparseLU factorization failed", solve_shifted.hpp:108-110).
 * The returned handle is a session: use eigsol_power_begin/step/query/finish/trace/kernel_info.
 * lambda_k = x_{k+1}^H A x_{k+1} is evaluated as sigma + conj(x_k^H y_k)/||y_k||^2 (A y_k = x_k +
 * sigma y_k), so an iteration reads only the factor. */
int eigsol_shifted_create_csr(eigsol_csr* A, const void* sigma, int32_t trace_capacity,
                              eigsol_power** out);
int eigsol_shifted_create_dense(eigsol_dense* A, const void* sigma, int32_t trace_capacity,
                                eigsol_power** out);
int eigsol_shifted_inverse_csr(eigsol_csr* A, const void* sigma, const eigsol_solver_options* opts,
                               const void* x0, void* lambda_out, void* x_out, int32_t* iterations,
                               int32_t* converged);
int eigsol_shifted_inverse_dense(eigsol_dense* A, const void* sigma,
                                 const eigsol_solver_options* opts, const void* x0,
                                 void* lambda_out, void* x_out, int32_t* iterations,
                                 int32_t* converged);
/* solve_shifted<S>(M, sigma, b) (solve_shifted.hpp:48-118): x = (A - sigma I)^{-1} b, host
 * buffers of nb scalars.  Status mirrors the reference's exceptions: NOT_SQUARE, SIZE_MISMATCH,
 * SOLVER. */
int eigsol_solve_shifted_csr(eigsol_csr* A, const void* sigma, const void* b, int64_t nb, void* x);
int eigsol_solve_shifted_dense(eigsol_dense* A, const void* sigma, const void* b, int64_t nb,
                               void* x);

/* ---------------------------------------------------------------- QR method (dense)
 * Host column-major buffers in and out; the work runs on the context's device.
 * to_hessenberg_dense<S>   (to_hessenberg.hpp:23-80): H = Householder reduction of A (n x n).
 * qr_decompose_dense<S>    (qr_decompose.hpp:25-86):  A (m x n) = Q (m x m) R (m x n); m or n
 *                          == 0 fails with EIGSOL_E_EMPTY ("qr_decompose_dense: empty matrix").
 * qr_eigenvalues_dense<S>  (qr_eigenvalues.hpp:40-108):
 *   variant EIGSOL_QR_UNSHIFTED — the reference algorithm exactly: Hessenberg, then H <- R Q until
 *     max|h(i,i-1)| <= tol (1 + ||H||_F); eigenvalues = diag(H) (eig_re_or_c: n scalars of the
 *     dtype; eig_im unused); iterations = iter + 1 (maxIter + 1 when not converged);
 *   variant EIGSOL_QR_FRANCIS (north_star; real matrices) — Hessenberg, then Francis multishift
 *     double-shift sweeps to quasi-triangular form with deflation at unit roundoff.  eig_re_or_c
 *     receives the real parts (= diag of the standardised real Schur form), eig_im (optional) the
 *     imaginary parts; iterations = the most sweeps any single deflation needed (>= 1), and
 *     converged = 0 when that exceeded maxIterations (so iterations <= maxIterations exactly when
 *     converged, as in the reference).  Complex matrices (EIGSOL_C128) run complex multishift
 *     sweeps and return the eigenvalues themselves in eig_re_or_c.
 *     EIGSOL_DD / EIGSOL_CDD (long double): the fp64 sweeps on the rounded double-double Hessenberg
 *     matrix, then every eigenvalue refined in double-double by Newton's method on det(H - mu I)
 *     (Hyman's recurrence, n <= 8192); eig_re_or_c receives n dd (real parts) / n cdd values, and
 *     for EIGSOL_DD eig_im (optional) the imaginary parts as n {hi, lo} pairs (2n doubles).
 * n == 0: iterations 0, converged 1 (qr_eigenvalues.hpp:55-57). */
#define EIGSOL_QR_FRANCIS 0
#define EIGSOL_QR_UNSHIFTED 1
int eigsol_hessenberg_dense(eigsol_ctx* ctx, int dtype, int64_t n, const void* A_colmajor,
                            void* H_out);
int eigsol_qr_decompose_dense(eigsol_ctx* ctx, int dtype, int64_t m, int64_t n,
                              const void* A_colmajor, void* Q_out, void* R_out);
int eigsol_qr_eigenvalues_dense(eigsol_ctx* ctx, int dtype, int64_t n, const void* A_colmajor,
                                const eigsol_solver_options* opts, int variant,
                                void* eig_re_or_c, double* eig_im, int32_t* iterations,
                                int32_t* converged);

/* ---------------------------------------------------------------- row-sharded power iteration
 * One process per GPU; RCCL over xGMI (the reference has no distribution: SURVEY.md §2.1).
 * Rank r owns global rows [row_begins[r], row_begins[r+1]).  Bootstrap: rank 0 calls
 * eigsol_dist_get_unique_id, broadcasts the bytes with any transport, every rank calls
 * eigsol_ctx_create_dist.  eigsol_csr_create_dist is collective; the resulting matrix is used with
 * the eigsol_power_* session functions unchanged (x0 / x_out hold the rank's own rows).  Each
 * iteration exchanges x plus one 32-byte all-gather of rank partials; every rank reaches the same
 * termination decision.  The x exchange (chosen collectively, eigsol_exchange_mode):
 *   EIGSOL_EXCHANGE_HALO      only the entries other ranks read, point to point (banded matrices);
 *   EIGSOL_EXCHANGE_ALLGATHER every rank keeps all of x and the row blocks are all-gathered
 *                             (unstructured columns, where a rank reads most of x anyway). */
#define EIGSOL_EXCHANGE_HALO 0
#define EIGSOL_EXCHANGE_ALLGATHER 1
int eigsol_dist_unique_id_bytes(void);
int eigsol_dist_get_unique_id(void* id_out);
/* Test transport: an id that makes eigsol_ctx_create_dist join an in-process loopback world of
 * nranks ranks instead of an RCCL communicator (one host thread per rank, any devices of this
 * process, e.g. all on one GPU).  Every exchange of the row-sharded path runs as device copies
 * between the ranks' buffers, so the whole device-side path (ghost layout, pack, halo and
 * all-gather slots, rank-order partials) can be tested where RCCL cannot run several ranks. */
int eigsol_dist_loopback_id(int nranks, void* id_out);
int eigsol_ctx_create_dist(int device, int rank, int nranks, const void* unique_id,
                           eigsol_ctx** out);
int eigsol_csr_create_dist(eigsol_ctx* ctx, eigsol_dtype dtype, const int64_t* row_begins,
                           int64_t nnz_local, const int32_t* rowptr_local,
                           const int32_t* colidx_global, const void* values, eigsol_csr** out);
/* Host-only planning used by eigsol_csr_create_dist (no device, no communication): remaps global
 * columns to the local x-space [ghosts of lower ranks | own rows | ghosts of higher ranks] and
 * lists the ghosts (ascending global index) with their per-owner counts. */
int eigsol_ghost_plan(int nranks, const int64_t* row_begins, int rank, int64_t nnz_local,
                      const int32_t* colidx_global, int32_t* colidx_local, int64_t* nghost,
                      int64_t* ghost_global, int64_t* recv_counts);
/* Host-only: the exchange every rank of eigsol_csr_create_dist selects from the P x P ghost counts
 * (ghost_counts[r * P + q] = entries rank r reads from rank q): all-gather when some rank reads at
 * least a quarter of the rows it does not own, else halo.  EIGSOL_DIST_EXCHANGE=halo|allgather
 * overrides. */
int eigsol_exchange_mode(int nranks, const int64_t* row_begins, const int64_t* ghost_counts, int* mode);
/* The exchange a row-sharded matrix uses (EIGSOL_EXCHANGE_*) and its number of ghost entries. */
int eigsol_csr_dist_info(const eigsol_csr* A, int* mode, int64_t* nghost);

/* Host-collective bootstrap, no RCCL communicator: `allgather` gathers bytes_per_rank host bytes
 * from every rank into recv (rank order) and returns 0 on success; the library calls it for its
 * setup steps only (ghost plan counts and request lists, inbox addresses / IPC handles, barriers)
 * and never from a kernel-issuing hot loop.  Any host transport works (MPI, torch.distributed
 * gloo, sockets).  Row-sharded sessions on such a context use the device-side peer exchange. */
typedef int (*eigsol_allgather_fn)(const void* send, void* recv, size_t bytes_per_rank, void* user);
int eigsol_ctx_create_dist_host(int device, int rank, int nranks, eigsol_allgather_fn allgather,
                                void* user, eigsol_ctx** out);

/* Per-iteration transport of a power session (eigsol_power_transport):
 *   EIGSOL_TRANSPORT_LOCAL     one GPU, nothing to exchange;
 *   EIGSOL_TRANSPORT_COLLECTIVE host-enqueued pack kernel + RCCL group (or loopback copies) after
 *                              every launch (all-gather exchange, non-sliced layouts);
 *   EIGSOL_TRANSPORT_PEER      device-side: the fused SpMV's epilogue stores the halo rows and the
 *                              rank partial straight into every peer's inbox (IPC-mapped over xGMI,
 *                              or same-device pointers in a loopback world) and raises an epoch
 *                              flag there; the next launch's prologue waits for the peers' flags.
 *                              No host round trip, no extra launch.  EIGSOL_DIST_TRANSPORT=
 *                              collective|peer overrides the collective choice (halo matrices in
 *                              the sliced layout use peer by default). */
#define EIGSOL_TRANSPORT_LOCAL 0
#define EIGSOL_TRANSPORT_COLLECTIVE 1
#define EIGSOL_TRANSPORT_PEER 2
int eigsol_power_transport(const eigsol_power* s, int* transport);

/* Host-only planning of the peer exchange (no device): this rank's push list.  requests holds
 * the global rows other ranks read from this rank, grouped by requesting rank in rank order with
 * counts ghost_counts[q * P + rank] (each group ascending, as eigsol_ghost_plan lists them);
 * ghost_counts is the all-gathered P x P matrix of eigsol_ghost_plan's recv_counts.  Output: per
 * request an entry {local row, peer, slot, 0}, where slot indexes the peer's ghost list (its
 * [lower | upper] ghost order), sorted by local row. */
int eigsol_peer_plan(int nranks, int rank, const int64_t* row_begins, const int64_t* ghost_counts,
                     const int64_t* requests, int64_t nreq, int32_t* push_out);
/* This context's place in the world: device, rank, ranks, and how it exchanges (0 none, 1 RCCL
 * communicator, 2 in-process loopback world, 3 caller's host all-gather + device peer inboxes). */
int eigsol_ctx_info(eigsol_ctx* ctx, int* device, int* rank, int* nranks, int* comm_kind);

/* ---------------------------------------------------------------- measurement
 * The device's practical HBM bandwidth ("verify the spec with a STREAM-like kernel
 * on the box"): hand-written gfx950 streams over `bytes` (use >= 2 GiB: beyond the 256 MB
 * Infinity Cache) with non-temporal loads / stores, four in flight per lane, timed with HIP events
 * over `reps` launches on the context's stream, best over 1/2/4/8 workgroups per CU.
 * read = load only (16- and 8-byte loads, the better), copy = load + store (both directions
 * counted), write = store only (GB/s). */
int eigsol_hbm_probe(eigsol_ctx* ctx, size_t bytes, int reps, double* read_gbps, double* copy_gbps,
                     double* write_gbps, int* best_blocks_per_cu);
/* The headline SpMV's read / write mix (12 reads : 1 write of 16-byte non-temporal words) over
 * `bytes` of reads: GB/s of both directions, best over 1/2/4/8 workgroups per CU. */
int eigsol_hbm_probe_mix(eigsol_ctx* ctx, size_t bytes, int reps, double* mix_gbps, int* best_blocks_per_cu);

/* ---------------------------------------------------------------- sparse LU analysis (host only)
 * The symbolic factorization the general-sparse shifted solve runs before choosing the exact LU
 * over ILU(0) (variant 18 vs 7): the pattern of A with its diagonal inserted, closed under fill
 * for LU without pivoting (row i = its own columns plus, for every k < i in it in ascending order,
 * fill included, row k's columns past k).  Stops once the pattern would pass `cap` entries.
 * *nnz_out = the filled pattern's entries, or -1 when it exceeds cap; *lower_levels_out (optional)
 * = dependency levels of its strict lower part (the numeric factorization's launches).  Rows must
 * be sorted; needs no device. */
int eigsol_sparse_lu_fill(int64_t n, const int32_t* rowptr, const int32_t* colidx, int64_t cap, int64_t* nnz_out,
                          int32_t* lower_levels_out);

/* The nested-dissection multifrontal plan of the general-sparse shifted solve (variant 19; host
 * only): the ordering of the pattern of A + A^T and the supernodal structure.  perm_out (n
 * entries, new -> old) and fronts_out (4 int32 per front: first column, pivots, struct size,
 * parent front or -1; fronts in postorder) may be null; fronts_cap = room in fronts_out (fronts).
 * stats_out[8] = fronts, tree heights, largest front order, most pivots of a front, stored factor
 * entries, sum of squared front orders, factorization flops (complex arithmetic if is_complex),
 * 1.0 when the plan is consistent.  Call once with fronts_out = null to size it. */
int eigsol_mf_analyze(int64_t n, const int32_t* rowptr, const int32_t* colidx, int32_t leaf, int32_t is_complex,
                      int32_t* perm_out, int32_t* fronts_out, int64_t fronts_cap, double* stats_out);

#ifdef __cplusplus
}
#endif
#endif /* EIGSOL_HIP_H */

// Device-resident CSR matrix and the fused power-iteration SpMV for gfx950.
//
// Replaces the numeric core behind powerMethod<S> (src/power_method/power_method.hpp:135-148):
// the two Eigen products per iteration (:69 and :81), y.norm() (:72), x = y/normY (:78), the
// Rayleigh dot (:81) and the is_close_relative test (:83-91, tolerance.hpp:28-33) become ONE
// kernel launch per iteration:
//
//   launch t:  x_t = y_{t-1} / ||y_{t-1}||  (division on the gather, bitwise the reference's x)
//              y_t = A x_t                 (row tiles staged through LDS, CSR-stream)
//              partials ||y_t||^2, x_t^H y_t  -> block partials -> last-arriver rank partial
//              prologue of launch t+1 turns the rank partials into the reference's decisions.
//
// Row tiles: consecutive rows whose nonzeros fit one LDS tile (4096 f64 / 2048 c128 products,
// <= 256 rows).  Phase 1 streams the tile's values/columns coalesced (16 B per lane), gathers x
// and writes the products to LDS; phase 2 gives each row to one lane, which sums its products
// sequentially in ascending column order — exactly the per-row order of the reference's
// Eigen CSC scatter, so every y_i is bitwise the reference's.  Rows longer than a tile get a tile
// of their own and a fixed-order strided block reduction (deterministic, tolerance-checked).
// Tiles are assigned XCD-contiguously (block b serves XCD group b % 8), so neighbouring row
// tiles — which gather overlapping x windows for banded matrices — share one XCD's L2.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <type_traits>
#include <vector>

#include "kernels_common.hpp"
#include "wide.hpp"

namespace eigsol {
namespace dev {

template <class S> struct Tile;
// kNnz: LDS products per tile; kCap: nonzeros a tile may hold (f64 lanes load aligned pairs, so a
// tile starting at an odd index needs one spare slot).
template <> struct Tile<double> { static constexpr int kNnz = 2048; static constexpr int kCap = kNnz - 1; };
template <> struct Tile<cplx> { static constexpr int kNnz = 1024; static constexpr int kCap = kNnz; };
constexpr int kTileRows = 256;

// One pad element every 32 keeps the lane-per-row phase-2 reads spread over the 64 banks.
__device__ __forceinline__ int lds_idx(int k) { return k + (k >> 5); }

// Tile metadata is read-only for the whole launch and indexed uniformly: scalar loads (constant
// address space) keep it off the vector memory counter.
__device__ __forceinline__ int4 ld_uniform(const int4* p, int i) {
    using cp = const __attribute__((address_space(4))) int*;
    const cp q = (cp)(uintptr_t)(p + i);
    return make_int4(q[0], q[1], q[2], q[3]);
}
__device__ __forceinline__ int2 ld_uniform(const int2* p, int i) {
    using cp = const __attribute__((address_space(4))) int*;
    const cp q = (cp)(uintptr_t)(p + i);
    return make_int2(q[0], q[1]);
}

template <class S>
struct CsrArgs {
    const int32_t* rowptr;
    const int32_t* col;
    const uint16_t* col16;   // windowed matrices: column - tile window start (< kWin)
    const S* val;
    // sliced layout (csr_slice_kernel): 64 rows per slice, entry (k, lane) at off + 64 k + lane
    const int4* slice_meta;  // per slice {entry offset, window start (-1: gather slice), K | ragged << 8, window length}
    const S* sval;
    const uint32_t* scol8;   // window slices: column - window start, 8 bits, 4 entries per lane-dword
    const int32_t* scol32;   // gather slices: x-space column
    const uint8_t* slen;     // row lengths (read for ragged slices only)
    int32_t nslices;
    int32_t nseg;                    // stream segments; 1: no per-slice segment lookup
    int64_t seg_val[kMaxSliceSeg];   // element offset of each stream segment (slice meta .z bits 21..24)
    int64_t seg_c8[kMaxSliceSeg];
    int64_t seg_c32[kMaxSliceSeg];
    const int4* tile_meta;   // per tile {r0, r1, e0, e1}: short tiles first, then long rows
    const int2* tile_win;    // per short tile: x window [w0, w1] covering its columns and rows
    int32_t ntiles;
    int32_t nshort;
    int32_t xlen;            // entries of the input vector (own + ghost)
    int32_t xoff;            // x-space index of local row 0 (lower ghosts precede the own rows)
    int32_t nrows;
    const S* x_plain;        // plain SpMV input (kPower == false)
    S* y_plain;              // plain SpMV output
    S* buf0;                 // power: y buffers, launch t reads buf[(t-1)&1], writes buf[t&1]
    S* buf1;
    PowerCtl* ctl;
    const part4* rank_part;
    int32_t nranks;
    part4* my_part;
    part4* blk_part;
    S* trace;
    PeerArgs peer;           // row-sharded session on the device-side peer exchange (kDist kernels)
    int32_t cb_carry;        // column-block pass > 0 (csr_kernel): row sums start from y's partials
    int32_t cb_epi;          // last (or only) pass: fused power epilogue (norm / Rayleigh partials)
    // column-binned layout (csr_bin_kernel): entries as (row in chunk << cbits | column in block)
    const uint32_t* bpk;
    const S* bval;
    const int4* bstep;       // per step {first level, levels | barrier << 8, first run, block}
    const int2* blev;        // per level {entry offset, runs}
    const int32_t* bchunk;   // per chunk: its steps [bchunk[c], bchunk[c + 1])
    int32_t nchunks;
    int32_t brows;           // rows per chunk (<= kBinRows of the instantiation)
    int32_t bcbits;          // log2 of the columns per block
    int32_t cbeg, cend;      // chunks of this launch (an iteration split in two row parts)
    int32_t cont;            // second part: read the first part's decision, add to its partial
};

// Registers holding one tile's stream for one lane: P slots of (values, columns) plus the lane's
// row pointers.  f64 slots carry a 16-byte pair of values and an 8-byte pair of columns.
template <class S> struct Slot;
template <> struct Slot<double> {
    static constexpr int kNnz = 2;
    double2 v;
    int2 c;
};
template <> struct Slot<cplx> {
    static constexpr int kNnz = 1;
    cplx v;
    int c;
};
template <class S>
struct TileRegs {
    static constexpr int P = Tile<S>::kNnz / (Slot<S>::kNnz * kThreads);
    Slot<S> s[P];
    int rp0, rp1;
};

// Issue every load of a short tile's value/column stream and of the lane's row pointers.
// Branch-free on purpose: an exec-masked branch around each load makes hipcc wait vmcnt(0) per
// load (MI355X guide §5 "Projection GEMM" item 4(c)), which serialises the pipeline.  The streams
// are padded by one tile on the device, and every column index (padding included) is valid.
template <class S>
__device__ __forceinline__ void load_tile(const CsrArgs<S>& a, int4 m, TileRegs<S>& R) {
    constexpr int P = TileRegs<S>::P;
    const int tid = threadIdx.x;
    if constexpr (std::is_same_v<S, double>) {
        const int q0 = m.z & ~1;
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const uint32_t q = (uint32_t)(q0 + 2 * (tid + p * kThreads));
            R.s[p].v = ldg_stream(reinterpret_cast<const double2*>(a.val), q >> 1);
            R.s[p].c = ldg_stream(reinterpret_cast<const int2*>(a.col), q >> 1);
        }
    } else {
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const uint32_t q = (uint32_t)(m.z + tid + p * kThreads);
            R.s[p].v = ldg_stream(a.val, q);
            R.s[p].c = ldg_stream(a.col, q);
        }
    }
    const uint32_t r = (uint32_t)min(m.x + tid, a.nrows - 1);
    R.rp0 = ldg(a.rowptr, r);
    R.rp1 = ldg(a.rowptr, r + 1);
}

// Gathers of one tile's x entries (all in flight together; unconditional, see load_tile).
template <class S, int kMode>
__device__ __forceinline__ void issue_gathers(const TileRegs<S>& R, const S* xin,
                                              S (&xg)[TileRegs<S>::P][Slot<S>::kNnz]) {
    constexpr int P = TileRegs<S>::P;
#pragma unroll
    for (int p = 0; p < P; ++p) {
        // The empty asm pins each column's first use here: without it hipcc computes the gather
        // address as soon as the prefetched column lands (before the previous barrier) and
        // waits for the whole prefetch there.
        if constexpr (std::is_same_v<S, double>) {
            int c0 = R.s[p].c.x, c1 = R.s[p].c.y;
            asm volatile("" : "+v"(c0), "+v"(c1));
            xg[p][0] = kMode == 1 ? 1.0 : xin[c0];
            xg[p][1] = kMode == 1 ? 1.0 : xin[c1];
        } else {
            int c0 = R.s[p].c;
            asm volatile("" : "+v"(c0));
            xg[p][0] = xin[c0];
        }
    }
}

// products a_ij * x_j (x_j = y_j / nrm, the reference's x = y / normY) -> LDS.  Slots outside
// the tile write to the scratch element `dummy`.
template <class S, bool kPower, int kMode>
__device__ __forceinline__ void write_products(const TileRegs<S>& R, int4 m,
                                               const S (&xg)[TileRegs<S>::P][Slot<S>::kNnz],
                                               double nrm, double rnrm, S* prod, int dummy) {
    constexpr int P = TileRegs<S>::P;
    constexpr int NPS = Slot<S>::kNnz;
    const int tid = threadIdx.x;
    const int q0 = std::is_same_v<S, double> ? (m.z & ~1) : m.z;
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const int qb = q0 + NPS * (tid + p * kThreads);
        if constexpr (std::is_same_v<S, double>) {
            double x0 = xg[p][0], x1 = xg[p][1];
            if constexpr (kPower && kMode == 2) {
                x0 = x0 * rnrm;
                x1 = x1 * rnrm;
            } else if constexpr (kPower) {
                x0 = scale_in(x0, nrm);
                x1 = scale_in(x1, nrm);
            }
            const int i0 = (qb >= m.z && qb < m.w) ? lds_idx(qb - m.z) : dummy;
            const int i1 = (qb + 1 < m.w) ? lds_idx(qb + 1 - m.z) : dummy;
            prod[i0] = R.s[p].v.x * x0;
            prod[i1] = R.s[p].v.y * x1;
        } else {
            S xv = xg[p][0];
            if constexpr (kPower) xv = scale_in(xv, nrm);
            const int i0 = qb < m.w ? lds_idx(qb - m.z) : dummy;
            prod[i0] = mul(R.s[p].v, xv);
        }
    }
}

// Long rows (one row per tile, longer than an LDS tile): strided partial sums and a fixed-order
// block reduction (deterministic); tiles dealt round-robin over the grid.
template <class S, bool kPower>
__device__ __forceinline__ void long_rows_pass(const CsrArgs<S>& a, const S* xin, S* yout,
                                               double nrm, double& n2, double& rr, double& ri,
                                               double* sm) {
    const int tid = threadIdx.x;
    for (int lt = a.nshort + blockIdx.x; lt < a.ntiles; lt += gridDim.x) {
        const int4 m = a.tile_meta[lt];
        double pr = 0.0, pi = 0.0, dummy = 0.0;
        for (int q = m.z + tid; q < m.w; q += kThreads) {
            S xv = xin[a.col[q]];
            if constexpr (kPower) xv = scale_in(xv, nrm);
            const S pq = mul(a.val[q], xv);
            if constexpr (std::is_same_v<S, double>) {
                pr += pq;
            } else {
                pr += pq.re;
                pi += pq.im;
            }
        }
        block_sum3(pr, pi, dummy, sm);
        if (tid == 0) {
            S sacc;
            set_re_im(sacc, pr, pi);
            yout[m.x] = sacc;
            if constexpr (kPower) {
                const S xi = scale_in(xin[m.x + a.xoff], nrm);
                n2 += sq_abs(sacc);
                acc_dot(rr, ri, xi, sacc);
            }
        }
    }
}

// Sequential ascending-column sum of one row's products from LDS (the reference's order).
template <class S, int kMode = 0>
__device__ __forceinline__ S row_sum(const S* pb, int k0, int k1) {
    S sacc = s_zero<S>();
    if constexpr (kMode == 3) {
        if (k1 > k0) sacc = pb[lds_idx(k0)];
    } else {
        for (int k = k0; k < k1; ++k) sacc = add(sacc, pb[lds_idx(k)]);
    }
    return sacc;
}

// kMode (diagnostic ablations, EIGSOL_CSR_ABLATION): 0 full; 1 no x gather; 2 reciprocal scaling;
// 3 no phase-2 row sums.  Only mode 0 is a product path.
//
// Short tiles run as a software pipeline with ONE barrier per tile and two LDS product buffers:
//   iteration i:  issue gathers of tile i+1 | issue stream loads of tile i+2
//                 row sums of tile i (LDS buffer b)          <- overlaps the gathers' latency
//                 products of tile i+1 -> LDS buffer b^1 ; barrier
// Buffer b^1 was last read by the row sums of iteration i-1, which precede the barrier that
// ended iteration i-1, so one barrier per tile orders both hazards.
template <class S, bool kPower, int kMode = 0>
__global__ __launch_bounds__(kThreads) void csr_kernel(CsrArgs<S> a, int parity) {
    constexpr int TN = Tile<S>::kNnz;
    constexpr int P = TileRegs<S>::P;
    constexpr int NPS = Slot<S>::kNnz;
    constexpr int LDSN = TN + TN / 32;
    __shared__ S prod[2 * LDSN];
    __shared__ int2 rows[2][kThreads];
    __shared__ S xrows[kPower ? 2 : 1][kThreads];
    __shared__ double sm[3 * kWaves];
    __shared__ Prologue pro;
    __shared__ int s_last;

    const S* xin;
    S* yout;
    double nrm = 0.0;
    if constexpr (kPower) {
        power_prologue<S>(a.ctl, a.rank_part, a.nranks, parity, a.trace, &pro);
        if (!__builtin_amdgcn_readfirstlane(pro.go)) return;   // block-uniform exit
        nrm = pro.nrm;
        xin = parity ? a.buf0 : a.buf1;
        yout = (parity ? a.buf1 : a.buf0) + a.xoff;   // y rows land at their x-space slots
    } else {
        xin = a.x_plain;
        yout = a.y_plain;
    }
    const double rnrm = nrm > 0.0 ? 1.0 / nrm : 1.0;
    (void)rnrm;
    const int tid = threadIdx.x;
    double n2 = 0.0, rr = 0.0, ri = 0.0;

    // XCD-contiguous ranges of short tiles: block b works in group b % 8 on that group's chunk.
    const int nb = gridDim.x >> 3;
    const int chunk = (a.nshort + 7) >> 3;
    const int tbeg = (blockIdx.x & 7) * chunk;
    const int tend = min(a.nshort, tbeg + chunk);
    int t = tbeg + (blockIdx.x >> 3);

    if (t < tend) {
        // Loop-carried per-row state (row pointers, x_i for the Rayleigh term) goes through LDS so
        // the only registers live across the back-edge are the prefetched stream: keeps hipcc's
        // s_waitcnt counting exact instead of vmcnt(0) at the first use of a loop-carried value.
        const int last = tend - 1;
        int4 mc = a.tile_meta[t];
        TileRegs<S> Rc;
        load_tile(a, mc, Rc);
        S xg[P][NPS];
        issue_gathers<S, kMode>(Rc, xin, xg);
        S xrow = s_zero<S>();
        if constexpr (kPower) xrow = xin[min(mc.x + tid, a.nrows - 1) + a.xoff];
        int tn = t + nb;
        int4 mn = a.tile_meta[min(tn, last)];
        TileRegs<S> Rn;
        load_tile(a, mn, Rn);
        write_products<S, kPower, kMode>(Rc, mc, xg, nrm, rnrm, prod, LDSN - 1);
        rows[0][tid] = make_int2(Rc.rp0, Rc.rp1);
        if constexpr (kPower) xrows[0][tid] = xrow;
        __syncthreads();
        int b = 0;
        // One pipeline step.  `Rnx` holds the next tile's stream (already in flight), `Rld`
        // receives the stream two tiles ahead.  The loop is unrolled by two with the register
        // sets swapping roles, so the prefetch is never copied (a copy would force its wait).
        auto step = [&](TileRegs<S>& Rnx, TileRegs<S>& Rld) -> bool {
            const int t2 = tn + nb;
            // meta first, so its wait does not cover the gathers issued after it
            const int4 m2 = a.tile_meta[min(t2, last)];
            issue_gathers<S, kMode>(Rnx, xin, xg);
            if constexpr (kPower) xrow = xin[min(mn.x + tid, a.nrows - 1) + a.xoff];
            load_tile(a, m2, Rld);
            // row sums of the current tile from LDS buffer b (ascending-column sequential sums)
            if (tid < mc.y - mc.x) {
                const S* pb = prod + b * LDSN;
                const int2 rp = rows[b][tid];
                const int k0 = rp.x - mc.z;
                const int k1 = rp.y - mc.z;
                // column-block passes continue the previous block's partial (same summation order)
                S sacc = a.cb_carry ? yout[mc.x + tid] : s_zero<S>();
                if constexpr (kMode == 3) {
                    if (k1 > k0) sacc = pb[lds_idx(k0)];
                } else {
                    for (int k = k0; k < k1; ++k) sacc = add(sacc, pb[lds_idx(k)]);
                }
                yout[mc.x + tid] = sacc;
                if constexpr (kPower) {
                    if (a.cb_epi) {
                        const S xi = scale_in(xrows[b][tid], nrm);
                        n2 += sq_abs(sacc);
                        acc_dot(rr, ri, xi, sacc);
                    }
                }
            }
            if (tn >= tend) return true;
            write_products<S, kPower, kMode>(Rnx, mn, xg, nrm, rnrm, prod + (b ^ 1) * LDSN, LDSN - 1);
            rows[b ^ 1][tid] = make_int2(Rnx.rp0, Rnx.rp1);
            if constexpr (kPower) xrows[b ^ 1][tid] = xrow;
            // keep the next step's address arithmetic (which waits for the prefetch) below this
            // barrier: hipcc otherwise hoists it and waits for the prefetched stream here.
            __builtin_amdgcn_sched_barrier(0);
            __syncthreads();
            __builtin_amdgcn_sched_barrier(0);
            b ^= 1;
            mc = mn;
            mn = m2;
            tn = t2;
            return false;
        };
        TileRegs<S>& Ra = Rn;
        TileRegs<S>& Rb = Rc;   // Rc's stream is consumed: reuse its registers
        for (;;) {
            if (step(Ra, Rb)) break;
            if (step(Rb, Ra)) break;
        }
    }

    long_rows_pass<S, kPower>(a, xin, yout, nrm, n2, rr, ri, sm);   // (column blocks have no long rows)
    if constexpr (kPower) {
        if (a.cb_epi) {   // launch-uniform
            block_sum3(n2, rr, ri, sm);
            last_arriver_reduce(n2, rr, ri, a.blk_part, &a.ctl->counter, a.my_part, sm, &s_last);
        }
    }
}

// ============================================================================ windowed pipeline
// For tiles whose columns (and rows) fall in a window of at most kWin entries — banded and
// locality-ordered matrices, the multi-GPU headline — the tile's slice of x is staged into LDS with
// coalesced loads (scaled by 1/||y|| once per element) and the products gather from LDS instead of
// global memory.  Per step (one tile), two barriers:
//   issue: stream + window loads of tile i+2          (registers, two tiles ahead)
//   store window of tile i+1 -> xwin[b^1]            (loaded one step ago)
//   row sums of tile i (prod, xwin[b])               ; barrier A
//   products of tile i+1 (xwin[b^1]) -> prod, rows   ; barrier B
template <class S> struct Win;
template <> struct Win<double> { static constexpr int kWin = 512; };
template <> struct Win<cplx> { static constexpr int kWin = 256; };

template <class S>
struct WinRegs {
    static constexpr int K = Win<S>::kWin / kThreads;
    S v[K];
};

// Branch-free window load: indices past the end of x are clamped (those slots lie beyond w1).
template <class S>
__device__ __forceinline__ void load_window(const S* xin, int2 w, int xlen, WinRegs<S>& W) {
#pragma unroll
    for (int k = 0; k < WinRegs<S>::K; ++k)
        W.v[k] = ldg(xin, (uint32_t)min(w.x + (int)threadIdx.x + k * kThreads, xlen - 1));
}

template <class S, bool kPower>
__device__ __forceinline__ void store_window(const WinRegs<S>& W, double nrm, S* xw) {
#pragma unroll
    for (int k = 0; k < WinRegs<S>::K; ++k) {
        S v = W.v[k];
        if constexpr (kPower) v = scale_in(v, nrm);
        xw[threadIdx.x + k * kThreads] = v;
    }
}

// products of a short tile with x read from the LDS window
template <class S>
__device__ __forceinline__ void win_products(const TileRegs<S>& R, int4 m, int w0, const S* xw,
                                             S* prod, int dummy) {
    constexpr int P = TileRegs<S>::P;
    constexpr int NPS = Slot<S>::kNnz;
    const int tid = threadIdx.x;
    const int q0 = std::is_same_v<S, double> ? (m.z & ~1) : m.z;
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const int qb = q0 + NPS * (tid + p * kThreads);
        if constexpr (std::is_same_v<S, double>) {
            const bool v0 = qb >= m.z && qb < m.w;
            const bool v1 = qb + 1 < m.w;
            const double x0 = xw[v0 ? R.s[p].c.x - w0 : 0];
            const double x1 = xw[v1 ? R.s[p].c.y - w0 : 0];
            prod[v0 ? lds_idx(qb - m.z) : dummy] = R.s[p].v.x * x0;
            prod[v1 ? lds_idx(qb + 1 - m.z) : dummy] = R.s[p].v.y * x1;
        } else {
            const bool v0 = qb < m.w;
            const S x0 = xw[v0 ? R.s[p].c - w0 : 0];
            prod[v0 ? lds_idx(qb - m.z) : dummy] = mul(R.s[p].v, x0);
        }
    }
}

// Windowed tiles stream 16-bit window-relative column offsets instead of int32 columns: 10 bytes
// per nonzero instead of 12 for f64 (the windows are at most kWin = 512 wide by construction).
// Algorithmic bytes are still counted for the int32 CSR layout; the PMC traffic
// in profiles/ shows the bytes actually moved.
template <class S> struct WSlot;
template <> struct WSlot<double> {
    static constexpr int kNnz = 2;
    double2 v;
    uint32_t c;     // two 16-bit offsets
};
template <> struct WSlot<cplx> {
    static constexpr int kNnz = 1;
    cplx v;
    uint32_t c;     // one 16-bit offset
};
template <class S>
struct WTileRegs {
    static constexpr int P = Tile<S>::kNnz / (WSlot<S>::kNnz * kThreads);
    WSlot<S> s[P];
    int rp0, rp1;
};

template <class S>
__device__ __forceinline__ void load_tile_w(const CsrArgs<S>& a, int4 m, WTileRegs<S>& R) {
    constexpr int P = WTileRegs<S>::P;
    const int tid = threadIdx.x;
    if constexpr (std::is_same_v<S, double>) {
        const int q0 = m.z & ~1;
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const uint32_t q = (uint32_t)(q0 + 2 * (tid + p * kThreads));
            R.s[p].v = ldg_stream(reinterpret_cast<const double2*>(a.val), q >> 1);
            R.s[p].c = ldg_stream(reinterpret_cast<const uint32_t*>(a.col16), q >> 1);
        }
    } else {
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const uint32_t q = (uint32_t)(m.z + tid + p * kThreads);
            R.s[p].v = ldg_stream(a.val, q);
            R.s[p].c = ldg_stream(a.col16, q);
        }
    }
    const uint32_t r = (uint32_t)min(m.x + tid, a.nrows - 1);
    R.rp0 = ldg(a.rowptr, r);
    R.rp1 = ldg(a.rowptr, r + 1);
}

// LDS product index of the windowed kernel: f64 products are written as 16-byte pairs, so the
// padding (one pair per 32 products, which spreads the lane-per-row reads over the banks) keeps
// every pair 16-byte aligned; complex products are 16 bytes each.
#ifndef EIGSOL_WPAD_SHIFT
#define EIGSOL_WPAD_SHIFT 5
#endif
template <class S>
__device__ __forceinline__ int wlds(int k) {
    if constexpr (std::is_same_v<S, double>) return k + 2 * (k >> EIGSOL_WPAD_SHIFT);
    else return k + (k >> 5);
}
template <class S>
__device__ __forceinline__ int wbase(int4 m) {
    return std::is_same_v<S, double> ? (m.z & ~1) : m.z;   // stream index of LDS product slot 0
}

// Products of a short tile with x from the LDS window, written unconditionally: slots outside the
// tile's [e0, e1) (the pair partner before e0, the stream beyond e1) hold products no row sum
// reads, and every 16-bit offset in the stream is a valid window index (< kWin) by construction.
template <class S>
__device__ __forceinline__ void win_products_w(const WTileRegs<S>& R, int4 m, const S* xw, S* prod) {
    constexpr int P = WTileRegs<S>::P;
    constexpr int NPS = WSlot<S>::kNnz;
    const int tid = threadIdx.x;
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const int k = NPS * (tid + p * kThreads);   // slot of this lane's first product
        if constexpr (std::is_same_v<S, double>) {
            const double x0 = xw[R.s[p].c & 0xffffu];
            const double x1 = xw[R.s[p].c >> 16];
            *reinterpret_cast<double2*>(prod + wlds<S>(k)) = make_double2(R.s[p].v.x * x0, R.s[p].v.y * x1);
        } else {
            prod[wlds<S>(k)] = mul(R.s[p].v, xw[R.s[p].c]);
        }
    }
    (void)m;
}

template <class S>
__device__ __forceinline__ S row_sum_w(const S* pb, int k0, int k1) {
    S sacc = s_zero<S>();
    for (int k = k0; k < k1; ++k) sacc = add(sacc, pb[wlds<S>(k)]);
    return sacc;
}

template <class S, bool kPower>
__global__ __launch_bounds__(kThreads) void csr_win_kernel(CsrArgs<S> a, int parity) {
    constexpr int TN = Tile<S>::kNnz;
    constexpr int LDSN = TN + (std::is_same_v<S, double> ? 2 * (TN >> EIGSOL_WPAD_SHIFT) : TN / 32);
    constexpr int KW = Win<S>::kWin;
    __shared__ __align__(16) S prod[LDSN];
    __shared__ S xwin[2][KW];
    __shared__ int2 rows[kThreads];
    __shared__ double sm[3 * kWaves];
    __shared__ Prologue pro;
    __shared__ int s_last;

    const S* xin;
    S* yout;
    double nrm = 0.0;
    if constexpr (kPower) {
        power_prologue<S>(a.ctl, a.rank_part, a.nranks, parity, a.trace, &pro);
        if (!__builtin_amdgcn_readfirstlane(pro.go)) return;   // block-uniform exit
        nrm = pro.nrm;
        xin = parity ? a.buf0 : a.buf1;
        yout = (parity ? a.buf1 : a.buf0) + a.xoff;   // y rows land at their x-space slots
    } else {
        xin = a.x_plain;
        yout = a.y_plain;
    }
    const int tid = threadIdx.x;
    double n2 = 0.0, rr = 0.0, ri = 0.0;

    const int nb = gridDim.x >> 3;
    const int chunk = (a.nshort + 7) >> 3;
    const int tbeg = (blockIdx.x & 7) * chunk;
    const int tend = min(a.nshort, tbeg + chunk);
    const int t = tbeg + (blockIdx.x >> 3);

    if (t < tend) {
        const int last = tend - 1;
        // Fill: tile t -> products in LDS; tile t+nb -> stream + window in registers; metadata
        // of tile t+2nb requested (scalar loads, one step ahead of its use).
        int4 mc = ld_uniform(a.tile_meta, t);
        int2 wc = ld_uniform(a.tile_win, t);
        int tn = t + nb;
        int4 mn = ld_uniform(a.tile_meta, min(tn, last));
        int2 wn = ld_uniform(a.tile_win, min(tn, last));
        int4 m2 = ld_uniform(a.tile_meta, min(tn + nb, last));
        int2 w2 = ld_uniform(a.tile_win, min(tn + nb, last));
        WTileRegs<S> Ra, Rb;
        WinRegs<S> Wa, Wb;
        load_tile_w(a, mc, Rb);
        load_window(xin, wc, a.xlen, Wb);
        load_tile_w(a, mn, Ra);
        load_window(xin, wn, a.xlen, Wa);
        int b = 0;
        store_window<S, kPower>(Wb, nrm, xwin[0]);
        __syncthreads();
        win_products_w(Rb, mc, xwin[0], prod);
        rows[tid] = make_int2(Rb.rp0, Rb.rp1);
        __syncthreads();

        // step i: Rnx/Wnx = tile i+1 (in flight since step i-1), Rld/Wld <- tile i+2.  Unrolled
        // by two with the register sets swapping roles, so the prefetch is never copied (a copy
        // would force its wait).
        auto step = [&](WTileRegs<S>& Rnx, WinRegs<S>& Wnx, WTileRegs<S>& Rld, WinRegs<S>& Wld) -> bool {
            const int t3 = tn + 2 * nb;
            const int4 m3 = ld_uniform(a.tile_meta, min(t3, last));
            const int2 w3 = ld_uniform(a.tile_win, min(t3, last));
            load_tile_w(a, m2, Rld);
            load_window(xin, w2, a.xlen, Wld);
            store_window<S, kPower>(Wnx, nrm, xwin[b ^ 1]);   // unconditional: no branch around the wait
            // row sums of the current tile (x_i for the Rayleigh term from the scaled window)
            if (tid < mc.y - mc.x) {
                const int2 rp = rows[tid];
                const int qb = wbase<S>(mc);
                const S sacc = row_sum_w<S>(prod, rp.x - qb, rp.y - qb);
                yout[mc.x + tid] = sacc;
                if constexpr (kPower) {
                    const S xi = xwin[b][mc.x + a.xoff + tid - wc.x];
                    n2 += sq_abs(sacc);
                    acc_dot(rr, ri, xi, sacc);
                }
            }
            if (tn >= tend) return true;
            __builtin_amdgcn_sched_barrier(0);
            __syncthreads();
            __builtin_amdgcn_sched_barrier(0);
            win_products_w(Rnx, mn, xwin[b ^ 1], prod);
            rows[tid] = make_int2(Rnx.rp0, Rnx.rp1);
            __builtin_amdgcn_sched_barrier(0);
            __syncthreads();
            __builtin_amdgcn_sched_barrier(0);
            b ^= 1;
            mc = mn;
            wc = wn;
            mn = m2;
            wn = w2;
            m2 = m3;
            w2 = w3;
            tn += nb;
            return false;
        };
        for (;;) {
            if (step(Ra, Wa, Rb, Wb)) break;
            if (step(Rb, Wb, Ra, Wa)) break;
        }
    }

    long_rows_pass<S, kPower>(a, xin, yout, nrm, n2, rr, ri, sm);   // (column blocks have no long rows)
    if constexpr (kPower) {
        if (a.cb_epi) {   // launch-uniform
            block_sum3(n2, rr, ri, sm);
            last_arriver_reduce(n2, rr, ri, a.blk_part, &a.ctl->counter, a.my_part, sm, &s_last);
        }
    }
}

// ============================================================================ sliced pipeline
// Rows in slices of 64, one row per lane.  Values are stored slice by slice in (k, lane) order, so
// every value load is one coalesced 64-lane access and each lane sums its own row in ascending
// column order (the reference's order) in registers: no LDS product round trip and no block
// barrier.  A slice whose x window (its columns and its own rows) spans at most kSliceWin entries
// stages the window, scaled once per element, in a wave-private LDS region, and streams 8-bit
// window offsets packed four per lane-dword; other slices gather x from global memory with int32
// columns.  Slices are taken XCD-contiguously like the tiles of the other kernels.
// meta per slice: {value entry offset, window start (-1: gather slice), K | ragged << 8 | wl << 9,
//                  column offset (dwords of packed 8-bit offsets, or int32 entries)}
constexpr int kSliceRows = 64;
constexpr int kSliceMaxK = 64;
constexpr int kSliceWin = 256;

// x-space entry e of a ghost-reading slice on the peer exchange: own rows from the input vector,
// ghosts (e < xoff, e >= xoff + nrows) from the inbox's ghost area with system-scope loads.
template <class S>
__device__ __forceinline__ S ld_x_peer(const CsrArgs<S>& a, const S* xin, const S* gin, int e) {
    const bool lo = e < a.xoff, hi = e >= a.xoff + a.nrows;
    if (lo || hi) return ld_sys_s(gin + (lo ? e : e - a.nrows));
    return xin[e];
}

// Real scalars travel in pairs (double2: 16-byte lane loads; float2: 8-byte), complex ones alone.
template <class S> struct Pair2 { using type = S; };
template <> struct Pair2<double> { using type = double2; };
template <> struct Pair2<float> { using type = float2; };
template <class S> using pair_t = typename Pair2<S>::type;
// Value groups of the slice stream: entries of a row held together in one 16-byte lane load
// (f64: pairs; f32: quads; complex: one entry)
template <class S> struct VGroup { using type = S; static constexpr int n = 1; };
template <> struct VGroup<double> { using type = double2; static constexpr int n = 2; };
template <> struct VGroup<float> { using type = float4; static constexpr int n = 4; };
template <class S> using vgroup_t = typename VGroup<S>::type;
template <class S> inline constexpr int kVG = VGroup<S>::n;

template <class S, int KB, bool kG>
struct SliceRegs {
    // window loads: real in pairs (window start even, length even), complex one per lane
    static constexpr int NW = is_real_v<S> ? kSliceWin / 128 : kSliceWin / 64;
    using WT = pair_t<S>;
    // real values are stored in lane groups (entries g j .. g j + g - 1 of a row adjacent, g = 2 for
    // f64, 4 for f32): one 16-byte load per group
    static constexpr int NV = (KB + kVG<S> - 1) / kVG<S>;
    using VT = vgroup_t<S>;
    VT v[NV];
    // window slices: packed 8-bit offsets in c[0 .. ceil(KB/4)); gather slices (kG): int32 columns
    uint32_t c[kG ? KB : (KB + 3) / 4];
    WT w[NW];
    int len;          // the lane's row length
};

template <class S, int KB, bool kG>
__device__ __forceinline__ S slice_val(const SliceRegs<S, KB, kG>& R, int u) {
    if constexpr (kVG<S> == 2) return (u & 1) ? R.v[u >> 1].y : R.v[u >> 1].x;
    else if constexpr (kVG<S> == 4) {
        const float4 q = R.v[u >> 2];
        return (u & 3) == 0 ? q.x : (u & 3) == 1 ? q.y : (u & 3) == 2 ? q.z : q.w;
    } else return R.v[u];
}
// stream index of entry (k, lane) of a slice whose values start at off
template <class S>
__device__ __forceinline__ uint32_t slice_entry(uint32_t off, int k, int lane) {
    constexpr uint32_t g = kVG<S>;
    return off + 64u * g * (uint32_t)(k / (int)g) + g * (uint32_t)lane + (uint32_t)(k % (int)g);
}

// Every load of one slice's first KB entries, its window and the row lengths.  Loads are clamped
// (to entry K-1, window entry wl-1): same cache lines, no extra bytes, no exec-masked loads.
template <class S, int KB, bool kG, bool kDist = false>
__device__ __forceinline__ void slice_issue(const CsrArgs<S>& a, const S* xin, int slice, int4 m,
                                            SliceRegs<S, KB, kG>& R, const S* gin = nullptr) {
    const int lane = threadIdx.x & 63;
    // K = 0 (all rows empty) clamps to entry 0 of the slice: the streams carry one slice of
    // padding past their end, so even an empty last slice loads in bounds
    const int K = max(m.z & 0xff, 1);
    const S* sval = a.sval;
    const uint32_t* scol8 = a.scol8;
    const int32_t* scol32 = a.scol32;
    if (a.nseg > 1) {   // a dynamically indexed kernel argument costs a scalar load per slice
        const int seg = (m.z >> kSliceSegShift) & (kMaxSliceSeg - 1);   // wave-uniform
        sval += a.seg_val[seg];
        scol8 += a.seg_c8[seg];
        scol32 += a.seg_c32[seg];
    }
    const uint32_t base = (uint32_t)m.x + (uint32_t)lane;
    R.len = m.z & 0xff;
    if (m.z & 0x100) R.len = a.slen[min(slice * kSliceRows + lane, a.nrows - 1)];
    if constexpr (is_real_v<S>) {
        constexpr int g = kVG<S>;
        const int Kg = (K + g - 1) / g;
        const uint32_t bg = ((uint32_t)m.x / (uint32_t)g) + (uint32_t)lane;
#pragma unroll
        for (int j = 0; j < SliceRegs<S, KB, kG>::NV; ++j)
            R.v[j] = ldg_stream(reinterpret_cast<const vgroup_t<S>*>(sval), bg + 64u * (uint32_t)min(j, Kg - 1));
    } else {
#pragma unroll
        for (int u = 0; u < KB; ++u) R.v[u] = ldg_stream(sval, base + 64u * (uint32_t)min(u, K - 1));
    }
    if (m.y >= 0) {
        const int nw = (K + 3) >> 2;
#pragma unroll
        for (int g = 0; g < (KB + 3) / 4; ++g)
            R.c[g] = ldg_stream(scol8, (uint32_t)m.w + 64u * (uint32_t)min(g, nw - 1) + (uint32_t)lane);
        // the window always holds the slice's own rows (the Rayleigh term reads them)
        const int wl = max((m.z >> 9) & 0x1ff, 1);
        if (kDist && (m.z & kGhostSliceBit)) {
#pragma unroll
            for (int j = 0; j < SliceRegs<S, KB, kG>::NW; ++j) {
                if constexpr (is_real_v<S>) {
                    const int e = m.y + 2 * min(lane + 64 * j, (wl >> 1) - 1);
                    R.w[j].x = ld_x_peer(a, xin, gin, e);
                    R.w[j].y = ld_x_peer(a, xin, gin, e + 1);
                } else {
                    R.w[j] = ld_x_peer(a, xin, gin, m.y + min(lane + 64 * j, wl - 1));
                }
            }
        } else
#pragma unroll
        for (int j = 0; j < SliceRegs<S, KB, kG>::NW; ++j)
            if constexpr (is_real_v<S>)
                R.w[j] = ldg(reinterpret_cast<const pair_t<S>*>(xin),
                             (uint32_t)((m.y >> 1) + min(lane + 64 * j, (wl >> 1) - 1)));
            else
                R.w[j] = ldg(xin, (uint32_t)(m.y + min(lane + 64 * j, wl - 1)));
    } else if constexpr (kG) {
#pragma unroll
        for (int u = 0; u < KB; ++u)
            R.c[u] = (uint32_t)ldg_stream(scol32, (uint32_t)m.w + 64u * (uint32_t)min(u, K - 1) + (uint32_t)lane);
    }
}

// Row sums of one slice from its registers (window slices: x from the wave's LDS window).
template <class S>
__device__ __forceinline__ S shfl_s(S v, int src) {
    if constexpr (is_real_v<S>) return __shfl(v, src, 64);
    else return S{__shfl(v.re, src, 64), __shfl(v.im, src, 64)};
}

template <class S, bool kPower, int KB, bool kG, bool kDist = false>
__device__ __forceinline__ void slice_compute(const CsrArgs<S>& a, const S* xin, S* yout, double nrm,
                                              const SliceRegs<S, KB, kG>& R, int4 mc, int sl, S* xw,
                                              double& n2, double& rr, double& ri, const S* gin = nullptr,
                                              int parity = 0) {
    const int lane = threadIdx.x & 63;
    const int K = mc.z & 0xff;
    const S* sval = a.sval;
    const uint32_t* scol8 = a.scol8;
    const int32_t* scol32 = a.scol32;
    if (a.nseg > 1) {
        const int seg = (mc.z >> kSliceSegShift) & (kMaxSliceSeg - 1);
        sval += a.seg_val[seg];
        scol8 += a.seg_c8[seg];
        scol32 += a.seg_c32[seg];
    }
    const int row = sl * kSliceRows + lane;
    const bool valid = row < a.nrows;
    const int rowc = valid ? row : a.nrows - 1;
    S sacc = s_zero<S>();
    S xi = s_zero<S>();
    if (mc.y >= 0) {
        const int w0 = mc.y, wl = (mc.z >> 9) & 0x1ff;
#pragma unroll
        for (int j = 0; j < SliceRegs<S, KB, kG>::NW; ++j) {
            if constexpr (is_real_v<S>) {
                pair_t<S> v = R.w[j];
                if constexpr (kPower) {
                    v.x = scale_in(v.x, nrm);
                    v.y = scale_in(v.y, nrm);
                }
                if (2 * (lane + 64 * j) < wl) *reinterpret_cast<pair_t<S>*>(xw + 2 * (lane + 64 * j)) = v;
            } else {
                S v = R.w[j];
                if constexpr (kPower) v = scale_in(v, nrm);
                if (lane + 64 * j < wl) xw[lane + 64 * j] = v;
            }
        }
        // wave-private region: LDS executes one wave's accesses in order; the fences only keep
        // the compiler from moving the reads above the stores
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int u = 0; u < KB; ++u) {
            const S pr = mul(slice_val(R, u), xw[(R.c[u >> 2] >> (8 * (u & 3))) & 0xffu]);
            if (u < R.len) sacc = add(sacc, pr);
        }
        for (int k0 = KB & ~3; k0 < K; k0 += 4) {  // rows longer than KB entries (offset words of 4)
            const uint32_t cw = ldg(scol8, (uint32_t)mc.w + 64u * (uint32_t)(k0 >> 2) + (uint32_t)lane);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const S pr = mul(ldg(sval, slice_entry<S>((uint32_t)mc.x, min(k0 + u, K - 1), lane)),
                                 xw[(cw >> (8 * u)) & 0xffu]);
                if (k0 + u >= KB && k0 + u < R.len) sacc = add(sacc, pr);
            }
        }
        if constexpr (kPower) xi = xw[min(max(rowc + a.xoff - w0, 0), wl - 1)];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    } else if constexpr (kG) {
        S xv[KB];
        const bool ghost = kDist && (mc.z & kGhostSliceBit);
        if (ghost) {
#pragma unroll
            for (int u = 0; u < KB; ++u) xv[u] = ld_x_peer(a, xin, gin, (int)R.c[u]);
        } else {
#pragma unroll
            for (int u = 0; u < KB; ++u) xv[u] = ldg(xin, R.c[u]);
        }
#pragma unroll
        for (int u = 0; u < KB; ++u) {
            S x = xv[u];
            if constexpr (kPower) x = scale_in(x, nrm);
            const S pr = mul(slice_val(R, u), x);
            if (u < R.len) sacc = add(sacc, pr);
        }
        for (int k0 = KB; k0 < K; ++k0) {
            const uint32_t q = (uint32_t)lane + 64u * (uint32_t)k0;
            const uint32_t cc = (uint32_t)ldg(scol32, (uint32_t)mc.w + q);
            S x = ghost ? ld_x_peer(a, xin, gin, (int)cc) : ldg(xin, cc);
            if constexpr (kPower) x = scale_in(x, nrm);
            const S pr = mul(ldg(sval, slice_entry<S>((uint32_t)mc.x, k0, lane)), x);
            if (k0 < R.len) sacc = add(sacc, pr);
        }
        if constexpr (kPower) xi = scale_in(xin[rowc + a.xoff], nrm);
    }
    if (valid) {
        yout[row] = sacc;   // a non-temporal store measured slower: the next launch reads y as x
        if constexpr (kPower) {
            n2 += sq_abs(sacc);
            acc_dot(rr, ri, xi, sacc);
        }
    }
    if constexpr (kDist) {
        // halo: the rows other ranks read go straight into their inboxes (system-scope stores,
        // drained before the block's ticket); a slice's entries are contiguous in the push list
        const int2 pr = ld_uniform(a.peer.slice_push, sl);
        for (int e0 = pr.x; e0 < pr.y; e0 += 64) {
            const int e = e0 + lane;
            const int4 en = a.peer.push[min(e, pr.y - 1)];
            const S v = shfl_s(sacc, en.x - sl * kSliceRows);
            if (e < pr.y) st_sys_s(peer_ghosts<S>(a.peer.peers[en.y], parity, a.peer.ghost_stride) + en.z, v);
        }
    }
}

// Rounds of slice loads a wave keeps in flight (software pipeline depth) and slices per round,
// from the size of one slice's registers: band10m (f64, 12 entries per row, 36 VGPRs per slice)
// measured 205.6 us unpipelined with two slices per round, 194.5 us at depth 1 and 191 us at
// depth 2 with one slice per round (depth 3+: register pressure, 214 us).  EIGSOL_SLICE_PIPE /
// EIGSOL_SLICE_NS (compile time) override for A/B builds.
template <class S, int KB, bool kG>
struct SlicePlan {
    static constexpr int bytes = (int)sizeof(SliceRegs<S, KB, kG>);
#ifdef EIGSOL_SLICE_PIPE
    static constexpr int pipe = EIGSOL_SLICE_PIPE;
#else
    static constexpr int pipe = bytes <= 160 ? 2 : (bytes <= 320 ? 1 : 0);
#endif
#ifdef EIGSOL_SLICE_NS
    static constexpr int ns = EIGSOL_SLICE_NS;
#else
    static constexpr int ns = pipe > 0 ? 1 : 2;
#endif
};
// float: a slice's registers are small enough that four slices per round, all loads issued before
// any is consumed, beat the software pipeline: band10m f32 149.3 -> 130.9 us (6.16 -> 7.03 TB/s
// algorithmic), 1M x 16 band 23.6 -> 21.6 us; two / three slices with a pipeline 141-142 / 136 us
// (tools/f32_ab.sh)
#if !defined(EIGSOL_SLICE_PIPE) && !defined(EIGSOL_SLICE_NS)
template <int KB, bool kG>
struct SlicePlan<float, KB, kG> {
    static constexpr int bytes = (int)sizeof(SliceRegs<float, KB, kG>);
    static constexpr int pipe = 0;
    static constexpr int ns = 4;
};
#endif

template <class S, bool kPower, int KB, bool kG, bool kDist = false>
__global__ __launch_bounds__(kThreads) void csr_slice_kernel(CsrArgs<S> a, int parity) {
    constexpr int kSliceNS = SlicePlan<S, KB, kG>::ns;   // slices per round
    constexpr int kPipe = SlicePlan<S, KB, kG>::pipe;    // rounds in flight while one computes
    __shared__ __align__(16) S xw_all[kWaves][kSliceNS][kSliceWin];
    __shared__ double sm[3 * kWaves];
    __shared__ Prologue pro;
    __shared__ int s_last;

    const S* xin;
    S* yout;
    double nrm = 0.0;
    const S* gin = nullptr;   // peer exchange: ghost entries of the input (inbox, previous parity)
    if constexpr (kPower) {
        power_prologue<S>(a.ctl, a.rank_part, a.nranks, parity, a.trace, &pro, kDist ? &a.peer : nullptr);
        if (!__builtin_amdgcn_readfirstlane(pro.go)) return;   // block-uniform exit
        nrm = pro.nrm;
        xin = parity ? a.buf0 : a.buf1;
        yout = (parity ? a.buf1 : a.buf0) + a.xoff;   // y rows land at their x-space slots
        if constexpr (kDist) gin = peer_ghosts<S>(a.peer.inbox, parity ^ 1, a.peer.ghost_stride);
    } else {
        xin = a.x_plain;
        yout = a.y_plain;
    }
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double n2 = 0.0, rr = 0.0, ri = 0.0;

    // XCD-contiguous slice ranges; each wave takes kSliceNS slices (wpg apart) per round, all
    // of whose loads are issued before any of them is consumed
    const int wpg = (gridDim.x >> 3) * kWaves;          // waves per XCD group (grid % 8 == 0)
    const int chunk = (a.nslices + 7) >> 3;
    const int sbeg = (blockIdx.x & 7) * chunk;
    const int send = min(a.nslices, sbeg + chunk);
    const int step = kSliceNS * wpg;
    auto issue = [&](SliceRegs<S, KB, kG>(&R)[kSliceNS], int4(&mc)[kSliceNS], int s0) {
#pragma unroll
        for (int i = 0; i < kSliceNS; ++i) mc[i] = ld_uniform(a.slice_meta, min(s0 + i * wpg, send - 1));
#pragma unroll
        for (int i = 0; i < kSliceNS; ++i)   // past the range: reloads the last slice, unused
            slice_issue<S, KB, kG, kDist>(a, xin, min(s0 + i * wpg, send - 1), mc[i], R[i], gin);
    };
    auto compute = [&](const SliceRegs<S, KB, kG>(&R)[kSliceNS], const int4(&mc)[kSliceNS], int s0) {
#pragma unroll
        for (int i = 0; i < kSliceNS; ++i)
            if (i == 0 || s0 + i * wpg < send)
                slice_compute<S, kPower, KB, kG, kDist>(a, xin, yout, nrm, R[i], mc[i], s0 + i * wpg, xw_all[wave][i],
                                                        n2, rr, ri, gin, parity);
    };
    int sl = sbeg + (blockIdx.x >> 3) * kWaves + wave;
    if constexpr (kPipe == 1) {
        // software pipeline, unrolled by two so both register sets have static names: the next
        // round's loads are in flight while this round computes
        SliceRegs<S, KB, kG> RA[kSliceNS], RB[kSliceNS];
        int4 ma[kSliceNS], mb[kSliceNS];
        if (sl < send) issue(RA, ma, sl);
        while (sl < send) {
            if (sl + step < send) issue(RB, mb, sl + step);
            compute(RA, ma, sl);
            sl += step;
            if (sl >= send) break;
            if (sl + step < send) issue(RA, ma, sl + step);
            compute(RB, mb, sl);
            sl += step;
        }
    } else if constexpr (kPipe >= 2) {
        // two rounds in flight while one computes (unrolled by three)
        SliceRegs<S, KB, kG> RA[kSliceNS], RB[kSliceNS], RC[kSliceNS];
        int4 ma[kSliceNS], mb[kSliceNS], mcc[kSliceNS];
        if (sl < send) issue(RA, ma, sl);
        if (sl + step < send) issue(RB, mb, sl + step);
        while (sl < send) {
            if (sl + 2 * step < send) issue(RC, mcc, sl + 2 * step);
            compute(RA, ma, sl);
            sl += step;
            if (sl >= send) break;
            if (sl + 2 * step < send) issue(RA, ma, sl + 2 * step);
            compute(RB, mb, sl);
            sl += step;
            if (sl >= send) break;
            if (sl + 2 * step < send) issue(RB, mb, sl + 2 * step);
            compute(RC, mcc, sl);
            sl += step;
        }
    } else {
        for (; sl < send; sl += step) {
            SliceRegs<S, KB, kG> R[kSliceNS];
            int4 mc[kSliceNS];
            issue(R, mc, sl);
            compute(R, mc, sl);
        }
    }
    if constexpr (kPower) {
        if constexpr (kDist) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // halo stores drained
        block_sum3(n2, rr, ri, sm);
        last_arriver_reduce(n2, rr, ri, a.blk_part, &a.ctl->counter, a.my_part, sm, &s_last);
        if constexpr (kDist) {
            if (threadIdx.x == 0 && s_last) {
                const part4 mine = *a.my_part;
                peer_publish(a.peer, parity, mine, (uint64_t)pro.t + 2);
            }
        }
    }
}

// Start of a peer-exchange session (begin(), after the x0 norm partial): x0's halo rows and the
// rank partial go to every inbox's parity-1 slots (launch 0 reads them as "launch -1"), then flag
// epoch 1.  One block.
template <class S>
__global__ __launch_bounds__(kThreads) void peer_begin_kernel(PeerArgs pa, const S* x_own, int64_t npush,
                                                              const part4* mine) {
    for (int64_t e = threadIdx.x; e < npush; e += kThreads) {
        const int4 en = pa.push[e];
        st_sys_s(peer_ghosts<S>(pa.peers[en.y], 1, pa.ghost_stride) + en.z, x_own[en.x]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) peer_publish(pa, 1, *mine, 1);
}

// ||x||^2 partials of the start vector (x.normalize(), power_method.hpp:62).
template <class S>
__global__ __launch_bounds__(kThreads) void norm_partial_kernel(const S* x, int64_t n, PowerCtl* ctl,
                                                                part4* blk_part, part4* out) {
    __shared__ double sm[3 * kWaves];
    __shared__ int s_last;
    double n2 = 0.0, z1 = 0.0, z2 = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kThreads)
        n2 += sq_abs(x[i]);
    block_sum3(n2, z1, z2, sm);
    last_arriver_reduce(n2, z1, z2, blk_part, &ctl->counter, out, sm, &s_last);
}

// Single-precision matrices the sliced layout cannot hold (a row longer than 64 entries, or
// too much padding): one row per lane, its entries summed sequentially in ascending column order
// (the reference's CSC scatter order, bitwise), fused power epilogue.  Uncoalesced, but only the
// fallback layout of the float / complex<float> instantiations.
template <class S, bool kPower>
__global__ __launch_bounds__(kThreads) void csr_row_kernel(CsrArgs<S> a, int parity) {
    __shared__ double sm[3 * kWaves];
    __shared__ Prologue pro;
    __shared__ int s_last;
    const S* xin;
    S* yout;
    double nrm = 0.0;
    if constexpr (kPower) {
        power_prologue<S>(a.ctl, a.rank_part, a.nranks, parity, a.trace, &pro);
        if (!__builtin_amdgcn_readfirstlane(pro.go)) return;   // block-uniform exit
        nrm = pro.nrm;
        xin = parity ? a.buf0 : a.buf1;
        yout = (parity ? a.buf1 : a.buf0) + a.xoff;
    } else {
        xin = a.x_plain;
        yout = a.y_plain;
    }
    double n2 = 0.0, rr = 0.0, ri = 0.0;
    for (int r = blockIdx.x * kThreads + threadIdx.x; r < a.nrows; r += gridDim.x * kThreads) {
        S acc = s_zero<S>();
        const int e1 = a.rowptr[r + 1];
        for (int e = a.rowptr[r]; e < e1; ++e) {
            S x = xin[a.col[e]];
            if constexpr (kPower) x = scale_in(x, nrm);
            acc = add(acc, mul(a.val[e], x));
        }
        yout[r] = acc;
        if constexpr (kPower) {
            const S xi = scale_in(xin[r + a.xoff], nrm);
            n2 += sq_abs(acc);
            acc_dot(rr, ri, xi, acc);
        }
    }
    if constexpr (kPower) {
        block_sum3(n2, rr, ri, sm);
        last_arriver_reduce(n2, rr, ri, a.blk_part, &a.ctl->counter, a.my_part, sm, &s_last);
    }
}

// Column-binned SpMV for gather-bound matrices (uniform columns, x larger than the L2s).  Rows go
// in chunks of kBinRows<S> whose row sums live in LDS, and a chunk's entries are grouped by column
// block.  A workgroup walks its chunk block by block, so the resident workgroups sweep x together
// and each block's gathers hit the L2 after the first touch, instead of one cache line fetched from
// the Infinity Cache per gathered word.  Inside a block, a row's entries form one run (its entries
// are ascending); runs are sorted longest first and run i belongs to lane i % kNT of the step that
// covers it.  Level l of the block holds the l-th entry of every run longer than l, so the lanes'
// loads of one level are contiguous (16-byte-free but coalesced), and a lane adds its run's entries
// to the row sum in register, in ascending column order.  A row has one run per block, so only the
// block boundaries need a barrier; every row is summed in ascending column order across blocks --
// the reference's CSC scatter order, bit for bit.  Entries pack (row in chunk, column in block) in
// 32 bits: 12 bytes per f64 entry, the CSR stream's size, and no row pointers.
// kKB: KB of LDS row sums per workgroup (16: more workgroups per CU, for matrices with few row
// chunks; 64: more rows per chunk, hence more runs per step); kNT threads per workgroup.
// Step (int4): {index of its first level in the level table, levels | barrier << 8, first run, block};
// level table (int2): {entry offset, runs at this level}.  A step covers runs [first, first + kNT)
// and at most kBinLev levels; the host cuts longer runs into several steps (same lanes, no barrier).
template <class S, int kKB> inline constexpr int kBinRows = kKB * 1024 / (int)sizeof(S);
constexpr int kBinLev = 4;
// the largest row-sum array one workgroup can hold beside its other LDS (160 KiB per CU): one
// workgroup per CU, e.g. 10M f64 rows in two exact rounds of 19532-row chunks over 256 CUs
constexpr int kBinKBMax = 153;
#ifndef EIGSOL_BIN_COND
#define EIGSOL_BIN_COND 1
#endif
constexpr bool kBinCondLoads = EIGSOL_BIN_COND;   // levels >= 1: loads only in waves that use them

template <class S>
struct BinRegs {
    uint32_t pk[kBinLev];
    S v[kBinLev];
    S x[kBinLev];
    int c[kBinLev];   // runs at each level (wave-uniform)
    int nl, bar, i;   // levels, barrier after, this lane's run
    uint32_t xb;
};

// LDS-only barrier: the row sums are the only data the waves share, so only the LDS counter is
// drained; loads of later steps stay in flight across it (__syncthreads would drain them too).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <class S, bool kPower, int kKB, int kNT>
__global__ __launch_bounds__(kNT) void csr_bin_kernel(CsrArgs<S> a, int parity) {
    constexpr int kRows = kBinRows<S, kKB>;
    __shared__ S acc[kRows + 1];
    __shared__ double sm[3 * (kNT / 64)];
    __shared__ Prologue pro;
    __shared__ int s_last;
    const S* xin;
    S* yout;
    double nrm = 0.0;
    if constexpr (kPower) {
        power_prologue<S>(a.ctl, a.rank_part, a.nranks, parity, a.trace, &pro, nullptr, a.cont != 0);
        if (!__builtin_amdgcn_readfirstlane(pro.go)) return;   // block-uniform exit
        nrm = pro.nrm;
        xin = parity ? a.buf0 : a.buf1;
        yout = (parity ? a.buf1 : a.buf0) + a.xoff;   // y rows land at their x-space slots (row shards)
    } else {
        xin = a.x_plain;
        yout = a.y_plain;
    }
    const int cb = a.bcbits;
    const uint32_t cmask = (1u << cb) - 1u;
    const int tid = threadIdx.x;
    const int wbase = __builtin_amdgcn_readfirstlane(tid & ~63);
    // three steps in flight: entries of step s+2 loading, x of step s+1 gathering, step s adding.
    // Level 0 loads are unconditional (clamped); levels >= 1, which few runs reach, are loaded only
    // by waves with a lane there (10M uniform: 0.89 ms against 1.29 ms with every level loaded).
    auto load_pv = [&](BinRegs<S>& R, int st) {
        const int4 m = ld_uniform(a.bstep, st);
        R.nl = m.y & 0xff;
        R.bar = m.y & 0x100;
        R.i = m.z + tid;
        R.xb = (uint32_t)m.w << cb;
#pragma unroll
        for (int l = 0; l < kBinLev; ++l) {
            const int2 lv = ld_uniform(a.blev, m.x + min(l, R.nl - 1));
            R.c[l] = l < R.nl ? lv.y : 0;
            const uint32_t e = (uint32_t)lv.x + (uint32_t)min(R.i, lv.y - 1);
            if (kBinCondLoads && l > 0 && m.z + wbase >= R.c[l]) continue;   // no lane of this wave at level l
            R.pk[l] = ldg_stream(a.bpk, e);
            R.v[l] = ldg_stream(a.bval, e);
        }
    };
    auto load_x = [&](BinRegs<S>& R) {
#pragma unroll
        for (int l = 0; l < kBinLev; ++l) {
            if (kBinCondLoads && l > 0 && (R.i - tid) + wbase >= R.c[l]) continue;
            R.x[l] = ldg(xin, R.xb + (R.pk[l] & cmask));
        }
    };
    auto apply = [&](const BinRegs<S>& R) {
        // lanes without a run add into the spare slot acc[kRows]
        const int r = R.i < R.c[0] ? (int)(R.pk[0] >> cb) : kRows;
        S sum = acc[r];
#pragma unroll
        for (int l = 0; l < kBinLev; ++l) {
            if (l > 0 && (R.i - tid) + wbase >= R.c[l]) break;   // no lane of this wave at level l
            S xv = R.x[l];
            if constexpr (kPower) xv = scale_in(xv, nrm);
            const S t = add(sum, mul(R.v[l], xv));
            sum = R.i < R.c[l] ? t : sum;
        }
        acc[r] = sum;
        if (R.bar) lds_barrier();   // the next block's runs may belong to other lanes
    };
    double n2 = 0.0, rr = 0.0, ri = 0.0;
    for (int c = a.cbeg + blockIdx.x; c < a.cend; c += gridDim.x) {
        const int r0 = c * a.brows;
        const int nr = min(a.brows, a.nrows - r0);
        for (int i = tid; i < nr; i += kNT) acc[i] = s_zero<S>();
        __syncthreads();
        const int s0 = a.bchunk[c], s1 = a.bchunk[c + 1];
        if (s0 < s1) {
            const int sl = s1 - 1;
            BinRegs<S> RA, RB, RC;
            load_pv(RA, s0);
            load_pv(RB, min(s0 + 1, sl));
            load_x(RA);
            for (int st = s0;; st += 3) {
                load_pv(RC, min(st + 2, sl));
                load_x(RB);
                apply(RA);
                if (st + 1 > sl) break;
                load_pv(RA, min(st + 3, sl));
                load_x(RC);
                apply(RB);
                if (st + 2 > sl) break;
                load_pv(RB, min(st + 4, sl));
                load_x(RA);
                apply(RC);
                if (st + 3 > sl) break;
            }
        }
        __syncthreads();
        for (int i = tid; i < nr; i += kNT) {
            const S y = acc[i];
            yout[r0 + i] = y;
            if constexpr (kPower) {
                const S xi = scale_in(xin[r0 + i + a.xoff], nrm);
                n2 += sq_abs(y);
                acc_dot(rr, ri, xi, y);
            }
        }
        __syncthreads();   // the next chunk clears acc
    }
    if constexpr (kPower) {
        block_sum3<kNT>(n2, rr, ri, sm);
        last_arriver_reduce<kNT>(n2, rr, ri, a.blk_part, &a.ctl->counter, a.my_part, sm, &s_last, a.cont != 0);
    }
}

// x_out = src / nrm (the reference's x = y / normY of the final iterate; unchanged if nrm == 0).
template <class S>
__global__ __launch_bounds__(kThreads) void scale_out_kernel(const S* src, double nrm, S* dst,
                                                             int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kThreads)
        dst[i] = scale_in(src[i], nrm);
}

}  // namespace dev
}  // namespace eigsol

using namespace eigsol;
using namespace eigsol::dev;

namespace eigsol {

void csr_retain(eigsol_csr* A) { A->refs.fetch_add(1); }

void csr_release(eigsol_csr* A) {
    if (!A || A->refs.fetch_sub(1) != 1) return;
    (void)hipSetDevice(A->ctx->device);
    (void)hipStreamSynchronize(A->ctx->stream);
    if (A->rowptr) (void)hipFree(A->rowptr);
    if (A->col) (void)hipFree(A->col);
    if (A->col16) (void)hipFree(A->col16);
    if (A->val) (void)hipFree(A->val);
    if (A->tile_meta) (void)hipFree(A->tile_meta);
    if (A->tile_win) (void)hipFree(A->tile_win);
    for (void* q : {(void*)A->slice_meta, A->sval, (void*)A->scol8, (void*)A->scol32, (void*)A->slen})
        if (q) (void)hipFree(q);
    if (A->send_idx) (void)hipFree(A->send_idx);
    if (A->send_buf) (void)hipFree(A->send_buf);
    for (eigsol_csr* B : A->cblk) csr_release(B);
    if (A->shadow) csr_release(A->shadow);
    for (void* q : {(void*)A->bpk, A->bval, (void*)A->bstep, (void*)A->blev, (void*)A->bchunk})
        if (q) (void)hipFree(q);
    eigsol_ctx* c = A->ctx;
    delete A;
    ctx_release(c);
}

// ---------------------------------------------------------------- host: CSR build / upload
// Row tiles: short tiles (consecutive rows, <= kTileRows rows, <= tile_nnz nonzeros) first, in
// row order, then one tile per long row.  meta = {r0, r1, e0, e1} per tile.
static int build_tiles(const int32_t* rowptr, const int32_t* col, int64_t nrows, int64_t xoff,
                       int tile_nnz, int win_cap, std::vector<int32_t>& meta, std::vector<int32_t>& win,
                       int32_t& nshort, int32_t& max_rows, int32_t& windowed) {
    std::vector<int32_t> shorts, longs;
    shorts.reserve(4 * (nrows / 64 + 2));
    max_rows = 0;
    auto push = [](std::vector<int32_t>& v, int64_t r0, int64_t r1, const int32_t* rp) {
        v.push_back((int32_t)r0);
        v.push_back((int32_t)r1);
        v.push_back(rp[r0]);
        v.push_back(rp[r1]);
    };
    int64_t r = 0;
    while (r < nrows) {
        const int64_t len = rowptr[r + 1] - rowptr[r];
        if (len > tile_nnz) {
            push(longs, r, r + 1, rowptr);
            ++r;
            continue;
        }
        int64_t nz = len;
        int64_t rr = r + 1;
        while (rr < nrows && rr - r < kTileRows) {
            const int64_t l2 = rowptr[rr + 1] - rowptr[rr];
            if (l2 > tile_nnz || nz + l2 > tile_nnz) break;
            nz += l2;
            ++rr;
        }
        max_rows = std::max(max_rows, (int32_t)(rr - r));
        push(shorts, r, rr, rowptr);
        r = rr;
    }
    nshort = (int32_t)(shorts.size() / 4);
    // x window of each short tile: [min(first row, min column), max(last row, max column)]
    win.assign(2 * std::max<int32_t>(nshort, 1), 0);
    windowed = nshort > 0 ? 1 : 0;
    for (int32_t i = 0; i < nshort; ++i) {
        const int32_t r0 = shorts[4 * i] + xoff, r1 = shorts[4 * i + 1] + xoff;   // x-space rows
        int32_t w0 = r0, w1 = r1 - 1;
        for (int32_t k = shorts[4 * i + 2]; k < shorts[4 * i + 3]; ++k) {
            w0 = std::min(w0, col[k]);
            w1 = std::max(w1, col[k]);
        }
        win[2 * i] = w0;
        win[2 * i + 1] = w1;
        if (w1 - w0 + 1 > win_cap) windowed = 0;
    }
    meta = std::move(shorts);
    meta.insert(meta.end(), longs.begin(), longs.end());
    if (meta.empty()) meta.assign(4, 0);
    return (int)(nshort + longs.size() / 4);
}

// Sliced layout: slices of 64 rows, K_s = longest row of the slice, value entry (k, lane) at
// off_s + 64 k + lane (padding entries: value 0, masked by the row length).  Columns: window
// slices hold 8-bit offsets from the window start, entry (k, lane) in byte k % 4 of dword
// coff_s + 64 (k / 4) + lane; gather slices hold int32 x-space columns at goff_s + 64 k + lane.
// Used when every row has at most kSliceMaxK entries and padding adds at most 1/8 of the entries.
struct SliceLayout {
    std::vector<int32_t> meta;
    std::vector<unsigned char> val;
    std::vector<uint32_t> c8;
    std::vector<int32_t> c32;
    std::vector<uint8_t> len;
    int maxk = 0;
    bool any_gather = false;   // some slice's window does not fit: gather instantiation
    int nseg = 1;              // stream segments (kSliceSegShift): element offsets of their starts
    int64_t seg_val[kMaxSliceSeg] = {0}, seg_c8[kMaxSliceSeg] = {0}, seg_c32[kMaxSliceSeg] = {0};
};

// Largest stream segment in bytes (32-bit offsets inside a segment).  EIGSOL_SLICE_SEG_BYTES
// lowers it so that tests exercise several segments on small matrices.
static int64_t slice_seg_bytes() {
    int64_t lim = (int64_t(1) << 32) - (int64_t(1) << 20);
    if (const char* e = std::getenv("EIGSOL_SLICE_SEG_BYTES")) lim = std::max<int64_t>(1 << 16, std::min<int64_t>(lim, std::atoll(e)));
    return lim;
}

static bool build_slices(const int32_t* rowptr, const int32_t* col, const void* values, size_t sb, int vg,
                         int64_t nrows, int64_t nnz, int64_t xoff, int64_t xlen, SliceLayout& L) {
    if (nrows == 0 || xlen == 0) return false;
    const int64_t ns = (nrows + kSliceRows - 1) / kSliceRows;
    int64_t total = 0, ctot8 = 0, ctot32 = 0;
    bool any_ragged = false;
    const int64_t seg_lim = slice_seg_bytes();
    int seg = 0;
    L.meta.assign(4 * ns, 0);
    for (int64_t s = 0; s < ns; ++s) {
        const int64_t r0 = s * kSliceRows, r1 = std::min<int64_t>(nrows, r0 + kSliceRows);
        int K = 0, kmin = INT32_MAX;
        int32_t w0 = (int32_t)(r0 + xoff), w1 = (int32_t)(r1 - 1 + xoff);
        for (int64_t r = r0; r < r1; ++r) {
            const int l = rowptr[r + 1] - rowptr[r];
            if (l > kSliceMaxK) return false;
            K = std::max(K, l);
            kmin = std::min(kmin, l);
            for (int32_t e = rowptr[r]; e < rowptr[r + 1]; ++e) {
                w0 = std::min(w0, col[e]);
                w1 = std::max(w1, col[e]);
            }
        }
        const bool ragged = kmin != K || (r1 - r0) != kSliceRows;
        // rows past the end of x (rectangular plain SpMV) need no x entry of their own
        w1 = (int32_t)std::min<int64_t>(w1, xlen - 1);
        w0 = std::min(w0, w1);
        bool win = true;
        const bool pairs = vg > 1;   // real scalars
        if (pairs) {
            // real windows load in aligned pairs: even start and even length inside x
            w0 &= ~1;
            if (((int64_t)w1 - w0 + 1) & 1) {
                if (w1 + 1 < xlen) ++w1;
                else win = false;
            }
        }
        const int64_t wl = (int64_t)w1 - w0 + 1;
        win = win && wl <= kSliceWin;
        // row-sharded x-space: does the slice read ghost entries (x-space indices outside its own
        // rank's rows)?  Only the peer-exchange kernel looks at the bit.
        bool ghost = false;
        if (win) {
            ghost = w0 < xoff || (int64_t)w1 >= xoff + nrows;
        } else {
            for (int64_t e = rowptr[r0]; e < rowptr[r1] && !ghost; ++e)
                ghost = col[e] < xoff || col[e] >= xoff + nrows;
        }
        any_ragged |= ragged;
        L.maxk = std::max(L.maxk, K);
        const int64_t nv = (int64_t)((K + vg - 1) / vg * vg) * kSliceRows;   // whole lane groups
        const int64_t n8 = win ? (int64_t)((K + 3) / 4) * kSliceRows : 0;
        const int64_t n32 = win ? 0 : (int64_t)K * kSliceRows;
        // a slice never straddles two segments: start a new one when a stream would pass the limit
        // (the margin covers the clamped loads of an empty slice)
        const int64_t pad = 2 * kSliceMaxK * kSliceRows;
        if ((total - L.seg_val[seg] + nv + pad) * (int64_t)sb > seg_lim ||
            (ctot8 - L.seg_c8[seg] + n8 + pad) * 4 > seg_lim || (ctot32 - L.seg_c32[seg] + n32 + pad) * 4 > seg_lim) {
            if (++seg >= kMaxSliceSeg) return false;
            L.seg_val[seg] = total;
            L.seg_c8[seg] = ctot8;
            L.seg_c32[seg] = ctot32;
        }
        L.meta[4 * s] = (int32_t)(total - L.seg_val[seg]);
        L.meta[4 * s + 1] = win ? w0 : -1;
        L.meta[4 * s + 2] = K | (ragged ? 0x100 : 0) | (win ? (int32_t)(wl << 9) : 0) | (ghost ? kGhostSliceBit : 0) |
                            (seg << kSliceSegShift);
        L.meta[4 * s + 3] = (int32_t)(win ? ctot8 - L.seg_c8[seg] : ctot32 - L.seg_c32[seg]);
        total += nv;
        ctot8 += n8;
        ctot32 += n32;
        L.any_gather |= !win;
        // padding beyond the lane-group rounding at most 1/8 of the entries
        if (total > nnz + nnz / 8 + (int64_t)(vg - 1) * kSliceRows * (s + 1) + 64 * kSliceRows) return false;
    }
    L.nseg = seg + 1;
    // one slice of padding past each stream's end (clamped loads of empty slices stay in bounds)
    L.val.assign((size_t)(total + kSliceRows) * sb, 0);
    L.c8.assign((size_t)(ctot8 + kSliceRows), 0);
    L.c32.assign((size_t)(ctot32 + kSliceRows), 0);
    if (any_ragged) L.len.assign((size_t)nrows, 0);
    for (int64_t s = 0; s < ns; ++s) {
        const int64_t r0 = s * kSliceRows, r1 = std::min<int64_t>(nrows, r0 + kSliceRows);
        const int sg = (L.meta[4 * s + 2] >> kSliceSegShift) & (kMaxSliceSeg - 1);
        const int32_t w0 = L.meta[4 * s + 1];
        const int64_t off = L.seg_val[sg] + L.meta[4 * s];
        const int64_t coff = (w0 >= 0 ? L.seg_c8[sg] : L.seg_c32[sg]) + L.meta[4 * s + 3];
        const int K = L.meta[4 * s + 2] & 0xff;
        for (int64_t r = r0; r < r1; ++r) {
            const int64_t lane = r - r0;
            const int l = rowptr[r + 1] - rowptr[r];
            if (any_ragged) L.len[r] = (uint8_t)l;
            for (int k = 0; k < l; ++k) {
                const int32_t e = rowptr[r] + k;
                const size_t q = (size_t)(off + (int64_t)(k / vg) * vg * kSliceRows + vg * lane + (k % vg));
                std::memcpy(&L.val[q * sb], (const unsigned char*)values + (size_t)e * sb, sb);
                if (w0 >= 0)
                    L.c8[(size_t)(coff + (int64_t)(k / 4) * kSliceRows + lane)] |= (uint32_t)(col[e] - w0) << (8 * (k % 4));
                else
                    L.c32[(size_t)(coff + (int64_t)k * kSliceRows + lane)] = col[e];
            }
            // padding: offset 0 is in the window; gather padding reads the row's own x entry
            if (w0 < 0)
                for (int k = l; k < K; ++k)
                    L.c32[(size_t)(coff + (int64_t)k * kSliceRows + lane)] = (int32_t)std::min<int64_t>(r + xoff, xlen - 1);
        }
    }
    return true;
}

// xoff: x-space index of local row 0 (0 on one GPU; the lower-ghost count when row-sharded)
static int build_col_blocks(eigsol_csr* A, const int32_t* rowptr, const int32_t* col, const void* val);
static int build_bins(eigsol_csr* A, const int32_t* rowptr, const int32_t* col, const void* val);
static thread_local int g_upload_plain = 0;   // > 0: building a column block (tiles only, no blocks)

int csr_upload(eigsol_ctx* ctx, int dtype, int64_t nrows, int64_t ncols, int64_t nnz,
               const int32_t* rowptr, const int32_t* colidx, const void* values, eigsol_csr** out,
               int64_t xoff) {
    const size_t sb = scalar_bytes(dtype);
    // sort columns inside rows when needed (keeps the reference's ascending-column row order)
    std::vector<int32_t> col_sorted;
    std::vector<unsigned char> val_sorted;
    const int32_t* col_use = colidx;
    const void* val_use = values;
    bool sorted = true;
    for (int64_t i = 0; i < nrows && sorted; ++i)
        for (int32_t k = rowptr[i] + 1; k < rowptr[i + 1]; ++k)
            if (colidx[k] < colidx[k - 1]) { sorted = false; break; }
    if (!sorted) {
        col_sorted.assign(colidx, colidx + nnz);
        val_sorted.resize((size_t)nnz * sb);
        std::vector<int32_t> perm;
        for (int64_t i = 0; i < nrows; ++i) {
            const int32_t b = rowptr[i], e = rowptr[i + 1];
            perm.resize(e - b);
            std::iota(perm.begin(), perm.end(), b);
            std::stable_sort(perm.begin(), perm.end(),
                             [&](int32_t x, int32_t y) { return colidx[x] < colidx[y]; });
            for (int32_t k = b; k < e; ++k) {
                col_sorted[k] = colidx[perm[k - b]];
                std::memcpy(&val_sorted[(size_t)k * sb],
                            (const unsigned char*)values + (size_t)perm[k - b] * sb, sb);
            }
        }
        col_use = col_sorted.data();
        val_use = val_sorted.data();
    }
    std::vector<int32_t> meta, win;
    int32_t nshort = 0, max_rows = 0, windowed = 0;
    const bool cx = dtype == EIGSOL_C128;
    const int ntiles = build_tiles(rowptr, col_use, nrows, xoff, cx ? Tile<cplx>::kCap : Tile<double>::kCap,
                                   cx ? Win<cplx>::kWin : Win<double>::kWin, meta, win, nshort,
                                   max_rows, windowed);
    if (const char* env = std::getenv("EIGSOL_CSR_NO_WINDOW")) if (std::atoi(env)) windowed = 0;
    SliceLayout SL;
    bool sliced = g_upload_plain == 0;
    if (g_upload_plain) windowed = 0;
    if (const char* env = std::getenv("EIGSOL_CSR_NO_SLICE")) if (std::atoi(env)) sliced = false;
    if (sliced)
        sliced = build_slices(rowptr, col_use, val_use, sb,
                              dtype == EIGSOL_F64 ? 2 : (dtype == EIGSOL_F32 ? 4 : 1), nrows, nnz, xoff, ncols, SL);

    // the kernels index every stream with 32-bit byte offsets (ldg).  The sliced layout cuts its
    // streams into < 4 GiB segments, so only the vectors are bounded there (n * sizeof(S) < 4 GiB:
    // 536M f64 rows); the tile layouts keep the whole value stream under 4 GiB
    const size_t tile_pad = (size_t)(dtype == EIGSOL_C128 ? Tile<cplx>::kNnz : Tile<double>::kNnz) + 8;
    if ((size_t)(std::max(nrows, ncols) + 64) * sb >= (size_t(1) << 32))
        return fail(EIGSOL_E_UNSUPPORTED, "eigsol_csr_create: the vectors exceed 4 GiB on one device; shard the rows over more ranks");
    if (!sliced && (size_t)(nnz + tile_pad) * sb >= (size_t(1) << 32))
        return fail(EIGSOL_E_UNSUPPORTED, "eigsol_csr_create: a per-device stream exceeds 4 GiB outside the sliced layout; shard the rows over more ranks");
    auto* A = new eigsol_csr();
    A->ctx = ctx;
    ctx_retain(ctx);
    A->dtype = dtype;
    A->nrows = nrows;
    A->ncols = ncols;
    A->nnz = nnz;
    A->ntiles = ntiles;
    A->nshort = nshort;
    A->xoff = xoff;
    A->windowed = windowed;
    A->max_tile_rows = max_rows;
    A->sliced = sliced ? 1 : 0;
    A->nslices = sliced ? (int32_t)(SL.meta.size() / 4) : 0;
    // register capacity KB of a row: 4 / 8 / 12 / 16.  Measured and rejected (round 5,
    // tools/kb10_ab.sh): KB = 10 for the headline's 10-entry rows (five 16-byte value loads per
    // lane instead of six, the sixth a clamped repeat): 192.0 -> 263.9 us per launch
    A->slice_kb = SL.maxk <= 4 ? 4 : SL.maxk <= 8 ? 8 : SL.maxk <= 12 ? 12 : 16;
    A->slice_gather = SL.any_gather ? 1 : 0;
    A->nseg = SL.nseg;
    for (int g = 0; g < kMaxSliceSeg; ++g) {
        A->seg_val[g] = SL.seg_val[g];
        A->seg_c8[g] = SL.seg_c8[g];
        A->seg_c32[g] = SL.seg_c32[g];
    }
    if (const char* env = std::getenv("EIGSOL_SLICE_FORCE_GATHER")) if (std::atoi(env)) A->slice_gather = 1;   // A/B
    const size_t pad = (size_t)(dtype == EIGSOL_C128 ? Tile<cplx>::kNnz : Tile<double>::kNnz) + 8;   // branch-free tile loads
    auto cleanup = [&]() { csr_release(A); };
    hipError_t e;
    if ((e = hipMalloc(&A->rowptr, (nrows + 1) * sizeof(int32_t))) != hipSuccess ||
        (e = hipMalloc(&A->col, (nnz + pad) * sizeof(int32_t))) != hipSuccess ||
        (e = hipMalloc(&A->val, (nnz + pad) * sb)) != hipSuccess ||
        (e = hipMalloc(&A->tile_meta, meta.size() * sizeof(int32_t))) != hipSuccess ||
        (e = hipMalloc(&A->tile_win, win.size() * sizeof(int32_t))) != hipSuccess) {
        cleanup();
        return fail(EIGSOL_E_HIP, std::string("eigsol_csr_create: hipMalloc: ") + hipGetErrorString(e));
    }
    hipStream_t s = ctx->stream;
    if ((e = hipMemsetAsync(A->col, 0, (nnz + pad) * sizeof(int32_t), s)) != hipSuccess ||
        (e = hipMemsetAsync(A->val, 0, (nnz + pad) * sb, s)) != hipSuccess ||
        (e = hipMemcpyAsync(A->rowptr, rowptr, (nrows + 1) * sizeof(int32_t), hipMemcpyHostToDevice, s)) != hipSuccess ||
        (nnz && (e = hipMemcpyAsync(A->col, col_use, nnz * sizeof(int32_t), hipMemcpyHostToDevice, s)) != hipSuccess) ||
        (nnz && (e = hipMemcpyAsync(A->val, val_use, nnz * sb, hipMemcpyHostToDevice, s)) != hipSuccess) ||
        (e = hipMemcpyAsync(A->tile_meta, meta.data(), meta.size() * sizeof(int32_t), hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(A->tile_win, win.data(), win.size() * sizeof(int32_t), hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess) {
        cleanup();
        return fail(EIGSOL_E_HIP, std::string("eigsol_csr_create: upload: ") + hipGetErrorString(e));
    }
    if (windowed && !sliced) {
        // 16-bit window-relative columns of the short tiles (long rows keep using int32 columns)
        std::vector<uint16_t> c16((size_t)(nnz + pad), 0);
        for (int32_t t = 0; t < nshort; ++t) {
            const int32_t w0 = win[2 * t];
            for (int32_t k = meta[4 * t + 2]; k < meta[4 * t + 3]; ++k) c16[k] = (uint16_t)(col_use[k] - w0);
        }
        if ((e = hipMalloc(&A->col16, c16.size() * sizeof(uint16_t))) != hipSuccess ||
            (e = hipMemcpyAsync(A->col16, c16.data(), c16.size() * sizeof(uint16_t), hipMemcpyHostToDevice, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess) {
            cleanup();
            return fail(EIGSOL_E_HIP, std::string("eigsol_csr_create: upload: ") + hipGetErrorString(e));
        }
    }
    if (A->sliced) {
        auto upl = [&](void** dst, const void* src, size_t bytes) -> hipError_t {
            hipError_t r = hipMalloc(dst, std::max<size_t>(bytes, 16));
            if (r == hipSuccess && bytes) r = hipMemcpyAsync(*dst, src, bytes, hipMemcpyHostToDevice, s);
            return r;
        };
        if ((e = upl((void**)&A->slice_meta, SL.meta.data(), SL.meta.size() * 4)) != hipSuccess ||
            (e = upl(&A->sval, SL.val.data(), SL.val.size())) != hipSuccess ||
            (e = upl((void**)&A->scol8, SL.c8.data(), SL.c8.size() * 4)) != hipSuccess ||
            (e = upl((void**)&A->scol32, SL.c32.data(), SL.c32.size() * 4)) != hipSuccess ||
            (!SL.len.empty() && (e = upl((void**)&A->slen, SL.len.data(), SL.len.size())) != hipSuccess) ||
            (e = hipStreamSynchronize(s)) != hipSuccess) {
            cleanup();
            return fail(EIGSOL_E_HIP, std::string("eigsol_csr_create: slice upload: ") + hipGetErrorString(e));
        }
    }
    int rcb = build_bins(A, rowptr, col_use, val_use);
    if (rcb == EIGSOL_OK && !A->binned) rcb = build_col_blocks(A, rowptr, col_use, val_use);
    if (rcb != EIGSOL_OK) {
        cleanup();
        return rcb;
    }
    *out = A;
    return EIGSOL_OK;
}

// Column blocks for gather-bound products (uniform columns): when the matrix gathers x (gather
// slices or plain tiles) and x is larger than kCblkMinBytes, split the columns into blocks of about
// kCblkBytes of x (one XCD's L2 is 4 MB) so that each pass's gathers hit L2.  Rows keep their
// ascending column order across the passes, so every row sum is the reference's, bit for bit.
// EIGSOL_CSR_CBLK=0 disables (=2 skips the entries-per-block rule); EIGSOL_CSR_CBLK_BYTES sets the block size of x in bytes;
// EIGSOL_CSR_CBLK_MIN the x size from which blocks are built.  Measured on config 3's 1M x 16 uniform
// matrix (x 8 MB, tools/cblk_ab.sh): 1 block 166 us, 2 blocks (4 MB) 140 us, 3 blocks 181 us,
// 4 blocks 233 us, 8 blocks 430 us -- each pass re-reads and re-writes y and walks every row, so
// only a split into blocks of a whole L2 pays, and only for rows with >= 8 entries per block.
static int build_col_blocks(eigsol_csr* A, const int32_t* rowptr, const int32_t* col, const void* val) {
    if (g_upload_plain || A->xoff != 0 || A->dist) return EIGSOL_OK;
    if (A->dtype != EIGSOL_F64 && A->dtype != EIGSOL_C128) return EIGSOL_OK;
    int mode = 1;   // EIGSOL_CSR_CBLK: 0 off, 1 by the rules below, 2 regardless of row lengths (tests)
    if (const char* e = std::getenv("EIGSOL_CSR_CBLK")) mode = std::atoi(e);
    if (!mode) return EIGSOL_OK;
    const bool gathers = A->sliced ? A->slice_gather != 0 : !A->windowed;
    if (!gathers || A->nrows != A->ncols || A->nnz == 0) return EIGSOL_OK;
    const size_t sb = scalar_bytes(A->dtype);
    double blk_bytes = 4.0 * 1024 * 1024, min_bytes = 6.0 * 1024 * 1024;
    if (const char* e = std::getenv("EIGSOL_CSR_CBLK_BYTES")) blk_bytes = std::max(1024.0, std::atof(e));
    if (const char* e = std::getenv("EIGSOL_CSR_CBLK_MIN")) min_bytes = std::atof(e);
    const double xbytes = (double)A->ncols * (double)sb;
    if (xbytes < min_bytes) return EIGSOL_OK;
    const int B = (int)std::ceil(xbytes / blk_bytes);
    // every pass visits every row: blocks pay only while rows keep >= 2 entries per block on average
    const double avg = (double)A->nnz / (double)A->nrows;
    if (B < 2 || B > 64 || (mode != 2 && avg < 8.0 * B)) return EIGSOL_OK;
    const int64_t n = A->nrows, nc = A->ncols;
    auto blk_of = [&](int32_t c) { return (int)(((int64_t)c * B) / nc); };
    // one pass over the entries, in row order: each block's rows stay ascending
    std::vector<std::vector<int32_t>> rp(B, std::vector<int32_t>(n + 1, 0)), ci(B);
    std::vector<std::vector<unsigned char>> vv(B);
    for (int b = 0; b < B; ++b) {
        ci[b].reserve((size_t)(A->nnz / B + 16));
        vv[b].reserve((size_t)(A->nnz / B + 16) * sb);
    }
    const int tile_cap = A->dtype == EIGSOL_C128 ? Tile<cplx>::kCap : Tile<double>::kCap;
    for (int64_t i = 0; i < n; ++i) {
        for (int32_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
            const int b = blk_of(col[k]);
            ci[b].push_back(col[k]);
            const unsigned char* src = (const unsigned char*)val + (size_t)k * sb;
            vv[b].insert(vv[b].end(), src, src + sb);
        }
        for (int b = 0; b < B; ++b) {
            rp[b][i + 1] = (int32_t)ci[b].size();
            if (rp[b][i + 1] - rp[b][i] > tile_cap / 2) return EIGSOL_OK;   // a long row: keep one pass
        }
    }
    for (int b = 0; b < B; ++b) {
        if (ci[b].empty()) { ci[b].push_back(0); vv[b].resize(sb, 0); }
        eigsol_csr* Bm = nullptr;
        ++g_upload_plain;
        const int rc = csr_upload(A->ctx, A->dtype, n, nc, rp[b][n], rp[b].data(), ci[b].data(), vv[b].data(), &Bm, 0);
        --g_upload_plain;
        if (rc != EIGSOL_OK) {
            for (eigsol_csr* q : A->cblk) csr_release(q);
            A->cblk.clear();
            return rc;
        }
        A->cblk.push_back(Bm);
        std::vector<int32_t>().swap(rp[b]);
        std::vector<int32_t>().swap(ci[b]);
        std::vector<unsigned char>().swap(vv[b]);
    }
    return EIGSOL_OK;
}

// Column-binned layout (csr_bin_kernel) for gather-bound matrices: built for matrices (square,
// rectangular or row shards) that gather x (gather slices or plain tiles) when x exceeds
// EIGSOL_CSR_BIN_MIN bytes (default 4 MB: one XCD's L2).  EIGSOL_CSR_BIN=0 disables, =2 builds regardless of x's size (tests);
// EIGSOL_CSR_BIN_BYTES (default 1 MB) is the x block a chunk's steps gather from.
static int build_bins(eigsol_csr* A, const int32_t* rowptr, const int32_t* col, const void* val) {
    if (g_upload_plain) return EIGSOL_OK;
    int mode = 1;
    if (const char* e = std::getenv("EIGSOL_CSR_BIN")) mode = std::atoi(e);
    if (!mode) return EIGSOL_OK;
    // gathering products of any shape: square matrices, row shards (x-space columns, rows at xoff)
    const bool gathers = A->sliced ? A->slice_gather != 0 : !A->windowed;
    if (!gathers || A->nnz == 0) return EIGSOL_OK;
    const size_t sb = scalar_bytes(A->dtype);
    // complex<double>: the 16-byte gathers already fetch 4 entries per 64-byte line and its
    // kernel runs at 3 waves per SIMD; config 5's triangular product measured 0.198 ms sliced
    // against 0.356 ms binned, so it keeps the slices
    if (sb > 8 && mode != 2) return EIGSOL_OK;
    double blk_bytes = 1024.0 * 1024, min_bytes = 4.0 * 1024 * 1024;
    if (const char* e = std::getenv("EIGSOL_CSR_BIN_BYTES")) blk_bytes = std::max(1024.0, std::atof(e));
    if (const char* e = std::getenv("EIGSOL_CSR_BIN_MIN")) min_bytes = std::atof(e);
    if (mode != 2 && (double)A->ncols * (double)sb < min_bytes) return EIGSOL_OK;
    // KB of row sums per workgroup: 153 (one workgroup per CU) where the rows' sums exceed 64 MB,
    // else 16 (EIGSOL_CSR_BIN_LDS = 16 | 64 | 128 | 153); threads per workgroup 1024 or 256
    // (EIGSOL_CSR_BIN_NT).  Round 4 A/B (tools/bin_balance_ab.py, balanced chunks): 10M x 10 uniform
    // 16 / 64 / 128 / 153 KB 1.733 / 0.859 / 0.761 / 0.751 ms (fewer chunk rounds: fewer sweeps of x);
    // 1M x 16 0.123 / 0.123 / 0.125 / 0.125 ms
    int lds_kb = (double)A->nrows * (double)sb >= 1024.0 * 65536.0 ? kBinKBMax : 16;
    if (const char* e = std::getenv("EIGSOL_CSR_BIN_LDS")) {
        const int v = std::atoi(e);
        lds_kb = v == kBinKBMax ? kBinKBMax : v == 128 ? 128 : v == 64 ? 64 : 16;
    }
    int nt = sb >= 16 ? 256 : 1024;   // complex<double>: the 1024-thread instantiation spills
    if (const char* e = std::getenv("EIGSOL_CSR_BIN_NT")) {
        const int v = std::atoi(e);
        nt = v == 256 ? 256 : v == 512 ? 512 : 1024;
    }
    const int Rmax = lds_kb * 1024 / (int)sb;   // kBinRows<S, lds_kb>
    int R = Rmax;
    // Balanced chunks (EIGSOL_CSR_BIN_BALANCE, default on): the resident workgroups take the chunks
    // round-robin, so R rows per chunk are chosen to make the chunk count an exact multiple of the
    // grid (every workgroup gets the same number of equal chunks) with the fewest rounds that fit
    // the LDS; otherwise a partial last round leaves part of the chip idle while every round still
    // sweeps x (10M uniform at 64 KB: 1221 chunks over 512 workgroups, the third round 38 % full)
    int balance = 1;
    if (const char* e = std::getenv("EIGSOL_CSR_BIN_BALANCE")) balance = std::atoi(e);
    if (balance) {
        const int per_cu = std::max(1, std::min(2, (160 * 1024) / (lds_kb * 1024 + 2048)));
        const int64_t G = (int64_t)per_cu * A->ctx->num_cus;
        const int64_t rounds = std::max<int64_t>(1, (A->nrows + G * Rmax - 1) / (G * Rmax));
        int64_t r = (A->nrows + rounds * G - 1) / (rounds * G);
        r = ((r + 63) / 64) * 64;
        R = (int)std::max<int64_t>(64, std::min<int64_t>(Rmax, r));
    }
    int rbits = 0;
    while ((1 << rbits) < R) ++rbits;
    int cbits = 0;
    while (cbits < 31 && (double)(int64_t(2) << cbits) * (double)sb <= blk_bytes) ++cbits;
    cbits = std::min(cbits, 32 - rbits);
    const int64_t n = A->nrows, nc = A->ncols;
    const int64_t nblk = (nc + (int64_t(1) << cbits) - 1) >> cbits;
    if (nblk > 65535 || (double)A->nnz * (double)sb >= 4294967296.0) return EIGSOL_OK;   // 32-bit byte offsets
    const int64_t nchunks = (n + R - 1) / R;
    std::vector<uint32_t> pk((size_t)A->nnz);
    std::vector<unsigned char> bv((size_t)A->nnz * sb);
    std::vector<int32_t> steps, levtab, chunk((size_t)nchunks + 1, 0);
    struct Run { int32_t blk, row, start, len; };
    std::vector<Run> runs, sorted;
    std::vector<int64_t> bcnt;
    std::vector<int32_t> lcnt;
    const uint32_t cm = (1u << cbits) - 1u;
    int64_t out = 0;
    for (int64_t c = 0; c < nchunks; ++c) {
        const int64_t r0 = c * R, r1 = std::min(n, r0 + R);
        // runs: a row's entries inside one column block (contiguous: the row is ascending)
        runs.clear();
        for (int64_t i = r0; i < r1; ++i)
            for (int32_t k = rowptr[i]; k < rowptr[i + 1];) {
                const int32_t b = col[k] >> cbits;
                int32_t k2 = k + 1;
                while (k2 < rowptr[i + 1] && (col[k2] >> cbits) == b) ++k2;
                runs.push_back({b, (int32_t)(i - r0), k, k2 - k});
                k = k2;
            }
        // by block (stable: row order)
        bcnt.assign((size_t)nblk + 1, 0);
        for (const Run& q : runs) ++bcnt[(size_t)q.blk + 1];
        for (int64_t b = 0; b < nblk; ++b) bcnt[b + 1] += bcnt[b];
        sorted.resize(runs.size());
        {
            std::vector<int64_t> pos(bcnt.begin(), bcnt.end() - 1);
            for (const Run& q : runs) sorted[(size_t)pos[(size_t)q.blk]++] = q;
        }
        for (int64_t b = 0; b < nblk; ++b) {
            const int64_t q0 = bcnt[b], q1 = bcnt[b + 1];
            if (q0 == q1) continue;
            // longest runs first (stable: row order among equal lengths)
            int32_t maxlen = 0;
            for (int64_t q = q0; q < q1; ++q) maxlen = std::max(maxlen, sorted[q].len);
            if (maxlen > 1) {
                if (maxlen <= 256) {
                    lcnt.assign((size_t)maxlen + 2, 0);
                    for (int64_t q = q0; q < q1; ++q) ++lcnt[(size_t)(maxlen - sorted[q].len) + 1];
                    for (int32_t l = 0; l <= maxlen; ++l) lcnt[l + 1] += lcnt[l];
                    runs.assign(sorted.begin() + q0, sorted.begin() + q1);
                    for (const Run& q : runs) sorted[(size_t)(q0 + lcnt[(size_t)(maxlen - q.len)]++)] = q;
                } else {
                    std::stable_sort(sorted.begin() + q0, sorted.begin() + q1,
                                     [](const Run& x, const Run& y) { return x.len > y.len; });
                }
            }
            // levels: level l holds the l-th entry of the c_l runs longer than l
            const int32_t lbase = (int32_t)(levtab.size() / 2);
            int64_t cl = q1 - q0;   // runs longer than l (prefix of the sorted runs)
            for (int32_t l = 0; l < maxlen; ++l) {
                while (cl > 0 && sorted[q0 + cl - 1].len <= l) --cl;
                levtab.push_back((int32_t)out);
                levtab.push_back((int32_t)cl);
                for (int64_t i = 0; i < cl; ++i) {
                    const Run& q = sorted[q0 + i];
                    const int64_t k = q.start + l;
                    pk[out] = ((uint32_t)q.row << cbits) | ((uint32_t)col[k] & cm);
                    std::memcpy(&bv[(size_t)out * sb], (const unsigned char*)val + (size_t)k * sb, sb);
                    ++out;
                }
            }
            // steps: runs [r, r + nt) x levels [l0, l0 + kBinLev); one barrier after the block
            const size_t sfirst = steps.size();
            for (int64_t r = 0; r < q1 - q0; r += nt) {
                int32_t lr = 0;   // levels holding runs >= r
                while (lr < maxlen && levtab[2 * (lbase + lr) + 1] > r) ++lr;
                for (int32_t l0 = 0; l0 < lr; l0 += kBinLev) {
                    steps.push_back(lbase + l0);
                    steps.push_back(std::min(kBinLev, lr - l0));
                    steps.push_back((int32_t)r);
                    steps.push_back((int32_t)b);
                }
            }
            if (steps.size() > sfirst) steps[steps.size() - 3] |= 0x100;
        }
        chunk[(size_t)c + 1] = (int32_t)(steps.size() / 4);
    }
    A->nchunks = (int32_t)nchunks;
    A->bcbits = cbits;
    A->nbsteps = (int32_t)(steps.size() / 4);
    hipStream_t s = A->ctx->stream;
    auto upl = [&](void** dst, const void* src, size_t bytes) -> hipError_t {
        hipError_t r = hipMalloc(dst, std::max<size_t>(bytes, 16));
        if (r == hipSuccess && bytes) r = hipMemcpyAsync(*dst, src, bytes, hipMemcpyHostToDevice, s);
        return r;
    };
    hipError_t e;
    if ((e = upl((void**)&A->bpk, pk.data(), pk.size() * 4)) != hipSuccess ||
        (e = upl(&A->bval, bv.data(), bv.size())) != hipSuccess ||
        (e = upl((void**)&A->bstep, steps.data(), steps.size() * 4)) != hipSuccess ||
        (e = upl((void**)&A->blev, levtab.data(), levtab.size() * 4)) != hipSuccess ||
        (e = upl((void**)&A->bchunk, chunk.data(), chunk.size() * 4)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess)
        return fail(EIGSOL_E_HIP, std::string("eigsol_csr_create: binned upload: ") + hipGetErrorString(e));
    A->binned = lds_kb;
    A->bin_nt = nt;
    A->bin_rows = R;
    return EIGSOL_OK;
}

static int validate_compressed(const char* who, int64_t nouter, int64_t ninner, int64_t nnz,
                               const int32_t* ptr, const int32_t* idx) {
    if (nouter < 0 || ninner < 0 || nnz < 0)
        return fail(EIGSOL_E_INVALID, std::string(who) + ": negative dimension");
    if (nnz > INT32_MAX - 16)
        return fail(EIGSOL_E_INVALID, std::string(who) + ": nnz exceeds int32 storage index");
    if (!ptr || (nnz && !idx)) return fail(EIGSOL_E_INVALID, std::string(who) + ": null array");
    if (ptr[0] != 0 || ptr[nouter] != nnz)
        return fail(EIGSOL_E_INVALID, std::string(who) + ": pointer array must start at 0 and end at nnz");
    for (int64_t i = 0; i < nouter; ++i)
        if (ptr[i + 1] < ptr[i])
            return fail(EIGSOL_E_INVALID, std::string(who) + ": pointer array not monotone");
    for (int64_t k = 0; k < nnz; ++k)
        if (idx[k] < 0 || idx[k] >= ninner)
            return fail(EIGSOL_E_INVALID, std::string(who) + ": index out of range");
    return EIGSOL_OK;
}

// ---------------------------------------------------------------- occupancy-derived grid
// Residency from the kernel's own resources (MI355X_MICROARCH.md § Register files: waves per SIMD
// = floor(512 / VGPR allocation), 4 waves per block, 160 KiB LDS per CU).
static int resident_grid(eigsol_ctx* ctx, const void* kernel, int64_t ntiles, int* grid, int cap = 8,
                         int waves = kWaves) {
    hipFuncAttributes fa;
    EIGSOL_HIP(hipFuncGetAttributes(&fa, kernel));
    const int vgpr_alloc = std::max(8, ((fa.numRegs + 7) / 8) * 8);
    const int by_vgpr = std::max(1, std::min(8, 512 / vgpr_alloc) * 4 / waves);
    const int by_lds = fa.sharedSizeBytes ? (int)(160 * 1024 / fa.sharedSizeBytes) : 8;
    int per_cu = std::max(1, std::min({by_vgpr, by_lds, cap}));
    if (const char* env = std::getenv("EIGSOL_CSR_BLOCKS_PER_CU")) per_cu = std::max(1, std::atoi(env));
    int64_t g = (int64_t)per_cu * ctx->num_cus;
    const int64_t need = ((ntiles + 7) / 8) * 8;
    g = std::min(g, std::max<int64_t>(need, 8));
    g = std::max<int64_t>(8, (g / 8) * 8);
    *grid = (int)g;
    return EIGSOL_OK;
}

// the device-side peer exchange (row-sharded sessions): every scalar type has the peer kernels
template <class S> inline constexpr bool kPeerOk = true;

template <class S, bool kPower, int kKB>
static const void* bin_kernel_ptr_kb(int nt) {
    return nt == 1024  ? reinterpret_cast<const void*>(csr_bin_kernel<S, kPower, kKB, 1024>)
           : nt == 512 ? reinterpret_cast<const void*>(csr_bin_kernel<S, kPower, kKB, 512>)
                       : reinterpret_cast<const void*>(csr_bin_kernel<S, kPower, kKB, 256>);
}
template <class S, bool kPower>
static const void* bin_kernel_ptr(const eigsol_csr* A) {
    return A->binned == kBinKBMax ? bin_kernel_ptr_kb<S, kPower, kBinKBMax>(A->bin_nt)
           : A->binned == 128     ? bin_kernel_ptr_kb<S, kPower, 128>(A->bin_nt)
           : A->binned == 64      ? bin_kernel_ptr_kb<S, kPower, 64>(A->bin_nt)
                                  : bin_kernel_ptr_kb<S, kPower, 16>(A->bin_nt);
}

template <class S>
static const void* power_kernel_ptr(const eigsol_csr* A, bool peer = false) {
    if (A->binned && !peer)
        return bin_kernel_ptr<S, true>(A);
    if constexpr (std::is_same_v<S, double> || std::is_same_v<S, cplx>)
        if (!A->cblk.empty() && !peer) return reinterpret_cast<const void*>(csr_kernel<S, true>);
    if (A->sliced) {
#define EIGSOL_SLICE_PTR(KB)                                                                                 \
    if (peer)                                                                                                \
        return A->slice_gather ? reinterpret_cast<const void*>(csr_slice_kernel<S, true, KB, true, kPeerOk<S>>)   \
                               : reinterpret_cast<const void*>(csr_slice_kernel<S, true, KB, false, kPeerOk<S>>); \
    return A->slice_gather ? reinterpret_cast<const void*>(csr_slice_kernel<S, true, KB, true>)             \
                           : reinterpret_cast<const void*>(csr_slice_kernel<S, true, KB, false>);
        switch (A->slice_kb) {
            case 4: EIGSOL_SLICE_PTR(4)
            case 8: EIGSOL_SLICE_PTR(8)
            case 12: EIGSOL_SLICE_PTR(12)
            default: EIGSOL_SLICE_PTR(16)
        }
#undef EIGSOL_SLICE_PTR
    }
    if constexpr (std::is_same_v<S, float> || std::is_same_v<S, cplxf>)
        return reinterpret_cast<const void*>(csr_row_kernel<S, true>);
    else
        return A->windowed ? reinterpret_cast<const void*>(csr_win_kernel<S, true>)
                           : reinterpret_cast<const void*>(csr_kernel<S, true>);
}

const void* csr_power_kernel(const eigsol_csr* A, bool peer) {
    return A->dtype == EIGSOL_C128  ? power_kernel_ptr<cplx>(A, peer)
           : A->dtype == EIGSOL_F32 ? power_kernel_ptr<float>(A, peer)
           : A->dtype == EIGSOL_C64 ? power_kernel_ptr<cplxf>(A, peer)
                                    : power_kernel_ptr<double>(A, peer);
}

int csr_grid(eigsol_csr* A, int* grid, bool peer) {
    const void* k = A->dtype == EIGSOL_C128  ? power_kernel_ptr<cplx>(A, peer)
                    : A->dtype == EIGSOL_F32 ? power_kernel_ptr<float>(A, peer)
                    : A->dtype == EIGSOL_C64 ? power_kernel_ptr<cplxf>(A, peer)
                                             : power_kernel_ptr<double>(A, peer);
    // work units: tiles (one per block step) or slices (one per wave step)
    int64_t units = A->sliced ? (A->nslices + kWaves - 1) / kWaves : A->ntiles;
    if (A->binned && !peer) return resident_grid(A->ctx, k, A->nchunks, grid, 8, A->bin_nt / 64);
    if (!A->cblk.empty() && !peer) {   // column blocks: csr_kernel passes over the blocks' tiles
        units = 0;
        for (const eigsol_csr* B : A->cblk) units = std::max<int64_t>(units, B->ntiles);
        return resident_grid(A->ctx, k, units, grid, 8);
    }
    // sliced: two blocks (8 waves, 16 slices in flight) per CU measured fastest on band10m f64
    // (round 4, tools/slice_grid_ab.py: 2 / 3 / 4 / 6 blocks 188.8 / 201.9 / 226.6 / 225.1 us); more
    // concurrent streams per CU cost more than the latency they hide.  float (four slices per round,
    // no pipeline) peaks at three: 128.8 / 125.8 / 128.8 / 156.2 us
    if (dtype_single(A->dtype) && !A->sliced)   // row-per-lane fallback: rows / threads
        return resident_grid(A->ctx, k, (A->nrows + kThreads - 1) / kThreads, grid, 8);
    return resident_grid(A->ctx, k, units, grid, A->sliced ? (A->dtype == EIGSOL_F32 ? 3 : 2) : 8);
}

template <class S>
static CsrArgs<S> make_args(const eigsol_csr* A, int64_t xlen) {
    CsrArgs<S> a{};
    a.rowptr = A->rowptr;
    a.col = A->col;
    a.col16 = A->col16;
    a.val = (const S*)A->val;
    a.tile_meta = (const int4*)A->tile_meta;
    a.tile_win = (const int2*)A->tile_win;
    a.slice_meta = (const int4*)A->slice_meta;
    a.sval = (const S*)A->sval;
    a.scol8 = A->scol8;
    a.scol32 = A->scol32;
    a.slen = A->slen;
    a.nslices = A->nslices;
    a.nseg = A->nseg;
    for (int g = 0; g < kMaxSliceSeg; ++g) {
        a.seg_val[g] = A->seg_val[g];
        a.seg_c8[g] = A->seg_c8[g];
        a.seg_c32[g] = A->seg_c32[g];
    }
    a.ntiles = A->ntiles;
    a.nshort = A->nshort;
    a.xlen = (int32_t)xlen;
    a.nrows = (int32_t)A->nrows;
    a.xoff = (int32_t)A->xoff;
    a.cb_carry = 0;
    a.cb_epi = 1;
    a.bpk = A->bpk;
    a.bval = (const S*)A->bval;
    a.bstep = (const int4*)A->bstep;
    a.blev = (const int2*)A->blev;
    a.bchunk = A->bchunk;
    a.nchunks = A->nchunks;
    a.brows = A->bin_rows;
    a.bcbits = A->bcbits;
    a.cbeg = 0;
    a.cend = A->nchunks;
    a.cont = 0;
    return a;
}

template <class S>
static int launch_csr(eigsol_csr* A, const CsrArgs<S>& args, bool power, int parity, int grid, bool peer = false) {
    hipStream_t s = A->ctx->stream;
    if (A->binned && !peer) {
        const void* k = power ? bin_kernel_ptr<S, true>(A) : bin_kernel_ptr<S, false>(A);
        CsrArgs<S> av = args;
        int pv = parity;
        void* argv[] = {&av, &pv};
        EIGSOL_HIP(hipLaunchKernel(k, dim3(grid), dim3(A->bin_nt), argv, 0, s));
        EIGSOL_HIP(hipGetLastError());
        return EIGSOL_OK;
    }
    if constexpr (std::is_same_v<S, double> || std::is_same_v<S, cplx>) {
        if (!A->cblk.empty() && !peer) {
            // column blocks: one csr_kernel pass per block, partials carried in y (stream order)
            const int B = (int)A->cblk.size();
            for (int b = 0; b < B; ++b) {
                CsrArgs<S> ab = make_args<S>(A->cblk[b], args.xlen);
                ab.x_plain = args.x_plain;
                ab.y_plain = args.y_plain;
                ab.buf0 = args.buf0;
                ab.buf1 = args.buf1;
                ab.ctl = args.ctl;
                ab.rank_part = args.rank_part;
                ab.nranks = args.nranks;
                ab.my_part = args.my_part;
                ab.blk_part = args.blk_part;
                ab.trace = args.trace;
                ab.cb_carry = b > 0;
                ab.cb_epi = b == B - 1;
                if (power) hipLaunchKernelGGL((csr_kernel<S, true>), dim3(grid), dim3(kThreads), 0, s, ab, parity);
                else hipLaunchKernelGGL((csr_kernel<S, false>), dim3(grid), dim3(kThreads), 0, s, ab, parity);
            }
            EIGSOL_HIP(hipGetLastError());
            return EIGSOL_OK;
        }
    }
    static const int mode = [] {
        const char* e = std::getenv("EIGSOL_CSR_ABLATION");
        return e ? std::atoi(e) : 0;
    }();
    if constexpr (std::is_same_v<S, double>) {
        if (power && mode > 0 && !A->windowed && !A->sliced) {
            if (mode == 1) hipLaunchKernelGGL((csr_kernel<S, true, 1>), dim3(grid), dim3(kThreads), 0, s, args, parity);
            else if (mode == 2) hipLaunchKernelGGL((csr_kernel<S, true, 2>), dim3(grid), dim3(kThreads), 0, s, args, parity);
            else hipLaunchKernelGGL((csr_kernel<S, true, 3>), dim3(grid), dim3(kThreads), 0, s, args, parity);
            EIGSOL_HIP(hipGetLastError());
            return EIGSOL_OK;
        }
    }
    if (A->sliced) {
#define EIGSOL_SLICE_LAUNCH2(KB, G)                                                                                     \
    if (power && peer)                                                                                                  \
        hipLaunchKernelGGL((csr_slice_kernel<S, true, KB, G, kPeerOk<S>>), dim3(grid), dim3(kThreads), 0, s, args, parity); \
    else if (power) hipLaunchKernelGGL((csr_slice_kernel<S, true, KB, G>), dim3(grid), dim3(kThreads), 0, s, args, parity); \
    else hipLaunchKernelGGL((csr_slice_kernel<S, false, KB, G>), dim3(grid), dim3(kThreads), 0, s, args, parity);
#define EIGSOL_SLICE_LAUNCH(KB)                                  \
    if (A->slice_gather) { EIGSOL_SLICE_LAUNCH2(KB, true) }      \
    else { EIGSOL_SLICE_LAUNCH2(KB, false) }
        switch (A->slice_kb) {
            case 4: EIGSOL_SLICE_LAUNCH(4) break;
            case 8: EIGSOL_SLICE_LAUNCH(8) break;
            case 12: EIGSOL_SLICE_LAUNCH(12) break;
            default: EIGSOL_SLICE_LAUNCH(16) break;
        }
#undef EIGSOL_SLICE_LAUNCH
#undef EIGSOL_SLICE_LAUNCH2
    } else if constexpr (std::is_same_v<S, float> || std::is_same_v<S, cplxf>) {
        if (power) hipLaunchKernelGGL((csr_row_kernel<S, true>), dim3(grid), dim3(kThreads), 0, s, args, parity);
        else hipLaunchKernelGGL((csr_row_kernel<S, false>), dim3(grid), dim3(kThreads), 0, s, args, parity);
    } else if (A->windowed) {
        if (power) hipLaunchKernelGGL((csr_win_kernel<S, true>), dim3(grid), dim3(kThreads), 0, s, args, parity);
        else hipLaunchKernelGGL((csr_win_kernel<S, false>), dim3(grid), dim3(kThreads), 0, s, args, parity);
    } else {
        if (power) hipLaunchKernelGGL((csr_kernel<S, true>), dim3(grid), dim3(kThreads), 0, s, args, parity);
        else hipLaunchKernelGGL((csr_kernel<S, false>), dim3(grid), dim3(kThreads), 0, s, args, parity);
    }
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

// First chunk of the second row part of an iteration split in two (binned layout).
static int32_t bin_split_chunk(const eigsol_csr* A) { return (A->nchunks + 1) / 2; }

template <class S>
static int power_launch_t(eigsol_csr* A, int64_t xlen, void* buf0, void* buf1, PowerCtl* ctl,
                          const void* rank_part, int nranks, void* my_part, void* blk_part,
                          void* trace, int parity, int grid, const PeerArgs* peer, int part) {
    CsrArgs<S> a = make_args<S>(A, xlen);
    if (part >= 0) {   // one of the two row parts of a split iteration (binned layout only)
        a.cbeg = part == 0 ? 0 : bin_split_chunk(A);
        a.cend = part == 0 ? bin_split_chunk(A) : A->nchunks;
        a.cont = part;
    }
    a.buf0 = (S*)buf0;
    a.buf1 = (S*)buf1;
    a.ctl = ctl;
    a.rank_part = (const part4*)rank_part;
    a.nranks = nranks;
    a.my_part = (part4*)my_part;
    a.blk_part = (part4*)blk_part;
    a.trace = (S*)trace;
    if (peer) a.peer = *peer;
    return launch_csr<S>(A, a, true, parity, grid, peer != nullptr);
}

// entry point used by power_session.cpp (xlen: entries of the y buffers, own + ghost)
int csr_power_launch(eigsol_csr* A, int64_t xlen, void* buf0, void* buf1, PowerCtl* ctl,
                     const void* rank_part, int nranks, void* my_part, void* blk_part, void* trace,
                     int parity, int grid, const PeerArgs* peer, int part) {
    if (peer && !A->sliced) return fail(EIGSOL_E_UNSUPPORTED, "peer exchange needs the sliced CSR layout");
    if (part >= 0 && (peer || !A->binned)) return fail(EIGSOL_E_INVALID, "split iteration needs the binned layout");
    if (A->dtype == EIGSOL_C128)
        return power_launch_t<cplx>(A, xlen, buf0, buf1, ctl, rank_part, nranks, my_part, blk_part,
                                    trace, parity, grid, peer, part);
    if (A->dtype == EIGSOL_F32)
        return power_launch_t<float>(A, xlen, buf0, buf1, ctl, rank_part, nranks, my_part, blk_part,
                                     trace, parity, grid, peer, part);
    if (A->dtype == EIGSOL_C64)
        return power_launch_t<cplxf>(A, xlen, buf0, buf1, ctl, rank_part, nranks, my_part, blk_part,
                                     trace, parity, grid, peer, part);
    return power_launch_t<double>(A, xlen, buf0, buf1, ctl, rank_part, nranks, my_part, blk_part,
                                  trace, parity, grid, peer, part);
}

// Own rows in the first part of a split iteration (binned layout): whole chunks of the first half.
int64_t csr_bin_split_row(const eigsol_csr* A) {
    if (!A->binned) return A->nrows;
    const int64_t rows = A->bin_rows;   // rows per chunk
    return std::min<int64_t>(A->nrows, (int64_t)bin_split_chunk(A) * rows);
}

int peer_begin_launch(eigsol_ctx* ctx, int dtype, const PeerArgs& pa, const void* x_own, int64_t npush,
                      const void* mine) {
    hipStream_t s = ctx->stream;
    if (dtype == EIGSOL_C128)
        hipLaunchKernelGGL(peer_begin_kernel<cplx>, dim3(1), dim3(kThreads), 0, s, pa, (const cplx*)x_own, npush,
                           (const part4*)mine);
    else if (dtype == EIGSOL_F32)
        hipLaunchKernelGGL(peer_begin_kernel<float>, dim3(1), dim3(kThreads), 0, s, pa, (const float*)x_own, npush,
                           (const part4*)mine);
    else if (dtype == EIGSOL_C64)
        hipLaunchKernelGGL(peer_begin_kernel<cplxf>, dim3(1), dim3(kThreads), 0, s, pa, (const cplxf*)x_own, npush,
                           (const part4*)mine);
    else
        hipLaunchKernelGGL(peer_begin_kernel<double>, dim3(1), dim3(kThreads), 0, s, pa, (const double*)x_own,
                           npush, (const part4*)mine);
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

int norm_partial_launch(eigsol_ctx* ctx, int dtype, const void* x, int64_t n, PowerCtl* ctl,
                        void* blk_part, void* out, int grid) {
    hipStream_t s = ctx->stream;
    if (dtype == EIGSOL_C128)
        hipLaunchKernelGGL(norm_partial_kernel<cplx>, dim3(grid), dim3(kThreads), 0, s,
                           (const cplx*)x, n, ctl, (part4*)blk_part, (part4*)out);
    else if (dtype == EIGSOL_F32)
        hipLaunchKernelGGL(norm_partial_kernel<float>, dim3(grid), dim3(kThreads), 0, s,
                           (const float*)x, n, ctl, (part4*)blk_part, (part4*)out);
    else if (dtype == EIGSOL_C64)
        hipLaunchKernelGGL(norm_partial_kernel<cplxf>, dim3(grid), dim3(kThreads), 0, s,
                           (const cplxf*)x, n, ctl, (part4*)blk_part, (part4*)out);
    else
        hipLaunchKernelGGL(norm_partial_kernel<double>, dim3(grid), dim3(kThreads), 0, s,
                           (const double*)x, n, ctl, (part4*)blk_part, (part4*)out);
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

int scale_out_launch(eigsol_ctx* ctx, int dtype, const void* src, double nrm, void* dst, int64_t n) {
    hipStream_t s = ctx->stream;
    const int grid = (int)std::min<int64_t>(4096, std::max<int64_t>(1, (n + kThreads - 1) / kThreads));
    if (dtype == EIGSOL_C128)
        hipLaunchKernelGGL(scale_out_kernel<cplx>, dim3(grid), dim3(kThreads), 0, s, (const cplx*)src,
                           nrm, (cplx*)dst, n);
    else if (dtype == EIGSOL_F32)
        hipLaunchKernelGGL(scale_out_kernel<float>, dim3(grid), dim3(kThreads), 0, s, (const float*)src,
                           nrm, (float*)dst, n);
    else if (dtype == EIGSOL_C64)
        hipLaunchKernelGGL(scale_out_kernel<cplxf>, dim3(grid), dim3(kThreads), 0, s, (const cplxf*)src,
                           nrm, (cplxf*)dst, n);
    else
        hipLaunchKernelGGL(scale_out_kernel<double>, dim3(grid), dim3(kThreads), 0, s,
                           (const double*)src, nrm, (double*)dst, n);
    EIGSOL_HIP(hipGetLastError());
    return EIGSOL_OK;
}

int wide_csr_upload(eigsol_ctx* ctx, int dtype, int64_t nrows, int64_t ncols, int64_t nnz, const int32_t* rowptr,
                    const int32_t* colidx, const void* values, eigsol_csr** out);   // wide.hip
int wide_csr_spmv(eigsol_csr* A, const void* x, void* y);

// the row-ordered CSR of any dtype: the fp64 / fp32 layouts, or the double-double plain CSR
static int upload_any(eigsol_ctx* ctx, int dtype, int64_t nrows, int64_t ncols, int64_t nnz, const int32_t* rowptr,
                      const int32_t* colidx, const void* values, eigsol_csr** out) {
    if (dtype_wide(dtype)) return wide_csr_upload(ctx, dtype, nrows, ncols, nnz, rowptr, colidx, values, out);
    return csr_upload(ctx, dtype, nrows, ncols, nnz, rowptr, colidx, values, out, 0);
}

}  // namespace eigsol

// ---------------------------------------------------------------- C ABI
extern "C" {

int eigsol_csr_create(eigsol_ctx* ctx, eigsol_dtype dtype, int64_t nrows, int64_t ncols,
                      int64_t nnz, const int32_t* rowptr, const int32_t* colidx,
                      const void* values, eigsol_csr** out) {
    if (!ctx || !out) return fail(EIGSOL_E_INVALID, "eigsol_csr_create: null ctx/out");
    *out = nullptr;
    if (!dtype_valid(dtype) && !dtype_wide(dtype)) return fail(EIGSOL_E_INVALID, "eigsol_csr_create: unknown dtype");
    if (nrows > INT32_MAX - 1 || ncols > INT32_MAX - 1)
        return fail(EIGSOL_E_INVALID, "eigsol_csr_create: dimension exceeds int32 storage index");
    EIGSOL_TRY(validate_compressed("eigsol_csr_create", nrows, ncols, nnz, rowptr, colidx));
    if (nnz && !values) return fail(EIGSOL_E_INVALID, "eigsol_csr_create: null values");
    EIGSOL_HIP(hipSetDevice(ctx->device));
    return upload_any(ctx, dtype, nrows, ncols, nnz, rowptr, colidx, values, out);
}

int eigsol_csr_create_from_csc(eigsol_ctx* ctx, eigsol_dtype dtype, int64_t nrows, int64_t ncols,
                               int64_t nnz, const int32_t* colptr, const int32_t* rowidx,
                               const void* values, eigsol_csr** out) {
    if (!ctx || !out) return fail(EIGSOL_E_INVALID, "eigsol_csr_create_from_csc: null ctx/out");
    *out = nullptr;
    if (!dtype_valid(dtype) && !dtype_wide(dtype)) return fail(EIGSOL_E_INVALID, "eigsol_csr_create_from_csc: unknown dtype");
    if (nrows > INT32_MAX - 1 || ncols > INT32_MAX - 1)
        return fail(EIGSOL_E_INVALID, "eigsol_csr_create_from_csc: dimension exceeds int32");
    EIGSOL_TRY(validate_compressed("eigsol_csr_create_from_csc", ncols, nrows, nnz, colptr, rowidx));
    if (nnz && !values) return fail(EIGSOL_E_INVALID, "eigsol_csr_create_from_csc: null values");
    // CSC -> CSR by counting sort; scanning columns in ascending order leaves every row's
    // columns ascending (the reference's CSC scatter order, power_method.hpp:69).
    const size_t sb = scalar_bytes(dtype);
    std::vector<int32_t> rp(nrows + 1, 0), ci(nnz);
    std::vector<unsigned char> v((size_t)nnz * sb);
    for (int64_t k = 0; k < nnz; ++k) rp[rowidx[k] + 1]++;
    for (int64_t i = 0; i < nrows; ++i) rp[i + 1] += rp[i];
    std::vector<int32_t> fill(rp.begin(), rp.end() - 1);
    for (int64_t j = 0; j < ncols; ++j)
        for (int32_t k = colptr[j]; k < colptr[j + 1]; ++k) {
            const int32_t d = fill[rowidx[k]]++;
            ci[d] = (int32_t)j;
            std::memcpy(&v[(size_t)d * sb], (const unsigned char*)values + (size_t)k * sb, sb);
        }
    EIGSOL_HIP(hipSetDevice(ctx->device));
    return upload_any(ctx, dtype, nrows, ncols, nnz, rp.data(), ci.data(), v.data(), out);
}

int eigsol_csr_create_from_coo(eigsol_ctx* ctx, eigsol_dtype dtype, int64_t nrows, int64_t ncols,
                               int64_t nnz, const int32_t* rowidx, const int32_t* colidx,
                               const void* values, eigsol_csr** out) {
    if (!ctx || !out) return fail(EIGSOL_E_INVALID, "eigsol_csr_create_from_coo: null ctx/out");
    *out = nullptr;
    if (!dtype_valid(dtype) && !dtype_wide(dtype)) return fail(EIGSOL_E_INVALID, "eigsol_csr_create_from_coo: unknown dtype");
    if (nrows < 0 || ncols < 0 || nnz < 0) return fail(EIGSOL_E_INVALID, "eigsol_csr_create_from_coo: negative dimension");
    if (nrows > INT32_MAX - 1 || ncols > INT32_MAX - 1 || nnz > INT32_MAX - 16)
        return fail(EIGSOL_E_INVALID, "eigsol_csr_create_from_coo: dimension exceeds int32 storage index");
    if (nnz && (!rowidx || !colidx || !values)) return fail(EIGSOL_E_INVALID, "eigsol_csr_create_from_coo: null array");
    for (int64_t k = 0; k < nnz; ++k)
        if (rowidx[k] < 0 || rowidx[k] >= nrows || colidx[k] < 0 || colidx[k] >= ncols)
            return fail(EIGSOL_E_INVALID, "eigsol_csr_create_from_coo: index out of range");
    // Two stable counting sorts (by column, then by row) order the triplets by (row, column) and
    // keep equal positions in input order; duplicates are then summed in input order, which is
    // what Matrix::Sparse's compression does with repeated insert()s (SparseMatrix::compress).
    const size_t sb = scalar_bytes(dtype);
    const auto* vin = static_cast<const unsigned char*>(values);
    std::vector<int32_t> by_col(nnz), cptr(ncols + 1, 0), rp(nrows + 1, 0);
    for (int64_t k = 0; k < nnz; ++k) cptr[colidx[k] + 1]++;
    for (int64_t j = 0; j < ncols; ++j) cptr[j + 1] += cptr[j];
    for (int64_t k = 0; k < nnz; ++k) by_col[cptr[colidx[k]]++] = (int32_t)k;
    for (int64_t k = 0; k < nnz; ++k) rp[rowidx[k] + 1]++;
    for (int64_t i = 0; i < nrows; ++i) rp[i + 1] += rp[i];
    std::vector<int32_t> perm(nnz), fill(rp.begin(), rp.end() - 1);
    for (int64_t t = 0; t < nnz; ++t) {
        const int32_t k = by_col[t];
        perm[fill[rowidx[k]]++] = k;
    }
    std::vector<int32_t>().swap(by_col);
    std::vector<int32_t> ci;
    std::vector<unsigned char> v;
    ci.reserve(nnz);
    v.reserve((size_t)nnz * sb);
    std::vector<int32_t> crp(nrows + 1, 0);
    auto accumulate = [&](unsigned char* dst, const unsigned char* src) {
        if (dtype_wide(dtype)) {   // double-double pairs: the sum in double-double
            for (size_t w = 0; w < sb / 16; ++w) {
                dd a, b;
                std::memcpy(&a, dst + 16 * w, 16);
                std::memcpy(&b, src + 16 * w, 16);
                a = dd_add(a, b);
                std::memcpy(dst + 16 * w, &a, 16);
            }
        } else if (dtype == EIGSOL_F64 || dtype == EIGSOL_C128) {
            for (size_t w = 0; w < sb / 8; ++w) {
                double a, b;
                std::memcpy(&a, dst + 8 * w, 8);
                std::memcpy(&b, src + 8 * w, 8);
                a += b;
                std::memcpy(dst + 8 * w, &a, 8);
            }
        } else {
            for (size_t w = 0; w < sb / 4; ++w) {
                float a, b;
                std::memcpy(&a, dst + 4 * w, 4);
                std::memcpy(&b, src + 4 * w, 4);
                a += b;
                std::memcpy(dst + 4 * w, &a, 4);
            }
        }
    };
    for (int64_t i = 0; i < nrows; ++i) {
        for (int32_t t = rp[i]; t < rp[i + 1]; ++t) {
            const int32_t k = perm[t];
            const unsigned char* src = vin + (size_t)k * sb;
            if ((int64_t)ci.size() > crp[i] && ci.back() == colidx[k]) {
                accumulate(v.data() + v.size() - sb, src);
                continue;
            }
            ci.push_back(colidx[k]);
            v.insert(v.end(), src, src + sb);
        }
        crp[i + 1] = (int32_t)ci.size();
    }
    EIGSOL_HIP(hipSetDevice(ctx->device));
    return upload_any(ctx, dtype, nrows, ncols, (int64_t)ci.size(), crp.data(), ci.data(), v.data(), out);
}

int eigsol_csr_download(eigsol_csr* A, int32_t* rowptr, int32_t* colidx, void* values) {
    if (!A) return fail(EIGSOL_E_INVALID, "eigsol_csr_download: null matrix");
    if (A->dist) return fail(EIGSOL_E_UNSUPPORTED, "eigsol_csr_download: row-sharded matrix");
    if (!rowptr || (A->nnz && (!colidx || !values))) return fail(EIGSOL_E_INVALID, "eigsol_csr_download: null array");
    EIGSOL_HIP(hipSetDevice(A->ctx->device));
    hipStream_t s = A->ctx->stream;
    EIGSOL_HIP(hipMemcpyAsync(rowptr, A->rowptr, (A->nrows + 1) * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (A->nnz) {
        EIGSOL_HIP(hipMemcpyAsync(colidx, A->col, A->nnz * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        EIGSOL_HIP(hipMemcpyAsync(values, A->val, A->nnz * scalar_bytes(A->dtype), hipMemcpyDeviceToHost, s));
    }
    EIGSOL_HIP(hipStreamSynchronize(s));
    return EIGSOL_OK;
}

int eigsol_csr_destroy(eigsol_csr* A) {
    csr_release(A);
    return EIGSOL_OK;
}

int eigsol_csr_info(eigsol_csr* A, int64_t* nrows, int64_t* ncols, int64_t* nnz, int* dtype) {
    if (!A) return fail(EIGSOL_E_INVALID, "eigsol_csr_info: null matrix");
    if (nrows) *nrows = A->nrows;
    if (ncols) *ncols = A->ncols;
    if (nnz) *nnz = A->nnz;
    if (dtype) *dtype = A->dtype;
    return EIGSOL_OK;
}

int eigsol_csr_spmv(eigsol_csr* A, const void* x_dev, void* y_dev) {
    if (!A || (!x_dev && A->ncols) || (!y_dev && A->nrows))
        return fail(EIGSOL_E_INVALID, "eigsol_csr_spmv: null pointer");
    if (A->nrows == 0) return EIGSOL_OK;
    EIGSOL_HIP(hipSetDevice(A->ctx->device));
    if (dtype_wide(A->dtype)) return wide_csr_spmv(A, x_dev, y_dev);
    int grid = 8;
    EIGSOL_TRY(csr_grid(A, &grid, false));
    auto run = [&](auto tag) {
        using S = decltype(tag);
        CsrArgs<S> a = make_args<S>(A, A->ncols);
        a.x_plain = (const S*)x_dev;
        a.y_plain = (S*)y_dev;
        return launch_csr<S>(A, a, false, 0, grid);
    };
    switch (A->dtype) {
        case EIGSOL_C128: return run(cplx{});
        case EIGSOL_F32: return run(0.0f);
        case EIGSOL_C64: return run(cplxf{});
        default: return run(0.0);
    }
}

}  // extern "C"

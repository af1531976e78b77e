// Device helpers shared by the gfx950 kernels: scalar arithmetic with the reference's rounding,
// deterministic wave/block reductions and the last-arriver hand-off of block partials.
#pragma once

#include "internal.hpp"

// Products and sums keep the reference's separate roundings (g++, no -march => no FMA).  This
// makes every CSR row sum bitwise equal to the reference's CSC scatter (oracle-checked).
#pragma clang fp contract(off)

namespace eigsol {
namespace dev {

constexpr int kThreads = 256;   // 4 wave64 per block
constexpr int kWaves = kThreads / 64;

struct alignas(32) part4 {
    double a, b, c, d;   // a = sum |y|^2, (b, c) = sum conj(x) y, d unused
};

__device__ __forceinline__ double mul(double a, double b) { return a * b; }
__device__ __forceinline__ cplx mul(cplx a, cplx b) {
    return cplx{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
__device__ __forceinline__ double add(double a, double b) { return a + b; }
__device__ __forceinline__ cplx add(cplx a, cplx b) { return cplx{a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ double sub(double a, double b) { return a - b; }
__device__ __forceinline__ cplx sub(cplx a, cplx b) { return cplx{a.re - b.re, a.im - b.im}; }
// x = y / normY (power_method.hpp:78): elementwise division by a real scalar.
__device__ __forceinline__ double divr(double a, double r) { return a / r; }
__device__ __forceinline__ cplx divr(cplx a, double r) { return cplx{a.re / r, a.im / r}; }
// conj(x) * y accumulated into (rr, ri) (Eigen dot conjugates its first argument).
__device__ __forceinline__ void acc_dot(double& rr, double& /*ri*/, double x, double y) {
    rr += x * y;
}
__device__ __forceinline__ void acc_dot(double& rr, double& ri, cplx x, cplx y) {
    rr += x.re * y.re + x.im * y.im;
    ri += x.re * y.im - x.im * y.re;
}
__device__ __forceinline__ void set_re_im(double& dst, double re, double /*im*/) { dst = re; }
__device__ __forceinline__ void set_re_im(cplx& dst, double re, double im) { dst = cplx{re, im}; }

// single precision (float, std::complex<float>): float products and sums, norm / dot partials in
// double (exact products of floats); x = y / normY divides by the float normY like the reference
__device__ __forceinline__ float mul(float a, float b) { return a * b; }
__device__ __forceinline__ cplxf mul(cplxf a, cplxf b) {
    return cplxf{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
__device__ __forceinline__ float add(float a, float b) { return a + b; }
__device__ __forceinline__ cplxf add(cplxf a, cplxf b) { return cplxf{a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ float sub(float a, float b) { return a - b; }
__device__ __forceinline__ cplxf sub(cplxf a, cplxf b) { return cplxf{a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ float divr(float a, double r) { return a / (float)r; }
__device__ __forceinline__ cplxf divr(cplxf a, double r) {
    const float f = (float)r;
    return cplxf{a.re / f, a.im / f};
}
__device__ __forceinline__ void acc_dot(double& rr, double& /*ri*/, float x, float y) {
    rr += (double)x * (double)y;
}
__device__ __forceinline__ void acc_dot(double& rr, double& ri, cplxf x, cplxf y) {
    const double xr = x.re, xi = x.im, yr = y.re, yi = y.im;
    rr += xr * yr + xi * yi;
    ri += xr * yi - xi * yr;
}
__device__ __forceinline__ void set_re_im(float& dst, double re, double /*im*/) { dst = (float)re; }
__device__ __forceinline__ void set_re_im(cplxf& dst, double re, double im) { dst = cplxf{(float)re, (float)im}; }

// Deterministic xor-butterfly: every lane ends with the same bits.
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Block sum of three doubles in a fixed order; result valid in thread 0.
template <int NT = kThreads>
__device__ __forceinline__ void block_sum3(double& a, double& b, double& c, double* sm /*3*NT/64*/) {
    constexpr int W = NT / 64;
    a = wave_sum(a);
    b = wave_sum(b);
    c = wave_sum(c);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sm[w] = a;
        sm[W + w] = b;
        sm[2 * W + w] = c;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a = sm[0]; b = sm[W]; c = sm[2 * W];
#pragma unroll
        for (int i = 1; i < W; ++i) {
            a += sm[i];
            b += sm[W + i];
            c += sm[2 * W + i];
        }
    }
    __syncthreads();
}

__device__ __forceinline__ void st_agent(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent(const double* p) {
    return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// In-launch reduction of per-block partials (MI355X guide §6 Guideline 16, counter form):
// thread 0 of every block stores its partial write-through (agent-scope sc1 stores), drains
// them, and takes a ticket; the block that draws G-1 reads every partial with sc1 loads and sums
// them in block order (deterministic), then publishes the rank partial with plain stores (its
// consumers run after the kernel boundary).  Must be reached by every block of the grid.
// accum: add to *out instead of overwriting it (the second launch of an iteration split in two
// row parts; the first part's launch wrote *out, so the sum order is fixed: part 0, then part 1).
template <int NT = kThreads>
__device__ __forceinline__ void last_arriver_reduce(double a, double b, double c, part4* blk_part,
                                                    uint32_t* counter, part4* out, double* sm,
                                                    int* s_last, bool accum = false) {
    const uint32_t G = gridDim.x;
    if (threadIdx.x == 0) {
        part4* p = blk_part + blockIdx.x;
        st_agent(&p->a, a);
        st_agent(&p->b, b);
        st_agent(&p->c, c);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t tk = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
        *s_last = (tk == G - 1) ? 1 : 0;
    }
    __syncthreads();
    if (!*s_last) return;
    double sa = 0.0, sb = 0.0, sc = 0.0;
    for (uint32_t i = threadIdx.x; i < G; i += NT) {
        sa += ld_agent(&blk_part[i].a);
        sb += ld_agent(&blk_part[i].b);
        sc += ld_agent(&blk_part[i].c);
    }
    block_sum3<NT>(sa, sb, sc, sm);
    if (threadIdx.x == 0) {
        if (accum) {
            sa = out->a + sa;
            sb = out->b + sb;
            sc = out->c + sc;
        }
        out->a = sa;
        out->b = sb;
        out->c = sc;
        out->d = 0.0;
        __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ------------------------------------------------------------------ device-side peer exchange
// Every rank of a row-sharded session owns one inbox (fine-grained-free, uncached device memory,
// exported to the other ranks by IPC handle or, in a loopback world, by plain pointer):
//   flag[q]          epoch written by rank q: q has delivered everything of its launch flag - 2
//   part[p][q]       rank q's partial sums of its launch t, p = t & 1
//   ghosts[p][...]   x-space ghost entries (this rank's [lower | upper] ghost order) of y_t, p = t & 1
// Producers store with system-scope (sc0 sc1) stores and drain them (s_waitcnt vmcnt(0)) before
// the block's ticket; the last-arriving block then stores the partial and, after a second drain,
// the flag.  Consumers poll the flag and read partials and ghosts with system-scope loads only
// (MI355X_MICROARCH.md, inter-workgroup visibility: every store and every load of the handed-off
// bytes bypasses the non-coherent caches, so no acquire fence is needed).
constexpr int kMaxPeerRanks = 64;
struct alignas(128) PeerInbox {
    uint64_t flag[kMaxPeerRanks];
    part4 part[2][kMaxPeerRanks];
};
constexpr int kGhostSliceBit = 1 << 20;   // slice meta .z: the slice reads ghost x entries
// slice meta .z bits 21..24: the slice's stream segment.  Slice streams larger than 4 GiB are cut
// into segments of < 4 GiB; a slice's 32-bit offsets are relative to its segment's base, so the
// kernels keep 32-bit address arithmetic for any matrix that fits HBM.
constexpr int kSliceSegShift = 21;
constexpr int kMaxSliceSeg = 16;

struct PeerArgs {
    PeerInbox* const* peers;   // peers[q]: rank q's inbox as mapped in this process (peers[me] = own)
    PeerInbox* inbox;          // own inbox
    const int4* push;          // {local row, peer, slot, 0} sorted by row
    const int2* slice_push;    // per slice: [begin, end) of its rows' entries in push
    int64_t ghost_stride;      // scalars per parity in a ghost area
    int32_t me, P;
};

template <class S>
__device__ __forceinline__ S* peer_ghosts(PeerInbox* b, int parity, int64_t stride) {
    return reinterpret_cast<S*>(b + 1) + parity * stride;
}
__device__ __forceinline__ double ld_sys(const double* p) {
    return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p) {
    return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ double ld_sys_s(const double* p) { return ld_sys(p); }
__device__ __forceinline__ cplx ld_sys_s(const cplx* p) {
    return cplx{ld_sys(&p->re), ld_sys(&p->im)};
}
__device__ __forceinline__ float ld_sys_s(const float* p) {
    return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ cplxf ld_sys_s(const cplxf* p) { return cplxf{ld_sys_s(&p->re), ld_sys_s(&p->im)}; }
__device__ __forceinline__ void st_sys_s(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys_s(cplxf* p, cplxf v) {
    st_sys_s(&p->re, v.re);
    st_sys_s(&p->im, v.im);
}
__device__ __forceinline__ void st_sys_s(double* p, double v) { st_sys(p, v); }
__device__ __forceinline__ void st_sys_s(cplx* p, cplx v) {
    st_sys(&p->re, v.re);
    st_sys(&p->im, v.im);
}

// Poll budget of a peer wait: 10 s of the 100 MHz constant clock (s_memrealtime).  A wait that
// runs out marks the session faulted instead of hanging the GPU.
constexpr uint64_t kPeerWaitTicks = 1000000000ull;

// Thread 0 only: wait until every peer's flag reached `epoch`; on timeout returns 1 + the peer
// that did not deliver (0: all delivered).
__device__ __forceinline__ int peer_wait(PeerInbox* inbox, int P, int me, uint64_t epoch) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int q = 0; q < P; ++q) {
        if (q == me) continue;
        while (ld_sys(&inbox->flag[q]) < epoch) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > kPeerWaitTicks) return 1 + q;
        }
    }
    return 0;
}

// Thread 0 of the last-arriving block: this rank's partial to part[parity][me] of every inbox,
// drained, then the epoch flag of every peer.
__device__ __forceinline__ void peer_publish(const PeerArgs& pa, int parity, const part4& mine,
                                             uint64_t epoch) {
    for (int q = 0; q < pa.P; ++q) {
        part4* d = &pa.peers[q]->part[parity][pa.me];
        st_sys(&d->a, mine.a);
        st_sys(&d->b, mine.b);
        st_sys(&d->c, mine.c);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int q = 0; q < pa.P; ++q)
        if (q != pa.me) st_sys(&pa.peers[q]->flag[pa.me], epoch);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Launch prologue of the fused power iteration, evaluated by thread 0 and broadcast through LDS.
struct alignas(16) Prologue {
    double nrm;       // ||y_{t-1}||: x_t = y_{t-1} / nrm (nrm == 0 only at t == 0: x0 == 0, kept as is)
    int32_t go;       // 1: this launch computes; 0: the loop has ended
    int32_t t;
    double s;         // multi-solve launches (shift_multi_prologue): the power of two scaling solves 1..K-1
};

// peer != nullptr: row-sharded session on the device-side peer exchange — wait for every peer's
// flag of the previous launch (epoch t + 1), then read the rank partials from the own inbox.
//
// cont: the second launch of an iteration split in two row parts (row-sharded sessions that
// overlap the first part's all-gather with the second part's product): the first launch's
// prologue already decided and advanced the carry, so this one only reads its decision.
template <class S>
__device__ __forceinline__ void power_prologue(PowerCtl* ctl, const part4* rank_part, int nranks,
                                               int parity, S* trace, Prologue* out,
                                               const PeerArgs* peer = nullptr, bool cont = false) {
    if (cont) {
        if (threadIdx.x == 0) {
            Prologue pr{0.0, 0, 0};
            if (!__hip_atomic_load(&ctl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                const PowerCarry o = ctl->st[parity ^ 1];
                pr.go = 1;
                pr.nrm = o.nrm;
                pr.t = o.t;
            }
            *out = pr;
        }
        __syncthreads();
        return;
    }
    if (threadIdx.x == 0) {
        Prologue pr{0.0, 0, 0};
        int done = __hip_atomic_load(&ctl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const PowerCarry in = ctl->st[parity];
        const int32_t t = in.t + 1;
        bool ok = true;
        if (!done && peer) {
            // a faulted session stops at once (later launches must not wait again)
            ok = __hip_atomic_load(&ctl->fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
            const int miss = ok ? peer_wait(peer->inbox, peer->P, peer->me, (uint64_t)t + 1) : 0;
            if (miss) {
                ok = false;
                // which peer, at which launch: (peer + 1) | t << 8
                __hip_atomic_store(&ctl->fault, miss | (t << 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (!done && ok) {
            double n2 = 0.0, rr = 0.0, ri = 0.0;
            if (peer) {
                const part4* rp = peer->inbox->part[parity ^ 1];
                for (int r = 0; r < nranks; ++r) {   // rank order: identical on every rank
                    n2 += ld_sys(&rp[r].a);
                    rr += ld_sys(&rp[r].b);
                    ri += ld_sys(&rp[r].c);
                }
            } else {
                for (int r = 0; r < nranks; ++r) {   // rank order: identical on every rank
                    n2 += rank_part[r].a;
                    rr += rank_part[r].b;
                    ri += rank_part[r].c;
                }
            }
            const double nrm = sqrt(n2);
            const bool cplx_ = is_cplx_v<S>;
            const PowerDecision d = power_decide(t, ctl->max_iter, ctl->tol, cplx_, nrm, rr, ri,
                                                 in.rho_re, in.rho_im);
            if (blockIdx.x == 0) {
                PowerCarry o;
                o.rho_re = rr;
                o.rho_im = ri;
                o.nrm = nrm;
                o.t = t;
                o.pad = 0;
                ctl->st[parity ^ 1] = o;
                ctl->launches = t + 1;
                if (d.record) ctl->ntrace = d.k + 1;
                if (d.record && trace && d.k < ctl->trace_cap) set_re_im(trace[d.k], d.lam_re, d.lam_im);
                if (d.done) {
                    ctl->lam_re = d.lam_re;
                    ctl->lam_im = d.lam_im;
                    ctl->iters = d.iters;
                    ctl->converged = d.converged ? 1 : 0;
                    ctl->final_parity = parity;   // x_final = y_{t-2} / ||y_{t-2}|| in B[t & 1]
                    ctl->final_norm = in.nrm;
                    __hip_atomic_store(&ctl->done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            pr.go = d.done ? 0 : 1;
            pr.nrm = nrm;
            pr.t = t;
        }
        *out = pr;
    }
    __syncthreads();
}

template <class S>
__device__ __forceinline__ S scale_in(S y, double nrm) {
    return nrm > 0.0 ? divr(y, nrm) : y;   // Eigen normalize(): unchanged when the norm is 0
}

// base + 32-bit element index: lets hipcc use the SGPR-base + 32-bit VGPR-offset form of
// global_load instead of per-lane 64-bit address arithmetic.  Every stream the kernels index
// this way is < 4 GiB (checked at upload).
template <class T>
__device__ __forceinline__ T ldg(const T* base, uint32_t i) {
    return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) +
                                       (uint64_t)(i * (uint32_t)sizeof(T)));
}
// streaming (read-once) variant: non-temporal, so the matrix stream does not evict the x windows
#ifndef EIGSOL_STREAM_NT
#define EIGSOL_STREAM_NT 1
#endif
template <class T>
__device__ __forceinline__ T ldg_stream(const T* base, uint32_t i) {
    const T* p = reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + (uint64_t)(i * (uint32_t)sizeof(T)));
#if EIGSOL_STREAM_NT
    if constexpr (std::is_arithmetic_v<T>) {
        return __builtin_nontemporal_load(p);
    } else if constexpr (sizeof(T) == 16) {           // double2, cplx, int4
        typedef double d2v __attribute__((ext_vector_type(2)));
        const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
        T r;
        __builtin_memcpy(&r, &v, 16);
        return r;
    } else {                                          // int2 and other 8-byte aggregates
        static_assert(sizeof(T) == 8, "ldg_stream: unsupported width");
        const long long v = __builtin_nontemporal_load(reinterpret_cast<const long long*>(p));
        T r;
        __builtin_memcpy(&r, &v, 8);
        return r;
    }
#else
    return *p;
#endif
}

}  // namespace dev
}  // namespace eigsol

namespace eigsol {
namespace dev {

__device__ __forceinline__ cplx cdiv(cplx a, cplx b) {
    // textbook quotient with one real division by |b|^2 (b is a pivot, never tiny in practice)
    const double d = b.re * b.re + b.im * b.im;
    return cplx{(a.re * b.re + a.im * b.im) / d, (a.im * b.re - a.re * b.im) / d};
}
__device__ __forceinline__ double sdiv(double a, double b) { return a / b; }
__device__ __forceinline__ cplx sdiv(cplx a, cplx b) { return cdiv(a, b); }
__device__ __forceinline__ float sdiv(float a, float b) { return a / b; }
__device__ __forceinline__ cplxf sdiv(cplxf a, cplxf b) {
    const float d = b.re * b.re + b.im * b.im;
    return cplxf{(a.re * b.re + a.im * b.im) / d, (a.im * b.re - a.re * b.im) / d};
}

// Launch prologue of the fused shifted-inverse iteration (shiftedInversePowerImpl,
// src/power_method/shifted_inverse_power_solver.hpp:48-76).  Launch t solves (A - sigma I) y_t = x_t
// with x_t = y_{t-1} / ||y_{t-1}||; its partials are ||y_t||^2 and p_t = x_t^H y_t.  Because
// A y_t = x_t + sigma y_t, the reference's Rayleigh quotient on A (:62) of x_{t+1} = y_t/||y_t|| is
//     lambda_t = sigma + conj(p_t) / ||y_t||^2
// so the prologue of launch t+1 completes reference iteration k = t with no extra product.
// Carry record: rho = lambda_{t-1} (previous estimate), nrm = ||y_{t-1}||.
template <class S>
__device__ __forceinline__ void shift_prologue(PowerCtl* ctl, const part4* rank_part, int parity,
                                               S* trace, double sig_re, double sig_im,
                                               Prologue* out) {
    if (threadIdx.x == 0) {
        Prologue pr{0.0, 0, 0};
        const int done = __hip_atomic_load(&ctl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!done) {
            const PowerCarry in = ctl->st[parity];
            const int32_t t = in.t + 1;
            const double n2 = rank_part[0].a, pr_ = rank_part[0].b, pi_ = rank_part[0].c;
            const double nrm = sqrt(n2);
            const bool cplx_ = is_cplx_v<S>;
            bool fin = false, conv = false, rec = false;
            int32_t iters = 0, fpar = 0;
            double lre = in.rho_re, lim = in.rho_im, fnorm = 0.0;
            if (t >= 1) {
                const int32_t k = t - 1;
                if (nrm == 0.0) {                 // normY == 0 (:55-58): x, lambda unchanged
                    fin = true;
                    iters = t;
                    fpar = parity;                // x_{t-1} = y_{t-2} / ||y_{t-2}||
                    fnorm = in.nrm;
                    if (t < 2) { lre = 0.0; lim = 0.0; }
                } else {
                    lre = sig_re + pr_ / n2;
                    lim = cplx_ ? sig_im - pi_ / n2 : 0.0;
                    rec = true;
                    fpar = parity ^ 1;            // x_{t} = y_{t-1} / ||y_{t-1}||
                    fnorm = nrm;
                    if (k >= 1 && close_rel(lre, lim, in.rho_re, in.rho_im, ctl->tol, cplx_)) {
                        fin = true;               // :64-70
                        conv = true;
                        iters = t;
                    } else if (t >= ctl->max_iter) {
                        fin = true;               // loop bound :48
                        iters = t;
                    }
                }
            }
            if (blockIdx.x == 0) {
                PowerCarry o;
                o.rho_re = lre;
                o.rho_im = lim;
                o.nrm = nrm;
                o.t = t;
                o.pad = 0;
                ctl->st[parity ^ 1] = o;
                ctl->launches = t + 1;
                if (rec) ctl->ntrace = t;
                if (rec && trace && t - 1 < ctl->trace_cap) set_re_im(trace[t - 1], lre, lim);
                if (fin) {
                    ctl->lam_re = lre;
                    ctl->lam_im = lim;
                    ctl->iters = iters;
                    ctl->converged = conv ? 1 : 0;
                    ctl->final_parity = fpar;
                    ctl->final_norm = fnorm;
                    __hip_atomic_store(&ctl->done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            pr.go = fin ? 0 : 1;
            pr.nrm = nrm;
            pr.t = t;
        }
        *out = pr;
    }
    __syncthreads();
}

// Multi-solve launches (triangular factors; shifted.hip, sptrsv_chunk_role_kernel): launch 0 is an
// ordinary single solve (reference iteration 0), launch t >= 1 runs reference iterations
// k_j = 1 + K (t - 1) + j, j = 0..K-1, together.  Solve 0 is w_0 = (A - sigma I)^{-1} x
// with x = v / ||v|| (v the previous launch's last solution), exactly as a single launch does;
// solve j >= 1 is w_j = (A - sigma I)^{-1} (s w_{j-1}) with s = 2^-e an exact power of two near
// 1 / ||w_0|| (e from the previous launch's growth ||w_0||, which launch 0 measures, so the chain
// stays near unit size instead of growing as ||w_0||^K).  The reference's
// iterate of k_j (j >= 1) is y = (A - sigma I)^{-1} (w_{j-1} / ||w_{j-1}||) = w_j / (s ||w_{j-1}||):
// solve j defers the normalisation to after the solve (linearity), which is what lets it start
// before ||w_{j-1}|| exists, one dependency round behind solve j - 1.  It differs from the
// reference's y only by the rounding of that division (the factor paths are
// tolerance parity).  Partials of solve j: {||w_j||^2, w_{j-1}^H w_j} (w_{-1} = x; j = 0 in
// part0, j >= 1 in kpart[j - 1]); the Rayleigh quotients are
//     lambda_k0 = sigma + conj(x^H w_0) / ||w_0||^2,   lambda_kj = sigma + s conj(w_{j-1}^H w_j) / ||w_j||^2
// and the prologue of launch t+1 applies the reference's tests (normY == 0, is_close_relative,
// maxIterations; shifted_inverse_power_solver.hpp:48-76) to k_0, k_1, ... in order, so the
// iteration count is the reference's; the work past the stopping iteration is discarded.
// Final iterate x: w_j / ||w_j|| (final_parity 2 + j: the factor's buffer aux[j], j < K - 1;
// B[parity ^ 1] for j = K - 1); a zero norm at k_j keeps the previous x (w_{j-1}, or the
// previous input B[parity]).  Carry: rho = last lambda, nrm = ||v|| (this launch's input norm),
// pad = e (this launch's exponent, read back for the lambdas).
template <class S>
__device__ __forceinline__ void shift_multi_prologue(PowerCtl* ctl, const part4* part0, const part4* kpart, int K,
                                                     int parity, S* trace, double sig_re, double sig_im,
                                                     Prologue* out) {
    if (threadIdx.x == 0) {
        Prologue pr{0.0, 0, 0, 1.0};
        const int done = __hip_atomic_load(&ctl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!done) {
            const PowerCarry in = ctl->st[parity];
            const int32_t t = in.t + 1;
            const bool cplx_ = is_cplx_v<S>;
            bool fin = false, conv = false;
            int32_t iters = 0, fpar = 0, ntr = -1, e = 0;
            double lre = in.rho_re, lim = in.rho_im, fnorm = 0.0, nrm;
            if (t == 0) {
                nrm = sqrt(part0[0].a);   // ||x0||^2 from begin()
            } else {
                // launch 0 of a multi-solve session is an ordinary single solve (shift_launch_t): with
                // no growth estimate yet, a chain of K solves would grow as g^K and could overflow
                const bool prev_single = t == 1;
                const int Kp = prev_single ? 1 : K;
                const int32_t kbase = prev_single ? 0 : 1 + K * (t - 2);
                const double s_prev = ldexp(1.0, -in.pad);
                double prev_n = in.nrm;   // norm of the previous x's buffer
                int prev_par = parity;    // ... and its final_parity code
                for (int j = 0; j < Kp && !fin; ++j) {
                    const part4 pj = j ? kpart[j - 1] : part0[0];
                    const int32_t k = kbase + j;
                    const int code = j == Kp - 1 ? (parity ^ 1) : 2 + j;
                    if (pj.a == 0.0) {                    // normY == 0 (:55-58): x, lambda unchanged
                        fin = true;
                        iters = k + 1;
                        fpar = prev_par;
                        fnorm = prev_n;
                        if (k == 0) { lre = 0.0; lim = 0.0; }
                        break;
                    }
                    const double sc = j ? s_prev : 1.0;
                    const double lr = sig_re + sc * pj.b / pj.a;
                    const double li = cplx_ ? sig_im - sc * pj.c / pj.a : 0.0;
                    ntr = k + 1;
                    if (trace && k < ctl->trace_cap && blockIdx.x == 0) set_re_im(trace[k], lr, li);
                    fpar = code;
                    fnorm = sqrt(pj.a);
                    if (k >= 1 && close_rel(lr, li, lre, lim, ctl->tol, cplx_)) {
                        fin = true;                       // :64-70
                        conv = true;
                        iters = k + 1;
                    } else if (k + 1 >= ctl->max_iter) {
                        fin = true;                       // loop bound :48
                        iters = k + 1;
                    }
                    lre = lr;
                    lim = li;
                    prev_n = fnorm;
                    prev_par = code;
                }
                nrm = sqrt((Kp > 1 ? kpart[Kp - 2] : part0[0]).a);
                // growth of the previous launch's first solve from a unit input
                const double g = sqrt(part0[0].a);
                if (g > 0.0 && g < INFINITY) e = min(max(ilogb(g), -900), 900);
                if constexpr (!std::is_same_v<S, double> && !std::is_same_v<S, cplx>)
                    e = min(max(e, -100), 100);
            }
            if (blockIdx.x == 0) {
                PowerCarry o;
                o.rho_re = lre;
                o.rho_im = lim;
                o.nrm = nrm;
                o.t = t;
                o.pad = e;
                ctl->st[parity ^ 1] = o;
                ctl->launches = t + 1;
                if (ntr >= 0) ctl->ntrace = ntr;
                if (fin) {
                    ctl->lam_re = lre;
                    ctl->lam_im = lim;
                    ctl->iters = iters;
                    ctl->converged = conv ? 1 : 0;
                    ctl->final_parity = fpar;
                    ctl->final_norm = fnorm;
                    __hip_atomic_store(&ctl->done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            pr.go = fin ? 0 : 1;
            pr.nrm = nrm;
            pr.t = t;
            pr.s = ldexp(1.0, -e);
        }
        *out = pr;
    }
    __syncthreads();
}

}  // namespace dev
}  // namespace eigsol

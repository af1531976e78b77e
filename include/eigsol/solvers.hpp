// EigSol drop-in façade — solver entry points, same names, signatures, check order and exception
// messages as the reference, numeric core on the gfx950 device through the C ABI.
//
//   powerMethod<S>                 src/power_method/power_method.hpp:135-148
//   shiftedInversePowerMethod<S>   src/power_method/shifted_inverse_power_solver.hpp:112-125
//   solve_shifted<S>               src/matrix/solve_shifted.hpp:48-118
//   to_hessenberg<S> / _dense      src/qr_method/to_hessenberg.hpp:23-119
//   qr_decompose<S> / _dense       src/qr_method/qr_decompose.hpp:25-132
//   qr_eigenvalues<S> / _dense     src/qr_method/qr_eigenvalues.hpp:40-147
//
// Scalars: double and std::complex<double> natively; float and std::complex<float> natively for the
// power method and the triangular-CSR shifted inverse, promoted to fp64 for the other solvers
// (core.hpp, PromotedScalar); long double / std::complex<long double> in double-double on the
// device (core.hpp, WideScalar: every solver; qr_eigenvalues' Francis variant refines the fp64
// sweeps' eigenvalues in double-double).
//
// Start vector: the reference draws x0 with Eigen's Vector::Random (std::rand, not reproducible
// across Eigen versions).  Here x0 comes from a documented generator
// (std::mt19937_64 seeded with EigSol::random_seed(), U(-1, 1) per real/imaginary component);
// overloads taking an explicit x0 are provided.  Iteration semantics (counts, convergence test,
// zero-norm and maxIterations <= 0 cases) are the reference's, evaluated on the device.
#pragma once

#include <random>
#include <typeinfo>
#include <utility>

#include "matrix.hpp"

namespace EigSol {

inline std::uint64_t& random_seed() {
    static std::uint64_t seed = 0x5eed5eedULL;
    return seed;
}

namespace detail {
struct RandomState {
    std::mt19937_64 gen{random_seed()};
    std::uint64_t seeded = random_seed();
};
inline RandomState& random_state() {
    static RandomState st;
    return st;
}
// One generator for every scalar type; re-seeded whenever EigSol::random_seed() holds a new value
// since the last draw (so setting the seed between solves takes effect, like std::srand before the
// reference's Eigen Vector::Random).
inline std::mt19937_64& random_engine() {
    RandomState& st = random_state();
    if (st.seeded != random_seed()) {
        st.seeded = random_seed();
        st.gen.seed(st.seeded);
    }
    return st.gen;
}
}  // namespace detail

// std::srand counterpart: always restarts the start-vector sequence, also for an unchanged seed.
inline void set_random_seed(std::uint64_t seed) {
    random_seed() = seed;
    detail::random_state().seeded = seed;
    detail::random_state().gen.seed(seed);
}

template <ScalarConcept S>
Vector<S> random_vector(std::size_t n) {
    std::mt19937_64& gen = detail::random_engine();
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    Vector<S> v(n);
    for (std::size_t i = 0; i < n; ++i) {
        if constexpr (is_complex_of_floating<S>::value) {
            const double re = u(gen);
            const double im = u(gen);
            v(i) = S(re, im);
        } else {
            v(i) = S(u(gen));
        }
    }
    return v;
}

template <typename S>
void DenseMatrix<S>::setRandom() {
    Vector<S> v = random_vector<S>(static_cast<std::size_t>(size()));
    std::copy(v.begin(), v.end(), d_.begin());
}

// QR iteration variant.  Francis (Hessenberg + implicit multishift sweeps with aggressive early
// deflation, the north_star path) is the default of every overload, as in the Python binding: it
// converges on general real and complex matrices (the reference's loop does not),
// deflates at LAPACK's threshold, reports `iterations` as the most sweeps any deflation needed
// (within [1, maxIterations] exactly when converged) and returns the real parts in `eigenvalues`
// with the complex eigenvalues in `eigenvalues_complex`.  The reference's own unshifted H <- RQ
// iteration (qr_eigenvalues.hpp:62-105: identical iteration counts, `converged` and positional
// diag(H)) is QRVariant::Unshifted.  The reference's tests check sorted eigenvalues, `converged`
// and 1 <= iterations <= maxIterations (qr_algorithms_test.cpp:253-332), which both satisfy.
enum class QRVariant { Francis = EIGSOL_QR_FRANCIS, Unshifted = EIGSOL_QR_UNSHIFTED };

namespace detail {

inline eigsol_solver_options copts(const SolverOptions& o) {
    eigsol_solver_options c;
    c.max_iterations = o.maxIterations;
    c.tolerance = o.tolerance;
    return c;
}

template <typename S>
void require_device_scalar(const char* who) {
    if constexpr (!DeviceCapable<S>)
        throw std::runtime_error(std::string(who) + ": scalar type not supported by the device path "
                                                    "(double, std::complex<double>, float, std::complex<float>)");
}

// element-wise conversions between a scalar type and its device (fp64) type
template <typename T, typename U>
Vector<T> convert_vec(const Vector<U>& v) {
    if constexpr (std::is_same_v<T, U>) return v;
    else {
        Vector<T> w(v.size());
        for (std::size_t i = 0; i < v.size(); ++i) w(i) = static_cast<T>(v(i));
        return w;
    }
}
template <typename T, typename U>
DenseMatrix<T> convert_dense(const DenseMatrix<U>& a) {
    DenseMatrix<T> b(a.rows(), a.cols());
    for (std::int64_t i = 0; i < a.size(); ++i) b.data()[i] = static_cast<T>(a.data()[i]);
    return b;
}

// long double: the same run with the vectors, the shift and the results as double-double pairs
template <typename S>
int power_run_wide(const DeviceMatrix& d, bool dense, const eigsol_solver_options& o, const Vector<S>& xs0,
                   const S* shift, EigenResult<S>& out) {
    using Wt = wire_t<S>;
    const std::vector<Wt> xw = to_wire_vec(xs0.data(), xs0.size());
    const Wt sh = shift ? to_wire(*shift) : to_wire(S(0));
    Wt lam{};
    std::vector<Wt> x(xs0.size());
    std::int32_t it = 0, conv = 0;
    int st;
    if (shift)
        st = dense ? eigsol_shifted_inverse_dense(d.dense(), &sh, &o, xw.data(), &lam, x.data(), &it, &conv)
                   : eigsol_shifted_inverse_csr(d.csr(), &sh, &o, xw.data(), &lam, x.data(), &it, &conv);
    else
        st = dense ? eigsol_power_dense(d.dense(), &o, xw.data(), &lam, x.data(), &it, &conv)
                   : eigsol_power_csr(d.csr(), &o, xw.data(), &lam, x.data(), &it, &conv);
    if (st == EIGSOL_OK) {
        Vector<S> xs(x.size());
        for (std::size_t i = 0; i < x.size(); ++i) xs(i) = from_wire(x[i]);
        out = EigenResult<S>(from_wire(lam), xs, it, conv != 0);
    }
    return st;
}

// One device run in scalar type D (S itself, or its fp64 promotion).
template <typename D, typename S>
int power_run(const DeviceMatrix& d, bool dense, const eigsol_solver_options& o, const Vector<S>& xs0,
              const S* shift, EigenResult<S>& out) {
    const Vector<D> xs = convert_vec<D>(xs0);
    const D sh = shift ? static_cast<D>(*shift) : D{};
    D lam{};
    Vector<D> x(xs0.size());
    std::int32_t it = 0, conv = 0;
    int st;
    if (shift)
        st = dense ? eigsol_shifted_inverse_dense(d.dense(), &sh, &o, xs.data(), &lam, x.data(), &it, &conv)
                   : eigsol_shifted_inverse_csr(d.csr(), &sh, &o, xs.data(), &lam, x.data(), &it, &conv);
    else
        st = dense ? eigsol_power_dense(d.dense(), &o, xs.data(), &lam, x.data(), &it, &conv)
                   : eigsol_power_csr(d.csr(), &o, xs.data(), &lam, x.data(), &it, &conv);
    if (st == EIGSOL_OK) out = EigenResult<S>(static_cast<S>(lam), convert_vec<S>(x), it, conv != 0);
    return st;
}

template <typename S>
EigenResult<S> power_like(const Matrix& M, const SolverOptions& opts, const Vector<S>* x0, const S* shift,
                          const char* who) {
    if (M.scalar_type() != typeid(S)) throw std::runtime_error(std::string(who) + ": scalar type mismatch");
    const std::int64_t r = M.rows(), c = M.cols();
    if (r != c) throw std::runtime_error(std::string(who) + ": matrix must be square");
    if (r == 0) throw std::runtime_error(std::string(who) + ": matrix has zero size");
    require_device_scalar<S>(who);
    EigenResult<S> res;
    if constexpr (DeviceCapable<S>) {
        Vector<S> xs0 = x0 ? *x0 : random_vector<S>(static_cast<std::size_t>(r));
        if (xs0.size() != static_cast<std::size_t>(r))
            throw std::runtime_error(std::string(who) + ": start vector size mismatch");
        const eigsol_solver_options o = copts(opts);
        // single precision runs natively (power method; shifted inverse on dense, banded and
        // triangular factors); only a general sparse pattern with neither a usable band nor a dense
        // factor that fits (ILU(0)-GMRES, double-only) is promoted to fp64
        int st = EIGSOL_E_UNSUPPORTED;
        if constexpr (WideScalar<S>) {   // long double: double-double kernels (see core.hpp)
            st = power_run_wide<S>(M.device<S>(), M.isDense(), o, xs0, shift, res);
        } else {
            st = power_run<S>(M.device<S>(), M.isDense(), o, xs0, shift, res);
        }
        if constexpr (PromotedScalar<S>) {
            if (st == EIGSOL_E_UNSUPPORTED && shift)
                st = power_run<device_scalar_t<S>>(M.device_fp64<S>(), M.isDense(), o, xs0, shift, res);
        }
        check(st, who);
    }
    return res;
}

template <typename S>
void dense_square_check(const DenseMatrix<S>& A, const char* who) {
    if (A.rows() != A.cols()) throw std::runtime_error(std::string(who) + ": A must be square");
}

}  // namespace detail

// ------------------------------------------------------------------------------ power methods
template <ScalarConcept S>
EigenResult<S> powerMethod(const Matrix& M, const SolverOptions& opts = SolverOptions{}) {
    return detail::power_like<S>(M, opts, nullptr, nullptr, "powerMethod");
}
template <ScalarConcept S>
EigenResult<S> powerMethod(const Matrix& M, const SolverOptions& opts, const Vector<S>& x0) {
    return detail::power_like<S>(M, opts, &x0, nullptr, "powerMethod");
}

template <ScalarConcept S>
EigenResult<S> shiftedInversePowerMethod(const Matrix& M,
                                         const ShiftedSolverOptions<S>& opts = ShiftedSolverOptions<S>{}) {
    return detail::power_like<S>(M, opts, nullptr, &opts.shift, "shiftedInversePowerMethod");
}
template <ScalarConcept S>
EigenResult<S> shiftedInversePowerMethod(const Matrix& M, const ShiftedSolverOptions<S>& opts, const Vector<S>& x0) {
    return detail::power_like<S>(M, opts, &x0, &opts.shift, "shiftedInversePowerMethod");
}

// --------------------------------------------------------------------------------- solve_shifted
template <ScalarConcept S>
Vector<S> solve_shifted(const Matrix& A, const S shift, const Vector<S>& b) {
    if (A.scalar_type() != typeid(S)) throw std::runtime_error("solve_shifted: scalar type mismatch");
    const char* kind = A.isDense() ? "dense" : "sparse";
    if (A.rows() != A.cols())
        throw std::runtime_error(std::string("solve_shifted: A must be square (") + kind + " case)");
    if (A.rows() != static_cast<std::int64_t>(b.size()))
        throw std::runtime_error(std::string("solve_shifted: size mismatch between A and b (") + kind + " case)");
    detail::require_device_scalar<S>("solve_shifted");
    Vector<S> x(b.size());
    if constexpr (DeviceCapable<S>) {
        if (b.size() == 0) return x;
        const std::int64_t n = static_cast<std::int64_t>(b.size());
        auto run = [&](auto tag, const detail::DeviceMatrix& d) {
            using D = decltype(tag);
            const D sh = static_cast<D>(shift);
            const Vector<D> bd = detail::convert_vec<D>(b);
            Vector<D> xd(b.size());
            const int st = A.isDense() ? eigsol_solve_shifted_dense(d.dense(), &sh, bd.data(), n, xd.data())
                                       : eigsol_solve_shifted_csr(d.csr(), &sh, bd.data(), n, xd.data());
            if (st == EIGSOL_OK) x = detail::convert_vec<S>(xd);
            return st;
        };
        // single precision natively (dense, banded and triangular factors in float); the fp64
        // factor only where the single-precision one is not built (general sparse via GMRES)
        int st = EIGSOL_E_UNSUPPORTED;
        if constexpr (WideScalar<S>) {   // double-double pairs in and out
            const detail::DeviceMatrix& d = A.device<S>();
            const wire_t<S> sh = to_wire(shift);
            const auto bw = to_wire_vec(b.data(), b.size());
            std::vector<wire_t<S>> xw(b.size());
            st = A.isDense() ? eigsol_solve_shifted_dense(d.dense(), &sh, bw.data(), n, xw.data())
                             : eigsol_solve_shifted_csr(d.csr(), &sh, bw.data(), n, xw.data());
            if (st == EIGSOL_OK)
                for (std::size_t i = 0; i < xw.size(); ++i) x(i) = from_wire(xw[i]);
        } else {
            st = run(S{}, A.device<S>());
        }
        if constexpr (PromotedScalar<S>)
            if (st == EIGSOL_E_UNSUPPORTED) st = run(device_scalar_t<S>{}, A.device_fp64<S>());
        detail::check(st, "solve_shifted");
    }
    return x;
}

// ------------------------------------------------------------------------------------ QR method
template <ScalarConcept S>
DenseMatrix<S> to_hessenberg_dense(const DenseMatrix<S>& A) {
    detail::dense_square_check(A, "to_hessenberg_dense");
    detail::require_device_scalar<S>("to_hessenberg_dense");
    DenseMatrix<S> H(A.rows(), A.cols());
    if constexpr (WideScalar<S>) {   // double-double reflectors
        if (A.rows() > 0) {
            const auto aw = to_wire_vec(A.data(), static_cast<std::size_t>(A.size()));
            std::vector<wire_t<S>> hw(aw.size());
            detail::check(eigsol_hessenberg_dense(detail::ctx(), detail::dtype_of<S>(), A.rows(), aw.data(), hw.data()),
                          "to_hessenberg_dense");
            for (std::size_t i = 0; i < hw.size(); ++i) H.data()[i] = from_wire(hw[i]);
        }
        return H;
    }
    if constexpr (DeviceScalar<S> || PromotedScalar<S>) {   // single precision: native float reduction
        if (A.rows() > 0)
            detail::check(eigsol_hessenberg_dense(detail::ctx(), detail::dtype_of<S>(), A.rows(), A.data(), H.data()),
                          "to_hessenberg_dense");
    }
    return H;
}

template <ScalarConcept S>
DenseMatrix<S> to_hessenberg(const Matrix& A) {
    if (!A.isDense()) throw std::runtime_error("to_hessenberg(Matrix): only dense matrices are supported");
    if (A.scalar_type() != typeid(S)) throw std::runtime_error("to_hessenberg(Matrix): scalar type mismatch");
    return to_hessenberg_dense<S>(A.cast<DenseMatrix<S>>());
}

template <ScalarConcept S>
void qr_decompose_dense(const DenseMatrix<S>& A, DenseMatrix<S>& Q, DenseMatrix<S>& R) {
    if (A.rows() == 0 || A.cols() == 0) throw std::runtime_error("qr_decompose_dense: empty matrix");
    detail::require_device_scalar<S>("qr_decompose_dense");
    if constexpr (WideScalar<S>) {   // double-double reflectors
        const auto aw = to_wire_vec(A.data(), static_cast<std::size_t>(A.size()));
        std::vector<wire_t<S>> qw(static_cast<std::size_t>(A.rows() * A.rows())), rw(aw.size());
        detail::check(eigsol_qr_decompose_dense(detail::ctx(), detail::dtype_of<S>(), A.rows(), A.cols(), aw.data(),
                                                qw.data(), rw.data()),
                      "qr_decompose_dense");
        Q = DenseMatrix<S>(A.rows(), A.rows());
        R = DenseMatrix<S>(A.rows(), A.cols());
        for (std::size_t i = 0; i < qw.size(); ++i) Q.data()[i] = from_wire(qw[i]);
        for (std::size_t i = 0; i < rw.size(); ++i) R.data()[i] = from_wire(rw[i]);
        return;
    }
    Q = DenseMatrix<S>(A.rows(), A.rows());
    R = DenseMatrix<S>(A.rows(), A.cols());
    if constexpr (DeviceScalar<S> || PromotedScalar<S>)   // single precision: native float QR
        detail::check(eigsol_qr_decompose_dense(detail::ctx(), detail::dtype_of<S>(), A.rows(), A.cols(), A.data(),
                                                Q.data(), R.data()),
                      "qr_decompose_dense");
}

template <ScalarConcept S>
std::pair<DenseMatrix<S>, DenseMatrix<S>> qr_decompose(const Matrix& A) {
    if (!A.isDense()) throw std::runtime_error("qr_decompose(Matrix): only dense matrices are supported");
    if (A.scalar_type() != typeid(S)) throw std::runtime_error("qr_decompose(Matrix): scalar type mismatch");
    DenseMatrix<S> Q, R;
    qr_decompose_dense<S>(A.cast<DenseMatrix<S>>(), Q, R);
    return {Q, R};
}

template <ScalarConcept S>
QRResult<S> qr_eigenvalues_dense(const DenseMatrix<S>& A, const SolverOptions& opts,
                                 QRVariant variant = QRVariant::Francis) {
    detail::dense_square_check(A, "qr_eigenvalues_dense");
    const std::int64_t n = A.rows();
    if (n == 0) return QRResult<S>(Vector<S>(), 0, true);   // qr_eigenvalues.hpp:55-57
    detail::require_device_scalar<S>("qr_eigenvalues_dense");
    if constexpr (WideScalar<S>) {
        // long double: Unshifted = the reference's own algorithm (H <- R Q, qr_eigenvalues.hpp:62-105)
        // in double-double; Francis = the fp64 multishift sweeps on the rounded double-double
        // Hessenberg matrix, every eigenvalue then refined in double-double by Newton's method on
        // det(H - mu I) (wide.hip), so no eigenvalue keeps fp64 accuracy only
        const auto aw = to_wire_vec(A.data(), static_cast<std::size_t>(A.size()));
        std::vector<wire_t<S>> ew(static_cast<std::size_t>(n));
        std::vector<double> eim(2 * static_cast<std::size_t>(n), 0.0);   // real long double: imaginary dd parts
        std::int32_t it = 0, conv = 0;
        const eigsol_solver_options o = detail::copts(opts);
        const bool francis = variant == QRVariant::Francis;
        detail::check(eigsol_qr_eigenvalues_dense(detail::ctx(), detail::dtype_of<S>(), n, aw.data(), &o,
                                                  static_cast<int>(variant), ew.data(),
                                                  francis ? eim.data() : nullptr, &it, &conv),
                      "qr_eigenvalues_dense");
        Vector<S> ev(static_cast<std::size_t>(n));
        for (std::int64_t i = 0; i < n; ++i) ev(i) = from_wire(ew[static_cast<std::size_t>(i)]);
        QRResult<S> r(ev, it, conv != 0);
        if (francis) {
            r.eigenvalues_complex_extended.resize(static_cast<std::size_t>(n));
            r.eigenvalues_complex.resize(static_cast<std::size_t>(n));
            for (std::int64_t i = 0; i < n; ++i) {
                std::complex<long double> z;
                if constexpr (std::is_same_v<S, long double>)
                    z = {ev(i), static_cast<long double>(eim[2 * i]) + static_cast<long double>(eim[2 * i + 1])};
                else z = ev(i);
                r.eigenvalues_complex_extended[i] = z;
                r.eigenvalues_complex[i] = {static_cast<double>(z.real()), static_cast<double>(z.imag())};
            }
        }
        return r;
    }
    // single precision: the reference's unshifted iteration natively in float; the Francis sweeps
    // (double kernels) on the fp64 promotion, eigenvalues rounded back
    if constexpr (PromotedScalar<S>) if (variant == QRVariant::Francis) {
        using D = device_scalar_t<S>;
        const QRResult<D> rd = qr_eigenvalues_dense<D>(detail::convert_dense<D>(A), opts, variant);
        QRResult<S> rs(detail::convert_vec<S>(rd.eigenvalues), rd.iterations, rd.converged);
        rs.eigenvalues_complex = rd.eigenvalues_complex;
        return rs;
    }
    QRResult<S> res;
    if constexpr (DeviceScalar<S> || PromotedScalar<S>) {
        Vector<S> ev(static_cast<std::size_t>(n));
        std::vector<double> wi(static_cast<std::size_t>(n), 0.0);
        std::int32_t it = 0, conv = 0;
        const eigsol_solver_options o = detail::copts(opts);
        detail::check(eigsol_qr_eigenvalues_dense(detail::ctx(), detail::dtype_of<S>(), n, A.data(), &o,
                                                  static_cast<int>(variant), ev.data(), wi.data(), &it, &conv),
                      "qr_eigenvalues_dense");
        res = QRResult<S>(ev, it, conv != 0);
        if (variant == QRVariant::Francis) {
            res.eigenvalues_complex.resize(static_cast<std::size_t>(n));
            for (std::int64_t i = 0; i < n; ++i) {
                if constexpr (std::is_same_v<S, double>) res.eigenvalues_complex[i] = {ev(i), wi[i]};
                else res.eigenvalues_complex[i] = ev(i);   // complex sweeps return the eigenvalues themselves
            }
        }
    }
    return res;
}

template <ScalarConcept S>
QRResult<S> qr_eigenvalues(const Matrix& A, const SolverOptions& opts, QRVariant variant = QRVariant::Francis) {
    if (!A.isDense()) throw std::runtime_error("qr_eigenvalues(Matrix): only dense matrices are supported");
    if (A.scalar_type() != typeid(S)) throw std::runtime_error("qr_eigenvalues(Matrix): scalar type mismatch");
    return qr_eigenvalues_dense<S>(A.cast<DenseMatrix<S>>(), opts, variant);
}

}  // namespace EigSol

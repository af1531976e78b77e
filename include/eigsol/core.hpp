// EigSol drop-in façade — value types (no Eigen dependency).
//
// Mirrors the reference's public types so that code written against
// hugoheziyang/PCSC_Eigenvalue_Solver_Project compiles unchanged for the scalar types the
// device path supports (double, std::complex<double>):
//   ScalarConcept / Vector<S>        src/core/types.hpp:16-33
//   is_close_relative                src/core/tolerance.hpp:28-33
//   SolverOptions                    src/option/solver_option.hpp:14-20
//   ShiftedSolverOptions<S>          src/option/shifted_solver_option.hpp:24-68
//   EigenResult<S>                   src/result/eigen_result.hpp:22-52
//   QRResult<S>                      src/result/qr_result.hpp:25-43
// Matrix::Dense<S> / Matrix::Sparse<S> are the column-major DenseMatrix<S> and the CSC
// SparseMatrix<S> below (the storage Eigen uses for the reference's canonical types,
// matrix.hpp:39-44), with the subset of Eigen's interface the reference's API and tests use.
#pragma once

#include <algorithm>
#include <cmath>
#include <complex>
#include <limits>
#include <cstdint>
#include <deque>
#include <initializer_list>
#include <iomanip>
#include <ios>
#include <ostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

// Eigen interop (the reference's storage types, matrix.hpp:39-44): compiled only where Eigen's
// headers are on the include path.  This image has no Eigen, so the conversions below are
// compile-unverified here.
#if __has_include(<Eigen/Dense>) && __has_include(<Eigen/Sparse>)
#include <Eigen/Dense>
#include <Eigen/Sparse>
#define EIGSOL_HAVE_EIGEN 1
#else
#define EIGSOL_HAVE_EIGEN 0
#endif

namespace EigSol {

template <typename T>
struct is_complex_of_floating : std::false_type {};
template <typename Inner>
struct is_complex_of_floating<std::complex<Inner>> : std::bool_constant<std::is_floating_point_v<Inner>> {};

// The reference's concept (src/core/types.hpp:28-30), spelled the same way: a C++20 concept, so
// reference-style callers written as `template <EigSol::ScalarConcept S>` compile unchanged.
template <typename S>
concept ScalarConcept = std::is_floating_point_v<S> || is_complex_of_floating<S>::value;

// Scalars with a device path (gfx950 kernels compute in fp64 / complex fp64).
template <typename S>
inline constexpr bool DeviceScalar = std::is_same_v<S, double> || std::is_same_v<S, std::complex<double>>;

// float and std::complex<float> have native single-precision kernels for the power method (CSR
// and dense), plain products and the triangular-CSR shifted inverse (values stored and multiplied
// in single precision, norm/dot partials in double).  The other solvers (dense and general-sparse
// shifted inverse, solve_shifted on a non-triangular matrix, Hessenberg, QR) promote the matrix,
// vectors and shift to double on the host and round the results back (a deliberate deviation:
// fp64 arithmetic, at least as accurate as the reference's single precision).
// long double and std::complex<long double> (WideScalar) run on the device in double-double
// (EIGSOL_DD / EIGSOL_CDD, a 106-bit significand against the x87 format's 64): values cross the C
// ABI as exact {hi, lo} double pairs (to_wire below), so nothing is rounded on the way in; the
// results come back rounded to the nearest long double.
template <typename S>
inline constexpr bool PromotedScalar = std::is_same_v<S, float> || std::is_same_v<S, std::complex<float>>;
template <typename S>
inline constexpr bool WideScalar = std::is_same_v<S, long double> || std::is_same_v<S, std::complex<long double>>;
template <typename S>
inline constexpr bool DeviceCapable = DeviceScalar<S> || PromotedScalar<S> || WideScalar<S>;
template <typename S>
struct device_scalar { using type = S; };
template <>
struct device_scalar<float> { using type = double; };
template <>
struct device_scalar<std::complex<float>> { using type = std::complex<double>; };
template <typename S>
using device_scalar_t = typename device_scalar<S>::type;

template <typename S>
struct real_of { using type = S; };
template <typename R>
struct real_of<std::complex<R>> { using type = R; };

// ------------------------------------------------------------------ double-double wire format
// long double (x87: 64-bit significand) as the unevaluated sum of two doubles.  hi = v rounded to
// double, lo = v - hi (exact in long double, at most 11 significant bits): exact for every finite
// v inside the double exponent range; beyond it the conversion throws instead of rounding.
struct DDWire {
    double hi, lo;
};
struct CDDWire {
    DDWire re, im;
};
// Exact for the x87 80-bit format (64-bit significand: hi holds 53 bits, lo the remaining 11) as long
// as lo's bits stay above the subnormal grid, i.e. |v| >= ~2^-1010 (1e-304); below that the pair is
// the double-double nearest v.  A long double with a wider significand (IEEE binary128, e.g. aarch64)
// does not fit {hi, lo} and is refused at compile time.
static_assert(std::numeric_limits<long double>::digits == 64,
              "EigSol: the double-double wire format assumes the x87 80-bit long double");
inline DDWire to_wire(long double v) {
    const double hi = static_cast<double>(v);
    if (std::isfinite(v) && !std::isfinite(hi))
        throw std::runtime_error("EigSol: long double value outside the double-double range (|v| >= 1.8e308)");
    return DDWire{hi, static_cast<double>(v - static_cast<long double>(hi))};
}
inline CDDWire to_wire(const std::complex<long double>& v) { return CDDWire{to_wire(v.real()), to_wire(v.imag())}; }
inline long double from_wire(const DDWire& w) { return static_cast<long double>(w.hi) + static_cast<long double>(w.lo); }
inline std::complex<long double> from_wire(const CDDWire& w) {
    return std::complex<long double>(from_wire(w.re), from_wire(w.im));
}
template <typename S>
struct wire_of { using type = S; };
template <>
struct wire_of<long double> { using type = DDWire; };
template <>
struct wire_of<std::complex<long double>> { using type = CDDWire; };
template <typename S>
using wire_t = typename wire_of<S>::type;
template <typename S>
std::vector<wire_t<S>> to_wire_vec(const S* v, std::size_t n) {
    if constexpr (std::is_same_v<wire_t<S>, S>) {
        return std::vector<S>(v, v + n);   // the device types travel as they are
    } else {
        std::vector<wire_t<S>> w(n);
        for (std::size_t i = 0; i < n; ++i) w[i] = to_wire(v[i]);
        return w;
    }
}

// ------------------------------------------------------------------------------------- Vector
template <typename S>
class Vector {
    static_assert(ScalarConcept<S>, "EigSol::Vector: scalar must be floating point or complex");

public:
    using Scalar = S;
    Vector() = default;
    explicit Vector(std::size_t n) : d_(n, S(0)) {}
    Vector(std::initializer_list<S> v) : d_(v) {}
    explicit Vector(std::vector<S> v) : d_(std::move(v)) {}

    std::size_t size() const { return d_.size(); }
    S& operator()(std::size_t i) { return d_[i]; }
    const S& operator()(std::size_t i) const { return d_[i]; }
    S& operator[](std::size_t i) { return d_[i]; }
    const S& operator[](std::size_t i) const { return d_[i]; }
    S* data() { return d_.data(); }
    const S* data() const { return d_.data(); }
    auto begin() { return d_.begin(); }
    auto end() { return d_.end(); }
    auto begin() const { return d_.begin(); }
    auto end() const { return d_.end(); }
    void resize(std::size_t n) { d_.resize(n, S(0)); }
    const std::vector<S>& std() const { return d_; }

    typename real_of<S>::type squaredNorm() const {
        typename real_of<S>::type s = 0;
        for (const S& x : d_) s += std::norm(x);
        return s;
    }
    typename real_of<S>::type norm() const { return std::sqrt(squaredNorm()); }
    // x^H y (the first argument is conjugated, like Eigen's dot)
    S dot(const Vector& o) const {
        S s = S(0);
        for (std::size_t i = 0; i < d_.size(); ++i) s += conj_(d_[i]) * o.d_[i];
        return s;
    }
    Vector operator-() const {
        Vector r(*this);
        for (S& x : r.d_) x = -x;
        return r;
    }
    friend Vector operator-(const Vector& a, const Vector& b) {
        Vector r(a);
        for (std::size_t i = 0; i < r.size(); ++i) r.d_[i] -= b.d_[i];
        return r;
    }
    friend Vector operator*(const S& s, const Vector& a) {
        Vector r(a);
        for (S& x : r.d_) x *= s;
        return r;
    }
    // comma initialisation: v << 1, 2, 3;
    struct Filler {
        Vector* v;
        std::size_t i;
        Filler& operator,(const S& x) {
            (*v)(i++) = x;
            return *this;
        }
    };
    Filler operator<<(const S& x) {
        d_.at(0) = x;
        return Filler{this, 1};
    }

    // Row view for printing, as in the reference demo's `std::cout << v.transpose()` (main.cpp:38):
    // the entries on one line, separated by spaces, padded to a common width (Eigen's default
    // IOFormat for a row vector).
    struct RowView {
        const Vector* v;
        friend std::ostream& operator<<(std::ostream& os, const RowView& r) {
            std::vector<std::string> cells;
            std::size_t w = 0;
            for (const S& x : r.v->std()) {
                std::ostringstream c;
                c.precision(os.precision());
                c.flags(os.flags());
                c << x;
                cells.push_back(c.str());
                w = std::max(w, cells.back().size());
            }
            for (std::size_t i = 0; i < cells.size(); ++i)
                os << (i ? " " : "") << std::setw(static_cast<int>(w)) << cells[i];
            return os;
        }
    };
    RowView transpose() const { return RowView{this}; }
#if EIGSOL_HAVE_EIGEN
    // Vector<S> of the reference is Eigen::Matrix<S, Dynamic, 1> (types.hpp:33)
    operator Eigen::Matrix<S, Eigen::Dynamic, 1>() const {
        Eigen::Matrix<S, Eigen::Dynamic, 1> e(static_cast<Eigen::Index>(d_.size()));
        for (std::size_t i = 0; i < d_.size(); ++i) e(static_cast<Eigen::Index>(i)) = d_[i];
        return e;
    }
#endif

private:
    static S conj_(const S& x) {
        if constexpr (is_complex_of_floating<S>::value) return std::conj(x);
        else return x;
    }
    std::vector<S> d_;
};

// -------------------------------------------------------------------------------- DenseMatrix
// Column-major rows x cols (Eigen::Matrix<S, Dynamic, Dynamic> default storage).
template <typename S>
class DenseMatrix {
    static_assert(ScalarConcept<S>, "EigSol::DenseMatrix: scalar must be floating point or complex");

public:
    using Scalar = S;
    DenseMatrix() = default;
    DenseMatrix(std::int64_t rows, std::int64_t cols)
        : r_(rows), c_(cols), d_(static_cast<std::size_t>(std::max<std::int64_t>(rows * cols, 0)), S(0)) {}

    static DenseMatrix Zero(std::int64_t r, std::int64_t c) { return DenseMatrix(r, c); }
    static DenseMatrix Identity(std::int64_t r, std::int64_t c) {
        DenseMatrix m(r, c);
        for (std::int64_t i = 0; i < std::min(r, c); ++i) m(i, i) = S(1);
        return m;
    }
    std::int64_t rows() const { return r_; }
    std::int64_t cols() const { return c_; }
    std::int64_t size() const { return r_ * c_; }
    S& operator()(std::int64_t i, std::int64_t j) { return d_[static_cast<std::size_t>(i + j * r_)]; }
    const S& operator()(std::int64_t i, std::int64_t j) const { return d_[static_cast<std::size_t>(i + j * r_)]; }
    S* data() { return d_.data(); }
    const S* data() const { return d_.data(); }
    void setIdentity() { *this = Identity(r_, c_); }
    void setZero() { std::fill(d_.begin(), d_.end(), S(0)); }
    void resize(std::int64_t r, std::int64_t c) { *this = DenseMatrix(r, c); }

    DenseMatrix adjoint() const {
        DenseMatrix t(c_, r_);
        for (std::int64_t j = 0; j < c_; ++j)
            for (std::int64_t i = 0; i < r_; ++i) {
                if constexpr (is_complex_of_floating<S>::value) t(j, i) = std::conj((*this)(i, j));
                else t(j, i) = (*this)(i, j);
            }
        return t;
    }
    friend DenseMatrix operator*(const DenseMatrix& a, const DenseMatrix& b) {
        if (a.c_ != b.r_) throw std::runtime_error("DenseMatrix: product dimension mismatch");
        DenseMatrix m(a.r_, b.c_);
        for (std::int64_t j = 0; j < b.c_; ++j)
            for (std::int64_t k = 0; k < a.c_; ++k) {
                const S bk = b(k, j);
                for (std::int64_t i = 0; i < a.r_; ++i) m(i, j) += a(i, k) * bk;
            }
        return m;
    }
    friend Vector<S> operator*(const DenseMatrix& a, const Vector<S>& x) {
        if (static_cast<std::size_t>(a.c_) != x.size()) throw std::runtime_error("DenseMatrix: size mismatch");
        Vector<S> y(static_cast<std::size_t>(a.r_));
        for (std::int64_t j = 0; j < a.c_; ++j)
            for (std::int64_t i = 0; i < a.r_; ++i) y(i) += a(i, j) * x(j);
        return y;
    }
    friend DenseMatrix operator-(const DenseMatrix& a, const DenseMatrix& b) {
        DenseMatrix m(a);
        for (std::size_t i = 0; i < m.d_.size(); ++i) m.d_[i] -= b.d_[i];
        return m;
    }
    friend DenseMatrix operator*(const S& s, const DenseMatrix& a) {
        DenseMatrix m(a);
        for (S& x : m.d_) x *= s;
        return m;
    }
    // comma initialisation in row-major order: A << 1, 2, 3, 4;
    struct Filler {
        DenseMatrix* m;
        std::int64_t k;
        Filler& operator,(const S& x) {
            m->set_rowmajor(k++, x);
            return *this;
        }
    };
    Filler operator<<(const S& x) {
        set_rowmajor(0, x);
        return Filler{this, 1};
    }
    void setRandom();   // defined in solvers.hpp (uses the façade's documented generator)

#if EIGSOL_HAVE_EIGEN
    // Matrix::Dense<S> of the reference is Eigen::Matrix<S, Dynamic, Dynamic> (matrix.hpp:39-41):
    // both are column-major, so the conversion is one copy of the storage.
    template <typename Derived>
    static DenseMatrix fromEigen(const Eigen::MatrixBase<Derived>& m) {
        const Eigen::Matrix<S, Eigen::Dynamic, Eigen::Dynamic> e = m;   // evaluates any expression
        DenseMatrix d(e.rows(), e.cols());
        std::copy(e.data(), e.data() + e.size(), d.d_.begin());
        return d;
    }
    operator Eigen::Matrix<S, Eigen::Dynamic, Eigen::Dynamic>() const {
        Eigen::Matrix<S, Eigen::Dynamic, Eigen::Dynamic> e(r_, c_);
        std::copy(d_.begin(), d_.end(), e.data());
        return e;
    }
#endif

    // Eigen's default matrix print (main.cpp:117, :123-127): one row per line, columns separated
    // by a space and right-aligned to the widest entry.
    friend std::ostream& operator<<(std::ostream& os, const DenseMatrix& m) {
        std::vector<std::string> cells(m.d_.size());
        std::size_t w = 0;
        for (std::int64_t i = 0; i < m.r_; ++i)
            for (std::int64_t j = 0; j < m.c_; ++j) {
                std::ostringstream c;
                c.precision(os.precision());
                c.flags(os.flags());
                c << m(i, j);
                std::string& cell = cells[static_cast<std::size_t>(i + j * m.r_)];
                cell = c.str();
                w = std::max(w, cell.size());
            }
        for (std::int64_t i = 0; i < m.r_; ++i) {
            if (i) os << "\n";
            for (std::int64_t j = 0; j < m.c_; ++j)
                os << (j ? " " : "") << std::setw(static_cast<int>(w)) << cells[static_cast<std::size_t>(i + j * m.r_)];
        }
        return os;
    }

private:
    void set_rowmajor(std::int64_t k, const S& x) {
        if (k >= size()) throw std::runtime_error("DenseMatrix: too many coefficients in comma initializer");
        (*this)(k / c_, k % c_) = x;
    }
    std::int64_t r_ = 0, c_ = 0;
    std::vector<S> d_;
};

// ------------------------------------------------------------------------------- SparseMatrix
// Compressed sparse column with int32 indices (Eigen::SparseMatrix<S> = ColMajor, int).
// insert(r, c) builds an uncompressed triplet list (duplicates are summed on compression).
template <typename S>
class SparseMatrix {
    static_assert(ScalarConcept<S>, "EigSol::SparseMatrix: scalar must be floating point or complex");

public:
    using Scalar = S;
    using StorageIndex = std::int32_t;
    SparseMatrix() = default;
    SparseMatrix(std::int64_t rows, std::int64_t cols) : r_(rows), c_(cols), outer_(cols + 1, 0) {}

    std::int64_t rows() const { return r_; }
    std::int64_t cols() const { return c_; }
    std::int64_t nonZeros() const {
        compress();
        return static_cast<std::int64_t>(val_.size());
    }
    void reserve(std::int64_t) {}
    S& insert(std::int64_t r, std::int64_t c) {
        if (r < 0 || r >= r_ || c < 0 || c >= c_) throw std::out_of_range("SparseMatrix::insert: index out of range");
        pend_.push_back({r, c, S(0)});   // deque: the returned reference stays valid
        dirty_ = true;
        return pend_.back().v;
    }
    void makeCompressed() const { compress(); }
    void setIdentity() {
        pend_.clear();
        outer_.assign(c_ + 1, 0);
        inner_.clear();
        val_.clear();
        for (std::int64_t i = 0; i < std::min(r_, c_); ++i) insert(i, i) = S(1);
        compress();
    }
    S coeff(std::int64_t r, std::int64_t c) const {
        compress();
        for (std::int32_t e = outer_[c]; e < outer_[c + 1]; ++e)
            if (inner_[e] == r) return val_[e];
        return S(0);
    }
    S& coeffRef(std::int64_t r, std::int64_t c) {
        compress();
        for (std::int32_t e = outer_[c]; e < outer_[c + 1]; ++e)
            if (inner_[e] == r) return val_[e];
        return insert(r, c);
    }
    const std::int32_t* outerIndexPtr() const { compress(); return outer_.data(); }
    const std::int32_t* innerIndexPtr() const { compress(); return inner_.data(); }
    const S* valuePtr() const { compress(); return val_.data(); }

    static SparseMatrix fromDense(const DenseMatrix<S>& d) {
        SparseMatrix s(d.rows(), d.cols());
        for (std::int64_t j = 0; j < d.cols(); ++j)
            for (std::int64_t i = 0; i < d.rows(); ++i)
                if (d(i, j) != S(0)) s.insert(i, j) = d(i, j);
        s.compress();
        return s;
    }
#if EIGSOL_HAVE_EIGEN
    // Matrix::Sparse<S> of the reference is Eigen::SparseMatrix<S> (ColMajor, int; matrix.hpp:43-44)
    template <int Options, typename Index>
    static SparseMatrix fromEigen(const Eigen::SparseMatrix<S, Options, Index>& m) {
        SparseMatrix s(m.rows(), m.cols());
        for (Eigen::Index k = 0; k < m.outerSize(); ++k)
            for (typename Eigen::SparseMatrix<S, Options, Index>::InnerIterator it(m, k); it; ++it)
                s.insert(it.row(), it.col()) = it.value();
        s.compress();
        return s;
    }
#endif
    DenseMatrix<S> toDense() const {
        compress();
        DenseMatrix<S> d(r_, c_);
        for (std::int64_t j = 0; j < c_; ++j)
            for (std::int32_t e = outer_[j]; e < outer_[j + 1]; ++e) d(inner_[e], j) += val_[e];
        return d;
    }

private:
    struct Trip {
        std::int64_t r, c;
        S v;
    };
    void compress() const {
        if (!dirty_) return;
        std::vector<Trip> all;
        all.reserve(val_.size() + pend_.size());
        for (std::int64_t j = 0; j < c_; ++j)
            for (std::int32_t e = outer_[j]; e < outer_[j + 1]; ++e) all.push_back({inner_[e], j, val_[e]});
        for (const Trip& t : pend_) all.push_back(t);
        std::stable_sort(all.begin(), all.end(),
                         [](const Trip& a, const Trip& b) { return a.c != b.c ? a.c < b.c : a.r < b.r; });
        outer_.assign(c_ + 1, 0);
        inner_.clear();
        val_.clear();
        for (std::size_t k = 0; k < all.size(); ++k) {
            if (!inner_.empty() && k > 0 && all[k].c == all[k - 1].c && all[k].r == all[k - 1].r) {
                val_.back() += all[k].v;
                continue;
            }
            inner_.push_back(static_cast<std::int32_t>(all[k].r));
            val_.push_back(all[k].v);
            ++outer_[all[k].c + 1];
        }
        for (std::int64_t j = 0; j < c_; ++j) outer_[j + 1] += outer_[j];
        pend_.clear();
        dirty_ = false;
    }
    std::int64_t r_ = 0, c_ = 0;
    mutable std::vector<std::int32_t> outer_, inner_;
    mutable std::vector<S> val_;
    mutable std::deque<Trip> pend_;   // stable references for insert()
    mutable bool dirty_ = false;
};

// ------------------------------------------------------------------------------- options / results
template <typename S>
inline bool is_close_relative(S a, S b, double tol) {
    const double diff = std::abs(a - b);
    const double scale = 1.0 + std::abs(a);
    return diff <= tol * scale;
}

struct SolverOptions {
    int maxIterations = 1000;
    double tolerance = 1e-10;
};

template <typename S>
struct ShiftedSolverOptions : public SolverOptions {
    S shift;
    ShiftedSolverOptions() : SolverOptions(), shift(S(0)) {}
    ShiftedSolverOptions(S s) : SolverOptions(), shift(s) {}   // NOLINT: implicit like the reference
    ShiftedSolverOptions(S s, int maxIter, double tol) : SolverOptions(), shift(s) {
        maxIterations = maxIter;
        tolerance = tol;
    }
};

template <typename S>
struct EigenResult {
    S eigenvalue{};
    Vector<S> eigenvector;
    int iterations = 0;
    bool converged = false;
    EigenResult() = default;
    EigenResult(const S& lambda, const Vector<S>& vec, int iters, bool conv)
        : eigenvalue(lambda), eigenvector(vec), iterations(iters), converged(conv) {}
};

template <typename S>
struct QRResult {
    Vector<S> eigenvalues;
    int iterations = 0;
    bool converged = false;
    // Francis variant on a real matrix: the complex eigenvalues (eigenvalues = their real parts)
    std::vector<std::complex<double>> eigenvalues_complex;
    // Francis variant, long double / std::complex<long double>: the eigenvalues at extended
    // precision (double-double refined, rounded to long double); eigenvalues_complex holds them
    // rounded to double
    std::vector<std::complex<long double>> eigenvalues_complex_extended;
    QRResult() = default;
    QRResult(const Vector<S>& ev, int iters, bool conv) : eigenvalues(ev), iterations(iters), converged(conv) {}
};

}  // namespace EigSol

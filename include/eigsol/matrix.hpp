// EigSol drop-in façade — the type-erased Matrix (src/matrix/matrix.hpp:36-246,
// src/box/box.hpp:32-81, src/box/box_typed.hpp:27-79) and its device-resident mirror.
//
// Same contract as the reference: non-copyable and non-movable, built from a dense matrix, a
// sparse matrix or a row-major std::vector, queried with isDense() / scalar_type() / type(),
// unwrapped with cast<T>() (std::bad_cast on the wrong T).  New: the first solver call uploads the
// matrix to the device (eigsol_dense_create / eigsol_csr_create_from_csc) and the handle is
// cached for the Matrix's lifetime, so repeated solves do not re-upload.  Mutating the storage
// obtained through the non-const cast<T>() drops the cached device copy.
// Device-resident construction (the text reader's sparse path): a Matrix built from triplets owns
// a device CSR from the start (eigsol_csr_create_from_coo, no host CSC); the host Sparse<S> that
// cast<>() returns is materialised from the device copy the first time a caller asks for it.
#pragma once

#include <memory>
#include <typeinfo>
#include <vector>

#include "core.hpp"
#include "device.hpp"

namespace EigSol {

class Box {
public:
    Box() = default;
    Box(const Box&) = delete;
    Box& operator=(const Box&) = delete;
    virtual ~Box() = default;
    virtual const std::type_info& type() const noexcept = 0;
};

template <typename T>
class BoxTyped final : public Box {
public:
    explicit BoxTyped(T v) : v_(std::move(v)) {}
    const std::type_info& type() const noexcept override { return typeid(T); }
    T& get() { return v_; }
    const T& get() const { return v_; }

private:
    T v_;
};

// Entries of a sparse matrix as a reader collects them: position and value per entry, any order,
// repeated positions summed (in input order) like repeated Sparse<S>::insert()s.
template <typename S>
struct SparseTriplets {
    std::int64_t rows = 0, cols = 0;
    std::vector<std::int32_t> row, col;
    std::vector<S> val;
};

template <typename S>
inline constexpr bool has_device_storage_v =
    std::is_same_v<S, double> || std::is_same_v<S, float> || std::is_same_v<S, std::complex<double>> ||
    std::is_same_v<S, std::complex<float>> || WideScalar<S>;   // long double: double-double on the device

class Matrix {
public:
    template <typename S>
    using Dense = DenseMatrix<S>;
    template <typename S>
    using Sparse = SparseMatrix<S>;

    Matrix() = delete;
    Matrix(const Matrix&) = delete;
    Matrix& operator=(const Matrix&) = delete;
    Matrix(Matrix&&) = delete;
    Matrix& operator=(Matrix&&) = delete;

    template <ScalarConcept S>
    explicit Matrix(const DenseMatrix<S>& m)
        : dense_(true), scalar_(&typeid(S)), box_(std::make_unique<BoxTyped<DenseMatrix<S>>>(m)) {}

    template <ScalarConcept S>
    explicit Matrix(const SparseMatrix<S>& m)
        : dense_(false), scalar_(&typeid(S)), box_(std::make_unique<BoxTyped<SparseMatrix<S>>>(m)) {
        box_cast<SparseMatrix<S>>().makeCompressed();
    }

    // Triplets straight to the device.  A process without a usable device takes
    // the host route (insert + compress); the solvers then report the missing device on first use,
    // as for any other Matrix.
    template <ScalarConcept S>
    explicit Matrix(SparseTriplets<S>&& t) : dense_(false), scalar_(&typeid(S)), rows_(t.rows), cols_(t.cols) {
        if constexpr (has_device_storage_v<S>) {
            try {
                const std::int64_t nnz = static_cast<std::int64_t>(t.val.size());
                if constexpr (WideScalar<S>) {   // exact double-double pairs
                    const std::vector<wire_t<S>> w = to_wire_vec(t.val.data(), t.val.size());
                    dev_ = detail::DeviceMatrix::coo(detail::dtype_of<S>(), t.rows, t.cols, nnz, t.row.data(),
                                                     t.col.data(), w.data());
                } else {
                    dev_ = detail::DeviceMatrix::coo(detail::dtype_of<S>(), t.rows, t.cols, nnz, t.row.data(),
                                                     t.col.data(), t.val.data());
                }
                type_ = &typeid(SparseMatrix<S>);
                materialise_ = &Matrix::host_from_device<S>;
                return;
            } catch (const std::runtime_error&) {
                dev_.reset();
            }
        }
        SparseMatrix<S> s(t.rows, t.cols);
        for (std::size_t k = 0; k < t.val.size(); ++k) s.insert(t.row[k], t.col[k]) = t.val[k];
        s.makeCompressed();
        box_ = std::make_unique<BoxTyped<SparseMatrix<S>>>(std::move(s));
    }

#if EIGSOL_HAVE_EIGEN
    // Eigen inputs, as the reference's constructors take them (matrix.hpp:70-76, :89-94): any dense
    // expression is evaluated into column-major storage, a sparse matrix is copied entry by entry.
    template <typename Derived>
        requires ScalarConcept<typename Derived::Scalar>
    explicit Matrix(const Eigen::MatrixBase<Derived>& m)
        : Matrix(DenseMatrix<typename Derived::Scalar>::fromEigen(m)) {}
    template <ScalarConcept S, int Options, typename Index>
    explicit Matrix(const Eigen::SparseMatrix<S, Options, Index>& m) : Matrix(SparseMatrix<S>::fromEigen(m)) {}
#endif

    // row-major data (matrix.hpp:207-232)
    template <ScalarConcept S>
    Matrix(const std::vector<S>& data, std::size_t rows, std::size_t cols) : dense_(true), scalar_(&typeid(S)) {
        if (rows * cols != data.size()) throw std::runtime_error("Matrix: size mismatch in vector constructor");
        DenseMatrix<S> m(static_cast<std::int64_t>(rows), static_cast<std::int64_t>(cols));
        for (std::size_t i = 0; i < data.size(); ++i)
            m(static_cast<std::int64_t>(i / cols), static_cast<std::int64_t>(i % cols)) = data[i];
        box_ = std::make_unique<BoxTyped<DenseMatrix<S>>>(std::move(m));
    }

    bool isDense() const { return dense_; }
    const std::type_info& scalar_type() const { return *scalar_; }
    const std::type_info& type() const { return box_ ? box_->type() : *type_; }
    // true while the only copy of the entries is the device one (the host storage has not been
    // asked for yet)
    bool deviceResident() const { return !box_; }

    template <typename T>
    T& cast() {
        check<T>();
        materialise();
        dev_.reset();   // the caller may modify the storage
        dev64_.reset();
        return box_cast<T>();
    }
    template <typename T>
    const T& cast() const {
        check<T>();
        materialise();
        return static_cast<const BoxTyped<T>*>(box_.get())->get();
    }

    std::int64_t rows() const { return box_ ? visit([](const auto& m) { return m.rows(); }) : rows_; }
    std::int64_t cols() const { return box_ ? visit([](const auto& m) { return m.cols(); }) : cols_; }

    // Device mirror (created on first use by the solvers) in the storage's own precision
    // (double, float, long double and their complex types all have device storage).
    template <typename S>
    const detail::DeviceMatrix& device() const {
        if (!dev_) dev_ = upload<S, S>();
        return *dev_;
    }
    // fp64 mirror for the solvers without single-precision kernels (float / complex<float>
    // storage promoted on upload; the same mirror as device<S>() for double scalars).
    template <typename S>
    const detail::DeviceMatrix& device_fp64() const {
        using D = device_scalar_t<S>;
        if constexpr (std::is_same_v<D, S>) {
            return device<S>();
        } else {
            if (!dev64_) dev64_ = upload<S, D>();
            return *dev64_;
        }
    }

private:
    template <typename T>
    void check() const {
        if (type() != typeid(T)) throw std::bad_cast{};
    }
    void materialise() const {
        if (!box_) box_ = materialise_(*dev_);
    }
    // host Sparse<S> (CSC) from the device CSR: download, then a counting-sort transpose
    template <typename S>
    static std::unique_ptr<Box> host_from_device(const detail::DeviceMatrix& d) {
        std::int64_t r = 0, c = 0, nnz = 0;
        detail::check(eigsol_csr_info(d.csr(), &r, &c, &nnz, nullptr), "eigsol_csr_info");
        std::vector<std::int32_t> rp(r + 1), ci(nnz);
        std::vector<wire_t<S>> v(nnz);
        detail::check(eigsol_csr_download(d.csr(), rp.data(), ci.data(), v.data()), "eigsol_csr_download");
        SparseMatrix<S> s(r, c);
        for (std::int64_t i = 0; i < r; ++i)
            for (std::int32_t e = rp[i]; e < rp[i + 1]; ++e) {
                if constexpr (WideScalar<S>) s.insert(i, ci[e]) = from_wire(v[e]);
                else s.insert(i, ci[e]) = v[e];
            }
        s.makeCompressed();
        return std::make_unique<BoxTyped<SparseMatrix<S>>>(std::move(s));
    }
    template <typename T>
    T& box_cast() {
        return static_cast<BoxTyped<T>*>(box_.get())->get();
    }
    template <typename F>
    std::int64_t visit(F f) const {
        const std::type_info& t = box_->type();
        if (t == typeid(DenseMatrix<double>)) return f(cast<DenseMatrix<double>>());
        if (t == typeid(DenseMatrix<std::complex<double>>)) return f(cast<DenseMatrix<std::complex<double>>>());
        if (t == typeid(SparseMatrix<double>)) return f(cast<SparseMatrix<double>>());
        if (t == typeid(SparseMatrix<std::complex<double>>)) return f(cast<SparseMatrix<std::complex<double>>>());
        if (t == typeid(DenseMatrix<float>)) return f(cast<DenseMatrix<float>>());
        if (t == typeid(SparseMatrix<float>)) return f(cast<SparseMatrix<float>>());
        if (t == typeid(DenseMatrix<std::complex<float>>)) return f(cast<DenseMatrix<std::complex<float>>>());
        if (t == typeid(SparseMatrix<std::complex<float>>)) return f(cast<SparseMatrix<std::complex<float>>>());
        if (t == typeid(DenseMatrix<long double>)) return f(cast<DenseMatrix<long double>>());
        if (t == typeid(SparseMatrix<long double>)) return f(cast<SparseMatrix<long double>>());
        if (t == typeid(DenseMatrix<std::complex<long double>>)) return f(cast<DenseMatrix<std::complex<long double>>>());
        if (t == typeid(SparseMatrix<std::complex<long double>>))
            return f(cast<SparseMatrix<std::complex<long double>>>());
        return -1;
    }

    template <typename S, typename D>
    std::shared_ptr<detail::DeviceMatrix> upload() const {
        materialise();
        if constexpr (WideScalar<S>) {   // long double: exact double-double pairs (core.hpp, to_wire)
            if (dense_) {
                const auto& d = cast<DenseMatrix<S>>();
                const auto w = to_wire_vec(d.data(), static_cast<std::size_t>(d.size()));
                return detail::DeviceMatrix::dense(detail::dtype_of<S>(), d.rows(), d.cols(), w.data());
            }
            const auto& sm = cast<SparseMatrix<S>>();
            const auto w = to_wire_vec(sm.valuePtr(), static_cast<std::size_t>(sm.nonZeros()));
            return detail::DeviceMatrix::csc(detail::dtype_of<S>(), sm.rows(), sm.cols(), sm.nonZeros(),
                                             sm.outerIndexPtr(), sm.innerIndexPtr(), w.data());
        }
        if (dense_) {
            const auto& d = cast<DenseMatrix<S>>();
            if constexpr (std::is_same_v<D, S>) {
                return detail::DeviceMatrix::dense(detail::dtype_of<D>(), d.rows(), d.cols(), d.data());
            } else {
                std::vector<D> w(d.data(), d.data() + d.size());
                return detail::DeviceMatrix::dense(detail::dtype_of<D>(), d.rows(), d.cols(), w.data());
            }
        }
        const auto& s = cast<SparseMatrix<S>>();
        if constexpr (std::is_same_v<D, S>) {
            return detail::DeviceMatrix::csc(detail::dtype_of<D>(), s.rows(), s.cols(), s.nonZeros(),
                                             s.outerIndexPtr(), s.innerIndexPtr(), s.valuePtr());
        } else {
            std::vector<D> w(s.valuePtr(), s.valuePtr() + s.nonZeros());
            return detail::DeviceMatrix::csc(detail::dtype_of<D>(), s.rows(), s.cols(), s.nonZeros(),
                                             s.outerIndexPtr(), s.innerIndexPtr(), w.data());
        }
    }

    bool dense_;
    const std::type_info* scalar_;
    const std::type_info* type_ = nullptr;   // storage type while box_ is empty
    std::int64_t rows_ = 0, cols_ = 0;
    mutable std::unique_ptr<Box> box_;        // empty until a device-resident matrix is cast
    std::unique_ptr<Box> (*materialise_)(const detail::DeviceMatrix&) = nullptr;
    mutable std::shared_ptr<detail::DeviceMatrix> dev_;
    mutable std::shared_ptr<detail::DeviceMatrix> dev64_;
};

}  // namespace EigSol

// C++ façade tests: the reference's GoogleTest cases (test/*.cpp) restated against
// <eigsol/eigsol.hpp> with a minimal harness (GoogleTest is not available in this image).
// Each TEST names the reference case it restates.  Needs a gfx950 device at run time.
#include <eigsol/eigsol.hpp>

#include <algorithm>
#include <array>
#include <cstdio>
#include <functional>
#include <string>
#include <type_traits>
#include <vector>

static int g_fail = 0, g_checks = 0;
static std::vector<std::pair<std::string, std::function<void()>>>& registry() {
    static std::vector<std::pair<std::string, std::function<void()>>> r;
    return r;
}
struct Reg {
    Reg(const char* n, std::function<void()> f) { registry().emplace_back(n, std::move(f)); }
};
#define TEST(suite, name)                                   \
    static void suite##_##name();                           \
    static Reg reg_##suite##_##name(#suite "." #name, suite##_##name); \
    static void suite##_##name()
#define EXPECT_TRUE(c)                                                                   \
    do {                                                                                 \
        ++g_checks;                                                                      \
        if (!(c)) { ++g_fail; std::printf("  FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); } \
    } while (0)
#define EXPECT_FALSE(c) EXPECT_TRUE(!(c))
#define EXPECT_EQ(a, b) EXPECT_TRUE((a) == (b))
#define EXPECT_GT(a, b) EXPECT_TRUE((a) > (b))
#define EXPECT_GE(a, b) EXPECT_TRUE((a) >= (b))
#define EXPECT_LE(a, b) EXPECT_TRUE((a) <= (b))
#define EXPECT_NEAR(a, b, t) EXPECT_TRUE(std::abs((a) - (b)) <= (t))
#define EXPECT_THROW(stmt, ex)                      \
    do {                                            \
        bool thrown_ = false;                       \
        try { stmt; } catch (const ex&) { thrown_ = true; } catch (...) {} \
        EXPECT_TRUE(thrown_);                       \
    } while (0)
#define EXPECT_NO_THROW(stmt)                       \
    do {                                            \
        bool ok_ = true;                            \
        try { stmt; } catch (...) { ok_ = false; }  \
        EXPECT_TRUE(ok_);                           \
    } while (0)

using DenseMat = EigSol::Matrix::Dense<double>;
using SparseMat = EigSol::Matrix::Sparse<double>;
using C = std::complex<double>;

static_assert(!std::is_default_constructible_v<EigSol::Matrix>);
static_assert(!std::is_copy_constructible_v<EigSol::Matrix>);
static_assert(!std::is_copy_assignable_v<EigSol::Matrix>);
static_assert(!std::is_move_constructible_v<EigSol::Matrix>);
static_assert(!std::is_move_assignable_v<EigSol::Matrix>);

// ---------------------------------------------------------------- matrix_wrapper_test.cpp
TEST(MatrixWrapperTest, ConstructFromDense) {
    DenseMat A(2, 2);
    A << 1.0, 2.0, 3.0, 4.0;
    EigSol::Matrix M(A);
    EXPECT_TRUE(M.isDense());
    EXPECT_TRUE(M.scalar_type() == typeid(double));
    DenseMat& B = M.cast<DenseMat>();
    EXPECT_EQ(B(0, 0), 1.0);
    EXPECT_EQ(B(1, 1), 4.0);
}
TEST(MatrixWrapperTest, ConstructFromSparse) {
    SparseMat S(3, 3);
    S.insert(0, 0) = 5.0;
    S.insert(1, 2) = 7.0;
    EigSol::Matrix M(S);
    EXPECT_FALSE(M.isDense());
    SparseMat& T = M.cast<SparseMat>();
    EXPECT_EQ(T.coeff(0, 0), 5.0);
    EXPECT_EQ(T.coeff(1, 2), 7.0);
}
TEST(MatrixWrapperTest, ConstructFromStdVector) {
    std::vector<double> v = {1, 2, 3, 4};
    EigSol::Matrix M(v, 2, 2);
    DenseMat& A = M.cast<DenseMat>();
    EXPECT_EQ(A(0, 1), 2.0);
    EXPECT_EQ(A(1, 0), 3.0);
    EXPECT_THROW(EigSol::Matrix(v, 3, 2), std::runtime_error);
}
TEST(MatrixWrapperTest, CastAndTypeQueries) {
    EigSol::Matrix M(DenseMat::Identity(3, 3));
    EXPECT_THROW(M.cast<SparseMat>(), std::bad_cast);
    EXPECT_NO_THROW(M.cast<DenseMat>());
    EXPECT_TRUE(M.type() == typeid(DenseMat));
}

// ---------------------------------------------------------------- power_method_test.cpp
TEST(PowerMethodTest, DenseSimpleMatrix) {
    DenseMat A(2, 2);
    A << 2.0, 0.0, 0.0, 1.0;
    EigSol::Matrix M(A);
    EigSol::SolverOptions opts;
    opts.maxIterations = 1000;
    opts.tolerance = 1e-10;
    auto r = EigSol::powerMethod<double>(M, opts);
    EXPECT_TRUE(r.converged);
    EXPECT_GT(r.iterations, 0);
    EXPECT_TRUE(EigSol::is_close_relative(2.0, r.eigenvalue, 1e-5));
    auto lhs = A * r.eigenvector;
    for (std::size_t i = 0; i < lhs.size(); ++i)
        EXPECT_TRUE(EigSol::is_close_relative(lhs(i), r.eigenvalue * r.eigenvector(i), 1e-5));
}
TEST(PowerMethodTest, SparseMatrix) {
    DenseMat Ad(2, 2);
    Ad << 3.0, 1.0, 0.0, 2.0;
    EigSol::Matrix M(SparseMat::fromDense(Ad));
    EigSol::SolverOptions opts;
    opts.tolerance = 1e-8;
    auto r = EigSol::powerMethod<double>(M, opts);
    EXPECT_TRUE(r.converged);
    EXPECT_TRUE(EigSol::is_close_relative(3.0, r.eigenvalue, 1e-6));
}
TEST(PowerMethodTest, ErrorsAndFewIterations) {
    EigSol::Matrix N(DenseMat(2, 3));
    EXPECT_THROW(EigSol::powerMethod<double>(N), std::runtime_error);
    EigSol::Matrix Z(DenseMat(0, 0));
    EXPECT_THROW(EigSol::powerMethod<double>(Z), std::runtime_error);
    EXPECT_THROW(EigSol::powerMethod<C>(EigSol::Matrix(DenseMat::Identity(2, 2))), std::runtime_error);
    DenseMat A(2, 2);
    A << 5.0, 1.0, 1.0, 4.0;
    EigSol::Matrix M(A);
    EigSol::SolverOptions opts;
    opts.maxIterations = 1;
    opts.tolerance = 1e-12;
    auto r = EigSol::powerMethod<double>(M, opts);
    EXPECT_EQ(r.iterations, opts.maxIterations);
    try {
        EigSol::powerMethod<double>(N);
    } catch (const std::runtime_error& e) {
        EXPECT_EQ(std::string(e.what()), std::string("powerMethod: matrix must be square"));
    }
}
TEST(PowerMethodTest, DataFileAsDouble) {
    // main.cpp reads data/A.txt (complex layout) as double: dominant eigenvalue 1 + sqrt(15)
    EigSol::Matrix A = EigSol::readMatrixFromFile<double>(EIGSOL_TEST_DATA "/A.txt");
    EigSol::SolverOptions opts;
    auto r = EigSol::powerMethod<double>(A, opts);
    EXPECT_TRUE(r.converged);
    EXPECT_NEAR(r.eigenvalue, 1.0 + std::sqrt(15.0), 1e-8);
    EXPECT_THROW(EigSol::readMatrixFromFile<double>(EIGSOL_TEST_DATA "/B.txt"), std::runtime_error);
    EigSol::Matrix B = EigSol::readMatrixFromFile<C>(EIGSOL_TEST_DATA "/B.txt");
    EXPECT_FALSE(B.isDense());
    EigSol::ShiftedSolverOptions<C> so(C(2.3, 0.0));
    auto rs = EigSol::shiftedInversePowerMethod<C>(B, so);
    EXPECT_TRUE(rs.converged);
    EXPECT_NEAR(std::abs(rs.eigenvalue - C(3, 2)), 0.0, 1e-6);
}

TEST(ReaderTest, SparseFileStraightToDevice) {
    // triplets in file order, unsorted, with a repeated position: the device CSR is built from
    // them directly; the host Sparse<S> appears only when cast<>() asks for it
    const char* path = "/tmp/eigsol_reader_coo.txt";
    {
        std::FILE* f = std::fopen(path, "w");
        std::fputs("sparse\n4 4\n7\n3 3 1.0\n0 1 2.0\n0 0 4.0\n2 2 0.5\n0 1 0.25\n1 0 1.0\n1 1 3.0\n", f);
        std::fclose(f);
    }
    EigSol::Matrix M = EigSol::readMatrixFromFile<double>(path);
    EXPECT_FALSE(M.isDense());
    EXPECT_TRUE(M.deviceResident());
    EXPECT_TRUE(M.type() == typeid(SparseMat));
    EXPECT_EQ(M.rows(), 4);
    EXPECT_EQ(M.cols(), 4);
    EigSol::SolverOptions opts;
    opts.tolerance = 1e-12;
    EigSol::set_random_seed(11);
    auto r = EigSol::powerMethod<double>(M, opts);
    EXPECT_TRUE(M.deviceResident());
    EXPECT_TRUE(r.converged);
    const SparseMat& S = M.cast<SparseMat>();
    EXPECT_FALSE(M.deviceResident());
    EXPECT_EQ(S.nonZeros(), 6);
    EXPECT_EQ(S.coeff(0, 1), 2.25);
    EXPECT_EQ(S.coeff(1, 0), 1.0);
    EXPECT_NEAR(r.eigenvalue, (7.0 + std::sqrt(10.0)) / 2, 1e-9);
    EXPECT_EQ(S.coeff(3, 3), 1.0);
    EXPECT_EQ(S.coeff(2, 3), 0.0);
    EigSol::set_random_seed(11);
    auto r2 = EigSol::powerMethod<double>(M, opts);   // re-uploaded from the host copy: same run
    EXPECT_EQ(r2.iterations, r.iterations);
    EXPECT_EQ(r2.eigenvalue, r.eigenvalue);
    EXPECT_THROW(M.cast<DenseMat>(), std::bad_cast);
    EigSol::set_random_seed(0x5eed5eedULL);   // leave the default sequence to later cases
    std::remove(path);
}

// ---------------------------------------------------------------- shifted_inverse_power_method_test.cpp
TEST(ShiftedInversePowerMethodTest, DenseShifts) {
    DenseMat A(2, 2);
    A << 2.0, 0.0, 0.0, 5.0;
    EigSol::Matrix M(A);
    for (double sh : {1.9, 4.9}) {
        EigSol::ShiftedSolverOptions<double> opts;
        opts.shift = sh;
        opts.maxIterations = 1000;
        opts.tolerance = 1e-10;
        auto r = EigSol::shiftedInversePowerMethod<double>(M, opts);
        EXPECT_TRUE(r.converged);
        EXPECT_GT(r.iterations, 0);
        EXPECT_TRUE(EigSol::is_close_relative(sh < 3 ? 2.0 : 5.0, r.eigenvalue, 1e-5));
    }
}
TEST(ShiftedInversePowerMethodTest, SparseMatrixAndErrors) {
    DenseMat Ad = DenseMat::Zero(3, 3);
    Ad(0, 0) = 1.0;
    Ad(1, 1) = 3.0;
    Ad(2, 2) = 10.0;
    EigSol::Matrix M(SparseMat::fromDense(Ad));
    EigSol::ShiftedSolverOptions<double> opts(2.9, 1000, 1e-8);
    auto r = EigSol::shiftedInversePowerMethod<double>(M, opts);
    EXPECT_TRUE(r.converged);
    EXPECT_TRUE(EigSol::is_close_relative(3.0, r.eigenvalue, 1e-5));
    EXPECT_THROW(EigSol::shiftedInversePowerMethod<double>(EigSol::Matrix(DenseMat(2, 3)), opts), std::runtime_error);
    EXPECT_THROW(EigSol::shiftedInversePowerMethod<double>(EigSol::Matrix(DenseMat(0, 0)), opts), std::runtime_error);
    DenseMat B(2, 2);
    B << 5.0, 1.0, 1.0, 4.0;
    EigSol::ShiftedSolverOptions<double> o1(4.0, 1, 1e-12);
    EXPECT_EQ(EigSol::shiftedInversePowerMethod<double>(EigSol::Matrix(B), o1).iterations, 1);
}

// ---------------------------------------------------------------- solve_shifted_test.cpp
TEST(SolveShiftedLinearSystem, DenseAndSparse) {
    EigSol::Vector<double> b(3);
    b << 1.0, -2.0, 3.0;
    auto x = EigSol::solve_shifted<double>(EigSol::Matrix(DenseMat::Identity(3, 3)), 2.0, b);
    for (int i = 0; i < 3; ++i) EXPECT_NEAR(x(i), -b(i), 1e-12);
    SparseMat S(3, 3);
    S.setIdentity();
    auto xs = EigSol::solve_shifted<double>(EigSol::Matrix(S), 2.0, b);
    for (int i = 0; i < 3; ++i) EXPECT_NEAR(xs(i), -b(i), 1e-12);
    DenseMat A(2, 2);
    A << 3.0, 1.0, 0.0, 4.0;
    EigSol::Vector<double> b2(2);
    b2 << 2.0, -1.0;
    auto x2 = EigSol::solve_shifted<double>(EigSol::Matrix(A), 1.5, b2);
    DenseMat Ms = A - 1.5 * DenseMat::Identity(2, 2);
    auto res = Ms * x2 - b2;
    EXPECT_NEAR(res.norm(), 0.0, 1e-10);
}
TEST(SolveShiftedLinearSystem, ComplexAndErrors) {
    EigSol::Matrix::Dense<C> A(2, 2);
    A << C(1, 1), C(2, -1), C(0.5, 0), C(3, 2);
    const C lam(0.7, -0.3);
    EigSol::Vector<C> b(2);
    b << C(1, 0), C(-2, 1);
    auto x = EigSol::solve_shifted<C>(EigSol::Matrix(A), lam, b);
    auto M = A - lam * EigSol::Matrix::Dense<C>::Identity(2, 2);
    EXPECT_NEAR((M * x - b).norm(), 0.0, 1e-10);
    EigSol::Vector<double> ones(2);
    ones << 1.0, 1.0;
    DenseMat R(2, 3);
    EXPECT_THROW(EigSol::solve_shifted<double>(EigSol::Matrix(R), 1.0, ones), std::runtime_error);
    SparseMat S23(2, 3);
    S23.insert(0, 0) = 1.0;
    S23.insert(1, 2) = 2.0;
    EXPECT_THROW(EigSol::solve_shifted<double>(EigSol::Matrix(S23), 0.5, ones), std::runtime_error);
    EXPECT_THROW(EigSol::solve_shifted<double>(EigSol::Matrix(DenseMat::Identity(3, 3)), 1.0, ones), std::runtime_error);
    DenseMat Rr(2, 2);
    Rr << 1.0, 2.0, 3.0, 4.0;
    EigSol::Vector<C> bc(2);
    EXPECT_THROW(EigSol::solve_shifted<C>(EigSol::Matrix(Rr), C(1, 0), bc), std::runtime_error);
}

// ---------------------------------------------------------------- qr_algorithms_test.cpp
TEST(ToHessenbergDenseTest, RealAndComplex) {
    DenseMat A(3, 3);
    A << 4.0, 1.0, -2.0, 1.0, 3.0, 0.0, 2.0, 1.0, 1.0;
    DenseMat H = EigSol::to_hessenberg_dense<double>(A);
    EXPECT_NEAR(H(2, 0), 0.0, 1e-12);
    EXPECT_NEAR(H(1, 0), -2.2360679774997902, 1e-12);
    EXPECT_NEAR(H(0, 1), 1.3416407864998736, 1e-12);
    DenseMat H2 = EigSol::to_hessenberg<double>(EigSol::Matrix(A));
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) EXPECT_NEAR(H(i, j), H2(i, j), 1e-10);
    EigSol::Matrix::Dense<C> Ac(3, 3);
    Ac << C(4, 1), C(1, 0), C(-2, 2), C(1, 0), C(3, -1), C(0, 1), C(2, 0), C(1, 2), C(1, 0);
    auto Hc = EigSol::to_hessenberg_dense<C>(Ac);
    EXPECT_NEAR(std::abs(Hc(2, 0)), 0.0, 1e-12);
    EXPECT_THROW(EigSol::to_hessenberg_dense<double>(DenseMat(2, 3)), std::runtime_error);
    SparseMat S(2, 2);
    S.setIdentity();
    EXPECT_THROW(EigSol::to_hessenberg<double>(EigSol::Matrix(S)), std::runtime_error);
}
TEST(QRDecomposeDenseTest, RealRectangularAndComplex) {
    DenseMat A(3, 2);
    A << 1.0, 2.0, 3.0, 4.0, 5.0, 6.0;
    DenseMat Q, R;
    EigSol::qr_decompose_dense<double>(A, Q, R);
    EXPECT_EQ(Q.rows(), 3);
    EXPECT_EQ(Q.cols(), 3);
    EXPECT_EQ(R.rows(), 3);
    EXPECT_EQ(R.cols(), 2);
    DenseMat QR = Q * R;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 2; ++j) EXPECT_NEAR(QR(i, j), A(i, j), 1e-10);
    DenseMat QtQ = Q.adjoint() * Q;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) EXPECT_NEAR(QtQ(i, j), i == j ? 1.0 : 0.0, 1e-10);
    EXPECT_NEAR(R(0, 0), -5.916079783099616, 1e-12);
    auto [Q2, R2] = EigSol::qr_decompose<double>(EigSol::Matrix(A));
    EXPECT_NEAR(Q2(2, 0), Q(2, 0), 1e-12);
    EigSol::Matrix::Dense<C> B(2, 2);
    B << C(1, 1), C(2, -1), C(0.5, 0), C(3, 2);
    EigSol::Matrix::Dense<C> Qc, Rc;
    EigSol::qr_decompose_dense<C>(B, Qc, Rc);
    auto QRc = Qc * Rc;
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) EXPECT_NEAR(std::abs(QRc(i, j) - B(i, j)), 0.0, 1e-10);
    EXPECT_NEAR(std::abs(Rc(1, 0)), 0.0, 1e-10);
    DenseMat E0(0, 0), q, r;
    EXPECT_THROW(EigSol::qr_decompose_dense<double>(E0, q, r), std::runtime_error);
}
TEST(QREigenvaluesDenseTest, Real2x2BothVariantsAndComplex) {
    DenseMat A(2, 2);
    A << 2.0, 1.0, 1.0, 2.0;
    EigSol::SolverOptions opts;
    opts.maxIterations = 1000;
    opts.tolerance = 1e-12;
    for (auto v : {EigSol::QRVariant::Francis, EigSol::QRVariant::Unshifted}) {
        auto r = EigSol::qr_eigenvalues_dense<double>(A, opts, v);
        EXPECT_TRUE(r.converged);
        EXPECT_EQ(r.eigenvalues.size(), 2u);
        EXPECT_GE(r.iterations, 1);
        EXPECT_LE(r.iterations, opts.maxIterations);
        const double hi = std::max(r.eigenvalues(0), r.eigenvalues(1));
        const double lo = std::min(r.eigenvalues(0), r.eigenvalues(1));
        EXPECT_NEAR(hi, 3.0, 1e-8);
        EXPECT_NEAR(lo, 1.0, 1e-8);
    }
    // reference algorithm: 25 iterations at 1e-12 (golden)
    EXPECT_EQ(EigSol::qr_eigenvalues_dense<double>(A, opts, EigSol::QRVariant::Unshifted).iterations, 25);
    // the reference-signature call runs the default (Francis) path; the reference test's checks
    // (qr_algorithms_test.cpp:253-266) hold for it
    auto r2 = EigSol::qr_eigenvalues<double>(EigSol::Matrix(A), opts);
    EXPECT_EQ(r2.eigenvalues.size(), 2u);
    EXPECT_GE(r2.iterations, 1);
    EXPECT_LE(r2.iterations, opts.maxIterations);
    EXPECT_TRUE(r2.converged);
    EXPECT_NEAR(std::max(r2.eigenvalues(0), r2.eigenvalues(1)), 3.0, 1e-8);
    EXPECT_EQ(EigSol::qr_eigenvalues<double>(EigSol::Matrix(A), opts, EigSol::QRVariant::Unshifted).iterations, 25);
    EigSol::Matrix::Dense<C> Ac(2, 2);
    Ac << C(2, 0), C(1, 0), C(1, 0), C(2, 0);
    auto rc = EigSol::qr_eigenvalues_dense<C>(Ac, opts);
    EXPECT_TRUE(rc.converged);
    const double hc = std::max(rc.eigenvalues(0).real(), rc.eigenvalues(1).real());
    EXPECT_NEAR(hc, 3.0, 1e-8);
    EXPECT_THROW(EigSol::qr_eigenvalues_dense<double>(DenseMat(2, 3), opts), std::runtime_error);
    // complex-conjugate pair reported through eigenvalues_complex
    DenseMat Rot(2, 2);
    Rot << 0.0, -1.0, 1.0, 0.0;
    auto rr = EigSol::qr_eigenvalues_dense<double>(Rot, opts, EigSol::QRVariant::Francis);
    EXPECT_TRUE(rr.converged);
    EXPECT_NEAR(std::abs(std::abs(rr.eigenvalues_complex[0].imag()) - 1.0), 0.0, 1e-12);
}

// ---------------------------------------------------------------- single precision (promoted)
// ScalarConcept admits float and std::complex<float> (types.hpp:28-30): they run on the fp64
// kernels (promoted on the host, rounded back).
TEST(SinglePrecision, PowerShiftedSolveAndQR) {
    EigSol::Matrix::Dense<float> A(2, 2);
    A << 2.0f, 0.0f, 0.0f, 1.0f;
    EigSol::Matrix M(A);
    auto r = EigSol::powerMethod<float>(M, EigSol::SolverOptions{});
    EXPECT_TRUE(r.converged);
    EXPECT_NEAR(r.eigenvalue, 2.0f, 1e-6f);
    EXPECT_EQ(r.eigenvector.size(), 2u);
    EigSol::ShiftedSolverOptions<float> so;
    so.shift = 0.9f;
    auto rs = EigSol::shiftedInversePowerMethod<float>(M, so);
    EXPECT_NEAR(rs.eigenvalue, 1.0f, 1e-6f);
    EigSol::Vector<float> b(2);
    b << 4.0f, 2.0f;
    auto x = EigSol::solve_shifted<float>(M, 0.5f, b);   // (A - 0.5 I) x = b
    EXPECT_NEAR(x(0), 4.0f / 1.5f, 1e-6f);
    EXPECT_NEAR(x(1), 4.0f, 1e-6f);
    EigSol::Matrix::Dense<float> B(2, 2);
    B << 2.0f, 1.0f, 1.0f, 2.0f;
    auto q = EigSol::qr_eigenvalues<float>(EigSol::Matrix(B), EigSol::SolverOptions{});
    EXPECT_TRUE(q.converged);
    std::array<float, 2> ev{q.eigenvalues(0), q.eigenvalues(1)};
    std::sort(ev.begin(), ev.end());
    EXPECT_NEAR(ev[0], 1.0f, 1e-5f);
    EXPECT_NEAR(ev[1], 3.0f, 1e-5f);
    auto H = EigSol::to_hessenberg<float>(EigSol::Matrix(B));
    EXPECT_EQ(H.rows(), 2);
    EigSol::Matrix::Sparse<std::complex<float>> Sc(2, 2);
    Sc.insert(0, 0) = std::complex<float>(1.0f, 3.0f);
    Sc.insert(0, 1) = std::complex<float>(3.0f, 5.0f);
    Sc.insert(1, 1) = std::complex<float>(5.0f, -1.0f);
    EigSol::Matrix Ms(Sc);
    auto rc = EigSol::powerMethod<std::complex<float>>(Ms, EigSol::SolverOptions{});
    EXPECT_NEAR(std::abs(rc.eigenvalue - std::complex<float>(5.0f, -1.0f)), 0.0f, 1e-4f);
    EXPECT_EQ(Ms.rows(), 2);
}

// long double / std::complex<long double>: double-double on the device (EIGSOL_DD / EIGSOL_CDD),
// every entry point of the reference's API, at more than double precision
TEST(WidePrecision, LongDoubleInDoubleDouble) {
    using LD = long double;
    using CLD = std::complex<long double>;
    const LD tiny = std::ldexp(1.0L, -60);   // below double resolution at 1, inside the x87 significand
    EigSol::Matrix::Dense<LD> L(2, 2);
    L << 1.0L + tiny, 0.0L, 0.0L, 0.5L;
    EigSol::Matrix Ml(L);
    EigSol::Vector<LD> x0(2);
    x0 << 0.8L, 0.6L;
    auto r = EigSol::powerMethod<LD>(Ml, EigSol::SolverOptions{1000, 1e-20}, x0);
    EXPECT_TRUE(r.converged);
    EXPECT_NEAR(r.eigenvalue, 1.0L + tiny, std::ldexp(1.0L, -62));   // fp64 would return exactly 1
    EXPECT_TRUE(r.eigenvalue != 1.0L);
    EigSol::ShiftedSolverOptions<LD> so(0.45L, 1000, 1e-18);
    auto rs = EigSol::shiftedInversePowerMethod<LD>(Ml, so, x0);
    EXPECT_TRUE(rs.converged);
    EXPECT_NEAR(rs.eigenvalue, 0.5L, std::ldexp(1.0L, -62));
    EigSol::Vector<LD> b(2);
    b << 4.0L, 2.0L;
    auto x = EigSol::solve_shifted<LD>(Ml, 0.0L, b);
    EXPECT_NEAR(x(0), 4.0L / (1.0L + tiny), std::ldexp(1.0L, -61));
    EXPECT_TRUE(x(0) != 4.0L);
    EXPECT_NEAR(x(1), 4.0L, 1e-18L);
    EigSol::Matrix::Dense<LD> B(2, 2);
    B << 2.0L, 1.0L, 1.0L, 2.0L;
    auto q = EigSol::qr_eigenvalues<LD>(EigSol::Matrix(B), EigSol::SolverOptions{1000, 1e-12},
                                        EigSol::QRVariant::Unshifted);
    EXPECT_TRUE(q.converged);
    EXPECT_EQ(q.iterations, 25);   // the reference iteration (qr_algorithms_test.cpp): same count
    auto H = EigSol::to_hessenberg<LD>(EigSol::Matrix(B));
    EXPECT_EQ(H.rows(), 2);
    EigSol::Matrix::Sparse<CLD> Sc(3, 3);
    Sc.insert(0, 0) = CLD(1.0L, 3.0L);
    Sc.insert(0, 1) = CLD(3.0L, 5.0L);
    Sc.insert(1, 1) = CLD(5.0L, -1.0L);
    Sc.insert(2, 2) = CLD(2.0L, 4.0L);
    EigSol::Matrix Ms(Sc);
    auto rc = EigSol::powerMethod<CLD>(Ms, EigSol::SolverOptions{});
    EXPECT_NEAR(std::abs(rc.eigenvalue - CLD(5.0L, -1.0L)), 0.0L, 1e-8L);
    EigSol::ShiftedSolverOptions<CLD> sc(CLD(2.1L, 3.9L), 1000, 1e-20);
    auto rsc = EigSol::shiftedInversePowerMethod<CLD>(Ms, sc);
    EXPECT_TRUE(rsc.converged);
    EXPECT_NEAR(std::abs(rsc.eigenvalue - CLD(2.0L, 4.0L)), 0.0L, 1e-18L);
    EigSol::Matrix::Dense<CLD> Dc(2, 2);
    Dc << CLD(1, 1), CLD(2, 0), CLD(0, 0), CLD(3, -1);
    // long double Francis: fp64 sweeps, then each eigenvalue refined in double-double (triangular
    // input: the diagonal, exactly)
    auto qc = EigSol::qr_eigenvalues<CLD>(EigSol::Matrix(Dc), EigSol::SolverOptions{}, EigSol::QRVariant::Francis);
    EXPECT_TRUE(qc.converged);
    EXPECT_EQ(qc.iterations, 1);
    EXPECT_NEAR(std::abs(qc.eigenvalues(0) - CLD(1, 1)), 0.0L, 1e-18L);
    EXPECT_NEAR(std::abs(qc.eigenvalues(1) - CLD(3, -1)), 0.0L, 1e-18L);
    // real long double Francis: eigenvalues 1 and 3 of [[2, 1], [1, 2]] at extended precision, the
    // complex form in eigenvalues_complex_extended
    auto qf = EigSol::qr_eigenvalues<LD>(EigSol::Matrix(B), EigSol::SolverOptions{1000, 1e-12});
    EXPECT_TRUE(qf.converged);
    EXPECT_EQ(qf.eigenvalues_complex_extended.size(), 2u);
    const LD lo = std::min(qf.eigenvalues(0), qf.eigenvalues(1)), hi = std::max(qf.eigenvalues(0), qf.eigenvalues(1));
    EXPECT_NEAR(lo, 1.0L, 1e-18L);
    EXPECT_NEAR(hi, 3.0L, 1e-18L);
    EXPECT_NEAR(std::abs(qf.eigenvalues_complex_extended[0].imag()), 0.0L, 0.0L);
}

// ---------------------------------------------------------------- reference caller shapes
// A helper constrained on the concept, as reference callers write it (power_method.hpp:135).
template <EigSol::ScalarConcept S>
S dominant_eigenvalue(const EigSol::Matrix& M) {
    return EigSol::powerMethod<S>(M, EigSol::SolverOptions{}).eigenvalue;
}
static_assert(EigSol::ScalarConcept<float> && EigSol::ScalarConcept<std::complex<double>>);
static_assert(!EigSol::ScalarConcept<int> && !EigSol::ScalarConcept<std::complex<int>>);

TEST(StartVector, SeedChangesTakeEffect) {
    EigSol::random_seed() = 11;
    auto a = EigSol::random_vector<double>(5);
    EigSol::random_seed() = 12;
    auto b = EigSol::random_vector<double>(5);
    EigSol::random_seed() = 11;
    auto c = EigSol::random_vector<double>(5);
    EXPECT_TRUE(a.std() == c.std());
    EXPECT_TRUE(a.std() != b.std());
    EigSol::set_random_seed(11);   // same value again: restarts the sequence like std::srand
    auto d = EigSol::random_vector<double>(5);
    EXPECT_TRUE(a.std() == d.std());
    DenseMat A(2, 2);
    A << 2.0, 0.0, 0.0, 1.0;
    EXPECT_NEAR(dominant_eigenvalue<double>(EigSol::Matrix(A)), 2.0, 1e-8);
}

int main() {
    for (auto& [name, fn] : registry()) {
        const int before = g_fail;
        try {
            fn();
        } catch (const std::exception& e) {
            ++g_fail;
            std::printf("  FAIL %s: unexpected exception: %s\n", name.c_str(), e.what());
        }
        std::printf("%s %s\n", g_fail == before ? "[ OK ]" : "[FAIL]", name.c_str());
    }
    std::printf("%d checks, %d failures\n", g_checks, g_fail);
    if (g_fail == 0) std::printf("ALL PASSED\n");
    return g_fail == 0 ? 0 : 1;
}

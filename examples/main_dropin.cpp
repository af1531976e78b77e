// A caller in the shape of the reference demo (main.cpp:1-149), compiled against the drop-in.
//
// What a maintainer changes when switching a reference caller over (INTEGRATION.md §"Caller
// changes"): the include path (-I<repo>/include/eigsol/compat -I<repo>/include keeps every
// `#include "src/..."` line as it is), the Eigen include (not needed), and the one spot that
// names Eigen's dense type (`Eigen::Matrix<...> H_A = to_hessenberg(...)` becomes
// `EigSol::Matrix::Dense<Scalar>`, or `Eigen::Matrix` again where Eigen is on the include path:
// the façade converts both ways then).  Everything else — the helpers constrained on
// EigSol::ScalarConcept, `v.transpose()` printing, `Q_A * R_A`, structured bindings, the solver
// calls and their option structs — is the reference caller's code shape unchanged.
//
//   g++ -std=c++20 -I include/eigsol/compat -I include examples/main_dropin.cpp
//       -L pcsc_eigenvalue_solver_project_amd -leigsol_hip -o main_dropin
//   ./main_dropin tests/golden/A.txt tests/golden/B.txt
#include <iomanip>
#include <iostream>

#include "src/core/tolerance.hpp"
#include "src/core/types.hpp"
#include "src/matrix/matrix.hpp"
#include "src/option/shifted_solver_option.hpp"
#include "src/option/solver_option.hpp"
#include "src/power_method/power_method.hpp"
#include "src/power_method/shifted_inverse_power_solver.hpp"
#include "src/qr_method/qr_decompose.hpp"
#include "src/qr_method/qr_eigenvalues.hpp"
#include "src/qr_method/to_hessenberg.hpp"
#include "src/reader/file_matrix_reader.hpp"
#include "src/result/eigen_result.hpp"

template <typename VectorType>
void printVector(const VectorType& v, const std::string& name) {
    std::cout << name << std::endl << "(" << v.transpose() << ")" << std::endl << std::endl;
}

// helpers constrained on the concept, the way reference-side code is written
template <EigSol::ScalarConcept S>
void reportPower(const char* label, const EigSol::EigenResult<S>& r) {
    std::cout << label << std::endl
              << "Converged : " << std::boolalpha << r.converged << std::endl
              << "Iterations: " << r.iterations << std::endl
              << "Eigenvalue: " << r.eigenvalue << std::endl;
    printVector(r.eigenvector, "Eigenvector:");
}

template <EigSol::ScalarConcept S>
void reportQR(const char* label, const EigSol::QRResult<S>& r) {
    std::cout << "QR eigenvalues for " << label << std::endl
              << "Converged              : " << std::boolalpha << r.converged << std::endl
              << "Iterations             : " << r.iterations << std::endl
              << "Eigenvalues (diag of H): " << std::endl
              << r.eigenvalues.transpose() << std::endl << std::endl;
}

int main(int argc, char** argv) {
    using Scalar = std::complex<double>;
    const std::string fileA = argc > 1 ? argv[1] : "../data/A.txt";
    const std::string fileB = argc > 2 ? argv[2] : "../data/B.txt";
    EigSol::random_seed() = 20251226;   // reproducible start vectors (Vector::Random in the reference)

    EigSol::Matrix A = EigSol::readMatrixFromFile<Scalar>(fileA);
    EigSol::Matrix B = EigSol::readMatrixFromFile<Scalar>(fileB);

    std::cout << "===== Power method =====" << std::endl;
    EigSol::SolverOptions opts;
    opts.maxIterations = 1000;
    opts.tolerance = 1e-10;
    reportPower("Matrix A", EigSol::powerMethod<Scalar>(A, opts));
    reportPower("Matrix B", EigSol::powerMethod<Scalar>(B, opts));

    std::cout << "===== Shifted inverse power method =====" << std::endl;
    EigSol::ShiftedSolverOptions<Scalar> shiftedOptsA;
    shiftedOptsA.shift = 3.1;
    shiftedOptsA.maxIterations = 1000;
    shiftedOptsA.tolerance = 1e-12;
    reportPower("Matrix A", EigSol::shiftedInversePowerMethod<Scalar>(A, shiftedOptsA));
    EigSol::ShiftedSolverOptions<Scalar> shiftedOptsB;
    shiftedOptsB.shift = 2.3;
    shiftedOptsB.maxIterations = 1000;
    shiftedOptsB.tolerance = 1e-12;
    reportPower("Matrix B", EigSol::shiftedInversePowerMethod<Scalar>(B, shiftedOptsB));

    std::cout << "===== QR eigenvalue method =====" << std::endl;
    EigSol::SolverOptions qrOpts;
    qrOpts.maxIterations = 1000;
    qrOpts.tolerance = 1e-10;
    try {
        std::cout << "Hessenberg reduction of Matrix A" << std::endl;
        EigSol::Matrix::Dense<Scalar> H_A = EigSol::to_hessenberg<Scalar>(A);
        std::cout << "H(A) = " << std::endl << H_A << std::endl << std::endl;
        std::cout << "QR decomposition of Matrix A" << std::endl;
        auto [Q_A, R_A] = EigSol::qr_decompose<Scalar>(A);
        std::cout << "Q_A = " << std::endl << Q_A << std::endl << std::endl;
        std::cout << "R_A = " << std::endl << R_A << std::endl << std::endl;
        std::cout << "Q_A * R_A (should approximate A) = " << std::endl << Q_A * R_A << std::endl << std::endl;
        reportQR("Matrix A", EigSol::qr_eigenvalues<Scalar>(A, qrOpts));
    } catch (const std::exception& e) {
        std::cerr << "QR-related computation failed for Matrix A: " << e.what() << std::endl;
    }
    try {
        reportQR("Matrix B", EigSol::qr_eigenvalues<Scalar>(B, qrOpts));
    } catch (const std::exception& e) {
        // B is sparse: the reference's qr_eigenvalues throws on it as well (qr_eigenvalues.hpp:131-133)
        std::cerr << "QR-related computation failed for Matrix B: " << e.what() << std::endl;
    }
    return 0;
}

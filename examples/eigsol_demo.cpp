// eigsol_demo — command-line counterpart of the reference's demo program (main.cpp:41-149),
// written against the drop-in façade: read two matrices from text files, then run the power
// method, the shifted inverse power method, the Hessenberg reduction, the QR decomposition and the
// QR eigenvalue method on the gfx950 device, printing the same fields as the reference demo.
//
//   eigsol_demo [--real] [--shift-a S] [--shift-b S] [--tol T] [--max-iter N] [A.txt [B.txt]]
//
// Defaults mirror main.cpp: complex<double> scalars, shifts 3.1 (A) and 2.3 (B), power tolerance
// 1e-10, shifted tolerance 1e-12, 1000 iterations.  File format: include/eigsol/reader.hpp.
#include <complex>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <iostream>
#include <string>

#include <eigsol/eigsol.hpp>

namespace {

template <class S>
void put(std::ostream& o, const S& x) {
    if constexpr (EigSol::is_complex_of_floating<S>::value) o << "(" << x.real() << "," << x.imag() << ")";
    else o << x;
}

template <class S>
void print_vector(const EigSol::Vector<S>& v, const char* name) {
    std::cout << name << "\n(";
    for (std::size_t i = 0; i < v.size(); ++i) {
        if (i) std::cout << " ";
        put(std::cout, v(i));
    }
    std::cout << ")\n\n";
}

template <class S>
void print_matrix(const EigSol::DenseMatrix<S>& m, const char* name) {
    std::cout << name << "\n";
    for (std::int64_t i = 0; i < m.rows(); ++i) {
        for (std::int64_t j = 0; j < m.cols(); ++j) {
            if (j) std::cout << " ";
            put(std::cout, m(i, j));
        }
        std::cout << "\n";
    }
    std::cout << "\n";
}

template <class S>
void power_section(const EigSol::Matrix& M, const char* label, const EigSol::SolverOptions& o) {
    auto r = EigSol::powerMethod<S>(M, o);
    std::cout << label << "\nConverged : " << std::boolalpha << r.converged << "\nIterations: " << r.iterations
              << "\nEigenvalue: ";
    put(std::cout, r.eigenvalue);
    std::cout << "\n";
    print_vector(r.eigenvector, "Eigenvector:");
}

template <class S>
void shifted_section(const EigSol::Matrix& M, const char* label, double shift) {
    EigSol::ShiftedSolverOptions<S> o;
    o.shift = S(shift);
    o.maxIterations = 1000;
    o.tolerance = 1e-12;
    auto r = EigSol::shiftedInversePowerMethod<S>(M, o);
    std::cout << label << "\nConverged                : " << std::boolalpha << r.converged
              << "\nIterations               : " << r.iterations << "\nEigenvalue near the shift: ";
    put(std::cout, r.eigenvalue);
    std::cout << "\n";
    print_vector(r.eigenvector, "Eigenvector:");
}

template <class S>
void qr_section(const EigSol::Matrix& M, const char* label, const EigSol::SolverOptions& o, bool factors) {
    try {
        if (factors) {
            std::cout << "Hessenberg reduction of " << label << "\n";
            print_matrix(EigSol::to_hessenberg<S>(M), "H =");
            std::cout << "QR decomposition of " << label << "\n";
            auto qr = EigSol::qr_decompose<S>(M);
            print_matrix(qr.first, "Q =");
            print_matrix(qr.second, "R =");
            print_matrix(qr.first * qr.second, "Q * R (should approximate the matrix) =");
        }
        auto r = EigSol::qr_eigenvalues<S>(M, o);
        std::cout << "QR eigenvalues for " << label << "\nConverged              : " << std::boolalpha
                  << r.converged << "\nIterations             : " << r.iterations << "\n";
        print_vector(r.eigenvalues, "Eigenvalues (diag of H):");
    } catch (const std::exception& e) {
        std::cerr << "QR-related computation failed for " << label << ": " << e.what() << "\n";
    }
}

template <class S>
int run(const std::string& fa, const std::string& fb, double sa, double sb, EigSol::SolverOptions o) {
    EigSol::Matrix A = EigSol::readMatrixFromFile<S>(fa);
    std::cout << "===== Power method =====\n";
    power_section<S>(A, "Matrix A", o);
    if (!fb.empty()) {
        EigSol::Matrix B = EigSol::readMatrixFromFile<S>(fb);
        power_section<S>(B, "Matrix B", o);
        std::cout << "===== Shifted inverse power method =====\n";
        shifted_section<S>(A, "Matrix A", sa);
        shifted_section<S>(B, "Matrix B", sb);
        std::cout << "===== QR eigenvalue method =====\n";
        qr_section<S>(A, "Matrix A", o, true);
        qr_section<S>(B, "Matrix B", o, false);
    } else {
        std::cout << "===== Shifted inverse power method =====\n";
        shifted_section<S>(A, "Matrix A", sa);
        std::cout << "===== QR eigenvalue method =====\n";
        qr_section<S>(A, "Matrix A", o, true);
    }
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    bool real = false;
    double sa = 3.1, sb = 2.3;
    EigSol::SolverOptions o;
    o.maxIterations = 1000;
    o.tolerance = 1e-10;
    std::string files[2];
    int nf = 0;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) { std::cerr << "missing value after " << a << "\n"; std::exit(2); }
            return argv[++i];
        };
        if (a == "--real") real = true;
        else if (a == "--shift-a") sa = std::atof(next());
        else if (a == "--shift-b") sb = std::atof(next());
        else if (a == "--tol") o.tolerance = std::atof(next());
        else if (a == "--max-iter") o.maxIterations = std::atoi(next());
        else if (a == "-h" || a == "--help") {
            std::cout << "usage: eigsol_demo [--real] [--shift-a S] [--shift-b S] [--tol T] [--max-iter N] "
                         "[A.txt [B.txt]]\n";
            return 0;
        } else if (nf < 2) files[nf++] = a;
        else { std::cerr << "unexpected argument " << a << "\n"; return 2; }
    }
    if (nf == 0) {
        files[0] = "data/A.txt";
        files[1] = "data/B.txt";
    }
    try {
        return real ? run<double>(files[0], files[1], sa, sb, o)
                    : run<std::complex<double>>(files[0], files[1], sa, sb, o);
    } catch (const std::exception& e) {
        std::cerr << "eigsol_demo: " << e.what() << "\n";
        return 1;
    }
}

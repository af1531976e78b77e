// Host-only checks of the façade and the library's host planning, built with AddressSanitizer and
// UndefinedBehaviorSanitizer (tests/test_sanitizers.py).  No device: every call here either never
// touches HIP or fails cleanly without a GPU (the reader then keeps host storage).
#include <eigsol/eigsol.hpp>

#include <cstdio>
#include <numeric>
#include <random>
#include <string>
#include <vector>

static int g_fail = 0;
#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) { ++g_fail; std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); } \
    } while (0)

template <typename F>
static std::string message_of(F f) {
    try {
        f();
    } catch (const std::exception& e) {
        return e.what();
    }
    return "";
}

static void reader_cases(const std::string& data) {
    EigSol::Matrix A = EigSol::readMatrixFromFile<double>(data + "/A.txt");
    CHECK(A.isDense() && A.rows() == 3 && A.cols() == 3);
    const auto& d = A.cast<EigSol::Matrix::Dense<double>>();
    CHECK(d(1, 0) == 5.0 && d(2, 2) == 2.0);
    EigSol::Matrix B = EigSol::readMatrixFromFile<std::complex<double>>(data + "/B.txt");
    CHECK(!B.isDense() && B.rows() == 5);
    const auto& s = B.cast<EigSol::Matrix::Sparse<std::complex<double>>>();
    CHECK(s.nonZeros() == 8 && s.coeff(0, 0) == std::complex<double>(2.0, 3.0));
    const char* path = "/tmp/eigsol_sanitize_reader.txt";
    auto write = [&](const char* text) {
        std::FILE* f = std::fopen(path, "w");
        std::fputs(text, f);
        std::fclose(f);
    };
    write("sparse\n3 3\n4\n0 0 1.0\n2 1 2.0\n0 0 0.5\n1 2 -1.0\n");
    EigSol::Matrix C = EigSol::readMatrixFromFile<double>(path);
    const auto& cs = C.cast<EigSol::Matrix::Sparse<double>>();
    CHECK(cs.nonZeros() == 3 && cs.coeff(0, 0) == 1.5 && cs.coeff(2, 1) == 2.0);
    write("sparse\n3 3\n2\n0 0 1.0\n3 1 2.0\n");
    CHECK(message_of([&] { EigSol::readMatrixFromFile<double>(path); }) == "Sparse indices out of range");
    write("sparse\n3 3\n0\n");
    CHECK(message_of([&] { EigSol::readMatrixFromFile<double>(path); }) ==
          "number of non-zero entries must be positive in a sparse matrix");
    write("banded\n3 3\n");
    CHECK(message_of([&] { EigSol::readMatrixFromFile<double>(path); }) == "Unknown storage type: banded");
    write("dense\n2 2\n1 2 3\n");
    CHECK(message_of([&] { EigSol::readMatrixFromFile<double>(path); }) ==
          "Failed to read scalar entry in dense matrix");
    CHECK(message_of([&] { EigSol::readMatrixFromFile<double>("/nonexistent/x.txt"); }) ==
          "Impossible to open the file: /nonexistent/x.txt");
    std::remove(path);
}

static void matrix_cases() {
    EigSol::Matrix::Sparse<double> S(4, 4);
    for (int i = 0; i < 4; ++i) S.insert(i, (i + 1) % 4) = 1.0 + i;
    S.insert(2, 3) = 0.25;   // repeated position: summed on compression
    EigSol::Matrix M(S);
    const auto& T = M.cast<EigSol::Matrix::Sparse<double>>();
    CHECK(T.nonZeros() == 4 && T.coeff(2, 3) == 3.25);
    CHECK(T.toDense()(3, 0) == 4.0);
    bool bad = false;
    try {
        (void)M.cast<EigSol::Matrix::Dense<double>>();
    } catch (const std::bad_cast&) {
        bad = true;
    }
    CHECK(bad);
    std::vector<float> v = {1, 2, 3, 4, 5, 6};
    EigSol::Matrix R(v, 2, 3);
    CHECK(R.rows() == 2 && R.cols() == 3 && R.cast<EigSol::Matrix::Dense<float>>()(1, 0) == 4.0f);
    // no device: the first solver call reports it (no host fallback)
    CHECK(!message_of([&] { EigSol::powerMethod<double>(M); }).empty());
}

static void plan_cases() {
    const int P = 4;
    const int64_t n = 4000;
    std::vector<int64_t> rb(P + 1);
    for (int q = 0; q <= P; ++q) rb[q] = n * q / P;
    std::mt19937 gen(7);
    std::vector<int64_t> counts((size_t)P * P, 0);
    std::vector<std::vector<int64_t>> ghosts(P);
    for (int r = 0; r < P; ++r) {
        const int64_t rows = rb[r + 1] - rb[r];
        std::vector<int32_t> cols;
        for (int64_t i = 0; i < rows; ++i)
            for (int k = 0; k < 6; ++k) {
                const int64_t g = rb[r] + i + (int64_t)(gen() % 129) - 64;
                cols.push_back((int32_t)std::min<int64_t>(std::max<int64_t>(g, 0), n - 1));
            }
        std::vector<int32_t> local(cols.size());
        std::vector<int64_t> gg(cols.size()), recv(P);
        int64_t ng = 0;
        CHECK(eigsol_ghost_plan(P, rb.data(), r, (int64_t)cols.size(), cols.data(), local.data(), &ng, gg.data(),
                                recv.data()) == EIGSOL_OK);
        gg.resize(ng);
        ghosts[r] = gg;
        for (int q = 0; q < P; ++q) counts[(size_t)r * P + q] = recv[q];
        for (size_t k = 0; k < cols.size(); ++k) CHECK(local[k] >= 0 && local[k] < rows + ng);
    }
    int mode = -1;
    CHECK(eigsol_exchange_mode(P, rb.data(), counts.data(), &mode) == EIGSOL_OK && mode == EIGSOL_EXCHANGE_HALO);
    for (int me = 0; me < P; ++me) {
        std::vector<int64_t> req;
        for (int q = 0; q < P; ++q)
            for (int64_t g : ghosts[q])
                if (g >= rb[me] && g < rb[me + 1]) req.push_back(g);
        std::vector<int32_t> push(4 * std::max<size_t>(req.size(), 1));
        CHECK(eigsol_peer_plan(P, me, rb.data(), counts.data(), req.data(), (int64_t)req.size(), push.data()) ==
              EIGSOL_OK);
    }
    // malformed input is rejected before anything is read past the arrays
    int64_t bad_rb[3] = {1, 2, 3};
    CHECK(eigsol_exchange_mode(2, bad_rb, counts.data(), &mode) != EIGSOL_OK ||
          eigsol_ghost_plan(2, bad_rb, 0, 0, nullptr, nullptr, nullptr, nullptr, nullptr) != EIGSOL_OK);
    CHECK(eigsol_csr_create(nullptr, EIGSOL_F64, 1, 1, 0, nullptr, nullptr, nullptr, nullptr) == EIGSOL_E_INVALID);
    CHECK(eigsol_csr_create_from_coo(nullptr, EIGSOL_F64, 1, 1, 0, nullptr, nullptr, nullptr, nullptr) ==
          EIGSOL_E_INVALID);
    for (int s = 0; s <= 12; ++s) CHECK(eigsol_status_string(s) != nullptr);
}

int main(int argc, char** argv) {
    const std::string data = argc > 1 ? argv[1] : "tests/golden";
    reader_cases(data);
    matrix_cases();
    plan_cases();
    std::printf("sanitize_host: %s\n", g_fail ? "FAILED" : "ok");
    return g_fail ? 1 : 0;
}

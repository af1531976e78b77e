// EigSol drop-in façade — text matrix reader (src/reader/file_matrix_reader.hpp:33-200).
//
// Same file format and messages: "dense" or "sparse", then rows cols; dense entries row by row
// (complex as "re im" pairs); sparse: nnz, then "row col value" (or "row col re im") triplets.
// Integer fields are parsed as int like the reference (so "3.0" in an index position fails with
// "Error when trying to read indices in sparse matrix").
#pragma once

#include <fstream>
#include <string>

#include "matrix.hpp"

namespace EigSol {

template <typename S>
Matrix readInsideDenseMatrix(std::ifstream& in, int rows, int cols) {
    if (rows < 0 || cols < 0) throw std::runtime_error("Negative matrix dimensions");
    DenseMatrix<S> d(rows, cols);
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < cols; ++c) {
            if constexpr (is_complex_of_floating<S>::value) {
                typename S::value_type re{}, im{};
                if (!(in >> re >> im)) throw std::runtime_error("Failed to read complex entry in dense matrix");
                d(r, c) = S(re, im);
            } else {
                S v{};
                if (!(in >> v)) throw std::runtime_error("Failed to read scalar entry in dense matrix");
                d(r, c) = v;
            }
        }
    return Matrix(d);
}

// Sparse entries go straight to the device: the triplets become a device CSR (no host CSC, SURVEY
// §8f rank 2) and the Matrix materialises its host Sparse<S> only if a caller casts to it.
template <typename S>
Matrix readInsideSparseMatrix(std::ifstream& in, int rows, int cols) {
    if (rows < 0 || cols < 0) throw std::runtime_error("Negative matrix dimensions");
    int nnz = 0;
    if (!(in >> nnz)) throw std::runtime_error("Cannot read number of non-zero entries in the sparse matrix");
    if (nnz <= 0) throw std::runtime_error("number of non-zero entries must be positive in a sparse matrix");
    SparseTriplets<S> t;
    t.rows = rows;
    t.cols = cols;
    t.row.reserve(nnz);
    t.col.reserve(nnz);
    t.val.reserve(nnz);
    for (int k = 0; k < nnz; ++k) {
        int r{}, c{};
        if (!(in >> r >> c)) throw std::runtime_error("Error when trying to read indices in sparse matrix");
        if (r < 0 || r >= rows || c < 0 || c >= cols) throw std::runtime_error("Sparse indices out of range");
        if constexpr (is_complex_of_floating<S>::value) {
            typename S::value_type re{}, im{};
            if (!(in >> re >> im)) throw std::runtime_error("Failed to read scalar entry in sparse matrix");
            t.val.push_back(S(re, im));
        } else {
            S v{};
            if (!(in >> v)) throw std::runtime_error("Failed to read scalar entry in sparse matrix");
            t.val.push_back(v);
        }
        t.row.push_back(r);
        t.col.push_back(c);
    }
    return Matrix(std::move(t));
}

enum class StorageType { Dense, Sparse };

inline StorageType translateStorageType(const std::string& s) {
    if (s == "dense") return StorageType::Dense;
    if (s == "sparse") return StorageType::Sparse;
    throw std::runtime_error("Unknown storage type: " + s);
}

// Matrix is non-copyable and non-movable: returned as a prvalue (C++17 guaranteed elision),
// exactly like the reference's by-value signature.
template <typename S>
Matrix readMatrixFromFile(const std::string& filename) {
    std::ifstream in(filename);
    if (!in.is_open()) throw std::runtime_error("Impossible to open the file: " + filename);
    std::string storage;
    if (!(in >> storage)) throw std::runtime_error("Failed to read matrix storage type");
    const StorageType st = translateStorageType(storage);
    int rows = 0, cols = 0;
    if (!(in >> rows >> cols)) throw std::runtime_error("Failed to read matrix dimensions");
    if (rows <= 0 || cols <= 0) throw std::runtime_error("Matrix dimensions must be positive");
    if (st == StorageType::Dense) return readInsideDenseMatrix<S>(in, rows, cols);
    return readInsideSparseMatrix<S>(in, rows, cols);
}

}  // namespace EigSol

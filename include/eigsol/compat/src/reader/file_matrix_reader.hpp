// Drop-in path for the reference header src/reader/file_matrix_reader.hpp: with -I<repo>/include/eigsol/compat and
// -I<repo>/include a caller keeps its #include "src/reader/file_matrix_reader.hpp" line unchanged.
#pragma once
#include <eigsol/eigsol.hpp>

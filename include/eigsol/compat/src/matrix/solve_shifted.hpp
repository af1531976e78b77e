// Drop-in path for the reference header src/matrix/solve_shifted.hpp: with -I<repo>/include/eigsol/compat and
// -I<repo>/include a caller keeps its #include "src/matrix/solve_shifted.hpp" line unchanged.
#pragma once
#include <eigsol/eigsol.hpp>

// Drop-in path for the reference header src/option/shifted_solver_option.hpp: with -I<repo>/include/eigsol/compat and
// -I<repo>/include a caller keeps its #include "src/option/shifted_solver_option.hpp" line unchanged.
#pragma once
#include <eigsol/eigsol.hpp>

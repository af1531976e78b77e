// Drop-in path for the reference header src/power_method/shifted_inverse_power_solver.hpp: with -I<repo>/include/eigsol/compat and
// -I<repo>/include a caller keeps its #include "src/power_method/shifted_inverse_power_solver.hpp" line unchanged.
#pragma once
#include <eigsol/eigsol.hpp>

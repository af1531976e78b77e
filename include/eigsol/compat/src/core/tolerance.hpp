// Drop-in path for the reference header src/core/tolerance.hpp: with -I<repo>/include/eigsol/compat and
// -I<repo>/include a caller keeps its #include "src/core/tolerance.hpp" line unchanged.
#pragma once
#include <eigsol/eigsol.hpp>

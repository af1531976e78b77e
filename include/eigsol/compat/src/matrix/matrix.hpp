// Drop-in path for the reference header src/matrix/matrix.hpp: with -I<repo>/include/eigsol/compat and
// -I<repo>/include a caller keeps its #include "src/matrix/matrix.hpp" line unchanged.
#pragma once
#include <eigsol/eigsol.hpp>

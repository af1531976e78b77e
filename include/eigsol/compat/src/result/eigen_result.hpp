// Drop-in path for the reference header src/result/eigen_result.hpp: with -I<repo>/include/eigsol/compat and
// -I<repo>/include a caller keeps its #include "src/result/eigen_result.hpp" line unchanged.
#pragma once
#include <eigsol/eigsol.hpp>

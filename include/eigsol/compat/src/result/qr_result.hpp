// Drop-in path for the reference header src/result/qr_result.hpp: with -I<repo>/include/eigsol/compat and
// -I<repo>/include a caller keeps its #include "src/result/qr_result.hpp" line unchanged.
#pragma once
#include <eigsol/eigsol.hpp>

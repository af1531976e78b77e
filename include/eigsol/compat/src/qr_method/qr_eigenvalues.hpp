// Drop-in path for the reference header src/qr_method/qr_eigenvalues.hpp: with -I<repo>/include/eigsol/compat and
// -I<repo>/include a caller keeps its #include "src/qr_method/qr_eigenvalues.hpp" line unchanged.
#pragma once
#include <eigsol/eigsol.hpp>

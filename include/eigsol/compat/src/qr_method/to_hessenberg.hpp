// Drop-in path for the reference header src/qr_method/to_hessenberg.hpp: with -I<repo>/include/eigsol/compat and
// -I<repo>/include a caller keeps its #include "src/qr_method/to_hessenberg.hpp" line unchanged.
#pragma once
#include <eigsol/eigsol.hpp>

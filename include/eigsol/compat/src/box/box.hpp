// Drop-in path for the reference header src/box/box.hpp: with -I<repo>/include/eigsol/compat and
// -I<repo>/include a caller keeps its #include "src/box/box.hpp" line unchanged.
#pragma once
#include <eigsol/eigsol.hpp>

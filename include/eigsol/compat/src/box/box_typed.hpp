// Drop-in path for the reference header src/box/box_typed.hpp: with -I<repo>/include/eigsol/compat and
// -I<repo>/include a caller keeps its #include "src/box/box_typed.hpp" line unchanged.
#pragma once
#include <eigsol/eigsol.hpp>

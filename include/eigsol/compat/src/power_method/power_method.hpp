// Drop-in path for the reference header src/power_method/power_method.hpp: with -I<repo>/include/eigsol/compat and
// -I<repo>/include a caller keeps its #include "src/power_method/power_method.hpp" line unchanged.
#pragma once
#include <eigsol/eigsol.hpp>

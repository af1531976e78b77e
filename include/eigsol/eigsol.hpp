// EigSol — MI355X (gfx950) drop-in for the C++ API of hugoheziyang/PCSC_Eigenvalue_Solver_Project.
//
//   #include <eigsol/eigsol.hpp>        (add -I<repo>/include, link -leigsol_hip)
//
// Everything lives in namespace EigSol with the reference's names; see core.hpp (types),
// matrix.hpp (Matrix), solvers.hpp (power / shifted inverse / solve_shifted / QR), reader.hpp.
#pragma once

#include "core.hpp"
#include "device.hpp"
#include "matrix.hpp"
#include "reader.hpp"
#include "solvers.hpp"

// mfem.hpp — lets a driver written against MFEM keep `#include "mfem.hpp"` and
// `using namespace mfem;` (linear_convection_diffusion_2D.cpp:15,37): the names resolve to the
// MFEM-shaped host API over libcdfem.so (cdfem_mfem.hpp).  The PETSc front end of that header
// (MFEMInitializePetsc, PetscParMatrix, PetscLinearSolver) is what MFEM_USE_PETSC guards in the
// reference drivers (:19-21).
#pragma once
#include "cdfem_mfem.hpp"

#ifndef MFEM_USE_PETSC
#define MFEM_USE_PETSC
#endif
#ifndef MFEM_USE_MPI
#define MFEM_USE_MPI
#endif

namespace mfem = cdfem::mfem;

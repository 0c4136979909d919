// Drop-in names for code written against the reference (include/BH_tDMRG.hpp,
// include/OptimalControl.hpp): `OptimalControl<BH_tDMRG>` with IQMPS states,
// BoseHubbard sites and Args{cutoff, maxm} compiles against the MI355X engine.
#pragma once

#include "ControlBasis.hpp"
#include "ControlBasisFactory.hpp"
#include "GpuTDMRG.hpp"
#include "MPS.hpp"
#include "OptimalControl.hpp"
#include "SeedGenerator.hpp"

using BH_tDMRG = ocmps::GpuTDMRG;
using IQMPS = ocmps::MPS;
using ocmps::Args;
using ocmps::BoseHubbard;
using ocmps::Cplx;
using stdvec = ocmps::stdvec;
using rowmat = ocmps::rowmat;

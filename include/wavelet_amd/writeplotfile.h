// writeplotfile.h — AMReX plotfile writer without AMReX (src/writeplotfile.h,
// src/writeplotfile.cpp:118-231).  Produces the files amrex::WriteMultiLevelPlotfile
// writes for a single-rank run: Header, Level_N/Cell_H, Level_N/Cell_D_00000.
#pragma once

#include <string>
#include <vector>

#include "box-structs.h"

void write_plotfiles(std::vector<std::vector<std::vector<multiBox3D>>> data, LocDimData locations,
                     LocDimData dimensions, std::vector<std::string> files, int num_levels, int num_components,
                     std::vector<std::string> comp_names, AMReXInfo amrexinfo, std::string out);

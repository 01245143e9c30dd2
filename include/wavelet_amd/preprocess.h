// preprocess.h — AMReX plotfile reading without AMReX (src/preprocess.h,
// src/preprocess.cpp:14-307): plotfile Header, Level_N/Cell_H (VisMF "new
// format") and the Cell_D FAB files (IEEE fp64).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "box-structs.h"

// src/preprocess.cpp:107: every selected component of every box of every
// (file, level), narrowed to float, with locations, dimensions, box counts,
// running min/max and the AMReX metadata.
AllData preprocess_data(std::vector<std::string> files, std::vector<std::string> components,
                        std::vector<int> levels);

namespace wavelet_amd {

// One FAB of a level: where its bytes are and what box it covers.
struct FabRef {
    std::string file;   // Level_N/Cell_D_xxxxx
    uint64_t offset;    // of the FAB's text header line
    int lo[3], hi[3];
    int ncomp;
    bool big_endian;
};

// Header of one plotfile, parsed the way src/preprocess.cpp:131-242 does.
struct PlotHeader {
    std::vector<std::string> names;
    int dim = 0;
    long double true_time = 0;
    std::vector<double> geomcell;  // prob_lo[3], prob_hi[3]
    std::vector<int> ref_ratios;   // `dim` values from the ratio line (0 where absent)
    int xDim = 0, yDim = 0, zDim = 0;
    std::vector<int> steps;        // every value on the level-steps line
};

PlotHeader read_plot_header(const std::string& plotfile);

// Cell_H of <plotfile>/Level_<level>/Cell -> FABs in file order (= MFIter order).
std::vector<FabRef> read_level_index(const std::string& plotfile, int level);

// Components `comps` of one FAB as fp64 (comp-major, x fastest) into dst.
void read_fab(const FabRef& fab, const std::vector<int>& comps, double* dst);

// Header indices of `components`, in Header order (src/preprocess.cpp:149-165);
// empty if any name is missing.
std::vector<int> match_components(const PlotHeader& h, const std::vector<std::string>& components);

}  // namespace wavelet_amd

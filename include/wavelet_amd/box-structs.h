// box-structs.h — the reference's data types (src/box-structs.h:7-70).
#pragma once

#include <string>
#include <utility>
#include <vector>

#include "grid.h"

using Box3D = Grid3D<float>;            // one component of one box
using multiBox3D = std::vector<Box3D>;  // all components of one box
using Location = std::vector<int>;
using Dimensions = std::vector<int>;

// Compressed form of one Box3D (src/box-structs.h:65-70).
struct CompressedWavelet {
    std::vector<int> shape;                          // {W, H, D}
    std::vector<int> coeff_shape;                    // {W * H * D}
    std::vector<std::pair<int, float>> rle_encoded;  // (zeros before, value)
    bool need32 = false;                             // computed, never serialized
};

// Location or dimension data of every box of a run: [t][lev][box][xyz]
// (src/box-structs.h:19).
using LocDimData = std::vector<std::vector<std::vector<std::vector<int>>>>;

// What decompression needs to know about a compression run (src/box-structs.h:22-28).
struct RunInfo {
    std::vector<std::string> files;       // plotfile directories, in time order
    int min_level = 0;
    int max_level = 0;
    std::vector<std::string> components;  // names as given by the user
    std::vector<int> comp_idxs;           // their indices in the plotfile Header
};

// One level of one timestep (src/box-structs.h:31-38).
struct LevelData {
    std::vector<multiBox3D> boxes;
    std::vector<Location> locations;
    std::vector<Dimensions> dimensions;
    int box_count = 0;
    std::vector<float> min_values;
    std::vector<float> max_values;
};

// Plotfile metadata needed to write plotfiles back (src/box-structs.h:42-50).
struct AMReXInfo {
    std::vector<std::vector<double>> geomcellinfo;  // per time: prob_lo[3], prob_hi[3]
    std::vector<int> ref_ratios;                    // per dimension
    std::vector<long double> true_times;            // per time
    std::vector<std::vector<int>> level_steps;      // [t][lev]
    int xDim = 0, yDim = 0, zDim = 0;               // level-0 domain size
};

// Everything a compression run reads (src/box-structs.h:53-62).
struct AllData {
    std::vector<std::vector<std::vector<multiBox3D>>> boxes;  // [t][lev][box][comp]
    LocDimData locations;
    LocDimData dimensions;
    std::vector<std::vector<int>> box_counts;  // [t][lev]
    std::vector<float> min_values;             // per component
    std::vector<float> max_values;
    AMReXInfo amrexinfo;
    std::vector<int> comp_idxs;
};

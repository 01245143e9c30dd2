// box-structs.h — the reference's codec data types (src/box-structs.h:7-70).
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

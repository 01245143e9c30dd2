// decompressor.h — drop-in for the reference's src/decompressor.h:6-18.
#pragma once

#include "box-structs.h"

// Read one .xz file, decode it on the GPU and return the Box3D
// (src/decompressor.cpp:238-255; only file_path is used, as in the reference).
Box3D decompress(std::string file_path, int time, int level, int component, int box_idx);

// Payload bytes -> CompressedWavelet (src/decompressor.cpp:35-74).
CompressedWavelet deserialize_compressed_wavelet(const std::string& data);

// Flat coefficients -> Box3D, on the GPU (src/decompressor.cpp:79-159).
Box3D inverse_wavelet_decompose(std::vector<float> flat, int x, int y, int z);

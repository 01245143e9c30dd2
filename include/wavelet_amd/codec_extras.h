// codec_extras.h — routines the reference keeps file-static
// (src/compressor.cpp:24-185, src/decompressor.cpp:14-30), exported here so the
// reference's unit tests can be restated against this library.
#pragma once

#include <string>
#include <utility>
#include <vector>

#include "box-structs.h"

namespace wavelet_amd {

// wavelet_decompose (GPU): Box3D -> flat coefficients, x slowest.
std::vector<float> wavelet_decompose(const Box3D& box);

// rle_encode over an explicit mask (host; the GPU path never materialises a mask).
std::vector<std::pair<int, float>> rle_encode(const std::vector<bool>& mask, const std::vector<float>& values);

// serialize_compressed_wavelet (host).
std::string serialize_compressed_wavelet(const CompressedWavelet& compressed);

// rle_decode (host; the GPU decode is K5 inside decompress()).
std::vector<float> rle_decode(const std::vector<std::pair<int, float>>& rle_encoded, int total_length);

// xz helpers: liblzma easy encoder preset 6 + CRC64, and the stream decoder.
std::string xz_compress(const std::string& payload);
std::string xz_decompress(const std::string& xz);

}  // namespace wavelet_amd

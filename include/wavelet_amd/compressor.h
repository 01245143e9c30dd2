// compressor.h — drop-in for the reference's src/compressor.h:9-15.
// The transform, threshold and pack run on the GPU (libwavelet_amd.so, one
// batched wc_forward_host_units call for all components, each read from its
// Box3D); the xz write stays on the host (liblzma preset 6, CRC64, as
// src/compressor.cpp:256-291), the components' streams on a thread pool.
#pragma once

#include "box-structs.h"

std::vector<CompressedWavelet> compress(multiBox3D& box,
                                        std::vector<int> components,
                                        double keep,
                                        int time,
                                        int level,
                                        int box_index,
                                        std::string compressed_dir);

// xz_pool.h — the xz stage of compress()/decompress() (src/compressor.cpp:256-291,
// src/decompressor.cpp:164-234) over a pool of host threads: one independent
// .xz stream per unit, so units encode and decode in parallel.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace wavelet_amd {

// Threads for host stages: $WCAMD_THREADS, else $OMP_NUM_THREADS, else the core count.
int host_threads();

// Run fn(i) for i in [0, n) on `threads` threads (dynamic assignment).
void parallel_for(size_t n, int threads, const std::function<void(size_t)>& fn);

struct XzJob {
    const uint8_t* data;  // serialized payload
    size_t size;
    std::string path;     // output file
};

// Encode each job (preset 6, CRC64, as the reference) and write its file.  A
// file that cannot be opened is skipped (src/compressor.cpp:256-257); encoder
// failures exit.  Returns the bytes written.
uint64_t xz_write_files(const std::vector<XzJob>& jobs, int threads);

// Read and decode each file (stream decoder, concatenated streams).  Failures exit.
std::vector<std::string> xz_read_files(const std::vector<std::string>& paths, int threads);

// One buffer -> one .xz stream (preset 6, CRC64).
std::string xz_encode(const uint8_t* data, size_t size);

}  // namespace wavelet_amd

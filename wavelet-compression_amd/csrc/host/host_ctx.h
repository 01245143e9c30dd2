// host_ctx.h — shared pieces of the C++ mirror (not part of the public API).
#pragma once

#include <cstdio>
#include <cstdlib>
#include <string>

#include "wavelet_amd.h"

namespace wavelet_amd {

// One codec context per host thread on device $WCAMD_DEVICE (default 0), or
// the device set by set_thread_device() before first use; created on first
// use.  Exits like the reference's fatal paths if no GPU.
wc_ctx* thread_ctx();
void set_thread_device(int device);

// The reference logs with spdlog::error and calls exit(EXIT_FAILURE) on codec
// and I/O failures (src/compressor.cpp:263-283, src/decompressor.cpp:170-231).
[[noreturn]] inline void fatal(const std::string& msg) {
    std::fprintf(stderr, "[error] %s\n", msg.c_str());
    std::exit(EXIT_FAILURE);
}

inline void check(wc_ctx* c, int rc, const char* what) {
    if (rc != WC_OK) fatal(std::string(what) + ": " + wc_last_error(c));
}

}  // namespace wavelet_amd

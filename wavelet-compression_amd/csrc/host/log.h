// log.h — console messages of the driver (the reference logs with spdlog at
// info/error level; the wording of each message follows the reference's).
#pragma once

#include <cstdio>
#include <string>

namespace wavelet_amd {

inline void log_info(const std::string& m) {
    std::printf("[info] %s\n", m.c_str());
    std::fflush(stdout);
}
inline void log_error(const std::string& m) {
    std::fprintf(stderr, "[error] %s\n", m.c_str());
    std::fflush(stderr);
}

}  // namespace wavelet_amd

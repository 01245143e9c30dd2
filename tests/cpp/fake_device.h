// fake_device.h — controls of the CPU fake of the HIP runtime and of the
// device entry points (tests/cpp/fake_device.cpp).  Test infrastructure.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "wavelet_amd.h"

struct wc_ctx;

namespace fake {
void fail_nth(const char* api, int k);  // the k-th next call of api fails (H2D, D2H, hipEventRecord, wc_forward, ...)
void clear_failures();
long calls();
size_t live_allocations();
extern int kernel_error_calls;  // the next k wc_forward calls raise a kernel-detected error
uint32_t kept_of(const wc_unit& u);
std::vector<uint8_t> payload_of(const wc_unit& u, const void* cells, int dtype);
void release_context_tables(const wc_ctx* c);
}  // namespace fake

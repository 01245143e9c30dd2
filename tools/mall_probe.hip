// mall_probe.hip — does the Infinity Cache (256 MiB L3) absorb a staging
// round trip?  Timing-only probe for the C5 cohort-forward design (DESIGN.md
// "C5 cohort forward"); the data read back is never checked.
//
//   write S      : one launch writes S bytes (float4, coalesced), repeated:
//                  above ~6 TB/s for small S => rewritten dirty lines are
//                  absorbed on-die (no HBM write per pass)
//   write+read S : the same S written then read back, repeated
//   mix ring R   : one launch of items of 64 KiB: read the item's cells
//                  (streamed, 4 GiB in all), write a 64 KiB staging block into
//                  ring slot i mod R, read ring slot (i - R/2) mod R back,
//                  write 58 KiB of output (streamed).  Ring = 4 GiB is the
//                  staged forward today; a small ring is the cohort design.
//
// usage: mall_probe  (prints one JSON line per case)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            std::exit(2);                                                          \
        }                                                                          \
    } while (0)

__global__ __launch_bounds__(256) void k_write(float4* __restrict__ p, size_t n4, float v) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
        p[i] = make_float4(v, v, v, v);
}

__global__ __launch_bounds__(256) void k_read(const float4* __restrict__ p, size_t n4, float* __restrict__ sink) {
    float s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const float4 v = p[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.678f) sink[0] = s;  // keeps the loads
}

constexpr int kItemF4 = 65536 / 16;  // float4 per 64 KiB item
constexpr int kOutF4 = 59392 / 16;   // 58 KiB output per item

__global__ __launch_bounds__(256) void k_mix(const float4* __restrict__ cells, float4* __restrict__ ring,
                                             float4* __restrict__ out, uint32_t ring_items, float* __restrict__ sink) {
    const uint32_t i = blockIdx.x;
    const int t = threadIdx.x;
    const float4* c = cells + (size_t)i * kItemF4;
    float4 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = c[k * 256 + t];
    float4* w = ring + (size_t)(i % ring_items) * kItemF4;
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k * 256 + t] = v[k];
    const uint32_t j = (i + ring_items - ring_items / 2) % ring_items;
    const float4* r = ring + (size_t)j * kItemF4;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const float4 x = r[k * 256 + t];
        s += x.x + x.y + x.z + x.w;
    }
    float4* o = out + (size_t)i * kOutF4;
    for (int k = t; k < kOutF4; k += 256) o[k] = make_float4(s, s, s, s);
    if (s == 12345.678f) sink[0] = s;
}

int main() {
    const size_t big = size_t(4) << 30;
    float4 *a = nullptr, *cells = nullptr, *out = nullptr;
    float* sink = nullptr;
    CK(hipMalloc(&a, big));
    CK(hipMalloc(&cells, big));
    const uint32_t items = (uint32_t)(big / 65536);
    CK(hipMalloc(&out, (size_t)items * kOutF4 * 16));
    CK(hipMalloc(&sink, 16));
    CK(hipMemset(a, 0, big));
    CK(hipMemset(cells, 0, big));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grid = 2048 * 4;
    const size_t sizes_mb[] = {16, 32, 64, 96, 128, 192, 256, 384, 1024, 4096};
    for (size_t mb : sizes_mb) {
        const size_t S = mb << 20, n4 = S / 16;
        const int reps = (int)std::max<size_t>(4, (size_t(16) << 30) / S);
        for (int mode = 0; mode < 2; ++mode) {
            for (int w = 0; w < 2; ++w) {  // warm-up pass, then the timed pass
                CK(hipEventRecord(e0));
                for (int r = 0; r < reps; ++r) {
                    k_write<<<grid, 256>>>(a, n4, (float)r);
                    if (mode == 1) k_read<<<grid, 256>>>(a, n4, sink);
                }
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
            }
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double bytes = (double)S * reps * (mode == 1 ? 2 : 1);
            std::printf("{\"case\": \"%s\", \"mb\": %zu, \"reps\": %d, \"ms\": %.4f, \"tb_s\": %.3f}\n",
                        mode ? "write+read" : "write", mb, reps, ms, bytes / (ms * 1e-3) / 1e12);
        }
    }
    const uint32_t rings_mb[] = {16, 32, 64, 96, 128, 192, 256, 512, 4096};
    for (uint32_t rmb : rings_mb) {
        const uint32_t ring_items = (uint32_t)(((size_t)rmb << 20) / 65536);
        float best = 1e30f;
        for (int w = 0; w < 4; ++w) {
            CK(hipEventRecord(e0));
            k_mix<<<items, 256>>>(cells, a, out, ring_items, sink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (w > 0 && ms < best) best = ms;
        }
        const double alg = (double)items * (65536.0 + 59392.0);  // cells + output (the bytes that must move)
        const double all = (double)items * (65536.0 * 3 + 59392.0);
        std::printf("{\"case\": \"mix\", \"ring_mb\": %u, \"ms\": %.4f, \"alg_tb_s\": %.3f, \"all_tb_s\": %.3f}\n", rmb,
                    best, alg / (best * 1e-3) / 1e12, all / (best * 1e-3) / 1e12);
    }
    CK(hipDeviceSynchronize());
    return 0;
}

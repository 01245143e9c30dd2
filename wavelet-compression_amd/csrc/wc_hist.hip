// wc_hist.hip — coefficient-magnitude histogram of the staged forward
// coefficients, for the opt-in global-threshold mode (wc_forward_stage /
// wc_forward_emit in include/wavelet_amd.h).
//
// Not part of the reference's codec: src/compressor.cpp:212-216 thresholds
// every box at (its own max) * (1 - keep).  The histogram mode replaces that
// per-box rule with ONE threshold for a whole run (all units on all ranks),
// picked from the all-reduced histogram (RCCL, one WC_HIST_BINS x u64 buffer)
// so that a chosen fraction of all coefficients is retained.  Payload format,
// run-length rule and decoder are unchanged.
//
// Bin of a coefficient c: fp32 bits of |c| >> WC_HIST_SHIFT (monotone in |c|,
// 8 exponent + 3 mantissa bits, 4096 bins up to +inf; NaN is not counted),
// so "every coefficient in bins >= b" is exactly "|c| > float(b << 19) - 1ulp",
// the strict test the emit kernels already apply.
//
// HBM-bound: one 16-B load per 4 coefficients (4 B/coefficient read), LDS
// privatized bins per workgroup, one 64-bit global atomic per nonzero bin per
// workgroup at the end.
#include "wc_device.h"

namespace wc {

constexpr int kHistThreads = 256;

// Workgroup g folds flat tiles g, g + G, ... (kFlatTile coefficients of one
// unit each, in the staged flat scratch at coef + coef_off) into its LDS bins,
// then adds its nonzero bins to hist with 64-bit atomics (integer sums: the
// result does not depend on their order).  skip_fast: only the units of the
// generic transform (k_transform_hist has binned the fast units' coefficients
// while it staged them).
__global__ __launch_bounds__(kHistThreads) void k_hist(const UnitDev* __restrict__ units,
                                                     const FTile* __restrict__ ftiles, uint32_t nftiles,
                                                     const float* __restrict__ coef,
                                                     unsigned long long* __restrict__ hist, int skip_fast) {
    __shared__ uint32_t h[kHistBins];
    for (int i = threadIdx.x; i < kHistBins; i += kHistThreads) h[i] = 0u;
    __syncthreads();
    for (uint32_t t = blockIdx.x; t < nftiles; t += gridDim.x) {
        const FTile ft = ftiles[t];
        const UnitDev& U = units[ft.unit];
        if (skip_fast && U.fast) continue;  // uniform
        const uint64_t start = (uint64_t)ft.index * kFlatTile;
        const uint32_t len = (uint32_t)min((uint64_t)kFlatTile, U.ncells - start);
        // coef_off is 16-B aligned and kFlatTile a multiple of 4: float4 loads
        const float4* __restrict__ p4 = reinterpret_cast<const float4*>(coef + U.coef_off + start);
        constexpr int kIt = kFlatTile / (4 * kHistThreads);  // 4: every load of the tile in flight at once
        float4 v[kIt];
#pragma unroll
        for (int it = 0; it < kIt; ++it) {
            const uint32_t q = it * kHistThreads + threadIdx.x;
            v[it] = 4 * q < len ? p4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int it = 0; it < kIt; ++it) {
            const uint32_t e = 4 * (it * kHistThreads + threadIdx.x);
            hist_add(h, v[it].x, e < len);
            hist_add(h, v[it].y, e + 1 < len);
            hist_add(h, v[it].z, e + 2 < len);
            hist_add(h, v[it].w, e + 3 < len);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kHistBins; i += kHistThreads)
        if (h[i]) atomicAdd(hist + i, (unsigned long long)h[i]);
}

hipError_t launch_hist(hipStream_t st, const UnitDev* units, const FTile* ftiles, uint32_t nftiles,
                       const float* coef, uint32_t max_blocks, unsigned long long* hist, bool skip_fast) {
    if (nftiles == 0) return hipSuccess;
    const uint32_t g = nftiles < max_blocks ? nftiles : max_blocks;
    k_hist<<<g, kHistThreads, 0, st>>>(units, ftiles, nftiles, coef, hist, skip_fast ? 1 : 0);
    return hipGetLastError();
}

}  // namespace wc

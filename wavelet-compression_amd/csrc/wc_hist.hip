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
// privatized bins per workgroup, per-workgroup rows written once and summed
// column-wise by a second small kernel (no global atomics, deterministic).
#include "wc_device.h"

namespace wc {

namespace {

constexpr int kHistBins = 4096;
constexpr int kHistShift = 19;
constexpr int kHistThreads = 256;

__device__ __forceinline__ void hist_add(uint32_t* h, float v) {
    const uint32_t b = __float_as_uint(v) & 0x7fffffffu;
    if (b <= 0x7f800000u) atomicAdd(h + (b >> kHistShift), 1u);
}

}  // namespace

// Workgroup g folds flat tiles g, g + G, ... (kFlatTile coefficients of one
// unit each, in the staged flat scratch at coef + coef_off) into its LDS bins
// and writes them as row g of rows[G][kHistBins].
__global__ __launch_bounds__(kHistThreads) void k_hist_rows(const UnitDev* __restrict__ units,
                                                          const FTile* __restrict__ ftiles, uint32_t nftiles,
                                                          const float* __restrict__ coef,
                                                          uint32_t* __restrict__ rows) {
    __shared__ uint32_t h[kHistBins];
    for (int i = threadIdx.x; i < kHistBins; i += kHistThreads) h[i] = 0u;
    __syncthreads();
    for (uint32_t t = blockIdx.x; t < nftiles; t += gridDim.x) {
        const FTile ft = ftiles[t];
        const UnitDev& U = units[ft.unit];
        const uint64_t start = (uint64_t)ft.index * kFlatTile;
        const uint32_t len = (uint32_t)min((uint64_t)kFlatTile, U.ncells - start);
        // coef_off is 16-B aligned and kFlatTile a multiple of 4: float4 loads
        const float4* __restrict__ p4 = reinterpret_cast<const float4*>(coef + U.coef_off + start);
#pragma unroll 4
        for (uint32_t q = threadIdx.x; 4 * q < len; q += kHistThreads) {
            const float4 v = p4[q];
            const uint32_t e = 4 * q;
            hist_add(h, v.x);
            if (e + 1 < len) hist_add(h, v.y);
            if (e + 2 < len) hist_add(h, v.z);
            if (e + 3 < len) hist_add(h, v.w);
        }
    }
    __syncthreads();
    uint32_t* row = rows + (uint64_t)blockIdx.x * kHistBins;
    for (int i = threadIdx.x; i < kHistBins; i += kHistThreads) row[i] = h[i];
}

// hist[b] += sum over rows of rows[r][b]: one thread per bin, coalesced rows.
__global__ __launch_bounds__(kHistThreads) void k_hist_sum(const uint32_t* __restrict__ rows, uint32_t nrows,
                                                         unsigned long long* __restrict__ hist) {
    const int b = blockIdx.x * kHistThreads + threadIdx.x;
    unsigned long long s = 0;
    for (uint32_t r = 0; r < nrows; ++r) s += rows[(uint64_t)r * kHistBins + b];
    hist[b] += s;
}

hipError_t launch_hist(hipStream_t st, const UnitDev* units, const FTile* ftiles, uint32_t nftiles,
                       const float* coef, uint32_t* rows, uint32_t nrows, unsigned long long* hist) {
    if (nftiles == 0) return hipSuccess;
    const uint32_t g = nftiles < nrows ? nftiles : nrows;
    k_hist_rows<<<g, kHistThreads, 0, st>>>(units, ftiles, nftiles, coef, rows);
    k_hist_sum<<<kHistBins / kHistThreads, kHistThreads, 0, st>>>(rows, g, hist);
    return hipGetLastError();
}

}  // namespace wc

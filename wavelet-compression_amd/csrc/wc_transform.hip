// wc_transform.hip — K1: one-level 3-D Haar, cells -> flat coefficients.
//   k_transform       generic tiles (any dims, odd tails)     src/compressor.cpp:85-185
//   k_transform_fast  even dims, D % 8 == 0 (4 z-blocks per thread)
// Both also reduce the unit's max-|c| key (src/compressor.cpp:212-215).
// The tile bodies live in wc_xform.h (shared with the pipelined kernel).
//
// Numerics (bit-exact with the reference): the reference
// pair `(a + b) / 2.0` is a float add, an exact halving in double and one
// rounding to float == `(a + b) * 0.5f` here; built with -ffp-contract=off and
// -fno-gpu-flush-denormals-to-zero so subnormals round identically.
#include "wc_xform.h"

namespace wc {

// Output position of a unit's flat coefficients: 0 the dense flat scratch
// (coef_off), 1 at the unit's cell offset (wc_decompose), 2 its slot in the
// chunked forward's coefficient slots (ring_off).
__device__ __forceinline__ uint64_t out_base(const UnitDev& U, int mode) {
    return mode == 1 ? U.cell_off : mode == 2 ? U.ring_off : U.coef_off;
}

// ---------------------------------------------------------------------------
// K1 kernels of the staged path: one tile per workgroup, coefficients written
// to the flat scratch (plain stores: the next kernel reads them), the unit's
// max key reduced with one 64-bit atomicMax per wave.
template <typename T, bool KEYS>
__global__ __launch_bounds__(kThreads) void k_transform(
    const T* __restrict__ cells, const UnitDev* __restrict__ units, const XTile* __restrict__ tiles,
    float* __restrict__ out, int out_mode, unsigned long long* __restrict__ unit_key) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const XTile td = tiles[blockIdx.x];
    const UnitDev& U = units[td.unit];
    xform_generic_p1<T>(cells + U.cell_off, U, td, lds, threadIdx.x);
    __syncthreads();
    float* __restrict__ dst = out + out_base(U, out_mode);
    unsigned long long kmax = xform_generic_p2<KEYS>(U, td, lds, threadIdx.x, [&](int64_t f, float v) { dst[f] = v; });
    if constexpr (KEYS) {
        kmax = wave_max_u64(kmax);
        if (lane_id() == 0 && kmax != 0) atomicMax(unit_key + td.unit, kmax);
    }
}

// Even W, H, D with D % 8 == 0: 4 z-blocks per thread, 16-B LDS and global stores.
template <typename T, bool KEYS>
__global__ __launch_bounds__(kThreads) void k_transform_fast(
    const T* __restrict__ cells, const UnitDev* __restrict__ units, const XTile* __restrict__ tiles,
    float* __restrict__ out, int out_mode, unsigned long long* __restrict__ unit_key) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const XTile td = tiles[blockIdx.x];
    const UnitDev& U = units[td.unit];
    xform_fast_p1<T>(cells + U.cell_off, U, td, lds, threadIdx.x);
    __syncthreads();
    const uint64_t obase = out_base(U, out_mode);
    float* __restrict__ dst = out + obase;
    unsigned long long kmax;
    if ((obase & 3) == 0) {
        kmax = xform_fast_p2<KEYS>(U, td, lds, threadIdx.x,
                                   [&](int64_t f, float4 v) { *reinterpret_cast<float4*>(dst + f) = v; });
    } else {
        kmax = xform_fast_p2<KEYS>(U, td, lds, threadIdx.x, [&](int64_t f, float4 v) {
            dst[f] = v.x;
            dst[f + 1] = v.y;
            dst[f + 2] = v.z;
            dst[f + 3] = v.w;
        });
    }
    if constexpr (KEYS) {
        kmax = wave_max_u64(kmax);
        if (lane_id() == 0 && kmax != 0) atomicMax(unit_key + td.unit, kmax);
    }
}

// ---------------------------------------------------------------------------
// Launch wrappers
size_t transform_lds_bytes(int lbx, int lby, int lbz) {
    return (size_t)4 * (1 << lbx) * (1 << lby) * (2 * (1 << lbz) + 1) * sizeof(float);
}

size_t transform_fast_lds_bytes(int lbx, int lby, int lbz) {
    return (size_t)4 * (1 << lbx) * (1 << lby) * (2 * (1 << lbz) + 4) * sizeof(float);
}

hipError_t launch_transform(hipStream_t st, const void* cells, int dtype, const UnitDev* units,
                            const XTile* tiles, uint32_t ntiles, size_t lds, float* out,
                            int out_mode, unsigned long long* keys) {
    if (ntiles == 0) return hipSuccess;
    if (dtype == 1) {
        if (keys)
            k_transform<double, true><<<ntiles, kThreads, lds, st>>>((const double*)cells, units, tiles, out,
                                                                   out_mode, keys);
        else
            k_transform<double, false><<<ntiles, kThreads, lds, st>>>((const double*)cells, units, tiles, out,
                                                                    out_mode, keys);
    } else {
        if (keys)
            k_transform<float, true><<<ntiles, kThreads, lds, st>>>((const float*)cells, units, tiles, out,
                                                                  out_mode, keys);
        else
            k_transform<float, false><<<ntiles, kThreads, lds, st>>>((const float*)cells, units, tiles, out,
                                                                   out_mode, keys);
    }
    return hipGetLastError();
}

hipError_t launch_transform_fast(hipStream_t st, const void* cells, int dtype, const UnitDev* units,
                                 const XTile* tiles, uint32_t ntiles, size_t lds, float* out,
                                 int out_mode, unsigned long long* keys) {
    if (ntiles == 0) return hipSuccess;
    if (dtype == 1) {
        if (keys)
            k_transform_fast<double, true><<<ntiles, kThreads, lds, st>>>((const double*)cells, units, tiles, out,
                                                                        out_mode, keys);
        else
            k_transform_fast<double, false><<<ntiles, kThreads, lds, st>>>((const double*)cells, units, tiles, out,
                                                                         out_mode, keys);
    } else {
        if (keys)
            k_transform_fast<float, true><<<ntiles, kThreads, lds, st>>>((const float*)cells, units, tiles, out,
                                                                       out_mode, keys);
        else
            k_transform_fast<float, false><<<ntiles, kThreads, lds, st>>>((const float*)cells, units, tiles, out,
                                                                        out_mode, keys);
    }
    return hipGetLastError();
}

}  // namespace wc

// wc_transform.hip — K1: one-level 3-D Haar, cells -> flat coefficients.
//   k_transform       generic tiles (any dims, odd tails)     src/compressor.cpp:85-185
//   k_transform_fast  even dims, D % 8 == 0 (4 z-blocks per thread)
//   k_transform_hist  the fast tiles with the global-threshold mode's
//                     magnitude histogram folded in (wc_forward_stage)
// All also reduce the unit's max-|c| key (src/compressor.cpp:212-215).
// The tile bodies live in wc_xform.h.
//
// Numerics (bit-exact with the reference): the reference
// pair `(a + b) / 2.0` is a float add, an exact halving in double and one
// rounding to float == `(a + b) * 0.5f` here; built with -ffp-contract=off and
// -fno-gpu-flush-denormals-to-zero so subnormals round identically.
#include "wc_xform.h"

#include <algorithm>

namespace wc {

// Output position of a unit's flat coefficients: 0 the dense flat scratch
// (coef_off), 1 at the unit's cell offset (wc_decompose).
__device__ __forceinline__ uint64_t out_base(const UnitDev& U, int mode) {
    return mode == 1 ? U.cell_off : U.coef_off;
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
        __shared__ unsigned long long s_key[kThreads / kWave];
        block_key_max(kmax, s_key, unit_key + td.unit);
    }
}

// Even W, H, D with D % 8 == 0: 4 z-blocks per thread, 16-B LDS and global stores.
// flags != null (staged forward): units with U.sparse store only the flagged
// 32-coefficient segments (xform_fast_p2_sparse).
template <typename T, bool KEYS>
__global__ __launch_bounds__(kThreads) void k_transform_fast(
    const T* __restrict__ cells, const UnitDev* __restrict__ units, const XTile* __restrict__ tiles,
    float* __restrict__ out, int out_mode, unsigned long long* __restrict__ unit_key,
    uint8_t* __restrict__ flags, uint32_t* __restrict__ spos, double keep) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ unsigned long long s_key[kThreads / kWave];
    __shared__ uint32_t s_mag[kThreads / kWave];
    const XTile td = tiles[blockIdx.x];
    const UnitDev& U = units[td.unit];
    const uint64_t obase = out_base(U, out_mode);
    float* __restrict__ dst = out + obase;
    if constexpr (KEYS) {
        if (flags && U.sparse) {  // uniform; coef_off is 128-B aligned here
            const bool s32 = s32_ok(U);  // uniform: the 32 x 1 x 32 tile shape specialised
            uint32_t mag = s32 ? xform_fast_p1<T, false, true, true>(cells + U.cell_off, U, td, lds, threadIdx.x)
                               : xform_fast_p1<T, false, true>(cells + U.cell_off, U, td, lds, threadIdx.x);
            mag = wave_max_u32_u(mag);
            if ((threadIdx.x & 63) == 0) s_mag[threadIdx.x >> 6] = mag;
            __syncthreads();
            mag = max(max(s_mag[0], s_mag[1]), max(s_mag[2], s_mag[3]));
            const double bound = sparse_bound(mag, keep);
            if (threadIdx.x == 0 && bound >= 0.0) atomicOr(spos + td.unit, 1u);  // a sparsely staged tile
            // mag >> 1: the tile's largest |c| bits (NaN patterns above +inf's)
            const unsigned long long kmax =
                s32 ? xform_fast_p2_sparse_s32(U, td, lds, threadIdx.x, bound, mag >> 1, flags, dst)
                    : xform_fast_p2_sparse(U, td, lds, threadIdx.x, bound, mag >> 1, flags,
                                           [&](int64_t f, float4 v) { stage_store4(dst + f, v); });
            block_key_max(kmax, s_key, unit_key + td.unit);
            return;
        }
    }
    xform_fast_p1<T>(cells + U.cell_off, U, td, lds, threadIdx.x);
    __syncthreads();
    unsigned long long kmax;
    if ((obase & 3) == 0) {
        kmax = xform_fast_p2<KEYS>(U, td, lds, threadIdx.x,
                                   [&](int64_t f, float4 v) { stage_store4(dst + f, v); });
    } else {
        kmax = xform_fast_p2<KEYS>(U, td, lds, threadIdx.x, [&](int64_t f, float4 v) {
            dst[f] = v.x;
            dst[f + 1] = v.y;
            dst[f + 2] = v.z;
            dst[f + 3] = v.w;
        });
    }
    if constexpr (KEYS) block_key_max(kmax, s_key, unit_key + td.unit);
}

// Sparse-staged units whose thresh is < 0 (negative signed max, or keep > 1:
// every coefficient is kept, src/compressor.cpp:216-226) need every
// coefficient; those with a sparsely staged tile (spos: a tile whose own
// largest magnitude is negative stages densely, so this takes a unit whose
// tiles disagree in sign) are re-staged densely.  One launch checks and
// re-stages: workgroup b owns units b, b + G, b + 2G, ... (G = grid); its
// threads check 256 of them at once (one key load each), list the needy ones
// in LDS, and the workgroup re-stages those tile by tile.  With none, every
// workgroup exits after one round of loads.
template <typename T>
__global__ __launch_bounds__(kThreads) void k_transform_fallback(const T* __restrict__ cells,
                                                               const UnitDev* __restrict__ units, int n,
                                                               const XTile* __restrict__ tiles, float* __restrict__ out,
                                                               const unsigned long long* __restrict__ unit_key,
                                                               const uint32_t* __restrict__ spos, double keep) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ uint32_t s_list[kThreads];
    __shared__ uint32_t s_cnt;
    const int tid = threadIdx.x;
    for (int64_t base = blockIdx.x; base < n; base += (int64_t)gridDim.x * kThreads) {
        if (tid == 0) s_cnt = 0;
        __syncthreads();
        const int64_t u = base + (int64_t)tid * gridDim.x;
        if (u < n && spos[u] && key_thresh(unit_key[u], keep) < 0.0) s_list[atomicAdd(&s_cnt, 1u)] = (uint32_t)u;
        __syncthreads();
        const uint32_t cnt = s_cnt;
        for (uint32_t i = 0; i < cnt; ++i) {
            const UnitDev& U = units[s_list[i]];
            float* __restrict__ dst = out + U.coef_off;
            for (uint32_t t = 0; t < U.ntx; ++t) {
                const XTile td = tiles[U.xt_begin + t];
                xform_fast_p1<T>(cells + U.cell_off, U, td, lds, tid);
                __syncthreads();
                (void)xform_fast_p2<false>(U, td, lds, tid,
                                           [&](int64_t f, float4 v) { stage_store4(dst + f, v); });
                __syncthreads();
            }
        }
        __syncthreads();  // s_cnt / s_list reused by the next round
    }
}

// fp32 cells, fast tiles, persistent: a tile of fp32 cells is half the bytes
// of an fp64 one, so with the LDS-bound 4 tiles per CU the plain kernel keeps
// too few bytes in flight.  Each workgroup walks tiles t, t + grid, ... and
// loads tile t + grid's cells into registers before transforming tile t
// (two column buffers, alternating).
template <bool KEYS>
__global__ __launch_bounds__(kThreads) void k_transform_fast_pf(
    const float* __restrict__ cells, const UnitDev* __restrict__ units, const XTile* __restrict__ tiles,
    uint32_t ntiles, float* __restrict__ out, int out_mode, unsigned long long* __restrict__ unit_key) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ unsigned long long s_key[kThreads / kWave];
    const int tid = threadIdx.x;
    FastCol buf[2];
    uint32_t t = blockIdx.x;
    if (t >= ntiles) return;
    XTile td[2];
    bool have[2];
    td[0] = tiles[t];
    have[0] = fast_load<float>(cells + units[td[0].unit].cell_off, units[td[0].unit], td[0], tid, buf[0]);
    auto step = [&](int cb) {
        const int nb = cb ^ 1;
        const uint32_t tn = t + gridDim.x;
        have[nb] = false;
        if (tn < ntiles) {
            td[nb] = tiles[tn];
            const UnitDev& Un = units[td[nb].unit];
            have[nb] = fast_load<float>(cells + Un.cell_off, Un, td[nb], tid, buf[nb]);
        }
        const UnitDev& U = units[td[cb].unit];
        if (have[cb]) fast_butterfly(U, buf[cb], lds, tid);
        __syncthreads();
        const uint64_t obase = out_base(U, out_mode);
        float* __restrict__ dst = out + obase;
        unsigned long long kmax;
        if ((obase & 3) == 0) {
            kmax = xform_fast_p2<KEYS>(U, td[cb], lds, tid,
                                       [&](int64_t f, float4 v) { stage_store4(dst + f, v); });
        } else {
            kmax = xform_fast_p2<KEYS>(U, td[cb], lds, tid, [&](int64_t f, float4 v) {
                dst[f] = v.x;
                dst[f + 1] = v.y;
                dst[f + 2] = v.z;
                dst[f + 3] = v.w;
            });
        }
        if constexpr (KEYS) block_key_max(kmax, s_key, unit_key + td[cb].unit);
        __syncthreads();  // LDS rows reused by the next tile
        t = tn;
    };
    for (;;) {
        step(0);
        if (t >= ntiles) break;
        step(1);
        if (t >= ntiles) break;
    }
}

// The opt-in global-threshold mode's stage (wc_forward_stage with a
// histogram) over the fast tiles: dense staging, unit keys, AND the
// coefficient-magnitude histogram (wc_hist.hip's bins) folded into the store
// of phase 2, where every coefficient is already in registers, so no kernel
// re-reads the staged coefficients for it (4 B per coefficient saved).
// Workgroup b takes tiles b, b + G, ... with G = tiles / kHistTilesPerWg (at
// least the resident workgroups): its LDS bins (16 KiB past the tile rows) add
// up its ~32 tiles and reach `hist` once, as one 64-bit atomic per nonzero
// bin.  C4 K1: 8.38-8.43 ms at 32 tiles per workgroup, 8.44-8.46 at 16, 8.54-
// 8.60 at 64, 8.82-8.93 with a resident (persistent) grid, 12.5 at one tile
// per workgroup (the flush atomics) (profiles/r06/experiments/gpu_hist_tpw.txt).
template <typename T>
__global__ __launch_bounds__(kThreads) void k_transform_hist(
    const T* __restrict__ cells, const UnitDev* __restrict__ units, const XTile* __restrict__ tiles,
    uint32_t ntiles, uint32_t tile_floats, float* __restrict__ out, unsigned long long* __restrict__ unit_key,
    unsigned long long* __restrict__ hist) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ unsigned long long s_key[kThreads / kWave];
    uint32_t* __restrict__ h = reinterpret_cast<uint32_t*>(lds + tile_floats);
    const int tid = threadIdx.x;
    for (int i = tid; i < kHistBins; i += kThreads) h[i] = 0u;  // ordered before any add by the barrier after p1
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const XTile td = tiles[t];
        const UnitDev& U = units[td.unit];
        xform_fast_p1<T>(cells + U.cell_off, U, td, lds, tid);
        __syncthreads();
        float* __restrict__ dst = out + U.coef_off;  // 128-B aligned: 16-B stores
        const unsigned long long kmax = xform_fast_p2<true>(U, td, lds, tid, [&](int64_t f, float4 v) {
            stage_store4(dst + f, v);
            hist_add(h, v.x, true);
            hist_add(h, v.y, true);
            hist_add(h, v.z, true);
            hist_add(h, v.w, true);
        });
        block_key_max(kmax, s_key, unit_key + td.unit);  // its barrier: the rows are free for the next tile
    }
    __syncthreads();
    for (int i = tid; i < kHistBins; i += kThreads)
        if (h[i]) atomicAdd(hist + i, (unsigned long long)h[i]);
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

// Workgroups of k_transform_fast_pf that fit on the current device at once
// (keys and no-keys forms share the register budget; the caller caches it).
uint32_t transform_pf_grid(size_t lds) {
    int per_cu = 0, ncu = 0, dev = 0;
    (void)hipGetDevice(&dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_transform_fast_pf<true>, kThreads, lds) !=
            hipSuccess ||
        per_cu < 1)
        per_cu = 2;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1) ncu = 256;
    return (uint32_t)per_cu * (uint32_t)ncu;
}

// Dynamic LDS of k_transform_hist: the tile rows, then the bins.
size_t transform_hist_lds_bytes(size_t lds_fast) { return ((lds_fast + 15) & ~size_t(15)) + 4 * kHistBins; }

uint32_t transform_hist_grid(size_t lds) {
    int per_cu = 0, ncu = 0, dev = 0;
    (void)hipGetDevice(&dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_transform_hist<double>, kThreads, lds) !=
            hipSuccess ||
        per_cu < 1)
        per_cu = 2;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1) ncu = 256;
    return (uint32_t)per_cu * (uint32_t)ncu;
}

constexpr uint32_t kHistTilesPerWg = 32;

// grid: the resident workgroups of k_transform_hist (transform_hist_grid).
hipError_t launch_transform_hist(hipStream_t st, const void* cells, int dtype, const UnitDev* units,
                                 const XTile* tiles, uint32_t ntiles, size_t lds_fast, float* out,
                                 unsigned long long* keys, unsigned long long* hist, uint32_t grid) {
    if (ntiles == 0) return hipSuccess;
    const size_t lds = transform_hist_lds_bytes(lds_fast);
    const uint32_t tf = (uint32_t)((lds - 4 * kHistBins) / sizeof(float));
    const uint32_t g = std::min(ntiles, std::max({1u, grid, (ntiles + kHistTilesPerWg - 1) / kHistTilesPerWg}));
    if (dtype == 1)
        k_transform_hist<double><<<g, kThreads, lds, st>>>((const double*)cells, units, tiles, ntiles, tf, out, keys,
                                                           hist);
    else
        k_transform_hist<float><<<g, kThreads, lds, st>>>((const float*)cells, units, tiles, ntiles, tf, out, keys,
                                                          hist);
    return hipGetLastError();
}

hipError_t launch_transform_fast(hipStream_t st, const void* cells, int dtype, const UnitDev* units,
                                 const XTile* tiles, uint32_t ntiles, size_t lds, float* out,
                                 int out_mode, unsigned long long* keys, uint8_t* flags, uint32_t* spos, double keep,
                                 uint32_t pf_grid) {
    if (ntiles == 0) return hipSuccess;
    if (dtype != 1 && !flags) {  // fp32 cells, dense staging: persistent, next tile's cells in flight
        const uint32_t grid = std::min(ntiles, std::max(1u, pf_grid));
        if (keys)
            k_transform_fast_pf<true><<<grid, kThreads, lds, st>>>((const float*)cells, units, tiles, ntiles, out,
                                                                 out_mode, keys);
        else
            k_transform_fast_pf<false><<<grid, kThreads, lds, st>>>((const float*)cells, units, tiles, ntiles, out,
                                                                  out_mode, keys);
        return hipGetLastError();
    }
    if (dtype == 1) {
        if (keys)
            k_transform_fast<double, true><<<ntiles, kThreads, lds, st>>>((const double*)cells, units, tiles, out,
                                                                  out_mode, keys, flags, spos, keep);
        else
            k_transform_fast<double, false><<<ntiles, kThreads, lds, st>>>((const double*)cells, units, tiles, out,
                                                                  out_mode, keys, flags, spos, keep);
    } else {
        if (keys)
            k_transform_fast<float, true><<<ntiles, kThreads, lds, st>>>((const float*)cells, units, tiles, out,
                                                                  out_mode, keys, flags, spos, keep);
        else
            k_transform_fast<float, false><<<ntiles, kThreads, lds, st>>>((const float*)cells, units, tiles, out,
                                                                  out_mode, keys, flags, spos, keep);
    }
    return hipGetLastError();
}

hipError_t launch_transform_fallback(hipStream_t st, const void* cells, int dtype, const UnitDev* units, int n,
                                     const XTile* tiles, size_t lds, float* out, const unsigned long long* keys,
                                     const uint32_t* spos, double keep) {
    if (n == 0) return hipSuccess;
    const int grid = std::min(n, 2048);  // <= 4 workgroups per CU of the LDS-bound tile: one dispatch round
    if (dtype == 1)
        k_transform_fallback<double><<<grid, kThreads, lds, st>>>((const double*)cells, units, n, tiles, out, keys,
                                                                  spos, keep);
    else
        k_transform_fallback<float><<<grid, kThreads, lds, st>>>((const float*)cells, units, n, tiles, out, keys,
                                                                 spos, keep);
    return hipGetLastError();
}

}  // namespace wc

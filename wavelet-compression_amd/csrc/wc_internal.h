// wc_internal.h — device-side plan structures shared by the HIP kernels and
// the C-ABI host code.  Not part of the public boundary (include/wavelet_amd.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wc {

constexpr int kThreads = 256;          // 4 waves of 64 lanes
constexpr int kWave = 64;
constexpr int kMaxTileBlocks = 1024;   // 2x2x2 blocks per transform tile (8192 coefficients)
constexpr int kFlatTile = 4096;        // coefficients per threshold/compaction tile
constexpr int kFlatPerThread = kFlatTile / kThreads;  // 16 = 4 x float4

// One Box3D component in the batch, with its transform tiling.
// Blocks: the reference's axis sweeps pair (2b, 2b+1) on every axis
// (src/compressor.cpp:107-111), so coefficient (I,J,K) depends only on the
// 2x2x2 input block (I mod h, J mod h, K mod h); an odd axis adds one
// pass-through "tail" block at b = n/2.
struct UnitDev {
    uint64_t cell_off;   // element offset of the unit's cells
    uint64_t coef_off;   // element offset in the flat coefficient scratch (16-B aligned)
    uint64_t ncells;     // W*H*D
    int32_t nx, ny, nz;  // W, H, D
    int32_t hx, hy, hz;  // n/2 per axis (number of pairs)
    int32_t nbx, nby, nbz;  // blocks per axis = ceil(n/2)
    int32_t lbx, lby, lbz;  // log2 of the transform tile shape in blocks
    uint32_t ftile_begin;   // first flat (threshold/compaction) tile of this unit
    uint32_t nftiles;       // number of flat tiles = ceil(ncells / kFlatTile)
    uint64_t pay_off;       // payload slot: prefix of worst-case sizes, == 4 (mod 8)
    uint64_t tab_off;       // fused units: first row-table granule (4 rows per granule)
    uint32_t xt_begin;      // fused units: first tile in the fused tile list
    uint32_t ntile_u;       // fused units: tiles G of this unit
    int32_t ntz;            // z tiles per unit (segments per flat row half)
    int32_t fused;          // 1: handled by k_forward_fused, 0: staged path
};

// A transform tile: a (1<<lbx) x (1<<lby) x (1<<lbz) box of 2x2x2 blocks.
struct XTile {
    uint32_t unit;
    uint32_t bx0, by0, bz0;
};

// A flat tile: kFlatTile consecutive coefficients (flat order) of one unit.
struct FTile {
    uint32_t unit;
    uint32_t index;  // tile index within the unit
};

// Sentinel for a unit whose flat[0] is NaN: std::max_element then returns
// flat[0] itself (every comparison with NaN is false), so thresh is NaN.
constexpr unsigned long long kKeyNaNFirst = ~0ull;

// Error bits raised by kernels (ctx->d_err).
constexpr uint32_t kErrHeader = 1u;      // payload header disagrees with the unit
constexpr uint32_t kErrNegativeRun = 2u; // a run length < 0 (reference: UB)
constexpr uint32_t kErrTooManyPairs = 4u;// nrle > ncoeff
constexpr uint32_t kErrTimeout = 8u;     // a fused-kernel hand-off wait hit its bound

// The fused forward kernel keeps a unit's G tiles co-resident; cap G well
// below the resident grid (>= 1024 tiles of 256 threads on 256 CUs).
constexpr uint32_t kMaxFusedTiles = 256;
// ... and the unit's row table (one 14-bit record per flat row, kept in LDS).
constexpr uint64_t kMaxFusedRows = 4096;

// Parameter block of k_forward_fused (wc_fused.hip), filled by wc_capi.cpp.
struct FusedParams {
    const void* cells;
    const UnitDev* units;
    const XTile* tiles;           // fused tiles, unit-major
    uint32_t ntiles;
    int n;
    uint32_t* ticket;             // zeroed per call
    unsigned long long* keyslot;  // [ntiles], zeroed per call
    unsigned long long* table;    // row-table granules, zeroed per call
    uint8_t* payload;
    uint64_t* offsets;            // [n + 1]
    uint32_t* kept;               // [n]
    uint32_t* err;
    double keep;
};

}  // namespace wc

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
    uint64_t coef_off;   // element offset in the flat coefficient scratch (128-B aligned)
    uint64_t ncells;     // W*H*D
    int32_t nx, ny, nz;  // W, H, D
    int32_t hx, hy, hz;  // n/2 per axis (number of pairs)
    int32_t nbx, nby, nbz;  // blocks per axis = ceil(n/2)
    int32_t lbx, lby, lbz;  // log2 of the transform tile shape in blocks
    uint32_t ftile_begin;   // first flat tile (kFlatTile) of this unit: staged forward, decode, RMSE
    uint32_t nftiles;       // number of flat tiles = ceil(ncells / kFlatTile)
    uint64_t pay_off;       // payload slot: prefix of worst-case sizes, == 4 (mod 8)
    int32_t ntz;            // z tiles per unit
    int32_t fast;           // 1: even dims, D % 8 == 0 -> the fast transform body
    uint32_t ntx;           // transform tiles of the unit
    uint32_t xt_begin;      // first transform tile of the unit in the plan's tile list
    uint32_t et_begin;      // first emit tile (kEmitTile coefficients) of the unit
    uint32_t net;           // emit tiles = max(1, ceil(ncells / kEmitTile))
    uint32_t sparse;        // 1: staged forward stores only flagged 32-coefficient segments (wc_xform.h)
    // inverse (wc_inverse.hip)
    uint32_t dt_begin;      // first decode tile (kFlatTile pairs) of the unit: look-back status index
    uint32_t ndt;           // decode tiles launched for the unit
    int32_t rix;            // 1: row-indexed inverse (K5 row index + K6r), 0: dense flat scratch
    int32_t ilbx, ilby;     // log2 of K6r's tile in blocks along x and y (all of z)
    uint64_t row_off;       // first rowinfo entry of the unit (W*H + 1 entries)
    uint32_t rt_begin;      // first K6r tile of the unit (row-indexed units)
    uint32_t nrt;           // K6r tiles of the unit
    uint64_t dmagic;        // m | (31 + l) << 32: row = floor(position / D) = (position * m) >> (31 + l)
    uint64_t flag_off;      // sparse units: byte offset of the segment flags (whole 2048-coefficient blocks, flag_pos)
};

// A transform tile: a (1<<lbx) x (1<<lby) x (1<<lbz) box of 2x2x2 blocks.
struct XTile {
    uint32_t unit;
    uint32_t bx0, by0, bz0;
};

// A K6r tile (row-indexed inverse, wc_inverse.hip): everything the kernel
// needs about the tile and its unit in one record (one scalar load batch).
struct RTile {
    uint64_t row_off;   // the unit's first rowinfo entry
    uint64_t cell_off;  // the unit's first output cell
    uint32_t unit;
    int32_t bx0, by0;   // first block of the tile along x and y (all of z)
    int32_t W, H, D;
    int32_t lbx, lby;   // log2 of the tile's blocks along x and y
    int32_t tyv;        // blocks along y in this tile (<= 1 << lby at the unit's edge)
    uint32_t nat;       // index in unit order (the fused RMSE's partial-sum slot)
};

// LDS layout of a K6r tile: 4 wave regions of TX ranges of RS = TY*D + 4
// floats, regions 16 floats apart (bank offset), 16-B aligned.
#ifndef WC_RIX_RSPAD
#define WC_RIX_RSPAD 4   // floats between ranges (bank offset)
#endif
#ifndef WC_RIX_WRPAD
#define WC_RIX_WRPAD 16  // floats between wave regions
#endif
__host__ __device__ inline int rix_rs(int lby, int D) { return (D << lby) + WC_RIX_RSPAD; }
__host__ __device__ inline int rix_wr(int lbx, int lby, int D) { return (rix_rs(lby, D) << lbx) + WC_RIX_WRPAD; }

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

constexpr uint32_t kEpochMask = 0x3fffffffu;  // epoch bits of a look-back granule (wc_device.h granule_e)

#ifndef WC_EMIT_EW
#define WC_EMIT_EW 4  // waves per emit block of the small-unit launch (2048 coefficients per wave)
#endif
constexpr int kEmitTile = WC_EMIT_EW * 2048;  // coefficients per emit tile (32 per thread)
constexpr int kEmitTileBig = 16384;      // emit tile of units of >= kEmitBigCells (8 waves)
constexpr uint64_t kEmitBigCells = uint64_t(1) << 21;  // 128^3: longer tiles pay

// Parameter block of k_emit (wc_emit.hip), filled by wc_capi.cpp.
// An emit block: its tile and every unit field the emit reads, so that a
// block's first memory round trip (one uniform load) already yields the
// addresses of its flags, key and coefficients.
struct EmitDesc {
    uint64_t coef_off;  // the unit's staged coefficients (UnitDev::coef_off)
    uint64_t pay_off;   // the unit's payload slot
    uint32_t ncells;    // W*H*D (< 2^31)
    uint32_t unit;
    uint32_t index;     // tile index within the unit (the ordered form's)
    uint32_t et_begin;  // the unit's first look-back granule
    uint32_t net;       // emit tiles of the unit
    int32_t nx, ny, nz;
    uint32_t mode;      // bit 0: UnitDev::sparse; bits 1-3: lbz, log2 of the staged segment length;
                        // bits 8-15: the row divisor's shift (div_rows)
    uint32_t flag_off;  // UnitDev::flag_off (the plan keeps every flag range below 4 GiB)
    uint32_t row_off;   // the unit's first row-index entry (UnitDev::row_off; the plan keeps it < 2^32)
    uint32_t dmul;      // the row divisor's multiplier (div_rows; UnitDev::dmagic); row_shift 0: no row index
};
static_assert(sizeof(EmitDesc) == 64, "one 64-B descriptor per emit block (one scalar load)");

struct EmitParams {
    const UnitDev* units;
    const EmitDesc* edesc;         // emit blocks in launch order (interleaved, wc_capi.cpp build_etiles)
    int n;
    uint32_t ordered;              // 1: tile index from edesc (dispatch order), 0: from tickets[unit]
    uint32_t* tickets;             // per-unit tile tickets (ticket form), zeroed per call
    const unsigned long long* key; // unit max keys (wc_xform.h coef_key)
    unsigned long long* status;    // decoupled look-back granules, per emit tile, zeroed per call
    uint8_t* payload;
    uint64_t* offsets;             // [n + 1]
    uint32_t* kept;                // [n]
    uint32_t* err;                 // the context's error word (atomicOr; read and cleared at wc_synchronize)
    double keep;
    uint32_t use_gthresh;          // 1: every unit uses gthresh (global histogram mode), 0: reference rule
    float gthresh;                 // fp32 threshold: keep |c| > gthresh
    const uint8_t* flags;          // sparse-staging segment flags (null: every unit dense)
    uint2* rowinfo;                // wc_forward_rows: the payloads' row index out (null: not written);
                                   // unit u's entries at units[u].row_off, units with dmagic != 0
};

constexpr int kSegShift = 4;    // sparse staging: flag index space of 16 coefficients per byte (min segment)
// Byte position of sparse-staging segment s (= flat index >> sh, sh = log2 of
// the segment length, 4 or 5) in its unit's flag range: within
// each 2048-coefficient block of a unit (one emit wave's share of a tile) the
// 8 flags one emit thread reads (element groups it = 0..7: segment it * G + g,
// G = 256 >> sh, g = its lane group) sit in 8 consecutive bytes, g * 8 + it:
// one 8-B load instead of eight byte loads (wc_emit.hip).  Each sparse unit's
// flag range (UnitDev::flag_off) is 8-B aligned and spans whole blocks, so
// permuted positions never leave it.
__host__ __device__ inline uint64_t flag_pos(uint64_t s, int sh) {
    const int lb = 11 - sh, lg = 8 - sh;
    const uint64_t sw = s & ((1ull << lb) - 1);
    return (s & ~((1ull << lb) - 1)) | ((sw & ((1ull << lg) - 1)) << 3) | (sw >> lg);
}
// flag_pos on 32-bit segment indices (K1's S32 form: units of < 2^30 cells).
__host__ __device__ inline uint32_t flag_pos32(uint32_t s, int sh) {
    const int lb = 11 - sh, lg = 8 - sh;
    const uint32_t sw = s & ((1u << lb) - 1);
    return (s & ~((1u << lb) - 1)) | ((sw & ((1u << lg) - 1)) << 3) | (sw >> lg);
}
#ifndef WC_RIX_TILE
#define WC_RIX_TILE 4096
#endif
constexpr int kRixTile = WC_RIX_TILE;   // pairs per row-index (K5) tile
constexpr int kRixRounds5 = kRixTile / kThreads;
constexpr int kRixLds = 9216;   // K6r tile: default LDS budget in floats (36 KB: 4 workgroups per CU)

}  // namespace wc

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
    // pipelined forward (wc_pipe.hip)
    uint64_t ring_off;      // element offset of the unit's coefficients in the ring (chunk aligned)
    uint32_t ntx;           // transform tiles of the unit
    uint32_t et_begin;      // first emit tile (kEmitTile coefficients) of the unit
    uint32_t net;           // look-back emit tiles = max(1, ceil(ncells / kEmitTile)); 0 = packed whole
    uint32_t wl_off;        // ring wait list: units whose emit tiles must finish before
    uint32_t wl_len;        //   this unit's transform tiles overwrite their ring chunks
    uint32_t xt_begin;      // first transform tile of the unit in the plan's tile list
    uint32_t ewant;         // pipe: emit items of the unit (1 = one whole-unit item, else net tiles)
    uint32_t sparse;        // 1: staged forward stores only flagged 32-coefficient segments (wc_xform.h)
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

// Pipelined forward kernel (wc_pipe.hip).
constexpr int kEmitTile = 8192;          // coefficients per emit tile (32 per thread)
constexpr uint32_t kRingChunk = 4096;    // ring allocation granule (floats); one writer per chunk per lap

// Pipe diagnostics (s_memrealtime ticks, 100 MHz), summed over workgroups.
enum PipeStat {
    kStT = 0,        // transform items: ticks from start to end
    kStTWait,        // ... of which waiting for ring space
    kStE,            // emit items: ticks from start to end
    kStEWait,        // ... of which waiting for the unit's transform tiles
    kStELook,        // ... of which in the look-back
    kStClaim,        // waiting for a claimed ticket to return
    kStNT,           // transform items
    kStNE,           // emit items
    kPipeStats = 8
};

// Parameter block of k_forward_pipe, filled by wc_capi.cpp.
struct PipeParams {
    const void* cells;
    const UnitDev* units;
    const XTile* xtiles;           // transform tiles, unit-major
    const FTile* etiles;           // emit tiles, unit-major
    const uint32_t* items;         // work list: bit 31 set = emit tile, else transform tile
    const uint32_t* waits;         // ring wait lists (unit indices)
    float* ring;                   // coefficient ring (MALL-resident by size)
    uint32_t ring_bytes;
    uint32_t nitems;
    int n;
    uint32_t claim;                // items per ticket (consecutive), >= 1
    uint32_t prefetch;             // 1: claim the next batch while working on the current one
    unsigned long long* stats;     // optional (WC_OPT_PIPE_STATS): kPipeStats counters, or null
    // per-call state, zeroed by one memset: [ticket | key[n] | tdone[n] | edone[n] | status[net]]
    uint32_t* ticket;
    unsigned long long* key;       // unit max keys (wc_xform.h coef_key)
    uint32_t* tdone;               // transform tiles finished, per unit
    uint32_t* edone;               // emit tiles that finished reading the ring, per unit
    unsigned long long* status;    // decoupled look-back granules, per emit tile
    uint8_t* payload;
    uint64_t* offsets;             // [n + 1]
    uint32_t* kept;                // [n]
    uint32_t* err;
    double keep;
    const uint32_t* segs;          // k_emit: units packed whole, one workgroup each
    const uint32_t* eunits;        // k_emit: unit of each look-back block (interleaved order), or null
    const uint32_t* eidx;          // k_emit: tile index of each look-back block (same order as eunits)
    uint32_t seg_base;             // k_emit: first entry of segs in this launch
    uint32_t etile_base;           // k_emit: first look-back emit tile of this launch
    uint32_t ring_coefs;           // k_emit: 1 = coefficients at ring_off (chunk slots), 0 = coef_off
    uint32_t use_gthresh;          // 1: every unit uses gthresh (global histogram mode), 0: reference rule
    float gthresh;                 // fp32 threshold: keep |c| > gthresh
    const uint8_t* flags;          // k_emit: sparse-staging segment flags (null: every unit dense)
};

constexpr int kSegShift = 4;  // sparse staging: flag index space of 16 coefficients per byte (min segment)

}  // namespace wc

// wc_emit.hip — K2: keep threshold + ordered pack of the staged coefficients.
//
//   src/compressor.cpp:212-216  signed max, thresh  -> unit key (K1's 64-bit atomicMax) -> fp32 threshold
//   src/compressor.cpp:222-238  mask + rle_encode   -> emit tiles with decoupled look-back
//   src/compressor.cpp:55-80    serialize           -> header + pairs written in the unit's slot
//
// An emit tile is kEmitTile consecutive flat coefficients of one unit (flat
// order, x slowest / z fastest, src/compressor.cpp:178-181).  Per tile: load
// the staged coefficients (only the flagged segments under sparse staging),
// keep bits |c| > tf, publish (kept count, last kept index + 1) in the tile's
// 8-B look-back granule, sum the unit's earlier tiles' granules for the pair
// offset and the previous kept index, and write the (run, value) pairs
// contiguously (staged per wave in LDS).  The unit's last tile writes the
// header.
//
// Tile index within the unit, two runtime forms (wc_set_option WC_OPT_ORDERED):
//   1 (default): from the launch order.  Blocks are listed so that a tile's
//      look-back waits only on tiles of its unit with LOWER block ids, which
//      in-order dispatch has started.  No atomic per block.
//   0: from a per-unit ticket (atomicAdd): a tile's predecessors have always
//      started.  One atomic round trip per block.
// Neither form's progress depends on dispatch order: a predecessor that has
// not published within the wait bound is counted by the waiting wave itself
// from its staged coefficients (emit_tile_agg; DESIGN.md §Forward progress).
// P.ordered 2 (test hook WC_OPT_REVERSE_TILES): the launch-order form with
// each unit's tile indices reversed, the worst dispatch order for the waits.
#include "wc_emit.h"

namespace wc {

#ifndef WC_EMIT_MINB
#define WC_EMIT_MINB 8  // 4-wave launch: workgroups per CU the register budget is sized for (64 VGPRs)
#endif
#ifndef WC_EMIT_MINB_ROWS
#define WC_EMIT_MINB_ROWS 7  // the same with the row-index output (wc_forward_rows): 72 VGPRs
#endif
#ifndef WC_EMIT_MINB8
#define WC_EMIT_MINB8 2  // 8-wave launch (units of >= 2^21 cells)
#endif
// One block per emit tile (EW waves: EW * 2048 coefficients).  Block b packs
// the tile edesc[b] in the ordered form, or the next ticket of edesc[b]'s unit
// in the ticket form.  The plan lists blocks interleaved by tile index across
// the units of a group, groups in reverse transform order (wc_capi.cpp
// build_etiles); units of kEmitBigCells or more cells form the 8-wave launch.
// ROWS (wc_forward_rows): the emit also writes the payloads' row index.
template <int EW, bool ROWS>
__global__ __launch_bounds__(EW * kWave, EW == 8 ? WC_EMIT_MINB8 : (ROWS ? WC_EMIT_MINB_ROWS : WC_EMIT_MINB)) void k_emit(EmitParams P,
                                                                           const float* __restrict__ coef) {
    __shared__ __attribute__((aligned(16))) uint32_t sm[32];
    __shared__ uint2 stage_all[EW][256 * WC_EMIT_SB];  // per-wave pair stage (emit_pairs)
    const int tid = threadIdx.x;
    uint2* stage = stage_all[tid >> 6];
    const EmitDesc E = P.edesc[blockIdx.x];
    if (P.ordered) {
        emit_tile<EW, ROWS>(P, PlainSrc{coef}, E, P.ordered == 2 ? E.net - 1u - E.index : E.index, sm, stage, tid);
        return;
    }
    if (tid == 0) sm[31] = atomicAdd(P.tickets + E.unit, 1u);
    __syncthreads();
    const uint32_t index = __builtin_amdgcn_readfirstlane(sm[31]);
    emit_tile<EW, ROWS>(P, PlainSrc{coef}, E, index, sm, stage, tid);
}

hipError_t launch_emit(hipStream_t st, const EmitParams& p, const float* coef, uint32_t nsmall, uint32_t nbig) {
    static_assert(kEmitTile == WC_EMIT_EW * 2048 && kEmitTileBig == 8 * 2048, "emit tile sizes");
    EmitParams q = p;
    q.edesc = p.edesc + nsmall;
    if (p.rowinfo) {
        if (nsmall) k_emit<WC_EMIT_EW, true><<<nsmall, WC_EMIT_EW * kWave, 0, st>>>(p, coef);
        if (nbig) k_emit<8, true><<<nbig, 8 * kWave, 0, st>>>(q, coef);
    } else {
        if (nsmall) k_emit<WC_EMIT_EW, false><<<nsmall, WC_EMIT_EW * kWave, 0, st>>>(p, coef);
        if (nbig) k_emit<8, false><<<nbig, 8 * kWave, 0, st>>>(q, coef);
    }
    return hipGetLastError();
}

}  // namespace wc

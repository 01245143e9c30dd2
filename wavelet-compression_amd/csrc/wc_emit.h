// wc_emit.h — the emit tile body (K2: keep threshold + ordered pack of staged
// coefficients) of k_emit (wc_emit.hip).  See wc_emit.hip for the algorithm
// and its reference lines.
#pragma once

#include "wc_xform.h"

#ifndef WC_EMIT_SB
#define WC_EMIT_SB 2  // 256-element blocks whose pairs share one copy-out (stage: 256 * WC_EMIT_SB pairs per wave)
#endif
#ifndef WC_EMIT_KEYPAR
#define WC_EMIT_KEYPAR 1  // the unit key loads beside the flags (bit 0: 4-wave launch, bit 1: 8-wave: +11 VGPRs there)
#endif

namespace wc {


// fp32 keep threshold of a unit: the reference rule from the unit's max key
// (src/compressor.cpp:212-216), or the one global threshold of the opt-in
// histogram mode (wc_forward_emit with a threshold).
__device__ __forceinline__ float unit_thresh(const EmitParams& P, unsigned long long key) {
    return P.use_gthresh ? P.gthresh : thresh_as_float(key_thresh(key, P.keep));
}

// Set bits of a 64-lane mask below this lane.
__device__ __forceinline__ uint32_t mbcnt64(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Row-index output of one unit (wc_forward_rows; dmagic == 0: none): its
// entries, the Granlund-Montgomery constant of D, and D.
struct RowOut {
    uint2* __restrict__ ri;
    uint64_t dmagic;
    uint32_t D;
};

// Emit the kept coefficients of one kEmitTile chunk held in q (thread (w, l)
// owns elements w*2048 + it*256 + 4l + j; kb bit it*4 + j = kept) as (run,
// value) pairs: ranks from per-column ballots, run = f - prev - 1 (taken at
// the copy-out from the staged indices: no per-block scan).  rank /
// prev: this wave's first pair index and the unit-relative flat index of the
// last kept coefficient before this wave's elements (0xffffffff = none, so
// that run = f).  32-bit arithmetic: flat indices are < 2^31.
// The pairs of every WC_EMIT_SB consecutive 256-element blocks are first
// placed in this wave's LDS stage in rank order, then copied out with
// contiguous 8-B stores (one full 512-B row per instruction instead of up to
// four sparse, partial-line scatters; two blocks per copy-out fill the last
// row of a copy better).  A wave's LDS operations execute in order, so the
// stage needs no barrier.
//
// kRows (wc_forward_rows): pair k = rank + i at flat index f, the previous
// pair's index pf, also writes the row entries of the rows whose first flat
// position lies in (pf, f] (write_rows, wc_device.h): (k, f - r*D).
template <bool kRows>
__device__ __forceinline__ void emit_pairs(const float4 (&q)[8], uint32_t kb, uint32_t start, int w, int l,
                                           uint32_t rank, uint32_t prev, uint2* __restrict__ pairs, uint2* stage,
                                           const RowOut& ro) {
    uint32_t soff = 0;  // pairs staged since the last copy-out
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const uint32_t nib = (kb >> (it * 4)) & 0xfu;
        const unsigned long long any = __ballot(nib != 0);
        if (any) {
            // exclusive prefix of kept counts over lanes: one ballot per column j,
            // counted below this lane with mbcnt (ballots live in SGPRs)
            const unsigned long long b0 = __ballot(nib & 1u), b1 = __ballot(nib & 2u), b2 = __ballot(nib & 4u),
                                     b3 = __ballot(nib & 8u);
            const uint32_t pre = mbcnt64(b0) + mbcnt64(b1) + mbcnt64(b2) + mbcnt64(b3);
            const uint32_t itot = (uint32_t)(__popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3));
            const uint32_t ebase = start + (uint32_t)(w * 2048 + it * 256 + l * 4);
            uint32_t r = soff + pre;
            // staged as (flat index, value); runs are taken at the copy-out
            if (nib) {
                const float vv[4] = {q[it].x, q[it].y, q[it].z, q[it].w};
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (nib & (1u << j)) stage[r++] = make_uint2(ebase + (uint32_t)j, __float_as_uint(vv[j]));
            }
            soff += itot;
        }
        // copy-out every WC_EMIT_SB blocks of 256 elements (the stage holds their pairs)
        if (it % WC_EMIT_SB == WC_EMIT_SB - 1 && soff) {
            __builtin_amdgcn_wave_barrier();
            {
                // run = f - (previous pair's f) - 1: the previous pair is lane
                // l - 1's (a whole-wave DPP shift), for lane 0 the carry (the
                // last pair of the previous round, or prev)
                uint32_t carry = prev;
                uint2 e = make_uint2(0u, 0u);
                for (uint32_t k0 = 0; k0 < soff; k0 += 64) {  // uniform rounds, every lane active
                    const uint32_t k = k0 + (uint32_t)l;
                    e = k < soff ? stage[k] : make_uint2(0u, 0u);
                    const uint32_t left = dpp_u32<0x138, 0xf>(e.x);  // wave_shr:1
                    const uint32_t pf = l == 0 ? carry : left;
                    if (k < soff) pairs[rank + k] = make_uint2(e.x - pf - 1u, e.y);
                    if constexpr (kRows) {
                        if (ro.dmagic) {  // uniform: rows (floor(pf / D), floor(f / D)] start in (pf, f]
                            const int32_t rhi = k < soff ? (int32_t)div_rows(e.x, ro.dmagic) : -1;
                            const int32_t rlo = pf == 0xffffffffu ? 0 : (int32_t)div_rows(pf, ro.dmagic) + 1;
                            write_rows(ro.ri, (uint32_t)rlo, rhi >= rlo ? (uint32_t)(rhi - rlo + 1) : 0u, rank + k,
                                       e.x, ro.D, l);
                        }
                    }
                    carry = __builtin_amdgcn_readlane(e.x, 63);
                }
                prev = __builtin_amdgcn_readlane(e.x, (soff - 1u) & 63u);  // the last pair's index
            }
            __builtin_amdgcn_wave_barrier();
            rank += soff;
            soff = 0;
        }
    }
}

// Keep bits of a chunk: bit it*4 + j of element w*2048 + it*256 + 4l + j,
// |c| > tf for elements below len (src/compressor.cpp:225-226).
__device__ __forceinline__ uint32_t keep_bits(const float4 (&q)[8], float tf, uint32_t len, int w, int l) {
    uint32_t kb = 0;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const float e[4] = {q[it].x, q[it].y, q[it].z, q[it].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t idx = (uint32_t)(w * 2048 + it * 256 + l * 4 + j);
            kb |= (uint32_t)(idx < len && fabsf(e[j]) > tf) << (it * 4 + j);
        }
    }
    return kb;
}

// keep_bits of a full chunk (len == EW * 2048: every element in range).
__device__ __forceinline__ uint32_t keep_bits_full(const float4 (&q)[8], float tf) {
    uint32_t kb = 0;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        kb |= (uint32_t)(fabsf(q[it].x) > tf) << (it * 4);
        kb |= (uint32_t)(fabsf(q[it].y) > tf) << (it * 4 + 1);
        kb |= (uint32_t)(fabsf(q[it].z) > tf) << (it * 4 + 2);
        kb |= (uint32_t)(fabsf(q[it].w) > tf) << (it * 4 + 3);
    }
    return kb;
}

// Per-wave kept count and last kept (chunk-relative index + 1, 0 = none).
__device__ __forceinline__ void wave_totals(uint32_t kb, int w, int l, uint32_t& cnt, uint32_t& last) {
    cnt = wave_sum_u32_u((uint32_t)__popc(kb));
    const int hb = kb ? 31 - __clz(kb) : 0;
    last = wave_max_u32_u(kb ? (uint32_t)(w * 2048 + (hb >> 2) * 256 + l * 4 + (hb & 3) + 1) : 0u);
}

// Unit E.unit's header (src/compressor.cpp:55-80: int32 W, H, D, ncoeff,
// nrle), kept count and payload offset, once its pair count is known.
__device__ __forceinline__ void finish_unit(const EmitParams& P, const EmitDesc& E, uint32_t total) {
    const uint32_t u = E.unit;
    int32_t* hd = reinterpret_cast<int32_t*>(P.payload + E.pay_off);
    hd[0] = E.nx;
    hd[1] = E.ny;
    hd[2] = E.nz;
    hd[3] = (int32_t)E.ncells;
    hd[4] = (int32_t)total;
    P.kept[u] = total;
    P.offsets[u] = E.pay_off;
    if ((int)u == P.n - 1) P.offsets[P.n] = E.pay_off + 20 + 8ull * total;
}

constexpr unsigned long long kMask31 = 0x7fffffffull;

// Staged-coefficient source of emit_tile: coefficients and unit keys written
// by EARLIER launches (K1), read with plain (and scalar) loads.
struct PlainTile {
    const float4* __restrict__ p;
    __device__ __forceinline__ float4 operator[](int i) const {
        // the staged coefficients' last use: nontemporal (emit -8 % at C2, -11 % at C3,
        // profiles/r05/experiments/gpu_nt.txt; nontemporal payload stores measured +7 %: not used)
        const f32x4 x = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + i));
        return make_float4(x.x, x.y, x.z, x.w);
    }
};
struct PlainSrc {
    const float* __restrict__ coef;
    __device__ __forceinline__ unsigned long long key(const EmitParams& P, uint32_t u) const { return P.key[u]; }
    __device__ __forceinline__ PlainTile tile(const EmitDesc& U, uint32_t start) const {
        return PlainTile{reinterpret_cast<const float4*>(coef + U.coef_off + start)};
    }
    __device__ __forceinline__ const float* unit_coef(const EmitDesc& U) const { return coef + U.coef_off; }
    __device__ __forceinline__ void consumed(const EmitDesc&, int) const {}
};

// The look-back aggregate of full tile j of unit U (kept count, unit-relative
// last kept index + 1 or 0), derived by one wave from the tile's staged
// coefficients exactly as its own block counts them: the look-back's path
// when tile j has not published within the wait bound (its block may not have
// been dispatched).  Elements of unflagged segments of a sparse unit were
// never staged and count as 0, as in emit_tile.  Rare: one 4-B load per lane
// per 64 elements and a ballot.
template <int EW>
__device__ __forceinline__ uint2 emit_tile_agg(const uint8_t* __restrict__ flags, const float* __restrict__ c,
                                                         uint32_t flag_off, uint32_t j, int sh, bool dense, float tf,
                                                         int l) {
    constexpr uint32_t kTile = EW * 2048;
    const uint32_t s0 = j * kTile;
    const float* __restrict__ ct = c + s0;
    uint32_t C = 0, L = 0;
#pragma unroll 1
    for (uint32_t e0 = 0; e0 < kTile; e0 += 64) {  // one load per step: the 4-wave emit has no VGPR to spare
        // a sparse unit's flag of this lane's segment (unflagged: never staged, counts as 0)
        bool on = true;
        if (!dense) on = flags[flag_off + flag_pos32((s0 + e0 + (uint32_t)l) >> sh, sh)] != 0;
        const float v = on ? ct[e0 + (uint32_t)l] : 0.0f;
        const unsigned long long b = __ballot(fabsf(v) > tf);
        C += (uint32_t)__popcll(b);
        if (b) L = e0 + 64u - (uint32_t)__clzll(b);
    }
    return make_uint2(C, L ? s0 + L : 0u);
}


// Threshold + ordered pack of tile `index` of unit `u`.  Thread t = (wave w,
// lane l) owns elements w*2048 + it*256 + 4l + j, it 0..7.  sm: 16 LDS words.
// kRows: also the unit's row index (P.rowinfo; the pairs' rows in
// emit_pairs, the rows after the unit's last pair by its last tile).
template <int EW, bool kRows, class Src>
__device__ __forceinline__ void emit_tile(const EmitParams& P, const Src& src, const EmitDesc& U, uint32_t index,
                                          uint32_t* sm, uint2* stage, int tid) {
    constexpr uint32_t kTile = EW * 2048;
    const uint32_t u = U.unit;
    const uint32_t et = U.et_begin + index;
    const int w = tid >> 6, l = tid & 63;
    // Sparse staging: this thread's 8 segment flags, loaded before the key.
    const bool sparse = P.flags && (U.mode & 1u);
    constexpr bool kKeyPar = (WC_EMIT_KEYPAR >> (EW == 8 ? 1 : 0)) & 1;
    // The key's scalar load is issued with the flag load, and the threshold is
    // needed only by the keep test: the chain before the coefficient loads is
    // descriptor -> flags (not descriptor -> flags -> key).  A unit whose
    // thresh is < 0 (densely re-staged, k_transform_fallback) loads the
    // segments its flags skipped once the threshold is known (rare).
    unsigned long long ukey = 0;
    if constexpr (kKeyPar) ukey = src.key(P, u);
    RowOut ro{nullptr, 0ull, 0u};
    if constexpr (kRows) {  // from the descriptor (a load of the unit's record would stall the tile's start)
        ro.dmagic = (uint64_t)U.dmul | ((uint64_t)((U.mode >> 8) & 0xffu) << 32);
        ro.ri = P.rowinfo + U.row_off;
        ro.D = (uint32_t)U.nz;
    }
    uint32_t segf = 0xffu;  // bit it: group it may hold kept coefficients
    if (sparse) {
        // one flag byte per segment of TZ = 2^lbz coefficients (16 or 32)
        const int sh = (int)((U.mode >> 1) & 7u);  // lbz
        const uint8_t* fl = P.flags + U.flag_off + (((uint64_t)index * kTile) >> sh);
        // this thread's 8 flags in 8 consecutive bytes (flag_pos): bytes 0 / 1
        const uint2 f8 = *reinterpret_cast<const uint2*>(fl + ((uint32_t)w << (11 - sh)) + ((((uint32_t)l << 2) >> sh) << 3));
        segf = (f8.x & 1u) | ((f8.x >> 7) & 2u) | ((f8.x >> 14) & 4u) | ((f8.x >> 21) & 8u) | ((f8.y & 1u) << 4) |
               ((f8.y >> 3) & 0x20u) | ((f8.y >> 10) & 0x40u) | ((f8.y >> 17) & 0x80u);
    }
    // the unit key: a finished earlier launch wrote it, one uniform load
    float tf = 0.0f;
    if constexpr (!kKeyPar) tf = unit_thresh(P, src.key(P, u));
    const uint32_t start = index * kTile;
    const uint32_t len = min(kTile, U.ncells - start);

    // 1. coefficients -> keep bits (bit it*4 + j).  The flat scratch is 16-B
    // aligned per unit with kFlatTile slack past the last unit.  Sparse units
    // with thresh >= 0 skip unflagged segments (never stored); thresh < 0
    // units were re-staged densely (k_transform_fallback).
    const auto p4 = src.tile(U, start);  // p4[i]: float4 i of the tile (Src::Tile)
    if constexpr (!kKeyPar)
        if (!(tf >= 0.0f)) segf = 0xffu;
    float4 q[8];
    uint32_t kb;
    if (len == kTile) {  // uniform: a full tile, no range checks
#pragma unroll
        for (int it = 0; it < 8; ++it)
            q[it] = ((segf >> it) & 1u) ? p4[w * 512 + it * 64 + l] : make_float4(0, 0, 0, 0);
        if constexpr (kKeyPar) {
            tf = unit_thresh(P, ukey);
            if (!(tf >= 0.0f) && sparse) {  // uniform: the densely re-staged unit, every segment
#pragma unroll
                for (int it = 0; it < 8; ++it) q[it] = p4[w * 512 + it * 64 + l];
            }
        }
        kb = keep_bits_full(q, tf);
    } else {
#pragma unroll
        for (int it = 0; it < 8; ++it)
            q[it] = ((segf >> it) & 1u) && (uint32_t)(w * 2048 + it * 256 + 4 * l) < len ? p4[w * 512 + it * 64 + l]
                                                                                          : make_float4(0, 0, 0, 0);
        if constexpr (kKeyPar) {
            tf = unit_thresh(P, ukey);
            if (!(tf >= 0.0f) && sparse) {
#pragma unroll
                for (int it = 0; it < 8; ++it)
                    q[it] = (uint32_t)(w * 2048 + it * 256 + 4 * l) < len ? p4[w * 512 + it * 64 + l]
                                                                          : make_float4(0, 0, 0, 0);
            }
        }
        kb = keep_bits(q, tf, len, w, l);
    }
    uint32_t wcnt, wlast;
    wave_totals(kb, w, l, wcnt, wlast);
    if (l == 0) {
        sm[4 + w] = wcnt;
        sm[4 + EW + w] = wlast;
    }
    __syncthreads();
    src.consumed(U, tid);  // every wave's coefficient loads have returned (their values are counted)

    // 2. publish the aggregate, look back over the unit's earlier tiles (wave 0)
    if (w == 0) {
        uint32_t C = 0, L = 0;
#pragma unroll
        for (int i = 0; i < EW; ++i) {
            C += sm[4 + i];
            L = sm[4 + EW + i] > L ? sm[4 + EW + i] : L;
        }
        const uint32_t L1 = L ? start + L : 0u;  // unit-relative last kept + 1
        uint32_t ecnt = 0, elast = 0;            // exclusive: pairs before, last kept + 1 before
        if (index == 0) {
            if (l == 0) st_rlx(P.status + et, kFlagIncl | ((unsigned long long)C << 31) | L1);
        } else {
            if (l == 0) st_rlx(P.status + et, kFlagAgg | ((unsigned long long)C << 31) | L1);
            int32_t pos = (int32_t)et - 1;  // emit tiles of a launch: < 2^31
            const int32_t first = (int32_t)U.et_begin;
            // Window of the 64 nearest predecessors (lane l = tile et-1-l; tiles
            // before the unit read as an inclusive 0).  Lanes up to the nearest
            // inclusive one are summed once every one of them has published;
            // a run of published aggregates before the first unpublished tile
            // is summed and the window slides past it.  A tile still
            // unpublished after the wait bound is derived here and published
            // (publish_derived, wc_device.h), and any progress restarts the bound.
            for (uint32_t spins = 0;;) {
                const int32_t idx = pos - l;
                const unsigned long long v = idx >= first ? ld_rlx(P.status + idx) : kFlagIncl;
                const unsigned long long incl = __ballot((v >> 62) == 2);
                const unsigned long long zero = __ballot((v >> 62) == 0);
                const int kI = incl ? __ffsll((long long)incl) - 1 : 64;
                const int kZ = zero ? __ffsll((long long)zero) - 1 : 64;
                const int take = kI < kZ ? kI + 1 : kZ;  // lanes [0, take) are summed
                if (take > 0) {
                    const bool in = l < take;
                    ecnt += wave_sum_u32_u(in ? (uint32_t)((v >> 31) & kMask31) : 0u);
                    const unsigned long long hasl = __ballot(in && (v & kMask31) != 0);
                    const uint32_t hl = __builtin_amdgcn_readlane((uint32_t)(v & kMask31),
                                                                  hasl ? __ffsll((long long)hasl) - 1 : 0);  // uniform lane
                    if (elast == 0 && hasl) elast = hl;
                    spins = 0;
                }
                if (kI < kZ) break;
                pos -= take;
                if (take == 0 && spin_wait(spins, P.err)) {  // tile pos (lane 0's) unpublished: derive it here
                    const uint2 a = emit_tile_agg<EW>(P.flags, src.unit_coef(U), U.flag_off,
                                                      (uint32_t)(pos - first), (int)((U.mode >> 1) & 7u),
                                                      !sparse || !(tf >= 0.0f), tf, l);
                    if (l == 0) publish_derived(P.status + pos, v, kFlagAgg | ((unsigned long long)a.x << 31) | a.y);
                    ecnt += a.x;
                    if (elast == 0 && a.y) elast = a.y;
                    --pos;
                }
            }
            if (l == 0)
                st_rlx(P.status + et, kFlagIncl | ((unsigned long long)(ecnt + C) << 31) | (L1 ? L1 : elast));
        }
        if (l == 0) {
            sm[0] = ecnt;
            sm[1] = elast;
            if (index + 1 == U.net) {  // last tile
                finish_unit(P, U, ecnt + C);
                sm[2] = ecnt + C;           // the unit's pair count
                sm[3] = L1 ? L1 : elast;    // its last kept flat index + 1 (0: none)
            }
        }
    }
    __syncthreads();

    // 3. emit (run, value) pairs: ranks from wave ballots, run = f - prev - 1.
    // Flat indices are unit-relative and < 2^31: 32-bit arithmetic, with
    // "no previous kept" = 0xffffffff so that run = f - prev - 1 = f.
    uint32_t rank = sm[0];
    uint32_t prev = sm[1] - 1u;
    for (int i = 0; i < w; ++i) {
        rank += sm[4 + i];
        if (sm[4 + EW + i]) prev = start + sm[4 + EW + i] - 1u;
    }
    if constexpr (kRows) {  // wave-uniform: scalar registers
        rank = __builtin_amdgcn_readfirstlane(rank);
        prev = __builtin_amdgcn_readfirstlane(prev);
    }
    uint2* __restrict__ pairs = reinterpret_cast<uint2*>(P.payload + U.pay_off + 20);
    emit_pairs<kRows>(q, kb, start, w, l, rank, prev, pairs, stage, ro);
    if constexpr (kRows) {
        // the rows after the unit's last pair and the sentinel row W*H: (nrle,
        // ncoeff - r*D), as the virtual pair k = nrle at position ncoeff
        if (ro.dmagic && index + 1 == U.net) {  // uniform
            const uint32_t total = sm[2], last1 = sm[3];
            const uint32_t rows = (uint32_t)U.nx * (uint32_t)U.ny;
            const uint32_t nc = (uint32_t)U.ncells;
            for (uint32_t r = (last1 ? div_rows(last1 - 1u, ro.dmagic) + 1u : 0u) + (uint32_t)tid; r <= rows;
                 r += EW * kWave)
                ro.ri[r] = make_uint2(total, nc - r * ro.D);
        }
    }
}


}  // namespace wc

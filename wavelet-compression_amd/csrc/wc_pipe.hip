// wc_pipe.hip — pipelined forward path: transform + keep threshold + ordered
// pack for a whole batch in ONE persistent launch.
//
//   src/compressor.cpp:85-185  wavelet_decompose  -> transform items (wc_xform.h bodies)
//   src/compressor.cpp:212-216 signed max, thresh -> unit max key (64-bit atomicMax)
//   src/compressor.cpp:222-238 mask + rle_encode  -> emit items (decoupled look-back)
//   src/compressor.cpp:55-80   serialize          -> header + pairs written in the unit's slot
//
// The work list (built on the host, wc_capi.cpp) interleaves two streams:
//   T(u, g): transform tile g of unit u: read its cells once, transform, write
//            the fp32 coefficients into the unit's region of a coefficient
//            RING (write-through sc1 stores), fold its max key into key[u],
//            count tdone[u].
//   E(u, e): emit tile e of unit u = kEmitTile consecutive flat coefficients:
//            wait tdone[u] == ntx (all transform tiles of u), thresh from
//            key[u], read its coefficients from the ring (sc1 loads), count,
//            decoupled look-back over the unit's earlier emit tiles for the
//            pair offset and the previous kept index, emit (run, value) pairs.
// E items of a unit are placed `lag` cells of transform work after its last
// T item, so by the time an E item runs its unit is long finished: the waits
// confirm instead of block.  The ring is sized to a few tens of MB so the
// coefficients stay in the 256 MiB Infinity Cache between their write and
// read; a T item that reuses ring chunks first waits until the units that
// last wrote them have finished their emit reads (wait lists).
//
// Items are claimed in list order from one ticket counter, and every wait
// is on an item EARLIER in the list: the earliest unfinished item never
// waits, so the grid drains whatever the residency.  Every spin is bounded
// and raises kErrTimeout.
//
// Hand-offs (MI355X_MICROARCH.md, Valid forms, table row 1): ring stores are
// 16-B sc1 buffer stores drained by every storing wave before the workgroup
// barrier and the one-lane tdone add; consumers poll tdone with an sc1 load
// and read the ring only with sc1 loads after a barrier.  Look-back status
// words are self-validating 8-byte granules (R2).
#include "wc_xform.h"

namespace wc {

namespace {

constexpr unsigned long long kMask31 = 0x7fffffffull;

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Ring access: buffer instructions with aux = 16 (sc1): stores write through
// to the memory side, loads bypass this CU's L1.
__device__ __forceinline__ void ring_st4(__amdgpu_buffer_rsrc_t r, uint32_t byte, float4 v) {
    u32x4 d;
    d.x = __float_as_uint(v.x);
    d.y = __float_as_uint(v.y);
    d.z = __float_as_uint(v.z);
    d.w = __float_as_uint(v.w);
    __builtin_amdgcn_raw_buffer_store_b128(d, r, (int)byte, 0, 16);
}
__device__ __forceinline__ void ring_st1(__amdgpu_buffer_rsrc_t r, uint32_t byte, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)byte, 0, 16);
}
__device__ __forceinline__ float4 ring_ld4(__amdgpu_buffer_rsrc_t r, uint32_t byte) {
    const u32x4 d = __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte, 0, 16);
    return make_float4(__uint_as_float(d.x), __uint_as_float(d.y), __uint_as_float(d.z), __uint_as_float(d.w));
}

// fp32 keep threshold of a unit: the reference rule from the unit's max key
// (src/compressor.cpp:212-216), or the one global threshold of the opt-in
// histogram mode (wc_forward_emit with a threshold).
__device__ __forceinline__ float unit_thresh(const PipeParams& P, unsigned long long key) {
    return P.use_gthresh ? P.gthresh : thresh_as_float(key_thresh(key, P.keep));
}

__device__ __forceinline__ unsigned long long now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

// ---------------------------------------------------------------------------
// T item: transform tile `xt` into the ring.
template <typename T>
__device__ __forceinline__ void pipe_transform(const PipeParams& P, __amdgpu_buffer_rsrc_t ring, uint32_t xt,
                                               float* lds, int tid, unsigned long long* st, bool claim,
                                               uint32_t& next) {
    const XTile td = P.xtiles[xt];
    const UnitDev& U = P.units[td.unit];
    const T* src = static_cast<const T*>(P.cells) + U.cell_off;
    if (U.fast)
        xform_fast_p1<T, false>(src, U, td, lds, tid);
    else
        xform_generic_p1<T>(src, U, td, lds, tid);
    const int lane = tid & 63;
    // Ring reuse: the units that last wrote this unit's chunks must have
    // finished reading them (their emit tiles sit earlier in the list).
    if (tid < 64 && U.wl_len) {
        const unsigned long long t0 = P.stats ? now_ticks() : 0;
        for (uint32_t i0 = 0; i0 < U.wl_len; i0 += 64) {
            const uint32_t i = i0 + lane;
            const bool need = i < U.wl_len;
            const uint32_t v = need ? P.waits[U.wl_off + i] : 0u;
            const uint32_t want = need ? P.units[v].ewant : 0u;
            for (uint32_t spins = 0;;) {
                const bool ok = !need || ld_rlx(P.edone + v) >= want;
                if (__all(ok)) break;
                if (spin_fail(spins, P.err)) break;
            }
        }
        if (P.stats && tid == 0) st[kStTWait] += now_ticks() - t0;
    }
    __syncthreads();
    const uint32_t base = 4u * (uint32_t)U.ring_off;
    unsigned long long kmax;
    if (U.fast)
        kmax = xform_fast_p2<true>(U, td, lds, tid,
                                   [&](int64_t f, float4 v) { ring_st4(ring, base + 4u * (uint32_t)f, v); });
    else
        kmax = xform_generic_p2<true>(U, td, lds, tid,
                                      [&](int64_t f, float v) { ring_st1(ring, base + 4u * (uint32_t)f, v); });
    kmax = wave_max_u64(kmax);
    if (lane == 0 && kmax != 0)
        __hip_atomic_fetch_max(P.key + td.unit, kmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // claim the next item now: its round trip overlaps the store drain
    if (claim && tid == 0) next = atomicAdd(P.ticket, 1u);
    drain();  // every storing wave: ring stores and the key atomic are complete
    __syncthreads();
    if (tid == 0) add_rlx(P.tdone + td.unit, 1u);
}

// Emit the kept coefficients of one 8192-coefficient chunk held in q (thread
// (w, l) owns elements w*2048 + it*256 + 4l + j; kb bit it*4 + j = kept) as
// (run, value) pairs: ranks from per-column ballots, run =
// f - prev - 1.  rank / prev: this wave's first pair index and the unit-
// relative flat index of the last kept coefficient before this wave's
// elements (0xffffffff = none, so that run = f).  32-bit arithmetic: flat
// indices are < 2^31.
// Set bits of a 64-lane mask below this lane.
__device__ __forceinline__ uint32_t mbcnt64(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// STAGE: the pairs of each 256-element block are first placed in this wave's
// 256-entry LDS stage in rank order, then copied out with contiguous 8-B
// stores (one full 512-B row per instruction instead of up to four sparse,
// partial-line scatters: the pair stores, not the bytes, bounded the emit).
// A wave's LDS operations execute in order, so the stage needs no barrier.
template <bool STAGE, class Val>
__device__ __forceinline__ void emit_pairs(Val val, uint32_t kb, uint32_t start, int w, int l, uint32_t rank,
                                           uint32_t prev, uint2* __restrict__ pairs, uint2* stage) {
    const unsigned long long lt = (1ull << l) - 1ull;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const uint32_t nib = (kb >> (it * 4)) & 0xfu;
        const unsigned long long any = __ballot(nib != 0);
        if (!any) continue;
        // exclusive prefix of kept counts over lanes: one ballot per column j,
        // counted below this lane with mbcnt (ballots live in SGPRs)
        const unsigned long long b0 = __ballot(nib & 1u), b1 = __ballot(nib & 2u), b2 = __ballot(nib & 4u),
                                 b3 = __ballot(nib & 8u);
        const uint32_t pre = mbcnt64(b0) + mbcnt64(b1) + mbcnt64(b2) + mbcnt64(b3);
        const uint32_t itot = (uint32_t)(__popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3));
        const uint32_t ebase = start + (uint32_t)(w * 2048 + it * 256 + l * 4);
        const uint32_t lane_last = ebase + (nib ? 31u - (uint32_t)__clz(nib) : 0u);
        const unsigned long long below = any & lt;
        const uint32_t from_lane = __shfl(lane_last, below ? 63 - __clzll(below) : l);
        uint32_t p = below ? from_lane : prev;
        uint32_t r = STAGE ? pre : rank + pre;
        if (nib) {
            const float4 v4 = val(it);
            const float vv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (nib & (1u << j)) {
                    const uint32_t f = ebase + (uint32_t)j;
                    const uint2 pr = make_uint2(f - p - 1u, __float_as_uint(vv[j]));
                    if constexpr (STAGE)
                        stage[r] = pr;
                    else
                        pairs[r] = pr;
                    p = f;
                    ++r;
                }
            }
        }
        if constexpr (STAGE) {
            __builtin_amdgcn_wave_barrier();
            for (uint32_t k = (uint32_t)l; k < itot; k += 64) pairs[rank + k] = stage[k];
            __builtin_amdgcn_wave_barrier();
        }
        rank += itot;
        prev = __shfl(lane_last, 63 - __clzll(any));
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

// Per-wave kept count and last kept (chunk-relative index + 1, 0 = none).
__device__ __forceinline__ void wave_totals(uint32_t kb, int w, int l, uint32_t& cnt, uint32_t& last) {
    cnt = wave_sum((uint32_t)__popc(kb));
    const int hb = kb ? 31 - __clz(kb) : 0;
    last = wave_max_u32(kb ? (uint32_t)(w * 2048 + (hb >> 2) * 256 + l * 4 + (hb & 3) + 1) : 0u);
}

// Unit u's header (src/compressor.cpp:55-80: int32 W, H, D, ncoeff, nrle),
// kept count and payload offset, once its pair count is known.
__device__ __forceinline__ void finish_unit(const PipeParams& P, const UnitDev& U, uint32_t u, uint32_t total) {
    int32_t* hd = reinterpret_cast<int32_t*>(P.payload + U.pay_off);
    hd[0] = U.nx;
    hd[1] = U.ny;
    hd[2] = U.nz;
    hd[3] = (int32_t)U.ncells;
    hd[4] = (int32_t)total;
    P.kept[u] = total;
    P.offsets[u] = U.pay_off;
    if ((int)u == P.n - 1) P.offsets[P.n] = U.pay_off + 20 + 8ull * total;
}

// ---------------------------------------------------------------------------
// E item: threshold + ordered pack of emit tile `et`.
// Thread t = (wave w, lane l) owns elements w*2048 + it*256 + 4l + j, it 0..7.
// sm: 16 LDS words of scratch.
// RING: inside k_forward_pipe (coefficients in the ring, dependency waits);
// else inside k_emit_lb (coefficients in the staged flat scratch, written by
// an earlier launch).
template <bool RING>
__device__ __forceinline__ void pipe_emit(const PipeParams& P, __amdgpu_buffer_rsrc_t ring,
                                          const float* __restrict__ coef, uint32_t et, uint32_t* sm, uint2* stage,
                                          int tid, unsigned long long* st, const FTile* known = nullptr,
                                          bool key_ready = false) {
    // known (k_emit): the tile's unit and index are already known (ticket or
    // dispatch order); key_ready: its unit key already sits in sm[0..1].
    const FTile ft = known ? *known : P.etiles[et];
    const uint32_t u = ft.unit;
    const UnitDev& U = P.units[u];
    const int w = tid >> 6, l = tid & 63;
    unsigned long long* smk = reinterpret_cast<unsigned long long*>(sm);  // sm[0..1]: key
    // Sparse staging: this thread's 8 segment flags, loaded before the key
    // wait (wc_xform.h).
    const bool sparse = !RING && P.flags && U.sparse;
    uint32_t segf = 0xffu;  // bit it: group it may hold kept coefficients
    if (sparse) {
        // one flag byte per segment of TZ = 2^lbz coefficients (16 or 32)
        const uint8_t* fl = P.flags + (U.coef_off >> kSegShift) + (((uint64_t)ft.index * kEmitTile) >> U.lbz);
        const int sh = U.lbz;
        segf = 0;
#pragma unroll
        for (int it = 0; it < 8; ++it) segf |= (uint32_t)(fl[(w * 2048 + it * 256 + 4 * l) >> sh] != 0) << it;
    }

    // 1. the unit's transform tiles are all in the ring (RING); the unit key
    unsigned long long ukey;
    if constexpr (RING) {
        if (tid == 0) {
            const unsigned long long t0 = P.stats ? now_ticks() : 0;
            for (uint32_t spins = 0;;) {
                if (ld_rlx(P.tdone + u) >= U.ntx) break;
                if (spin_fail(spins, P.err)) break;
            }
            smk[0] = ld_rlx(P.key + u);
            if (P.stats) st[kStEWait] += now_ticks() - t0;
        }
        __syncthreads();
        ukey = smk[0];
    } else if (key_ready) {
        ukey = smk[0];  // stored before the caller's barrier
    } else {
        ukey = P.key[u];  // a finished earlier launch wrote it: one uniform load, no barrier
    }
    const float tf = unit_thresh(P, ukey);
    const uint32_t start = ft.index * (uint32_t)kEmitTile;
    const uint32_t len = (uint32_t)min((uint64_t)kEmitTile, U.ncells - start);

    // 2. coefficients -> keep bits (bit it*4 + j)
    float4 q[8];
    if constexpr (RING) {
        const uint32_t base = 4u * ((uint32_t)U.ring_off + start);
#pragma unroll
        for (int it = 0; it < 8; ++it) q[it] = ring_ld4(ring, base + 16u * (uint32_t)(w * 512 + it * 64 + l));
    } else {
        // flat scratch: 16-B aligned per unit, kFlatTile slack past the last unit
        const float4* __restrict__ p4 =
            reinterpret_cast<const float4*>(coef + (P.ring_coefs ? U.ring_off : U.coef_off) + start);
        // sparse units with thresh >= 0 skip unflagged segments (never stored);
        // thresh < 0 units were re-staged densely (k_transform_fallback)
        if (!(tf >= 0.0f)) segf = 0xffu;
#pragma unroll
        for (int it = 0; it < 8; ++it)
            q[it] = ((segf >> it) & 1u) && (uint32_t)(w * 2048 + it * 256 + 4 * l) < len ? p4[w * 512 + it * 64 + l]
                                                                                          : make_float4(0, 0, 0, 0);
    }
    const uint32_t kb = keep_bits(q, tf, len, w, l);
    uint32_t wcnt, wlast;
    wave_totals(kb, w, l, wcnt, wlast);
    if (l == 0) {
        sm[4 + w] = wcnt;
        sm[8 + w] = wlast;
    }
    __syncthreads();

    // 3. publish the aggregate, look back over the unit's earlier tiles (wave 0)
    if (w == 0) {
        uint32_t C = 0, L = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            C += sm[4 + i];
            L = sm[8 + i] > L ? sm[8 + i] : L;
        }
        const uint32_t L1 = L ? start + L : 0u;  // unit-relative last kept + 1
        uint32_t ecnt = 0, elast = 0;            // exclusive: pairs before, last kept + 1 before
        if (ft.index == 0) {
            if (l == 0) st_rlx(P.status + et, kFlagIncl | ((unsigned long long)C << 31) | L1);
        } else {
            if (l == 0) st_rlx(P.status + et, kFlagAgg | ((unsigned long long)C << 31) | L1);
            const unsigned long long t0 = (RING && P.stats) ? now_ticks() : 0;
            int64_t pos = (int64_t)et - 1;
            const int64_t first = U.et_begin;
            // Window of the 64 nearest predecessors (lane l = tile et-1-l; tiles
            // before the unit read as an inclusive 0).  Lanes up to the nearest
            // inclusive one are summed once every one of them has published;
            // a run of published aggregates before the first unpublished tile
            // is summed and the window slides past it.
            for (uint32_t spins = 0;;) {
                const int64_t idx = pos - l;
                const unsigned long long v = idx >= first ? ld_rlx(P.status + idx) : kFlagIncl;
                const unsigned long long incl = __ballot((v >> 62) == 2);
                const unsigned long long zero = __ballot((v >> 62) == 0);
                const int kI = incl ? __ffsll((long long)incl) - 1 : 64;
                const int kZ = zero ? __ffsll((long long)zero) - 1 : 64;
                const int take = kI < kZ ? kI + 1 : kZ;  // lanes [0, take) are summed
                if (take > 0) {
                    const bool in = l < take;
                    ecnt += wave_sum(in ? (uint32_t)((v >> 31) & kMask31) : 0u);
                    const unsigned long long hasl = __ballot(in && (v & kMask31) != 0);
                    const uint32_t hl = __shfl((uint32_t)(v & kMask31), hasl ? __ffsll((long long)hasl) - 1 : 0);
                    if (elast == 0 && hasl) elast = hl;
                }
                if (kI < kZ) break;
                pos -= take;
                if (take == 0 && spin_fail(spins, P.err)) break;
            }
            if (l == 0)
                st_rlx(P.status + et, kFlagIncl | ((unsigned long long)(ecnt + C) << 31) | (L1 ? L1 : elast));
            if (RING && P.stats && l == 0) st[kStELook] += now_ticks() - t0;
        }
        if (l == 0) {
            sm[0] = ecnt;
            sm[1] = elast;
            // ring reads of this tile are done (all waves passed the barrier above)
            if constexpr (RING) add_rlx(P.edone + u, 1u);
            if (ft.index + 1 == U.net) finish_unit(P, U, u, ecnt + C);  // last tile
        }
    }
    __syncthreads();

    // 4. emit (run, value) pairs: ranks from wave ballots, run = f - prev - 1.
    // Flat indices are unit-relative and < 2^31: 32-bit arithmetic, with
    // "no previous kept" = 0xffffffff so that run = f - prev - 1 = f.
    uint32_t rank = sm[0];
    uint32_t prev = sm[1] - 1u;
    for (int i = 0; i < w; ++i) {
        rank += sm[4 + i];
        if (sm[8 + i]) prev = start + sm[8 + i] - 1u;
    }
    uint2* __restrict__ pairs = reinterpret_cast<uint2*>(P.payload + U.pay_off + 20);
    emit_pairs<!RING>([&](int it) { return q[it]; }, kb, start, w, l, rank, prev, pairs, stage);
}

// ---------------------------------------------------------------------------
// E item, unit granularity: one workgroup thresholds and packs a whole unit,
// streaming its ring region in kEmitTile chunks: a chunk's values are parked
// in LDS (each thread its own elements) so the next chunk's loads are in
// flight while this one is packed.  Pair offsets are a running sum (no
// look-back); one dependency wait per unit.
// sm: [0..1] key, [4..19] per-wave counts / lasts of two chunks (alternating,
// so one barrier per chunk suffices); stash: 32 KB of LDS.
__device__ __forceinline__ void ring_chunk(__amdgpu_buffer_rsrc_t ring, uint32_t rbase, uint32_t c, int w, int l,
                                           float4 (&q)[8]) {
#pragma unroll
    for (int it = 0; it < 8; ++it)
        q[it] = ring_ld4(ring, rbase + 4u * c * (uint32_t)kEmitTile + 16u * (uint32_t)(w * 512 + it * 64 + l));
}

__device__ __forceinline__ void pipe_emit_unit(const PipeParams& P, __amdgpu_buffer_rsrc_t ring, uint32_t u,
                                               uint32_t* sm, float* stash, int tid, unsigned long long* st) {
    const UnitDev& U = P.units[u];
    const int w = tid >> 6, l = tid & 63;
    unsigned long long* smk = reinterpret_cast<unsigned long long*>(sm);
    if (tid == 0) {
        const unsigned long long t0 = P.stats ? now_ticks() : 0;
        for (uint32_t spins = 0;;) {
            if (ld_rlx(P.tdone + u) >= U.ntx) break;
            if (spin_fail(spins, P.err)) break;
        }
        smk[0] = ld_rlx(P.key + u);
        if (P.stats) st[kStEWait] += now_ticks() - t0;
    }
    __syncthreads();
    const float tf = unit_thresh(P, smk[0]);
    const uint32_t nc = (uint32_t)U.ncells;
    const uint32_t nch = (nc + kEmitTile - 1) / kEmitTile;
    const uint32_t rbase = 4u * (uint32_t)U.ring_off;
    uint2* __restrict__ pairs = reinterpret_cast<uint2*>(P.payload + U.pay_off + 20);
    uint32_t rank = 0, prev = 0xffffffffu;
    // This thread's stash slots (its own elements: no barrier needed).
    float4* mine = reinterpret_cast<float4*>(stash) + w * 512 + l;
    float4 q[8];
    if (nch) ring_chunk(ring, rbase, 0, w, l, q);
    for (uint32_t c = 0; c < nch; ++c) {
        uint32_t* cs = sm + 4 + 8 * (c & 1u);  // alternating: one barrier per chunk
        const uint32_t start = c * (uint32_t)kEmitTile;
        const uint32_t len = min((uint32_t)kEmitTile, nc - start);
        const uint32_t kb = keep_bits(q, tf, len, w, l);
        uint32_t wc, wl;
        wave_totals(kb, w, l, wc, wl);
#pragma unroll
        for (int it = 0; it < 8; ++it) mine[it * 64] = q[it];
        if (c + 1 < nch) ring_chunk(ring, rbase, c + 1, w, l, q);  // in flight while this chunk is packed
        if (l == 0) {
            cs[w] = wc;
            cs[4 + w] = wl;
        }
        __syncthreads();
        uint32_t r = rank, pv = prev, tot = 0, cl = prev;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t ci = cs[i], li = cs[4 + i];
            if (i < w) {
                r += ci;
                if (li) pv = start + li - 1u;
            }
            tot += ci;
            if (li) cl = start + li - 1u;
        }
        emit_pairs<false>([&](int it) { return mine[it * 64]; }, kb, start, w, l, r, pv, pairs, nullptr);
        rank += tot;
        prev = cl;
    }
    __syncthreads();  // every ring load of the unit has been consumed
    if (tid == 0) {
        add_rlx(P.edone + u, 1u);
        finish_unit(P, U, u, rank);
    }
}

// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kThreads, 4) void k_forward_pipe(PipeParams P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    uint32_t* ctl = reinterpret_cast<uint32_t*>(lds);   // [0]: next batch; [2..17]: stats (tid 0)
    uint32_t* sm = ctl + 18;                             // emit scratch (24 words)
    float* tl = lds + 48;                                // transform tile rows (192-B offset)
    const int tid = threadIdx.x;
    const __amdgpu_buffer_rsrc_t ring = __builtin_amdgcn_make_buffer_rsrc(P.ring, 0, (int)P.ring_bytes, 0x00020000);
    // stats accumulators (tid 0 only) live in LDS words ctl[2..]
    unsigned long long* st = reinterpret_cast<unsigned long long*>(ctl + 2);
    if (tid == 0) {
        for (int i = 0; i < kPipeStats; ++i) st[i] = 0;
        ctl[0] = atomicAdd(P.ticket, 1u);
    }
    __syncthreads();
    const uint32_t K = P.claim;
    uint32_t batch = __builtin_amdgcn_readfirstlane(ctl[0]);
    while (batch * K < P.nitems) {
        uint32_t next = 0;
        const uint32_t first = batch * K, last = min(first + K, P.nitems);
        bool claimed = false;
        for (uint32_t item = first; item < last; ++item) {
            if (tid == 0 && P.prefetch && item + 1 == last) next = atomicAdd(P.ticket, 1u);
            const unsigned long long t0 = (P.stats && tid == 0) ? now_ticks() : 0;
            const uint32_t code = P.items[item];
            if (code & 0x80000000u) {
                pipe_emit_unit(P, ring, code & 0x3fffffffu, sm, tl, tid, st);
                if (P.stats && tid == 0) {
                    st[kStE] += now_ticks() - t0;
                    st[kStNE] += 1;
                }
            } else {
                claimed = !P.prefetch && item + 1 == last;
                pipe_transform<T>(P, ring, code, tl, tid, st, claimed, next);
                if (P.stats && tid == 0) {
                    st[kStT] += now_ticks() - t0;
                    st[kStNT] += 1;
                }
            }
        }
        if (tid == 0) {
            const unsigned long long t0 = P.stats ? now_ticks() : 0;
            if (!P.prefetch && !claimed) next = atomicAdd(P.ticket, 1u);
            ctl[0] = next;
            if (P.stats) st[kStClaim] += now_ticks() - t0;
        }
        __syncthreads();
        batch = __builtin_amdgcn_readfirstlane(ctl[0]);
    }
    if (P.stats && tid == 0)
        for (int i = 0; i < kPipeStats; ++i) atomicAdd(P.stats + i, st[i]);
}

// ---------------------------------------------------------------------------
// Staged-path emit, whole units (k_emit blocks [0, nseg)): one workgroup
// thresholds and packs a unit of at most WC_OPT_EMIT_SEG_MAX emit tiles,
// streaming its coefficients in kEmitTile chunks with the next chunk's loads
// in flight while the current one is packed.  Pair ranks and the previous
// kept index are running values: no look-back, no tickets, no traffic
// between workgroups.  sm[4..11] / sm[12..19]: per-wave counts and lasts of
// even / odd chunks (alternating, so one barrier per chunk suffices).
__device__ __forceinline__ void seg_load(const float4* __restrict__ p4, uint32_t c, uint32_t nc, int w, int l,
                                         float4 (&q)[8]) {
    const uint32_t start = c * (uint32_t)kEmitTile;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const uint32_t e = start + (uint32_t)(w * 2048 + it * 256 + 4 * l);
        q[it] = e < nc ? p4[e >> 2] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

__device__ __forceinline__ void seg_pack(const float4 (&q)[8], float tf, uint32_t c, uint32_t nc, int w, int l,
                                         uint32_t* cs, uint32_t& rank, uint32_t& prev, uint2* __restrict__ pairs,
                                         uint2* stage) {
    const uint32_t start = c * (uint32_t)kEmitTile;
    const uint32_t kb = keep_bits(q, tf, min((uint32_t)kEmitTile, nc - start), w, l);
    uint32_t wc, wl;
    wave_totals(kb, w, l, wc, wl);
    if (l == 0) {
        cs[w] = wc;
        cs[4 + w] = wl;
    }
    __syncthreads();
    uint32_t r = rank, pv = prev, tot = 0, cl = prev;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t ci = cs[i], li = cs[4 + i];
        if (i < w) {
            r += ci;
            if (li) pv = start + li - 1u;
        }
        tot += ci;
        if (li) cl = start + li - 1u;
    }
    emit_pairs<true>([&](int it) { return q[it]; }, kb, start, w, l, r, pv, pairs, stage);
    rank += tot;
    prev = cl;
}

__device__ __forceinline__ void emit_seg(const PipeParams& P, const float* __restrict__ coef, uint32_t u,
                                         uint32_t* sm, uint2* stage, int tid) {
    const UnitDev& U = P.units[u];
    const int w = tid >> 6, l = tid & 63;
    const float tf = unit_thresh(P, P.key[u]);
    const uint32_t nc = (uint32_t)U.ncells;
    const uint32_t nch = (nc + kEmitTile - 1) / kEmitTile;
    const float4* __restrict__ p4 = reinterpret_cast<const float4*>(coef + (P.ring_coefs ? U.ring_off : U.coef_off));
    uint2* __restrict__ pairs = reinterpret_cast<uint2*>(P.payload + U.pay_off + 20);
    uint32_t rank = 0, prev = 0xffffffffu;
    float4 a[8], b[8];
    if (nch) seg_load(p4, 0, nc, w, l, a);
    for (uint32_t c = 0; c < nch; c += 2) {
        if (c + 1 < nch) seg_load(p4, c + 1, nc, w, l, b);
        seg_pack(a, tf, c, nc, w, l, sm + 4, rank, prev, pairs, stage);
        if (c + 1 == nch) break;
        if (c + 2 < nch) seg_load(p4, c + 2, nc, w, l, a);
        seg_pack(b, tf, c + 1, nc, w, l, sm + 12, rank, prev, pairs, stage);
    }
    if (tid == 0) finish_unit(P, U, u, rank);
}

// Staged-path emit, one launch: blocks [0, nseg) pack whole units
// (emit_seg); the rest pack the emit tiles of the other units with decoupled
// look-back (pipe_emit).  A look-back block takes its tile index within the
// unit from that unit's ticket (P.tdone[u], unused by the staged path), so a
// tile's predecessors have always started (forward progress without
// assuming dispatch order), and the ticket atomics spread over one address
// per unit.  SEG = false compiles the look-back path alone (its register
// budget is not raised by the whole-unit path's double buffer).
template <bool SEG>
#ifndef WC_EMIT_ORDERED
#define WC_EMIT_ORDERED 1  // 0: take the look-back tile index from a per-unit ticket atomic instead
#endif
#ifndef WC_EMIT_MINB
#define WC_EMIT_MINB 4  // workgroups per CU the register budget is sized for (tools/sweeps/emit_variants.sh)
#endif
__global__ __launch_bounds__(kThreads, WC_EMIT_MINB) void k_emit(PipeParams P, const float* __restrict__ coef, uint32_t nseg) {
    __shared__ __attribute__((aligned(16))) uint32_t sm[32];
    __shared__ uint2 stage_all[kThreads / kWave][256];  // per-wave pair stage (emit_pairs)
    const int tid = threadIdx.x;
    uint2* stage = stage_all[tid >> 6];
    if constexpr (SEG) {
        if (blockIdx.x < nseg) {
            emit_seg(P, coef, P.segs[P.seg_base + blockIdx.x], sm, stage, tid);
            return;
        }
    }
    __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc(nullptr, 0, 0, 0x00020000);
#if WC_EMIT_ORDERED
    // Tile index from the dispatch order: a block's look-back waits only on
    // lower-indexed tiles of its unit, which have lower block ids, and each
    // XCD dispatches its blocks in increasing id order, so no wait is on an
    // undispatched block (waits stay bounded by spin_fail regardless).
    if (P.eidx) {
        const uint32_t b = blockIdx.x - nseg;
        const FTile ft{P.eunits[b], P.eidx[b]};
        pipe_emit<false>(P, none, coef, P.units[ft.unit].et_begin + ft.index, sm, stage, tid, nullptr, &ft);
        return;
    }
#endif
    if (tid == 0) {
        const uint32_t b = blockIdx.x - nseg;
        const uint32_t u = P.eunits ? P.eunits[b] : P.etiles[P.etile_base + b].unit;
        // the unit key and the tile ticket in flight together
        const unsigned long long key = P.key[u];
        const uint32_t t = atomicAdd(P.tdone + u, 1u);
        reinterpret_cast<unsigned long long*>(sm)[0] = key;
        sm[16] = t;
        sm[17] = u;
    }
    __syncthreads();
    const FTile ft{(uint32_t)__builtin_amdgcn_readfirstlane(sm[17]), (uint32_t)__builtin_amdgcn_readfirstlane(sm[16])};
    const uint32_t et = P.units[ft.unit].et_begin + ft.index;
    pipe_emit<false>(P, none, coef, et, sm, stage, tid, nullptr, &ft, true);
}

// ---------------------------------------------------------------------------
// Chunked forward (WC_OPT_CHUNK): one launch per chunk on ONE stream.  Blocks
// [0, nE) pack the emit tiles of the previous chunk (look-back, as k_emit),
// blocks after them transform the tiles of this chunk into its coefficient
// slot.  The launch boundary orders every hand-off: chunk k's coefficients
// (slot k % 2) are complete when launch k + 1 reads them, and slot k % 2 is
// rewritten by launch k + 2 only after launch k + 1 has read it.  A slot is a
// few tens of MB, so the coefficients should stay in the 256 MiB Infinity
// Cache between their write and their read.
struct ChunkLaunch {
    uint32_t gen_b, gen_n, fast_b, fast_n;  // transform tiles of this chunk (xtiles ranges)
    uint32_t et_b, et_n;                    // emit tiles of the previous chunk
};

template <typename T>
__global__ __launch_bounds__(kThreads) void k_chunk(PipeParams P, ChunkLaunch C) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid = threadIdx.x;
    if (blockIdx.x < C.et_n) {
        uint32_t* sm = reinterpret_cast<uint32_t*>(lds);                   // 32 words
        uint2* stage = reinterpret_cast<uint2*>(lds + 32) + (tid >> 6) * 256;  // per-wave pair stage
        if (tid == 0) {
            const uint32_t u = P.etiles[C.et_b + blockIdx.x].unit;
            sm[16] = P.units[u].et_begin + atomicAdd(P.tdone + u, 1u);
        }
        __syncthreads();
        const uint32_t et = __builtin_amdgcn_readfirstlane(sm[16]);
        __syncthreads();
        __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc(nullptr, 0, 0, 0x00020000);
        pipe_emit<false>(P, none, P.ring, et, sm, stage, tid, nullptr);
        return;
    }
    const uint32_t b = blockIdx.x - C.et_n;
    const XTile td = P.xtiles[b < C.gen_n ? C.gen_b + b : C.fast_b + (b - C.gen_n)];
    const UnitDev& U = P.units[td.unit];
    const T* src = static_cast<const T*>(P.cells) + U.cell_off;
    float* __restrict__ dst = P.ring + U.ring_off;
    unsigned long long kmax;
    if (U.fast) {
        xform_fast_p1<T>(src, U, td, lds, tid);
        __syncthreads();
        kmax = xform_fast_p2<true>(U, td, lds, tid,
                                   [&](int64_t f, float4 v) { *reinterpret_cast<float4*>(dst + f) = v; });
    } else {
        xform_generic_p1<T>(src, U, td, lds, tid);
        __syncthreads();
        kmax = xform_generic_p2<true>(U, td, lds, tid, [&](int64_t f, float v) { dst[f] = v; });
    }
    kmax = wave_max_u64(kmax);
    if ((tid & 63) == 0 && kmax != 0) atomicMax(P.key + td.unit, kmax);
}

}  // namespace

hipError_t launch_emit(hipStream_t st, const PipeParams& p, const float* coef, uint32_t nseg, uint32_t netiles) {
    if (nseg)
        k_emit<true><<<nseg + netiles, kThreads, 0, st>>>(p, coef, nseg);
    else if (netiles)
        k_emit<false><<<netiles, kThreads, 0, st>>>(p, coef, 0u);
    return hipGetLastError();
}

size_t pipe_lds_bytes(size_t tile_lds) { return 192 + (tile_lds > 4u * kEmitTile ? tile_lds : 4u * kEmitTile); }

hipError_t launch_forward_pipe(hipStream_t st, int dtype, size_t lds, uint32_t grid, const PipeParams& p) {
    if (p.nitems == 0) return hipSuccess;
    if (dtype == 1)
        k_forward_pipe<double><<<grid, kThreads, lds, st>>>(p);
    else
        k_forward_pipe<float><<<grid, kThreads, lds, st>>>(p);
    return hipGetLastError();
}

// Workgroups that fit on the device at once (more would only find the
// ticket counter exhausted).  Residency is not needed for correctness.
uint32_t pipe_grid(int dtype, size_t lds, int max_per_cu) {
    int per_cu = 0, ncu = 0, dev = 0;
    (void)hipGetDevice(&dev);
    const void* fn = dtype == 1 ? (const void*)k_forward_pipe<double> : (const void*)k_forward_pipe<float>;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kThreads, lds) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per_cu < 1 ||
        ncu < 1)
        return 1024;
    if (max_per_cu > 0 && per_cu > max_per_cu) per_cu = max_per_cu;
    return (uint32_t)per_cu * (uint32_t)ncu;
}

size_t chunk_lds_bytes(size_t tile_lds) {
    const size_t emit = 4 * 32 + 8 * 256 * (kThreads / kWave);
    return tile_lds > emit ? tile_lds : emit;
}

hipError_t launch_chunk(hipStream_t st, int dtype, size_t lds, const PipeParams& p, uint32_t gen_b, uint32_t gen_n,
                        uint32_t fast_b, uint32_t fast_n, uint32_t et_b, uint32_t et_n) {
    const ChunkLaunch c{gen_b, gen_n, fast_b, fast_n, et_b, et_n};
    const uint32_t grid = gen_n + fast_n + et_n;
    if (grid == 0) return hipSuccess;
    if (dtype == 1)
        k_chunk<double><<<grid, kThreads, lds, st>>>(p, c);
    else
        k_chunk<float><<<grid, kThreads, lds, st>>>(p, c);
    return hipGetLastError();
}

}  // namespace wc

// wc_cohort.hip — the cohort forward: K1 (transform + max key) and K2 (keep
// threshold + ordered pack) of large units in ONE persistent launch, with the
// staged coefficients kept in a small ring that stays in the Infinity Cache.
//
//   src/compressor.cpp:85-185   wavelet_decompose     -> K1 items (S32 tile body, wc_xform.h)
//   src/compressor.cpp:212-216  max_element, thresh   -> unit key (atomicMax per workgroup)
//   src/compressor.cpp:222-238  mask + rle_encode     -> emit items (emit_tile, wc_emit.h)
//   src/compressor.cpp:55-80    serialize             -> header + pairs in the unit's slot
//
// Why (DESIGN.md "C5 cohort forward"): the staged forward of 128^3 fp32 units
// writes every coefficient to HBM in K1 and reads it back in the emit (C5:
// 4.1 GB each way of 16.3 GB of counter traffic).  A ring of a few units'
// staging slots, reused as the batch advances, keeps that round trip on-die
// (tools/mall_probe.hip: 1.86 vs 3.25 ms for the same flow through a 128 MiB
// vs a 4 GiB ring, profiles/r04/experiments/mall_probe.txt).
//
// Work list (host-built, wc_capi.cpp build_cohort): units in cohorts of S;
// phase p lists cohort p's K1 tiles interleaved with the emit tiles of cohort
// p - lag; unit u stages into ring slot u mod R, R = (lag + 2) S.  Block b
// runs item b, so every item waits only on items of lower block ids — a K1
// tile on the emit tiles of the slot's previous unit (edone), an emit tile on
// its unit's K1 tiles (kdone) and on its unit's earlier emit tiles
// (look-back).  Those sit 1-2 phases (>= 2 resident-block windows) back, so
// the waits rarely block.  A persistent dequeue form (workgroups claiming
// items from one counter: progress whatever the dispatch order) was built and
// measured 5-240x slower: claimed-but-queued items make convoys
// (profiles/r04/experiments/gpu_cohort_dequeue.txt).
//
// Hand-offs inside the launch (MI355X_MICROARCH.md Valid forms, row 1): every
// staged coefficient is stored write-through (sc1) and every emit load of it
// is an sc1 load; each storing wave drains (s_waitcnt vmcnt(0)) before the
// workgroup barrier, then ONE lane signals with an agent-scope atomic add; the
// consumer polls that counter relaxed.  The unit key is an agent-scope
// atomicMax read with an agent-scope load (never the scalar path).
#include "wc_emit.h"

// Diagnostic builds (tools/build_variants.sh; timing only, results invalid):
//   WC_COH_XP_NOWAIT  no kdone / edone waits;  WC_COH_XP_AUX=0  plain (not sc1)
//   ring loads and stores;  WC_COH_XP_K1ONLY / WC_COH_XP_EONLY  one item kind only.
#ifndef WC_COH_XP_AUX
#define WC_COH_XP_AUX 16
#endif

namespace wc {

using u32x4 = uint32_t __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ring_rsrc(const CohortParams& C) {
    // built from kernel arguments only: wave-uniform, no waterfall (cdna_hip_programming.md T20)
    return __builtin_amdgcn_make_buffer_rsrc(C.ring, (short)0, (int)C.ring_bytes, 0x00020000);
}

// One lane waits until *cnt >= want (relaxed agent-scope polls, bounded).
__device__ __forceinline__ void wait_geq(const uint32_t* cnt, uint32_t want, uint32_t* err) {
#ifdef WC_COH_XP_NOWAIT
    return;
#endif
    for (uint32_t spins = 0; ld_rlx(cnt) < want;)
        if (spin_fail(spins, err)) break;
}

// Emit source of the cohort: the unit's staged coefficients in its ring slot,
// written in this launch by K1 items with sc1 stores; every load is an sc1
// buffer load (bypasses the possibly stale L1).  consumed(): the tile's loads
// have returned, so the slot's next unit may overwrite it (edone).
struct RingTile {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t base;  // byte offset of the tile's first coefficient in the ring
    __device__ __forceinline__ float4 operator[](int i) const {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, base + (uint32_t)i * 16u, 0, WC_COH_XP_AUX);
        return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
    }
};
struct RingSrc {
    __amdgpu_buffer_rsrc_t rs;
    const unsigned long long* keys;
    uint32_t* edone;
    __device__ __forceinline__ unsigned long long key(const EmitParams&, uint32_t u) const { return ld_rlx(keys + u); }
    __device__ __forceinline__ RingTile tile(const EmitDesc& U, uint32_t start) const {
        return RingTile{rs, (uint32_t)(U.coef_off + start) * 4u};
    }
    __device__ __forceinline__ void consumed(const EmitDesc& U, int tid) const {
        if (tid == 0) add_rlx(edone + U.unit, 1u);
    }
};

// K1 phase 2 of an S32 tile for the cohort: EVERY coefficient stored
// write-through into the unit's ring slot (dense: no flags, no re-staging
// fallback), and this thread's max key (WC_K1_BFKEY form of
// xform_fast_p2_sparse_s32: only where |c| equals the tile's largest |c|;
// a tile holding a NaN takes every coefficient's key).
__device__ __forceinline__ unsigned long long xform_s32_p2_ring(const UnitDev& U, const XTile& td, const float* lds,
                                                                int tid, uint32_t amax, __amdgpu_buffer_rsrc_t rs,
                                                                uint32_t slot_bytes) {
    constexpr int lbz = 5, TZ = 32, rstride = 2 * TZ + 4;
    const int H = U.ny, D = U.nz, hx = U.hx, hy = U.hy, hz = U.hz;
    const int r0 = tid >> 4, col = (tid & 15) << 2;
    const int ssz = col >> lbz, bzl = col & (TZ - 1);
    const int K = td.bz0 + bzl + ssz * hz;
    const bool allkeys = amax > 0x7f800000u;
    const uint32_t HD = (uint32_t)H * (uint32_t)D;
    const uint32_t fb = ((uint32_t)(td.bx0 + r0) * (uint32_t)H + td.by0) * (uint32_t)D + (uint32_t)K;
    const uint32_t dA = 16u * HD, dB = (uint32_t)hx * HD, dC = (uint32_t)hy * (uint32_t)D;
    uint32_t best = 0;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const int row = r0 + 16 * it;
        const float4 v = *reinterpret_cast<const float4*>(lds + row * rstride + col);
        const uint32_t f0 = fb + ((it & 1) ? dA : 0u) + (((it >> 1) & 1) ? dB : 0u) + ((it >> 2) ? dC : 0u);
        const u32x4 w = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
        __builtin_amdgcn_raw_buffer_store_b128(w, rs, slot_bytes + (f0 << 2), 0, WC_COH_XP_AUX);  // sc1: write-through
        const float m4 = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
        if (__ballot(__float_as_uint(m4) == amax)) {
            best = key_lo_max(best, v.x, f0, amax);
            best = key_lo_max(best, v.y, f0 + 1u, amax);
            best = key_lo_max(best, v.z, f0 + 2u, amax);
            best = key_lo_max(best, v.w, f0 + 3u, amax);
        }
    }
    if (!allkeys) return key_from_lo(amax, best);
    unsigned long long kmax = 0;  // a NaN in the tile (rare): every key, as the generic form
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const int row = r0 + 16 * it;
        const int bxl = row & 31, ssx = (row >> 5) & 1, ssy = row >> 6;
        const int I = td.bx0 + bxl + ssx * hx, J = (int)td.by0 + ssy * hy;
        const uint32_t f0 = (uint32_t)(((int64_t)I * H + J) * D + K);
        const float4 v = *reinterpret_cast<const float4*>(lds + row * rstride + col);
        const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const unsigned long long k = coef_key(e[j], f0 + (uint32_t)j);
            kmax = k > kmax ? k : kmax;
        }
    }
    return kmax;
}

struct alignas(16) CohShared {
    uint32_t sm[32];                       // emit_tile words
    unsigned long long key[kThreads / kWave];
    uint32_t mag[kThreads / kWave];
    uint32_t pad[4];
};

template <typename T>
__device__ __forceinline__ void cohort_k1(const CohortParams& C, const T* __restrict__ cells, uint32_t xt, float* lds,
                                          CohShared& sh, int tid) {
    const XTile td = C.xtiles[xt];
    const uint32_t u = td.unit;
    const UnitDev& U = C.units[u];
    uint32_t mag = xform_fast_p1<T, false, true, true>(cells + U.cell_off, U, td, lds, tid);
    mag = wave_max_u32_u(mag);
    if ((tid & 63) == 0) sh.mag[tid >> 6] = mag;
    // the slot's previous unit: every emit tile has read it.  Waited for only
    // now (phase 1 reads cells and writes LDS): the poll's round trip overlaps
    // the cell loads instead of preceding them.
    if (u >= C.ring_units && tid == 0) {
        const uint32_t v = u - C.ring_units;
        wait_geq(C.edone + v, (uint32_t)((C.units[v].ncells + kEmitTile - 1) / kEmitTile), C.E.err);
    }
    __syncthreads();
    mag = max(max(sh.mag[0], sh.mag[1]), max(sh.mag[2], sh.mag[3]));
    const uint32_t slot_bytes = (u % C.ring_units) * (uint32_t)(C.ring_bytes / C.ring_units);
    const unsigned long long kmax = xform_s32_p2_ring(U, td, lds, tid, mag >> 1, ring_rsrc(C), slot_bytes);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains its sc1 stores
    block_key_max(kmax, sh.key, C.key + u);           // barrier; lane 0: one atomicMax
    if (tid == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the key's atomic has completed
        add_rlx(C.kdone + u, 1u);
    }
}

__device__ __forceinline__ void cohort_emit(const CohortParams& C, uint32_t ei, float* lds, CohShared& sh, int tid) {
    const EmitDesc E = C.E.edesc[ei];
    if (tid == 0) wait_geq(C.kdone + E.unit, C.units[E.unit].ntx, C.E.err);
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the poll
    uint2* stage = reinterpret_cast<uint2*>(lds) + (tid >> 6) * (256 * WC_EMIT_SB);
    emit_tile<4>(C.E, RingSrc{ring_rsrc(C), C.key, C.edone}, E, E.index, sh.sm, stage, tid);
}

}  // namespace

// One block per item, items in list order (blockIdx.x): the in-flight items
// are the resident blocks (~1024 consecutive items), and with the per-XCD
// in-order dispatch the other look-back kernels also rely on (DESIGN.md
// §Forward progress) every item waits only on blocks dispatched before it.
// wc_capi.cpp takes this path only where the launch-order form is in use;
// the ticket form runs the two-kernel path instead.
template <typename T>
__global__ __launch_bounds__(kThreads, 4) void k_cohort(CohortParams C, const T* __restrict__ cells) {
    extern __shared__ __attribute__((aligned(16))) float lds[];  // K1 rows | emit pair stage
    __shared__ CohShared sh;
    const int tid = threadIdx.x;
    const uint32_t it = cst(C.items)[blockIdx.x];
#ifdef WC_COH_XP_K1ONLY
    if (it >> 31) return;
#endif
#ifdef WC_COH_XP_EONLY
    if (!(it >> 31)) return;
#endif
    if (it >> 31)
        cohort_emit(C, it & 0x7fffffffu, lds, sh, tid);
    else
        cohort_k1<T>(C, cells, it, lds, sh, tid);
}

size_t cohort_lds_bytes() {
    const size_t k1 = (size_t)4 * 32 * (2 * 32 + 4) * sizeof(float);  // S32 tile rows (wc_xform.h)
    const size_t em = (size_t)4 * 256 * WC_EMIT_SB * sizeof(uint2);     // 4 waves' pair stages
    return k1 > em ? k1 : em;
}

hipError_t launch_cohort(hipStream_t st, const CohortParams& p, const void* cells, int dtype) {
    if (p.nitems == 0) return hipSuccess;
    const uint32_t g = p.nitems;
    if (dtype == 1)
        k_cohort<double><<<g, kThreads, cohort_lds_bytes(), st>>>(p, (const double*)cells);
    else
        k_cohort<float><<<g, kThreads, cohort_lds_bytes(), st>>>(p, (const float*)cells);
    return hipGetLastError();
}

}  // namespace wc

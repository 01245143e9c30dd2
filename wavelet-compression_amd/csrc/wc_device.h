// wc_device.h — device helpers shared by the codec kernels (wave64 reductions,
// block scans, x-pair loads, the Haar butterfly halves).
#pragma once

#include "wc_internal.h"

namespace wc {

__device__ __forceinline__ float haar_lo(float a, float b) { return (a + b) * 0.5f; }
__device__ __forceinline__ float haar_hi(float a, float b) { return (a - b) * 0.5f; }

// The reference keeps |c| iff (double)|c| > thresh (src/compressor.cpp:225-226).
// With tf = thresh rounded toward -inf to float, that is exactly |c| > tf for
// every float |c|: no float lies strictly between tf and thresh; NaN and
// +-inf thresholds map to themselves.
__device__ __forceinline__ float thresh_as_float(double thresh) { return __double2float_rd(thresh); }

__device__ __forceinline__ int lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0));
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Wave reductions on DPP lane moves (row_shr 1/2/4/8 inside 16-lane rows,
// then row_bcast 15 / 31 across them, as wave_incl_sum below): lane 63 ends
// with the reduction over all 64 lanes, returned uniformly by readlane.  A
// chain of six VALU ops instead of six LDS-crossbar bpermutes (__shfl_xor).
// Lanes whose DPP source is out of range read 0, the identity of the unsigned
// max and of the sum.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return __builtin_amdgcn_update_dpp(0u, v, CTRL, ROW_MASK, 0xf, false);
}

__device__ __forceinline__ uint32_t wave_max_u32_u(uint32_t v) {
    v = max(v, dpp_u32<0x111, 0xf>(v));
    v = max(v, dpp_u32<0x112, 0xf>(v));
    v = max(v, dpp_u32<0x114, 0xf>(v));
    v = max(v, dpp_u32<0x118, 0xf>(v));
    v = max(v, dpp_u32<0x142, 0xa>(v));
    v = max(v, dpp_u32<0x143, 0xc>(v));
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ uint32_t wave_sum_u32_u(uint32_t v) {
    v += dpp_u32<0x111, 0xf>(v);
    v += dpp_u32<0x112, 0xf>(v);
    v += dpp_u32<0x114, 0xf>(v);
    v += dpp_u32<0x118, 0xf>(v);
    v += dpp_u32<0x142, 0xa>(v);
    v += dpp_u32<0x143, 0xc>(v);
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ unsigned long long dpp_u64_max_step(unsigned long long v, uint32_t lo, uint32_t hi) {
    const unsigned long long w = ((unsigned long long)hi << 32) | lo;
    return w > v ? w : v;
}

__device__ __forceinline__ unsigned long long wave_max_u64_u(unsigned long long v) {
#define WC_MAX64_STEP(C, M) v = dpp_u64_max_step(v, dpp_u32<C, M>((uint32_t)v), dpp_u32<C, M>((uint32_t)(v >> 32)))
    WC_MAX64_STEP(0x111, 0xf);
    WC_MAX64_STEP(0x112, 0xf);
    WC_MAX64_STEP(0x114, 0xf);
    WC_MAX64_STEP(0x118, 0xf);
    WC_MAX64_STEP(0x142, 0xa);
    WC_MAX64_STEP(0x143, 0xc);
#undef WC_MAX64_STEP
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, 63), hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), 63);
    return ((unsigned long long)hi << 32) | lo;
}

// Load the x-pair (x, x+1) of a row as fp32 (fp64 cells narrowed RNE,
// src/preprocess.cpp:78).  `vec`: both elements in one aligned vector load.
// NT: non-temporal (streaming) vector load: the cells are read exactly once.
// Every K1 form loads its cells this way (round 6, profiles/r06/experiments/
// gpu_nt_cells.txt: C2 forward -6 %, K1 -12 % with the emit after it +6 %).
using f64x2 = double __attribute__((ext_vector_type(2)));
using f32x2 = float __attribute__((ext_vector_type(2)));
using f32x4 = float __attribute__((ext_vector_type(4)));

template <typename T, bool NT = false>
__device__ __forceinline__ void load_xpair(const T* __restrict__ p, bool two, bool vec,
                                           float& a, float& b) {
    if (two) {
        if (vec) {
            if constexpr (sizeof(T) == 8) {
                f64x2 d;
                if constexpr (NT)
                    d = __builtin_nontemporal_load(reinterpret_cast<const f64x2*>(p));
                else
                    d = *reinterpret_cast<const f64x2*>(p);
                a = (float)d.x;
                b = (float)d.y;
            } else {
                f32x2 d;
                if constexpr (NT)
                    d = __builtin_nontemporal_load(reinterpret_cast<const f32x2*>(p));
                else
                    d = *reinterpret_cast<const f32x2*>(p);
                a = d.x;
                b = d.y;
            }
        } else {
            a = (float)p[0];
            b = (float)p[1];
        }
    } else {
        a = (float)p[0];
        b = 0.0f;
    }
}

// Flat position of output index s (0 = low, 1 = high) of block b on an axis
// with h pairs and n cells: low -> b, high -> h + b, tail block (b == h) -> n - 1.
__device__ __forceinline__ int out_index(int b, int s, int h, int n) {
    return b < h ? b + s * h : n - 1;
}


// Block-wide (256 threads) exclusive sum + exclusive max, with carry-in.
struct ScanOut {
    uint64_t excl_sum, total_sum;
    uint32_t excl_max, total_max;
};

template <typename S>
__device__ __forceinline__ ScanOut block_scan_sum_max(S v, uint32_t m, S* s_sum, uint32_t* s_max) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    S incl = v;
    uint32_t im = m;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        S t = __shfl_up(incl, o);
        uint32_t tm = __shfl_up(im, o);
        if (l >= o) {
            incl += t;
            im = tm > im ? tm : im;
        }
    }
    if (l == 63) {
        s_sum[w] = incl;
        s_max[w] = im;
    }
    __syncthreads();
    S wbase = 0, tot = 0;
    uint32_t wmax = 0, totm = 0;
    for (int i = 0; i < 4; ++i) {
        if (i < w) {
            wbase += s_sum[i];
            wmax = s_max[i] > wmax ? s_max[i] : wmax;
        }
        tot += s_sum[i];
        totm = s_max[i] > totm ? s_max[i] : totm;
    }
    __syncthreads();
    ScanOut r;
    r.excl_sum = (uint64_t)(wbase + incl - v);
    // exclusive max: max over lanes < l in this wave and all earlier waves
    uint32_t em = __shfl_up(im, 1);
    if (l == 0) em = 0;
    r.excl_max = em > wmax ? em : wmax;
    r.total_sum = (uint64_t)tot;
    r.total_max = totm;
    return r;
}


// ---------------------------------------------------------------------------
// Hand-offs between workgroups of one launch (MI355X_MICROARCH.md, Valid
// forms): relaxed agent-scope atomics on self-validating 8-B granules (the
// word carries its own data, so no fence is needed), bounded waits.
constexpr uint32_t kSpinSelf = 64;  // polls (~0.1 ms with the backoff) before a wave derives a predecessor itself
constexpr unsigned long long kFlagAgg = 1ull << 62;   // granule holds this tile's aggregate
constexpr unsigned long long kFlagIncl = 2ull << 62;  // granule holds the inclusive prefix
constexpr unsigned long long kMask62 = (1ull << 62) - 1;

__device__ __forceinline__ uint32_t ld_rlx(const uint32_t* p) {
    return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_rlx(const unsigned long long* p) {
    return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void add_rlx(uint32_t* p, uint32_t v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A look-back wave that derived an unpublished predecessor's aggregate
// publishes it for the waves after it (one lane): swapped in only while the
// granule still holds `seen`, the unpublished value that lane polled.  The
// tile's own block, or another wave that derived it too, may have published
// meanwhile: the same aggregate, or the inclusive prefix, which is kept.
__device__ __forceinline__ void publish_derived(unsigned long long* p, unsigned long long seen,
                                                unsigned long long v) {
    __hip_atomic_compare_exchange_strong(p, &seen, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
}

// Look-back waits with backoff: pollers share the memory system with the
// streaming loads (MI355X_MICROARCH.md: 255 pollers cut chip bandwidth
// 37-71 %), so re-polls slow down from ~0.2 us to ~1.7 us.  A wait is never
// left to another workgroup's progress: once a wave has polled an
// unpublished predecessor tile err[1] times (WC_OPT_SPIN_LIMIT; 0 = the default
// kSpinSelf, ~0.1 ms), it derives that tile's aggregate from the tile's own
// inputs (which an earlier launch wrote) and moves on.  So no wait depends on
// which workgroups the hardware has dispatched, in any order, beside any other
// kernel (DESIGN.md §Forward progress).  err[1] is read only by a wave that is
// already waiting.  The derived aggregate is published into the predecessor's
// granule (publish_derived), so waves after it reuse it instead of deriving
// the same tile again, and a wave's poll count restarts whenever a poll makes
// progress: each unpublished tile costs one bounded wait and one derivation,
// not one per waiting wave (no O(tiles^2) work when a share of a launch's
// workgroups is held back, e.g. by another process on one XCD).
#ifndef WC_SPIN_S0
#define WC_SPIN_S0 8  // s_sleep units (64 clocks) before re-polls 1-3
#endif
#ifndef WC_SPIN_S1
#define WC_SPIN_S1 24  // ... before re-polls 4-15
#endif
__device__ __forceinline__ bool spin_wait(uint32_t& spins, const uint32_t* err) {
    const uint32_t lim = __hip_atomic_load(const_cast<uint32_t*>(err + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (spins >= (lim ? lim : kSpinSelf)) return true;  // lim 1: after the first unanswered poll
    ++spins;
    if (spins < 4)
        __builtin_amdgcn_s_sleep(WC_SPIN_S0);
    else if (spins < 16)
        __builtin_amdgcn_s_sleep(WC_SPIN_S1);
    else
        __builtin_amdgcn_s_sleep(64);
    return false;
}

// Decoupled look-back (one wave): exclusive prefix of tile t from granules
// st[0..t) of 62-bit sums.  A window of the 64 nearest predecessors (lane l =
// tile pos - l; indices below 0 read as an inclusive 0) is summed up to the
// nearest inclusive granule once every lane before it has published; a run
// of published aggregates before the first unpublished tile is summed and
// the window slides past it.  A predecessor still unpublished after the wait
// bound is summed from agg(tile) (a wave-uniform call by the whole wave: the
// tile's aggregate derived from its inputs, as its own block would publish it),
// and published there as an aggregate granule.
template <class Agg>
__device__ __forceinline__ unsigned long long lookback_sum62(unsigned long long* st, int64_t t, int l,
                                                             const uint32_t* err, Agg agg) {
    unsigned long long excl = 0;
    int64_t pos = t - 1;
    for (uint32_t spins = 0;;) {
        const int64_t idx = pos - l;
        const unsigned long long v = idx >= 0 ? ld_rlx(st + idx) : kFlagIncl;
        const unsigned long long incl = __ballot((v >> 62) == 2);
        const unsigned long long zero = __ballot((v >> 62) == 0);
        const int kI = incl ? __ffsll((long long)incl) - 1 : 64;
        const int kZ = zero ? __ffsll((long long)zero) - 1 : 64;
        const int take = kI < kZ ? kI + 1 : kZ;  // lanes [0, take) are summed
        if (take > 0) {
            excl += wave_sum(l < take ? (v & kMask62) : 0ull);
            spins = 0;  // progress: a later unpublished tile gets a full wait
        }
        if (kI < kZ) break;
        pos -= take;
        if (take == 0 && spin_wait(spins, err)) {  // tile pos (lane 0's): derived here
            const unsigned long long a = agg(pos) & kMask62;
            if (l == 0) publish_derived(st + pos, v, kFlagAgg | a);
            excl += a;
            --pos;
        }
    }
    return excl & kMask62;
}

// Epoch-tagged granules: flag (2 bits) | epoch (30 bits) | 32-bit saturated
// sum.  A granule of another epoch (an earlier call) reads as unpublished, so
// a buffer of such granules needs zeroing only once, when it is allocated.
__device__ __forceinline__ unsigned long long granule_e(unsigned long long flag, uint32_t epoch, uint32_t sum) {
    return flag | ((unsigned long long)(epoch & kEpochMask) << 32) | sum;
}

// lookback_sum62 over epoch-tagged granules; the result saturates at 2^32 - 1
// (agg: a tile's saturated 32-bit sum).
template <class Agg>
__device__ __forceinline__ uint32_t lookback_sum32e(unsigned long long* st, int64_t t, int l,
                                                    const uint32_t* err, uint32_t epoch, Agg agg) {
    unsigned long long excl = 0;
    int64_t pos = t - 1;
    const uint32_t ep = epoch & kEpochMask;
    for (uint32_t spins = 0;;) {
        const int64_t idx = pos - l;
        const unsigned long long raw = idx >= 0 ? ld_rlx(st + idx) : granule_e(kFlagIncl, ep, 0u);
        const unsigned long long v = (uint32_t)(raw >> 32 & kEpochMask) != ep ? 0ull : raw;  // earlier call's: unpublished
        const unsigned long long incl = __ballot((v >> 62) == 2);
        const unsigned long long zero = __ballot((v >> 62) == 0);
        const int kI = incl ? __ffsll((long long)incl) - 1 : 64;
        const int kZ = zero ? __ffsll((long long)zero) - 1 : 64;
        const int take = kI < kZ ? kI + 1 : kZ;  // lanes [0, take) are summed
        if (take > 0) {
            excl += wave_sum(l < take ? (v & 0xffffffffull) : 0ull);
            spins = 0;
        }
        if (kI < kZ) break;
        pos -= take;
        if (take == 0 && spin_wait(spins, err)) {  // tile pos (lane 0's): derived here, published
            const uint32_t a = agg(pos);
            if (l == 0) publish_derived(st + pos, raw, granule_e(kFlagAgg, ep, a));
            excl += a;
            --pos;
        }
    }
    return excl > 0xffffffffull ? 0xffffffffu : (uint32_t)excl;
}

// Wave-wide inclusive sum (64 lanes) on DPP lane moves, GFX9 pattern:
// row_shr 1/2/4/8 within 16-lane rows, then row_bcast:15 and row_bcast:31
// carry into the next rows.  Lanes whose source is out of range read 0.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_update_dpp(0u, (uint32_t)v, CTRL, ROW_MASK, 0xf, false);
    const uint32_t hi = __builtin_amdgcn_update_dpp(0u, (uint32_t)(v >> 32), CTRL, ROW_MASK, 0xf, false);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_incl_sum(uint64_t v) {
    v += dpp_u64<0x111, 0xf>(v);  // row_shr:1
    v += dpp_u64<0x112, 0xf>(v);  // row_shr:2
    v += dpp_u64<0x114, 0xf>(v);  // row_shr:4
    v += dpp_u64<0x118, 0xf>(v);  // row_shr:8
    v += dpp_u64<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
    v += dpp_u64<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
    return v;
}

// Wave-wide inclusive sum of 32-bit values on DPP lane moves (wave_incl_sum's
// pattern); lanes whose source is out of range read 0.
__device__ __forceinline__ uint32_t wave_incl_sum32(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

// ---------------------------------------------------------------------------
// The row index of a payload (include/wavelet_amd.h wc_rowindex_bytes): for
// every flat row r = I*H + J of a unit (D consecutive flat coefficients, x
// slowest / z fastest, src/compressor.cpp:178-181) the entry (k, p_k - r*D),
// k the first pair whose flat position p_k is >= r*D (nrle and ncoeff when
// there is none), plus the sentinel row W*H.  Written by the row index kernel
// from a payload (wc_inverse.hip k_rowindex) or by the emit as it packs the
// pairs (wc_emit.h, wc_forward_rows); read by K6r.

// floor(p / D) for p < 2^31 (Granlund-Montgomery, N = 31): dmagic = m |
// (31 + l) << 32, l = ceil(log2 D), m = floor(2^(31+l) / D) + 1 < 2^32; for
// D a power of two m = 0 and the high word is log2 D: a shift (uniform branch).
__device__ __forceinline__ uint32_t div_rows(uint32_t p, uint64_t dmagic) {
    if ((uint32_t)dmagic == 0u) return p >> (uint32_t)(dmagic >> 32);
    return (uint32_t)(((uint64_t)p * (uint32_t)dmagic) >> (uint32_t)(dmagic >> 32));
}

// Rows [r_lo, r_lo + cnt) of this lane get (k, p - r * D).  Most lanes write 0
// or 1 row.  A lane whose pair follows a long run of zeros (an empty
// stretch of rows: the high-frequency sub-bands of a smooth field) has many:
// ranges of more than WC_ROWS_BIG rows are written by the whole wave, one
// range at a time, with coalesced stores; shorter ones by their own lane.
// Every lane of the wave calls it (uniform control flow).
#ifndef WC_ROWS_BIG
#define WC_ROWS_BIG 4
#endif
__device__ __forceinline__ void write_rows(uint2* __restrict__ ri, uint32_t r_lo, uint32_t cnt, uint32_t k,
                                           uint32_t p, uint32_t D, int l) {
    if (!__ballot(cnt > 1)) {
        if (cnt) ri[r_lo] = make_uint2(k, p - r_lo * D);
        return;
    }
    for (unsigned long long big = __ballot(cnt > WC_ROWS_BIG); big; big &= big - 1) {  // uniform
        const int src = __ffsll((long long)big) - 1;
        const uint32_t rl = __builtin_amdgcn_readlane(r_lo, src), c = __builtin_amdgcn_readlane(cnt, src);
        const uint32_t kk = __builtin_amdgcn_readlane(k, src), pp = __builtin_amdgcn_readlane(p, src);
        for (uint32_t j = (uint32_t)l; j < c; j += 64) ri[rl + j] = make_uint2(kk, pp - (rl + j) * D);
    }
    if (cnt <= WC_ROWS_BIG)
        for (uint32_t j = 0; j < cnt; ++j) ri[r_lo + j] = make_uint2(k, p - (r_lo + j) * D);
}

// Uniform reads of launch-constant tables (plan descriptors, tile lists) through
// the constant address space: scalar loads even after the kernel has stored to
// global memory (a vector load's vmcnt wait would also wait for loads in flight).
#if defined(__HIP_DEVICE_COMPILE__)
template <class T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* cst(const T* p) {
    return (const __attribute__((address_space(4))) T*)(uintptr_t)p;
}
#else  // host pass of the same source: kernels are not compiled for the host
template <class T>
__device__ __forceinline__ const T* cst(const T* p) {
    return p;
}
#endif

// Workgroup barrier for LDS hand-offs only: unlike __syncthreads() it does not
// wait for this wave's outstanding global loads (a prefetch stays in flight).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Workgroup max of a 64-bit key folded into *dst with ONE atomicMax per
// workgroup (all tiles of a unit update the same key word).  s: 4 LDS
// slots; contains a barrier (call from uniform control flow).
template <bool LDS_ONLY = false>
__device__ __forceinline__ void block_key_max(unsigned long long v, unsigned long long* s,
                                              unsigned long long* dst) {
    v = wave_max_u64_u(v);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
    if constexpr (LDS_ONLY)
        lds_barrier();
    else
        __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = s[0];
        for (int i = 1; i < (int)(blockDim.x >> 6); ++i) m = s[i] > m ? s[i] : m;
        if (m != 0) atomicMax(dst, m);
    }
}

// Coefficient-magnitude histogram of the opt-in global-threshold mode
// (wc_hist.hip, k_transform_hist): bin = fp32 bits of |c| >> kHistShift,
// NaN not counted.  One LDS atomic per coefficient: a wave-aggregated form
// (the first pending lane's bin counted by ballot, one atomic for its lanes)
// measured 1.6 ms slower in C4's K1 (profiles/r06/experiments/gpu_hist_split.txt).
constexpr int kHistBins = 4096;
constexpr int kHistShift = 19;

__device__ __forceinline__ void hist_add(uint32_t* h, float v, bool valid) {
    const uint32_t m = __float_as_uint(v) & 0x7fffffffu;
    if (valid && m <= 0x7f800000u) atomicAdd(h + (m >> kHistShift), 1u);  // NaN is not counted
}

}  // namespace wc

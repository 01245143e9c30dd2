// wc_compact.hip — staged threshold + ordered pack over flat fp32 coefficients
// (the path for units the fused kernel does not take; wc_fused.hip).
//   K2a k_flat_count    per flat tile: kept count + last kept   src/compressor.cpp:216-234
//   K2b k_unit_scan     per unit: exclusive scan over its tiles
//   K2c k_unit_offsets  payload slot offsets + 20-byte headers  src/compressor.cpp:55-71
//   K2d k_flat_emit     ordered compaction -> (run, value) pairs src/compressor.cpp:24-42, :73-77
#include "wc_device.h"

namespace wc {

// thresh = (signed max) * (1 - keep)   src/compressor.cpp:212-216
__device__ __forceinline__ double unit_thresh(const UnitDev& U, unsigned long long key,
                                              const float* __restrict__ coef, double keep) {
    if (key == kKeyNaNFirst) return __longlong_as_double(0x7ff8000000000000ll);
    const uint32_t f = 0xffffffffu - (uint32_t)(key & 0xffffffffull);
    const double max_val = (double)coef[U.coef_off + f];
    return max_val * (1.0 - keep);
}

// ---------------------------------------------------------------------------
// K2a: kept count and last kept flat index (+1, 0 = none) per flat tile.
// Thread t = (wave w, lane l) owns elements w*1024 + it*256 + 4l + j.
__global__ __launch_bounds__(kThreads) void k_flat_count(
    const float* __restrict__ coef, const UnitDev* __restrict__ units, const FTile* __restrict__ tiles,
    const unsigned long long* __restrict__ unit_key, double keep, uint32_t* __restrict__ tcount,
    uint32_t* __restrict__ tlast) {
    __shared__ uint32_t s_cnt[4], s_last[4];
    const FTile ft = tiles[blockIdx.x];
    const UnitDev& U = units[ft.unit];
    const float tf = thresh_as_float(unit_thresh(U, unit_key[ft.unit], coef, keep));
    const int64_t start = (int64_t)ft.index * kFlatTile;
    const int len = (int)min((int64_t)kFlatTile, (int64_t)U.ncells - start);
    const float4* __restrict__ p4 = reinterpret_cast<const float4*>(coef + U.coef_off + start);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;

    float4 q[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) q[it] = p4[w * 256 + it * 64 + l];

    uint32_t cnt = 0, last = 0;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const float e[4] = {q[it].x, q[it].y, q[it].z, q[it].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int idx = w * 1024 + it * 256 + l * 4 + j;
            const bool k = idx < len && fabsf(e[j]) > tf;
            cnt += k;
            if (k) last = (uint32_t)(start + idx + 1);
        }
    }
    cnt = wave_sum(cnt);
    last = wave_max_u32(last);
    if (l == 0) {
        s_cnt[w] = cnt;
        s_last[w] = last;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t c = 0, m = 0;
        for (int i = 0; i < 4; ++i) {
            c += s_cnt[i];
            m = s_last[i] > m ? s_last[i] : m;
        }
        tcount[blockIdx.x] = c;
        tlast[blockIdx.x] = m;
    }
}

// ---------------------------------------------------------------------------
// K2b: per unit, exclusive scan of its tiles' kept counts / last kept.
__global__ __launch_bounds__(kThreads) void k_unit_scan(
    const UnitDev* __restrict__ units, const uint32_t* __restrict__ tcount,
    const uint32_t* __restrict__ tlast, uint32_t* __restrict__ toff, uint32_t* __restrict__ tprev,
    uint32_t* __restrict__ kept) {
    __shared__ uint32_t s_sum[4], s_max[4];
    const UnitDev& U = units[blockIdx.x];
    if (U.fused) return;  // kept/offsets/header come from k_forward_fused
    uint32_t base = 0, prev = 0;
    for (uint32_t c0 = 0; c0 < U.nftiles; c0 += kThreads) {
        const uint32_t i = c0 + threadIdx.x;
        const bool ok = i < U.nftiles;
        const uint32_t t = U.ftile_begin + i;
        const uint32_t cnt = ok ? tcount[t] : 0;
        const uint32_t lst = ok ? tlast[t] : 0;
        ScanOut s = block_scan_sum_max<uint32_t>(cnt, lst, s_sum, s_max);
        if (ok) {
            toff[t] = base + (uint32_t)s.excl_sum;
            tprev[t] = s.excl_max > prev ? s.excl_max : prev;
        }
        base += (uint32_t)s.total_sum;
        prev = s.total_max > prev ? s.total_max : prev;
    }
    if (threadIdx.x == 0) kept[blockIdx.x] = base;
}

// ---------------------------------------------------------------------------
// K2c: slot offsets (fixed: prefix of worst-case sizes, so no cross-unit scan)
// and the 20-byte header (src/compressor.cpp:59-71) of every staged unit.
__global__ __launch_bounds__(256) void k_unit_offsets(const UnitDev* __restrict__ units, int n,
                                                    const uint32_t* __restrict__ kept,
                                                    uint8_t* __restrict__ payload,
                                                    uint64_t* __restrict__ offsets) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= n) return;
    const UnitDev& U = units[u];
    if (U.fused) return;
    const uint32_t k = kept[u];
    int32_t* h = reinterpret_cast<int32_t*>(payload + U.pay_off);
    h[0] = U.nx;
    h[1] = U.ny;
    h[2] = U.nz;
    h[3] = (int32_t)U.ncells;
    h[4] = (int32_t)k;
    offsets[u] = U.pay_off;
    if (u == n - 1) offsets[n] = U.pay_off + 20 + 8ull * k;
}

// Host-path compaction: packed offsets (== 4 mod 8) from kept counts ...
__global__ __launch_bounds__(1024) void k_pack_offsets(int n, const uint32_t* __restrict__ kept,
                                                     uint64_t* __restrict__ packed) {
    __shared__ uint64_t s_w[16];
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t carry = 4;
    for (int c0 = 0; c0 < n; c0 += 1024) {
        const int u = c0 + threadIdx.x;
        const bool ok = u < n;
        const uint64_t k = ok ? kept[u] : 0;
        const uint64_t sz = ok ? 24 + 8 * k : 0;
        uint64_t incl = sz;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            uint64_t t = __shfl_up(incl, o);
            if (l >= o) incl += t;
        }
        if (l == 63) s_w[w] = incl;
        __syncthreads();
        uint64_t wb = 0, tot = 0;
        for (int i = 0; i < 16; ++i) {
            if (i < w) wb += s_w[i];
            tot += s_w[i];
        }
        __syncthreads();
        if (ok) {
            const uint64_t off = carry + wb + incl - sz;
            packed[u] = off;
            if (u == n - 1) packed[n] = off + 20 + 8 * k;
        }
        carry += tot;
    }
}

// ... and the copy of each unit's bytes from its slot to its packed offset.
__global__ __launch_bounds__(256) void k_pack_copy(const UnitDev* __restrict__ units,
                                                 const uint32_t* __restrict__ kept,
                                                 const uint8_t* __restrict__ src, const uint64_t* __restrict__ packed,
                                                 uint8_t* __restrict__ dst) {
    const int u = blockIdx.x;
    const UnitDev& U = units[u];
    const uint64_t words = (20 + 8ull * kept[u]) / 4;
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src + U.pay_off);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst + packed[u]);
    for (uint64_t i = threadIdx.x; i < words; i += blockDim.x) d[i] = s[i];
}

// ---------------------------------------------------------------------------
// K2d: ordered compaction.  The keep mask of each element is re-derived from
// the coefficient; ranks come from wave ballots + a 4-wave prefix; the run
// length is the distance to the previous kept flat index (rle_encode's
// "falses since the last true", src/compressor.cpp:31-38).
__global__ __launch_bounds__(kThreads) void k_flat_emit(
    const float* __restrict__ coef, const UnitDev* __restrict__ units, const FTile* __restrict__ tiles,
    const unsigned long long* __restrict__ unit_key, double keep, const uint32_t* __restrict__ toff,
    const uint32_t* __restrict__ tprev, const uint64_t* __restrict__ offsets,
    uint8_t* __restrict__ payload) {
    __shared__ uint32_t s_cnt[4], s_last[4];
    const FTile ft = tiles[blockIdx.x];
    const UnitDev& U = units[ft.unit];
    const float tf = thresh_as_float(unit_thresh(U, unit_key[ft.unit], coef, keep));
    const int64_t start = (int64_t)ft.index * kFlatTile;
    const int len = (int)min((int64_t)kFlatTile, (int64_t)U.ncells - start);
    const float4* __restrict__ p4 = reinterpret_cast<const float4*>(coef + U.coef_off + start);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const unsigned long long lt = (1ull << l) - 1ull;

    float4 q[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) q[it] = p4[w * 256 + it * 64 + l];

    uint32_t kb = 0;  // keep bits, bit it*4 + j
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const float e[4] = {q[it].x, q[it].y, q[it].z, q[it].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int idx = w * 1024 + it * 256 + l * 4 + j;
            const bool k = idx < len && fabsf(e[j]) > tf;
            kb |= (uint32_t)k << (it * 4 + j);
        }
    }
    // Wave totals: count and last kept (local index + 1).
    const uint32_t wcnt = wave_sum((uint32_t)__popc(kb));
    uint32_t mylast = kb ? (uint32_t)(w * 1024 + (31 - __clz(kb)) / 4 * 256 + l * 4 + ((31 - __clz(kb)) & 3) + 1) : 0u;
    const uint32_t wlast = wave_max_u32(mylast);
    if (l == 0) {
        s_cnt[w] = wcnt;
        s_last[w] = wlast;
    }
    __syncthreads();
    uint32_t base = toff[blockIdx.x];
    // prev kept flat index (unit-relative), -1 = none
    int64_t prev = (int64_t)tprev[blockIdx.x] - 1;
    for (int i = 0; i < w; ++i) {
        base += s_cnt[i];
        if (s_last[i]) prev = start + (int64_t)s_last[i] - 1;
    }
    uint8_t* __restrict__ pairs = payload + U.pay_off + 20;

#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const uint32_t nib = (kb >> (it * 4)) & 0xfu;
        const unsigned long long b0 = __ballot(nib & 1), b1 = __ballot(nib & 2),
                                 b2 = __ballot(nib & 4), b3 = __ballot(nib & 8);
        const unsigned long long any = b0 | b1 | b2 | b3;
        const uint32_t pre = __popcll(b0 & lt) + __popcll(b1 & lt) + __popcll(b2 & lt) + __popcll(b3 & lt);
        const uint32_t itot = __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
        const int64_t ebase = start + w * 1024 + it * 256;  // unit-relative flat index of lane 0, j 0
        const int lastj = nib ? 31 - __clz(nib) : 0;
        const int64_t lane_last = ebase + l * 4 + lastj;
        // previous kept element before this lane: highest lower lane with any kept
        const unsigned long long below = any & lt;
        const int src = below ? 63 - __clzll(below) : l;
        const int64_t from_lane = __shfl(lane_last, src);
        int64_t p = below ? from_lane : prev;
        uint32_t r = base + pre;
        if (nib) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (nib & (1u << j)) {
                    const int64_t f = ebase + l * 4 + j;
                    uint2 pr;
                    pr.x = (uint32_t)(int32_t)(f - p - 1);
                    pr.y = __float_as_uint(j == 0 ? q[it].x : j == 1 ? q[it].y : j == 2 ? q[it].z : q[it].w);
                    *reinterpret_cast<uint2*>(pairs + 8ull * r) = pr;
                    p = f;
                    ++r;
                }
            }
        }
        base += itot;
        if (any) {
            const int top = 63 - __clzll(any);
            prev = __shfl(lane_last, top);
        }
    }
}

// ---------------------------------------------------------------------------
// Launch wrappers
hipError_t launch_flat_count(hipStream_t st, const float* coef, const UnitDev* units, const FTile* ftiles,
                             uint32_t nft, const unsigned long long* keys, double keep, uint32_t* tcount,
                             uint32_t* tlast) {
    if (nft) k_flat_count<<<nft, kThreads, 0, st>>>(coef, units, ftiles, keys, keep, tcount, tlast);
    return hipGetLastError();
}

hipError_t launch_unit_scan(hipStream_t st, const UnitDev* units, int n, const uint32_t* tcount,
                            const uint32_t* tlast, uint32_t* toff, uint32_t* tprev, uint32_t* kept) {
    k_unit_scan<<<n, kThreads, 0, st>>>(units, tcount, tlast, toff, tprev, kept);
    return hipGetLastError();
}

hipError_t launch_unit_offsets(hipStream_t st, const UnitDev* units, int n, const uint32_t* kept,
                               uint8_t* payload, uint64_t* offsets) {
    k_unit_offsets<<<(n + 255) / 256, 256, 0, st>>>(units, n, kept, payload, offsets);
    return hipGetLastError();
}

hipError_t launch_pack(hipStream_t st, const UnitDev* units, int n, const uint32_t* kept, const uint8_t* src,
                       uint64_t* packed, uint8_t* dst) {
    k_pack_offsets<<<1, 1024, 0, st>>>(n, kept, packed);
    k_pack_copy<<<n, 256, 0, st>>>(units, kept, src, packed, dst);
    return hipGetLastError();
}

hipError_t launch_flat_emit(hipStream_t st, const float* coef, const UnitDev* units, const FTile* ftiles,
                            uint32_t nft, const unsigned long long* keys, double keep, const uint32_t* toff,
                            const uint32_t* tprev, const uint64_t* offsets, uint8_t* payload) {
    if (nft)
        k_flat_emit<<<nft, kThreads, 0, st>>>(coef, units, ftiles, keys, keep, toff, tprev, offsets, payload);
    return hipGetLastError();
}

}  // namespace wc

// wc_fused.hip — single-read forward path: transform + keep threshold + ordered
// pack in ONE kernel, for units with even W, H and D % 8 == 0 whose tile count
// G fits comfortably in the resident grid.
//
//   src/compressor.cpp:85-185  wavelet_decompose  -> phase 1 (coefficients stay in LDS)
//   src/compressor.cpp:212-216 signed max, thresh -> phase 2 (box-wide max exchange)
//   src/compressor.cpp:222-238 mask + rle_encode  -> phases 3-5 (segment scan, emit)
//   src/compressor.cpp:55-80   serialize          -> header + pairs written in place
//
// A unit (one Box3D component) is cut into G transform tiles (the fast K1 tile:
// up to 32 x-blocks x 32 z-blocks, 4 z-blocks per thread).  Every tile:
//   1. takes a ticket (atomic counter) -> tile index.  Tiles of one unit have
//      consecutive tickets, so a tile only ever waits for tiles that have
//      already started; with >= G resident slots the grid cannot deadlock.
//   2. loads its cells once, transforms them into LDS rows keyed by flat row
//      (I, J) and reduces its max-|c| key (|c| bits, first flat index, sign).
//   3. publishes the key as one self-validating 8-byte granule and waits for
//      all G granules of its unit -> thresh = signed max * (1 - keep).
//   4. thresholds its rows (wave ballots) and publishes one record per
//      segment (a TZ-long piece of a flat row: kept count, last kept).
//   5. the last tile of the unit to arrive scans the unit's records in flat
//      order (exclusive count -> pair offset, exclusive max -> previous kept
//      flat index) and publishes them; the others wait for its ready flag.
//   6. every tile emits its kept coefficients as (run, value) pairs straight
//      into the unit's payload slot.
// Hand-offs follow MI355X_MICROARCH.md "Valid forms": sc1 (agent-scope relaxed
// atomic) stores drained by s_waitcnt vmcnt(0) before a workgroup barrier and
// the signalling atomic; sc1 loads after the poll/ticket.  Every spin is
// bounded and raises kErrTimeout instead of hanging.
#include "wc_device.h"

namespace wc {

constexpr unsigned long long kValid = 1ull << 63;
constexpr uint32_t kSpinLimit = 1u << 22;
// Segment records the last arriver scans per thread (plan caps a fused unit at
// kThreads * kScanPer segments).
constexpr int kScanPer = 32;

__device__ __forceinline__ void st_rlx(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_rlx(const uint32_t* p) {
    return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_rlx(const unsigned long long* p) {
    return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Fused max key: valid | |c| bits (62..32) | (0x7fffffff - f) (31..1) | sign (0).
// Larger key = larger magnitude, then smaller flat index (std::max_element's
// first-wins); the sign rides along so thresh needs no second lookup.
__device__ __forceinline__ unsigned long long fused_key(float c, uint32_t f) {
    const uint32_t bits = __float_as_uint(c);
    const uint32_t ab = bits & 0x7fffffffu;
    if (ab > 0x7f800000u) return f == 0 ? ~0ull : 0ull;  // NaN: only flat[0] can win (NaN thresh)
    return ((unsigned long long)ab << 32) | ((unsigned long long)(0x7fffffffu - f) << 1) | (bits >> 31);
}

__device__ __forceinline__ double key_thresh(unsigned long long key, double keep) {
    const uint32_t ab = (uint32_t)(key >> 32) & 0x7fffffffu;
    if (ab == 0x7fffffffu) return __longlong_as_double(0x7ff8000000000000ll);
    const float maxv = __uint_as_float(ab | ((uint32_t)(key & 1ull) << 31));
    return (double)maxv * (1.0 - keep);
}


// Segment id of (flat row (I, J), z half sz, z tile tz): flat order.
__device__ __forceinline__ uint32_t seg_id(int I, int J, int H, int sz, int tz, int ntz) {
    return (uint32_t)((((int64_t)I * H + J) * 2 + sz) * ntz + tz);
}

template <typename T>
__global__ __launch_bounds__(kThreads, 4) void k_forward_fused(FusedParams P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;

    // Carve the tail of the dynamic LDS: misc words first (fixed), the tile after.
    unsigned long long* misc = reinterpret_cast<unsigned long long*>(lds);  // 16 words
    // misc[0]: ticket   misc[1]: thresh (double bits)   misc[2]: last-arriver flag
    // misc[4..7]: per-wave key maxima   misc[8..11]: per-wave scan totals
    if (tid == 0) misc[0] = atomicAdd(P.ticket, 1u);
    __syncthreads();
    const uint32_t t = (uint32_t)misc[0];
    if (t >= P.ntiles) return;
    const XTile td = P.tiles[t];
    const UnitDev& U = P.units[td.unit];
    const int W = U.nx, H = U.ny, D = U.nz;
    const int hx = U.hx, hy = U.hy, hz = U.hz;
    const int lbx = U.lbx, lby = U.lby, lbz = U.lbz;
    const int TX = 1 << lbx, TY = 1 << lby, TZ = 1 << lbz;
    const int rowlen = 2 * TZ, rstride = rowlen + 4;
    const int nrows = 4 * TX * TY;
    const int nelem = nrows * rowlen;
    const int nchunk = (nelem + 63) >> 6;
    const int tz = td.bz0 >> lbz;
    float* rows = lds + 32;                                                  // after misc (128 B)
    unsigned long long* masks = reinterpret_cast<unsigned long long*>(rows + nrows * rstride);

    // ---- phase 1: load + transform into LDS rows, local max key ----------
    const int64_t sy = W, sz = (int64_t)W * H;
    const T* __restrict__ src = static_cast<const T*>(P.cells) + U.cell_off;
    const bool vec = (U.cell_off & 1) == 0;
    const int ncol = (TX * TY * TZ) >> 2;
    unsigned long long kmax = 0;
    for (int ci = tid; ci < ncol; ci += kThreads) {
        const int bxl = ci & (TX - 1);
        const int byl = (ci >> lbx) & (TY - 1);
        const int bzq = ci >> (lbx + lby);
        const int bx = td.bx0 + bxl, by = td.by0 + byl, bzb = td.bz0 + 4 * bzq;
        if (bx >= hx || by >= hy || bzb >= hz) continue;
        float v[8][2][2];
        const T* p0 = src + 2 * (int64_t)bx + sy * (2 * by) + sz * (2 * (int64_t)bzb);
#pragma unroll
        for (int zp = 0; zp < 8; ++zp)
#pragma unroll
            for (int dy = 0; dy < 2; ++dy) load_xpair<T>(p0 + sz * zp + sy * dy, true, vec, v[zp][dy][0], v[zp][dy][1]);
        float c[4][2][2][2];  // [q][sz][sy][sx]
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float a[2][2][2];
#pragma unroll
            for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                for (int dx = 0; dx < 2; ++dx) {
                    a[0][dy][dx] = haar_lo(v[2 * q][dy][dx], v[2 * q + 1][dy][dx]);
                    a[1][dy][dx] = haar_hi(v[2 * q][dy][dx], v[2 * q + 1][dy][dx]);
                }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                float b[2][2];
#pragma unroll
                for (int dx = 0; dx < 2; ++dx) {
                    b[0][dx] = haar_lo(a[s][0][dx], a[s][1][dx]);
                    b[1][dx] = haar_hi(a[s][0][dx], a[s][1][dx]);
                }
#pragma unroll
                for (int tt = 0; tt < 2; ++tt) {
                    c[q][s][tt][0] = haar_lo(b[tt][0], b[tt][1]);
                    c[q][s][tt][1] = haar_hi(b[tt][0], b[tt][1]);
                }
            }
        }
#pragma unroll
        for (int ssz = 0; ssz < 2; ++ssz)
#pragma unroll
            for (int ssy = 0; ssy < 2; ++ssy)
#pragma unroll
                for (int ssx = 0; ssx < 2; ++ssx) {
                    const int row = ((((ssy << lby) + byl) * 2 + ssx) << lbx) + bxl;
                    *reinterpret_cast<float4*>(rows + row * rstride + (ssz << lbz) + 4 * bzq) =
                        make_float4(c[0][ssz][ssy][ssx], c[1][ssz][ssy][ssx], c[2][ssz][ssy][ssx],
                                    c[3][ssz][ssy][ssx]);
                    const int I = bx + ssx * hx, J = by + ssy * hy, K = bzb + ssz * hz;
                    const uint32_t f0 = (uint32_t)(((int64_t)I * H + J) * D + K);
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const unsigned long long k = fused_key(c[q][ssz][ssy][ssx], f0 + q);
                        kmax = k > kmax ? k : kmax;
                    }
                }
    }
    kmax = wave_max_u64(kmax);
    if (lane == 0) misc[4 + w] = kmax;
    __syncthreads();

    // ---- phase 2: publish the key granule, wait for the unit's G granules --
    const uint32_t G = U.ntile_u, gbase = U.xt_begin;
    if (tid == 0) {
        unsigned long long k = misc[4];
        for (int i = 1; i < 4; ++i) k = misc[4 + i] > k ? misc[4 + i] : k;
        st_rlx(P.keyslot + t, k | kValid);
    }
    if (w == 0) {
        unsigned long long best = 0;
        for (uint32_t g0 = 0; g0 < G; g0 += 64) {
            const uint32_t gi = g0 + lane;
            const bool need = gi < G;
            unsigned long long v = 0;
            for (uint32_t spin = 0;; ++spin) {
                if (need) v = ld_rlx(P.keyslot + gbase + gi);
                if (__all(!need || (v & kValid))) break;
                if (spin > kSpinLimit) {
                    if (lane == 0) atomicOr(P.err, kErrTimeout);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            best = v > best ? v : best;
        }
        best = wave_max_u64(best);
        if (lane == 0) misc[1] = (unsigned long long)__double_as_longlong(key_thresh(best, P.keep));
    }
    __syncthreads();
    const double thresh = __longlong_as_double((long long)misc[1]);

    // ---- phase 3: threshold rows -> ballot masks + segment records ---------
    const int lrow = lbz + 1;
    for (int ch = w; ch < nchunk; ch += 4) {
        const int e = (ch << 6) + lane;
        const int row = e >> lrow, col = e & (rowlen - 1);
        const int bxl = row & (TX - 1);
        int r2 = row >> lbx;
        const int ssx = r2 & 1;
        r2 >>= 1;
        const int byl = r2 & (TY - 1), ssy = r2 >> lby;
        const int ssz = col >> lbz, bzl = col & (TZ - 1);
        const int bx = td.bx0 + bxl, by = td.by0 + byl;
        const bool rv = e < nelem && bx < hx && by < hy;
        const bool ev = rv && (td.bz0 + bzl) < hz;
        const float cv = e < nelem ? rows[row * rstride + col] : 0.0f;
        const bool keepv = ev && (double)fabsf(cv) > thresh;
        const unsigned long long m = __ballot(keepv);
        if (lane == 0) masks[ch] = m;
        if (rv && bzl == 0) {
            const unsigned long long segm = TZ >= 64 ? ~0ull : ((1ull << TZ) - 1ull);
            const unsigned long long sb = (m >> lane) & segm;
            const uint32_t cnt = (uint32_t)__popcll(sb);
            const uint32_t last1 = sb ? (uint32_t)(64 - __clzll(sb)) : 0u;  // last local index + 1
            const int I = bx + ssx * hx, J = by + ssy * hy;
            st_rlx(P.segrec + U.seg_off + seg_id(I, J, H, ssz, tz, U.ntz), cnt | (last1 << 8));
        }
    }
    drain_stores();
    __syncthreads();
    if (tid == 0) misc[2] = (atomicAdd(P.arrive + td.unit, 1u) == G - 1) ? 1ull : 0ull;
    __syncthreads();

    // ---- phase 4: last arriver scans the unit's segments in flat order -----
    // Thread t owns records [t*per, t*per + per): all its loads are issued
    // before any is used (kScanPer in flight), then a local scan, one block
    // scan, and the (offset, prev) stores.
    if (misc[2]) {
        const uint32_t nseg = (uint32_t)W * (uint32_t)H * 2u * (uint32_t)U.ntz;
        const uint32_t per = (nseg + kThreads - 1) / kThreads;  // <= kScanPer (plan guarantees)
        const uint32_t s0 = min(nseg, (uint32_t)tid * per), s1 = min(nseg, s0 + per);
        const uint32_t* rec = P.segrec + U.seg_off;
        const int ntz = U.ntz;
        uint32_t r[kScanPer];
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) r[k] = (s0 + k < s1) ? ld_rlx(rec + s0 + k) : 0u;
        // segment flat start: s = ((I*H + J) * 2 + sz) * ntz + tz
        auto seg_start = [&](uint32_t s) -> uint32_t {
            const uint32_t rowi = s / (2u * ntz), rem = s - rowi * 2u * ntz;
            const uint32_t ssz = rem / ntz, ttz = rem - ssz * ntz;
            return (uint32_t)((uint64_t)rowi * D + ttz * TZ + ssz * hz);
        };
        uint32_t cnt = 0, mx = 0;  // mx: last kept flat index + 1 in my range
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            cnt += r[k] & 0xffu;
            if (r[k] >> 8) mx = seg_start(s0 + k) + (r[k] >> 8);
        }
        uint32_t* s_sum = reinterpret_cast<uint32_t*>(misc + 8);   // misc[8..9]
        uint32_t* s_max = reinterpret_cast<uint32_t*>(misc + 10);  // misc[10..11]
        ScanOut sc = block_scan_sum_max<uint32_t>(cnt, mx, s_sum, s_max);
        uint32_t off = (uint32_t)sc.excl_sum, prev = sc.excl_max;
        unsigned long long* so = reinterpret_cast<unsigned long long*>(P.segoff + U.seg_off);
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            if (s0 + k < s1) {
                st_rlx(so + s0 + k, (unsigned long long)off | ((unsigned long long)prev << 32));
                off += r[k] & 0xffu;
                if (r[k] >> 8) prev = seg_start(s0 + k) + (r[k] >> 8);
            }
        }
        if (tid == 0) {
            const uint32_t total = (uint32_t)sc.total_sum;
            int32_t* h = reinterpret_cast<int32_t*>(P.payload + U.pay_off);
            h[0] = W;
            h[1] = H;
            h[2] = D;
            h[3] = (int32_t)U.ncells;
            h[4] = (int32_t)total;
            P.kept[td.unit] = total;
            P.offsets[td.unit] = U.pay_off;
            if ((int)td.unit == P.n - 1) P.offsets[P.n] = U.pay_off + 20 + 8ull * total;
        }
        drain_stores();
        __syncthreads();
        if (tid == 0) st_rlx(P.ready + td.unit, 1u);
    } else {
        if (tid == 0) {
            for (uint32_t spin = 0; ld_rlx(P.ready + td.unit) == 0u; ++spin) {
                if (spin > kSpinLimit) {
                    atomicOr(P.err, kErrTimeout);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
    }

    // ---- phase 5: emit (run, value) pairs from LDS --------------------------
    uint8_t* __restrict__ pairs = P.payload + U.pay_off + 20;
    for (int ch = w; ch < nchunk; ch += 4) {
        const unsigned long long m = masks[ch];
        if (m == 0ull) continue;  // wave-uniform; lanes past nelem never have a mask bit
        const int e = (ch << 6) + lane;
        const int row = e >> lrow, col = e & (rowlen - 1);
        const int bxl = row & (TX - 1);
        int r2 = row >> lbx;
        const int ssx = r2 & 1;
        r2 >>= 1;
        const int byl = r2 & (TY - 1), ssy = r2 >> lby;
        const int ssz = col >> lbz, bzl = col & (TZ - 1);
        const int bx = td.bx0 + bxl, by = td.by0 + byl;
        const int I = bx + ssx * hx, J = by + ssy * hy, K = td.bz0 + bzl + ssz * hz;
        const int sl = lane & ~(TZ - 1);  // first lane of my segment
        unsigned long long so = 0;
        if (lane == sl && ((m >> lane) & (TZ >= 64 ? ~0ull : ((1ull << TZ) - 1ull))))
            so = ld_rlx(reinterpret_cast<const unsigned long long*>(P.segoff + U.seg_off +
                                                                    seg_id(I, J, H, ssz, tz, U.ntz)));
        so = __shfl(so, sl);
        if ((m >> lane) & 1ull) {
            const unsigned long long below = m & ((1ull << lane) - 1ull) & ~((1ull << sl) - 1ull);
            const uint32_t rank = (uint32_t)so + (uint32_t)__popcll(below);
            const uint32_t f = (uint32_t)(((int64_t)I * H + J) * D + K);
            int32_t run;
            if (below)
                run = lane - (63 - __clzll(below)) - 1;
            else
                run = (int32_t)(f - (uint32_t)(so >> 32));  // f - prev - 1, with so.y = prev + 1
            uint2 pr;
            pr.x = (uint32_t)run;
            pr.y = __float_as_uint(rows[row * rstride + col]);
            *reinterpret_cast<uint2*>(pairs + 8ull * rank) = pr;
        }
    }
}

size_t fused_lds_bytes(int lbx, int lby, int lbz) {
    const size_t nrows = (size_t)4 << (lbx + lby);
    const size_t rowlen = (size_t)2 << lbz;
    const size_t nchunk = (nrows * rowlen + 63) / 64;
    return 128 + nrows * (rowlen + 4) * sizeof(float) + nchunk * 8;
}

hipError_t launch_forward_fused(hipStream_t st, int dtype, size_t lds, const FusedParams& p) {
    if (p.ntiles == 0) return hipSuccess;
    if (dtype == 1)
        k_forward_fused<double><<<p.ntiles, kThreads, lds, st>>>(p);
    else
        k_forward_fused<float><<<p.ntiles, kThreads, lds, st>>>(p);
    return hipGetLastError();
}

}  // namespace wc

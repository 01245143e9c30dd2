// wc_fused.hip — single-read forward path: transform + keep threshold + ordered
// pack in ONE kernel, for units whose transform tiles span the full x and z
// extent (even W, H, D % 8 == 0, W <= 64, D <= 64, <= kMaxFusedTiles tiles).
//
//   src/compressor.cpp:85-185  wavelet_decompose  -> phase 1 (coefficients stay in LDS)
//   src/compressor.cpp:212-216 signed max, thresh -> phase 2 (unit-wide max exchange)
//   src/compressor.cpp:222-238 mask + rle_encode  -> phases 3-5 (row table, scan, emit)
//   src/compressor.cpp:55-80   serialize          -> header + pairs written in place
//
// A unit (one Box3D component) is cut along y into G tiles; each tile owns
// complete flat rows (I, J) (x-slowest / z-fastest, :178-181).  Every tile:
//   0. takes a ticket (atomic counter) -> tile index.  Tiles of one unit hold
//      consecutive tickets, so a tile only waits for tiles that have started;
//      with >= G resident slots the grid cannot deadlock.
//   1. loads its cells once and transforms them into LDS rows; reduces its
//      max-|c| key (|c| bits, first flat index, sign).
//   2. publishes the key as one self-validating 8-byte granule and waits for
//      the unit's G granules -> thresh = signed max * (1 - keep).
//   3. thresholds its rows (wave ballots) and publishes one 14-bit record per
//      row (kept count, last kept + 1), four per self-validating granule.
//   4. reads the whole unit's row table (every tile does: no serial scan, no
//      ready flag) and block-scans it in flat order -> for its own rows the
//      pair offset and the previous kept flat index.
//   5. emits its kept coefficients as (run, value) pairs into the unit's slot;
//      tile 0 writes the 20-byte header, kept[u] and offsets[u].
// Two hand-offs per tile, both "data is the flag" granules (MI355X_MICROARCH.md
// Valid forms, R2): one 8-byte sc1 store per granule, relaxed agent-scope
// (sc1) loads to poll.  Every spin is bounded and raises kErrTimeout.
#include "wc_device.h"

namespace wc {

constexpr unsigned long long kValid = 1ull << 63;
constexpr uint32_t kSpinLimit = 1u << 22;


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



// Per-tile descriptors are read-only for the whole launch: read them through
// the constant address space so uniform indices become scalar (SMEM) loads
// into SGPRs instead of per-lane copies in VGPRs.
#define WC_CONST __attribute__((address_space(4)))
__device__ __forceinline__ XTile tile_at(const FusedParams& P, uint32_t t) {
    const WC_CONST XTile* p = (const WC_CONST XTile*)(uintptr_t)P.tiles + t;
    XTile r;
    r.unit = p->unit;
    r.bx0 = p->bx0;
    r.by0 = p->by0;
    r.bz0 = p->bz0;
    return r;
}
__device__ __forceinline__ const WC_CONST UnitDev& unit_at(const FusedParams& P, uint32_t u) {
    return ((const WC_CONST UnitDev*)(uintptr_t)P.units)[u];
}

// Lane-explicit wave64 shuffles (ds_bpermute from a caller-supplied lane):
// inside the persistent loop `lane` is opaque, so the compiler cannot hoist
// the per-lane shuffle addresses out of the loop and keep them live.
__device__ __forceinline__ uint32_t bperm(uint32_t v, int src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}
__device__ __forceinline__ unsigned long long bperm64(unsigned long long v, int src) {
    return (unsigned long long)bperm((uint32_t)v, src) | ((unsigned long long)bperm((uint32_t)(v >> 32), src) << 32);
}
__device__ __forceinline__ unsigned long long wmax64(unsigned long long v, int lane) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long x = bperm64(v, lane ^ o);
        v = x > v ? x : v;
    }
    return v;
}
// Block-wide (kThreads) exclusive sum + exclusive max; scratch s[0..3], s[64..67].
__device__ __forceinline__ void block_scan2(uint32_t v, uint32_t m, int tid, uint32_t* s, uint32_t& esum,
                                            uint32_t& emax, uint32_t& tsum) {
    const int l = tid & 63, w = tid >> 6;
    uint32_t incl = v, im = m;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int src = l >= o ? l - o : l;
        const uint32_t a = bperm(incl, src), b = bperm(im, src);
        if (l >= o) {
            incl += a;
            im = b > im ? b : im;
        }
    }
    if (l == 63) {
        s[w] = incl;
        s[64 + w] = im;
    }
    __syncthreads();
    uint32_t wbase = 0, wmax = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kThreads / 64; ++i) {
        if (i < w) {
            wbase += s[i];
            wmax = s[64 + i] > wmax ? s[64 + i] : wmax;
        }
        tot += s[i];
    }
    __syncthreads();
    uint32_t em = bperm(im, l > 0 ? l - 1 : 0);
    if (l == 0) em = 0;
    esum = wbase + incl - v;
    emax = em > wmax ? em : wmax;
    tsum = tot;
}

template <typename T>
struct Pair2;
template <>
struct Pair2<double> {
    using type = double2;
};
template <>
struct Pair2<float> {
    using type = float2;
};

// One transform column of a tile: x-pair x y-pair x 8 z-planes of raw cells
// (4 z-blocks), held in registers from issue to use so the loads of the
// next tile stay in flight while the current tile waits on its unit.
template <typename T>
struct RawCol {
    typename Pair2<T>::type r[8][2];
    bool act;
};

template <typename T>
__device__ __forceinline__ void issue_col(const FusedParams& P, const XTile& td, const WC_CONST UnitDev& U, int ci,
                                          RawCol<T>& c) {
    const int lbx = U.lbx, lby = U.lby;
    const int TX = 1 << lbx, TY = 1 << lby, TZ = 1 << U.lbz;
    const int bxl = ci & (TX - 1), byl = (ci >> lbx) & (TY - 1), bzq = ci >> (lbx + lby);
    const int bx = td.bx0 + bxl, by = td.by0 + byl, bzb = td.bz0 + 4 * bzq;
    c.act = ci < ((TX * TY * TZ) >> 2) && bx < U.hx && by < U.hy && bzb < U.hz;
    // fused units have an even cell offset (host check): x-pairs are aligned vectors
    const uint32_t sy = (uint32_t)U.nx, sz = (uint32_t)U.nx * (uint32_t)U.ny;
    const uint32_t o0 = c.act ? 2u * bx + sy * (2u * by) + sz * (2u * bzb) : 0u;
    const T* __restrict__ base = static_cast<const T*>(P.cells) + U.cell_off;
    using V = typename Pair2<T>::type;
#pragma unroll
    for (int zp = 0; zp < 8; ++zp)
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) {
            if (c.act)
                c.r[zp][dy] = *reinterpret_cast<const V*>(base + (o0 + sz * zp + sy * dy));
            else
                c.r[zp][dy] = V{0, 0};
        }
}

template <typename T>
__global__ __launch_bounds__(kThreads, 3) void k_forward_fused(FusedParams P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid0 = threadIdx.x;
    // misc[0] current tile, misc[1] thresh bits, misc[2] prefetched tile, misc[4..7] wave key maxima
    unsigned long long* misc = reinterpret_cast<unsigned long long*>(lds);
    if (tid0 == 0) misc[0] = atomicAdd(P.ticket, 1u);
    __syncthreads();
    uint32_t t = __builtin_amdgcn_readfirstlane((uint32_t)misc[0]);
    if (t >= P.ntiles) return;
    RawCol<T> raw;
    {
        const XTile tt = tile_at(P, t);
        issue_col<T>(P, tt, unit_at(P, tt.unit), tid0, raw);
    }

    // Persistent loop.  Tickets are claimed in order, so a unit's tiles hold
    // consecutive tickets; a workgroup waits only on its current tile's unit
    // and prefetches only a ticket of a LATER unit, so every waited-on tile is
    // either running or unclaimed (claimable by a finishing workgroup).
    for (;;) {
    int tid;  // opaque per iteration: keeps lane-derived values from being hoisted and held live
    asm volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"(tid0));
    const int w = tid >> 6, lane = tid & 63;
    const XTile td = tile_at(P, t);
    const WC_CONST UnitDev& U = unit_at(P, td.unit);
    const int W = U.nx, H = U.ny, D = U.nz;
    const int hx = U.hx, hy = U.hy, hz = U.hz;
    const int lbx = U.lbx, lby = U.lby, lbz = U.lbz;
    const int TX = 1 << lbx, TY = 1 << lby, TZ = 1 << lbz;
    const int rowlen = 2 * TZ, rstride = rowlen + 4;   // the tile spans all of z
    const int nrows = 4 * TX * TY;
    const uint32_t G = U.ntile_u;
    const uint32_t gme = t - U.xt_begin;               // my tile index within the unit (along y)
    // LDS carve (16-B aligned pieces)
    uint32_t* slab = reinterpret_cast<uint32_t*>(lds + 32);  // block-scan scratch
    float* rows = lds + 32 + 128;
    unsigned long long* masks = reinterpret_cast<unsigned long long*>(rows + nrows * rstride);  // per row
    uint32_t* own_off = reinterpret_cast<uint32_t*>(masks + nrows);
    uint32_t* own_prev = own_off + nrows;
    uint16_t* tab = reinterpret_cast<uint16_t*>(own_prev + nrows + 2 * kThreads);  // 4096 records; rec[] aliases

    // ---- phase 1: transform the landed column into LDS rows, local max key -
    unsigned long long kmax = 0;
    if (raw.act) {
        const int ci = tid;
        const int bxl = ci & (TX - 1);
        const int byl = (ci >> lbx) & (TY - 1);
        const int bzq = ci >> (lbx + lby);
        const int bx = td.bx0 + bxl, by = td.by0 + byl, bzb = td.bz0 + 4 * bzq;
        float v[8][2][2];
#pragma unroll
        for (int zp = 0; zp < 8; ++zp)
#pragma unroll
            for (int dy = 0; dy < 2; ++dy) {
                v[zp][dy][0] = (float)raw.r[zp][dy].x;  // fp64 -> fp32 RNE, src/preprocess.cpp:78
                v[zp][dy][1] = (float)raw.r[zp][dy].y;
            }
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
    kmax = wmax64(kmax, lane);
    if (lane == 0) misc[4 + w] = kmax;
    // claim the next tile now, so its loads overlap this tile's hand-offs --
    // only when the counter has already passed my unit: it never decreases,
    // so the ticket the add returns is then of a later unit too.
    if (tid == 0) {
        const uint32_t later = U.xt_begin + G;  // first ticket of a later unit
        const uint32_t cur = __hip_atomic_load(P.ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t nxt = 0xffffffffu;
        if (cur >= later && cur < P.ntiles) nxt = atomicAdd(P.ticket, 1u);
        misc[2] = nxt;
    }
    __syncthreads();
    const uint32_t tnext = __builtin_amdgcn_readfirstlane((uint32_t)misc[2]);
    if (tnext < P.ntiles) {
        const XTile tt = tile_at(P, tnext);
        issue_col<T>(P, tt, unit_at(P, tt.unit), tid, raw);
    }

    // ---- phase 2: publish the key granule, wait for the unit's G granules --
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
                if (need) v = ld_rlx(P.keyslot + U.xt_begin + gi);
                if (__all(!need || (v & kValid))) break;
                if (spin > kSpinLimit) {
                    if (lane == 0) atomicOr(P.err, kErrTimeout);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            best = v > best ? v : best;
        }
        best = wmax64(best, lane);
        if (lane == 0) misc[1] = (unsigned long long)__double_as_longlong(key_thresh(best, P.keep));
    }
    __syncthreads();
    const double thresh = __longlong_as_double((long long)misc[1]);

    // ---- phase 3: threshold rows -> per-row keep masks + records ----------
    // 4 consecutive columns per lane (one 16-B LDS read), lpr lanes per row.
    // Column c holds K = (c mod TZ) + (c / TZ) * hz; hz % 4 == 0, so a lane's
    // four columns are all valid or all padding and map to 4 consecutive K.
    const int lpr = rowlen >> 2, llpr = lbz - 1;  // lanes per row, log2
    const int rpw = 64 >> llpr;                    // rows per wave-iteration
    const float tf = thresh_as_float(thresh);
    uint16_t* rec = tab;  // my records, published below, then overwritten by the table
    for (int rb = w * rpw; rb < nrows; rb += 4 * rpw) {
        const int row = rb + (lane >> llpr), q = lane & (lpr - 1);
        const int bxl = row & (TX - 1);
        const int byl = ((row >> lbx) >> 1) & (TY - 1);
        const int zc = (4 * q) & (TZ - 1), kb = zc + ((4 * q) >> lbz) * hz;  // column -> K offset
        const bool rv = row < nrows && td.bx0 + bxl < hx && td.by0 + byl < hy && zc < hz;
        unsigned long long m = 0;
        if (rv) {
            const float4 v4 = *reinterpret_cast<const float4*>(rows + row * rstride + 4 * q);
            const uint32_t nib = (uint32_t)(fabsf(v4.x) > tf) | ((uint32_t)(fabsf(v4.y) > tf) << 1) |
                                 ((uint32_t)(fabsf(v4.z) > tf) << 2) | ((uint32_t)(fabsf(v4.w) > tf) << 3);
            m = (unsigned long long)nib << kb;  // masks are in flat K order (bit K of row (I, J))
        }
        for (int o = 1; o < lpr; o <<= 1) m |= bperm64(m, lane ^ o);
        if (q == 0 && row < nrows) {
            masks[row] = m;
            const uint32_t last1 = m ? (uint32_t)(64 - __clzll(m)) : 0u;
            rec[row] = (uint16_t)((uint32_t)__popcll(m) | (last1 << 7));
        }
    }
    __syncthreads();
    unsigned long long* mytab = P.table + U.tab_off + (uint64_t)gme * (nrows >> 2);
    for (int i = tid; i < (nrows >> 2); i += kThreads) {
        const unsigned long long g = kValid | (unsigned long long)rec[4 * i] |
                                     ((unsigned long long)rec[4 * i + 1] << 14) |
                                     ((unsigned long long)rec[4 * i + 2] << 28) |
                                     ((unsigned long long)rec[4 * i + 3] << 42);
        st_rlx(mytab + i, g);
    }
    __syncthreads();  // rec[] is read before the table overwrites it

    // ---- phase 4: read the unit's row table into LDS, in flat (I, J) order -
    // Granule i of tile g holds local rows 4*(i mod nrows/4) .. +3; local row
    // r = (((h*TY + jj) * 2 + sx) << lbx) + bxl is flat row
    // (I, J) = (bxl + sx*hx, g*TY + jj + h*hy).  Every valid (I, J) has exactly
    // one writer, so ft[0 .. W*H) ends up fully defined.
    uint16_t* ft = tab;
    const uint32_t ngr = G * (uint32_t)(nrows >> 2);
    const unsigned long long* utab = P.table + U.tab_off;
    const int lgq = lbx + lby;  // log2(nrows / 4)
    for (uint32_t i = tid; i < ngr; i += kThreads) {
        unsigned long long v = 0;
        for (uint32_t spin = 0;; ++spin) {
            v = ld_rlx(utab + i);
            if (v & kValid) break;
            if (spin > kSpinLimit) {
                atomicOr(P.err, kErrTimeout);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const uint32_t g = i >> lgq;
        const uint32_t r0 = (i & ((1u << lgq) - 1u)) << 2;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint32_t r = r0 + e;
            const uint32_t bxl = r & (TX - 1), sxv = (r >> lbx) & 1u;
            const uint32_t jj = (r >> (lbx + 1)) & (TY - 1), h = r >> (lbx + 1 + lby);
            const uint32_t jy = (g << lby) + jj;
            if (bxl < (uint32_t)hx && jy < (uint32_t)hy)
                ft[(bxl + sxv * hx) * (uint32_t)H + jy + h * hy] = (uint16_t)((v >> (14 * e)) & 0x3fffu);
        }
    }
    __syncthreads();

    // ---- phase 5: pair offsets of my rows ----------------------------------
    // Block scan over the W*H flat rows, 16 per thread (two 16-B LDS reads):
    // chunk prefix = pairs before the chunk, and last kept flat index + 1
    // before it.  Then each own row adds the (< 16) rows of its chunk before it.
    const uint32_t nflat = (uint32_t)W * (uint32_t)H;  // <= kMaxFusedRows
    uint32_t* cp_sum = own_prev + nrows;                // [256] chunk prefixes
    uint32_t* cp_last = cp_sum + kThreads;
    auto chunk_scan = [&](uint32_t c, uint32_t lim, uint32_t& sum, uint32_t& last) {
        // sum / last over flat rows [16c, min(16c + lim, nflat))
        const uint4* q = reinterpret_cast<const uint4*>(ft + 16 * c);
        const uint4 a = q[0], b = q[1];
        const uint32_t wd[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        sum = 0;
        last = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t fr = 16 * c + k;
            const uint32_t rc = (k & 1) ? (wd[k >> 1] >> 16) : (wd[k >> 1] & 0xffffu);
            if ((uint32_t)k < lim && fr < nflat) {
                sum += rc & 0x7fu;
                if (rc >> 7) last = fr * (uint32_t)D + (rc >> 7);
            }
        }
    };
    {
        uint32_t csum, clast, esum, emax, total;
        chunk_scan(tid, 16, csum, clast);
        block_scan2(csum, clast, tid, slab, esum, emax, total);
        cp_sum[tid] = esum;
        cp_last[tid] = emax;
        if (gme == 0 && tid == 0) {
            int32_t* hd = reinterpret_cast<int32_t*>(P.payload + U.pay_off);
            hd[0] = W;
            hd[1] = H;
            hd[2] = D;
            hd[3] = (int32_t)U.ncells;
            hd[4] = (int32_t)total;
            P.kept[td.unit] = total;
            P.offsets[td.unit] = U.pay_off;
            if ((int)td.unit == P.n - 1) P.offsets[P.n] = U.pay_off + 20 + 8ull * total;
        }
        __syncthreads();
        for (int r = tid; r < nrows; r += kThreads) {
            const uint32_t bxl = r & (TX - 1), sxv = (r >> lbx) & 1u;
            const uint32_t jj = (r >> (lbx + 1)) & (TY - 1), h = r >> (lbx + 1 + lby);
            const uint32_t bx = td.bx0 + bxl, byv = td.by0 + jj;
            uint32_t off = 0, prev = 0;
            if (bx < (uint32_t)hx && byv < (uint32_t)hy) {
                const uint32_t fr = (bx + sxv * hx) * (uint32_t)H + byv + h * hy;
                uint32_t ps, pl;
                chunk_scan(fr >> 4, fr & 15u, ps, pl);
                off = cp_sum[fr >> 4] + ps;
                prev = pl ? pl : cp_last[fr >> 4];
            }
            own_off[r] = off;
            own_prev[r] = prev;
        }
    }
    __syncthreads();

    // ---- phase 6: emit (run, value) pairs, 4 columns per lane ---------------
    uint8_t* __restrict__ pairs = P.payload + U.pay_off + 20;
    for (int rb = w * rpw; rb < nrows; rb += 4 * rpw) {
        const int row = rb + (lane >> llpr), q = lane & (lpr - 1);
        const int zc = (4 * q) & (TZ - 1), kb = zc + ((4 * q) >> lbz) * hz;
        const unsigned long long m = row < nrows ? masks[row] : 0ull;
        const uint32_t nib = zc < hz ? (uint32_t)(m >> kb) & 0xfu : 0u;
        if (nib) {
            const int bxl = row & (TX - 1);
            int r2 = row >> lbx;
            const int ssx = r2 & 1;
            r2 >>= 1;
            const int byl = r2 & (TY - 1), ssy = r2 >> lby;
            const uint32_t I = td.bx0 + bxl + ssx * hx, J = td.by0 + byl + ssy * hy;
            const uint32_t fbase = (I * (uint32_t)H + J) * (uint32_t)D;
            const unsigned long long below = m & ((1ull << kb) - 1ull);
            uint32_t rank = own_off[row] + (uint32_t)__popcll(below);
            // previous kept flat index + 1
            uint32_t prev1 = below ? fbase + (uint32_t)(64 - __clzll(below)) : own_prev[row];
            const float4 v4 = *reinterpret_cast<const float4*>(rows + row * rstride + 4 * q);
            const float vv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (nib & (1u << j)) {
                    const uint32_t f = fbase + kb + j;
                    uint2 pr;
                    pr.x = f - prev1;  // run = f - prev - 1
                    pr.y = __float_as_uint(vv[j]);
                    *reinterpret_cast<uint2*>(pairs + 8ull * rank) = pr;
                    ++rank;
                    prev1 = f + 1;
                }
            }
        }
    }

    __syncthreads();  // this tile's LDS is free
    if (tnext < P.ntiles) {
        t = tnext;
        continue;
    }
    if (tid0 == 0) misc[0] = atomicAdd(P.ticket, 1u);
    __syncthreads();
    t = __builtin_amdgcn_readfirstlane((uint32_t)misc[0]);
    if (t >= P.ntiles) return;
    {
        const XTile tt = tile_at(P, t);
        issue_col<T>(P, tt, unit_at(P, tt.unit), tid, raw);
    }
    }
}

size_t fused_lds_bytes(int lbx, int lby, int lbz, uint32_t ntile) {
    const size_t nrows = (size_t)4 << (lbx + lby);
    const size_t rowlen = (size_t)2 << lbz;
    // misc 128 | slab 512 | rows | masks, own_off, own_prev (16 B/row) | chunk prefixes 2 KB |
    // flat row table (kThreads * 16 records, read as 32-B chunks)
    (void)ntile;
    return 128 + 512 + nrows * (rowlen + 4) * sizeof(float) + nrows * 16 + 2 * kThreads * 4 +
           16 * kThreads * 2;
}

// Persistent grid: one workgroup per resident slot (never more than the tiles).
// Residency is not needed for correctness (tickets order the work), only for
// not launching workgroups that would find the ticket counter exhausted.
template <typename T>
static uint32_t fused_grid(size_t lds, uint32_t ntiles) {
    static thread_local size_t c_lds = 0;
    static thread_local uint32_t c_slots = 0;
    static thread_local int c_dev = -1;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (c_lds != lds || c_dev != dev) {
        int per_cu = 0, ncu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_forward_fused<T>, kThreads, lds) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per_cu < 1 ||
            ncu < 1)
            return ntiles;
        c_lds = lds;
        c_dev = dev;
        c_slots = (uint32_t)per_cu * (uint32_t)ncu;
    }
    return ntiles < c_slots ? ntiles : c_slots;
}

hipError_t launch_forward_fused(hipStream_t st, int dtype, size_t lds, const FusedParams& p) {
    if (p.ntiles == 0) return hipSuccess;
    if (dtype == 1)
        k_forward_fused<double><<<fused_grid<double>(lds, p.ntiles), kThreads, lds, st>>>(p);
    else
        k_forward_fused<float><<<fused_grid<float>(lds, p.ntiles), kThreads, lds, st>>>(p);
    return hipGetLastError();
}

}  // namespace wc

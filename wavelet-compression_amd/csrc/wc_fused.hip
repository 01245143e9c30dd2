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



template <typename T>
__global__ __launch_bounds__(kThreads, 3) void k_forward_fused(FusedParams P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    // misc[0] ticket, misc[1] thresh bits, misc[4..7] wave key maxima, misc[8..11] scan scratch
    unsigned long long* misc = reinterpret_cast<unsigned long long*>(lds);
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
    const int rowlen = 2 * TZ, rstride = rowlen + 4;   // rowlen == D: the tile spans all of z
    const int nrows = 4 * TX * TY;
    const uint32_t G = U.ntile_u;
    const uint32_t gme = t - U.xt_begin;               // my tile index within the unit (along y)
    // LDS carve (16-B aligned pieces)
    uint32_t* slab = reinterpret_cast<uint32_t*>(lds + 32);  // [0,64) slab totals/bases, [64,128) slab last
    float* rows = lds + 32 + 128;
    unsigned long long* masks = reinterpret_cast<unsigned long long*>(rows + nrows * rstride);  // per row
    uint32_t* own_off = reinterpret_cast<uint32_t*>(masks + nrows);
    uint32_t* own_prev = own_off + nrows;
    uint16_t* tab = reinterpret_cast<uint16_t*>(own_prev + nrows + 2 * kThreads);  // 4096 records; rec[] aliases

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
    if (tid == 0) {
        unsigned long long k = misc[4];
        for (int i = 1; i < 4; ++i) k = misc[4 + i] > k ? misc[4 + i] : k;
        st_rlx(P.keyslot + t, k | kValid);
    }
    if (w == 0 && (P.diag & 1u)) {
        if (lane == 0) misc[1] = (unsigned long long)__double_as_longlong(key_thresh(misc[4], P.keep));
    } else if (w == 0) {
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
        best = wave_max_u64(best);
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
    for (int rb = w * rpw; rb < ((P.diag & 16u) ? 0 : nrows); rb += 4 * rpw) {
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
        for (int o = 1; o < lpr; o <<= 1) m |= __shfl_xor(m, o);
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
    const uint32_t ngr = (P.diag & 2u) ? 0u : G * (uint32_t)(nrows >> 2);
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
    if (!(P.diag & 4u)) {
        uint32_t csum, clast;
        chunk_scan(tid, 16, csum, clast);
        const ScanOut so = block_scan_sum_max<uint32_t>(csum, clast, slab, slab + 64);
        cp_sum[tid] = (uint32_t)so.excl_sum;
        cp_last[tid] = so.excl_max;
        if (gme == 0 && tid == 0) {
            const uint32_t total = (uint32_t)so.total_sum;
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
    for (int rb = w * rpw; rb < ((P.diag & 8u) ? 0 : nrows); rb += 4 * rpw) {
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

hipError_t launch_forward_fused(hipStream_t st, int dtype, size_t lds, const FusedParams& p) {
    if (p.ntiles == 0) return hipSuccess;
    if (dtype == 1)
        k_forward_fused<double><<<p.ntiles, kThreads, lds, st>>>(p);
    else
        k_forward_fused<float><<<p.ntiles, kThreads, lds, st>>>(p);
    return hipGetLastError();
}

}  // namespace wc

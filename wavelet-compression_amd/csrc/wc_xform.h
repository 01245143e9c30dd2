// wc_xform.h — the transform-tile bodies (K1) of wc_transform.hip and the
// helpers the emit and inverse kernels share with them.
//
// One-level 3-D Haar, src/compressor.cpp:85-185: a coefficient (I, J, K)
// depends only on the 2x2x2 input block (I mod hx, J mod hy, K mod hz), so a
// tile of blocks is transformed in registers (Z, then Y, then X pairs — the
// reference's sweep order) and its outputs land in LDS rows keyed by flat row
// (I, J) (flat order is x-slowest / z-fastest, :178-181).  Phase 2 streams
// the rows out along K through a caller-supplied store functor.
//
// Max key (src/compressor.cpp:212-215, std::max_element by |c|):
//   bits 62..32 |c| bits, 31..1 (0x7fffffff - flat index), bit 0 sign.
// Larger key = larger magnitude, then SMALLER flat index (first wins); the
// sign rides along so thresh needs no second lookup.  A NaN at flat index 0
// (max_element then returns flat[0]: every comparison with NaN is false)
// is the sentinel ~0 -> thresh NaN -> nothing kept; later NaNs never win.
#pragma once

#include "wc_device.h"

namespace wc {

__device__ __forceinline__ unsigned long long coef_key(float c, uint32_t f) {
    const uint32_t bits = __float_as_uint(c);
    const uint32_t ab = bits & 0x7fffffffu;
    if (ab > 0x7f800000u) return f == 0 ? kKeyNaNFirst : 0ull;
    return ((unsigned long long)ab << 32) | ((unsigned long long)(0x7fffffffu - f) << 1) | (bits >> 31);
}

// thresh = (signed max) * (1 - keep), src/compressor.cpp:216.  key 0 (no
// coefficients or all NaN) gives max 0 -> thresh 0, as max_element on an
// all-NaN range returns flat[0] only when it is the sentinel case.
__device__ __forceinline__ double key_thresh(unsigned long long key, double keep) {
    if (key == kKeyNaNFirst) return __longlong_as_double(0x7ff8000000000000ll);
    const uint32_t ab = (uint32_t)(key >> 32) & 0x7fffffffu;
    const float maxv = __uint_as_float(ab | ((uint32_t)(key & 1ull) << 31));
    return (double)maxv * (1.0 - keep);
}

__device__ __forceinline__ void row_of(int row, int lbx, int lby, int& bxl, int& ssx, int& byl, int& ssy) {
    bxl = row & ((1 << lbx) - 1);
    int r2 = row >> lbx;
    ssx = r2 & 1;
    r2 >>= 1;
    byl = r2 & ((1 << lby) - 1);
    ssy = r2 >> lby;
}

// ---------------------------------------------------------------------------
// Generic tile: any dims (odd tails pass through on that axis).  LDS row
// stride 2*TZ + 1 floats.
template <typename T>
__device__ __forceinline__ void xform_generic_p1(const T* __restrict__ src, const UnitDev& U,
                                                               const XTile& td, float* lds, int tid) {
    const int H = U.ny, W = U.nx;
    const int hx = U.hx, hy = U.hy, hz = U.hz;
    const int lbx = U.lbx, lby = U.lby, lbz = U.lbz;
    const int TX = 1 << lbx, TY = 1 << lby, TZ = 1 << lbz;
    const int rstride = 2 * TZ + 1;
    const int nblk = TX * TY * TZ;
    const int64_t sy = W, sz = (int64_t)W * H;
    const bool vec = ((U.cell_off & 1) == 0) && ((W & 1) == 0);
    for (int b = tid; b < nblk; b += kThreads) {
        const int bxl = b & (TX - 1);
        const int byl = (b >> lbx) & (TY - 1);
        const int bzl = b >> (lbx + lby);
        const int bx = td.bx0 + bxl, by = td.by0 + byl, bz = td.bz0 + bzl;
        if (bx >= U.nbx || by >= U.nby || bz >= U.nbz) continue;
        const bool px = bx < hx, py = by < hy, pz = bz < hz;
        float v[2][2][2];  // [dz][dy][dx]
#pragma unroll
        for (int dz = 0; dz < 2; ++dz)
#pragma unroll
            for (int dy = 0; dy < 2; ++dy) {
                if ((dz == 0 || pz) && (dy == 0 || py)) {
                    const T* p = src + 2 * (int64_t)bx + sy * (2 * by + dy) + sz * (2 * bz + dz);
                    load_xpair<T, true>(p, px, vec, v[dz][dy][0], v[dz][dy][1]);
                } else {
                    v[dz][dy][0] = 0.0f;
                    v[dz][dy][1] = 0.0f;
                }
            }
        float a[2][2][2];  // Z sweep (src/compressor.cpp:98-125): a[sz][dy][dx]
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx) {
                a[0][dy][dx] = pz ? haar_lo(v[0][dy][dx], v[1][dy][dx]) : v[0][dy][dx];
                a[1][dy][dx] = pz ? haar_hi(v[0][dy][dx], v[1][dy][dx]) : 0.0f;
            }
        float c2[2][2][2];  // Y sweep (:128-150): c2[sz][sy][dx]
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx) {
                c2[s][0][dx] = py ? haar_lo(a[s][0][dx], a[s][1][dx]) : a[s][0][dx];
                c2[s][1][dx] = py ? haar_hi(a[s][0][dx], a[s][1][dx]) : 0.0f;
            }
        float c[2][2][2];  // X sweep (:153-175): c[sz][sy][sx]
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                c[s][t][0] = px ? haar_lo(c2[s][t][0], c2[s][t][1]) : c2[s][t][0];
                c[s][t][1] = px ? haar_hi(c2[s][t][0], c2[s][t][1]) : 0.0f;
            }
#pragma unroll
        for (int ssz = 0; ssz < 2; ++ssz)
#pragma unroll
            for (int ssy = 0; ssy < 2; ++ssy)
#pragma unroll
                for (int ssx = 0; ssx < 2; ++ssx) {
                    if ((ssx && !px) || (ssy && !py) || (ssz && !pz)) continue;
                    const float cv = c[ssz][ssy][ssx];
                    const int row = ((((ssy << lby) + byl) * 2 + ssx) << lbx) + bxl;
                    lds[row * rstride + (ssz << lbz) + bzl] = cv;
                }
    }
}

// Phase 2 of a generic tile: st(flat index within the unit, value).  With
// KEYS, also returns this thread's max key over the values it stores (keys
// are computed here rather than in phase 1, where every coefficient of the
// thread's blocks is live in registers).
template <bool KEYS, class Store1>
__device__ __forceinline__ unsigned long long xform_generic_p2(const UnitDev& U, const XTile& td, const float* lds,
                                                               int tid, Store1 st) {
    unsigned long long kmax = 0;
    const int W = U.nx, H = U.ny, D = U.nz;
    const int hx = U.hx, hy = U.hy, hz = U.hz;
    const int lbx = U.lbx, lby = U.lby, lbz = U.lbz;
    const int TX = 1 << lbx, TY = 1 << lby, TZ = 1 << lbz;
    const int rowlen = 2 * TZ, rstride = rowlen + 1;
    const int nrows = 4 * TX * TY;
    const int total = nrows * rowlen;
    const int lrow = lbz + 1;
    for (int e = tid; e < total; e += kThreads) {
        const int row = e >> lrow;
        const int col = e & (rowlen - 1);
        const int ssz = col >> lbz, bzl = col & (TZ - 1);
        int bxl, ssx, byl, ssy;
        row_of(row, lbx, lby, bxl, ssx, byl, ssy);
        const int bx = td.bx0 + bxl, by = td.by0 + byl, bz = td.bz0 + bzl;
        if (bx >= U.nbx || by >= U.nby || bz >= U.nbz) continue;
        if ((ssx && bx >= hx) || (ssy && by >= hy) || (ssz && bz >= hz)) continue;
        const int I = out_index(bx, ssx, hx, W), J = out_index(by, ssy, hy, H), K = out_index(bz, ssz, hz, D);
        const int64_t f = ((int64_t)I * H + J) * D + K;
        const float v = lds[row * rstride + col];
        st(f, v);
        if constexpr (KEYS) {
            const unsigned long long k = coef_key(v, (uint32_t)f);
            kmax = k > kmax ? k : kmax;
        }
    }
    return kmax;
}

// ---------------------------------------------------------------------------
// Fast tile: even W, H, D with D % 8 == 0 (no tails).  A thread owns a column
// of 4 consecutive z-blocks (bx, by, bz..bz+3): 16 independent x-pair loads in
// flight, and each of its 8 output rows gets 4 consecutive K -> one 16-B LDS
// write.  LDS row stride 2*TZ + 4 floats (16-B rows; b128 writes of 8 lanes
// hit 32 banks).  Keys come from phase 2.
// MAG: also return the max of this thread's (|c| bits << 1 | sign) (NaN
// patterns are above +inf's): the largest magnitude for the sparse-staging
// bound, and in bit 0 whether some coefficient of that magnitude is negative.
// S32 (template): the tile shape is the compile-time 32 x 1 x 32 blocks, the
// unit's hx and hz are multiples of 32 and its cells 16-B / 8-B aligned
// (s32_ok): no bounds checks, no unaligned-load branches, index arithmetic
// folded (the shape of every C2 and C5 unit).
template <typename T, bool SPLIT = false, bool MAG = false, bool S32 = false>
__device__ __forceinline__ uint32_t xform_fast_p1(const T* __restrict__ src, const UnitDev& U,
                                                  const XTile& td, float* lds, int tid) {
    uint32_t mag = 0;
    const int W = U.nx, H = U.ny;
    const int hx = U.hx, hy = U.hy, hz = U.hz;
    const int lbx = S32 ? 5 : U.lbx, lby = S32 ? 0 : U.lby, lbz = S32 ? 5 : U.lbz;
    const int TX = 1 << lbx, TY = 1 << lby, TZ = 1 << lbz;
    const int rstride = 2 * TZ + 4;
    const int ncol = (TX * TY * TZ) >> 2;
    const int64_t sy = W, sz = (int64_t)W * H;
    const bool vec = S32 || (U.cell_off & 1) == 0;
    for (int ci = tid; ci < ncol; ci += kThreads) {
        const int bxl = ci & (TX - 1);
        const int byl = (ci >> lbx) & (TY - 1);
        const int bzq = ci >> (lbx + lby);  // quad of z-blocks within the tile
        const int bx = td.bx0 + bxl, by = td.by0 + byl, bzb = td.bz0 + 4 * bzq;
        if (!S32 && (bx >= hx || by >= hy || bzb >= hz)) continue;
        const T* p0 = src + 2 * (int64_t)bx + sy * (2 * by) + sz * (2 * (int64_t)bzb);
        float c[4][2][2][2];  // [q][sz][sy][sx]
        // Two halves of 4 z-planes (8 x-pair loads in flight each): bounds the
        // raw fp64 registers so 4 workgroups fit per CU.
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float v[4][2][2];  // [z plane 4h..4h+3][dy][dx]
#pragma unroll
            for (int zp = 0; zp < 4; ++zp)
#pragma unroll
                for (int dy = 0; dy < 2; ++dy)
                    load_xpair<T, true>(p0 + sz * (4 * h + zp) + sy * dy, true, vec, v[zp][dy][0], v[zp][dy][1]);
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                const int q = 2 * h + qq;
                float a[2][2][2];
#pragma unroll
                for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                    for (int dx = 0; dx < 2; ++dx) {
                        a[0][dy][dx] = haar_lo(v[2 * qq][dy][dx], v[2 * qq + 1][dy][dx]);
                        a[1][dy][dx] = haar_hi(v[2 * qq][dy][dx], v[2 * qq + 1][dy][dx]);
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
                    for (int t = 0; t < 2; ++t) {
                        c[q][s][t][0] = haar_lo(b[t][0], b[t][1]);
                        c[q][s][t][1] = haar_hi(b[t][0], b[t][1]);
                    }
                }
            }
            if (SPLIT && h == 0) __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int ssz = 0; ssz < 2; ++ssz)
#pragma unroll
            for (int ssy = 0; ssy < 2; ++ssy)
#pragma unroll
                for (int ssx = 0; ssx < 2; ++ssx) {
                    const int row = ((((ssy << lby) + byl) * 2 + ssx) << lbx) + bxl;
                    *reinterpret_cast<float4*>(lds + row * rstride + (ssz << lbz) + 4 * bzq) =
                        make_float4(c[0][ssz][ssy][ssx], c[1][ssz][ssy][ssx], c[2][ssz][ssy][ssx],
                                    c[3][ssz][ssy][ssx]);
                    if constexpr (MAG) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const uint32_t bits = __float_as_uint(c[q][ssz][ssy][ssx]);
                            mag = max(mag, (bits << 1) | (bits >> 31));
                        }
                    }
                }
    }
    return mag;
}

// Split form of the fast phase 1 for a persistent kernel that keeps the next
// tile's cells in flight while it transforms the current one: a fast tile
// has at most kThreads columns (kMaxTileBlocks / 4), so a thread owns at most
// one.  fast_load reads thread tid's column; fast_butterfly transforms it into
// the LDS rows exactly as xform_fast_p1 does.
struct FastCol {
    float v[8][2][2];  // [z plane][dy][dx]
};

template <typename T>
__device__ __forceinline__ bool fast_load(const T* __restrict__ src, const UnitDev& U, const XTile& td, int tid,
                                          FastCol& c) {
    const int lbx = U.lbx, lby = U.lby, lbz = U.lbz;
    const int TX = 1 << lbx, TY = 1 << lby, TZ = 1 << lbz;
    const int ci = tid;
    if (ci >= ((TX * TY * TZ) >> 2)) return false;
    const int bx = td.bx0 + (ci & (TX - 1)), by = td.by0 + ((ci >> lbx) & (TY - 1));
    const int bzb = td.bz0 + 4 * (ci >> (lbx + lby));
    if (bx >= U.hx || by >= U.hy || bzb >= U.hz) return false;
    const int64_t sy = U.nx, sz = (int64_t)U.nx * U.ny;
    const bool vec = (U.cell_off & 1) == 0;
    const T* p0 = src + 2 * (int64_t)bx + sy * (2 * by) + sz * (2 * (int64_t)bzb);
#pragma unroll
    for (int zp = 0; zp < 8; ++zp)
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) load_xpair<T, true>(p0 + sz * zp + sy * dy, true, vec, c.v[zp][dy][0], c.v[zp][dy][1]);
    return true;
}

__device__ __forceinline__ void fast_butterfly(const UnitDev& U, const FastCol& col, float* lds, int tid) {
    const int lbx = U.lbx, lby = U.lby, lbz = U.lbz;
    const int TX = 1 << lbx, TY = 1 << lby, TZ = 1 << lbz;
    const int rstride = 2 * TZ + 4;
    const int bxl = tid & (TX - 1), byl = (tid >> lbx) & (TY - 1), bzq = tid >> (lbx + lby);
    float c[4][2][2][2];  // [q][sz][sy][sx]
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        float a[2][2][2];
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx) {
                a[0][dy][dx] = haar_lo(col.v[2 * q][dy][dx], col.v[2 * q + 1][dy][dx]);
                a[1][dy][dx] = haar_hi(col.v[2 * q][dy][dx], col.v[2 * q + 1][dy][dx]);
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
            for (int t = 0; t < 2; ++t) {
                c[q][s][t][0] = haar_lo(b[t][0], b[t][1]);
                c[q][s][t][1] = haar_hi(b[t][0], b[t][1]);
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
                *reinterpret_cast<float4*>(lds + row * rstride + (ssz << lbz) + 4 * bzq) =
                    make_float4(c[0][ssz][ssy][ssx], c[1][ssz][ssy][ssx], c[2][ssz][ssy][ssx], c[3][ssz][ssy][ssx]);
            }
}

// Phase 2 of a fast tile: st(flat index within the unit (multiple of 4), float4);
// with KEYS, returns this thread's max key.
template <bool KEYS, class Store4>
__device__ __forceinline__ unsigned long long xform_fast_p2(const UnitDev& U, const XTile& td, const float* lds,
                                                            int tid, Store4 st) {
    unsigned long long kmax = 0;
    const int H = U.ny, D = U.nz;
    const int hx = U.hx, hy = U.hy, hz = U.hz;
    const int lbx = U.lbx, lby = U.lby, lbz = U.lbz;
    const int TX = 1 << lbx, TY = 1 << lby, TZ = 1 << lbz;
    const int rstride = 2 * TZ + 4;
    const int nrows = 4 * TX * TY;
    const int q4 = lbz - 1;  // log2(rowlen / 4)
    const int total4 = nrows << q4;
    for (int e = tid; e < total4; e += kThreads) {
        const int row = e >> q4;
        const int col = (e & ((1 << q4) - 1)) << 2;
        const int ssz = col >> lbz, bzl = col & (TZ - 1);
        int bxl, ssx, byl, ssy;
        row_of(row, lbx, lby, bxl, ssx, byl, ssy);
        const int bx = td.bx0 + bxl, by = td.by0 + byl, bz = td.bz0 + bzl;
        if (bx >= hx || by >= hy || bz >= hz) continue;
        const int I = bx + ssx * hx, J = by + ssy * hy, K = bz + ssz * hz;
        const int64_t f = ((int64_t)I * H + J) * D + K;
        const float4 v = *reinterpret_cast<const float4*>(lds + row * rstride + col);
        st(f, v);
        if constexpr (KEYS) {
            const uint32_t f0 = (uint32_t)f;
            unsigned long long k = coef_key(v.x, f0);
            kmax = k > kmax ? k : kmax;
            k = coef_key(v.y, f0 + 1);
            kmax = k > kmax ? k : kmax;
            k = coef_key(v.z, f0 + 2);
            kmax = k > kmax ? k : kmax;
            k = coef_key(v.w, f0 + 3);
            kmax = k > kmax ? k : kmax;
        }
    }
    return kmax;
}


// Sparse staging (U.sparse: TZ >= 16 blocks per z tile and hz % TZ == 0, so
// each TZ-coefficient flat segment belongs to one tile and to one aligned
// group of TZ/4 lanes).  A tile whose largest magnitude belongs to a negative
// coefficient stages densely (the unit's signed max may be that coefficient:
// thresh < 0 keeps everything); the others flag their unit (spos), so only a
// unit with a negative max AND a sparsely staged tile needs the re-staging
// fallback.  Flag byte of segment s of a unit: (coef_off >> 4) + s,
// inside the unit's 16-coefficient index range (UnitDev::flag_off; byte order: flag_pos).  With m = the tile's max |c| (from phase 1), bound = m * (1 - keep)
// (fp64, as src/compressor.cpp:216) is <= the unit's thresh whenever
// thresh >= 0 (|tile max| <= |unit max|), so a segment with no |c| > bound
// holds no kept coefficient.  A NaN in the tile, or a bound that is not >= 0,
// flags every segment.  Units whose thresh turns out < 0 (negative signed
// max: everything kept) are re-staged densely by k_transform_fallback.
__device__ __forceinline__ bool s32_ok(const UnitDev& U) {
    return U.lbx == 5 && U.lby == 0 && U.lbz == 5 && ((U.hx | U.hz) & 31) == 0 && (U.cell_off & 1) == 0 &&
           U.ncells < (1ull << 30);  // 32-bit byte offsets of the flat coefficients
}

__device__ __forceinline__ double sparse_bound(uint32_t magkey, double keep) {
    const uint32_t magbits = magkey >> 1;
    if (magbits > 0x7f800000u || (magkey & 1u)) return -1.0;  // NaN in the tile, or a negative max: dense
    const double b = (double)__uint_as_float(magbits) * (1.0 - keep);
    return b >= 0.0 ? b : -1.0;
}

// Branch-free max key: with amax = the tile's largest |c| bits
// and no NaN in the tile, only coefficients with |c| bits == amax can carry
// the tile's max key, and among those coef_key orders by the low word alone
// ((0x7fffffff - f) << 1 | sign: smallest flat index first).  So each
// coefficient costs a compare and a select into one 32-bit running max
// (`best`, 0 = none) instead of a branch around a 64-bit key; the key is
// (amax << 32) | best.  A tile holding a NaN (amax > +inf's bits) takes the
// per-coefficient coef_key pass instead (kKeyNaNFirst at flat index 0).
// Staged coefficients are written with nontemporal stores (their next reader
// is another kernel): K1 -2 % at C2, -4 % at C5 (profiles/r05/experiments/gpu_nt.txt).
__device__ __forceinline__ void stage_store4(float* __restrict__ p, const float4& v) {
    const f32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f32x4*>(p));
}
__device__ __forceinline__ uint32_t key_lo_max(uint32_t best, float c, uint32_t f, uint32_t amax) {
    const uint32_t bits = __float_as_uint(c);
    const uint32_t lo = ((0x7fffffffu - f) << 1) | (bits >> 31);
    return (bits & 0x7fffffffu) == amax ? max(best, lo) : best;
}

__device__ __forceinline__ unsigned long long key_from_lo(uint32_t amax, uint32_t best) {
    return best ? ((unsigned long long)amax << 32) | best : 0ull;
}

// Phase 2 with sparse staging: stores only segments with some |c| > bound,
// writes EVERY segment's flag byte (the emit skips the others' loads), and
// returns this thread's max key over all its coefficients.
template <class Store4>
__device__ __forceinline__ unsigned long long xform_fast_p2_sparse(const UnitDev& U, const XTile& td,
                                                                   const float* lds, int tid, double bound,
                                                                   uint32_t amax, uint8_t* __restrict__ flags,
                                                                   Store4 st) {
    const bool bf = amax <= 0x7f800000u;  // uniform: no NaN in the tile
    uint32_t best = 0;
    const int H = U.ny, D = U.nz;
    const int hx = U.hx, hy = U.hy, hz = U.hz;
    const int lbx = U.lbx, lby = U.lby, lbz = U.lbz;
    const int TX = 1 << lbx, TY = 1 << lby, TZ = 1 << lbz;
    const int rstride = 2 * TZ + 4;
    const int nrows = 4 * TX * TY;
    const int q4 = lbz - 1;
    const int total4 = nrows << q4;
    const int glanes = TZ >> 2;  // lanes per segment: 4 (TZ 16) or 8 (TZ 32)
    const int g0 = (tid & 63) & ~(glanes - 1);
    const unsigned long long gmask = (1ull << glanes) - 1ull;
    unsigned long long kmax = 0;
    for (int e = tid; e < total4; e += kThreads) {
        const int row = e >> q4;
        const int col = (e & ((1 << q4) - 1)) << 2;
        const int ssz = col >> lbz, bzl = col & (TZ - 1);
        int bxl, ssx, byl, ssy;
        row_of(row, lbx, lby, bxl, ssx, byl, ssy);
        const int bx = td.bx0 + bxl, by = td.by0 + byl, bz = td.bz0 + bzl;
        if (bx >= hx || by >= hy || bz >= hz) continue;  // uniform per 8-lane segment
        const int I = bx + ssx * hx, J = by + ssy * hy, K = bz + ssz * hz;
        const int64_t f = ((int64_t)I * H + J) * D + K;
        const float4 v = *reinterpret_cast<const float4*>(lds + row * rstride + col);
        const bool cand = (double)fabsf(v.x) > bound || (double)fabsf(v.y) > bound ||
                          (double)fabsf(v.z) > bound || (double)fabsf(v.w) > bound;
        // bound < 0 (dense tile): every segment, all-NaN ones included
        const bool flag = ((__ballot(cand) >> g0) & gmask) != 0 || !(bound >= 0.0);
        if (flag) st(f, v);
        if ((tid & (glanes - 1)) == 0) flags[U.flag_off + flag_pos((uint64_t)f >> lbz, lbz)] = flag ? 1 : 0;
        const uint32_t f0 = (uint32_t)f;
        if (bf) {
            best = key_lo_max(best, v.x, f0, amax);
            best = key_lo_max(best, v.y, f0 + 1, amax);
            best = key_lo_max(best, v.z, f0 + 2, amax);
            best = key_lo_max(best, v.w, f0 + 3, amax);
            continue;
        }
        unsigned long long k = coef_key(v.x, f0);
        kmax = k > kmax ? k : kmax;
        k = coef_key(v.y, f0 + 1);
        kmax = k > kmax ? k : kmax;
        k = coef_key(v.z, f0 + 2);
        kmax = k > kmax ? k : kmax;
        k = coef_key(v.w, f0 + 3);
        kmax = k > kmax ? k : kmax;
    }
    return bf ? key_from_lo(amax, best) : kmax;
}

// xform_fast_p2_sparse for the S32 shape (s32_ok), in fewer instructions:
//  * the candidate test |c| > bound in fp32 against bf = bound rounded toward
//    -inf (thresh_as_float: exact for every float |c|) instead of fp64;
//  * the max key only where it can win: amax = the tile's largest non-NaN |c|
//    bits (from phase 1's MAG, passed in; ~0u when the tile holds a NaN, then
//    every coefficient gets its key as in xform_fast_p2_sparse); a coefficient
//    whose |c| bits differ from amax cannot carry the tile's max key, and a NaN
//    at flat index 0 (the kKeyNaNFirst sentinel) is checked where it can sit;
//  * the loop unrolled over the constant shape (8 float4 per thread: row
//    (tid >> 4) + 16 it, 4 K from (tid & 15) * 4).
__device__ __forceinline__ unsigned long long xform_fast_p2_sparse_s32(const UnitDev& U, const XTile& td,
                                                                       const float* lds, int tid, double bound,
                                                                       uint32_t amax, uint8_t* __restrict__ flags,
                                                                       float* __restrict__ dst) {
    constexpr int lbz = 5, TZ = 32, rstride = 2 * TZ + 4;
    const int H = U.ny, D = U.nz, hx = U.hx, hy = U.hy, hz = U.hz;
    const int r0 = tid >> 4, col = (tid & 15) << 2;
    const int ssz = col >> lbz, bzl = col & (TZ - 1);
    const int K = td.bz0 + bzl + ssz * hz;
    const int g0 = (tid & 63) & ~7;  // 8 lanes per 32-coefficient segment
    const bool dense = !(bound >= 0.0);
    const float bf = thresh_as_float(bound);
    const bool allkeys = amax > 0x7f800000u;  // a NaN in the tile: every key as in the generic form
    unsigned long long kmax = 0;
    uint32_t best = 0;  // running low word of the branch-free max key
    // 32-bit unit-relative indices (s32_ok: < 2^30 cells): row r0 + 16 it has
    // flat index fb + (it & 1) 16 H D + ssx hx H D + ssy hy D, uniform steps;
    // stores through the uniform bases with 32-bit offsets.
    const uint32_t HD = (uint32_t)H * (uint32_t)D;
    const uint32_t fb = ((uint32_t)(td.bx0 + r0) * (uint32_t)H + td.by0) * (uint32_t)D + (uint32_t)K;
    const uint32_t dA = 16u * HD, dB = (uint32_t)hx * HD, dC = (uint32_t)hy * (uint32_t)D;
    uint8_t* __restrict__ fl = flags + U.flag_off;
    char* __restrict__ dstb = reinterpret_cast<char*>(dst);
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const int row = r0 + 16 * it;  // row_of with lbx 5, lby 0: bxl, ssx, ssy
        const float4 v = *reinterpret_cast<const float4*>(lds + row * rstride + col);
        // largest |c| of the four (NaNs ignored, as the per-element compares)
        const float m4 = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
        const bool cand = m4 > bf;
        const bool flag = ((__ballot(cand) >> g0) & 0xffull) != 0 || dense;
        const uint32_t f0 = fb + ((it & 1) ? dA : 0u) + (((it >> 1) & 1) ? dB : 0u) + ((it >> 2) ? dC : 0u);
        if (flag) stage_store4(reinterpret_cast<float*>(dstb + (f0 << 2)), v);
        if ((tid & 7) == 0) fl[flag_pos32(f0 >> lbz, lbz)] = flag ? 1 : 0;
        const float e[4] = {v.x, v.y, v.z, v.w};
        // only a wave with a lane holding the tile's largest |c| can raise the
        // key (no NaN here: allkeys tiles redo every key below)
        if (__ballot(__float_as_uint(m4) == amax)) {
#pragma unroll
            for (int j = 0; j < 4; ++j) best = key_lo_max(best, e[j], f0 + (uint32_t)j, amax);
        }
    }
    if (!allkeys) return key_from_lo(amax, best);
    // a NaN in the tile (rare): every coefficient's key, as the generic form
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

}  // namespace wc

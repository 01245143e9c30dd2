// wc_kernels.hip — gfx950 kernels of the wavelet codec hot path.
//
//   K1 k_transform      cells (fp64|fp32, x-fastest) -> flat fp32 coefficients
//                       (x-slowest) + per-unit max-|c| key      src/compressor.cpp:85-185, :212-215
//   K2a k_flat_count    per flat tile: kept count + last kept   src/compressor.cpp:216-234
//   K2b k_unit_scan     per unit: exclusive scan over its tiles
//   K2c k_unit_offsets  payload offsets + 20-byte headers      src/compressor.cpp:55-71
//   K2d k_flat_emit     ordered compaction -> (run, value) pairs src/compressor.cpp:24-42, :73-77
//   K5a/b/c             rle_decode as scan + scatter            src/decompressor.cpp:14-30
//   K6 k_inverse        flat coefficients -> fp32 Box3D         src/decompressor.cpp:79-159
//   K7 k_rmse_*         per-unit RMSE                           src/calc-loss.cpp:12-43
//
// Numerics (bit-exact with the reference):
//   * forward pair  (a + b) / 2.0 in the reference = float add, exact halving,
//     one rounding to float  ==  (a + b) * 0.5f here (no FTZ: built with
//     -fno-gpu-flush-denormals-to-zero, -ffp-contract=off).
//   * inverse pair  avg +/- diff in double then stored to float  ==  a float
//     add (53 >= 2*24 + 2, so the double rounding is innocuous).
//   * keep test     |c| > thresh in double, thresh = signed max * (1 - keep).
#include "wc_internal.h"

namespace wc {

__device__ __forceinline__ float haar_lo(float a, float b) { return (a + b) * 0.5f; }
__device__ __forceinline__ float haar_hi(float a, float b) { return (a - b) * 0.5f; }

__device__ __forceinline__ int lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0));
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}

// Load the x-pair (x, x+1) of a row as fp32 (fp64 cells narrowed RNE,
// src/preprocess.cpp:78).  `vec`: both elements in one aligned vector load.
template <typename T>
__device__ __forceinline__ void load_xpair(const T* __restrict__ p, bool two, bool vec,
                                           float& a, float& b) {
    if (two) {
        if (vec) {
            if constexpr (sizeof(T) == 8) {
                const double2 d = *reinterpret_cast<const double2*>(p);
                a = (float)d.x;
                b = (float)d.y;
            } else {
                const float2 d = *reinterpret_cast<const float2*>(p);
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

// ---------------------------------------------------------------------------
// K1: one-level 3-D Haar over a tile of 2x2x2 blocks.
// Phase 1: each thread transforms whole blocks in registers (z, then y, then x
//          pairs — the reference's sweep order) and stores the 8 outputs in LDS
//          rows keyed by flat row (I, J).
// Phase 2: rows are streamed to global memory along K (flat order is
//          z-fastest), so the x-fastest -> z-fastest transpose costs one LDS trip.
// KEYS: also reduce the unit's max-|c| key (|c| bits << 32 | ~flat_index) so the
//       FIRST largest magnitude wins, exactly like std::max_element.
template <typename T, bool KEYS>
__global__ __launch_bounds__(kThreads) void k_transform(
    const T* __restrict__ cells, const UnitDev* __restrict__ units, const XTile* __restrict__ tiles,
    float* __restrict__ out, int out_at_cell_off, unsigned long long* __restrict__ unit_key) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const XTile td = tiles[blockIdx.x];
    const UnitDev& U = units[td.unit];
    const int W = U.nx, H = U.ny, D = U.nz;
    const int hx = U.hx, hy = U.hy, hz = U.hz;
    const int lbx = U.lbx, lby = U.lby, lbz = U.lbz;
    const int TX = 1 << lbx, TY = 1 << lby, TZ = 1 << lbz;
    const int rowlen = 2 * TZ, rstride = rowlen + 1;
    const int nblk = TX * TY * TZ;
    const int64_t sy = W, sz = (int64_t)W * H;
    const T* __restrict__ src = cells + U.cell_off;
    const bool vec = ((U.cell_off & 1) == 0) && ((W & 1) == 0);

    unsigned long long kmax = 0;

    for (int b = threadIdx.x; b < nblk; b += kThreads) {
        const int bxl = b & (TX - 1);
        const int byl = (b >> lbx) & (TY - 1);
        const int bzl = b >> (lbx + lby);
        const int bx = td.bx0 + bxl, by = td.by0 + byl, bz = td.bz0 + bzl;
        if (bx >= U.nbx || by >= U.nby || bz >= U.nbz) continue;
        const bool px = bx < hx, py = by < hy, pz = bz < hz;

        // v[dz][dy][dx]
        float v[2][2][2];
#pragma unroll
        for (int dz = 0; dz < 2; ++dz)
#pragma unroll
            for (int dy = 0; dy < 2; ++dy) {
                if ((dz == 0 || pz) && (dy == 0 || py)) {
                    const T* p = src + 2 * (int64_t)bx + sy * (2 * by + dy) + sz * (2 * bz + dz);
                    load_xpair<T>(p, px, vec, v[dz][dy][0], v[dz][dy][1]);
                } else {
                    v[dz][dy][0] = 0.0f;
                    v[dz][dy][1] = 0.0f;
                }
            }
        // Z sweep first (src/compressor.cpp:98-125): a[sz][dy][dx]
        float a[2][2][2];
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx) {
                if (pz) {
                    a[0][dy][dx] = haar_lo(v[0][dy][dx], v[1][dy][dx]);
                    a[1][dy][dx] = haar_hi(v[0][dy][dx], v[1][dy][dx]);
                } else {
                    a[0][dy][dx] = v[0][dy][dx];
                    a[1][dy][dx] = 0.0f;
                }
            }
        // Y sweep (:128-150): c2[sz][sy][dx]
        float c2[2][2][2];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx) {
                if (py) {
                    c2[s][0][dx] = haar_lo(a[s][0][dx], a[s][1][dx]);
                    c2[s][1][dx] = haar_hi(a[s][0][dx], a[s][1][dx]);
                } else {
                    c2[s][0][dx] = a[s][0][dx];
                    c2[s][1][dx] = 0.0f;
                }
            }
        // X sweep (:153-175): c[sz][sy][sx]
        float c[2][2][2];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                if (px) {
                    c[s][t][0] = haar_lo(c2[s][t][0], c2[s][t][1]);
                    c[s][t][1] = haar_hi(c2[s][t][0], c2[s][t][1]);
                } else {
                    c[s][t][0] = c2[s][t][0];
                    c[s][t][1] = 0.0f;
                }
            }

        const int I0 = out_index(bx, 0, hx, W), I1 = bx + hx;
        const int J0 = out_index(by, 0, hy, H), J1 = by + hy;
        const int K0 = out_index(bz, 0, hz, D), K1 = bz + hz;
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
                    if constexpr (KEYS) {
                        const int I = ssx ? I1 : I0, J = ssy ? J1 : J0, K = ssz ? K1 : K0;
                        const uint32_t f = (uint32_t)(((int64_t)I * H + J) * D + K);
                        const uint32_t ab = __float_as_uint(cv) & 0x7fffffffu;
                        unsigned long long key;
                        if (ab > 0x7f800000u) {
                            key = (f == 0) ? kKeyNaNFirst : 0ull;
                        } else {
                            key = ((unsigned long long)ab << 32) | (unsigned long long)(0xffffffffu - f);
                        }
                        kmax = key > kmax ? key : kmax;
                    }
                }
    }
    __syncthreads();

    // Phase 2: LDS rows -> flat coefficients, consecutive lanes on consecutive K.
    float* __restrict__ dst = out + (out_at_cell_off ? U.cell_off : U.coef_off);
    const int nrows = 4 * TX * TY;
    const int total = nrows * rowlen;
    const int lrow = lbz + 1;
    for (int e = threadIdx.x; e < total; e += kThreads) {
        const int row = e >> lrow;
        const int col = e & (rowlen - 1);
        const int ssz = col >> lbz, bzl = col & (TZ - 1);
        const int bxl = row & (TX - 1);
        int r2 = row >> lbx;
        const int ssx = r2 & 1;
        r2 >>= 1;
        const int byl = r2 & (TY - 1), ssy = r2 >> lby;
        const int bx = td.bx0 + bxl, by = td.by0 + byl, bz = td.bz0 + bzl;
        if (bx >= U.nbx || by >= U.nby || bz >= U.nbz) continue;
        if ((ssx && bx >= hx) || (ssy && by >= hy) || (ssz && bz >= hz)) continue;
        const int I = out_index(bx, ssx, hx, W), J = out_index(by, ssy, hy, H),
                  K = out_index(bz, ssz, hz, D);
        dst[((int64_t)I * H + J) * D + K] = lds[row * rstride + col];
    }

    if constexpr (KEYS) {
        kmax = wave_max_u64(kmax);
        if (lane_id() == 0 && kmax != 0) atomicMax(unit_key + td.unit, kmax);
    }
}

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
    const double thresh = unit_thresh(U, unit_key[ft.unit], coef, keep);
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
            const bool k = idx < len && (double)fabsf(e[j]) > thresh;
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
// K2b: per unit, exclusive scan of its tiles' kept counts / last kept.
__global__ __launch_bounds__(kThreads) void k_unit_scan(
    const UnitDev* __restrict__ units, const uint32_t* __restrict__ tcount,
    const uint32_t* __restrict__ tlast, uint32_t* __restrict__ toff, uint32_t* __restrict__ tprev,
    uint32_t* __restrict__ kept) {
    __shared__ uint32_t s_sum[4], s_max[4];
    const UnitDev& U = units[blockIdx.x];
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
// K2c: payload offsets (unit u starts at offsets[u] == 4 mod 8, so pairs are
// 8-byte aligned) and the 20-byte header (src/compressor.cpp:59-71).
__global__ __launch_bounds__(1024) void k_unit_offsets(const UnitDev* __restrict__ units, int n,
                                                     const uint32_t* __restrict__ kept,
                                                     uint8_t* __restrict__ payload,
                                                     uint64_t* __restrict__ offsets) {
    __shared__ uint64_t s_w[16];
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t carry = 4;
    for (int c0 = 0; c0 < n; c0 += 1024) {
        const int u = c0 + threadIdx.x;
        const bool ok = u < n;
        const uint64_t k = ok ? kept[u] : 0;
        const uint64_t sz = ok ? 20 + 8 * k + 4 : 0;
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
            offsets[u] = off;
            const UnitDev& U = units[u];
            int32_t* h = reinterpret_cast<int32_t*>(payload + off);
            h[0] = U.nx;
            h[1] = U.ny;
            h[2] = U.nz;
            h[3] = (int32_t)U.ncells;
            h[4] = (int32_t)k;
            if (u == n - 1) offsets[n] = off + 20 + 8 * k;
        }
        carry += tot;
    }
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
    const double thresh = unit_thresh(U, unit_key[ft.unit], coef, keep);
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
            const bool k = idx < len && (double)fabsf(e[j]) > thresh;
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
    uint8_t* __restrict__ pairs = payload + offsets[ft.unit] + 20;

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
// K5a: validate headers and sum (run + 1) per pair tile (pair tiles reuse the
// flat-tile plan: nrle <= ncoeff for every valid payload).
__device__ __forceinline__ bool read_header(const UnitDev& U, const uint8_t* __restrict__ ph,
                                            int32_t& nrle) {
    const int32_t* h = reinterpret_cast<const int32_t*>(ph);
    nrle = h[4];
    return h[0] == U.nx && h[1] == U.ny && h[2] == U.nz && h[3] == (int32_t)U.ncells &&
           nrle >= 0 && (uint64_t)nrle <= U.ncells;
}

__global__ __launch_bounds__(kThreads) void k_decode_count(
    const UnitDev* __restrict__ units, const FTile* __restrict__ tiles,
    const uint8_t* __restrict__ payload, const uint64_t* __restrict__ offsets,
    uint64_t* __restrict__ tsum, uint32_t* __restrict__ err) {
    __shared__ uint64_t s_w[4];
    const FTile ft = tiles[blockIdx.x];
    const UnitDev& U = units[ft.unit];
    const uint8_t* ph = payload + offsets[ft.unit];
    int32_t nrle;
    const bool hok = read_header(U, ph, nrle);
    if (!hok && ft.index == 0 && threadIdx.x == 0) atomicOr(err, kErrHeader);
    const int64_t start = (int64_t)ft.index * kFlatTile;
    const int64_t n = hok ? nrle : 0;
    const int32_t* pr = reinterpret_cast<const int32_t*>(ph + 20);
    uint64_t s = 0;
    bool neg = false;
    for (int i = threadIdx.x; i < kFlatTile; i += kThreads) {
        const int64_t k = start + i;
        if (k < n) {
            const int32_t run = pr[2 * k];
            neg |= run < 0;
            s += (uint64_t)(int64_t)run + 1;
        }
    }
    if (neg) atomicOr(err, kErrNegativeRun);
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) tsum[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// K5b: per unit exclusive scan of the tile sums (64-bit).
__global__ __launch_bounds__(kThreads) void k_decode_scan(const UnitDev* __restrict__ units,
                                                        const uint64_t* __restrict__ tsum,
                                                        uint64_t* __restrict__ tbase) {
    __shared__ uint64_t s_sum[4];
    __shared__ uint32_t s_max[4];
    const UnitDev& U = units[blockIdx.x];
    uint64_t base = 0;
    for (uint32_t c0 = 0; c0 < U.nftiles; c0 += kThreads) {
        const uint32_t i = c0 + threadIdx.x;
        const bool ok = i < U.nftiles;
        const uint32_t t = U.ftile_begin + i;
        const uint64_t v = ok ? tsum[t] : 0;
        ScanOut s = block_scan_sum_max<uint64_t>(v, 0u, s_sum, s_max);
        if (ok) tbase[t] = base + s.excl_sum;
        base += s.total_sum;
    }
}

// K5c: scatter.  Thread-contiguous runs of 16 pairs; position of pair k is
// (sum of run+1 over pairs <= k) - 1, written only while < ncoeff — which is
// exactly rle_decode's `idx += run; if (idx < total) out[idx++] = val`.
__global__ __launch_bounds__(kThreads) void k_decode_scatter(
    const UnitDev* __restrict__ units, const FTile* __restrict__ tiles,
    const uint8_t* __restrict__ payload, const uint64_t* __restrict__ offsets,
    const uint64_t* __restrict__ tbase, float* __restrict__ flat) {
    __shared__ uint64_t s_sum[4];
    __shared__ uint32_t s_max[4];
    const FTile ft = tiles[blockIdx.x];
    const UnitDev& U = units[ft.unit];
    const uint8_t* ph = payload + offsets[ft.unit];
    int32_t nrle;
    const bool hok = read_header(U, ph, nrle);
    const int64_t start = (int64_t)ft.index * kFlatTile;
    const int64_t n = hok ? nrle : 0;
    const uint2* __restrict__ pr = reinterpret_cast<const uint2*>(ph + 20);
    constexpr int P = kFlatTile / kThreads;  // 16
    const int64_t k0 = start + (int64_t)threadIdx.x * P;
    uint2 q[P];
    uint64_t local = 0;
#pragma unroll
    for (int i = 0; i < P; ++i) {
        if (k0 + i < n) {
            q[i] = pr[k0 + i];
            local += (uint64_t)(int64_t)(int32_t)q[i].x + 1;
        } else {
            q[i] = make_uint2(0u, 0u);
        }
    }
    ScanOut s = block_scan_sum_max<uint64_t>(local, 0u, s_sum, s_max);
    uint64_t pos = tbase[blockIdx.x] + s.excl_sum;  // count of slots consumed before my first pair
    float* __restrict__ dst = flat + U.coef_off;
#pragma unroll
    for (int i = 0; i < P; ++i) {
        if (k0 + i < n) {
            const int32_t run = (int32_t)q[i].x;
            if (run < 0) break;  // flagged in K5a; stop scattering this thread's pairs
            pos += (uint64_t)run;  // idx += run
            if (pos < U.ncells) dst[pos] = __uint_as_float(q[i].y);
            pos += 1;
        }
    }
}

// ---------------------------------------------------------------------------
// K6: inverse transform over the same 2x2x2-block tiles as K1.
// Phase 1: flat rows (contiguous along K) -> LDS.  Phase 2: per block X, then Y,
// then Z synthesis (src/decompressor.cpp:89-156); blocks with an odd tail on any
// axis reconstruct to 0 (the reference's zero-initialised `restored`).
__global__ __launch_bounds__(kThreads) void k_inverse(const float* __restrict__ flat,
                                                    int flat_at_cell_off,
                                                    const UnitDev* __restrict__ units,
                                                    const XTile* __restrict__ tiles,
                                                    float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const XTile td = tiles[blockIdx.x];
    const UnitDev& U = units[td.unit];
    const int W = U.nx, H = U.ny, D = U.nz;
    const int hx = U.hx, hy = U.hy, hz = U.hz;
    const int lbx = U.lbx, lby = U.lby, lbz = U.lbz;
    const int TX = 1 << lbx, TY = 1 << lby, TZ = 1 << lbz;
    const int rowlen = 2 * TZ, rstride = rowlen + 1;
    const int64_t sy = W, sz = (int64_t)W * H;
    const float* __restrict__ srcf = flat + (flat_at_cell_off ? U.cell_off : U.coef_off);

    const int nrows = 4 * TX * TY;
    const int total = nrows * rowlen;
    const int lrow = lbz + 1;
    for (int e = threadIdx.x; e < total; e += kThreads) {
        const int row = e >> lrow;
        const int col = e & (rowlen - 1);
        const int ssz = col >> lbz, bzl = col & (TZ - 1);
        const int bxl = row & (TX - 1);
        int r2 = row >> lbx;
        const int ssx = r2 & 1;
        r2 >>= 1;
        const int byl = r2 & (TY - 1), ssy = r2 >> lby;
        const int bx = td.bx0 + bxl, by = td.by0 + byl, bz = td.bz0 + bzl;
        if (bx >= hx || by >= hy || bz >= hz) continue;  // tail blocks are not needed
        const int I = bx + ssx * hx, J = by + ssy * hy, K = bz + ssz * hz;
        lds[row * rstride + col] = srcf[((int64_t)I * H + J) * D + K];
    }
    __syncthreads();

    float* __restrict__ dst = out + U.cell_off;
    const bool vec = ((U.cell_off & 1) == 0) && ((W & 1) == 0);
    const int nblk = TX * TY * TZ;
    for (int b = threadIdx.x; b < nblk; b += kThreads) {
        const int bxl = b & (TX - 1);
        const int byl = (b >> lbx) & (TY - 1);
        const int bzl = b >> (lbx + lby);
        const int bx = td.bx0 + bxl, by = td.by0 + byl, bz = td.bz0 + bzl;
        if (bx >= U.nbx || by >= U.nby || bz >= U.nbz) continue;
        const bool px = bx < hx, py = by < hy, pz = bz < hz;
        float V[2][2][2];  // V[dz][dy][dx]
        if (px && py && pz) {
            float c[2][2][2];  // c[sz][sy][sx]
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int x = 0; x < 2; ++x) {
                        const int row = ((((t << lby) + byl) * 2 + x) << lbx) + bxl;
                        c[s][t][x] = lds[row * rstride + (s << lbz) + bzl];
                    }
            // X first: X[sz][sy][dx]
            float X[2][2][2];
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    X[s][t][0] = c[s][t][0] + c[s][t][1];
                    X[s][t][1] = c[s][t][0] - c[s][t][1];
                }
            // then Y: Y[sz][dy][dx]
            float Y[2][2][2];
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int x = 0; x < 2; ++x) {
                    Y[s][0][x] = X[s][0][x] + X[s][1][x];
                    Y[s][1][x] = X[s][0][x] - X[s][1][x];
                }
            // then Z
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int x = 0; x < 2; ++x) {
                    V[0][t][x] = Y[0][t][x] + Y[1][t][x];
                    V[1][t][x] = Y[0][t][x] - Y[1][t][x];
                }
        } else {
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int t = 0; t < 2; ++t) V[s][t][0] = V[s][t][1] = 0.0f;
        }
#pragma unroll
        for (int dz = 0; dz < 2; ++dz)
#pragma unroll
            for (int dy = 0; dy < 2; ++dy) {
                if ((dz && !pz) || (dy && !py)) continue;
                float* p = dst + 2 * (int64_t)bx + sy * (2 * by + dy) + sz * (2 * bz + dz);
                if (px) {
                    if (vec) {
                        *reinterpret_cast<float2*>(p) = make_float2(V[dz][dy][0], V[dz][dy][1]);
                    } else {
                        p[0] = V[dz][dy][0];
                        p[1] = V[dz][dy][1];
                    }
                } else {
                    p[0] = 0.0f;
                }
            }
    }
}

// ---------------------------------------------------------------------------
// K7: RMSE.  Partial sums per flat tile (cell order), then a fixed-order
// per-unit reduction so the result is reproducible run to run.
template <typename T>
__global__ __launch_bounds__(kThreads) void k_rmse_partial(const T* __restrict__ orig,
                                                         const float* __restrict__ regen,
                                                         const UnitDev* __restrict__ units,
                                                         const FTile* __restrict__ tiles,
                                                         double* __restrict__ part) {
    __shared__ double s_w[4];
    const FTile ft = tiles[blockIdx.x];
    const UnitDev& U = units[ft.unit];
    const int64_t start = (int64_t)ft.index * kFlatTile;
    const int64_t len = min((int64_t)kFlatTile, (int64_t)U.ncells - start);
    const T* a = orig + U.cell_off + start;
    const float* b = regen + U.cell_off + start;
    double s = 0.0;
    for (int i = threadIdx.x; i < len; i += kThreads) {
        const float d = (float)a[i] - b[i];  // float - float, then widened
        const double dd = d;
        s += dd * dd;
    }
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = ((s_w[0] + s_w[1]) + s_w[2]) + s_w[3];
}

__global__ __launch_bounds__(64) void k_rmse_final(const UnitDev* __restrict__ units, int n,
                                                 const double* __restrict__ part,
                                                 double* __restrict__ rmse) {
    const int u = blockIdx.x;
    const UnitDev& U = units[u];
    double s = 0.0;
    for (uint32_t i = threadIdx.x; i < U.nftiles; i += 64) s += part[U.ftile_begin + i];
    s = wave_sum(s);
    if (threadIdx.x == 0) {
        const int vol = U.nx * U.ny * U.nz;  // int product, as src/calc-loss.cpp:37
        rmse[u] = vol > 0 ? sqrt(s / (double)vol) : 0.0;
    }
}

// ---------------------------------------------------------------------------
// Launch wrappers (host side), called by wc_capi.cpp.
size_t transform_lds_bytes(int lbx, int lby, int lbz) {
    return (size_t)4 * (1 << lbx) * (1 << lby) * (2 * (1 << lbz) + 1) * sizeof(float);
}

hipError_t launch_transform(hipStream_t st, const void* cells, int dtype, const UnitDev* units,
                            const XTile* tiles, uint32_t ntiles, size_t lds, float* out,
                            int out_at_cell_off, unsigned long long* keys) {
    if (ntiles == 0) return hipSuccess;
    if (dtype == 1) {
        if (keys)
            k_transform<double, true><<<ntiles, kThreads, lds, st>>>((const double*)cells, units, tiles, out,
                                                                   out_at_cell_off, keys);
        else
            k_transform<double, false><<<ntiles, kThreads, lds, st>>>((const double*)cells, units, tiles, out,
                                                                    out_at_cell_off, keys);
    } else {
        if (keys)
            k_transform<float, true><<<ntiles, kThreads, lds, st>>>((const float*)cells, units, tiles, out,
                                                                  out_at_cell_off, keys);
        else
            k_transform<float, false><<<ntiles, kThreads, lds, st>>>((const float*)cells, units, tiles, out,
                                                                   out_at_cell_off, keys);
    }
    return hipGetLastError();
}

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
    k_unit_offsets<<<1, 1024, 0, st>>>(units, n, kept, payload, offsets);
    return hipGetLastError();
}

hipError_t launch_flat_emit(hipStream_t st, const float* coef, const UnitDev* units, const FTile* ftiles,
                            uint32_t nft, const unsigned long long* keys, double keep, const uint32_t* toff,
                            const uint32_t* tprev, const uint64_t* offsets, uint8_t* payload) {
    if (nft)
        k_flat_emit<<<nft, kThreads, 0, st>>>(coef, units, ftiles, keys, keep, toff, tprev, offsets, payload);
    return hipGetLastError();
}

hipError_t launch_decode(hipStream_t st, const UnitDev* units, int n, const FTile* ftiles, uint32_t nft,
                         const uint8_t* payload, const uint64_t* offsets, uint64_t* tsum,
                         uint64_t* tbase, float* flat, uint32_t* err) {
    if (nft == 0) return hipSuccess;
    k_decode_count<<<nft, kThreads, 0, st>>>(units, ftiles, payload, offsets, tsum, err);
    k_decode_scan<<<n, kThreads, 0, st>>>(units, tsum, tbase);
    k_decode_scatter<<<nft, kThreads, 0, st>>>(units, ftiles, payload, offsets, tbase, flat);
    return hipGetLastError();
}

hipError_t launch_inverse(hipStream_t st, const float* flat, int flat_at_cell_off, const UnitDev* units,
                          const XTile* tiles, uint32_t ntiles, size_t lds, float* out) {
    if (ntiles == 0) return hipSuccess;
    k_inverse<<<ntiles, kThreads, lds, st>>>(flat, flat_at_cell_off, units, tiles, out);
    return hipGetLastError();
}

hipError_t launch_rmse(hipStream_t st, const void* orig, int dtype, const float* regen,
                       const UnitDev* units, int n, const FTile* ftiles, uint32_t nft, double* part,
                       double* rmse) {
    if (nft) {
        if (dtype == 1)
            k_rmse_partial<double><<<nft, kThreads, 0, st>>>((const double*)orig, regen, units, ftiles, part);
        else
            k_rmse_partial<float><<<nft, kThreads, 0, st>>>((const float*)orig, regen, units, ftiles, part);
    }
    k_rmse_final<<<n, 64, 0, st>>>(units, n, part, rmse);
    return hipGetLastError();
}

}  // namespace wc

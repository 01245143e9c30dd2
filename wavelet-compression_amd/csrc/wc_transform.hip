// wc_transform.hip — K1: one-level 3-D Haar, cells -> flat coefficients.
//   k_transform       generic tiles (any dims, odd tails)     src/compressor.cpp:85-185
//   k_transform_fast  even dims, D % 8 == 0 (4 z-blocks per thread)
// Both also reduce the unit's max-|c| key (src/compressor.cpp:212-215).
//
// Numerics (bit-exact with the reference): the reference
// pair `(a + b) / 2.0` is a float add, an exact halving in double and one
// rounding to float == `(a + b) * 0.5f` here; built with -ffp-contract=off and
// -fno-gpu-flush-denormals-to-zero so subnormals round identically.
#include "wc_device.h"

namespace wc {

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

// K1 fast path for units with even W, H, D and D % 8 == 0 (no tails; every
// tile's z extent is a multiple of 4 blocks).  A thread owns a column of 4
// consecutive z-blocks (bx, by, bz..bz+3): 16 independent x-pair loads in
// flight, and each of its 8 output rows gets 4 consecutive K -> one 16-B LDS
// write; rows are streamed out as 16-B global stores.
template <typename T, bool KEYS>
__global__ __launch_bounds__(kThreads) void k_transform_fast(
    const T* __restrict__ cells, const UnitDev* __restrict__ units, const XTile* __restrict__ tiles,
    float* __restrict__ out, int out_at_cell_off, unsigned long long* __restrict__ unit_key) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const XTile td = tiles[blockIdx.x];
    const UnitDev& U = units[td.unit];
    const int W = U.nx, H = U.ny, D = U.nz;
    const int hx = U.hx, hy = U.hy, hz = U.hz;
    const int lbx = U.lbx, lby = U.lby, lbz = U.lbz;
    const int TX = 1 << lbx, TY = 1 << lby, TZ = 1 << lbz;
    const int rowlen = 2 * TZ, rstride = rowlen + 4;  // 16-B rows; b128 writes of 8 lanes hit 32 banks
    const int ncol = (TX * TY * TZ) >> 2;
    const int64_t sy = W, sz = (int64_t)W * H;
    const T* __restrict__ src = cells + U.cell_off;
    const bool vec = (U.cell_off & 1) == 0;

    unsigned long long kmax = 0;
    for (int ci = threadIdx.x; ci < ncol; ci += kThreads) {
        const int bxl = ci & (TX - 1);
        const int byl = (ci >> lbx) & (TY - 1);
        const int bzq = ci >> (lbx + lby);  // quad of z-blocks within the tile
        const int bx = td.bx0 + bxl, by = td.by0 + byl, bzb = td.bz0 + 4 * bzq;
        if (bx >= hx || by >= hy || bzb >= hz) continue;
        float v[8][2][2];  // [z plane 0..7][dy][dx]
        const T* p0 = src + 2 * (int64_t)bx + sy * (2 * by) + sz * (2 * (int64_t)bzb);
#pragma unroll
        for (int zp = 0; zp < 8; ++zp)
#pragma unroll
            for (int dy = 0; dy < 2; ++dy) load_xpair<T>(p0 + sz * zp + sy * dy, true, vec, v[zp][dy][0], v[zp][dy][1]);
        float c[4][2][2][2];  // [q][sz][sy][sx]
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float a[2][2][2];  // Z sweep: a[sz][dy][dx]
#pragma unroll
            for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                for (int dx = 0; dx < 2; ++dx) {
                    a[0][dy][dx] = haar_lo(v[2 * q][dy][dx], v[2 * q + 1][dy][dx]);
                    a[1][dy][dx] = haar_hi(v[2 * q][dy][dx], v[2 * q + 1][dy][dx]);
                }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                float b[2][2];  // Y sweep: b[sy][dx]
#pragma unroll
                for (int dx = 0; dx < 2; ++dx) {
                    b[0][dx] = haar_lo(a[s][0][dx], a[s][1][dx]);
                    b[1][dx] = haar_hi(a[s][0][dx], a[s][1][dx]);
                }
#pragma unroll
                for (int t = 0; t < 2; ++t) {  // X sweep
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
                    const float4 w = make_float4(c[0][ssz][ssy][ssx], c[1][ssz][ssy][ssx],
                                                 c[2][ssz][ssy][ssx], c[3][ssz][ssy][ssx]);
                    *reinterpret_cast<float4*>(lds + row * rstride + (ssz << lbz) + 4 * bzq) = w;
                    if constexpr (KEYS) {
                        const int I = bx + ssx * hx, J = by + ssy * hy, K = bzb + ssz * hz;
                        const uint32_t f0 = (uint32_t)(((int64_t)I * H + J) * D + K);
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const uint32_t f = f0 + q;
                            const uint32_t ab = __float_as_uint(c[q][ssz][ssy][ssx]) & 0x7fffffffu;
                            unsigned long long key;
                            if (ab > 0x7f800000u)
                                key = (f == 0) ? kKeyNaNFirst : 0ull;
                            else
                                key = ((unsigned long long)ab << 32) | (unsigned long long)(0xffffffffu - f);
                            kmax = key > kmax ? key : kmax;
                        }
                    }
                }
    }
    __syncthreads();

    const uint64_t obase = out_at_cell_off ? U.cell_off : U.coef_off;
    float* __restrict__ dst = out + obase;
    const bool vst = (obase & 3) == 0;
    const int nrows = 4 * TX * TY;
    const int q4 = lbz - 1;  // log2(rowlen / 4)
    const int total4 = nrows << q4;
    for (int e = threadIdx.x; e < total4; e += kThreads) {
        const int row = e >> q4;
        const int col = (e & ((1 << q4) - 1)) << 2;
        const int ssz = col >> lbz, bzl = col & (TZ - 1);
        const int bxl = row & (TX - 1);
        int r2 = row >> lbx;
        const int ssx = r2 & 1;
        r2 >>= 1;
        const int byl = r2 & (TY - 1), ssy = r2 >> lby;
        const int bx = td.bx0 + bxl, by = td.by0 + byl, bz = td.bz0 + bzl;
        if (bx >= hx || by >= hy || bz >= hz) continue;
        const int I = bx + ssx * hx, J = by + ssy * hy, K = bz + ssz * hz;
        const float4 val = *reinterpret_cast<const float4*>(lds + row * rstride + col);
        float* o = dst + ((int64_t)I * H + J) * D + K;
        if (vst) {
            *reinterpret_cast<float4*>(o) = val;
        } else {
            o[0] = val.x;
            o[1] = val.y;
            o[2] = val.z;
            o[3] = val.w;
        }
    }

    if constexpr (KEYS) {
        kmax = wave_max_u64(kmax);
        if (lane_id() == 0 && kmax != 0) atomicMax(unit_key + td.unit, kmax);
    }
}

// ---------------------------------------------------------------------------
// Launch wrappers
size_t transform_lds_bytes(int lbx, int lby, int lbz) {
    return (size_t)4 * (1 << lbx) * (1 << lby) * (2 * (1 << lbz) + 1) * sizeof(float);
}

size_t transform_fast_lds_bytes(int lbx, int lby, int lbz) {
    return (size_t)4 * (1 << lbx) * (1 << lby) * (2 * (1 << lbz) + 4) * sizeof(float);
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

hipError_t launch_transform_fast(hipStream_t st, const void* cells, int dtype, const UnitDev* units,
                                 const XTile* tiles, uint32_t ntiles, size_t lds, float* out,
                                 int out_at_cell_off, unsigned long long* keys) {
    if (ntiles == 0) return hipSuccess;
    if (dtype == 1) {
        if (keys)
            k_transform_fast<double, true><<<ntiles, kThreads, lds, st>>>((const double*)cells, units, tiles, out,
                                                                        out_at_cell_off, keys);
        else
            k_transform_fast<double, false><<<ntiles, kThreads, lds, st>>>((const double*)cells, units, tiles, out,
                                                                         out_at_cell_off, keys);
    } else {
        if (keys)
            k_transform_fast<float, true><<<ntiles, kThreads, lds, st>>>((const float*)cells, units, tiles, out,
                                                                       out_at_cell_off, keys);
        else
            k_transform_fast<float, false><<<ntiles, kThreads, lds, st>>>((const float*)cells, units, tiles, out,
                                                                        out_at_cell_off, keys);
    }
    return hipGetLastError();
}

}  // namespace wc

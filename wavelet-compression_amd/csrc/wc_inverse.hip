// wc_inverse.hip — decode, inverse transform and RMSE.
//   K5       k_decode: rle_decode into dense rows    src/decompressor.cpp:14-30
//   K6       k_inverse{,_fast}: flat -> Box3D        src/decompressor.cpp:79-159
//   K7       k_rmse_*: per-unit RMSE                 src/calc-loss.cpp:12-43
// The inverse pair `avg +/- diff` is evaluated in double and stored as float
// by the reference; a float add is bit-identical (53 >= 2*24 + 2).
#include "wc_xform.h"

namespace wc {

// ---------------------------------------------------------------------------
// K5: rle_decode (src/decompressor.cpp:14-30) straight into the dense flat
// scratch, in one pass and without a memset.  Pair tile t (kFlatTile pairs)
// of a unit owns the flat range [S_t, S_t+1): from just after the previous
// tile's last pair through its own last pair (the unit's last tile: through
// ncoeff - 1), and writes every element of it — zeros between pairs.  Pair k
// lands at (sum of run + 1 over pairs <= k) - 1 while that is < ncoeff, which
// is rle_decode's `idx += run; if (idx < total) out[idx++] = val`; every later
// pair is dropped.  S_t (the sum over the unit's earlier tiles) comes from a
// decoupled look-back; a block takes its tile index from a per-unit ticket,
// so a tile's predecessors have always started, and blocks past the unit's
// last pair tile exit.
//
// Pairs are loaded coalesced: wave w, round r, lane l holds pair
// w*1024 + r*64 + l of the tile; positions come from wave scans of run + 1.
// The range is written in kDecChunk-element rounds: zero an LDS chunk, drop
// the tile's pairs that fall in it, copy it out with 16-B stores.
constexpr int kDecRounds = kFlatTile / kThreads;  // 16 pairs per lane
constexpr int kDecChunk = 4096;                   // floats per write round (16 KB of LDS)

// Header check: the dims and ncoeff must be the unit's and nrle >= 0.  More
// pairs than coefficients are accepted: rle_decode drops every pair whose
// index reaches ncoeff (src/decompressor.cpp:20-27), as here.
__device__ __forceinline__ bool read_header(const UnitDev& U, const uint8_t* __restrict__ ph, int32_t& nrle) {
    const int32_t* h = reinterpret_cast<const int32_t*>(ph);
    nrle = h[4];
    return h[0] == U.nx && h[1] == U.ny && h[2] == U.nz && h[3] == (int32_t)U.ncells && nrle >= 0;
}

__global__ __launch_bounds__(kThreads) void k_decode(const UnitDev* __restrict__ units,
                                                   const FTile* __restrict__ tiles,
                                                   const uint8_t* __restrict__ payload,
                                                   const uint64_t* __restrict__ offsets, uint32_t* __restrict__ ticket,
                                                   unsigned long long* __restrict__ status, float* __restrict__ flat,
                                                   uint32_t* __restrict__ err, int ordered) {
    __shared__ __attribute__((aligned(16))) float buf[kDecChunk];
    __shared__ unsigned long long s_w[4];
    __shared__ unsigned long long s_x[2];
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const FTile ft = tiles[blockIdx.x];
    const uint32_t u = ft.unit;
    const UnitDev& U = units[u];
    const uint8_t* ph = payload + offsets[u];
    int32_t nrle;
    const bool hok = read_header(U, ph, nrle);
    const int64_t n = hok ? nrle : 0;
    const uint32_t ntile = n ? (uint32_t)((n + kFlatTile - 1) / kFlatTile) : 1u;
    // The plan launches ceil(ncoeff / kFlatTile) blocks per unit; those whose
    // plan index is past the payload's pair tiles exit before any atomic.
    if (ft.index >= ntile) return;  // uniform
    // Tile index: ordered form (WC_OPT_ORDERED 1) = plan index: the plan
    // interleaves tiles by index across units, so a tile's look-back waits
    // only on lower block ids of its unit (DESIGN.md §Forward progress);
    // ticket form = the unit's next ticket, whatever the dispatch order.
    uint32_t t = ft.index;
    if (!ordered) {
        if (tid == 0) s_x[0] = atomicAdd(ticket + u, 1u);
        __syncthreads();
        t = (uint32_t)s_x[0];
    }
    if (!hok && t == 0 && tid == 0) atomicOr(err, kErrHeader);

    // 1. this lane's pairs and their in-wave inclusive sums of (run + 1)
    const uint2* __restrict__ pr = reinterpret_cast<const uint2*>(ph + 20);
    const int64_t kw = (int64_t)t * kFlatTile + (int64_t)w * (kFlatTile / 4);
    uint2 q[kDecRounds];
#pragma unroll
    for (int r = 0; r < kDecRounds; ++r) {
        const int64_t k = kw + r * 64 + l;
        q[r] = k < n ? pr[k] : make_uint2(0u, 0u);
    }
    uint64_t incl[kDecRounds];
    uint64_t wsum = 0;
    bool neg = false;
#pragma unroll
    for (int r = 0; r < kDecRounds; ++r) {
        const int64_t k = kw + r * 64 + l;
        const int32_t run = (int32_t)q[r].x;
        neg |= k < n && run < 0;
        const uint64_t v = k < n ? (uint64_t)(int64_t)run + 1 : 0;
        const uint64_t s = wave_incl_sum(v);
        incl[r] = wsum + s;
        wsum += ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(s >> 32), 63) << 32) |
                __builtin_amdgcn_readlane((uint32_t)s, 63);
    }
    if (neg) atomicOr(err, kErrNegativeRun);
    if (l == 0) s_w[w] = wsum;
    __syncthreads();
    uint64_t wexcl = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        wexcl += i < w ? s_w[i] : 0;
        tot += s_w[i];
    }

    // 2. start of this tile's range: look-back over the unit's earlier tiles
    if (w == 0) {
        unsigned long long* st = status + U.ftile_begin;
        unsigned long long excl = 0;
        if (t == 0) {
            if (l == 0) st_rlx(st, kFlagIncl | (tot & kMask62));
        } else {
            if (l == 0) st_rlx(st + t, kFlagAgg | (tot & kMask62));
            excl = lookback_sum62(st, (int64_t)t, l, err);
            if (l == 0) st_rlx(st + t, kFlagIncl | ((excl + tot) & kMask62));
        }
        if (l == 0) s_x[1] = excl;
    }
    __syncthreads();
    const uint64_t nc = U.ncells;
    const uint64_t A = s_x[1];
    const uint64_t Ac = A < nc ? A : nc;
    const uint64_t B = (t + 1 == ntile || tot >= nc - Ac) ? nc : Ac + tot;
    const uint64_t base = A + wexcl - 1;  // + incl[r]: position of the lane's pair in round r

    // 3. write [Ac, B): zeros with this tile's pairs dropped in
    float* __restrict__ dst = flat + U.coef_off;
    float4* b4 = reinterpret_cast<float4*>(buf);
    for (uint64_t c0 = Ac & ~3ull; c0 < B; c0 += kDecChunk) {
        for (int i = tid; i < kDecChunk / 4; i += kThreads) b4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kDecRounds; ++r) {
            const int64_t k = kw + r * 64 + l;
            const uint64_t o = base + incl[r] - c0;
            if (k < n && o < (uint64_t)kDecChunk) buf[o] = __uint_as_float(q[r].y);
        }
        __syncthreads();
        for (int i = tid; i < kDecChunk / 4; i += kThreads) {
            const uint64_t g = c0 + 4ull * (uint64_t)i;
            if (g >= B) break;
            const float4 v = b4[i];
            if (g >= Ac && g + 4 <= B) {
                *reinterpret_cast<float4*>(dst + g) = v;
            } else {
                const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (g + j >= Ac && g + j < B) dst[g + j] = e[j];
            }
        }
        __syncthreads();
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

// K6, fast tiles (even W, H, D with D % 8 == 0, the forward's fast shape): a
// thread owns a column of 4 consecutive z-blocks.  Flat rows are staged with
// 16-B loads; each of the 8 sub-band values is read back as one float4 (the 4
// z-blocks), then X, Y, Z synthesis per block and 8-B x-pair stores.
__global__ __launch_bounds__(kThreads) void k_inverse_fast(const float* __restrict__ flat,
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
    const int rstride = 2 * TZ + 4;
    const uint64_t ibase = flat_at_cell_off ? U.cell_off : U.coef_off;
    const float* __restrict__ srcf = flat + ibase;
    const bool vin = (ibase & 3) == 0;

    const int nrows = 4 * TX * TY;
    const int q4 = lbz - 1;  // log2(row length / 4)
    const int total4 = nrows << q4;
    for (int e = threadIdx.x; e < total4; e += kThreads) {
        const int row = e >> q4;
        const int col = (e & ((1 << q4) - 1)) << 2;
        const int ssz = col >> lbz, bzl = col & (TZ - 1);
        int bxl, ssx, byl, ssy;
        row_of(row, lbx, lby, bxl, ssx, byl, ssy);
        const int bx = td.bx0 + bxl, by = td.by0 + byl, bz = td.bz0 + bzl;
        if (bx >= hx || by >= hy || bz >= hz) continue;
        const int I = bx + ssx * hx, J = by + ssy * hy, K = bz + ssz * hz;
        const float* p = srcf + ((int64_t)I * H + J) * D + K;
        float4 v;
        if (vin)
            v = *reinterpret_cast<const float4*>(p);
        else
            v = make_float4(p[0], p[1], p[2], p[3]);
        *reinterpret_cast<float4*>(lds + row * rstride + col) = v;
    }
    __syncthreads();

    float* __restrict__ dst = out + U.cell_off;
    const int64_t sy = W, sz = (int64_t)W * H;
    const bool vout = (U.cell_off & 1) == 0;
    const int ncol = (TX * TY * TZ) >> 2;
    for (int ci = threadIdx.x; ci < ncol; ci += kThreads) {
        const int bxl = ci & (TX - 1);
        const int byl = (ci >> lbx) & (TY - 1);
        const int bzq = ci >> (lbx + lby);
        const int bx = td.bx0 + bxl, by = td.by0 + byl, bzb = td.bz0 + 4 * bzq;
        if (bx >= hx || by >= hy || bzb >= hz) continue;
        float c[2][2][2][4];  // [sz][sy][sx][z-block]
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int x = 0; x < 2; ++x) {
                    const int row = ((((t << lby) + byl) * 2 + x) << lbx) + bxl;
                    const float4 v = *reinterpret_cast<const float4*>(lds + row * rstride + (s << lbz) + 4 * bzq);
                    c[s][t][x][0] = v.x;
                    c[s][t][x][1] = v.y;
                    c[s][t][x][2] = v.z;
                    c[s][t][x][3] = v.w;
                }
#pragma unroll
        for (int qb = 0; qb < 4; ++qb) {
            float X[2][2][2], Y[2][2][2], V[2][2][2];
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    X[s][t][0] = c[s][t][0][qb] + c[s][t][1][qb];
                    X[s][t][1] = c[s][t][0][qb] - c[s][t][1][qb];
                }
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int x = 0; x < 2; ++x) {
                    Y[s][0][x] = X[s][0][x] + X[s][1][x];
                    Y[s][1][x] = X[s][0][x] - X[s][1][x];
                }
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int x = 0; x < 2; ++x) {
                    V[0][t][x] = Y[0][t][x] + Y[1][t][x];
                    V[1][t][x] = Y[0][t][x] - Y[1][t][x];
                }
#pragma unroll
            for (int dz = 0; dz < 2; ++dz)
#pragma unroll
                for (int dy = 0; dy < 2; ++dy) {
                    float* p = dst + 2 * (int64_t)bx + sy * (2 * by + dy) + sz * (2 * (bzb + qb) + dz);
                    if (vout) {
                        *reinterpret_cast<float2*>(p) = make_float2(V[dz][dy][0], V[dz][dy][1]);
                    } else {
                        p[0] = V[dz][dy][0];
                        p[1] = V[dz][dy][1];
                    }
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
// Launch wrappers
hipError_t launch_decode(hipStream_t st, const UnitDev* units, const FTile* ftiles, uint32_t nft,
                         const uint8_t* payload, const uint64_t* offsets, uint32_t* ticket,
                         unsigned long long* status, float* flat, uint32_t* err, int ordered) {
    if (nft == 0) return hipSuccess;
    k_decode<<<nft, kThreads, 0, st>>>(units, ftiles, payload, offsets, ticket, status, flat, err, ordered);
    return hipGetLastError();
}

// Generic tiles [0, ngen) through k_inverse, fast tiles after them through
// k_inverse_fast (the plan's xtiles order).
hipError_t launch_inverse(hipStream_t st, const float* flat, int flat_at_cell_off, const UnitDev* units,
                          const XTile* tiles, uint32_t ngen, size_t lds_gen, uint32_t nfast, size_t lds_fast,
                          float* out) {
    if (ngen) k_inverse<<<ngen, kThreads, lds_gen, st>>>(flat, flat_at_cell_off, units, tiles, out);
    if (nfast) k_inverse_fast<<<nfast, kThreads, lds_fast, st>>>(flat, flat_at_cell_off, units, tiles + ngen, out);
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

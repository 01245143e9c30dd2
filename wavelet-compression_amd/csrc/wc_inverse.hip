// wc_inverse.hip — decode, inverse transform and RMSE.
//   K5a/b/c  rle_decode as scan + scatter            src/decompressor.cpp:14-30
//   K6       k_inverse: flat coefficients -> Box3D   src/decompressor.cpp:79-159
//   K7       k_rmse_*: per-unit RMSE                 src/calc-loss.cpp:12-43
// The inverse pair `avg +/- diff` is evaluated in double and stored as float
// by the reference; a float add is bit-identical (53 >= 2*24 + 2).
#include "wc_device.h"

namespace wc {

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
// Launch wrappers
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

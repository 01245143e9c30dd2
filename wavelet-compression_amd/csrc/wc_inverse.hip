// wc_inverse.hip — decode, inverse transform and RMSE.
//   K5   k_decode: rle_decode                        src/decompressor.cpp:14-30
//        - row-indexed units: a row index of the payload's pairs
//        - other units: dense flat coefficients
//   K6r  k_inverse_rows: pairs -> Box3D, row-indexed  src/decompressor.cpp:14-30, 79-159
//   K6   k_inverse{,_fast}: dense flat -> Box3D       src/decompressor.cpp:79-159
//   K7   k_rmse_*: per-unit RMSE                      src/calc-loss.cpp:12-43
// The inverse pair `avg +/- diff` is evaluated in double and stored as float
// by the reference; a float add is bit-identical (53 >= 2*24 + 2).
#include "wc_xform.h"

#include <algorithm>

namespace wc {

// ---------------------------------------------------------------------------
// K5: rle_decode (src/decompressor.cpp:14-30).  Pair k lands at flat position
// p_k = (sum of run + 1 over pairs <= k) - 1 while that is < ncoeff, which is
// rle_decode's `idx += run; if (idx < total) out[idx++] = val`; every later
// pair is dropped.  Pair tile t (kFlatTile pairs) gets the sum over the unit's
// earlier tiles from a decoupled look-back (tile index from the launch order
// or a per-unit ticket, WC_OPT_ORDERED); blocks past the payload's last pair
// tile exit.  Pairs are loaded coalesced: wave w, round r, lane l holds pair
// w*1024 + r*64 + l of the tile; positions come from wave scans of run + 1.
//
// Two forms:
//   k_rowindex  row-indexed units (U.rix, the even-dims fast shapes): writes
//               no coefficient.  For every flat row r = I*H + J (D
//               coefficients) whose first position r*D lies in (p_{k-1}, p_k]
//               it writes rowinfo[r] = (k, p_k - r*D): the row's pairs are k ..
//               rowinfo[r+1].x - 1 and the first lands at p_k.  The virtual
//               pair k = nrle at position ncoeff closes the table (rows past the
//               last pair and the sentinel row W*H); a dropped pair counts as
//               position ncoeff.  K6r then reads each tile's pairs straight
//               from the payload: the dense fp32 scratch is never materialised.
//   k_decode    other units: the tile owns the flat range [S_t, S_t+1) from just
//               after the previous tile's last pair through its own last pair
//               (the unit's last tile: through ncoeff - 1) and writes every
//               element of it — zeros between pairs — through LDS in
//               kDecChunk-element rounds (no memset of the scratch).
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

// The same with saturating adds (v_add_u32 clamp): positions at or past
// ncoeff (< 2^31) are all "dropped", so sums clamped at 2^32 - 1 decide the
// same rows as exact ones.
__device__ __forceinline__ uint32_t sat_add(uint32_t a, uint32_t b) { return __builtin_elementwise_add_sat(a, b); }

__device__ __forceinline__ uint32_t wave_incl_sum32_sat(uint32_t v) {
    v = sat_add(v, __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false));
    v = sat_add(v, __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false));
    v = sat_add(v, __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false));
    v = sat_add(v, __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false));
    v = sat_add(v, __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false));
    v = sat_add(v, __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false));
    return v;
}

// Row index of the row-indexed units.  Only the runs are needed (the values
// stay in the payload for K6r).  A negative run (malformed; the reference's
// behaviour is undefined) counts as run 0, so positions never decrease and
// every row entry is written: K6r never sees a stale or out-of-range entry.
//
// One block per pair tile of the plan (rdtiles: interleaved by tile index
// across units, so a tile's look-back waits only on lower block ids, DESIGN.md
// §Forward progress; or the tile index from a per-unit ticket); blocks past
// the payload's pair tiles exit after the header.  The look-back granules are
// epoch-tagged: no zeroing between calls.

#ifndef WC_RIX_MINB
#define WC_RIX_MINB 8  // waves per SIMD the register budget is sized for (4-wave blocks: 8 per CU, <= 64 VGPRs)
#endif
__global__ __launch_bounds__(kThreads, WC_RIX_MINB) void k_rowindex(const UnitDev* __restrict__ units,
                                                     const FTile* __restrict__ tiles, uint32_t* __restrict__ ticket,
                                                     const uint8_t* __restrict__ payload,
                                                     const uint64_t* __restrict__ offsets,
                                                     unsigned long long* __restrict__ status,
                                                     uint2* __restrict__ rowinfo, uint32_t* __restrict__ err,
                                                     int ordered, uint32_t epoch, uint32_t* __restrict__ npairs) {
    __shared__ uint32_t s_w[4];
    __shared__ uint32_t s_x[2];
    // the waves' inclusive sums, parked across the look-back (round r of thread
    // tid at [r][tid]: the row phase holds no 16-register array; 16 KB per workgroup)
    __shared__ uint32_t s_v[kRixRounds5][kThreads];
    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const FTile ft = cst(tiles)[blockIdx.x];
    const uint32_t u = ft.unit;
    const UnitDev U = cst(units)[u];  // scalar copy: no reloads after the stores below
    const uint8_t* ph = payload + cst(offsets)[u];
    int32_t nrle;
    const bool hok = read_header(U, ph, nrle);
    const uint32_t n = hok ? (uint32_t)nrle : 0u;
    if (ft.index == 0 && tid == 0) npairs[u] = n;  // K6r bounds its pair indices by it
    // tiles up to the one holding the virtual pair k = n (the plan launches
    // floor(ncoeff / kRixTile) + 1, enough for the first dropped pair)
    if (ft.index > n / (uint32_t)kRixTile) return;  // uniform
    uint32_t t = ordered == 2 ? n / (uint32_t)kRixTile - ft.index : ft.index;  // 2: reversed (test hook)
    if (!ordered) {
        if (tid == 0) s_x[0] = atomicAdd(ticket + u, 1u);
        __syncthreads();
        t = s_x[0];
    }
    const uint32_t* __restrict__ runs = reinterpret_cast<const uint32_t*>(ph + 20);
    uint32_t v[kRixRounds5];
    {
        const uint32_t kw = t * (uint32_t)kRixTile + (uint32_t)w * (kRixTile / 4);
#pragma unroll
        for (int r = 0; r < kRixRounds5; ++r) {
            const uint32_t k = kw + r * 64 + l;
            // nontemporal: K5 -12 % at C2, K6r after it +1 %, C5 even (profiles/r05/experiments/gpu_nt.txt)
            v[r] = k < n ? __builtin_nontemporal_load(runs + 2 * k) : 0u;
        }
    }
    if (!hok && t == 0 && tid == 0) atomicOr(err, kErrHeader);

    // 1. v = run + 1 (k < n), 0 (k >= n) -> saturating in-wave inclusive sums
    const uint32_t kw = t * (uint32_t)kRixTile + (uint32_t)w * (kRixTile / 4);
    bool neg = false;
    uint32_t wsum = 0;
#pragma unroll
    for (int r = 0; r < kRixRounds5; ++r) {
        const uint32_t k = kw + r * 64 + l;
        const int32_t run = (int32_t)v[r];
        neg |= k < n && run < 0;
        const uint32_t x = k < n ? (run < 0 ? 1u : (uint32_t)run + 1u) : 0u;
        const uint32_t s = wave_incl_sum32_sat(x);
        s_v[r][tid] = sat_add(wsum, s);
        wsum = sat_add(wsum, __builtin_amdgcn_readlane(s, 63));
    }
    if (neg) atomicOr(err, kErrNegativeRun);
    if (l == 0) s_w[w] = wsum;
    __syncthreads();
    uint32_t wexcl = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        wexcl = i < w ? sat_add(wexcl, s_w[i]) : wexcl;
        tot = sat_add(tot, s_w[i]);
    }

    // 2. the sum over the unit's earlier tiles: look-back
    if (w == 0) {
        unsigned long long* st = status + U.dt_begin;
        uint32_t excl = 0;
        if (t == 0) {
            if (l == 0) st_rlx(st, granule_e(kFlagIncl, epoch, tot));
        } else {
            if (l == 0) st_rlx(st + t, granule_e(kFlagAgg, epoch, tot));
            // a predecessor tile unpublished after the wait bound: its sum from its pairs
            excl = lookback_sum32e(st, (int64_t)t, l, err, epoch, [&](int64_t j) -> uint32_t {
                const uint32_t k0 = (uint32_t)j * (uint32_t)kRixTile, k1 = min(k0 + (uint32_t)kRixTile, n);
                uint32_t a = 0;
                for (uint32_t k = k0 + (uint32_t)l; k < k1; k += 64) {
                    const int32_t run = (int32_t)runs[2 * k];
                    a = sat_add(a, run < 0 ? 1u : (uint32_t)run + 1u);
                }
                return __builtin_amdgcn_readlane(wave_incl_sum32_sat(a), 63);
            });
            if (l == 0) st_rlx(st + t, granule_e(kFlagIncl, epoch, sat_add(excl, tot)));
        }
        if (l == 0) s_x[1] = (uint32_t)excl;
    }
    __syncthreads();
    const uint32_t nc = (uint32_t)U.ncells;
    const uint32_t A = sat_add(s_x[1], wexcl);

    // 3. row entries.  Pair k covers rows (rhi_{k-1}, rhi_k], rhi_k =
    // floor(ph_k / D) with ph_k = min(p_k, ncoeff) (p_k = S - 1, S the
    // saturating inclusive sum of run + 1; the virtual pair k == n sits at
    // ncoeff), and rhi_{-1} = -1.  Positions at or past ncoeff (< 2^31) clamp
    // to it, so saturated sums give the same rows.  rhi_{k-1} comes from the
    // lane below, the previous round's lane 63, or for the wave's first pair
    // from A (= p_{k-1} + 1): one division per pair.
    uint2* __restrict__ ri = rowinfo + U.row_off;
    const uint32_t D = (uint32_t)U.nz;
    int32_t carry = A == 0 ? -1 : (int32_t)div_rows(min(A - 1u, nc), U.dmagic);  // rhi of the pair before
#pragma unroll
    for (int r = 0; r < kRixRounds5; ++r) {
        const uint32_t k = kw + r * 64 + l;
        const uint32_t vr = s_v[r][tid];
        const uint32_t phk = k < n ? min(sat_add(A, vr) - 1u, nc) : nc;
        const int32_t rhi = k <= n ? (int32_t)div_rows(phk, U.dmagic) : -1;
        // rhi of pair k - 1: lane l - 1, the carry in lane 0
        const int32_t from = __builtin_amdgcn_update_dpp(0, rhi, 0x138, 0xf, 0xf, false);  // wave_shr:1
        const int32_t rlo = (l == 0 ? carry : from) + 1;
        const uint32_t cnt = (k <= n && rhi >= rlo) ? (uint32_t)(rhi - rlo + 1) : 0u;
        write_rows(ri, (uint32_t)rlo, cnt, k, phk, D, l);
        carry = __builtin_amdgcn_readlane(rhi, 63);
        if (carry < 0) break;  // uniform: lane 63 is past the virtual pair, so is every later round
    }
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
    uint32_t t = ordered == 2 ? ntile - 1u - ft.index : ft.index;  // 2: reversed (test hook)
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
        unsigned long long* st = status + U.dt_begin;
        unsigned long long excl = 0;
        if (t == 0) {
            if (l == 0) st_rlx(st, kFlagIncl | (tot & kMask62));
        } else {
            if (l == 0) st_rlx(st + t, kFlagAgg | (tot & kMask62));
            // a predecessor tile unpublished after the wait bound: its sum from its pairs
            excl = lookback_sum62(st, (int64_t)t, l, err, [&](int64_t j) -> unsigned long long {
                const int64_t k0 = j * kFlatTile, k1 = min(k0 + (int64_t)kFlatTile, n);
                unsigned long long a = 0;
                for (int64_t k = k0 + l; k < k1; k += 64) a += (unsigned long long)((int64_t)(int32_t)pr[k].x + 1);
                return wave_sum(a);
            });
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
// K6r: inverse of a row-indexed unit straight from its payload.  A tile is
// TX x TY blocks in (x, y) and all of z; its coefficients are the 4 TX
// "ranges" g = (ssx * 2 + ssy) * TX + bxl: I = bx0 + bxl + ssx * hx, flat rows
// I*H + J for J in [by0, by0 + TY) + ssy * hy — TY*D consecutive flat
// coefficients (x slowest, z fastest: src/compressor.cpp:178-181), so one
// contiguous run of pairs, rowinfo[r0].x .. rowinfo[r0 + TY].x - 1, whose
// first pair lands at rowinfo[r0].y within the range.
//
// Wave w owns the ranges g = w + 4j (lane j holds range j's row entries; every
// sub-band class in every wave) and an LDS region of its own.  It zeroes the
// region and walks its ranges one at a time, 64 pairs per round (range j's
// round m: lane l holds pair m*64 + l; rix_scatter_range).  Position in the
// range = first + (inclusive DPP scan of run + 1 over the range's pairs after
// its first); the value is dropped into LDS.  Then one block barrier, and X, Y,
// Z synthesis per 2x2x2 block (src/decompressor.cpp:89-156) from LDS sub-band
// reads with 16-B x-quad stores (8-B x-pair stores where the output is not
// 16-B aligned); with fp64 originals the fused RMSE sums the squared
// differences of the cells each thread has just synthesised.
//
// Persistent: workgroup b runs tiles b, b + G, ...  The latency of the
// dependent loads (tile record -> row entries + payload offset -> pairs) is
// hidden by a two-stage prefetch: while tile t is synthesised, the pairs of
// tile t + G are in flight (the first round of each range; the rest are loaded
// when scattered) and the row entries of tile t + 2G.
//
// The row index of a unit is complete and monotone whatever the payload
// (k_rowindex: every tile's look-back completes, negative runs count as 0),
// pair indices are clamped to the payload's pair count, and every LDS address
// is checked against the range: a malformed payload (reported by K5) or a row
// index of other payloads gives garbage cells, never an out-of-bounds access.
#ifndef WC_RIX_ROUNDS
#define WC_RIX_ROUNDS 16  // prefetch slots (one per range): 128 VGPRs with the x-quad synthesis, 4 waves per SIMD, no spills
#endif
constexpr int kRixRounds = WC_RIX_ROUNDS;
  // rounds of 64 pairs prefetched per wave

// Range info of this lane (range g = w + 4l of tile T, lanes l < TX).
struct RixRange {
    uint32_t ks, c0, e;  // rowinfo[r0] = (ks, c0), rowinfo[r0 + tyv].x = e
};

__device__ __forceinline__ RixRange rix_load_range(const RTile& T, const uint2* __restrict__ rowinfo, int w, int l) {
    RixRange R{0u, 0u, 0u};
    const int TX = 1 << T.lbx;
    if (l < TX) {
        const int g = w + 4 * l, bxl = g & (TX - 1), ssy = (g >> T.lbx) & 1, ssx = g >> (T.lbx + 1);
        const int bx = T.bx0 + bxl, hx = T.W >> 1, hy = T.H >> 1;
        if (bx < hx) {
            const uint64_t r0 = (uint64_t)(bx + ssx * hx) * T.H + T.by0 + ssy * hy;
            const uint2 a = rowinfo[T.row_off + r0];
            R.ks = a.x;
            R.c0 = a.y;
            R.e = rowinfo[T.row_off + r0 + T.tyv].x;
        }
    }
    return R;
}

// Tile T's pairs in the payload; npairs[unit]: their count, checked against
// the unit (k_rowindex or k_pair_counts: 0 for a header that disagrees).
__device__ __forceinline__ const uint2* rix_payload(const uint8_t* __restrict__ payload,
                                                    const uint64_t* __restrict__ offsets,
                                                    const uint32_t* __restrict__ npairs, const RTile& T,
                                                    uint32_t& np) {
    np = cst(npairs)[T.unit];
    return reinterpret_cast<const uint2*>(payload + offsets[T.unit] + 20);
}

// Per-lane range plan of a wave: pair count of range l (lanes < TX).
struct RixPlan {
    uint32_t cnt;
};

// Pair indices are clamped to the payload's pair count np (an entry past it,
// from a row index that does not belong to this payload, reads no pair) here,
// where the range is first used: clamping at the load would wait for the row
// entries there, behind the pair prefetch issued before them.
__device__ __forceinline__ RixPlan rix_plan(const RTile& T, RixRange& R, uint32_t np, int l) {
    const uint32_t rlen = (uint32_t)(T.tyv * T.D);
    R.ks = min(R.ks, np);
    const uint32_t e = min(R.e, np);
    RixPlan p;
    p.cnt = (l < (1 << T.lbx) && e > R.ks) ? min(e - R.ks, rlen) : 0u;
    return p;
}

// Rounds of 64 pairs, range-major (round 4; before: rounds in flat order over
// the wave's ranges, each round finding its range by a ballot and popcount,
// measured equal at C2 and 4 % slower at C5, profiles/r04/experiments/
// gpu_rangemajor.txt): prefetch slot j holds the first 64 pairs of range j
// (lane l: pair l), so a round's range is a compile-time constant of the
// unrolled loops and the row fields come from immediate-lane readlanes.  Later
// rounds of a range (more than 64 pairs) and ranges past the prefetch slots
// are loaded when scattered.
template <int J>
__device__ __forceinline__ uint2 rix_load_first(const uint2* __restrict__ pr, const RixRange& R, const RixPlan& p,
                                                int l) {
    const uint32_t cnt = __builtin_amdgcn_readlane(p.cnt, J);
    const uint32_t ks = __builtin_amdgcn_readlane(R.ks, J);
    return (uint32_t)l < cnt ? pr[ks + (uint32_t)l] : make_uint2(0u, 0u);
}

// One round of a range: pair i = m0 + l (q) lands at carry + the inclusive
// scan of run + 1 over the round (the range's first pair: + 0).  Returns the
// carry of the next round.
__device__ __forceinline__ uint32_t rix_round(float* __restrict__ rg, uint32_t rlen, uint2 q, uint32_t i,
                                              uint32_t cnt, uint32_t carry) {
    const int32_t run = (int32_t)q.x;
    const uint32_t x = (i < cnt && i > 0) ? (run < 0 ? 1u : (uint32_t)run + 1u) : 0u;
    const uint32_t pos = carry + wave_incl_sum32(x);
    if (i < cnt && pos < rlen) rg[pos] = __uint_as_float(q.y);
    return __builtin_amdgcn_readlane(pos, 63);
}

// Scatter range j's pairs from round m0 on (q0: round m0's pairs, or loaded
// here when !have0; later rounds are loaded here).
__device__ __forceinline__ void rix_scatter_range(float* __restrict__ reg, int RS, uint32_t rlen, uint2 q0, bool have0,
                                                  const uint2* __restrict__ pr, const RixRange& R, const RixPlan& p,
                                                  int l, int j, uint32_t m0 = 0, uint32_t carry0 = ~0u) {
    const uint32_t cnt = __builtin_amdgcn_readlane(p.cnt, j);
    const uint32_t ks = __builtin_amdgcn_readlane(R.ks, j);
    float* __restrict__ rg = reg + j * RS;
    uint32_t carry = m0 == 0 ? __builtin_amdgcn_readlane(R.c0, j) : carry0;
    for (uint32_t m = m0; m < cnt; m += 64) {  // uniform
        const uint32_t i = m + (uint32_t)l;
        uint2 q = q0;
        if (m != m0 || !have0) q = i < cnt ? pr[ks + i] : make_uint2(0u, 0u);
        carry = rix_round(rg, rlen, q, i, cnt, carry);
    }
}

// Inverse of one 2x2x2 block (src/decompressor.cpp:89-156: X, then Y, then Z
// pairs avg +/- diff): c[sz][sy][sx] -> V[dz][dy][dx].
__device__ __forceinline__ void synth_block(const float (&c)[2][2][2], float (&V)[2][2][2]) {
    float X[2][2][2], Y[2][2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            X[s][t][0] = c[s][t][0] + c[s][t][1];
            X[s][t][1] = c[s][t][0] - c[s][t][1];
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
}

// The prefetch of a tile's pairs into q: the first round of each range.
template <int NR>
__device__ __forceinline__ void rix_prefetch(uint2 (&q)[NR], const uint2* __restrict__ pr, const RixRange& R,
                                             const RixPlan& p, const RTile& T, int l) {
    const int TX = 1 << T.lbx;
#define WC_RIX_PF(J) if (J < NR && J < TX) q[J < NR ? J : 0] = rix_load_first<J>(pr, R, p, l);
    WC_RIX_PF(0) WC_RIX_PF(1) WC_RIX_PF(2) WC_RIX_PF(3) WC_RIX_PF(4) WC_RIX_PF(5) WC_RIX_PF(6) WC_RIX_PF(7)
    WC_RIX_PF(8) WC_RIX_PF(9) WC_RIX_PF(10) WC_RIX_PF(11) WC_RIX_PF(12) WC_RIX_PF(13) WC_RIX_PF(14) WC_RIX_PF(15)
#undef WC_RIX_PF
    static_assert(NR <= 16, "rix_prefetch: extend WC_RIX_PF");
}

#ifndef WC_RIX_RMSE_ROUNDS_LESS
// prefetch slots given up by the inline fused-RMSE form (OT 1): 3 is the fewest
// without spills; 9 measured 3 % faster at C3, 1 % at C2 (profiles/r05/
// experiments/gpu_k6r_rmse_slots.txt)
#define WC_RIX_RMSE_ROUNDS_LESS 9
#endif
#ifndef WC_RIX_RMSE_PASS_ROUNDS_LESS
#define WC_RIX_RMSE_PASS_ROUNDS_LESS 3  // the same for the separate-pass forms (OT 2, 3): no spills
#endif
// Original cells of one z-block pair of an x-quad column (fused RMSE): at
// cell index base + sy dy + sz dz, 4 consecutive x cells, narrowed to float
// as calc_rmse_per_box sees them (src/calc-loss.cpp:12-43 on Box3D floats).
template <int OT>
__device__ __forceinline__ void rix_load_orig(const void* __restrict__ orig, int64_t base, int64_t sy, int64_t sz,
                                              float (&o)[2][2][4]) {
#pragma unroll
    for (int dz = 0; dz < 2; ++dz)
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) {
            const int64_t i = base + sy * dy + sz * dz;
            if constexpr (OT == 1) {
                const f64x2* p = reinterpret_cast<const f64x2*>(static_cast<const double*>(orig) + i);
                const f64x2 a = p[0], b = p[1];
                o[dz][dy][0] = (float)a.x;
                o[dz][dy][1] = (float)a.y;
                o[dz][dy][2] = (float)b.x;
                o[dz][dy][3] = (float)b.y;
            } else {
                const float4 a = *reinterpret_cast<const float4*>(static_cast<const float*>(orig) + i);
                o[dz][dy][0] = a.x;
                o[dz][dy][1] = a.y;
                o[dz][dy][2] = a.z;
                o[dz][dy][3] = a.w;
            }
        }
}

// Tiles of workgroup b: blocked (a contiguous run of ceil(ntiles / G) tiles:
// consecutive tiles share the payload lines at their range boundaries and the
// unit's row entries) or strided (b, b + G, ...).
// OT (fused calc_rmse_per_box, wc_inverse_rmse): 0 none, 1 fp64 original
// cells (16-B aligned: summed inside the x-quad synthesis), 2 fp32 original
// cells, 3 fp64 original cells at a base that is not 16-B aligned (the
// separate pass below, scalar loads).  After the tile's synthesis (barrier), each
// wave re-reads part of the tile's output (L2-resident, just written) beside
// the original cells and adds ((float)orig - regen)^2 in double; the wave's
// sum goes to part[4 * tile + wave] and k_rmse_rows_final sums a unit's in
// order.  A pass of its own keeps the synthesis' registers untouched.
template <int OT>
#ifndef WC_RIX_MINW
#define WC_RIX_MINW 4  // K6r: waves per SIMD the register budget is sized for (4-wave blocks: workgroups per CU)
#endif
__global__ __launch_bounds__(kThreads, WC_RIX_MINW) void k_inverse_rows(const RTile* __restrict__ tiles, uint32_t ntiles,
                                                         const uint8_t* __restrict__ payload,
                                                         const uint64_t* __restrict__ offsets,
                                                         const uint2* __restrict__ rowinfo, float* __restrict__ out,
                                                         int blocked, const void* __restrict__ orig,
                                                         double* __restrict__ part,
                                                         const uint32_t* __restrict__ npairs) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    uint32_t G = gridDim.x, t = blockIdx.x, tend = ntiles;
    if (blocked) {
        const uint32_t per = (ntiles + gridDim.x - 1) / gridDim.x;
        t = blockIdx.x * per;
        tend = min(ntiles, t + per);
        G = 1;
    }
    if (t >= tend) return;

    // prologue: tile t's ranges and pairs in flight, tile t + G's row entries
    RTile T = tiles[t];
    uint32_t np;
    const uint2* pr = rix_payload(payload, offsets, npairs, T, np);
    RixRange R = rix_load_range(T, rowinfo, w, l);
    RixPlan PL = rix_plan(T, R, np, l);
    // prefetch slots, one per range (a wave owns at most 16 ranges at the
    // default WC_OPT_RIX_TX); the RMSE sums need registers
    constexpr int NR = OT == 1   ? kRixRounds - WC_RIX_RMSE_ROUNDS_LESS
                       : OT != 0 ? kRixRounds - WC_RIX_RMSE_PASS_ROUNDS_LESS
                                 : kRixRounds;
    uint2 q[NR];
    rix_prefetch<NR>(q, pr, R, PL, T, l);
    uint32_t t1 = t + G;
    RTile T1 = T;
    RixRange R1{0u, 0u, 0u};
    const uint2* pr1 = pr;
    uint32_t np1 = 0;
    if (t1 < tend) {
        T1 = tiles[t1];
        pr1 = rix_payload(payload, offsets, npairs, T1, np1);
        R1 = rix_load_range(T1, rowinfo, w, l);
    }

    for (;;) {
        const int TX = 1 << T.lbx, RS = rix_rs(T.lby, T.D);
        const int WR = rix_wr(T.lbx, T.lby, T.D);
        const uint32_t rlen = (uint32_t)(T.tyv * T.D);
        float* reg = lds + w * WR;
        // 1. zero the wave's region, scatter its pairs
        {
            float4* r4 = reinterpret_cast<float4*>(reg);
            const uint32_t n4 = (uint32_t)(TX * RS) >> 2;
            for (uint32_t i = l; i < n4; i += 64) r4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int j = 0; j < NR; ++j)
                if (j < TX) rix_scatter_range(reg, RS, rlen, q[j], true, pr, R, PL, l, j);
            for (int j = NR; j < TX; ++j) rix_scatter_range(reg, RS, rlen, q[0], false, pr, R, PL, l, j);
        }
        __syncthreads();

        // 2. prefetch: tile t1's pairs, tile t2's row entries
        const uint32_t t2 = t1 + G;
        RTile T2 = T1;
        RixRange R2{0u, 0u, 0u};
        const uint2* pr2 = pr1;
        uint32_t np2 = 0;
        RixPlan PL1{0u};
        if (t1 < tend) {
            PL1 = rix_plan(T1, R1, np1, l);
            rix_prefetch<NR>(q, pr1, R1, PL1, T1, l);
            if (t2 < tend) {
                T2 = tiles[t2];
                pr2 = rix_payload(payload, offsets, npairs, T2, np2);
                R2 = rix_load_range(T2, rowinfo, w, l);
            }
        }

        // 3. synthesis of tile t
        bool f4 = false;
        double racc = 0.0;  // fused RMSE of the x-quad path: this thread's squared differences
        {
            const int lbx = T.lbx, TYv = T.tyv;
            const int W = T.W, H = T.H, D = T.D, hx = W >> 1, hz = D >> 1;
            float* __restrict__ dst = out + T.cell_off;
            const int64_t sy = W, sz = (int64_t)W * H;
            const int64_t lo = (int64_t)(T.bx0 * 2);
            // x-quad (16-B) stores where the output allows them (uniform: out 16-B aligned)
            f4 = TX >= 2 && ((T.cell_off & 3) == 0) && ((W & 3) == 0);
            if (f4) {
                // two x-blocks x two z-blocks per thread: 16-B x-quad stores
                const int nq = (TX >> 1) * TYv * (hz >> 1);
                for (int ci = tid; ci < nq; ci += kThreads) {
                    const int bp = ci & ((TX >> 1) - 1), rest = ci >> (lbx - 1);
                    const int byl = rest % TYv, bq = rest / TYv;
                    const int bxl = 2 * bp, by = T.by0 + byl, bzb = 2 * bq;
                    if (T.bx0 + bxl >= hx) continue;
                    // fused RMSE (OT 1, fp64 originals: summed inside this synthesis, no
                    // re-read of the output): the original cells of z-block
                    // pair qb = 0, issued before the LDS reads (qb = 1: after qb 0)
                    float og[2][2][2][4];  // [qb][dz][dy][4 x-cells], original cells narrowed to float
                    if constexpr (OT == 1)
                        rix_load_orig<OT>(orig, T.cell_off + lo + 2 * bxl + sy * (2 * by) + sz * (2 * bzb), sy, sz, og[0]);
                    float c[2][2][2][2][2];  // [x-block][sz][sy][sx][z-block]
#pragma unroll
                    for (int e = 0; e < 2; ++e)
#pragma unroll
                        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                            for (int t3 = 0; t3 < 2; ++t3)
#pragma unroll
                                for (int x = 0; x < 2; ++x) {
                                    const int g = ((x * 2 + t3) << lbx) + bxl + e;
                                    const float2 v2 = *reinterpret_cast<const float2*>(
                                        lds + (g & 3) * WR + (g >> 2) * RS + byl * D + s2 * hz + bzb);
                                    c[e][s2][t3][x][0] = v2.x;
                                    c[e][s2][t3][x][1] = v2.y;
                                }
#pragma unroll
                    for (int qb = 0; qb < 2; ++qb) {
                        float V[2][2][2][2];  // [x-block][dz][dy][dx]
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            float cb[2][2][2];
#pragma unroll
                            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                                for (int t3 = 0; t3 < 2; ++t3)
#pragma unroll
                                    for (int x = 0; x < 2; ++x) cb[s2][t3][x] = c[e][s2][t3][x][qb];
                            synth_block(cb, V[e]);
                        }
#pragma unroll
                        for (int dz = 0; dz < 2; ++dz)
#pragma unroll
                            for (int dy = 0; dy < 2; ++dy) {
                                float* p = dst + lo + 2 * bxl + sy * (2 * by + dy) + sz * (2 * (bzb + qb) + dz);
                                // nontemporal where no RMSE pass re-reads the output (OT 2, 3 re-read it
                                // from L2): K6r -9 % at C2, -6 % at C3 (profiles/r05/experiments/gpu_nt.txt)
                                if constexpr (OT <= 1) {
                                    const f32x4 x = {V[0][dz][dy][0], V[0][dz][dy][1], V[1][dz][dy][0],
                                                     V[1][dz][dy][1]};
                                    __builtin_nontemporal_store(x, reinterpret_cast<f32x4*>(p));
                                } else {
                                    *reinterpret_cast<float4*>(p) = make_float4(V[0][dz][dy][0], V[0][dz][dy][1],
                                                                                V[1][dz][dy][0], V[1][dz][dy][1]);
                                }
                            }
                        if constexpr (OT == 1) {
                            if (qb == 0)  // the second z-block pair's originals, in flight during this one's sums
                                rix_load_orig<OT>(orig, T.cell_off + lo + 2 * bxl + sy * (2 * by) + sz * (2 * (bzb + 1)),
                                                  sy, sz, og[1]);
#pragma unroll
                            for (int dz = 0; dz < 2; ++dz)
#pragma unroll
                                for (int dy = 0; dy < 2; ++dy) {
                                    const float v[4] = {V[0][dz][dy][0], V[0][dz][dy][1], V[1][dz][dy][0],
                                                        V[1][dz][dy][1]};
#pragma unroll
                                    for (int k = 0; k < 4; ++k) {
                                        const float d = og[qb][dz][dy][k] - v[k];  // float - float, then widened
                                        racc += (double)d * (double)d;
                                    }
                                }
                        }
                    }
                }
            } else {
                const bool vout = (T.cell_off & 1) == 0;
                const int ncol = TX * TYv * (hz >> 2);
                for (int ci = tid; ci < ncol; ci += kThreads) {
                    const int bxl = ci & (TX - 1), rest = ci >> lbx;
                    const int byl = rest % TYv, bq = rest / TYv;
                    const int bx = T.bx0 + bxl, by = T.by0 + byl, bzb = 4 * bq;
                    if (bx >= hx) continue;
                    float c[2][2][2][4];  // [sz][sy][sx][z-block]
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                        for (int t3 = 0; t3 < 2; ++t3)
#pragma unroll
                            for (int x = 0; x < 2; ++x) {
                                const int g = ((x * 2 + t3) << lbx) + bxl;
                                const float4 v4 = *reinterpret_cast<const float4*>(lds + (g & 3) * WR + (g >> 2) * RS +
                                                                                   byl * D + s2 * hz + bzb);
                                c[s2][t3][x][0] = v4.x;
                                c[s2][t3][x][1] = v4.y;
                                c[s2][t3][x][2] = v4.z;
                                c[s2][t3][x][3] = v4.w;
                            }
#pragma unroll
                    for (int qb = 0; qb < 4; ++qb) {
                        float cb[2][2][2], V[2][2][2];
#pragma unroll
                        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                            for (int t3 = 0; t3 < 2; ++t3)
#pragma unroll
                                for (int x = 0; x < 2; ++x) cb[s2][t3][x] = c[s2][t3][x][qb];
                        synth_block(cb, V);
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
        }
        __syncthreads();
        if constexpr (OT == 1) {
            if (f4) {  // uniform: the x-quad synthesis summed its own cells
                const double acc = wave_sum(racc);
                if (l == 0) part[4 * (uint64_t)T.nat + w] = acc;
            }
        }
        if constexpr (OT != 0) if (!(OT == 1 && f4)) {  // 4. calc_rmse_per_box over tile t's cells (src/calc-loss.cpp:12-43)
            const int TX = 1 << T.lbx, txv = min(TX, (T.W >> 1) - T.bx0), ny2 = 2 * T.tyv;
            const uint32_t nc = (uint32_t)(T.D * ny2) << T.lbx;
            const int64_t sy = T.W, sz = (int64_t)T.W * T.H;
            const int64_t lo = T.cell_off + 2 * (int64_t)T.bx0 + 2 * (int64_t)T.by0 * sy;
            double acc = 0.0;
            for (uint32_t ci = tid; ci < nc; ci += kThreads) {
                const int x = (int)(ci & (uint32_t)(TX - 1));
                if (x >= txv) continue;
                const uint32_t row = ci >> T.lbx;
                const int64_t i = lo + 2 * x + sy * (int64_t)(row % (uint32_t)ny2) + sz * (int64_t)(row / (uint32_t)ny2);
                float o0, o1;
                if constexpr (OT == 1 || OT == 3) {
                    o0 = (float)((const double*)orig)[i];
                    o1 = (float)((const double*)orig)[i + 1];
                } else {
                    o0 = ((const float*)orig)[i];
                    o1 = ((const float*)orig)[i + 1];
                }
                const float d0 = o0 - out[i], d1 = o1 - out[i + 1];  // float - float, then widened
                acc += (double)d0 * (double)d0;
                acc += (double)d1 * (double)d1;
            }
            acc = wave_sum(acc);
            if (l == 0) part[4 * (uint64_t)T.nat + w] = acc;
        }
        if (t1 >= tend) break;
        T = T1;
        pr = pr1;
        R = R1;
        PL = PL1;
        t = t1;
        t1 = t2;
        T1 = T2;
        pr1 = pr2;
        np1 = np2;
        R1 = R2;
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
    // uniform: cell pairs, one vector load each (read once: nontemporal), where both are pair-aligned
    if ((reinterpret_cast<uintptr_t>(a) % (2 * sizeof(T))) == 0 && (reinterpret_cast<uintptr_t>(b) & 7u) == 0) {
        const int n2 = (int)(len >> 1);
        for (int i = threadIdx.x; i < n2; i += kThreads) {
            float o0, o1;
            load_xpair<T, true>(a + 2 * i, true, true, o0, o1);
            const f32x2 r = __builtin_nontemporal_load(reinterpret_cast<const f32x2*>(b + 2 * i));
            const float d0 = o0 - r.x, d1 = o1 - r.y;  // float - float, then widened
            s += (double)d0 * (double)d0;
            s += (double)d1 * (double)d1;
        }
        if ((len & 1) && threadIdx.x == 0) {
            const float d = (float)a[len - 1] - b[len - 1];
            s += (double)d * (double)d;
        }
    } else {
        for (int i = threadIdx.x; i < len; i += kThreads) {
            const float d = (float)a[i] - b[i];
            const double dd = d;
            s += dd * dd;
        }
    }
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = ((s_w[0] + s_w[1]) + s_w[2]) + s_w[3];
}

__global__ __launch_bounds__(64) void k_rmse_final(const UnitDev* __restrict__ units, int /*n*/,
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
// Workgroups of a kernel resident at once (persistent grids).
static uint32_t resident_grid(const void* fn, size_t lds) {
    int per_cu = 0, ncu = 0, dev = 0;
    (void)hipGetDevice(&dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kThreads, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1) ncu = 256;
    return (uint32_t)per_cu * (uint32_t)ncu;
}

// The pair count of every unit's payload, checked against the unit (the row
// index of wc_inverse_rows comes from the caller, so k_rowindex, which checks
// the headers otherwise, does not run): npairs[u] = nrle, or 0 and kErrHeader
// for a header that disagrees (read_header).
__global__ __launch_bounds__(kThreads) void k_pair_counts(const UnitDev* __restrict__ units, int n,
                                                        const uint8_t* __restrict__ payload,
                                                        const uint64_t* __restrict__ offsets,
                                                        uint32_t* __restrict__ npairs, uint32_t* __restrict__ err) {
    const int u = blockIdx.x * kThreads + threadIdx.x;
    if (u >= n) return;
    const UnitDev& U = units[u];
    if (!U.rix) return;
    int32_t nrle;
    const bool ok = read_header(U, payload + offsets[u], nrle);
    npairs[u] = ok ? (uint32_t)nrle : 0u;
    if (!ok) atomicOr(err, kErrHeader);
}

hipError_t launch_pair_counts(hipStream_t st, const UnitDev* units, int n, const uint8_t* payload,
                              const uint64_t* offsets, uint32_t* npairs, uint32_t* err) {
    k_pair_counts<<<(n + kThreads - 1) / kThreads, kThreads, 0, st>>>(units, n, payload, offsets, npairs, err);
    return hipGetLastError();
}

// K5.  Row-indexed units: the row index (epoch-tagged granules istate at
// dt_begin, never zeroed per call).  Other units: the dense decode (zeroed
// ticket / status).
hipError_t launch_decode(hipStream_t st, const UnitDev* units, const FTile* ftiles, uint32_t nft,
                         const FTile* rtiles, uint32_t nrt, unsigned long long* istate, uint32_t epoch,
                         const uint8_t* payload, const uint64_t* offsets, uint32_t* ticket,
                         unsigned long long* status, float* flat, uint2* rowinfo, uint32_t* err, int ordered,
                         uint32_t* npairs) {
    if (nrt)
        k_rowindex<<<nrt, kThreads, 0, st>>>(units, rtiles, ticket, payload, offsets, istate, rowinfo, err, ordered,
                                             epoch, npairs);
    if (nft) k_decode<<<nft, kThreads, 0, st>>>(units, ftiles, payload, offsets, ticket, status, flat, err, ordered);
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

// Workgroups of k_inverse_rows resident at once for `lds` bytes on the current
// device (persistent grid; the caller caches it per context and LDS size).
uint32_t inverse_rows_grid(size_t lds) { return resident_grid((const void*)k_inverse_rows<0>, lds); }

// calc_rmse_per_box of the fused form: unit u's K6r tile sums in tile order.
__global__ __launch_bounds__(64) void k_rmse_rows_final(const UnitDev* __restrict__ units,
                                                       const double* __restrict__ part, double* __restrict__ rmse) {
    const UnitDev& U = units[blockIdx.x];
    double s = 0.0;
    for (uint32_t i = threadIdx.x; i < 4 * U.nrt; i += 64) s += part[4 * (uint64_t)U.rt_begin + i];
    s = wave_sum(s);
    if (threadIdx.x == 0) {
        const int vol = U.nx * U.ny * U.nz;  // int product, as src/calc-loss.cpp:37
        rmse[blockIdx.x] = vol > 0 ? sqrt(s / (double)vol) : 0.0;
    }
}

// orig == null: the inverse alone; else also calc_rmse_per_box against orig
// (dtype 1 fp64, 0 fp32) into rmse[n] via part[ntiles].
// rmse_final: also launch k_rmse_rows_final (after the last group's tiles).
hipError_t launch_inverse_rows(hipStream_t st, const RTile* tiles, uint32_t ntiles, size_t lds, uint32_t max_grid,
                               const uint8_t* payload, const uint64_t* offsets, const uint2* rowinfo, float* out,
                               int blocked, const void* orig, int dtype, const UnitDev* units, int n, double* part,
                               double* rmse, bool rmse_final, const uint32_t* npairs) {
    if (!ntiles) {
        if (orig && rmse_final) k_rmse_rows_final<<<n, 64, 0, st>>>(units, part, rmse);
        return hipGetLastError();
    }
    const uint32_t grid = std::min(ntiles, std::max(1u, max_grid));
    if (!orig)
        k_inverse_rows<0><<<grid, kThreads, lds, st>>>(tiles, ntiles, payload, offsets, rowinfo, out, blocked, orig,
                                                       part, npairs);
    else if (dtype == 1 && ((uintptr_t)orig & 15) == 0)
        k_inverse_rows<1><<<grid, kThreads, lds, st>>>(tiles, ntiles, payload, offsets, rowinfo, out, blocked, orig,
                                                       part, npairs);
    else if (dtype == 1)
        k_inverse_rows<3><<<grid, kThreads, lds, st>>>(tiles, ntiles, payload, offsets, rowinfo, out, blocked, orig,
                                                       part, npairs);
    else
        k_inverse_rows<2><<<grid, kThreads, lds, st>>>(tiles, ntiles, payload, offsets, rowinfo, out, blocked, orig,
                                                       part, npairs);
    if (orig && rmse_final) k_rmse_rows_final<<<n, 64, 0, st>>>(units, part, rmse);
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

// wc_bench — torch-free C++ driver of the C-ABI, for rocprofv3 (--pmc) runs.
//
// Same workload as bench.py (N boxes of D^3, fp64 or fp32, keep 0.999f): the
// synthetic field of SURVEY.md §8(d) is generated on the device (hash-based
// Box-Muller noise), then wc_forward runs `steps` times.  Prints one JSON line.
//
// usage: wc_bench [boxes=1024] [dim=64|c3] [f64|f32] [keep=0.999] [steps=10] [warmup=2] [inverse=0|1|2]
//                 [check=0|1] [ordered=1] [sparse=1] [rows=1] [rix_lds=9216] [rix_tx=4] [rix_blocked=0]
//                 [rix_xcd=0] [inv_groups=1]
// check=1: also run the conservative configuration (ticket look-back, dense
// staging, dense inverse decode) once and compare every unit's payload bytes and, with inverse=1,
// every reconstructed cell ("paths_identical" in the JSON line).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "wavelet_amd.h"

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                    \
        }                                                                                    \
    } while (0)

__device__ inline unsigned long long mix64(unsigned long long z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <typename T>
__global__ void synth(T* out, int dim, long long nboxes, unsigned long long seed) {
    const long long per = (long long)dim * dim * dim;
    const long long total = per * nboxes;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long b = i / per, r = i % per;
        const int x = (int)(r % dim), y = (int)((r / dim) % dim), z = (int)(r / ((long long)dim * dim));
        const double gx = dim * (b % 16) + x, gy = dim * ((b / 16) % 8) + y, gz = dim * (b / 128) + z;
        const unsigned long long h1 = mix64(seed + 0x9E3779B97F4A7C15ull * (2 * i + 1));
        const unsigned long long h2 = mix64(seed + 0x9E3779B97F4A7C15ull * (2 * i + 2));
        const double u1 = ((double)(h1 >> 11) + 1.0) * (1.0 / 9007199254740992.0);
        const double u2 = (double)(h2 >> 11) * (1.0 / 9007199254740992.0);
        const double g = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
        out[i] = (T)(300.0 + 50.0 * sin(0.1 * gx) * cos(0.07 * gy) + 0.01 * gz + 0.05 * g);
    }
}

// per-component field mean and amplitude, as bench_workloads.py COMP_MEAN / COMP_AMP
// (components 3 and 7: negative signed max, the fallback's dense re-staging)
static const double kCompMean[8] = {300.0, 1000.0, 5.0, 0.0, 300.0, 1.0, 50.0, 0.0};
static const double kCompAmp[8] = {50.0, 120.0, 2.0, 40.0, 80.0, 0.5, 10.0, 3.0};

// Every unit of the C3 layout in ONE launch (block row y = unit y; a launch
// per unit made 46 080 dispatches at C4 size, which the counter passes do not
// survive): unit i's field (bench_workloads.py synth_cells: its component's
// mean + amplitude x sin(0.1 gx) cos(0.07 gy) + 0.01 gz + N(0, 0.05)) at its
// box origin.
struct SynthUnit {
    unsigned long long off;
    int W, H, D, gx, gy, gz;  // dims, origin
    double mean, amp;         // the component's (host-side table)
};
template <typename T>
__global__ void synth_units(T* out, const SynthUnit* units, unsigned long long seed0) {
    const SynthUnit u = units[blockIdx.y];
    const int i = (int)blockIdx.y;
    const int gx0 = u.gx, gy0 = u.gy, gz0 = u.gz;
    const double mean = u.mean, amp = u.amp;
    const unsigned long long seed = seed0 + (unsigned long long)i;
    const long long total = (long long)u.W * u.H * u.D;
    for (long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x; c < total;
         c += (long long)gridDim.x * blockDim.x) {
        const int x = (int)(c % u.W), y = (int)((c / u.W) % u.H), z = (int)(c / ((long long)u.W * u.H));
        const double gx = gx0 + x, gy = gy0 + y, gz = gz0 + z;
        const unsigned long long h1 = mix64(seed + 0x9E3779B97F4A7C15ull * (2 * c + 1));
        const unsigned long long h2 = mix64(seed + 0x9E3779B97F4A7C15ull * (2 * c + 2));
        const double u1 = ((double)(h1 >> 11) + 1.0) * (1.0 / 9007199254740992.0);
        const double u2 = (double)(h2 >> 11) * (1.0 / 9007199254740992.0);
        const double g = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
        out[u.off + c] = (T)(mean + amp * sin(0.1 * gx) * cos(0.07 * gy) + 0.01 * gz + 0.05 * g);
    }
}

// BASELINE configs[2] (C3) layout, SURVEY §8(d): L0 64 x 64^3, L1 96 x 64^3,
// L2 128 x 32^3, L3 256 x 16^3 + 32 x (48 x 32 x 16), `ncomp` units per box
// (c: component c % 8 of timestep c / 8, so 80 = C4's 10 timesteps x 8
// components).  Box origins as bench_workloads.py amr_levels (per level: boxes
// on a per_row x per_plane grid, the slabs from z 256), timestep t shifted 3t
// in x; `lo` gets each unit's origin.
// WCB_C3_MASK (diagnostic): bit g keeps group g of the five (L0, L1, L2, L3 cubes, L3 slabs).
struct Origin {
    int x, y, z;
};
static std::vector<wc_unit> c3_layout(int ncomp, std::vector<Origin>& lo) {
    std::vector<wc_unit> u;
    uint64_t off = 0;
    const char* me = std::getenv("WCB_C3_MASK");
    const int mask = me ? std::atoi(me) : 31;
    int group = 0;
    auto add = [&](int n, int W, int H, int D, int per_row, int per_plane, int z0) {
        if (!((mask >> group++) & 1)) return;
        for (int b = 0; b < n; ++b)
            for (int c = 0; c < ncomp; ++c) {
                u.push_back(wc_unit{off, W, H, D, 0});
                lo.push_back(Origin{(b % per_row) * W + 3 * (c / 8), ((b / per_row) % per_plane) * H,
                                    (b / (per_row * per_plane)) * D + z0});
                off += ((uint64_t)W * H * D + 3) & ~3ull;
            }
    };
    add(64, 64, 64, 64, 4, 4, 0);
    add(96, 64, 64, 64, 6, 4, 0);
    add(128, 32, 32, 32, 8, 4, 0);
    add(256, 16, 16, 16, 8, 8, 0);
    add(32, 48, 32, 16, 4, 4, 256);
    return u;
}

int main(int argc, char** argv) {
    // boxes/dim: N cubes of dim^3; dim "c3": the C3 layout with `boxes` components (4 in bench.py)
    const bool c3 = argc > 2 && std::strcmp(argv[2], "c3") == 0;
    const int boxes_arg = argc > 1 ? std::atoi(argv[1]) : 1024;
    const int dim = c3 ? 0 : (argc > 2 ? std::atoi(argv[2]) : 64);
    const bool f64 = argc > 3 ? std::strcmp(argv[3], "f32") != 0 : true;
    const double keep = (double)(float)(argc > 4 ? std::atof(argv[4]) : 0.999);
    const int steps = argc > 5 ? std::atoi(argv[5]) : 10;
    const int warmup = argc > 6 ? std::atoi(argv[6]) : 2;
    // 1 wc_inverse, 2 wc_inverse_rmse (fused calc_rmse_per_box), 3 the round trip with the forward's row
    // index (wc_forward_rows + wc_inverse_rows with the RMSE), 7 wc_inverse + wc_rmse (the separate calls)
    const int inv_mode = argc > 7 ? std::atoi(argv[7]) : 0;
    const bool inverse = inv_mode != 0;
    const bool check = argc > 8 ? std::atoi(argv[8]) != 0 : false;
    const int ordered = argc > 9 ? std::atoi(argv[9]) : 1;
    const int sparse = argc > 10 ? std::atoi(argv[10]) : 1;
    const int rows = argc > 11 ? std::atoi(argv[11]) : 1;
    const int rix_lds = argc > 12 ? std::atoi(argv[12]) : 9216;
    const int rix_tx = argc > 13 ? std::atoi(argv[13]) : 4;
    const int rix_blocked = argc > 14 ? std::atoi(argv[14]) : 0;
    const int rix_xcd = argc > 15 ? std::atoi(argv[15]) : 0;
    const int inv_groups = argc > 16 ? std::atoi(argv[16]) : 1;

    std::vector<wc_unit> units;
    std::vector<Origin> origins;
    if (c3) {
        units = c3_layout(boxes_arg, origins);
    } else {
        const unsigned long long per = (unsigned long long)dim * dim * dim;
        for (int i = 0; i < boxes_arg; ++i) units.push_back(wc_unit{per * i, dim, dim, dim, 0});
    }
    const int boxes = (int)units.size();
    const unsigned long long ncells = wc_cell_count(units.data(), boxes);
    const unsigned long long extent = units.back().cell_offset +
                                      (unsigned long long)units.back().nx * units.back().ny * units.back().nz;
    const size_t esz = f64 ? 8 : 4;
    void* cells = nullptr;
    CK(hipMalloc(&cells, esz * extent));
    if (c3) {
        std::vector<SynthUnit> su(boxes);
        for (int i = 0; i < boxes; ++i)
            su[i] = SynthUnit{units[i].cell_offset, units[i].nx, units[i].ny, units[i].nz, origins[i].x,
                              origins[i].y, origins[i].z, kCompMean[(i % boxes_arg) % 8],
                              kCompAmp[(i % boxes_arg) % 8]};
        SynthUnit* d_su = nullptr;
        CK(hipMalloc(&d_su, sizeof(SynthUnit) * boxes));
        CK(hipMemcpy(d_su, su.data(), sizeof(SynthUnit) * boxes, hipMemcpyHostToDevice));
        const dim3 grid(64, (unsigned)boxes);
        if (f64)
            synth_units<double><<<grid, 256>>>((double*)cells, d_su, 1234);
        else
            synth_units<float><<<grid, 256>>>((float*)cells, d_su, 1234);
        CK(hipDeviceSynchronize());
        CK(hipFree(d_su));
    } else if (f64) {
        synth<double><<<4096, 256>>>((double*)cells, dim, boxes, 1234);
    } else {
        synth<float><<<4096, 256>>>((float*)cells, dim, boxes, 1234);
    }
    CK(hipDeviceSynchronize());

    const uint64_t cap = wc_payload_bound(units.data(), boxes);
    uint8_t* payload = nullptr;
    uint64_t* offsets = nullptr;
    uint32_t* kept = nullptr;
    float* regen = nullptr;
    CK(hipMalloc(&payload, cap));
    CK(hipMalloc(&offsets, 8 * (2 * boxes + 1)));
    CK(hipMalloc(&kept, 4 * boxes));
    double* rmse = nullptr;
    if (inverse) CK(hipMalloc(&regen, 4 * extent));
    if (inv_mode >= 2) CK(hipMalloc(&rmse, 8 * boxes));
    void* rowinfo = nullptr;
    const uint64_t rowinfo_bytes = wc_rowindex_bytes(units.data(), boxes);
    // 4 (diagnostic): wc_forward_rows, then wc_inverse_rows WITHOUT the row index (the
    // row index kernel runs); 5: wc_inverse, then wc_inverse_rows with it, per step;
    // 6: wc_forward_rows + wc_inverse_rows without the RMSE
    if (inv_mode >= 3) CK(hipMalloc(&rowinfo, rowinfo_bytes));

    wc_ctx* ctx = nullptr;
    if (wc_ctx_create(0, &ctx) != WC_OK) {
        std::fprintf(stderr, "wc_ctx_create failed\n");
        return 2;
    }
    wc_set_option(ctx, WC_OPT_ORDERED, ordered);
    wc_set_option(ctx, WC_OPT_SPARSE, sparse);
    wc_set_option(ctx, WC_OPT_INVERSE_ROWS, rows);
    if (wc_set_option(ctx, WC_OPT_RIX_LDS, rix_lds) != WC_OK || wc_set_option(ctx, WC_OPT_RIX_TX, rix_tx) != WC_OK ||
        wc_set_option(ctx, WC_OPT_RIX_BLOCKED, rix_blocked) != WC_OK || wc_set_option(ctx, WC_OPT_RIX_XCD, rix_xcd) != WC_OK) {
        std::fprintf(stderr, "options: %s\n", wc_last_error(ctx));
        return 2;
    }
    // WCB_CHUNK=k (uniform cubes only, diagnostic): the forward as boxes/k calls of k
    // units each (same unit list, cells/payload pointers advanced per call), so the
    // context's coefficient staging is one k-unit buffer reused by every call.
    const char* chunk_env = std::getenv("WCB_CHUNK");
    const int chunk = (!c3 && chunk_env) ? std::atoi(chunk_env) : 0;
    // WCB_HIST=q: the opt-in global-threshold mode at quantile q (bench.py's c4
    // global_hist leg): wc_forward_stage with the histogram, its threshold on
    // the host (one rank: no all-reduce), wc_forward_emit with it.
    const char* hist_env = std::getenv("WCB_HIST");
    const double hist_q = hist_env ? std::atof(hist_env) : -1.0;
    uint64_t* d_hist = nullptr;
    std::vector<uint64_t> h_hist(WC_HIST_BINS);
    if (hist_q >= 0.0) CK(hipMalloc(&d_hist, 8 * WC_HIST_BINS));
    // WCB_SPLIT=us (diagnostic): the reference rule as wc_forward_stage + wc_synchronize + an idle
    // gap of `us` microseconds on the host + wc_forward_emit (stage + emit == wc_forward): does
    // the emit's time depend on how long ago K1 finished?
    const char* split_env = std::getenv("WCB_SPLIT");
    const int split_us = split_env ? std::atoi(split_env) : -1;
    auto fwd = [&]() {
        int rc = WC_OK;
        if (split_us >= 0 && hist_q < 0.0) {
            if ((rc = wc_forward_stage(ctx, cells, f64 ? WC_F64 : WC_F32, units.data(), boxes, nullptr)) == WC_OK &&
                (rc = wc_synchronize(ctx)) == WC_OK) {
                const auto t0 = std::chrono::steady_clock::now();
                while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() <
                       split_us) {
                }
                rc = wc_forward_emit(ctx, units.data(), boxes, keep, nullptr, payload, cap, offsets, kept);
            }
        } else if (hist_q >= 0.0) {
            float t = 0.0f;
            CK(hipMemset(d_hist, 0, 8 * WC_HIST_BINS));
            if ((rc = wc_forward_stage(ctx, cells, f64 ? WC_F64 : WC_F32, units.data(), boxes, d_hist)) == WC_OK &&
                (rc = wc_synchronize(ctx)) == WC_OK) {
                CK(hipMemcpy(h_hist.data(), d_hist, 8 * WC_HIST_BINS, hipMemcpyDeviceToHost));
                wc_hist_threshold(h_hist.data(), hist_q, &t, nullptr);
                rc = wc_forward_emit(ctx, units.data(), boxes, keep, &t, payload, cap, offsets, kept);
            }
        } else if (chunk > 0 && chunk < boxes && boxes % chunk == 0) {
            const uint64_t per = (uint64_t)dim * dim * dim;
            const uint64_t ccap = wc_payload_bound(units.data(), chunk);
            for (int g = 0; g < boxes / chunk && rc == WC_OK; ++g)
                rc = wc_forward(ctx, (uint8_t*)cells + esz * per * chunk * g, f64 ? WC_F64 : WC_F32, units.data(),
                                chunk, keep, payload + ccap * g, ccap, offsets + (chunk + 1) * g, kept + chunk * g);
        } else {
            rc = rowinfo ? wc_forward_rows(ctx, cells, f64 ? WC_F64 : WC_F32, units.data(), boxes, keep, payload, cap,
                                           offsets, kept, rowinfo, rowinfo_bytes)
                         : wc_forward(ctx, cells, f64 ? WC_F64 : WC_F32, units.data(), boxes, keep, payload, cap,
                                      offsets, kept);
        }
        if (rc != WC_OK) {
            std::fprintf(stderr, "wc_forward: %s\n", wc_last_error(ctx));
            std::exit(2);
        }
    };
    // WCB_TOUCH=payload|rows (diagnostic, inverse_mode 3): before each inverse, a
    // device-to-device copy that streams the payloads (or the row index) through
    // the caches, on the context's stream: does K6r wait on those reads?
    const char* touch = std::getenv("WCB_TOUCH");
    hipStream_t tstream = nullptr;
    void* tbuf = nullptr;
    if (touch) {
        CK(hipStreamCreate(&tstream));
        wc_set_stream(ctx, tstream);
        CK(hipMalloc(&tbuf, std::max<uint64_t>(cap, rowinfo_bytes)));
    }
    auto inv = [&]() {
        if (touch && std::strcmp(touch, "payload") == 0) CK(hipMemcpyAsync(tbuf, payload, cap, hipMemcpyDeviceToDevice, tstream));
        if (touch && std::strcmp(touch, "rows") == 0 && rowinfo)
            CK(hipMemcpyAsync(tbuf, rowinfo, rowinfo_bytes, hipMemcpyDeviceToDevice, tstream));
        if (inv_mode == 5 && wc_inverse(ctx, payload, offsets, units.data(), boxes, regen) != WC_OK) std::exit(2);
        if (inv_mode == 7) {
            if (wc_inverse(ctx, payload, offsets, units.data(), boxes, regen) != WC_OK ||
                wc_rmse(ctx, cells, f64 ? WC_F64 : WC_F32, regen, units.data(), boxes, rmse) != WC_OK) {
                std::fprintf(stderr, "wc_inverse + wc_rmse: %s\n", wc_last_error(ctx));
                std::exit(2);
            }
            return;
        }
        int rc = inv_mode == 3   ? wc_inverse_rows(ctx, payload, offsets, units.data(), boxes, rowinfo, rowinfo_bytes, cells,
                                                   f64 ? WC_F64 : WC_F32, regen, rmse)
                 : inv_mode == 4 ? wc_inverse_rows(ctx, payload, offsets, units.data(), boxes, nullptr, 0, cells,
                                                   f64 ? WC_F64 : WC_F32, regen, rmse)
                 : inv_mode == 5 || inv_mode == 6
                                 ? wc_inverse_rows(ctx, payload, offsets, units.data(), boxes, rowinfo, rowinfo_bytes, nullptr,
                                                   WC_F32, regen, nullptr)
                 : inv_mode == 2 ? wc_inverse_rmse(ctx, payload, offsets, units.data(), boxes, cells,
                                                   f64 ? WC_F64 : WC_F32, regen, rmse)
                                 : wc_inverse(ctx, payload, offsets, units.data(), boxes, regen);
        if (rc != WC_OK) {
            std::fprintf(stderr, "wc_inverse: %s\n", wc_last_error(ctx));
            std::exit(2);
        }
    };
    for (int i = 0; i < warmup; ++i) {
        fwd();
        if (inverse) inv();
    }
    wc_synchronize(ctx);
    wc_profile_enable(ctx, 1);
    double ms[WC_NUM_STAGES];
    uint32_t cnt[WC_NUM_STAGES];
    wc_profile_read(ctx, ms, cnt, WC_NUM_STAGES);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < steps; ++i) fwd();
    wc_synchronize(ctx);
    auto t1 = std::chrono::steady_clock::now();
    wc_profile_read(ctx, ms, cnt, WC_NUM_STAGES);
    double inv_ms = 0;
    double ims[WC_NUM_STAGES];
    uint32_t icnt[WC_NUM_STAGES];
    if (inverse) {
        auto a = std::chrono::steady_clock::now();
        for (int i = 0; i < steps; ++i) inv();
        wc_synchronize(ctx);
        auto b = std::chrono::steady_clock::now();
        inv_ms = std::chrono::duration<double, std::milli>(b - a).count() / steps;
        wc_profile_read(ctx, ims, icnt, WC_NUM_STAGES);
    }
    const double step_ms = std::chrono::duration<double, std::milli>(t1 - t0).count() / steps;
    int identical = -1;
    if (check) {
        // Configured path vs the conservative one (ticket look-back, dense
        // staging): every unit's serialized bytes and reconstructed cells.
        std::vector<uint64_t> off_a(boxes + 1), off_b(boxes + 1);
        std::vector<uint32_t> k_a(boxes), k_b(boxes);
        std::vector<uint8_t> pa(cap), pb(cap);
        std::vector<float> ra, rb;
        auto run = [&](std::vector<uint64_t>& off, std::vector<uint32_t>& k, std::vector<uint8_t>& pl,
                       std::vector<float>& rg) {
            CK(hipMemset(payload, 0xA5, cap));
            fwd();
            if (inverse) {
                CK(hipMemset(regen, 0xA5, 4 * extent));
                inv();
            }
            if (wc_synchronize(ctx) != WC_OK) {
                std::fprintf(stderr, "check: %s\n", wc_last_error(ctx));
                std::exit(2);
            }
            CK(hipMemcpy(off.data(), offsets, 8 * (boxes + 1), hipMemcpyDeviceToHost));
            CK(hipMemcpy(k.data(), kept, 4 * boxes, hipMemcpyDeviceToHost));
            CK(hipMemcpy(pl.data(), payload, cap, hipMemcpyDeviceToHost));
            if (inverse) {
                rg.resize(extent);
                CK(hipMemcpy(rg.data(), regen, 4 * extent, hipMemcpyDeviceToHost));
            }
        };
        run(off_a, k_a, pa, ra);
        wc_set_option(ctx, WC_OPT_ORDERED, 0);
        wc_set_option(ctx, WC_OPT_SPARSE, 0);
        wc_set_option(ctx, WC_OPT_INVERSE_ROWS, 0);
        run(off_b, k_b, pb, rb);
        wc_set_option(ctx, WC_OPT_ORDERED, ordered);
        wc_set_option(ctx, WC_OPT_SPARSE, sparse);
        wc_set_option(ctx, WC_OPT_INVERSE_ROWS, rows);
        identical = 1;
        for (int i = 0; i < boxes && identical; ++i) {
            if (k_a[i] != k_b[i] || off_a[i] != off_b[i]) identical = 0;
            else if (std::memcmp(pa.data() + off_a[i], pb.data() + off_b[i], 20 + 8ull * k_a[i]) != 0) identical = 0;
        }
        if (inverse && identical && std::memcmp(ra.data(), rb.data(), 4 * ra.size()) != 0) identical = 0;
    }
    uint64_t total = 0;
    CK(hipMemcpy(&total, offsets + boxes, 8, hipMemcpyDeviceToHost));
    std::vector<uint32_t> hk(boxes);
    CK(hipMemcpy(hk.data(), kept, 4 * boxes, hipMemcpyDeviceToHost));
    double ksum = 0;
    for (uint32_t k : hk) ksum += k;
    const char* names[WC_NUM_STAGES] = {"transform", "emit", "decode", "inverse", "rmse", "hist", "pairs"};
    std::printf("{\"boxes\": %d, \"dim\": %d, \"dtype\": \"%s\", \"keep\": %.17g, \"steps\": %d, "
                "\"ms_per_step\": %.4f, \"cells_per_s\": %.6e, \"kept_fraction\": %.6f, \"payload_bytes\": %llu, "
                "\"ordered\": %d, \"sparse\": %d, \"rows\": %d, \"rix\": [%d, %d, %d], \"paths_identical\": %d, \"stage_ms\": {",
                boxes, dim, f64 ? "f64" : "f32", keep, steps, step_ms, ncells / (step_ms * 1e-3),
                ksum / (double)ncells, (unsigned long long)total, ordered, sparse, rows, rix_lds, rix_tx, rix_blocked, identical);
    bool first = true;
    for (int s = 0; s < WC_NUM_STAGES; ++s)
        if (cnt[s]) {
            std::printf("%s\"%s\": %.4f", first ? "" : ", ", names[s], ms[s] / cnt[s]);
            first = false;
        }
    if (inverse) {
        std::printf("}, \"inverse_ms_per_step\": %.4f, \"inverse_stage_ms\": {", inv_ms);
        first = true;
        for (int s = 0; s < WC_NUM_STAGES; ++s)
            if (icnt[s]) {
                std::printf("%s\"%s\": %.4f", first ? "" : ", ", names[s], ims[s] / icnt[s]);
                first = false;
            }
    }
    std::printf("}");
    std::printf("}\n");
    wc_ctx_destroy(ctx);
    (void)hipFree(cells);
    (void)hipFree(payload);
    (void)hipFree(offsets);
    (void)hipFree(kept);
    if (regen) (void)hipFree(regen);
    if (rmse) (void)hipFree(rmse);
    if (d_hist) (void)hipFree(d_hist);
    if (rowinfo) (void)hipFree(rowinfo);
    return 0;
}

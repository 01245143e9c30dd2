// dropin_bench — the literal drop-in path (INTEGRATION.md Option A): the
// reference's own per-box loops calling the C++ mirror of its interface.
//
//   -c: for every (level, box) of the C3 layout, in the reference's order
//       (src/modes.cpp:100-103): compress(multiBox3D of ncomp fp32 Box3D,
//       components, keep, t, level, box, dir) -> GPU transform + threshold +
//       pack (one wc_forward_host_units call per box), the components' xz
//       streams at the current preset, one file per component;
//   -d: decompress(file) for every file (src/modes.cpp:151-166);
//   GPU stage alone: the same per-box wc_forward_host_units call without the
//       xz stage and the files (what compress() spends outside liblzma);
//   -c with write-behind (opt-in): the same loop, files queued to the xz
//       workers, flushed after it, compared byte for byte with the first pass.
// Prints one JSON line.  Benchmark tool: links only the product libraries.
//
// usage: dropin_bench <scratch dir> [ncomp=4] [keep=0.999] [boxes per level: all]
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <iterator>
#include <string>
#include <thread>
#include <vector>

#include "wavelet_amd.h"
#include "wavelet_amd/compressor.h"
#include "wavelet_amd/decompressor.h"
#include "wavelet_amd/xz_pool.h"

using clk = std::chrono::steady_clock;

static double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct BoxSpec {
    int lev, box, W, H, D, gx, gy, gz;
};

// BASELINE configs[2] (C3) layout, SURVEY §8(d): L0 64 x 64^3, L1 96 x 64^3,
// L2 128 x 32^3, L3 256 x 16^3 + 32 x (48 x 32 x 16) (bench_workloads.py amr_levels)
static std::vector<BoxSpec> c3_layout(int per_level_limit) {
    std::vector<BoxSpec> v;
    auto add = [&](int lev, int first, int n, int W, int H, int D, int per_row, int per_plane, int z0) {
        for (int i = 0; i < n && (per_level_limit <= 0 || first + i < per_level_limit); ++i)
            v.push_back({lev, first + i, W, H, D, (i % per_row) * W, ((i / per_row) % per_plane) * H,
                         (i / (per_row * per_plane)) * D + z0});
    };
    add(0, 0, 64, 64, 64, 64, 4, 4, 0);
    add(1, 0, 96, 64, 64, 64, 6, 4, 0);
    add(2, 0, 128, 32, 32, 32, 8, 4, 0);
    add(3, 0, 256, 16, 16, 16, 8, 8, 0);
    add(3, 256, 32, 48, 32, 16, 4, 4, 256);
    return v;
}

static const double kMean[8] = {300.0, 1000.0, 5.0, 0.0, 300.0, 1.0, 50.0, 0.0};
static const double kAmp[8] = {50.0, 120.0, 2.0, 40.0, 80.0, 0.5, 10.0, 3.0};

static multiBox3D make_box(const BoxSpec& s, int ncomp, uint64_t gid) {
    multiBox3D mb;
    for (int c = 0; c < ncomp; ++c) {
        Box3D b(s.W, s.H, s.D);
        float* p = b.data();
        for (int z = 0; z < s.D; ++z)
            for (int y = 0; y < s.H; ++y)
                for (int x = 0; x < s.W; ++x) {
                    const uint64_t i = (uint64_t)x + (uint64_t)s.W * (y + (uint64_t)s.H * z);
                    const uint64_t h1 = mix64((gid * 16 + c) * 0x9E3779B97F4A7C15ull + 2 * i + 1);
                    const uint64_t h2 = mix64((gid * 16 + c) * 0x9E3779B97F4A7C15ull + 2 * i + 2);
                    const double u1 = ((double)(h1 >> 11) + 1.0) * (1.0 / 9007199254740992.0);
                    const double u2 = (double)(h2 >> 11) * (1.0 / 9007199254740992.0);
                    const double g = std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
                    const double v = kMean[c % 8] + kAmp[c % 8] * std::sin(0.1 * (s.gx + x)) * std::cos(0.07 * (s.gy + y)) +
                                     0.01 * (s.gz + z) + 0.05 * g;
                    p[i] = (float)v;
                }
        mb.push_back(std::move(b));
    }
    return mb;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: dropin_bench <scratch dir> [ncomp=4] [keep=0.999] [boxes per level]\n");
        return 2;
    }
    const std::filesystem::path dir = argv[1];
    const int ncomp = argc > 2 ? std::atoi(argv[2]) : 4;
    const double keep = (double)(float)(argc > 3 ? std::atof(argv[3]) : 0.999);  // Config::keep is a float
    const int limit = argc > 4 ? std::atoi(argv[4]) : 0;
    std::filesystem::create_directories(dir);
    const std::vector<BoxSpec> specs = c3_layout(limit);
    std::vector<multiBox3D> boxes(specs.size());
    {
        const auto t0 = clk::now();
        wavelet_amd::parallel_for(specs.size(), wavelet_amd::host_threads(),
                                  [&](size_t i) { boxes[i] = make_box(specs[i], ncomp, i); });
        std::fprintf(stderr, "dropin_bench: %zu boxes x %d components generated in %.1f s\n", specs.size(), ncomp,
                     secs(t0, clk::now()));
    }
    uint64_t cells = 0;
    for (const multiBox3D& mb : boxes)
        for (const Box3D& b : mb) cells += b.data_size();
    std::vector<int> comps(ncomp);
    for (int c = 0; c < ncomp; ++c) comps[c] = c;

    // warm-up: the thread's context, plans, pools (first call of the process)
    {
        multiBox3D w = make_box(specs[0], ncomp, 999999);
        (void)compress(w, comps, keep, 9, 9, 9, dir.string());
    }
    // GPU stage alone, per box: the call compress() makes, without xz and files
    wc_ctx* ctx = nullptr;
    if (wc_ctx_create(0, &ctx) != WC_OK) {
        std::fprintf(stderr, "wc_ctx_create failed\n");
        return 2;
    }
    std::vector<uint8_t> pay;
    std::vector<uint64_t> offs;
    std::vector<uint32_t> kept;
    double gpu_s = 0.0;
    uint64_t kept_total = 0, payload_bytes = 0;
    for (int rep = 0; rep < 2; ++rep) {  // rep 0: warm (plans of every shape)
        gpu_s = 0.0;
        kept_total = payload_bytes = 0;
        for (size_t i = 0; i < specs.size(); ++i) {
            std::vector<wc_unit> units(ncomp);
            std::vector<const void*> ptrs(ncomp);
            for (int c = 0; c < ncomp; ++c) {
                const Box3D& b = boxes[i][c];
                units[c] = wc_unit{0, (int32_t)b.width(), (int32_t)b.height(), (int32_t)b.depth(), 0};
                ptrs[c] = b.data();
            }
            const uint64_t cap = wc_payload_bound(units.data(), ncomp);
            if (pay.size() < cap) pay.resize(cap);
            offs.resize(ncomp + 1);
            kept.resize(ncomp);
            const auto t0 = clk::now();
            if (wc_forward_host_units(ctx, ptrs.data(), WC_F32, units.data(), ncomp, keep, pay.data(), cap, offs.data(),
                                      kept.data()) != WC_OK) {
                std::fprintf(stderr, "wc_forward_host_units: %s\n", wc_last_error(ctx));
                return 2;
            }
            gpu_s += secs(t0, clk::now());
            for (uint32_t k : kept) kept_total += k;
            payload_bytes += offs[ncomp] - 4;
        }
    }
    wc_ctx_destroy(ctx);
    std::fprintf(stderr, "dropin_bench: GPU stage alone %.3f s per pass\n", gpu_s);

    // -c: compress() per box, the reference's loop order
    std::vector<double> per_box(specs.size());
    const auto c0 = clk::now();
    for (size_t i = 0; i < specs.size(); ++i) {
        const auto t0 = clk::now();
        std::vector<CompressedWavelet> cw = compress(boxes[i], comps, keep, 0, specs[i].lev, specs[i].box, dir.string());
        per_box[i] = secs(t0, clk::now());
        if ((int)cw.size() != ncomp) return 2;
        if ((i + 1) % 64 == 0) std::fprintf(stderr, "dropin_bench: -c %zu / %zu boxes\n", i + 1, specs.size());
    }
    const double c_s = secs(c0, clk::now());
    uint64_t xz_bytes = 0;
    std::vector<std::string> files;
    for (const BoxSpec& s : specs)
        for (int c = 0; c < ncomp; ++c) {
            const std::string f = (dir / ("compressed-wavelet-0-" + std::to_string(s.lev) + "-" + std::to_string(c) +
                                          "-" + std::to_string(s.box) + ".xz"))
                                      .string();
            xz_bytes += std::filesystem::file_size(f);
            files.push_back(f);
        }

    // -c again with write-behind (opt-in, xz_pool.h): compress() queues its
    // components' files and returns; the loop's time, the flush after it, and
    // every file compared byte for byte with the write-through pass's
    // ($DROPIN_WB_REPS = k: k passes, each timed; the JSON reports the first and lists all)
    const std::filesystem::path dir2 = dir / "write_behind";
    const char* reps_env = std::getenv("DROPIN_WB_REPS");
    const int wb_reps = std::max(1, reps_env ? std::atoi(reps_env) : 1);
    std::vector<double> wb_all;
    double wb_s = 0.0, wb_loop_s = 0.0;
    for (int r = 0; r < wb_reps; ++r) {
        std::filesystem::remove_all(dir2);
        std::filesystem::create_directories(dir2);
        wavelet_amd::set_write_behind(true);
        const auto w0 = clk::now();
        for (size_t i = 0; i < specs.size(); ++i)
            (void)compress(boxes[i], comps, keep, 0, specs[i].lev, specs[i].box, dir2.string());
        const double loop_s = secs(w0, clk::now());
        wavelet_amd::flush_writes();
        const double s_all = secs(w0, clk::now());
        wavelet_amd::set_write_behind(false);
        if (r == 0) {
            wb_s = s_all;
            wb_loop_s = loop_s;
        }
        wb_all.push_back(s_all);
    }
    bool wb_same = true;
    for (const std::string& f : files) {
        const std::filesystem::path g = dir2 / std::filesystem::path(f).filename();
        std::ifstream a(f, std::ios::binary), b(g, std::ios::binary);
        const std::string sa((std::istreambuf_iterator<char>(a)), std::istreambuf_iterator<char>());
        const std::string sb((std::istreambuf_iterator<char>(b)), std::istreambuf_iterator<char>());
        if (sa.empty() || sa != sb) wb_same = false;
    }
    std::filesystem::remove_all(dir2);
    std::fprintf(stderr, "dropin_bench: -c with write-behind %.1f s (loop %.1f s), files identical %d\n", wb_s,
                 wb_loop_s, (int)wb_same);

    // -d: decompress() per file; every box compared with the compressed one
    // through the same codec (lossy: rle_decode + inverse of the kept set)
    const auto d0 = clk::now();
    size_t fi = 0;
    double max_err = 0.0;
    for (size_t i = 0; i < specs.size(); ++i)
        for (int c = 0; c < ncomp; ++c, ++fi) {
            Box3D b = decompress(files[fi], 0, specs[i].lev, c, specs[i].box);
            const Box3D& o = boxes[i][c];
            if (b.data_size() != o.data_size()) return 3;
            for (size_t j = 0; j < b.data_size(); j += 997)
                max_err = std::max(max_err, (double)std::fabs(b.data()[j] - o.data()[j]));
        }
    const double d_s = secs(d0, clk::now());
    std::fprintf(stderr, "dropin_bench: -d %zu files in %.1f s\n", files.size(), d_s);
    std::sort(per_box.begin(), per_box.end());
    std::printf(
        "{\"workload\": \"C3 layout, %zu boxes x %d fp32 components (Box3D), keep %.9g\", \"boxes\": %zu, "
        "\"units\": %zu, \"cells\": %llu, \"xz_preset\": %u, \"host_threads\": %d, "
        "\"compress_s\": %.4f, \"compress_ms_per_box\": {\"mean\": %.4f, \"median\": %.4f, \"max\": %.4f}, "
        "\"compress_cells_per_s\": %.6e, \"gpu_stage_s\": %.4f, \"gpu_stage_ms_per_box\": %.4f, "
        "\"gpu_stage_cells_per_s\": %.6e, \"kept_fraction\": %.6f, \"payload_bytes\": %llu, \"xz_bytes\": %llu, "
        "\"decompress_s\": %.4f, \"decompress_ms_per_file\": %.4f, \"decompress_cells_per_s\": %.6e, "
        "\"max_abs_err_sampled\": %.6g, \"write_behind\": {\"compress_s\": %.4f, \"loop_s\": %.4f, "
        "\"compress_cells_per_s\": %.6e, \"files_identical\": %s, \"passes_s\": [%s]}}\n",
        specs.size(), ncomp, keep, specs.size(), specs.size() * ncomp, (unsigned long long)cells,
        wavelet_amd::xz_preset(), wavelet_amd::host_threads(), c_s, 1e3 * c_s / specs.size(),
        1e3 * per_box[per_box.size() / 2], 1e3 * per_box.back(), cells / c_s, gpu_s, 1e3 * gpu_s / specs.size(),
        cells / gpu_s, (double)kept_total / cells, (unsigned long long)payload_bytes, (unsigned long long)xz_bytes,
        d_s, 1e3 * d_s / files.size(), cells / d_s, max_err, wb_s, wb_loop_s, cells / wb_s, wb_same ? "true" : "false",
        [&] {
            std::string l;
            for (double v : wb_all) l += (l.empty() ? "" : ", ") + std::to_string(v);
            return l;
        }().c_str());
    std::filesystem::remove_all(dir);
    return 0;
}

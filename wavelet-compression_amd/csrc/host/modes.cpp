// modes.cpp — the reference's -c / -d / -estimate drivers (src/modes.cpp:24-327),
// batched for the GPU.
//
// The reference walks (t, lev, box) with AMRIterator and calls the per-box
// codec, one component and one unit at a time, after loading the whole run
// into memory.  Here the same work list is cut into chunks of whole boxes
// (about $WCAMD_CHUNK_CELLS cells, default 2^28 = 2 GiB of fp64): a chunk's
// FAB data is read straight into one fp64 buffer (the kernel narrows to fp32,
// as src/preprocess.cpp:78 does on load), all its units go through ONE
// wc_forward_host call, and the payloads are xz-encoded and written by the
// host thread pool while the next chunk is read and transformed.  Output
// files, names and bytes are the reference's.
#include <algorithm>
#include <charconv>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <thread>

#include "host_ctx.h"
#include "log.h"
#include "wavelet_amd/calc-loss.h"
#include "wavelet_amd/iterator.h"
#include "wavelet_amd/modes.h"
#include "wavelet_amd/preprocess.h"
#include "wavelet_amd/readandwrite.h"
#include "wavelet_amd/tmpdir.h"
#include "wavelet_amd/writeplotfile.h"
#include "wavelet_amd/xz_pool.h"

using namespace wavelet_amd;

namespace {

using Clock = std::chrono::high_resolution_clock;
double since(Clock::time_point t0) { return std::chrono::duration<double>(Clock::now() - t0).count(); }

// fmt's "{}" for a double: shortest representation that round-trips.
std::string fmt_double(double v) {
    char b[64];
    auto r = std::to_chars(b, b + sizeof b, v);
    return std::string(b, r.ptr);
}

// Cells per chunk: $WCAMD_CHUNK_CELLS, else 2^28 (2 GiB of fp64), cut to the
// run's share of each device (down to 2^24 cells) so every device gets work.
uint64_t chunk_cells(uint64_t total = 0, size_t ndev = 1) {
    if (const char* v = std::getenv("WCAMD_CHUNK_CELLS")) {
        const long long n = std::atoll(v);
        if (n > 0) return (uint64_t)n;
    }
    const uint64_t share = ndev > 1 ? (total + ndev - 1) / ndev : total;
    return std::clamp<uint64_t>(share, 1ull << 24, 1ull << 28);
}

// GPUs to spread a run over (units shard over the node's
// GPUs): every visible device by default; $WCAMD_DEVICES = "all" or a list
// "0,2,5" (a device may repeat: several host workers on one GPU) picks them;
// $WCAMD_DEVICE alone pins the run to one device.
std::vector<int> run_devices() {
    std::vector<int> d;
    const char* v = std::getenv("WCAMD_DEVICES");
    const char* one = std::getenv("WCAMD_DEVICE");
    if ((!v || !*v) && one && *one) return {std::atoi(one)};
    if (!v || !*v || std::string(v) == "all") {
        for (int i = 0; i < wc_device_count(); ++i) d.push_back(i);
        if (d.empty()) return {-1};  // no device: thread_ctx() fails loudly on first use
    } else {
        std::string cur;
        for (const char* p = v;; ++p) {
            if (*p == ',' || *p == 0) {
                if (!cur.empty()) d.push_back(std::atoi(cur.c_str()));
                cur.clear();
                if (*p == 0) break;
            } else {
                cur.push_back(*p);
            }
        }
    }
    if (d.empty()) fatal("WCAMD_DEVICES names no usable device");
    return d;
}

// Run worker(threads_per_device) on one host thread per device, for `work`
// items (chunks, timesteps): no more devices than items, so a small run keeps
// the whole host pool for its xz stage.
template <class F>
void on_devices(std::vector<int> devs, size_t work, F worker) {
    devs.resize(std::max<size_t>(1, std::min(devs.size(), work)));
    const int tpd = std::max(1, host_threads() / (int)devs.size());
    if (devs.size() == 1) {
        if (devs[0] >= 0) set_thread_device(devs[0]);
        worker(tpd);
        return;
    }
    std::vector<std::thread> th;
    for (int d : devs)
        th.emplace_back([d, tpd, &worker]() {
            set_thread_device(d);
            worker(tpd);
        });
    for (auto& t : th) t.join();
}

// The run's layout without its cell data: plotfile headers + FAB index.
struct RunIndex {
    std::vector<std::string> files;
    std::vector<int> levels;
    std::vector<int> comp_idxs;
    std::vector<std::vector<std::vector<FabRef>>> fabs;  // [t][lev][box]
    LocDimData locations, dimensions;
    std::vector<std::vector<int>> box_counts;
    AMReXInfo amrexinfo;
    bool ok = false;
};

RunIndex index_run(const std::vector<std::string>& files, const std::vector<std::string>& components,
                   const std::vector<int>& levels) {
    RunIndex r;
    r.files = files;
    r.levels = levels;
    for (size_t i = 0; i < files.size(); ++i) {
        const PlotHeader h = read_plot_header(files[i]);
        if (i == 0) {
            r.comp_idxs = match_components(h, components);
            if (r.comp_idxs.empty() && !components.empty()) {
                log_error("Some components you entered were not found. Check that the names you entered match "
                          "their names exactly in the AMReX Header files.");
                return r;
            }
            r.amrexinfo.ref_ratios = h.ref_ratios;
        }
        if (h.dim != 3) log_error("Error: you are using a 3D build to open a " + std::to_string(h.dim) + "D plotfile");
        r.amrexinfo.true_times.push_back(h.true_time);
        r.amrexinfo.geomcellinfo.push_back(h.geomcell);
        r.amrexinfo.xDim = h.xDim;
        r.amrexinfo.yDim = h.yDim;
        r.amrexinfo.zDim = h.zDim;
        std::vector<int> steps(levels.size(), 0);
        for (size_t l = 0; l < levels.size() && l < h.steps.size(); ++l) steps[l] = h.steps[l];
        r.amrexinfo.level_steps.push_back(steps);
        r.fabs.emplace_back();
        r.locations.emplace_back();
        r.dimensions.emplace_back();
        r.box_counts.emplace_back();
        for (int level : levels) {
            std::vector<FabRef> fl = read_level_index(files[i], level);
            std::vector<std::vector<int>> locs, dims;
            for (const FabRef& f : fl) {
                locs.push_back({f.lo[0], f.lo[1], f.lo[2]});
                dims.push_back({f.hi[0] - f.lo[0] + 1, f.hi[1] - f.lo[1] + 1, f.hi[2] - f.lo[2] + 1});
            }
            r.box_counts.back().push_back((int)fl.size());
            r.fabs.back().push_back(std::move(fl));
            r.locations.back().push_back(std::move(locs));
            r.dimensions.back().push_back(std::move(dims));
        }
    }
    r.ok = true;
    return r;
}

// A chunk of whole boxes, in iterator order.
struct BoxRef {
    int t, lev, box;
};

struct Chunk {
    std::vector<BoxRef> boxes;
    std::vector<wc_unit> units;     // nc units per box, comp-major within the box
    std::vector<double> cells;      // fp64 FAB data of the selected components
    uint64_t ncells = 0;
};

// Cut the run into chunks of about `budget` cells (at least one box each).
std::vector<Chunk> plan_chunks(const RunIndex& r, size_t nc, uint64_t budget) {
    std::vector<Chunk> out(1);
    AMRIterator it(r.files.size(), r.levels.size(), r.box_counts, nc);
    it.iterate([&](int t, int l, int b) {
        const FabRef& f = r.fabs[t][l][b];
        const uint64_t npts = (uint64_t)(f.hi[0] - f.lo[0] + 1) * (f.hi[1] - f.lo[1] + 1) * (f.hi[2] - f.lo[2] + 1);
        if (!out.back().boxes.empty() && out.back().ncells + npts * nc > budget) out.emplace_back();
        Chunk& c = out.back();
        c.boxes.push_back({t, l, b});
        for (size_t k = 0; k < nc; ++k) {
            c.units.push_back(wc_unit{c.ncells + k * npts, f.hi[0] - f.lo[0] + 1, f.hi[1] - f.lo[1] + 1,
                                      f.hi[2] - f.lo[2] + 1, 0});
        }
        c.ncells += npts * nc;
    });
    if (out.back().boxes.empty()) out.pop_back();
    return out;
}

void load_chunk(const RunIndex& r, Chunk& c, int threads) {
    c.cells.resize(std::max<uint64_t>(c.ncells, 1));
    const size_t nc = r.comp_idxs.size();
    parallel_for(c.boxes.size(), threads, [&](size_t i) {
        const BoxRef& b = c.boxes[i];
        read_fab(r.fabs[b.t][b.lev][b.box], r.comp_idxs, c.cells.data() + c.units[i * nc].cell_offset);
    });
}

struct Packed {
    // worst-case sized (every coefficient kept) and only partly written: not
    // zero-filled (a std::vector would memset the whole bound, 8 B per cell)
    std::unique_ptr<uint8_t[]> payload;
    std::vector<uint64_t> offsets;
    std::vector<uint32_t> kept;
    std::vector<double> rmse;  // round trip (estimate): calc_rmse_per_box of every unit
};

// The chunk's forward; round_trip: also decode the payloads again and take
// each unit's RMSE against its cells, on the device (wc_round_trip_host: the
// reconstruction never comes back to the host).
Packed forward_chunk(const Chunk& c, double keep, bool round_trip) {
    Packed p;
    const int n = (int)c.units.size();
    const uint64_t cap = wc_payload_bound(c.units.data(), n);
    p.payload.reset(new uint8_t[cap]);
    p.offsets.resize(n + 1);
    p.kept.resize(n);
    wc_ctx* ctx = thread_ctx();
    if (round_trip) {
        p.rmse.resize(n);
        check(ctx, wc_round_trip_host(ctx, c.cells.data(), WC_F64, c.units.data(), n, keep, p.payload.get(), cap,
                                      p.offsets.data(), p.kept.data(), p.rmse.data()),
              "GPU round trip");
    } else {
        check(ctx, wc_forward_host(ctx, c.cells.data(), WC_F64, c.units.data(), n, keep, p.payload.get(), cap,
                                   p.offsets.data(), p.kept.data()),
              "GPU forward");
    }
    return p;
}

std::string unit_name(int t, int lev, int comp, int box) {
    return "compressed-wavelet-" + std::to_string(t) + "-" + std::to_string(lev) + "-" + std::to_string(comp) + "-" +
           std::to_string(box) + ".xz";
}

// Payloads -> one buffer for wc_inverse_host (offsets = 4 mod 8: pairs 8-B aligned).
void inverse_batch(const std::vector<std::string>& payloads, const std::vector<wc_unit>& units, float* out) {
    std::vector<uint64_t> offs(payloads.size());
    uint64_t cur = 4;
    for (size_t i = 0; i < payloads.size(); ++i) {
        if (payloads[i].size() < 20) fatal("Deserialization failed: payload shorter than its header");
        // wc_inverse_host sizes the device copy from each header's nrle: a truncated
        // or corrupt stream must not make it read past this buffer
        int32_t nrle;
        std::memcpy(&nrle, payloads[i].data() + 16, 4);
        if (nrle < 0 || 20 + 8 * (uint64_t)nrle > payloads[i].size())
            fatal("Deserialization failed: payload holds fewer pairs than its header's nrle");
        offs[i] = cur;
        cur += (payloads[i].size() + 4 + 7) / 8 * 8;
    }
    std::vector<uint8_t> buf(cur + 8, 0);
    for (size_t i = 0; i < payloads.size(); ++i) std::memcpy(buf.data() + offs[i], payloads[i].data(), payloads[i].size());
    wc_ctx* ctx = thread_ctx();
    check(ctx, wc_inverse_host(ctx, buf.data(), offs.data(), units.data(), (int)units.size(), out), "GPU decompress");
}

// The run's cells over all (t, lev, box) and selected components.
uint64_t run_cells(const RunIndex& r, size_t nc) {
    uint64_t total = 0;
    for (const auto& t : r.fabs)
        for (const auto& l : t)
            for (const FabRef& f : l)
                total += (uint64_t)(f.hi[0] - f.lo[0] + 1) * (f.hi[1] - f.lo[1] + 1) * (f.hi[2] - f.lo[2] + 1) * nc;
    return total;
}

// Compress every unit of `r` into `dir` (file names joined as std::filesystem
// paths, src/compressor.cpp:250-254), chunks spread over `devs`.  `on_chunk(i,
// chunk, payloads)` sees chunk i (iterator order) after its forward pass
// (round_trip: with every unit's RMSE), on the device's host thread: chunks
// arrive in any order and concurrently, so it does its own locking.
template <class OnChunk>
void compress_run(const RunIndex& r, double keep, const std::filesystem::path& dir, OnChunk on_chunk,
                  const std::vector<int>& devs, bool round_trip = false) {
    const size_t nc = r.comp_idxs.size();
    std::vector<Chunk> chunks = plan_chunks(r, nc, chunk_cells(run_cells(r, nc), devs.size()));
    auto jobs_of = [&](const Chunk& c, const Packed& p) {
        std::vector<XzJob> jobs;
        for (size_t i = 0; i < c.boxes.size(); ++i)
            for (size_t k = 0; k < nc; ++k) {
                const size_t u = i * nc + k;
                const BoxRef& b = c.boxes[i];
                jobs.push_back(XzJob{p.payload.get() + p.offsets[u], 20 + 8ull * p.kept[u],
                                     (dir / unit_name(b.t, b.lev, r.comp_idxs[k], b.box)).string()});
            }
        return jobs;
    };
    std::atomic<size_t> next{0};
    on_devices(devs, chunks.size(), [&](int threads) {
        // per device: read + GPU pass of chunk i overlapped with the xz stage of chunk i-1
        std::future<void> xz_done;
        for (size_t i = next.fetch_add(1); i < chunks.size(); i = next.fetch_add(1)) {
            Chunk& c = chunks[i];
            load_chunk(r, c, threads);
            auto p = std::make_shared<Packed>(forward_chunk(c, keep, round_trip));
            std::vector<XzJob> jobs = jobs_of(c, *p);
            if (xz_done.valid()) xz_done.get();
            xz_done = std::async(std::launch::async,
                                 [jobs = std::move(jobs), p, threads]() { xz_write_files(jobs, threads); });
            on_chunk(i, c, *p);
            c.cells.clear();
            c.cells.shrink_to_fit();
        }
        if (xz_done.valid()) xz_done.get();
    });
}

}  // namespace

int compress(const Config& cfg) {
    if (cfg.xz_preset >= 0) set_xz_preset((uint32_t)cfg.xz_preset);
    if (xz_preset() != 6) log_info("xz preset " + std::to_string(xz_preset() & 0xff) +
                                   ((xz_preset() & 0x80000000u) ? "e" : "") + " (the reference's is 6)");
    const std::vector<std::string> files = format_files(cfg.data_dir, cfg.min_time, cfg.max_time);
    const std::vector<int> levels = format_levels(cfg.min_level, cfg.max_level);
    const int num_times = (int)files.size(), num_levels = (int)levels.size();
    const int num_components = (int)cfg.components.size();
    log_info("Processing data...");
    const auto t0 = Clock::now();
    RunIndex r = index_run(files, cfg.components, levels);
    if (!r.ok) return 1;
    RunInfo runinfo{files, cfg.min_level, cfg.max_level, cfg.components, r.comp_idxs};
    AMRIterator iterator(num_times, num_levels, r.box_counts, num_components);
    if (!cfg.compressed_dir.empty() && !std::filesystem::exists(cfg.compressed_dir)) {
        std::error_code ec;
        std::filesystem::create_directories(cfg.compressed_dir, ec);
        if (ec) log_error("Failed to create compressed directory " + cfg.compressed_dir + ": " + ec.message());
    }
    write_runinfo(runinfo, cfg.compressed_dir, "runinfo.raw");
    write_loc_dim_to_bin(r.locations, cfg.compressed_dir, "locations.raw", iterator);
    write_loc_dim_to_bin(r.dimensions, cfg.compressed_dir, "dimensions.raw", iterator);
    write_box_counts(r.box_counts, cfg.compressed_dir, "boxcounts.raw", num_times, num_levels);
    write_amrexinfo(r.amrexinfo, cfg.compressed_dir, "amrexinfo.raw");
    log_info("Successfully processed data in " + fmt_double(since(t0)) + " seconds. Beginning compression...");
    const auto t1 = Clock::now();
    compress_run(r, (double)cfg.keep, std::filesystem::path(cfg.compressed_dir),
                 [](size_t, const Chunk&, const Packed&) {}, run_devices());
    log_info("Compression completed in " + fmt_double(since(t1)) + " seconds.");
    return 0;
}

int decompress(const Config& cfg) {
    RunInfo runinfo = read_runinfo(cfg.compressed_dir, "runinfo.raw");
    const std::vector<int> levels = format_levels(runinfo.min_level, runinfo.max_level);
    const int num_times = (int)runinfo.files.size(), num_levels = (int)levels.size();
    const int num_components = (int)runinfo.components.size();
    if (num_times > 0)
        log_info("Decompressing data between timestep " + runinfo.files.front() + " and " + runinfo.files.back() +
                 ", level " + std::to_string(runinfo.min_level) + " and " + std::to_string(runinfo.max_level) +
                 ", for " + std::to_string(num_components) + " components");
    log_info("Beginning decompression...");
    const auto t0 = Clock::now();
    const std::vector<std::vector<int>> counts = read_box_counts(cfg.compressed_dir, "boxcounts.raw", num_times, num_levels);
    AMRIterator iterator(num_times, num_levels, counts, num_components);
    const AMReXInfo info = read_amrex_info(cfg.compressed_dir, "amrexinfo.raw");
    const LocDimData locs = read_loc_dim_from_bin(cfg.compressed_dir, "locations.raw", counts, iterator, num_times, num_levels);
    const LocDimData dims = read_loc_dim_from_bin(cfg.compressed_dir, "dimensions.raw", counts, iterator, num_times, num_levels);
    // One timestep at a time per device: decode its files on the pool, one GPU
    // inverse for all its units, then write its plotfile.
    std::atomic<int> next{0};
    on_devices(run_devices(), (size_t)std::max(num_times, 0), [&](int threads) {
        for (int t = next.fetch_add(1); t < num_times; t = next.fetch_add(1)) {
            std::vector<std::string> paths;
            std::vector<wc_unit> units;
            uint64_t cursor = 0;
            for (int l = 0; l < num_levels; ++l)
                for (int b = 0; b < counts[t][l]; ++b)
                    for (int comp : runinfo.comp_idxs)
                        paths.push_back(cfg.compressed_dir + unit_name(t, l, comp, b));  // string concatenation (src/modes.cpp:157)
            std::vector<std::string> payloads = xz_read_files(paths, threads);
            for (const std::string& p : payloads) {
                if (p.size() < 20) fatal("Deserialization failed: payload shorter than its header");
                int32_t h[3];
                std::memcpy(h, p.data(), sizeof h);
                wc_unit u{cursor, std::max(h[0], 0), std::max(h[1], 0), std::max(h[2], 0), 0};
                cursor += (uint64_t)u.nx * u.ny * u.nz;
                cursor = (cursor + 3) & ~uint64_t(3);
                units.push_back(u);
            }
            std::vector<float> cells(std::max<uint64_t>(cursor, 1));
            inverse_batch(payloads, units, cells.data());
            payloads.clear();
            std::vector<std::vector<std::vector<multiBox3D>>> regen(1);
            regen[0].resize(num_levels);
            size_t u = 0;
            for (int l = 0; l < num_levels; ++l)
                for (int b = 0; b < counts[t][l]; ++b) {
                    multiBox3D mb;
                    for (int c = 0; c < num_components; ++c, ++u) {
                        Box3D box(units[u].nx, units[u].ny, units[u].nz);
                        if (box.data_size())
                            std::memcpy(box.data(), cells.data() + units[u].cell_offset, 4 * box.data_size());
                        mb.push_back(std::move(box));
                    }
                    regen[0][l].push_back(std::move(mb));
                }
            AMReXInfo one = info;
            one.true_times = {info.true_times[t]};
            one.geomcellinfo = {info.geomcellinfo[t]};
            one.level_steps = {info.level_steps[t]};
            write_plotfiles(std::move(regen), {locs[t]}, {dims[t]}, {runinfo.files[t]}, num_levels, num_components,
                            runinfo.components, one, cfg.out_dir);
        }
    });
    const double t_decode = since(t0);
    log_info("Decompression completed in " + fmt_double(t_decode) + " seconds.");
    log_info("Sucessfully wrote plotfiles.");
    return 0;
}

int estimate(Config& cfg) {
    const int num_components = (int)cfg.components.size();
    TempDir scratch;
    const std::vector<std::string> files = format_files(cfg.data_dir, cfg.min_time, cfg.min_time);
    const std::vector<int> levels{cfg.min_level};
    RunIndex r = index_run(files, cfg.components, levels);
    if (!r.ok || files.empty()) return 1;
    const size_t nc = r.comp_idxs.size();
    // The reference compresses the boxes, reads the files back, decompresses
    // them and takes calc_rmse_per_box (src/modes.cpp:236-291).  Here each
    // chunk's round trip runs on the device right after its forward
    // (wc_round_trip_host): the files are still written (their sizes are the
    // estimate), the RMSE comes from the same payload bytes they hold.
    // min/max over the narrowed values.
    // Chunks run on every device; the per-box RMSEs are kept per chunk and
    // averaged in iterator order (the reference's order, so the mean is the
    // same double whatever the device count); min / max do not depend on order.
    std::vector<std::vector<double>> all_rmses(nc);
    std::vector<float> minv(nc, FLT_MAX), maxv(nc, FLT_MIN);  // src/preprocess.cpp:30-31 quirk
    std::map<size_t, std::vector<double>> chunk_rmse;  // chunk -> its units' RMSEs
    std::mutex mu;
    compress_run(r, (double)cfg.keep, scratch.path(), [&](size_t ci, Chunk& c, const Packed& p) {
        std::vector<float> lo(nc, FLT_MAX), hi(nc, FLT_MIN);
        for (size_t u = 0; u < c.units.size(); ++u) {
            const size_t k = u % nc;
            const uint64_t n = (uint64_t)c.units[u].nx * c.units[u].ny * c.units[u].nz;
            const double* s = c.cells.data() + c.units[u].cell_offset;
            for (uint64_t i = 0; i < n; ++i) {
                const float v = (float)s[i];
                if (v < lo[k]) lo[k] = v;
                if (v > hi[k]) hi[k] = v;
            }
        }
        std::lock_guard<std::mutex> g(mu);
        for (size_t k = 0; k < nc; ++k) {
            minv[k] = std::min(minv[k], lo[k]);
            maxv[k] = std::max(maxv[k], hi[k]);
        }
        chunk_rmse[ci] = p.rmse;
    }, run_devices(), /*round_trip=*/true);
    for (const auto& [ci, rm] : chunk_rmse)
        for (size_t u = 0; u < rm.size(); ++u) all_rmses[u % nc].push_back(rm[u]);
    // The reference reads every file back (src/modes.cpp:250-265) and exits on
    // one it cannot read; the RMSE here comes from the payloads in memory, so
    // check the files the size estimate counts exist and are not empty.
    for (int b = 0; b < r.box_counts[0][0]; ++b)
        for (int comp : r.comp_idxs) {
            const std::string f = (scratch.path() / unit_name(0, 0, comp, b)).string();
            std::error_code ec;
            const auto sz = std::filesystem::file_size(f, ec);
            if (ec) fatal("Error getting file size: " + ec.message() + " " + f);
            if (sz == 0) fatal("Failed to read file: " + f);
        }
    log_info("Compression complete.");
    log_info("Decompression complete.");
    for (int c = 0; c < num_components && c < (int)nc; ++c) {
        const double mean = std::accumulate(all_rmses[c].begin(), all_rmses[c].end(), 0.0) / all_rmses[c].size();
        log_info("Predicted RMSE, " + cfg.components[c] + " = " + fmt_double(mean));
        const double loss = calc_adj_loss(mean, maxv[c] - minv[c]);
        log_info("Predicted Adjusted loss, " + cfg.components[c] + " = " + fmt_double(loss));
    }
    // compressed size vs the level's raw size scaled to the compressed components (src/modes.cpp:294-324)
    std::ifstream x(files[0] + "/Header");
    if (!x.is_open()) log_error("Failed to open header file: " + files[0]);
    std::string str;
    int ncomp_file = 1;
    x >> str >> ncomp_file;
    double raw_size = calc_size(files[0] + "/Level_" + std::to_string(levels[0]) + "/");
    raw_size /= ncomp_file;
    raw_size *= num_components;
    const double compressed_size = calc_size(scratch.path().string());
    log_info("Predicted compressed size: " + fmt_double(compressed_size / raw_size * 100) + "%");
    return 0;
}

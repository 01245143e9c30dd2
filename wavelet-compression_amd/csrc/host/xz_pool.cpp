// xz_pool.cpp — the per-unit xz stage on a host thread pool.
//
// The reference encodes one unit at a time inside compress()
// (src/compressor.cpp:256-291: lzma_easy_encoder(6, CRC64), one
// lzma_code(FINISH) into a 1.1 x + 128 byte buffer) and decodes one file at a
// time in decompress() (src/decompressor.cpp:164-234).  Units are independent
// .xz streams, so here a batch of them runs on `threads` workers with dynamic
// assignment; each stream's bytes are exactly what the serial code produces.
#include <lzma.h>

#include <atomic>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <thread>

#include "host_ctx.h"
#include "wavelet_amd/codec_extras.h"
#include "wavelet_amd/xz_pool.h"

namespace wavelet_amd {

int host_threads() {
    for (const char* var : {"WCAMD_THREADS", "OMP_NUM_THREADS"}) {
        if (const char* v = std::getenv(var)) {
            const int n = std::atoi(v);
            if (n > 0) return n;
        }
    }
    const unsigned hc = std::thread::hardware_concurrency();
    return hc ? (int)hc : 1;
}

void parallel_for(size_t n, int threads, const std::function<void(size_t)>& fn) {
    if (n == 0) return;
    const size_t nt = std::min<size_t>(n, (size_t)std::max(1, threads));
    if (nt == 1) {
        for (size_t i = 0; i < n; ++i) fn(i);
        return;
    }
    std::atomic<size_t> next{0};
    auto worker = [&]() {
        for (size_t i = next.fetch_add(1); i < n; i = next.fetch_add(1)) fn(i);
    };
    std::vector<std::thread> pool;
    pool.reserve(nt - 1);
    for (size_t t = 1; t < nt; ++t) pool.emplace_back(worker);
    worker();
    for (auto& th : pool) th.join();
}

int parse_xz_preset(const char* text) {
    if (!text || text[0] < '0' || text[0] > '9') return -1;
    uint32_t v = (uint32_t)(text[0] - '0');
    if (text[1] == 'e' && text[2] == '\0') return (int)(v | LZMA_PRESET_EXTREME);
    return text[1] == '\0' ? (int)v : -1;
}

namespace {
std::atomic<int> g_preset{-1};  // -1: not chosen yet ($WCAMD_XZ_PRESET or 6)
}

uint32_t xz_preset() {
    int p = g_preset.load(std::memory_order_relaxed);
    if (p < 0) {
        p = 6;
        if (const char* e = std::getenv("WCAMD_XZ_PRESET")) {
            const int v = parse_xz_preset(e);
            if (v < 0) fatal(std::string("WCAMD_XZ_PRESET: 0-9, optionally followed by e, not ") + e);
            p = v;
        }
        int expect = -1;
        g_preset.compare_exchange_strong(expect, p);
        p = g_preset.load(std::memory_order_relaxed);
    }
    return (uint32_t)p;
}

void set_xz_preset(uint32_t preset) { g_preset.store((int)preset, std::memory_order_relaxed); }

bool xz_encode_try(const uint8_t* data, size_t size, std::string& out, const char*& err, int preset) {
    lzma_stream strm = LZMA_STREAM_INIT;
    const uint32_t pr = preset >= 0 ? (uint32_t)preset : xz_preset();
    if (lzma_easy_encoder(&strm, pr, LZMA_CHECK_CRC64) != LZMA_OK) {
        err = "Failed to initialize LZMA encoder";
        return false;
    }
    out.assign(static_cast<size_t>(size * 1.1) + 128, '\0');
    strm.next_in = data;
    strm.avail_in = size;
    strm.next_out = reinterpret_cast<uint8_t*>(out.data());
    strm.avail_out = out.size();
    const bool ok = lzma_code(&strm, LZMA_FINISH) == LZMA_STREAM_END;
    if (ok) out.resize(out.size() - strm.avail_out);
    lzma_end(&strm);
    if (!ok) err = "LZMA compression failed";
    return ok;
}

std::string xz_encode(const uint8_t* data, size_t size, int preset) {
    std::string out;
    const char* err = nullptr;
    if (!xz_encode_try(data, size, out, err, preset)) fatal(err);
    return out;
}

std::string xz_compress(const std::string& payload) {
    return xz_encode(reinterpret_cast<const uint8_t*>(payload.data()), payload.size());
}

uint64_t xz_write_files(const std::vector<XzJob>& jobs, int threads) {
    std::atomic<uint64_t> written{0};
    parallel_for(jobs.size(), threads, [&](size_t i) {
        const XzJob& j = jobs[i];
        std::ofstream f(j.path, std::ios::binary);
        if (!f.is_open()) return;  // the reference skips a file it cannot open
        const std::string xz = xz_encode(j.data, j.size);
        f.write(xz.data(), (std::streamsize)xz.size());
        written += xz.size();
    });
    return written.load();
}

static std::string slurp(const std::string& path) {
    std::error_code ec;
    const auto size = std::filesystem::file_size(path, ec);
    if (ec) fatal("Error getting file size: " + ec.message() + " " + path);
    std::ifstream f(path, std::ios::binary);
    if (!f) fatal("Failed to open file: " + path);
    std::string data(size, '\0');
    if (size && !f.read(data.data(), (std::streamsize)size)) fatal("Failed to read file: " + path);
    return data;
}

std::vector<std::string> xz_read_files(const std::vector<std::string>& paths, int threads) {
    std::vector<std::string> out(paths.size());
    parallel_for(paths.size(), threads, [&](size_t i) { out[i] = xz_decompress(slurp(paths[i])); });
    return out;
}

}  // namespace wavelet_amd

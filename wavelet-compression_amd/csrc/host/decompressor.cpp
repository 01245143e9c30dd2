// decompressor.cpp — C++ mirror of the reference's decompressor
// (src/decompressor.cpp:14-255).  xz decode on the host; rle_decode and the
// inverse transform on the GPU (wc_inverse_host).
#include <lzma.h>

#include <cstdint>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <vector>

#include "host_ctx.h"
#include "wavelet_amd/codec_extras.h"
#include "wavelet_amd/decompressor.h"
#include "wavelet_amd/xz_pool.h"

namespace wavelet_amd {

std::vector<float> rle_decode(const std::vector<std::pair<int, float>>& rle, int total) {
    std::vector<float> out(total > 0 ? total : 0, 0.0f);
    long long idx = 0;
    for (const auto& pr : rle) {
        idx += pr.first;
        if (idx >= 0 && idx < total) out[idx++] = pr.second;
    }
    return out;
}

std::string xz_decompress(const std::string& xz) {
    // lzma_stream_decoder(UINT64_MAX, LZMA_CONCATENATED), output doubled until
    // the stream ends (src/decompressor.cpp:188-220).
    lzma_stream strm = LZMA_STREAM_INIT;
    if (lzma_stream_decoder(&strm, UINT64_MAX, LZMA_CONCATENATED) != LZMA_OK) fatal("Failed to initialize LZMA decoder.");
    std::vector<uint8_t> out(4096);
    strm.next_in = reinterpret_cast<const uint8_t*>(xz.data());
    strm.avail_in = xz.size();
    strm.next_out = out.data();
    strm.avail_out = out.size();
    for (;;) {
        const lzma_ret r = lzma_code(&strm, LZMA_FINISH);
        if (r == LZMA_STREAM_END) break;
        if (r != LZMA_OK) {
            lzma_end(&strm);
            fatal("LZMA decompression failed with code: " + std::to_string((int)r));
        }
        const size_t old = out.size();
        out.resize(old * 2);
        strm.next_out = out.data() + old;
        strm.avail_out = old;
    }
    const size_t used = out.size() - strm.avail_out;
    lzma_end(&strm);
    return std::string(reinterpret_cast<const char*>(out.data()), used);
}

static std::string read_file(const std::string& path) {
    std::error_code ec;
    const auto size = std::filesystem::file_size(path, ec);
    if (ec) fatal("Error getting file size: " + ec.message() + " " + path);
    std::ifstream f(path, std::ios::binary);
    if (!f) fatal("Failed to open file: " + path);
    std::string data(size, '\0');
    if (!f.read(data.data(), (std::streamsize)size)) fatal("Failed to read file: " + path);
    return data;
}

}  // namespace wavelet_amd

using namespace wavelet_amd;

CompressedWavelet deserialize_compressed_wavelet(const std::string& data) {
    CompressedWavelet cw;
    auto get = [&data](size_t off) {
        int32_t v = 0;
        if (off + 4 <= data.size()) std::memcpy(&v, data.data() + off, 4);
        return v;
    };
    cw.shape = {get(0), get(4), get(8)};
    cw.coeff_shape = {get(12)};
    const int32_t n = get(16);
    if (n < 0 || 20 + 8ull * (uint64_t)n > data.size()) fatal("Deserialization failed: truncated payload");
    cw.rle_encoded.resize(n);
    for (int32_t i = 0; i < n; ++i) {
        float v;
        std::memcpy(&v, data.data() + 24 + 8ull * i, 4);
        cw.rle_encoded[i] = {get(20 + 8ull * i), v};
    }
    return cw;
}

Box3D inverse_wavelet_decompose(std::vector<float> flat, int x, int y, int z) {
    Box3D out(x, y, z);
    if (out.data_size() == 0) return out;
    if (flat.size() < out.data_size()) fatal("inverse_wavelet_decompose: flat shorter than x*y*z");
    wc_ctx* c = thread_ctx();
    wc_unit u{0, x, y, z, 0};
    check(c, wc_inverse_flat_host(c, flat.data(), &u, 1, out.data()), "GPU inverse transform");
    return out;
}

Box3D decompress(std::string file_path, int /*time*/, int /*level*/, int /*component*/, int /*box_idx*/) {
    flush_writes(file_path);  // this file, if compress() queued it (write-behind, opt-in), is complete first
    const std::string payload = xz_decompress(read_file(file_path));
    if (payload.size() < 20) fatal("Deserialization failed: payload shorter than its header");
    int32_t hdr[5];
    std::memcpy(hdr, payload.data(), sizeof hdr);
    Box3D out(hdr[0] > 0 ? hdr[0] : 0, hdr[1] > 0 ? hdr[1] : 0, hdr[2] > 0 ? hdr[2] : 0);
    if (out.data_size() == 0) return out;
    // stage as one unit at offset 4 (pairs 8-byte aligned)
    std::vector<uint8_t> buf(payload.size() + 8);
    std::memcpy(buf.data() + 4, payload.data(), payload.size());
    const uint64_t off = 4;
    wc_unit u{0, hdr[0], hdr[1], hdr[2], 0};
    wc_ctx* c = thread_ctx();
    check(c, wc_inverse_host(c, buf.data(), &off, &u, 1, out.data()), "GPU decompress");
    return out;
}

// compressor.cpp — C++ mirror of the reference's compress() (src/compressor.cpp:192-297).
//
// All components of the box go to the GPU in ONE wc_forward_host_units call,
// each straight from its Box3D (the reference loops per component, :203); the
// serialized payloads come back byte-identical to serialize_compressed_wavelet,
// and the host only does the xz stage and the file write, the components'
// independent xz streams on a pool of host threads (same bytes as one by one).
#include <lzma.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <memory>
#include <mutex>
#include <vector>

#include "host_ctx.h"
#include "wavelet_amd/codec_extras.h"
#include "wavelet_amd/compressor.h"
#include "wavelet_amd/decompressor.h"
#include "wavelet_amd/xz_pool.h"

namespace wavelet_amd {

static thread_local int t_device = -1;

void set_thread_device(int device) { t_device = device; }

wc_ctx* thread_ctx() {
    thread_local struct Holder {
        wc_ctx* c = nullptr;
        ~Holder() {
            if (c) wc_ctx_destroy(c);
        }
    } h;
    if (!h.c) {
        const char* dev = std::getenv("WCAMD_DEVICE");
        const int d = t_device >= 0 ? t_device : (dev ? std::atoi(dev) : 0);
        if (wc_ctx_create(d, &h.c) != WC_OK) fatal("wc_ctx_create failed: no usable HIP device");
    }
    return h.c;
}

std::vector<std::pair<int, float>> rle_encode(const std::vector<bool>& mask, const std::vector<float>& values) {
    std::vector<std::pair<int, float>> out;
    int gap = 0;
    size_t vi = 0;
    for (bool m : mask) {
        if (!m) {
            ++gap;
            continue;
        }
        out.emplace_back(gap, values[vi++]);
        gap = 0;
    }
    return out;
}

std::string serialize_compressed_wavelet(const CompressedWavelet& cw) {
    std::string buf;
    auto put = [&buf](const void* p, size_t n) { buf.append(static_cast<const char*>(p), n); };
    for (int d : cw.shape) put(&d, 4);
    for (int d : cw.coeff_shape) put(&d, 4);
    const int n = static_cast<int>(cw.rle_encoded.size());
    put(&n, 4);
    for (const auto& pr : cw.rle_encoded) {
        put(&pr.first, 4);
        put(&pr.second, 4);
    }
    return buf;
}

std::vector<float> wavelet_decompose(const Box3D& box) {
    wc_ctx* c = thread_ctx();
    wc_unit u{0, (int32_t)box.width(), (int32_t)box.height(), (int32_t)box.depth(), 0};
    std::vector<float> flat(box.data_size());
    if (flat.empty()) return flat;
    check(c, wc_decompose_host(c, box.data(), WC_F32, &u, 1, flat.data()), "wavelet_decompose");
    return flat;
}

}  // namespace wavelet_amd

using namespace wavelet_amd;

std::vector<CompressedWavelet> compress(multiBox3D& box, std::vector<int> components, double keep, int time,
                                        int level, int box_index, std::string compressed_dir) {
    const int n = static_cast<int>(components.size());
    std::vector<CompressedWavelet> out;
    if (n == 0) return out;
    // box[0..n) (positional, src/compressor.cpp:203-206), each component from
    // its own Box3D storage: no packing copy on the host
    std::vector<wc_unit> units(n);
    std::vector<const void*> cells(n);
    for (int c = 0; c < n; ++c) {
        const Box3D& b = box.at(c);
        units[c] = wc_unit{0, (int32_t)b.width(), (int32_t)b.height(), (int32_t)b.depth(), 0};
        cells[c] = b.data();
    }
    // the payload buffer of this thread, reused across calls (grow-only, never
    // zero-filled: the library writes every byte it reports)
    const uint64_t cap = wc_payload_bound(units.data(), n);
    thread_local std::unique_ptr<uint8_t[]> t_payload;
    thread_local uint64_t t_cap = 0;
    if (t_cap < cap) {
        t_payload.reset(new uint8_t[cap]);
        t_cap = cap;
    }
    std::vector<uint64_t> offsets(n + 1);
    std::vector<uint32_t> kept(n);
    wc_ctx* ctx = thread_ctx();
    check(ctx, wc_forward_host_units(ctx, cells.data(), WC_F32, units.data(), n, keep, t_payload.get(), cap,
                                     offsets.data(), kept.data()),
          "GPU forward");
    // per component: the struct, and the .xz file (src/compressor.cpp:250-291);
    // the components' xz streams are independent: encoded concurrently, or
    // queued for the write-behind workers (opt-in, xz_pool.h)
    out.resize(n);
    const uint8_t* payload = t_payload.get();
    const bool behind = write_behind();
    if (behind) note_write_behind_used();
    parallel_for((size_t)n, behind ? 1 : std::min(n, host_threads()), [&](size_t c) {
        std::string serialized(reinterpret_cast<const char*>(payload + offsets[c]), 20 + 8ull * kept[c]);
        CompressedWavelet cw = deserialize_compressed_wavelet(serialized);
        for (const auto& pr : cw.rle_encoded)
            if (std::fabs((double)pr.second) > INT16_MAX) cw.need32 = true;  // src/compressor.cpp:229
        const std::filesystem::path fname =
            std::filesystem::path(compressed_dir) / ("compressed-wavelet-" + std::to_string(time) + "-" +
                                                     std::to_string(level) + "-" + std::to_string(components[c]) +
                                                     "-" + std::to_string(box_index) + ".xz");
        if (behind) {
            write_behind_submit(std::move(serialized), fname.string());
        } else {
            std::ofstream file(fname, std::ios::binary);
            if (file.is_open()) {  // a failed open silently skips the file, as the reference does (:256-257)
                const std::string xz = xz_compress(serialized);
                file.write(xz.data(), (std::streamsize)xz.size());
            }
        }
        out[c] = std::move(cw);
    });
    return out;
}

// test_codec.cpp — the reference's codec unit tests restated against the C++
// mirror (include/wavelet_amd/*.h -> libwavelet_amd_host.so -> GPU kernels).
//   RLE Encode            src/compressor.cpp:300-339
//   Serialization         src/compressor.cpp:342-366
//   Wavelet decomposition src/compressor.cpp:369-384
//   File writing          src/compressor.cpp:387-406
//   Calc RMSE             src/calc-loss.cpp:68-86
// plus sign-quirk and odd-tail checks from SURVEY.md §8(c).
// Minimal runner (no doctest in this image): prints one line per case and
// exits non-zero on the first failed REQUIRE.
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <random>
#include <string>
#include <unistd.h>

#include "wavelet_amd/calc-loss.h"
#include "wavelet_amd/codec_extras.h"
#include "wavelet_amd/compressor.h"
#include "wavelet_amd/decompressor.h"
#include "wavelet_amd/xz_pool.h"
#include <fstream>
#include <iterator>

static int g_checks = 0;
#define REQUIRE(cond)                                                                   \
    do {                                                                                \
        ++g_checks;                                                                     \
        if (!(cond)) {                                                                  \
            std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond);      \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

using namespace wavelet_amd;
using Pairs = std::vector<std::pair<int, float>>;

static void rle_encode_case() {
    std::vector<float> values{1.0f, 2.0f, 3.0f, 4.0f, 5.0f};
    REQUIRE((rle_encode({true, true, false, false, true}, values) == Pairs{{0, 1.0f}, {0, 2.0f}, {2, 3.0f}}));
    REQUIRE((rle_encode({true, true, true, true, true}, values) ==
             Pairs{{0, 1.0f}, {0, 2.0f}, {0, 3.0f}, {0, 4.0f}, {0, 5.0f}}));
    REQUIRE(rle_encode({false, false, false, false, false}, values).empty());
}

static void serialization_case() {
    std::mt19937 gen(12345);
    std::uniform_int_distribution<> d(1, 100);
    CompressedWavelet t;
    t.shape = {d(gen), d(gen), d(gen)};
    t.coeff_shape = {d(gen)};
    t.rle_encoded = {{0, 1.0f}, {0, 2.0f}, {2, 3.0f}};
    t.need32 = false;
    CompressedWavelet r = deserialize_compressed_wavelet(serialize_compressed_wavelet(t));
    REQUIRE(t.shape == r.shape);
    REQUIRE(t.coeff_shape == r.coeff_shape);
    REQUIRE(t.rle_encoded == r.rle_encoded);
    REQUIRE(t.need32 == r.need32);
}

static void wavelet_case() {
    Box3D test(4, 8, 16, 5.0f);
    test.set(1, 2, 3, 8.5f);
    test.set(2, 5, 6, 5.44f);
    test.set(1, 1, 1, 3.3999932f);
    test.set(2, 2, 2, 3.19229f);
    test.set(3, 5, 12, 199.39029f);
    std::vector<float> w = wavelet_decompose(test);
    Box3D result = inverse_wavelet_decompose(w, 4, 8, 16);
    REQUIRE(test.equals(result, 1e-6f));
}

static std::filesystem::path scratch() {
    char tmpl[] = "/tmp/wavelet_amd_test.XXXXXX";
    char* p = mkdtemp(tmpl);
    REQUIRE(p != nullptr);
    return p;
}

static void file_writing_case() {
    Box3D box(4, 8, 16, 5.0f);
    multiBox3D test;
    test.push_back(std::move(box));
    const auto dir = scratch();
    compress(test, {0}, 0.999, 0, 0, 0, dir.string());
    Box3D result = decompress(dir.string() + "/compressed-wavelet-0-0-0-0.xz", 0, 0, 0, 0);
    REQUIRE(test[0].equals(result, 0));
    std::filesystem::remove_all(dir);
}

static void multi_component_and_quirks_case() {
    // components name the files; box[c] is positional (src/compressor.cpp:203-206, :253)
    multiBox3D mb;
    Box3D spike(4, 4, 4, 5.0f);
    spike.set(3, 2, 1, 7.5f);
    mb.push_back(std::move(spike));
    mb.push_back(Box3D(4, 4, 4, -5.0f));  // negative max -> everything kept
    mb.push_back(Box3D(3, 4, 2, 7.0f));   // odd width: x = 2 plane comes back 0
    const auto dir = scratch();
    auto cws = compress(mb, {6, 25, 3}, (double)0.999f, 2, 1, 7, dir.string());
    REQUIRE(cws.size() == 3);
    REQUIRE(cws[0].rle_encoded.size() == 15);
    REQUIRE(cws[1].rle_encoded.size() == 64);
    REQUIRE((cws[0].shape == std::vector<int>{4, 4, 4}) && (cws[0].coeff_shape == std::vector<int>{64}));
    REQUIRE(std::filesystem::exists(dir / "compressed-wavelet-2-1-6-7.xz"));
    REQUIRE(std::filesystem::exists(dir / "compressed-wavelet-2-1-25-7.xz"));
    Box3D odd = decompress((dir / "compressed-wavelet-2-1-3-7.xz").string(), 2, 1, 3, 7);
    for (int z = 0; z < 2; ++z)
        for (int y = 0; y < 4; ++y) {
            REQUIRE(odd.get(2, y, z) == 0.0f);
            REQUIRE(odd.get(0, y, z) == 7.0f && odd.get(1, y, z) == 7.0f);
        }
    // the components' xz streams were encoded concurrently: each file is
    // byte for byte the serial encoder's output of the component's payload
    const int comps[3] = {6, 25, 3};
    for (int c = 0; c < 3; ++c) {
        const std::string ser = serialize_compressed_wavelet(cws[c]);
        std::ifstream f(dir / ("compressed-wavelet-2-1-" + std::to_string(comps[c]) + "-7.xz"), std::ios::binary);
        const std::string file((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        REQUIRE(file == wavelet_amd::xz_encode(reinterpret_cast<const uint8_t*>(ser.data()), ser.size()));
    }
    std::vector<float> flat = rle_decode(cws[1].rle_encoded, cws[1].coeff_shape[0]);
    Box3D back = inverse_wavelet_decompose(flat, 4, 4, 4);
    REQUIRE(back.equals(mb[1], 0));
    REQUIRE(calc_size(dir.string()) > 0);
    std::filesystem::remove_all(dir);
}

// Write-behind (opt-in): compress() returns before its files exist; after
// flush_writes() every file holds the bytes the write-through compress()
// writes, and decompress() flushes by itself before it reads.
static void write_behind_case() {
    const auto d1 = scratch(), d2 = scratch();
    std::vector<multiBox3D> boxes;
    for (int b = 0; b < 24; ++b) {
        multiBox3D mb;
        for (int c = 0; c < 3; ++c) {
            Box3D x(8 + 2 * (b % 3), 8, 16, 0.0f);
            for (int z = 0; z < 16; ++z)
                for (int y = 0; y < 8; ++y)
                    for (int i = 0; i < x.width(); ++i)
                        x.set(i, y, z, (float)(c * 100 + b) + 0.5f * (float)((i * 7 + y * 3 + z * 5 + b) % 11));
            mb.push_back(std::move(x));
        }
        boxes.push_back(std::move(mb));
    }
    for (int b = 0; b < 24; ++b) compress(boxes[b], {0, 1, 2}, 0.99, 0, 1, b, d1.string());
    wavelet_amd::set_write_behind(true);
    REQUIRE(wavelet_amd::write_behind());
    for (int b = 0; b < 24; ++b) compress(boxes[b], {0, 1, 2}, 0.99, 0, 1, b, d2.string());
    // decompress() of a queued file: complete before it is read
    Box3D r = decompress((d2 / "compressed-wavelet-0-1-2-23.xz").string(), 0, 1, 2, 23);
    Box3D w = decompress((d1 / "compressed-wavelet-0-1-2-23.xz").string(), 0, 1, 2, 23);
    REQUIRE(r.equals(w, 0));
    wavelet_amd::flush_writes();
    for (int b = 0; b < 24; ++b)
        for (int c = 0; c < 3; ++c) {
            const std::string name = "compressed-wavelet-0-1-" + std::to_string(c) + "-" + std::to_string(b) + ".xz";
            std::ifstream f1(d1 / name, std::ios::binary), f2(d2 / name, std::ios::binary);
            const std::string a((std::istreambuf_iterator<char>(f1)), std::istreambuf_iterator<char>());
            const std::string e((std::istreambuf_iterator<char>(f2)), std::istreambuf_iterator<char>());
            REQUIRE(!a.empty() && a == e);
        }
    wavelet_amd::set_write_behind(false);
    REQUIRE(!wavelet_amd::write_behind());
    std::filesystem::remove_all(d1);
    std::filesystem::remove_all(d2);
}

static void calc_rmse_case() {
    Box3D a(2, 2, 2, 0.0f), b(2, 2, 2, 3.5f);
    multiBox3D t1, t2;
    t1.push_back(a.clone());
    t2.push_back(b.clone());
    t1.push_back(a.clone());
    t2.push_back(b.clone());
    REQUIRE((calc_rmse_per_box(t1, t2, 2) == std::vector<double>{3.5, 3.5}));
    REQUIRE(calc_adj_loss(3.5, 7.0) == 0.5);
}

int main() {
    struct {
        const char* name;
        void (*fn)();
    } cases[] = {{"RLE Encode", rle_encode_case},
                 {"Serialization", serialization_case},
                 {"Wavelet decomposition", wavelet_case},
                 {"File writing/compression", file_writing_case},
                 {"Multi-component + quirks", multi_component_and_quirks_case},
                 {"Write-behind", write_behind_case},
                 {"Calc RMSE", calc_rmse_case}};
    for (auto& c : cases) {
        c.fn();
        std::printf("[ok] %s\n", c.name);
    }
    std::printf("%zu cases, %d checks passed\n", sizeof(cases) / sizeof(cases[0]), g_checks);
    return 0;
}

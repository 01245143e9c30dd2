// test_hostpipe.cpp — the host pipeline of the C-ABI (wavelet-compression_amd/
// csrc/wc_hostpipe.cpp: wc_forward_host / wc_inverse_host) on the CPU, against
// the fake HIP runtime and device stand-ins of tests/cpp/fake_device.cpp, for
// the ASan/UBSan and TSan builds (`make asan` / `make tsan`, run by
// tests/test_sanitizers.py).  No GPU: what runs is the pipeline's own code —
// unit runs, the three streams and their events, the helper and prefault
// threads, pinned bounce slots, the dense pack, the ticket-form retry — and
// its error paths, by injected failures of every runtime call it makes.
//
// Checks: bytes and offsets of the packed payloads and the decoded boxes
// equal a sequential host computation of the same stand-in codec, for 1 and
// 16 runs, pinned and pageable sources (bounce slots above 64 MiB), 0..8 host
// threads; an injected failure in any call returns its error code, leaves no
// copy running into the caller's buffers (ASan: the test frees them at once)
// and the next call on the same context succeeds.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fake_device.h"
#include "wc_ctx.h"

static int g_checks = 0, g_fail = 0;
#define CHECK(c, ...)                                               \
    do {                                                            \
        ++g_checks;                                                 \
        if (!(c)) {                                                 \
            ++g_fail;                                               \
            std::fprintf(stderr, "FAIL %s:%d %s: ", __FILE__, __LINE__, #c); \
            std::fprintf(stderr, __VA_ARGS__);                      \
            std::fprintf(stderr, "\n");                             \
        }                                                           \
    } while (0)

static wc_ctx* make_ctx() {
    wc_ctx* c = new wc_ctx();
    c->device = 0;
    if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) std::abort();
    c->stream = c->own;
    if (wc::ensure(c, c->errflag, 16) != WC_OK || hipMemset(c->errflag.p, 0, 16) != hipSuccess) std::abort();
    return c;
}

static void destroy_ctx(wc_ctx* c) {
    for (hipStream_t s : {c->stream, c->up, c->down})
        if (s) (void)hipStreamSynchronize(s);
    c->plan.d_units.p = nullptr;  // the fake's own tables
    for (wc::DevBuf* b : {&c->errflag, &c->h_cells, &c->h_payload, &c->h_packed, &c->h_offsets, &c->h_poff, &c->h_kept,
                          &c->h_out, &c->h_rows, &c->h_rmse})
        if (b->p) (void)hipFree(b->p);
    for (hipEvent_t e : c->hev) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->bev) (void)hipEventDestroy(e);
    if (c->up) (void)hipStreamDestroy(c->up);
    if (c->down) (void)hipStreamDestroy(c->down);
    if (c->pinned) (void)hipHostFree(c->pinned);
    if (c->bounce) (void)hipHostFree(c->bounce);
    (void)hipStreamDestroy(c->own);
    fake::release_context_tables(c);
    delete c;
}

struct Batch {
    std::vector<wc_unit> units;
    uint64_t extent = 0;
    std::vector<double> cells;
};

// n units of assorted shapes, packed back to back (4-element aligned), a few
// empty ones and one gap between units (cells no unit owns)
static Batch make_batch(int n, uint64_t scale) {
    Batch b;
    uint64_t off = 0;
    for (int i = 0; i < n; ++i) {
        int W = 2 + (int)((i * 7) % 9), H = 2 + (int)((i * 3) % 5), D = 2 + (int)((i * 5) % 7);
        if (i % 11 == 10) W = 0;  // an empty unit
        D = (int)(D * scale);
        b.units.push_back(wc_unit{off, W, H, D, 0});
        off += ((uint64_t)W * H * D + 3) & ~3ull;
        if (i == n / 2) off += 8;  // a gap
    }
    b.extent = off;
    b.cells.resize(off);
    for (uint64_t j = 0; j < off; ++j) b.cells[j] = 0.25 * (double)(j % 1000) - 17.0;
    return b;
}

// the packed payload a correct pipeline returns: units back to back from 4
static std::vector<uint8_t> expected_payload(const Batch& b, std::vector<uint64_t>& offs, std::vector<uint32_t>& kept) {
    std::vector<uint8_t> out(4, 0);
    offs.assign(b.units.size() + 1, 0);
    kept.assign(b.units.size(), 0);
    for (size_t i = 0; i < b.units.size(); ++i) {
        offs[i] = out.size();
        std::vector<uint8_t> p = fake::payload_of(b.units[i], b.cells.data(), WC_F64);
        kept[i] = fake::kept_of(b.units[i]);
        out.insert(out.end(), p.begin(), p.end());
        if (i + 1 < b.units.size()) out.insert(out.end(), 4, 0);
    }
    offs[b.units.size()] = out.size();
    return out;
}

static std::vector<float> expected_boxes(const Batch& b, float fill) {
    std::vector<float> out(b.extent, fill);
    for (const wc_unit& u : b.units) {
        const uint64_t nc = (uint64_t)u.nx * u.ny * u.nz, k = fake::kept_of(u);
        for (uint64_t j = 0; j < nc; ++j) out[u.cell_offset + j] = j < k ? (float)b.cells[u.cell_offset + j] : 0.0f;
    }
    return out;
}

// one forward + inverse over the host entry points, checked
static void round_trip(wc_ctx* c, const Batch& b, const double* cells, const char* what) {
    const int n = (int)b.units.size();
    std::vector<uint64_t> woff;
    std::vector<uint32_t> wkept;
    const std::vector<uint8_t> want = expected_payload(b, woff, wkept);
    const uint64_t cap = wc_payload_bound(b.units.data(), n);
    std::vector<uint8_t> pay(cap, 0xEE);
    std::vector<uint64_t> offs(n + 1, 7);
    std::vector<uint32_t> kept(n, 7);
    int rc = wc_forward_host(c, cells, WC_F64, b.units.data(), n, 0.999, pay.data(), cap, offs.data(), kept.data());
    CHECK(rc == WC_OK, "%s: forward rc %d (%s)", what, rc, c->err.c_str());
    if (rc) return;
    CHECK(offs == woff, "%s: offsets", what);
    CHECK(kept == wkept, "%s: kept", what);
    bool same = true;
    for (int i = 0; i < n && same; ++i)
        same = std::memcmp(pay.data() + woff[i], want.data() + woff[i], 20 + 8ull * wkept[i]) == 0;
    CHECK(same, "%s: payload bytes", what);
    {  // the same units, each from its own pointer (the drop-in compress()'s call)
        std::vector<const void*> ptrs(n);
        for (int i = 0; i < n; ++i) ptrs[i] = cells + b.units[i].cell_offset;
        std::vector<uint8_t> pay2(cap, 0xDD);
        std::vector<uint64_t> offs2(n + 1, 7);
        std::vector<uint32_t> kept2(n, 7);
        rc = wc_forward_host_units(c, ptrs.data(), WC_F64, b.units.data(), n, 0.999, pay2.data(), cap, offs2.data(),
                                   kept2.data());
        CHECK(rc == WC_OK, "%s: forward_host_units rc %d (%s)", what, rc, c->err.c_str());
        bool same2 = rc == WC_OK && offs2 == woff && kept2 == wkept;
        for (int i = 0; i < n && same2; ++i)
            same2 = std::memcmp(pay2.data() + woff[i], want.data() + woff[i], 20 + 8ull * wkept[i]) == 0;
        CHECK(same2, "%s: forward_host_units bytes", what);
    }
    {  // the -estimate round trip: the same payloads, and each unit's RMSE against its decoded boxes
        std::vector<uint8_t> pay3(cap, 0xCC);
        std::vector<uint64_t> offs3(n + 1, 7);
        std::vector<uint32_t> kept3(n, 7);
        std::vector<double> rmse(n, -1.0);
        rc = wc_round_trip_host(c, cells, WC_F64, b.units.data(), n, 0.999, pay3.data(), cap, offs3.data(),
                                kept3.data(), rmse.data());
        CHECK(rc == WC_OK, "%s: round_trip_host rc %d (%s)", what, rc, c->err.c_str());
        bool same3 = rc == WC_OK && offs3 == woff && kept3 == wkept;
        for (int i = 0; i < n && same3; ++i)
            same3 = std::memcmp(pay3.data() + woff[i], want.data() + woff[i], 20 + 8ull * wkept[i]) == 0;
        CHECK(same3, "%s: round_trip_host bytes", what);
        const std::vector<float> box = expected_boxes(b, 0.0f);
        bool rm = rc == WC_OK;
        for (int i = 0; i < n && rm; ++i) {
            const wc_unit& u = b.units[i];
            const uint64_t nc = (uint64_t)u.nx * u.ny * u.nz;
            double s = 0.0;
            for (uint64_t j = 0; j < nc; ++j) {
                const float d = (float)b.cells[u.cell_offset + j] - box[u.cell_offset + j];
                s += (double)d * (double)d;
            }
            rm = rmse[i] == (nc ? std::sqrt(s / (double)nc) : 0.0);
        }
        CHECK(rm, "%s: round_trip_host rmse", what);
    }
    std::vector<float> out(b.extent, -3.0f);
    rc = wc_inverse_host(c, pay.data(), offs.data(), b.units.data(), n, out.data());
    CHECK(rc == WC_OK, "%s: inverse rc %d (%s)", what, rc, c->err.c_str());
    CHECK(out == expected_boxes(b, -3.0f), "%s: boxes (gap cells untouched)", what);
}

static void test_runs_and_threads() {
    const Batch b = make_batch(60, 1);
    for (int64_t chunk : {0, 64, 1 << 25})
        for (int threads : {0, 1, 3, 8})
            for (int thp : {0, 1}) {
                wc_ctx* c = make_ctx();
                c->opt_host_chunk = chunk;
                c->opt_host_threads = threads;
                c->opt_host_thp = thp != 0;
                const std::string w = "chunk " + std::to_string(chunk) + " threads " + std::to_string(threads) +
                                      " thp " + std::to_string(thp);
                round_trip(c, b, b.cells.data(), w.c_str());
                round_trip(c, b, b.cells.data(), (w + " (again)").c_str());
                destroy_ctx(c);
            }
}

// >= 64 MiB of pageable cells: the uploads go through the pinned bounce slots;
// the same cells from pinned memory go straight to the copy engine
static void test_bounce_slots() {
    const Batch b = make_batch(24, 4096);  // ~95 MB of fp64 cells
    CHECK(b.extent * 8 > (64u << 20), "batch too small for the bounce path: %llu", (unsigned long long)b.extent);
    wc_ctx* c = make_ctx();
    c->opt_host_threads = 4;
    c->opt_host_chunk = 0;  // one run: one upload of all cells
    round_trip(c, b, b.cells.data(), "bounce");
    CHECK(c->bounce != nullptr, "bounce slots were not used");
    c->opt_host_chunk = 1 << 22;  // runs of >= 64 MiB: bounce slots reused across runs and calls
    round_trip(c, b, b.cells.data(), "bounce, runs");
    double* pinned = nullptr;
    if (hipHostMalloc((void**)&pinned, 8 * b.extent, hipHostMallocDefault) == hipSuccess) {
        std::memcpy(pinned, b.cells.data(), 8 * b.extent);
        round_trip(c, b, pinned, "pinned source");
        (void)hipHostFree(pinned);
    }
    // no pinned memory for the slots: the runtime's own copy path
    wc_ctx* d = make_ctx();
    d->opt_host_threads = 4;
    fake::fail_nth("hipHostMalloc", 2);  // the first is the pinned metadata block
    round_trip(d, b, b.cells.data(), "bounce slots unavailable");
    fake::clear_failures();
    destroy_ctx(d);
    destroy_ctx(c);
}

// Every call of the pipeline can fail: the call returns the error, no copy
// outlives it (the buffers are freed at once: ASan), and the context works again.
static void test_failures() {
    const Batch b = make_batch(40, 64);
    const int n = (int)b.units.size();
    const char* apis[] = {"H2D",          "D2H",          "hipEventRecord", "hipStreamWaitEvent", "hipEventSynchronize",
                          "hipMalloc",    "launch_pack",  "wc_forward",     "wc_inverse",         "hipStreamSynchronize",
                          "hipSetDevice", "hipEventCreateWithFlags", "wc_rmse"};
    for (const char* api : apis)
        for (int k : {1, 2, 5})
            for (int64_t chunk : {0, 1 << 12}) {
                wc_ctx* c = make_ctx();
                c->opt_host_threads = 2;
                c->opt_host_chunk = chunk;
                const std::string w = std::string(api) + " #" + std::to_string(k) + " chunk " + std::to_string(chunk);
                {
                    const uint64_t cap = wc_payload_bound(b.units.data(), n);
                    std::vector<uint8_t> pay(cap);
                    std::vector<uint64_t> offs(n + 1);
                    std::vector<uint32_t> kept(n);
                    std::vector<float> out(b.extent);
                    fake::fail_nth(api, k);
                    const int rf = wc_forward_host(c, b.cells.data(), WC_F64, b.units.data(), n, 0.999, pay.data(), cap,
                                                   offs.data(), kept.data());
                    int ri = rf ? rf : wc_inverse_host(c, pay.data(), offs.data(), b.units.data(), n, out.data());
                    std::vector<double> rmse(n);
                    if (!ri)
                        ri = wc_round_trip_host(c, b.cells.data(), WC_F64, b.units.data(), n, 0.999, pay.data(), cap,
                                                offs.data(), kept.data(), rmse.data());
                    fake::clear_failures();
                    CHECK(ri == WC_OK || ri == WC_ERR_HIP || ri == WC_ERR_NOMEM, "%s: rc %d", w.c_str(), ri);
                    CHECK(ri == WC_OK || !c->err.empty(), "%s: no message", w.c_str());
                }  // the caller's buffers are gone: a copy still running would write into freed memory
                round_trip(c, b, b.cells.data(), (w + " then").c_str());
                destroy_ctx(c);
            }
}

// An error a kernel raises in one run of a pipelined _host call (the word is
// read at the call's end) fails the call after every copy has drained; the
// next call of the context succeeds.
static void test_kernel_error() {
    const Batch b = make_batch(30, 8);
    wc_ctx* c = make_ctx();
    c->opt_host_chunk = 1 << 10;
    const int n = (int)b.units.size();
    const uint64_t cap = wc_payload_bound(b.units.data(), n);
    {
        std::vector<uint8_t> pay(cap);
        std::vector<uint64_t> offs(n + 1);
        std::vector<uint32_t> kept(n);
        fake::kernel_error_calls = 1;
        const int rc = wc_forward_host(c, b.cells.data(), WC_F64, b.units.data(), n, 0.999, pay.data(), cap,
                                       offs.data(), kept.data());
        CHECK(rc == WC_ERR_FORMAT, "kernel error: rc %d", rc);
        CHECK(fake::kernel_error_calls == 0, "the error was not raised");
    }  // the caller's buffers are gone: a copy still running would write into freed memory
    round_trip(c, b, b.cells.data(), "after a kernel error");
    destroy_ctx(c);
}

static void test_argument_errors() {
    const Batch b = make_batch(5, 1);
    wc_ctx* c = make_ctx();
    const int n = (int)b.units.size();
    std::vector<uint8_t> pay(wc_payload_bound(b.units.data(), n));
    std::vector<uint64_t> offs(n + 1);
    std::vector<uint32_t> kept(n);
    CHECK(wc_forward_host(c, b.cells.data(), WC_F64, b.units.data(), n, 0.999, pay.data(), pay.size() - 1, offs.data(),
                          kept.data()) == WC_ERR_INVALID, "capacity");
    CHECK(wc_forward_host(c, nullptr, WC_F64, b.units.data(), n, 0.999, pay.data(), pay.size(), offs.data(),
                          kept.data()) == WC_ERR_INVALID, "null cells");
    CHECK(wc_forward_host(c, b.cells.data(), 7, b.units.data(), n, 0.999, pay.data(), pay.size(), offs.data(),
                          kept.data()) == WC_ERR_INVALID, "dtype");
    std::vector<uint64_t> odd(n, 6);
    std::vector<float> out(b.extent);
    CHECK(wc_inverse_host(c, pay.data(), odd.data(), b.units.data(), n, out.data()) == WC_ERR_INVALID, "offsets not multiples of 4");
    destroy_ctx(c);
}

int main() {
    test_argument_errors();
    test_runs_and_threads();
    test_kernel_error();
    test_failures();
    test_bounce_slots();
    std::printf("test_hostpipe: %d checks, %d failed, %ld fake runtime calls, %zu allocations left\n", g_checks, g_fail,
                fake::calls(), fake::live_allocations());
    return g_fail ? 1 : 0;
}

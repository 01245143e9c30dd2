// fake_device.cpp — test infrastructure for tests/cpp/test_hostpipe.cpp: a CPU
// implementation of the HIP runtime calls declared in fakehip/hip/hip_runtime.h,
// and CPU stand-ins for the device entry points the host pipeline calls
// (wc_forward, launch_pack, wc_inverse, ...), running on the fake streams.
//
// The stand-in "codec" is NOT the wavelet codec: a unit keeps its first
// kept_of(unit) cells as (run 0, value) pairs in the real payload
// layout (src/compressor.cpp:55-80), and the inverse is rle_decode of those
// pairs into zeroed boxes (src/decompressor.cpp:14-30) without a transform.
// What is under test is the pipeline around it: runs, streams, events, helper
// threads, bounce slots, destination prefault, packing, error paths.  Fault
// injection: fake::fail_nth(api, k) makes the k-th next call of `api` fail.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fake_device.h"
#include "wc_ctx.h"

// ---------------------------------------------------------------------------
// the fake runtime

struct FakeEvent {
    std::mutex mu;
    std::condition_variable cv;
    uint64_t recorded = 0, completed = 0;
};

struct FakeStream {
    std::mutex mu;
    std::condition_variable cv, idle;
    std::deque<std::function<void()>> q;
    bool stop = false, busy = false;
    std::thread th;
    FakeStream() : th([this] { loop(); }) {}
    ~FakeStream() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        th.join();
    }
    void loop() {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return stop || !q.empty(); });
            if (q.empty()) return;
            std::function<void()> f = std::move(q.front());
            q.pop_front();
            busy = true;
            lk.unlock();
            f();
            lk.lock();
            busy = false;
            if (q.empty()) idle.notify_all();
        }
    }
    void push(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> lk(mu);
            q.push_back(std::move(f));
        }
        cv.notify_all();
    }
    void drain() {
        std::unique_lock<std::mutex> lk(mu);
        idle.wait(lk, [&] { return q.empty() && !busy; });
    }
};

namespace {

std::mutex g_mu;
struct Alloc {
    size_t bytes;
    hipMemoryType type;
};
std::map<uintptr_t, Alloc> g_allocs;      // live hipMalloc / hipHostMalloc ranges
std::vector<FakeStream*> g_streams;       // live streams (hipFree drains them all)
thread_local hipError_t t_last = hipSuccess;
std::map<std::string, int> g_fail;        // api -> calls left until the injected failure
std::atomic<long> g_calls{0};

FakeStream* default_stream() {
    static FakeStream* s = [] {
        auto* p = new FakeStream();
        std::lock_guard<std::mutex> lk(g_mu);
        g_streams.push_back(p);
        return p;
    }();
    return s;
}

FakeStream* S(hipStream_t s) { return s ? s : default_stream(); }

bool injected(const char* api) {
    ++g_calls;
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_fail.find(api);
    if (it == g_fail.end()) return false;
    if (--it->second > 0) return false;
    g_fail.erase(it);
    return true;
}

hipError_t ret(hipError_t e) {
    if (e != hipSuccess) t_last = e;
    return e;
}

hipMemoryType type_of(const void* p) {
    std::lock_guard<std::mutex> lk(g_mu);
    const uintptr_t a = (uintptr_t)p;
    auto it = g_allocs.upper_bound(a);
    if (it == g_allocs.begin()) return hipMemoryTypeUnregistered;
    --it;
    return a < it->first + it->second.bytes ? it->second.type : hipMemoryTypeUnregistered;
}

void* alloc(size_t bytes, hipMemoryType t) {
    const size_t b = (std::max<size_t>(bytes, 1) + 255) & ~size_t(255);
    void* p = std::aligned_alloc(256, b);
    if (!p) return nullptr;
    std::lock_guard<std::mutex> lk(g_mu);
    g_allocs[(uintptr_t)p] = Alloc{b, t};
    return p;
}

hipError_t release(void* p, hipMemoryType t) {
    if (!p) return hipSuccess;
    std::vector<FakeStream*> ss;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_allocs.find((uintptr_t)p);
        if (it == g_allocs.end() || it->second.type != t) return ret(hipErrorInvalidValue);
        ss = g_streams;
    }
    for (FakeStream* s : ss) s->drain();  // as hipFree: no queued work may still use it
    {
        std::lock_guard<std::mutex> lk(g_mu);
        g_allocs.erase((uintptr_t)p);
    }
    std::free(p);
    return hipSuccess;
}

// Run f on stream s; a copy touching pageable host memory returns only when done.
void enqueue(hipStream_t s, std::function<void()> f, bool blocking) {
    FakeStream* st = S(s);
    if (!blocking) {
        st->push(std::move(f));
        return;
    }
    auto done = std::make_shared<std::pair<std::mutex, std::condition_variable>>();
    auto flag = std::make_shared<bool>(false);
    st->push([f = std::move(f), done, flag] {
        f();
        std::lock_guard<std::mutex> lk(done->first);
        *flag = true;
        done->second.notify_all();
    });
    std::unique_lock<std::mutex> lk(done->first);
    done->second.wait(lk, [&] { return *flag; });
}

}  // namespace

namespace fake {
void fail_nth(const char* api, int k) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_fail[api] = k;
}
void clear_failures() {
    std::lock_guard<std::mutex> lk(g_mu);
    g_fail.clear();
}
long calls() { return g_calls.load(); }
size_t live_allocations() {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_allocs.size();
}
}  // namespace fake

hipError_t hipMalloc(void** p, size_t bytes) {
    if (injected("hipMalloc")) return ret(hipErrorOutOfMemory);
    *p = alloc(bytes, hipMemoryTypeDevice);
    return *p ? hipSuccess : ret(hipErrorOutOfMemory);
}
hipError_t hipFree(void* p) { return release(p, hipMemoryTypeDevice); }
hipError_t hipHostMalloc(void** p, size_t bytes, unsigned) {
    if (injected("hipHostMalloc")) return ret(hipErrorOutOfMemory);
    *p = alloc(bytes, hipMemoryTypeHost);
    return *p ? hipSuccess : ret(hipErrorOutOfMemory);
}
hipError_t hipHostFree(void* p) { return release(p, hipMemoryTypeHost); }

hipError_t hipMemcpyAsync(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s) {
    const char* api = kind == hipMemcpyHostToDevice ? "H2D" : kind == hipMemcpyDeviceToHost ? "D2H" : "memcpy";
    if (injected(api) || injected("hipMemcpyAsync")) return ret(hipErrorUnknown);
    const bool pageable = (kind == hipMemcpyHostToDevice && type_of(src) == hipMemoryTypeUnregistered) ||
                          (kind == hipMemcpyDeviceToHost && type_of(dst) == hipMemoryTypeUnregistered);
    enqueue(s, [=] { std::memcpy(dst, src, bytes); }, pageable);
    return hipSuccess;
}
hipError_t hipMemsetAsync(void* dst, int v, size_t bytes, hipStream_t s) {
    if (injected("hipMemsetAsync")) return ret(hipErrorUnknown);
    enqueue(s, [=] { std::memset(dst, v, bytes); }, false);
    return hipSuccess;
}
hipError_t hipMemset(void* dst, int v, size_t bytes) {
    enqueue(nullptr, [=] { std::memset(dst, v, bytes); }, true);
    return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned) {
    if (injected("hipStreamCreateWithFlags")) return ret(hipErrorUnknown);
    auto* p = new FakeStream();
    std::lock_guard<std::mutex> lk(g_mu);
    g_streams.push_back(p);
    *s = p;
    return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
    if (!s) return ret(hipErrorInvalidValue);
    s->drain();
    {
        std::lock_guard<std::mutex> lk(g_mu);
        g_streams.erase(std::remove(g_streams.begin(), g_streams.end(), s), g_streams.end());
    }
    delete s;
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t s) {
    if (injected("hipStreamSynchronize")) return ret(hipErrorUnknown);
    S(s)->drain();
    return hipSuccess;
}
hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned) {
    if (injected("hipStreamWaitEvent")) return ret(hipErrorUnknown);
    uint64_t gen;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        gen = e->recorded;
    }
    enqueue(s, [e, gen] {
        std::unique_lock<std::mutex> lk(e->mu);
        e->cv.wait(lk, [&] { return e->completed >= gen; });
    }, false);
    return hipSuccess;
}
hipError_t hipEventCreate(hipEvent_t* e) {
    *e = new FakeEvent();
    return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
    if (injected("hipEventCreateWithFlags")) return ret(hipErrorUnknown);
    *e = new FakeEvent();
    return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e) {
    hipEventSynchronize(e);
    delete e;
    return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) {
    if (injected("hipEventRecord")) return ret(hipErrorUnknown);
    uint64_t gen;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        gen = ++e->recorded;
    }
    enqueue(s, [e, gen] {
        std::lock_guard<std::mutex> lk(e->mu);
        e->completed = std::max(e->completed, gen);
        e->cv.notify_all();
    }, false);
    return hipSuccess;
}
hipError_t hipEventSynchronize(hipEvent_t e) {
    if (injected("hipEventSynchronize")) return ret(hipErrorUnknown);
    std::unique_lock<std::mutex> lk(e->mu);
    const uint64_t gen = e->recorded;
    e->cv.wait(lk, [&] { return e->completed >= gen; });
    return hipSuccess;
}
hipError_t hipPointerGetAttributes(hipPointerAttribute_t* a, const void* p) {
    const hipMemoryType t = type_of(p);
    if (t == hipMemoryTypeUnregistered) return ret(hipErrorInvalidValue);
    *a = hipPointerAttribute_t{t, 0, (void*)p, (void*)p, 0, 0};
    return hipSuccess;
}
hipError_t hipGetLastError(void) {
    const hipError_t e = t_last;
    t_last = hipSuccess;
    return e;
}
hipError_t hipSetDevice(int d) {
    if (injected("hipSetDevice")) return ret(hipErrorUnknown);
    return d == 0 ? hipSuccess : ret(hipErrorInvalidValue);
}
hipError_t hipGetDevice(int* d) {
    *d = 0;
    return hipSuccess;
}
hipError_t hipGetDeviceCount(int* n) {
    *n = 1;
    return hipSuccess;
}
const char* hipGetErrorString(hipError_t e) {
    switch (e) {
        case hipSuccess: return "no error";
        case hipErrorInvalidValue: return "invalid argument (fake)";
        case hipErrorOutOfMemory: return "out of memory (fake)";
        default: return "injected failure (fake)";
    }
}

// ---------------------------------------------------------------------------
// stand-ins for the device entry points (the kernels' side of the pipeline)

namespace fake {
int kernel_error_calls = 0;  // the next k wc_forward calls raise a kernel-detected error (malformed header)

// unit u keeps its first kept_of(u) cells (a function of its shape alone: not
// of its run, nor of where its cells sit)
uint32_t kept_of(const wc_unit& u) {
    const uint64_t cells = (uint64_t)u.nx * u.ny * u.nz;
    return (uint32_t)((cells * ((uint64_t)(u.nx + 2 * u.ny + 3 * u.nz) % 5)) / 7);
}

std::vector<uint8_t> payload_of(const wc_unit& u, const void* cells, int dtype) {
    const uint64_t nc = (uint64_t)u.nx * u.ny * u.nz;
    const uint32_t k = kept_of(u);
    std::vector<uint8_t> out(20 + 8ull * k);
    const int32_t hdr[5] = {u.nx, u.ny, u.nz, (int32_t)nc, (int32_t)k};
    std::memcpy(out.data(), hdr, 20);
    for (uint32_t j = 0; j < k; ++j) {
        const float v = dtype == WC_F64 ? (float)((const double*)cells)[u.cell_offset + j]
                                        : ((const float*)cells)[u.cell_offset + j];
        const int32_t run = 0;
        std::memcpy(out.data() + 20 + 8ull * j, &run, 4);
        std::memcpy(out.data() + 24 + 8ull * j, &v, 4);
    }
    return out;
}
}  // namespace fake

namespace {
// descriptor tables of the calls, alive until the context is torn down
std::mutex g_tab_mu;
std::map<const wc_ctx*, std::vector<std::shared_ptr<std::vector<wc::UnitDev>>>> g_tabs;
}  // namespace

namespace fake {
void release_context_tables(const wc_ctx* c) {
    std::lock_guard<std::mutex> lk(g_tab_mu);
    g_tabs.erase(c);
}
}  // namespace fake

namespace wc {
hipError_t launch_pack(hipStream_t st, const UnitDev* units, int n, const uint32_t* kept, const uint8_t* src,
                       uint64_t* packed, uint8_t* dst) {
    if (injected("launch_pack")) return ret(hipErrorUnknown);
    enqueue(st, [=] {
        uint64_t off = 4;
        for (int u = 0; u < n; ++u) {
            packed[u] = off;
            std::memcpy(dst + off, src + units[u].pay_off, 20 + 8ull * kept[u]);
            off += 24 + 8ull * kept[u];
        }
        packed[n] = n ? packed[n - 1] + 20 + 8ull * kept[n - 1] : 4;
    }, false);
    return hipSuccess;
}
}  // namespace wc

using namespace wc;

extern "C" {

int wc_forward(wc_ctx* c, const void* d_cells, int dtype, const wc_unit* units, int n, double, uint8_t* d_payload,
               uint64_t cap, uint64_t* d_offsets, uint32_t* d_kept) {
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (n == 0) return WC_OK;
    if (cap < wc_payload_bound(units, n)) return fail(c, WC_ERR_INVALID, "payload_capacity < wc_payload_bound");
    if (injected("wc_forward")) return fail(c, WC_ERR_HIP, "wc_forward: injected launch failure (fake)");
    auto tab = std::make_shared<std::vector<UnitDev>>(n);
    uint64_t slot = 4;
    for (int i = 0; i < n; ++i) {
        (*tab)[i].pay_off = slot;
        slot += 24 + 8ull * units[i].nx * units[i].ny * units[i].nz;
    }
    {
        std::lock_guard<std::mutex> lk(g_tab_mu);
        g_tabs[c].push_back(tab);
    }
    c->plan.d_units.p = tab->data();  // launch_pack reads the slots from here
    std::vector<wc_unit> us(units, units + n);
    const bool kerr = fake::kernel_error_calls > 0;
    if (kerr) --fake::kernel_error_calls;
    uint32_t* err = (uint32_t*)c->errflag.p;
    enqueue(c->stream, [=] {
        for (int i = 0; i < n; ++i) {
            std::vector<uint8_t> p = fake::payload_of(us[i], d_cells, dtype);
            std::memcpy(d_payload + (*tab)[i].pay_off, p.data(), p.size());
            d_offsets[i] = (*tab)[i].pay_off;
            d_kept[i] = fake::kept_of(us[i]);
        }
        d_offsets[n] = d_offsets[n - 1] + 20 + 8ull * d_kept[n - 1];
        if (kerr) *err |= kErrHeader;
    }, false);
    c->err_check_pending = true;
    return WC_OK;
}

int wc_inverse(wc_ctx* c, const uint8_t* d_payload, const uint64_t* d_offsets, const wc_unit* units, int n,
               float* d_out) {
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (n == 0) return WC_OK;
    if (injected("wc_inverse")) return fail(c, WC_ERR_HIP, "wc_inverse: injected launch failure (fake)");
    std::vector<wc_unit> us(units, units + n);
    enqueue(c->stream, [=] {
        for (int i = 0; i < n; ++i) {
            const uint8_t* ph = d_payload + d_offsets[i];
            int32_t hdr[5];
            std::memcpy(hdr, ph, 20);
            const uint64_t nc = (uint64_t)us[i].nx * us[i].ny * us[i].nz;
            float* o = d_out + us[i].cell_offset;
            std::fill(o, o + nc, 0.0f);
            uint64_t idx = 0;
            for (int32_t k = 0; k < hdr[4]; ++k) {  // rle_decode, src/decompressor.cpp:14-30
                int32_t run;
                float v;
                std::memcpy(&run, ph + 20 + 8ull * k, 4);
                std::memcpy(&v, ph + 24 + 8ull * k, 4);
                idx += (uint64_t)run;
                if (idx < nc) o[idx++] = v;
            }
        }
    }, false);
    return WC_OK;
}

// wc_round_trip_host's calls: the row index is the device's business (the
// stand-in inverse decodes from the payloads), the RMSE is calc_rmse_per_box's
int wc_forward_rows(wc_ctx* c, const void* d_cells, int dtype, const wc_unit* units, int n, double keep,
                    uint8_t* d_payload, uint64_t cap, uint64_t* d_offsets, uint32_t* d_kept, void* d_rowinfo,
                    uint64_t rowinfo_capacity) {
    if (!d_rowinfo || rowinfo_capacity < wc_rowindex_bytes(units, n)) return fail(c, WC_ERR_INVALID, "fake: rows");
    return wc_forward(c, d_cells, dtype, units, n, keep, d_payload, cap, d_offsets, d_kept);
}

int wc_inverse_rows(wc_ctx* c, const uint8_t* d_payload, const uint64_t* d_offsets, const wc_unit* units, int n,
                    const void* d_rowinfo, uint64_t rowinfo_capacity, const void* d_orig, int, float* d_out, double*) {
    if (d_orig) return fail(c, WC_ERR_INVALID, "fake: fused RMSE");
    if (d_rowinfo && rowinfo_capacity < wc_rowindex_bytes(units, n)) return fail(c, WC_ERR_INVALID, "fake: rows");
    return wc_inverse(c, d_payload, d_offsets, units, n, d_out);
}

int wc_rmse(wc_ctx* c, const void* d_orig, int dtype, const float* d_regen, const wc_unit* units, int n,
            double* d_rmse) {
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (injected("wc_rmse")) return fail(c, WC_ERR_HIP, "wc_rmse: injected launch failure (fake)");
    std::vector<wc_unit> us(units, units + n);
    enqueue(c->stream, [=] {
        for (int i = 0; i < n; ++i) {
            const uint64_t nc = (uint64_t)us[i].nx * us[i].ny * us[i].nz;
            double s = 0.0;
            for (uint64_t j = 0; j < nc; ++j) {
                const uint64_t o = us[i].cell_offset + j;
                const float a = dtype == WC_F64 ? (float)((const double*)d_orig)[o] : ((const float*)d_orig)[o];
                const float d = a - d_regen[o];
                s += (double)d * (double)d;
            }
            d_rmse[i] = nc ? std::sqrt(s / (double)nc) : 0.0;
        }
    }, false);
    return WC_OK;
}

// the transform-only _host wrappers are not what this test covers
int wc_decompose(wc_ctx* c, const void*, int, const wc_unit*, int, float*) {
    return fail(c, WC_ERR_INVALID, "fake: wc_decompose");
}
int wc_inverse_flat(wc_ctx* c, const float*, const wc_unit*, int, float*) {
    return fail(c, WC_ERR_INVALID, "fake: wc_inverse_flat");
}

}  // extern "C"

// wc_hostpipe.cpp — the _host entry points of the C-ABI (include/wavelet_amd.h):
// host buffers in, host buffers out, over PCIe.
//
// A batch runs as up to 16 contiguous unit runs pipelined over three streams
// (upload, compute = the context stream, download); downloads run on a helper
// thread of the call beside the uploads (a copy from or to pageable memory
// returns only when it is done); large pageable uploads go through pinned
// bounce slots filled by a host pool; each download's destination pages are
// faulted in first (wc_hostmem.h).  The compute is the device entry points
// (wc_forward, wc_inverse, ...): this file launches no kernel of its own
// except the dense pack, and is also built against a CPU fake of the HIP
// runtime for the ASan/TSan tests of its concurrency and error paths
// (tests/cpp/test_hostpipe.cpp).
#include "wc_ctx.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

using namespace wc;

// ---- host-pointer variants -------------------------------------------------

// Unit runs of the host-buffer paths: boundaries rb[0] = 0 < ... < rb[nr] = n,
// runs of about opt_host_chunk cells (at least total / 16), one run unless the
// batch holds more than two chunks (or opt_host_chunk <= 0).
static std::vector<int> host_runs(const wc_ctx* c, const wc_unit* units, int n) {
    std::vector<int> rb{0};
    uint64_t total = 0;
    for (int i = 0; i < n; ++i) total += (uint64_t)units[i].nx * units[i].ny * units[i].nz;
    const uint64_t chunk =
        c->opt_host_chunk > 0 ? std::max<uint64_t>((uint64_t)c->opt_host_chunk, total / 16 + 1) : total + 1;
    if (total > 2 * chunk) {
        uint64_t acc = 0;
        for (int i = 0; i < n; ++i) {
            acc += (uint64_t)units[i].nx * units[i].ny * units[i].nz;
            if (acc >= chunk && i + 1 < n) {
                rb.push_back(i + 1);
                acc = 0;
            }
        }
    }
    rb.push_back(n);
    return rb;
}

// WCAMD_HOST_TRACE=1: the _host calls print their host-side timeline (ms
// since the call began) to stderr.  Diagnostic.
struct HostTrace {
    const bool on = std::getenv("WCAMD_HOST_TRACE") != nullptr;
    const std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    const char* call;
    explicit HostTrace(const char* name) : call(name) {}
    void operator()(const char* what, int r = -1) const {
        if (!on) return;
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::fprintf(stderr, "[%s] %8.2f ms %s %d\n", call, ms, what, r);
    }
};

// WC_OPT_HOST_THREADS unset: the job's CPU share (OMP_NUM_THREADS, 16 per GPU
// on the MI355X boxes, where nproc shows the whole host) or the cores, <= 16.
int wc::host_threads_default() {
    int t = 0;
    if (const char* e = std::getenv("OMP_NUM_THREADS")) t = std::atoi(e);
    if (t <= 0) t = (int)std::thread::hardware_concurrency();
    return std::clamp(t, 1, 16);
}

// Faulting in the pages of a host destination before a device-to-host copy
// lands there (wc_hostmem.h: the copy's own thread faults at 12–20 GB/s).
// Resolved on the call's thread before any helper thread starts; null = off.
struct Populate {
    wc::HostPool* pool = nullptr;
    bool on = false, thp = false;
    void operator()(void* p, size_t bytes) const {
        if (on && bytes) wc::populate_for_write(pool, p, bytes, thp);
    }
};

static Populate host_populate(wc_ctx* c) {
    if (c->opt_host_threads < 0) c->opt_host_threads = host_threads_default();
    Populate P;
    if (c->opt_host_threads == 0) return P;
    if (!c->hpool || c->hpool->threads() != c->opt_host_threads) {
        c->hpool.reset();
        try {
            c->hpool = std::make_unique<wc::HostPool>(c->opt_host_threads - 1);
        } catch (...) {  // no threads: the faults stay with the copies
            return P;
        }
    }
    P.pool = c->hpool.get();
    P.on = true;
    P.thp = c->opt_host_thp;
    return P;
}

// Is p pinned (or device) memory the DMA engines read directly?  A pageable
// pointer makes the query fail; its error is cleared so that no later launch
// check sees it.
static bool dma_ready(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost || a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged ||
           a.type == hipMemoryTypeUnified;
}

constexpr size_t kBounceSlot = size_t(16) << 20;  // bytes per pinned bounce slot
constexpr int kBounceSlots = 8;
constexpr int kBounceThreads = 8;                  // enough to outrun the link (~110 GB/s into pinned memory)

// Host-to-device copy of `bytes` from `src` on stream `st`.  Pinned (or
// device) sources and small copies go straight to the DMA engine.  A large
// pageable source goes through the context's pinned bounce slots: this
// thread's pool copies slot-sized pieces (8-16 threads: ~100 GB/s) while the
// previous pieces' DMA runs (57 GB/s), instead of the runtime pinning pages
// of a buffer it has not seen before (14-32 GB/s on the MI355X host,
// profiles/r04/experiments/gpu_host_prefault.txt).  Returns the first error.
static hipError_t host_upload(wc_ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st) {
    if (bytes < (size_t(64) << 20) || c->opt_host_threads == 0 || dma_ready(src))
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
    hipError_t e;
    if (!c->bounce) {
        if ((e = hipHostMalloc(&c->bounce, kBounceSlot * kBounceSlots, hipHostMallocDefault)) != hipSuccess) {
            c->bounce = nullptr;
            return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
        }
    }
    while ((int)c->bev.size() < kBounceSlots) {
        hipEvent_t ev;
        if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
        c->bev.push_back(ev);
        c->bev_live.push_back(false);
    }
    const int ut = std::min(c->opt_host_threads, kBounceThreads);
    if (!c->upool || c->upool->threads() != ut) {
        c->upool.reset();
        try {
            c->upool = std::make_unique<wc::HostPool>(ut - 1);
        } catch (...) {
            return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
        }
    }
    wc::HostPool& pool = *c->upool;
    for (size_t off = 0; off < bytes; off += kBounceSlot) {
        const int k = (int)(c->bnext++ % kBounceSlots);
        const size_t len = std::min(kBounceSlot, bytes - off);
        uint8_t* slot = (uint8_t*)c->bounce + kBounceSlot * k;
        // the slot's previous copy (this call's or an earlier one's) has been read
        if (c->bev_live[k] && (e = hipEventSynchronize(c->bev[k])) != hipSuccess) return e;
        const int T = pool.threads();
        const size_t per = (len / T + 4095) & ~size_t(4095);
        pool.run(T, [&](int i) {
            const size_t lo = std::min(len, per * i), hi = std::min(len, per * (i + 1));
            if (hi > lo) std::memcpy(slot + lo, (const uint8_t*)src + off + lo, hi - lo);
        });
        if ((e = hipMemcpyAsync((uint8_t*)dst + off, slot, len, hipMemcpyHostToDevice, st)) != hipSuccess ||
            (e = hipEventRecord(c->bev[k], st)) != hipSuccess)
            return e;
        c->bev_live[k] = true;
    }
    return hipSuccess;
}

// What a helper thread of a _host call ran into (applied to the context by
// the call's thread once the helper has joined).
struct HelperStatus {
    int rc = WC_OK;
    std::string msg;
    void hip(hipError_t e, const char* what) {
        if (rc == WC_OK) {
            rc = WC_ERR_HIP;
            msg = std::string(what) + ": " + hipGetErrorString(e);
        }
    }
    void invalid(const char* what) {
        if (rc == WC_OK) {
            rc = WC_ERR_INVALID;
            msg = what;
        }
    }
};

// Runs `body` on a helper thread (bound to the context's device) when the
// call has more than one run, else on the call's thread after `main`.
template <class Main, class Body>
static int with_helper(wc_ctx* c, int nr, wc::RunGate& gate, HelperStatus& hs, Main main, Body body) {
    std::thread helper;
    if (nr > 1) {
        try {
            helper = std::thread([&] {
                hipError_t e = hipSetDevice(c->device);
                if (e != hipSuccess) return hs.hip(e, "hipSetDevice (helper)");
                body();
            });
        } catch (...) {  // no thread: the body runs after main on this one
        }
    }
    const int rc = main();
    if (rc != WC_OK) gate.cancel();
    if (helper.joinable()) helper.join();
    else if (rc == WC_OK) body();
    if (rc != WC_OK || hs.rc != WC_OK) {
        // Copies queued before the failure may still read or write the
        // caller's buffers: none may outlive the call.
        for (hipStream_t st : {c->up, c->down, c->stream})
            if (st) (void)hipStreamSynchronize(st);
    }
    if (rc != WC_OK) return rc;
    if (hs.rc != WC_OK) return fail(c, hs.rc, hs.msg);
    return WC_OK;
}

// The copy streams (when there is more than one run) and 2 events per run.
static int host_streams(wc_ctx* c, int nr) {
    hipError_t e;
    if (nr > 1) {
        if (!c->up && (e = hipStreamCreateWithFlags(&c->up, hipStreamNonBlocking)) != hipSuccess)
            return hip_fail(c, e, "upload stream");
        if (!c->down && (e = hipStreamCreateWithFlags(&c->down, hipStreamNonBlocking)) != hipSuccess)
            return hip_fail(c, e, "download stream");
    }
    while ((int)c->hev.size() < 2 * nr) {
        hipEvent_t ev;
        if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return hip_fail(c, e, "event");
        c->hev.push_back(ev);
    }
    return WC_OK;
}

// Where a _host forward's cells come from: one host buffer at the units' cell
// offsets (wc_forward_host), or one host pointer per unit (wc_forward_host_units:
// the units' cell offsets are then the packed device layout).
struct CellSource {
    const uint8_t* base = nullptr;
    const void* const* per_unit = nullptr;
};

// rmse != null (wc_round_trip_host): each run's forward also writes its row
// index, and the run's payloads are decoded again on the device with it
// (wc_inverse_rows) and compared with the run's cells there (wc_rmse): the
// reconstruction never leaves the device, the cells cross PCIe once.
static int forward_host_once(wc_ctx* c, CellSource src, int dtype, const wc_unit* units, int n, double keep,
                             uint8_t* payload, uint64_t cap, uint64_t* offsets, uint32_t* kept, double* rmse) {
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (dtype != WC_F32 && dtype != WC_F64) return fail(c, WC_ERR_INVALID, "dtype");
    if (n == 0) return WC_OK;
    if ((!src.base && !src.per_unit) || !payload || !offsets || !kept) return fail(c, WC_ERR_INVALID, "null buffer");
    if (src.per_unit)
        for (int i = 0; i < n; ++i)
            if (!src.per_unit[i] && (uint64_t)units[i].nx * units[i].ny * units[i].nz)
                return fail(c, WC_ERR_INVALID, "null buffer (unit " + std::to_string(i) + ")");
    const uint64_t bound = wc_payload_bound(units, n);
    if (cap < bound) return fail(c, WC_ERR_INVALID, "payload_capacity < wc_payload_bound");
    if ((rc = set_device(c))) return rc;
    const size_t esz = dtype == WC_F64 ? 8 : 4;
    const uint64_t ext = cells_extent(units, n);
    const HostTrace mark("forward_host");

    // Runs of contiguous units of about opt_host_chunk cells (at most 16),
    // pipelined: run r's cells upload on `up` while run r-1 computes on the
    // context stream, and each run's packed payloads download on `down` once
    // its sizes are known.  The packed layout (== 4 mod 8 offsets) is the same
    // as one run's.
    std::vector<int> rb = host_runs(c, units, n);
    const int nr = (int)rb.size() - 1;
    // per run: payload slot base (device), metadata base (pinned): poff[n_r + 1] | kept[n_r]
    std::vector<uint64_t> pbase(nr + 1, 0);
    // (16-B aligned: each run's slots start like a device buffer's, pairs 8-B aligned)
    for (int r = 0; r < nr; ++r)
        pbase[r + 1] = round_up(pbase[r] + wc_payload_bound(units + rb[r], rb[r + 1] - rb[r]), 16);
    const size_t meta_bytes = sizeof(uint64_t) * (size_t)(n + nr) + 4ull * n;
    uint64_t rows_cap = 0;  // the largest run's row index (wc_round_trip_host)
    if (rmse) {
        for (int r = 0; r < nr; ++r) rows_cap = std::max(rows_cap, wc_rowindex_bytes(units + rb[r], rb[r + 1] - rb[r]));
        if ((rc = ensure(c, c->h_rows, rows_cap)) || (rc = ensure(c, c->h_out, sizeof(float) * ext)) ||
            (rc = ensure(c, c->h_rmse, sizeof(double) * n)))
            return rc;
    }
    if ((rc = ensure(c, c->h_cells, esz * ext)) || (rc = ensure(c, c->h_payload, pbase[nr])) ||
        (rc = ensure(c, c->h_packed, pbase[nr])) || (rc = ensure(c, c->h_offsets, sizeof(uint64_t) * (n + nr))) ||
        (rc = ensure(c, c->h_poff, sizeof(uint64_t) * (n + nr))) || (rc = ensure(c, c->h_kept, 4 * n)))
        return rc;
    hipError_t e = hipSuccess;
    if (c->pinned_bytes < meta_bytes) {
        if (c->pinned) (void)hipHostFree(c->pinned);
        c->pinned = nullptr;
        c->pinned_bytes = 0;
        if ((e = hipHostMalloc(&c->pinned, meta_bytes, hipHostMallocDefault)) != hipSuccess)
            return hip_fail(c, e, "pinned metadata");
        c->pinned_bytes = meta_bytes;
    }
    if ((rc = host_streams(c, nr))) return rc;
    uint64_t* pin_poff = (uint64_t*)c->pinned;                   // [n + nr]
    uint32_t* pin_kept = (uint32_t*)(pin_poff + (n + nr));       // [n]
    uint8_t* d_cells = (uint8_t*)c->h_cells.p;
    const Populate populate = host_populate(c);
    wc::RunGate gate;
    HelperStatus hs;
    uint64_t R = 4;  // run r's packed bytes [4, end) land at R (== 4 mod 8); the next run starts at R + end
    // The call's thread: uploads, kernels, each run's sizes to pinned memory.
    auto enqueue = [&]() -> int {
        for (int r = 0; r < nr; ++r) {
            const int a = rb[r], m = rb[r + 1] - rb[r];
            uint64_t lo = UINT64_MAX, hi = 0;
            for (int i = a; i < a + m; ++i) {
                const uint64_t cnt = (uint64_t)units[i].nx * units[i].ny * units[i].nz;
                if (!cnt) continue;
                lo = std::min(lo, units[i].cell_offset);
                hi = std::max(hi, units[i].cell_offset + cnt);
            }
            hipStream_t cs = nr > 1 ? c->up : c->stream;
            hipError_t e;
            if (src.base) {  // one span of the caller's buffer
                if (hi > lo &&
                    (e = host_upload(c, d_cells + esz * lo, src.base + esz * lo, esz * (hi - lo), cs)) != hipSuccess)
                    return hip_fail(c, e, "cells upload");
            } else {  // unit by unit, each from its own pointer
                for (int i = a; i < a + m; ++i) {
                    const uint64_t cnt = (uint64_t)units[i].nx * units[i].ny * units[i].nz;
                    if (cnt && (e = host_upload(c, d_cells + esz * units[i].cell_offset, src.per_unit[i], esz * cnt,
                                                cs)) != hipSuccess)
                        return hip_fail(c, e, "cells upload");
                }
            }
            if (nr > 1 && ((e = hipEventRecord(c->hev[2 * r], c->up)) != hipSuccess ||
                           (e = hipStreamWaitEvent(c->stream, c->hev[2 * r], 0)) != hipSuccess))
                return hip_fail(c, e, "upload event");
            uint8_t* pay = (uint8_t*)c->h_payload.p + pbase[r];
            uint8_t* packed = (uint8_t*)c->h_packed.p + pbase[r];
            uint64_t* doff = (uint64_t*)c->h_offsets.p + (a + r);
            uint64_t* dpoff = (uint64_t*)c->h_poff.p + (a + r);
            uint32_t* dkept = (uint32_t*)c->h_kept.p + a;
            int rc2;
            if ((rc2 = rmse ? wc_forward_rows(c, c->h_cells.p, dtype, units + a, m, keep, pay, pbase[r + 1] - pbase[r],
                                              doff, dkept, c->h_rows.p, rows_cap)
                            : wc_forward(c, c->h_cells.p, dtype, units + a, m, keep, pay, pbase[r + 1] - pbase[r], doff,
                                         dkept)))
                return rc2;
            // Pack the slots densely (offsets stay == 4 mod 8), sizes to pinned memory.
            e = launch_pack(c->stream, (const UnitDev*)c->plan.d_units.p, m, dkept, pay, dpoff, packed);
            if (e != hipSuccess) return hip_fail(c, e, "pack launch");
            if ((e = hipMemcpyAsync(pin_poff + (a + r), dpoff, sizeof(uint64_t) * (m + 1), hipMemcpyDeviceToHost,
                                    c->stream)) != hipSuccess ||
                (e = hipMemcpyAsync(pin_kept + a, dkept, 4ull * m, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
                (e = hipEventRecord(c->hev[2 * r + 1], c->stream)) != hipSuccess)
                return hip_fail(c, e, "sizes readback");
            gate.publish(r + 1);
            // the round trip: this run's payloads back to cells with the row
            // index just written, and calc_rmse_per_box against its cells
            if (rmse && ((rc2 = wc_inverse_rows(c, pay, doff, units + a, m, c->h_rows.p, rows_cap, nullptr, WC_F32,
                                                (float*)c->h_out.p, nullptr)) ||
                         (rc2 = wc_rmse(c, c->h_cells.p, dtype, (const float*)c->h_out.p, units + a, m,
                                        (double*)c->h_rmse.p + a))))
                return rc2;
        }
        mark("enqueued", nr);
        return WC_OK;
    };
    // The helper (or, with one run, the call's thread afterwards): each run's
    // sizes, offsets and kept counts, then its packed payloads to the caller.
    auto download = [&] {
        hipStream_t ds = nr > 1 ? c->down : c->stream;
        for (int r = 0; r < nr; ++r) {
            if (!gate.wait(r)) return;
            const int a = rb[r], m = rb[r + 1] - rb[r];
            hipError_t e;
            if ((e = hipEventSynchronize(c->hev[2 * r + 1])) != hipSuccess) return hs.hip(e, "sizes sync");
            mark("sizes", r);
            const uint64_t* po = pin_poff + (a + r);
            for (int i = 0; i < m; ++i) {
                offsets[a + i] = R - 4 + po[i];
                kept[a + i] = pin_kept[a + i];
            }
            const uint64_t span = po[m] - 4;
            if (R - 4 + po[m] > cap) return hs.invalid("payload_capacity");
            populate(payload + R, span);
            mark("populated", r);
            if (span && (e = hipMemcpyAsync(payload + R, (const uint8_t*)c->h_packed.p + pbase[r] + 4, span,
                                            hipMemcpyDeviceToHost, ds)) != hipSuccess)
                return hs.hip(e, "payload readback");
            mark("d2h issued", r);
            R += po[m];
        }
        hipError_t e;
        if (nr > 1 && (e = hipStreamSynchronize(c->down)) != hipSuccess) return hs.hip(e, "payload readback");
        mark("down synced");
    };
    if ((rc = with_helper(c, nr, gate, hs, enqueue, download))) return rc;
    offsets[n] = R - 4;
    hipError_t e2;
    if (rmse && (e2 = hipMemcpyAsync(rmse, c->h_rmse.p, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream)) !=
                    hipSuccess)
        return hip_fail(c, e2, "rmse readback");
    if ((e2 = hipStreamSynchronize(c->stream)) != hipSuccess) return hip_fail(c, e2, "sync");
    mark("done");
    return check_kernel_errors(c);
}

static int inverse_host_once(wc_ctx* c, const uint8_t* payload, const uint64_t* offsets, const wc_unit* units,
                             int n, float* out) {
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (n == 0) return WC_OK;
    if (!payload || !offsets || !out) return fail(c, WC_ERR_INVALID, "null buffer");
    for (int i = 0; i < n; ++i)
        if (offsets[i] & 3) return fail(c, WC_ERR_INVALID, "offsets must be multiples of 4");
    // Host-side bounds check of every header before anything reaches the device.
    uint64_t extent = 0;
    for (int i = 0; i < n; ++i) {
        int32_t hdr[5];
        std::memcpy(hdr, payload + offsets[i], sizeof hdr);
        if (hdr[4] < 0) return fail(c, WC_ERR_FORMAT, "unit " + std::to_string(i) + ": negative pair count");
        extent = std::max(extent, offsets[i] + 20 + 8 * (uint64_t)hdr[4]);
    }
    if ((rc = set_device(c))) return rc;
    const uint64_t ext = cells_extent(units, n);
    if ((rc = ensure(c, c->h_payload, extent)) || (rc = ensure(c, c->h_offsets, sizeof(uint64_t) * n)) ||
        (rc = ensure(c, c->h_out, sizeof(float) * ext)))
        return rc;
    // Runs of contiguous units of about opt_host_chunk cells (at most 16), as
    // in forward_host_once: run r's payload bytes upload on `up` while run r-1
    // decodes on the context stream and run r-2's boxes download on `down`.
    std::vector<int> rb = host_runs(c, units, n);
    const int nr = (int)rb.size() - 1;
    hipError_t e;
    const HostTrace mark("inverse_host");
    if ((rc = host_streams(c, nr))) return rc;
    if ((e = hipMemcpyAsync(c->h_offsets.p, offsets, sizeof(uint64_t) * n, hipMemcpyHostToDevice, c->stream)) !=
        hipSuccess)
        return hip_fail(c, e, "offsets upload");
    // Each run's boxes go back as one copy per span of back-to-back units:
    // exactly the cells the units own (the caller's buffer may have gaps).
    struct Span {
        int run;
        uint64_t lo, hi;  // cells
    };
    std::vector<Span> spans;
    std::vector<int> first_span(nr + 1, 0);
    for (int r = 0; r < nr; ++r) {
        first_span[r] = (int)spans.size();
        for (int i = rb[r]; i < rb[r + 1];) {
            const uint64_t o = units[i].cell_offset;
            uint64_t end = o + (uint64_t)units[i].nx * units[i].ny * units[i].nz;
            int j = i + 1;
            for (; j < rb[r + 1]; ++j) {
                const uint64_t cj = (uint64_t)units[j].nx * units[j].ny * units[j].nz;
                if (cj && units[j].cell_offset != end) break;
                end += cj;
            }
            if (end > o) spans.push_back({r, o, end});
            i = j;
        }
    }
    first_span[nr] = (int)spans.size();
    const Populate populate = host_populate(c);
    wc::RunGate gate, resident;
    HelperStatus hs;
    // The destination spans do not depend on the device: with several runs a
    // thread of its own faults them in ahead of the downloads.
    std::thread ahead;
    if (populate.on && nr > 1) {
        try {
            ahead = std::thread([&] {
                for (int r = 0; r < nr; ++r) {
                    for (int k = first_span[r]; k < first_span[r + 1]; ++k)
                        populate(out + spans[k].lo, sizeof(float) * (spans[k].hi - spans[k].lo));
                    resident.publish(r + 1);
                }
            });
        } catch (...) {  // no thread: the downloads fault their spans in themselves
        }
    }
    // The call's thread: payload uploads and decodes, run by run.
    auto enqueue = [&]() -> int {
        for (int r = 0; r < nr; ++r) {
            const int a = rb[r], m = rb[r + 1] - rb[r];
            uint64_t lo = UINT64_MAX, hi = 0;
            for (int i = a; i < a + m; ++i) {
                int32_t cnt;
                std::memcpy(&cnt, payload + offsets[i] + 16, 4);
                lo = std::min(lo, offsets[i]);
                hi = std::max(hi, offsets[i] + 20 + 8 * (uint64_t)cnt);
            }
            hipStream_t us = nr > 1 ? c->up : c->stream;
            hipError_t e;
            if (hi > lo && (e = host_upload(c, (uint8_t*)c->h_payload.p + lo, payload + lo, hi - lo, us)) != hipSuccess)
                return hip_fail(c, e, "payload upload");
            if (nr > 1 && ((e = hipEventRecord(c->hev[2 * r], c->up)) != hipSuccess ||
                           (e = hipStreamWaitEvent(c->stream, c->hev[2 * r], 0)) != hipSuccess))
                return hip_fail(c, e, "upload event");
            int rc2;
            if ((rc2 = wc_inverse(c, (const uint8_t*)c->h_payload.p, (const uint64_t*)c->h_offsets.p + a, units + a,
                                  m, (float*)c->h_out.p)))
                return rc2;
            if (nr > 1 && (e = hipEventRecord(c->hev[2 * r + 1], c->stream)) != hipSuccess)
                return hip_fail(c, e, "decode event");
            gate.publish(r + 1);
        }
        mark("enqueued", nr);
        return WC_OK;
    };
    // The helper (or, with one run, the call's thread afterwards): each run's
    // boxes to the caller once it is decoded and its spans are resident.
    auto download = [&] {
        hipStream_t ds = nr > 1 ? c->down : c->stream;
        for (int r = 0; r < nr; ++r) {
            if (!gate.wait(r)) return;
            hipError_t e;
            if (nr > 1 && (e = hipStreamWaitEvent(c->down, c->hev[2 * r + 1], 0)) != hipSuccess)
                return hs.hip(e, "decode event");
            if (ahead.joinable()) resident.wait(r);
            for (int k = first_span[r]; k < first_span[r + 1]; ++k) {
                const uint64_t o = spans[k].lo, bytes = sizeof(float) * (spans[k].hi - o);
                if (!ahead.joinable()) populate(out + o, bytes);
                if ((e = hipMemcpyAsync(out + o, (float*)c->h_out.p + o, bytes, hipMemcpyDeviceToHost, ds)) !=
                    hipSuccess)
                    return hs.hip(e, "box readback");
            }
            mark("d2h issued", r);
        }
        hipError_t e;
        if (nr > 1 && (e = hipStreamSynchronize(c->down)) != hipSuccess) return hs.hip(e, "box readback");
        mark("down synced");
    };
    rc = with_helper(c, nr, gate, hs, enqueue, download);
    if (ahead.joinable()) ahead.join();
    if (rc) return rc;
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return hip_fail(c, e, "sync");
    mark("done");
    return check_kernel_errors(c);
}

extern "C" {

int wc_forward_host(wc_ctx* c, const void* cells, int dtype, const wc_unit* units, int n, double keep,
                    uint8_t* payload, uint64_t cap, uint64_t* offsets, uint32_t* kept) {
    if (!c) return WC_ERR_INVALID;
    return forward_host_once(c, CellSource{(const uint8_t*)cells, nullptr}, dtype, units, n, keep, payload, cap,
                             offsets, kept, nullptr);
}

int wc_round_trip_host(wc_ctx* c, const void* cells, int dtype, const wc_unit* units, int n, double keep,
                       uint8_t* payload, uint64_t cap, uint64_t* offsets, uint32_t* kept, double* rmse) {
    if (!c) return WC_ERR_INVALID;
    if (n > 0 && !rmse) return fail(c, WC_ERR_INVALID, "null buffer");
    return forward_host_once(c, CellSource{(const uint8_t*)cells, nullptr}, dtype, units, n, keep, payload, cap,
                             offsets, kept, rmse);
}

int wc_forward_host_units(wc_ctx* c, const void* const* cells, int dtype, const wc_unit* units, int n, double keep,
                          uint8_t* payload, uint64_t cap, uint64_t* offsets, uint32_t* kept) {
    if (!c) return WC_ERR_INVALID;
    if (n < 0 || (n > 0 && (!units || !cells))) return fail(c, WC_ERR_INVALID, "null buffer");
    // the device layout: the units back to back, 4-element aligned (16-B loads)
    std::vector<wc_unit> packed(units, units + n);
    uint64_t cursor = 0;
    for (wc_unit& u : packed) {
        cursor = (cursor + 3) & ~uint64_t(3);
        u.cell_offset = cursor;
        if (u.nx > 0 && u.ny > 0 && u.nz > 0) cursor += (uint64_t)u.nx * u.ny * u.nz;
    }
    return forward_host_once(c, CellSource{nullptr, cells}, dtype, packed.data(), n, keep, payload, cap, offsets,
                             kept, nullptr);
}

int wc_inverse_host(wc_ctx* c, const uint8_t* payload, const uint64_t* offsets, const wc_unit* units, int n,
                    float* out) {
    if (!c) return WC_ERR_INVALID;
    return inverse_host_once(c, payload, offsets, units, n, out);
}

// Stage host arrays through the context's staging buffers for the
// transform-only, inverse-only and RMSE entry points.
int wc_decompose_host(wc_ctx* c, const void* cells, int dtype, const wc_unit* units, int n, float* flat) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (dtype != WC_F32 && dtype != WC_F64) return fail(c, WC_ERR_INVALID, "dtype");
    if (n == 0) return WC_OK;
    if (!cells || !flat) return fail(c, WC_ERR_INVALID, "null buffer");
    if ((rc = set_device(c))) return rc;
    const size_t esz = dtype == WC_F64 ? 8 : 4;
    const uint64_t ext = cells_extent(units, n);
    if ((rc = ensure(c, c->h_cells, esz * ext)) || (rc = ensure(c, c->h_out, sizeof(float) * ext))) return rc;
    hipError_t e = hipMemcpyAsync(c->h_cells.p, cells, esz * ext, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "cells upload");
    if ((rc = wc_decompose(c, c->h_cells.p, dtype, units, n, (float*)c->h_out.p))) return rc;
    if ((e = hipMemcpyAsync(flat, c->h_out.p, sizeof(float) * ext, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return hip_fail(c, e, "flat readback");
    return WC_OK;
}

int wc_inverse_flat_host(wc_ctx* c, const float* flat, const wc_unit* units, int n, float* out) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (n == 0) return WC_OK;
    if (!flat || !out) return fail(c, WC_ERR_INVALID, "null buffer");
    if ((rc = set_device(c))) return rc;
    const uint64_t ext = cells_extent(units, n);
    if ((rc = ensure(c, c->h_cells, sizeof(float) * ext)) || (rc = ensure(c, c->h_out, sizeof(float) * ext)))
        return rc;
    hipError_t e = hipMemcpyAsync(c->h_cells.p, flat, sizeof(float) * ext, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "flat upload");
    if ((rc = wc_inverse_flat(c, (const float*)c->h_cells.p, units, n, (float*)c->h_out.p))) return rc;
    if ((e = hipMemcpyAsync(out, c->h_out.p, sizeof(float) * ext, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return hip_fail(c, e, "box readback");
    return WC_OK;
}

int wc_rmse_host(wc_ctx* c, const void* orig, int dtype, const float* regen, const wc_unit* units, int n,
                 double* rmse) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (dtype != WC_F32 && dtype != WC_F64) return fail(c, WC_ERR_INVALID, "dtype");
    if (n == 0) return WC_OK;
    if (!orig || !regen || !rmse) return fail(c, WC_ERR_INVALID, "null buffer");
    if ((rc = set_device(c))) return rc;
    const size_t esz = dtype == WC_F64 ? 8 : 4;
    const uint64_t ext = cells_extent(units, n);
    if ((rc = ensure(c, c->h_cells, esz * ext)) || (rc = ensure(c, c->h_out, sizeof(float) * ext)) ||
        (rc = ensure(c, c->h_offsets, sizeof(double) * n)))
        return rc;
    hipError_t e;
    if ((e = hipMemcpyAsync(c->h_cells.p, orig, esz * ext, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(c->h_out.p, regen, sizeof(float) * ext, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
        return hip_fail(c, e, "rmse upload");
    if ((rc = wc_rmse(c, c->h_cells.p, dtype, (const float*)c->h_out.p, units, n, (double*)c->h_offsets.p))) return rc;
    if ((e = hipMemcpyAsync(rmse, c->h_offsets.p, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return hip_fail(c, e, "rmse readback");
    return WC_OK;
}

}  // extern "C"

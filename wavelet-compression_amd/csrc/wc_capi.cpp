// wc_capi.cpp — the extern "C" boundary (include/wavelet_amd.h).
//
// Owns the per-device context (stream, grow-only scratch in HBM, cached batch
// plans) and turns a batch of units into kernel launches (wc_kernels.hip).
// No CPU fallback exists: every entry point that computes launches HIP
// kernels, and fails with WC_ERR_HIP if the device or code object is absent.
#include "wavelet_amd.h"
#include "wc_internal.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace wc {
size_t transform_lds_bytes(int lbx, int lby, int lbz);
hipError_t launch_transform(hipStream_t, const void*, int, const UnitDev*, const XTile*, uint32_t, size_t,
                            float*, int, unsigned long long*);
hipError_t launch_flat_count(hipStream_t, const float*, const UnitDev*, const FTile*, uint32_t,
                             const unsigned long long*, double, uint32_t*, uint32_t*);
hipError_t launch_unit_scan(hipStream_t, const UnitDev*, int, const uint32_t*, const uint32_t*, uint32_t*,
                            uint32_t*, uint32_t*);
hipError_t launch_unit_offsets(hipStream_t, const UnitDev*, int, const uint32_t*, uint8_t*, uint64_t*);
hipError_t launch_flat_emit(hipStream_t, const float*, const UnitDev*, const FTile*, uint32_t,
                            const unsigned long long*, double, const uint32_t*, const uint32_t*,
                            const uint64_t*, uint8_t*);
hipError_t launch_decode(hipStream_t, const UnitDev*, int, const FTile*, uint32_t, const uint8_t*,
                         const uint64_t*, uint64_t*, uint64_t*, float*, uint32_t*);
hipError_t launch_inverse(hipStream_t, const float*, int, const UnitDev*, const XTile*, uint32_t, size_t,
                          float*);
hipError_t launch_rmse(hipStream_t, const void*, int, const float*, const UnitDev*, int, const FTile*,
                       uint32_t, double*, double*);
}  // namespace wc

using namespace wc;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

// A batch plan: unit descriptors + transform tiles + flat tiles, mirrored in HBM.
struct Plan {
    std::vector<wc_unit> key;  // the units it was built for
    std::vector<UnitDev> units;
    std::vector<XTile> xtiles;
    std::vector<FTile> ftiles;
    uint64_t coef_extent = 0;  // floats
    size_t lds_bytes = 0;
    DevBuf d_units, d_xtiles, d_ftiles;
};

int ceil_log2(int64_t v) {
    int l = 0;
    while ((int64_t(1) << l) < v) ++l;
    return l;
}

}  // namespace

struct wc_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    Plan plan;
    bool plan_valid = false;
    // scratch (grow-only)
    DevBuf coef, keys, tcount, tlast, toff, tprev, kept, tsum, tbase, part, errflag;
    // host-path staging
    DevBuf h_cells, h_payload, h_offsets, h_kept, h_out, h_rmse;
    // per-kernel event timing (wc_profile_enable / wc_profile_read)
    bool prof = false;
    std::vector<hipEvent_t> ev_pool;
    struct Mark { int stage; hipEvent_t a, b; };
    std::vector<Mark> marks;
};

namespace {

int fail(wc_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

int hip_fail(wc_ctx* c, hipError_t e, const char* what) {
    return fail(c, WC_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

int ensure(wc_ctx* c, DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return WC_OK;
    size_t want = std::max(bytes, b.bytes + b.bytes / 2);
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    hipError_t e = hipMalloc(&b.p, want);
    if (e != hipSuccess) {
        e = hipMalloc(&b.p, bytes);
        want = bytes;
    }
    if (e != hipSuccess) return fail(c, WC_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    b.bytes = want;
    return WC_OK;
}

int validate_units(wc_ctx* c, const wc_unit* units, int n) {
    if (n < 0) return fail(c, WC_ERR_INVALID, "n < 0");
    if (n > 0 && !units) return fail(c, WC_ERR_INVALID, "units is NULL");
    for (int i = 0; i < n; ++i) {
        const wc_unit& u = units[i];
        if (u.nx < 0 || u.ny < 0 || u.nz < 0 || u.reserved != 0)
            return fail(c, WC_ERR_INVALID, "unit " + std::to_string(i) + ": negative dims or reserved != 0");
        const uint64_t cells = (uint64_t)u.nx * u.ny * u.nz;
        // ncoeff is serialized as int32 (src/compressor.cpp:65-67)
        if (cells > 0x7fffffffull)
            return fail(c, WC_ERR_INVALID, "unit " + std::to_string(i) + ": more than 2^31-1 cells");
    }
    return WC_OK;
}

// Build (or reuse) the plan for this batch and upload it.
int get_plan(wc_ctx* c, const wc_unit* units, int n) {
    Plan& P = c->plan;
    if (c->plan_valid && (int)P.key.size() == n &&
        (n == 0 || std::memcmp(P.key.data(), units, sizeof(wc_unit) * n) == 0))
        return WC_OK;
    c->plan_valid = false;
    P.key.assign(units, units + n);
    P.units.clear();
    P.xtiles.clear();
    P.ftiles.clear();
    P.lds_bytes = 0;
    uint64_t cursor = 0;
    for (int i = 0; i < n; ++i) {
        const wc_unit& u = units[i];
        UnitDev d{};
        d.cell_off = u.cell_offset;
        d.ncells = (uint64_t)u.nx * u.ny * u.nz;
        d.nx = u.nx;
        d.ny = u.ny;
        d.nz = u.nz;
        d.hx = u.nx / 2;
        d.hy = u.ny / 2;
        d.hz = u.nz / 2;
        d.nbx = (u.nx + 1) / 2;
        d.nby = (u.ny + 1) / 2;
        d.nbz = (u.nz + 1) / 2;
        // Tile: up to 32 blocks along x (coalesced input rows) and z (contiguous
        // flat rows), the rest along y, at most kMaxTileBlocks blocks.
        d.lbx = std::min(5, ceil_log2(std::max(1, d.nbx)));
        d.lbz = std::min(5, ceil_log2(std::max(1, d.nbz)));
        d.lby = std::min(ceil_log2(std::max(1, d.nby)), 10 - d.lbx - d.lbz);
        d.coef_off = (cursor + 3) & ~uint64_t(3);
        cursor = d.coef_off + d.ncells;
        d.ftile_begin = (uint32_t)P.ftiles.size();
        d.nftiles = (uint32_t)((d.ncells + kFlatTile - 1) / kFlatTile);
        for (uint32_t t = 0; t < d.nftiles; ++t) P.ftiles.push_back(FTile{(uint32_t)i, t});
        if (d.ncells > 0) {
            const int TX = 1 << d.lbx, TY = 1 << d.lby, TZ = 1 << d.lbz;
            for (int bz = 0; bz < d.nbz; bz += TZ)
                for (int by = 0; by < d.nby; by += TY)
                    for (int bx = 0; bx < d.nbx; bx += TX)
                        P.xtiles.push_back(XTile{(uint32_t)i, (uint32_t)bx, (uint32_t)by, (uint32_t)bz});
            P.lds_bytes = std::max(P.lds_bytes, transform_lds_bytes(d.lbx, d.lby, d.lbz));
        }
        P.units.push_back(d);
    }
    P.coef_extent = cursor + kFlatTile;  // slack: flat tiles read whole float4 groups
    int rc;
    if ((rc = ensure(c, P.d_units, sizeof(UnitDev) * P.units.size())) ||
        (rc = ensure(c, P.d_xtiles, sizeof(XTile) * P.xtiles.size())) ||
        (rc = ensure(c, P.d_ftiles, sizeof(FTile) * P.ftiles.size())))
        return rc;
    hipError_t e;
    if (!P.units.empty() &&
        (e = hipMemcpyAsync(P.d_units.p, P.units.data(), sizeof(UnitDev) * P.units.size(),
                            hipMemcpyHostToDevice, c->stream)) != hipSuccess)
        return hip_fail(c, e, "upload units");
    if (!P.xtiles.empty() &&
        (e = hipMemcpyAsync(P.d_xtiles.p, P.xtiles.data(), sizeof(XTile) * P.xtiles.size(),
                            hipMemcpyHostToDevice, c->stream)) != hipSuccess)
        return hip_fail(c, e, "upload xtiles");
    if (!P.ftiles.empty() &&
        (e = hipMemcpyAsync(P.d_ftiles.p, P.ftiles.data(), sizeof(FTile) * P.ftiles.size(),
                            hipMemcpyHostToDevice, c->stream)) != hipSuccess)
        return hip_fail(c, e, "upload ftiles");
    // The host vectors back the async copies; keep them alive until the next
    // plan, which first synchronizes below.
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return hip_fail(c, e, "plan upload sync");
    c->plan_valid = true;
    return WC_OK;
}

int ensure_scratch(wc_ctx* c, bool need_coef) {
    const Plan& P = c->plan;
    const size_t n = P.units.size(), nft = P.ftiles.size();
    int rc;
    if (need_coef && (rc = ensure(c, c->coef, sizeof(float) * P.coef_extent))) return rc;
    if ((rc = ensure(c, c->keys, sizeof(unsigned long long) * n)) ||
        (rc = ensure(c, c->tcount, sizeof(uint32_t) * nft)) ||
        (rc = ensure(c, c->tlast, sizeof(uint32_t) * nft)) ||
        (rc = ensure(c, c->toff, sizeof(uint32_t) * nft)) ||
        (rc = ensure(c, c->tprev, sizeof(uint32_t) * nft)) ||
        (rc = ensure(c, c->tsum, sizeof(uint64_t) * nft)) ||
        (rc = ensure(c, c->tbase, sizeof(uint64_t) * nft)) ||
        (rc = ensure(c, c->part, sizeof(double) * nft)) ||
        (rc = ensure(c, c->errflag, sizeof(uint32_t) * 4)))
        return rc;
    return WC_OK;
}

hipEvent_t take_event(wc_ctx* c) {
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

// Bracket one launch with events when profiling is on.
struct StageTimer {
    wc_ctx* c;
    int stage;
    hipEvent_t a = nullptr;
    StageTimer(wc_ctx* c_, int s) : c(c_), stage(s) {
        if (c->prof) {
            a = take_event(c);
            (void)hipEventRecord(a, c->stream);
        }
    }
    ~StageTimer() {
        if (c->prof && a) {
            hipEvent_t b = take_event(c);
            (void)hipEventRecord(b, c->stream);
            c->marks.push_back({stage, a, b});
        }
    }
};

int set_device(wc_ctx* c) {
    hipError_t e = hipSetDevice(c->device);
    return e == hipSuccess ? WC_OK : hip_fail(c, e, "hipSetDevice");
}

}  // namespace

extern "C" {

const char* wc_version(void) {
    return "wavelet_amd 0.1 (gfx950; fp-contract=off, no denormal flush)";
}

int wc_ctx_create(int device, wc_ctx** out) {
    if (!out) return WC_ERR_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return WC_ERR_HIP;
    if (device < 0 || device >= ndev) return WC_ERR_INVALID;
    wc_ctx* c = new wc_ctx();
    c->device = device;
    if (set_device(c) != WC_OK) {
        delete c;
        return WC_ERR_HIP;
    }
    if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return WC_ERR_HIP;
    }
    c->stream = c->own;
    *out = c;
    return WC_OK;
}

void wc_ctx_destroy(wc_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    DevBuf* bufs[] = {&c->coef,  &c->keys,  &c->tcount,  &c->tlast,   &c->toff,     &c->tprev,
                      &c->kept,  &c->tsum,  &c->tbase,   &c->part,    &c->errflag,  &c->h_cells,
                      &c->h_payload, &c->h_offsets, &c->h_kept, &c->h_out, &c->h_rmse,
                      &c->plan.d_units, &c->plan.d_xtiles, &c->plan.d_ftiles};
    for (DevBuf* b : bufs)
        if (b->p) (void)hipFree(b->p);
    for (auto& m : c->marks) {
        c->ev_pool.push_back(m.a);
        c->ev_pool.push_back(m.b);
    }
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

const char* wc_last_error(const wc_ctx* c) { return c ? c->err.c_str() : "null context"; }

int wc_set_stream(wc_ctx* c, void* s) {
    if (!c) return WC_ERR_INVALID;
    c->stream = s ? (hipStream_t)s : c->own;
    return WC_OK;
}

int wc_synchronize(wc_ctx* c) {
    if (!c) return WC_ERR_INVALID;
    hipError_t e = hipStreamSynchronize(c->stream);
    return e == hipSuccess ? WC_OK : hip_fail(c, e, "hipStreamSynchronize");
}

uint64_t wc_payload_bound(const wc_unit* units, int n) {
    uint64_t b = 4;
    for (int i = 0; i < n; ++i) b += 24 + 8 * (uint64_t)units[i].nx * units[i].ny * units[i].nz;
    return b;
}

uint64_t wc_cell_count(const wc_unit* units, int n) {
    uint64_t s = 0;
    for (int i = 0; i < n; ++i) s += (uint64_t)units[i].nx * units[i].ny * units[i].nz;
    return s;
}

int wc_forward(wc_ctx* c, const void* d_cells, int dtype, const wc_unit* units, int n, double keep,
               uint8_t* d_payload, uint64_t cap, uint64_t* d_offsets, uint32_t* d_kept) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (dtype != WC_F32 && dtype != WC_F64) return fail(c, WC_ERR_INVALID, "dtype");
    if (n == 0) return WC_OK;
    if (!d_cells || !d_payload || !d_offsets || !d_kept) return fail(c, WC_ERR_INVALID, "null buffer");
    if (cap < wc_payload_bound(units, n)) return fail(c, WC_ERR_INVALID, "payload_capacity < wc_payload_bound");
    if ((rc = set_device(c)) || (rc = get_plan(c, units, n)) || (rc = ensure_scratch(c, true))) return rc;
    Plan& P = c->plan;
    hipError_t e = hipMemsetAsync(c->keys.p, 0, sizeof(unsigned long long) * n, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "memset keys");
    const UnitDev* du = (const UnitDev*)P.d_units.p;
    const FTile* dft = (const FTile*)P.d_ftiles.p;
    const uint32_t nft = (uint32_t)P.ftiles.size();
    const unsigned long long* keys = (const unsigned long long*)c->keys.p;
    {
        StageTimer t(c, WC_STAGE_TRANSFORM);
        e = launch_transform(c->stream, d_cells, dtype, du, (const XTile*)P.d_xtiles.p, (uint32_t)P.xtiles.size(),
                             P.lds_bytes, (float*)c->coef.p, 0, (unsigned long long*)c->keys.p);
    }
    if (e != hipSuccess) return hip_fail(c, e, "transform launch");
    {
        StageTimer t(c, WC_STAGE_COUNT);
        e = launch_flat_count(c->stream, (const float*)c->coef.p, du, dft, nft, keys, keep, (uint32_t*)c->tcount.p,
                              (uint32_t*)c->tlast.p);
    }
    if (e != hipSuccess) return hip_fail(c, e, "count launch");
    {
        StageTimer t(c, WC_STAGE_SCAN);
        e = launch_unit_scan(c->stream, du, n, (const uint32_t*)c->tcount.p, (const uint32_t*)c->tlast.p,
                             (uint32_t*)c->toff.p, (uint32_t*)c->tprev.p, d_kept);
    }
    if (e != hipSuccess) return hip_fail(c, e, "scan launch");
    {
        StageTimer t(c, WC_STAGE_OFFSETS);
        e = launch_unit_offsets(c->stream, du, n, d_kept, d_payload, d_offsets);
    }
    if (e != hipSuccess) return hip_fail(c, e, "offsets launch");
    {
        StageTimer t(c, WC_STAGE_EMIT);
        e = launch_flat_emit(c->stream, (const float*)c->coef.p, du, dft, nft, keys, keep,
                             (const uint32_t*)c->toff.p, (const uint32_t*)c->tprev.p, d_offsets, d_payload);
    }
    if (e != hipSuccess) return hip_fail(c, e, "emit launch");
    return WC_OK;
}

int wc_decompose(wc_ctx* c, const void* d_cells, int dtype, const wc_unit* units, int n, float* d_flat) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (dtype != WC_F32 && dtype != WC_F64) return fail(c, WC_ERR_INVALID, "dtype");
    if (n == 0) return WC_OK;
    if (!d_cells || !d_flat) return fail(c, WC_ERR_INVALID, "null buffer");
    if ((rc = set_device(c)) || (rc = get_plan(c, units, n))) return rc;
    Plan& P = c->plan;
    hipError_t e = launch_transform(c->stream, d_cells, dtype, (const UnitDev*)P.d_units.p,
                                    (const XTile*)P.d_xtiles.p, (uint32_t)P.xtiles.size(), P.lds_bytes,
                                    d_flat, 1, nullptr);
    return e == hipSuccess ? WC_OK : hip_fail(c, e, "transform launch");
}

int wc_inverse(wc_ctx* c, const uint8_t* d_payload, const uint64_t* d_offsets, const wc_unit* units, int n,
               float* d_out) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (n == 0) return WC_OK;
    if (!d_payload || !d_offsets || !d_out) return fail(c, WC_ERR_INVALID, "null buffer");
    if ((rc = set_device(c)) || (rc = get_plan(c, units, n)) || (rc = ensure_scratch(c, true))) return rc;
    Plan& P = c->plan;
    hipError_t e;
    if ((e = hipMemsetAsync(c->coef.p, 0, sizeof(float) * P.coef_extent, c->stream)) != hipSuccess ||
        (e = hipMemsetAsync(c->errflag.p, 0, sizeof(uint32_t), c->stream)) != hipSuccess)
        return hip_fail(c, e, "memset");
    {
        StageTimer t(c, WC_STAGE_DECODE);
        e = launch_decode(c->stream, (const UnitDev*)P.d_units.p, n, (const FTile*)P.d_ftiles.p,
                          (uint32_t)P.ftiles.size(), d_payload, d_offsets, (uint64_t*)c->tsum.p,
                          (uint64_t*)c->tbase.p, (float*)c->coef.p, (uint32_t*)c->errflag.p);
    }
    if (e != hipSuccess) return hip_fail(c, e, "decode launch");
    {
        StageTimer t(c, WC_STAGE_INVERSE);
        e = launch_inverse(c->stream, (const float*)c->coef.p, 0, (const UnitDev*)P.d_units.p,
                           (const XTile*)P.d_xtiles.p, (uint32_t)P.xtiles.size(), P.lds_bytes, d_out);
    }
    if (e != hipSuccess) return hip_fail(c, e, "inverse launch");
    // Malformed payloads end the reference with exit(EXIT_FAILURE)
    // (src/decompressor.cpp:228-231); here they return WC_ERR_FORMAT.
    uint32_t flag = 0;
    if ((e = hipMemcpyAsync(&flag, c->errflag.p, sizeof(flag), hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return hip_fail(c, e, "error flag readback");
    if (flag) {
        char buf[128];
        std::snprintf(buf, sizeof buf, "malformed payload (flags 0x%x: 1 header, 2 negative run)", flag);
        return fail(c, WC_ERR_FORMAT, buf);
    }
    return WC_OK;
}

int wc_inverse_flat(wc_ctx* c, const float* d_flat, const wc_unit* units, int n, float* d_out) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (n == 0) return WC_OK;
    if (!d_flat || !d_out) return fail(c, WC_ERR_INVALID, "null buffer");
    if ((rc = set_device(c)) || (rc = get_plan(c, units, n))) return rc;
    Plan& P = c->plan;
    hipError_t e = launch_inverse(c->stream, d_flat, 1, (const UnitDev*)P.d_units.p,
                                  (const XTile*)P.d_xtiles.p, (uint32_t)P.xtiles.size(), P.lds_bytes, d_out);
    return e == hipSuccess ? WC_OK : hip_fail(c, e, "inverse launch");
}

int wc_rmse(wc_ctx* c, const void* d_orig, int dtype, const float* d_regen, const wc_unit* units, int n,
            double* d_rmse) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (dtype != WC_F32 && dtype != WC_F64) return fail(c, WC_ERR_INVALID, "dtype");
    if (n == 0) return WC_OK;
    if (!d_orig || !d_regen || !d_rmse) return fail(c, WC_ERR_INVALID, "null buffer");
    if ((rc = set_device(c)) || (rc = get_plan(c, units, n)) || (rc = ensure_scratch(c, false))) return rc;
    Plan& P = c->plan;
    StageTimer t(c, WC_STAGE_RMSE);
    hipError_t e = launch_rmse(c->stream, d_orig, dtype, d_regen, (const UnitDev*)P.d_units.p, n,
                               (const FTile*)P.d_ftiles.p, (uint32_t)P.ftiles.size(), (double*)c->part.p,
                               d_rmse);
    return e == hipSuccess ? WC_OK : hip_fail(c, e, "rmse launch");
}

int wc_profile_enable(wc_ctx* c, int on) {
    if (!c) return WC_ERR_INVALID;
    c->prof = on != 0;
    return WC_OK;
}

int wc_profile_read(wc_ctx* c, double* total_ms, uint32_t* launches, int nstages) {
    if (!c || nstages < 0 || (nstages > 0 && (!total_ms || !launches))) return WC_ERR_INVALID;
    for (int i = 0; i < nstages; ++i) {
        total_ms[i] = 0.0;
        launches[i] = 0;
    }
    int rc = WC_OK;
    if (!c->marks.empty()) {
        hipError_t e = hipEventSynchronize(c->marks.back().b);
        if (e != hipSuccess) rc = hip_fail(c, e, "hipEventSynchronize");
    }
    for (auto& m : c->marks) {
        float ms = 0.f;
        if (rc == WC_OK && m.stage < nstages && hipEventElapsedTime(&ms, m.a, m.b) == hipSuccess) {
            total_ms[m.stage] += ms;
            launches[m.stage] += 1;
        }
        c->ev_pool.push_back(m.a);
        c->ev_pool.push_back(m.b);
    }
    c->marks.clear();
    return rc;
}

// ---- host-pointer variants -------------------------------------------------

static uint64_t cells_extent(const wc_unit* units, int n) {
    uint64_t ext = 0;
    for (int i = 0; i < n; ++i)
        ext = std::max(ext, units[i].cell_offset + (uint64_t)units[i].nx * units[i].ny * units[i].nz);
    return ext;
}

int wc_forward_host(wc_ctx* c, const void* cells, int dtype, const wc_unit* units, int n, double keep,
                    uint8_t* payload, uint64_t cap, uint64_t* offsets, uint32_t* kept) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (dtype != WC_F32 && dtype != WC_F64) return fail(c, WC_ERR_INVALID, "dtype");
    if (n == 0) return WC_OK;
    if (!cells || !payload || !offsets || !kept) return fail(c, WC_ERR_INVALID, "null buffer");
    const uint64_t bound = wc_payload_bound(units, n);
    if (cap < bound) return fail(c, WC_ERR_INVALID, "payload_capacity < wc_payload_bound");
    if ((rc = set_device(c))) return rc;
    const size_t esz = dtype == WC_F64 ? 8 : 4;
    const uint64_t ext = cells_extent(units, n);
    if ((rc = ensure(c, c->h_cells, esz * ext)) || (rc = ensure(c, c->h_payload, bound)) ||
        (rc = ensure(c, c->h_offsets, sizeof(uint64_t) * (n + 1))) || (rc = ensure(c, c->h_kept, 4 * n)))
        return rc;
    hipError_t e = hipMemcpyAsync(c->h_cells.p, cells, esz * ext, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "cells upload");
    if ((rc = wc_forward(c, c->h_cells.p, dtype, units, n, keep, (uint8_t*)c->h_payload.p, bound,
                         (uint64_t*)c->h_offsets.p, (uint32_t*)c->h_kept.p)))
        return rc;
    if ((e = hipMemcpyAsync(offsets, c->h_offsets.p, sizeof(uint64_t) * (n + 1), hipMemcpyDeviceToHost,
                            c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(kept, c->h_kept.p, 4 * n, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return hip_fail(c, e, "offsets readback");
    if ((e = hipMemcpyAsync(payload, c->h_payload.p, offsets[n], hipMemcpyDeviceToHost, c->stream)) !=
            hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return hip_fail(c, e, "payload readback");
    return WC_OK;
}

int wc_inverse_host(wc_ctx* c, const uint8_t* payload, const uint64_t* offsets, const wc_unit* units, int n,
                    float* out) {
    if (!c) return WC_ERR_INVALID;
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
    hipError_t e;
    if ((e = hipMemcpyAsync(c->h_payload.p, payload, extent, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(c->h_offsets.p, offsets, sizeof(uint64_t) * n, hipMemcpyHostToDevice, c->stream)) !=
            hipSuccess)
        return hip_fail(c, e, "payload upload");
    if ((rc = wc_inverse(c, (const uint8_t*)c->h_payload.p, (const uint64_t*)c->h_offsets.p, units, n,
                         (float*)c->h_out.p)))
        return rc;
    // Copy back exactly the cells the units own (the caller's buffer may have gaps).
    for (int i = 0; i < n; ++i) {
        const uint64_t cnt = (uint64_t)units[i].nx * units[i].ny * units[i].nz;
        if (!cnt) continue;
        if ((e = hipMemcpyAsync(out + units[i].cell_offset, (float*)c->h_out.p + units[i].cell_offset,
                                sizeof(float) * cnt, hipMemcpyDeviceToHost, c->stream)) != hipSuccess)
            return hip_fail(c, e, "box readback");
    }
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return hip_fail(c, e, "sync");
    return WC_OK;
}

}  // extern "C"

// wc_capi.cpp — the extern "C" boundary (include/wavelet_amd.h).
//
// Owns the per-device context (stream, grow-only scratch in HBM, cached batch
// plans) and turns a batch of units into kernel launches.  No CPU fallback
// exists: every computing entry point launches HIP kernels and fails with
// WC_ERR_HIP if the device or code object is absent.
//
// Forward path per batch (wc_forward):
//   fused units  (even dims, D % 8 == 0, W <= 64, D <= 64, <= kMaxFusedTiles tiles)
//       -> k_forward_fused: one read of the cells, pairs written in place
//   staged units (everything else: odd dims, short z, huge boxes)
//       -> k_transform{,_fast} -> flat coefficients in HBM scratch
//       -> k_flat_count -> k_unit_scan -> k_unit_offsets -> k_flat_emit
// Both write unit u's serialized bytes at its fixed slot offsets[u].
#include "wavelet_amd.h"
#include "wc_internal.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace wc {
size_t transform_lds_bytes(int lbx, int lby, int lbz);
size_t transform_fast_lds_bytes(int lbx, int lby, int lbz);
size_t fused_lds_bytes(int lbx, int lby, int lbz, uint32_t ntile);
hipError_t launch_transform(hipStream_t, const void*, int, const UnitDev*, const XTile*, uint32_t, size_t,
                            float*, int, unsigned long long*);
hipError_t launch_transform_fast(hipStream_t, const void*, int, const UnitDev*, const XTile*, uint32_t, size_t,
                                 float*, int, unsigned long long*);
hipError_t launch_flat_count(hipStream_t, const float*, const UnitDev*, const FTile*, uint32_t,
                             const unsigned long long*, double, uint32_t*, uint32_t*);
hipError_t launch_unit_scan(hipStream_t, const UnitDev*, int, const uint32_t*, const uint32_t*, uint32_t*,
                            uint32_t*, uint32_t*);
hipError_t launch_unit_offsets(hipStream_t, const UnitDev*, int, const uint32_t*, uint8_t*, uint64_t*);
hipError_t launch_flat_emit(hipStream_t, const float*, const UnitDev*, const FTile*, uint32_t,
                            const unsigned long long*, double, const uint32_t*, const uint32_t*,
                            const uint64_t*, uint8_t*);
hipError_t launch_pack(hipStream_t, const UnitDev*, int, const uint32_t*, const uint8_t*, uint64_t*, uint8_t*);
hipError_t launch_decode(hipStream_t, const UnitDev*, int, const FTile*, uint32_t, const uint8_t*,
                         const uint64_t*, uint64_t*, uint64_t*, float*, uint32_t*);
hipError_t launch_inverse(hipStream_t, const float*, int, const UnitDev*, const XTile*, uint32_t, size_t,
                          float*);
hipError_t launch_rmse(hipStream_t, const void*, int, const float*, const UnitDev*, int, const FTile*,
                       uint32_t, double*, double*);
hipError_t launch_forward_fused(hipStream_t, int, size_t, const FusedParams&);
}  // namespace wc

using namespace wc;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

// A batch plan: unit descriptors and tile lists, mirrored in HBM.
//   xtiles = [generic staged | fast staged | fused]  (unit-major in each part;
//            the inverse transform runs over all of them)
//   ftiles = [staged units | fused units]            (flat tiles; the staged
//            forward uses the first part, decode and RMSE use all)
struct Plan {
    std::vector<wc_unit> key;
    bool fused_enabled = true;
    std::vector<UnitDev> units;
    std::vector<XTile> xtiles;
    std::vector<FTile> ftiles;
    uint32_t ngen = 0, nfast = 0, nfused = 0;  // xtiles partition
    uint32_t nft_staged = 0;
    uint32_t nstaged_units = 0;  // units (including empty ones) the staged kernels finish
    uint64_t coef_extent = 0;  // floats of staged coefficient scratch
    uint64_t ntab = 0;         // fused row-table granules
    size_t lds_gen = 0, lds_fast = 0, lds_fused = 0, lds_inverse = 0;
    size_t flags_bytes = 0;    // ticket + keyslot[nfused]
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
    bool opt_fused = true;   // WC_OPT_FUSED default (see include/wavelet_amd.h)
    bool err_check_pending = false;
    // scratch (grow-only)
    DevBuf coef, keys, tcount, tlast, toff, tprev, tsum, tbase, part, errflag, flags, table;
    // host-path staging
    DevBuf h_cells, h_payload, h_packed, h_offsets, h_poff, h_kept, h_out;
    // per-kernel event timing (wc_profile_enable / wc_profile_read)
    bool prof = false;
    std::vector<hipEvent_t> ev_pool;
    struct Mark {
        int stage;
        hipEvent_t a, b;
    };
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

int upload(wc_ctx* c, DevBuf& d, const void* h, size_t bytes, const char* what) {
    int rc = ensure(c, d, bytes);
    if (rc) return rc;
    if (!bytes) return WC_OK;
    hipError_t e = hipMemcpyAsync(d.p, h, bytes, hipMemcpyHostToDevice, c->stream);
    return e == hipSuccess ? WC_OK : hip_fail(c, e, what);
}

void set_tiling(UnitDev& d) {
    // Up to 32 blocks along x (coalesced input rows) and z (contiguous flat
    // rows), the rest along y, at most kMaxTileBlocks blocks per tile.
    d.lbx = std::min(5, ceil_log2(std::max(1, d.nbx)));
    d.lbz = std::min(5, ceil_log2(std::max(1, d.nbz)));
    d.lby = std::min(ceil_log2(std::max(1, d.nby)), 10 - d.lbx - d.lbz);
}

void push_tiles(std::vector<XTile>& v, const UnitDev& d, uint32_t u) {
    const int TX = 1 << d.lbx, TY = 1 << d.lby, TZ = 1 << d.lbz;
    for (int bz = 0; bz < d.nbz; bz += TZ)
        for (int by = 0; by < d.nby; by += TY)
            for (int bx = 0; bx < d.nbx; bx += TX) v.push_back(XTile{u, (uint32_t)bx, (uint32_t)by, (uint32_t)bz});
}

// Build (or reuse) the plan for this batch and upload it.
int get_plan(wc_ctx* c, const wc_unit* units, int n) {
    Plan& P = c->plan;
    if (c->plan_valid && P.fused_enabled == c->opt_fused && (int)P.key.size() == n &&
        (n == 0 || std::memcmp(P.key.data(), units, sizeof(wc_unit) * n) == 0))
        return WC_OK;
    c->plan_valid = false;
    P.key.assign(units, units + n);
    P.fused_enabled = c->opt_fused;
    P.units.assign(n, UnitDev{});
    P.xtiles.clear();
    P.ftiles.clear();
    P.ngen = P.nfast = P.nfused = P.nft_staged = P.nstaged_units = 0;
    P.lds_gen = P.lds_fast = P.lds_fused = P.lds_inverse = 0;
    std::vector<XTile> gen, fast, fused;
    uint64_t coef_cursor = 0, pay_cursor = 4, tab_cursor = 0;
    for (int i = 0; i < n; ++i) {
        const wc_unit& u = units[i];
        UnitDev& d = P.units[i];
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
        set_tiling(d);
        d.ntz = (d.nbz + (1 << d.lbz) - 1) >> d.lbz;
        d.pay_off = pay_cursor;  // slot of 20 + 8*ncells bytes + 4 pad: next slot stays == 4 (mod 8)
        pay_cursor += 24 + 8 * d.ncells;
        if (d.ncells == 0) {
            ++P.nstaged_units;  // header-only payload, written by k_unit_offsets
            continue;
        }
        const bool fast_ok = (u.nx % 2 == 0) && (u.ny % 2 == 0) && (u.nz % 8 == 0);
        const uint64_t ntile = (uint64_t)((d.nbx + (1 << d.lbx) - 1) >> d.lbx) *
                               ((d.nby + (1 << d.lby) - 1) >> d.lby) * d.ntz;
        // fused: tiles span the whole x and z extent (one tile row per y block
        // range), G <= kMaxFusedTiles, the row table fits kMaxFusedRows.
        const uint64_t nrows_tile = (uint64_t)4 << (d.lbx + d.lby);
        const bool fused_ok = fast_ok && (u.cell_offset % 2 == 0) && d.nbx <= (1 << d.lbx) && d.ntz == 1 &&
                              ntile <= kMaxFusedTiles &&
                              ntile * nrows_tile <= kMaxFusedRows;
        if (fused_ok && c->opt_fused) {
            d.fused = 1;
            d.xt_begin = (uint32_t)fused.size();
            d.ntile_u = (uint32_t)ntile;
            d.tab_off = tab_cursor;
            tab_cursor += ntile * nrows_tile / 4;
            push_tiles(fused, d, (uint32_t)i);
            P.lds_fused = std::max(P.lds_fused, fused_lds_bytes(d.lbx, d.lby, d.lbz, (uint32_t)ntile));
        } else {
            ++P.nstaged_units;
            d.coef_off = (coef_cursor + 3) & ~uint64_t(3);
            coef_cursor = d.coef_off + d.ncells;
            if (fast_ok) {
                push_tiles(fast, d, (uint32_t)i);
                P.lds_fast = std::max(P.lds_fast, transform_fast_lds_bytes(d.lbx, d.lby, d.lbz));
            } else {
                push_tiles(gen, d, (uint32_t)i);
                P.lds_gen = std::max(P.lds_gen, transform_lds_bytes(d.lbx, d.lby, d.lbz));
            }
        }
        P.lds_inverse = std::max(P.lds_inverse, transform_lds_bytes(d.lbx, d.lby, d.lbz));
    }
    // flat tiles: staged units first, then fused units
    for (int pass = 0; pass < 2; ++pass) {
        for (int i = 0; i < n; ++i) {
            UnitDev& d = P.units[i];
            if ((pass == 0) == (d.fused != 0)) continue;
            d.ftile_begin = (uint32_t)P.ftiles.size();
            d.nftiles = (uint32_t)((d.ncells + kFlatTile - 1) / kFlatTile);
            for (uint32_t t = 0; t < d.nftiles; ++t) P.ftiles.push_back(FTile{(uint32_t)i, t});
        }
        if (pass == 0) P.nft_staged = (uint32_t)P.ftiles.size();
    }
    P.ngen = (uint32_t)gen.size();
    P.nfast = (uint32_t)fast.size();
    P.nfused = (uint32_t)fused.size();
    P.xtiles = std::move(gen);
    P.xtiles.insert(P.xtiles.end(), fast.begin(), fast.end());
    P.xtiles.insert(P.xtiles.end(), fused.begin(), fused.end());
    P.coef_extent = coef_cursor ? coef_cursor + kFlatTile : 0;  // slack: flat tiles read whole float4 groups
    P.ntab = tab_cursor;
    P.flags_bytes = 16 + 8 * (size_t)P.nfused;
    int rc;
    if ((rc = upload(c, P.d_units, P.units.data(), sizeof(UnitDev) * P.units.size(), "upload units")) ||
        (rc = upload(c, P.d_xtiles, P.xtiles.data(), sizeof(XTile) * P.xtiles.size(), "upload xtiles")) ||
        (rc = upload(c, P.d_ftiles, P.ftiles.data(), sizeof(FTile) * P.ftiles.size(), "upload ftiles")))
        return rc;
    // The host vectors back the async copies: finish them before returning.
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "plan upload sync");
    c->plan_valid = true;
    return WC_OK;
}

int ensure_scratch(wc_ctx* c) {
    const Plan& P = c->plan;
    const size_t n = P.units.size(), nft = P.ftiles.size();
    int rc;
    if ((rc = ensure(c, c->coef, sizeof(float) * std::max<uint64_t>(P.coef_extent, 1))) ||
        (rc = ensure(c, c->keys, sizeof(unsigned long long) * n)) ||
        (rc = ensure(c, c->tcount, sizeof(uint32_t) * nft)) || (rc = ensure(c, c->tlast, sizeof(uint32_t) * nft)) ||
        (rc = ensure(c, c->toff, sizeof(uint32_t) * nft)) || (rc = ensure(c, c->tprev, sizeof(uint32_t) * nft)) ||
        (rc = ensure(c, c->tsum, sizeof(uint64_t) * nft)) || (rc = ensure(c, c->tbase, sizeof(uint64_t) * nft)) ||
        (rc = ensure(c, c->part, sizeof(double) * nft)) || (rc = ensure(c, c->errflag, 16)) ||
        (rc = ensure(c, c->flags, P.flags_bytes)) || (rc = ensure(c, c->table, 8 * P.ntab)))
        return rc;
    return WC_OK;
}

int set_device(wc_ctx* c) {
    hipError_t e = hipSetDevice(c->device);
    return e == hipSuccess ? WC_OK : hip_fail(c, e, "hipSetDevice");
}

// Surface an error bit a kernel raised (fused hand-off timeout) at the next
// synchronisation point.
int check_kernel_errors(wc_ctx* c) {
    if (!c->err_check_pending) return WC_OK;
    c->err_check_pending = false;
    uint32_t flag = 0;
    hipError_t e = hipMemcpyAsync(&flag, c->errflag.p, 4, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "error flag readback");
    if (flag & kErrTimeout) return fail(c, WC_ERR_HIP, "fused forward: hand-off wait timed out");
    return WC_OK;
}

int forward_impl(wc_ctx* c, const void* d_cells, int dtype, int n, double keep, uint8_t* d_payload,
                 uint64_t* d_offsets, uint32_t* d_kept) {
    Plan& P = c->plan;
    const UnitDev* du = (const UnitDev*)P.d_units.p;
    const XTile* dxt = (const XTile*)P.d_xtiles.p;
    const FTile* dft = (const FTile*)P.d_ftiles.p;
    hipError_t e = hipSuccess;
    if (P.nfused) {
        uint8_t* fl = (uint8_t*)c->flags.p;
        if ((e = hipMemsetAsync(fl, 0, P.flags_bytes, c->stream)) != hipSuccess ||
            (e = hipMemsetAsync(c->table.p, 0, 8 * P.ntab, c->stream)) != hipSuccess ||
            (e = hipMemsetAsync(c->errflag.p, 0, 4, c->stream)) != hipSuccess)
            return hip_fail(c, e, "memset fused flags");
        FusedParams fp{};
        fp.cells = d_cells;
        fp.units = du;
        fp.tiles = dxt + P.ngen + P.nfast;
        fp.ntiles = P.nfused;
        fp.n = n;
        fp.ticket = (uint32_t*)fl;
        fp.keyslot = (unsigned long long*)(fl + 16);
        fp.table = (unsigned long long*)c->table.p;
        fp.payload = d_payload;
        fp.offsets = d_offsets;
        fp.kept = d_kept;
        fp.err = (uint32_t*)c->errflag.p;
        fp.keep = keep;
        {
            StageTimer t(c, WC_STAGE_FUSED);
            e = launch_forward_fused(c->stream, dtype, P.lds_fused, fp);
        }
        if (e != hipSuccess) return hip_fail(c, e, "fused launch");
        c->err_check_pending = true;
    }
    if (P.nstaged_units == 0) return WC_OK;  // every unit was fused
    if ((e = hipMemsetAsync(c->keys.p, 0, sizeof(unsigned long long) * n, c->stream)) != hipSuccess)
        return hip_fail(c, e, "memset keys");
    unsigned long long* keys = (unsigned long long*)c->keys.p;
    float* coef = (float*)c->coef.p;
    {
        StageTimer t(c, WC_STAGE_TRANSFORM);
        e = launch_transform(c->stream, d_cells, dtype, du, dxt, P.ngen, P.lds_gen, coef, 0, keys);
        if (e == hipSuccess)
            e = launch_transform_fast(c->stream, d_cells, dtype, du, dxt + P.ngen, P.nfast, P.lds_fast, coef, 0,
                                      keys);
    }
    if (e != hipSuccess) return hip_fail(c, e, "transform launch");
    {
        StageTimer t(c, WC_STAGE_COUNT);
        e = launch_flat_count(c->stream, coef, du, dft, P.nft_staged, keys, keep, (uint32_t*)c->tcount.p,
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
        e = launch_flat_emit(c->stream, coef, du, dft, P.nft_staged, keys, keep, (const uint32_t*)c->toff.p,
                             (const uint32_t*)c->tprev.p, d_offsets, d_payload);
    }
    if (e != hipSuccess) return hip_fail(c, e, "emit launch");
    return WC_OK;
}

uint64_t cells_extent(const wc_unit* units, int n) {
    uint64_t ext = 0;
    for (int i = 0; i < n; ++i)
        ext = std::max(ext, units[i].cell_offset + (uint64_t)units[i].nx * units[i].ny * units[i].nz);
    return ext;
}

// Plan with the fused path switched off (transform-only and inverse calls
// need flat coefficient scratch for every unit).
int get_plan_staged(wc_ctx* c, const wc_unit* units, int n) {
    const bool saved = c->opt_fused;
    c->opt_fused = false;
    int rc = get_plan(c, units, n);
    c->opt_fused = saved;
    return rc;
}

}  // namespace

extern "C" {

const char* wc_version(void) { return "wavelet_amd 0.2 (gfx950; fp-contract=off, no denormal flush)"; }

int wc_device_count(void) {
    int ndev = 0;
    return hipGetDeviceCount(&ndev) == hipSuccess ? ndev : 0;
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
    DevBuf* bufs[] = {&c->coef,      &c->keys,      &c->tcount,    &c->tlast,      &c->toff,
                      &c->tprev,     &c->tsum,      &c->tbase,     &c->part,       &c->errflag,
                      &c->flags,     &c->table,     &c->h_cells,    &c->h_payload,
                      &c->h_packed,  &c->h_offsets, &c->h_poff,    &c->h_kept,     &c->h_out,
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

int wc_set_option(wc_ctx* c, int option, int64_t value) {
    if (!c) return WC_ERR_INVALID;
    switch (option) {
        case WC_OPT_FUSED:
            c->opt_fused = value != 0;
            return WC_OK;
        default:
            return fail(c, WC_ERR_INVALID, "unknown option");
    }
}

int wc_synchronize(wc_ctx* c) {
    if (!c) return WC_ERR_INVALID;
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "hipStreamSynchronize");
    return check_kernel_errors(c);
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
    if ((rc = set_device(c)) || (rc = get_plan(c, units, n)) || (rc = ensure_scratch(c))) return rc;
    return forward_impl(c, d_cells, dtype, n, keep, d_payload, d_offsets, d_kept);
}

int wc_decompose(wc_ctx* c, const void* d_cells, int dtype, const wc_unit* units, int n, float* d_flat) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (dtype != WC_F32 && dtype != WC_F64) return fail(c, WC_ERR_INVALID, "dtype");
    if (n == 0) return WC_OK;
    if (!d_cells || !d_flat) return fail(c, WC_ERR_INVALID, "null buffer");
    if ((rc = set_device(c)) || (rc = get_plan_staged(c, units, n))) return rc;
    Plan& P = c->plan;
    const UnitDev* du = (const UnitDev*)P.d_units.p;
    const XTile* dxt = (const XTile*)P.d_xtiles.p;
    StageTimer t(c, WC_STAGE_TRANSFORM);
    hipError_t e = launch_transform(c->stream, d_cells, dtype, du, dxt, P.ngen, P.lds_gen, d_flat, 1, nullptr);
    if (e == hipSuccess)
        e = launch_transform_fast(c->stream, d_cells, dtype, du, dxt + P.ngen, P.nfast, P.lds_fast, d_flat, 1,
                                  nullptr);
    return e == hipSuccess ? WC_OK : hip_fail(c, e, "transform launch");
}

int wc_inverse(wc_ctx* c, const uint8_t* d_payload, const uint64_t* d_offsets, const wc_unit* units, int n,
               float* d_out) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (n == 0) return WC_OK;
    if (!d_payload || !d_offsets || !d_out) return fail(c, WC_ERR_INVALID, "null buffer");
    if ((rc = set_device(c)) || (rc = get_plan_staged(c, units, n)) || (rc = ensure_scratch(c))) return rc;
    Plan& P = c->plan;
    hipError_t e;
    if ((e = hipMemsetAsync(c->coef.p, 0, sizeof(float) * P.coef_extent, c->stream)) != hipSuccess ||
        (e = hipMemsetAsync(c->errflag.p, 0, 4, c->stream)) != hipSuccess)
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
                           (const XTile*)P.d_xtiles.p, (uint32_t)P.xtiles.size(), P.lds_inverse, d_out);
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
    StageTimer t(c, WC_STAGE_INVERSE);
    hipError_t e = launch_inverse(c->stream, d_flat, 1, (const UnitDev*)P.d_units.p, (const XTile*)P.d_xtiles.p,
                                  (uint32_t)P.xtiles.size(), P.lds_inverse, d_out);
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
    if ((rc = set_device(c)) || (rc = get_plan(c, units, n)) || (rc = ensure_scratch(c))) return rc;
    Plan& P = c->plan;
    StageTimer t(c, WC_STAGE_RMSE);
    hipError_t e = launch_rmse(c->stream, d_orig, dtype, d_regen, (const UnitDev*)P.d_units.p, n,
                               (const FTile*)P.d_ftiles.p, (uint32_t)P.ftiles.size(), (double*)c->part.p, d_rmse);
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
        (rc = ensure(c, c->h_packed, bound)) || (rc = ensure(c, c->h_offsets, sizeof(uint64_t) * (n + 1))) ||
        (rc = ensure(c, c->h_poff, sizeof(uint64_t) * (n + 1))) || (rc = ensure(c, c->h_kept, 4 * n)))
        return rc;
    hipError_t e = hipMemcpyAsync(c->h_cells.p, cells, esz * ext, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "cells upload");
    if ((rc = wc_forward(c, c->h_cells.p, dtype, units, n, keep, (uint8_t*)c->h_payload.p, bound,
                         (uint64_t*)c->h_offsets.p, (uint32_t*)c->h_kept.p)))
        return rc;
    // Pack the slots into a dense buffer before the copy back (offsets stay == 4 mod 8).
    e = launch_pack(c->stream, (const UnitDev*)c->plan.d_units.p, n, (const uint32_t*)c->h_kept.p,
                    (const uint8_t*)c->h_payload.p, (uint64_t*)c->h_poff.p, (uint8_t*)c->h_packed.p);
    if (e != hipSuccess) return hip_fail(c, e, "pack launch");
    if ((e = hipMemcpyAsync(offsets, c->h_poff.p, sizeof(uint64_t) * (n + 1), hipMemcpyDeviceToHost, c->stream)) !=
            hipSuccess ||
        (e = hipMemcpyAsync(kept, c->h_kept.p, 4 * n, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return hip_fail(c, e, "offsets readback");
    if ((rc = check_kernel_errors(c))) return rc;
    if ((e = hipMemcpyAsync(payload, c->h_packed.p, offsets[n], hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
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

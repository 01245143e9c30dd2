// wc_capi.cpp — the extern "C" boundary (include/wavelet_amd.h): context
// lifetime, options and the device-pointer entry points.
//
// The context (wc_ctx.h) owns the stream, grow-only scratch in HBM and the
// cached batch plans (wc_plan.cpp), and turns a batch of units into kernel
// launches.  No CPU fallback exists: every computing entry point launches HIP
// kernels and fails with WC_ERR_HIP if the device or code object is absent.
// The _host entry points are in wc_hostpipe.cpp.
//
// Forward path per batch (wc_forward), every unit shape: K1 k_transform{,_fast}
// -> flat coefficients in HBM scratch (sparse staging: only the flagged
// segments) + per-unit max keys -> k_transform_fallback (units whose thresh
// is < 0 re-staged densely) -> K2 k_emit (threshold + decoupled look-back +
// ordered pack), writing unit u's serialized bytes at its fixed slot
// offsets[u] (and with wc_forward_rows the payloads' row index).  Inverse:
// K5 k_rowindex (or the caller's row index) -> K6r k_inverse_rows from the
// payloads; units that are not row-indexable: k_decode -> dense flat scratch
// -> K6 k_inverse{,_fast}.
#include "wc_ctx.h"

#include <algorithm>
#include <cmath>
#include <cstring>

using namespace wc;

namespace {

// Staged forward, first half: K1 transform into the flat coefficient
// scratch + per-unit max keys (zeroed state).
int stage_transform(wc_ctx* c, const void* d_cells, int dtype, double keep, bool sparse) {
    Plan& P = c->plan;
    const UnitDev* du = (const UnitDev*)P.d_units.p;
    const XTile* dxt = (const XTile*)P.d_xtiles.p;
    hipError_t e = hipSuccess;
    if ((e = hipMemsetAsync(c->state.p, 0, P.state_bytes, c->stream)) != hipSuccess)
        return hip_fail(c, e, "memset state");
    unsigned long long* key = (unsigned long long*)((uint8_t*)c->state.p + 16);
    const size_t n = P.units.size();
    uint32_t* spos = (uint32_t*)((uint8_t*)c->state.p + 16 + 12 * n);
    float* coef = (float*)c->coef.p;
    uint8_t* flags = sparse && P.any_sparse ? (uint8_t*)c->flags.p : nullptr;
    {
        StageTimer t(c, WC_STAGE_TRANSFORM);
        e = launch_transform(c->stream, d_cells, dtype, du, dxt, P.ngen, P.lds_gen, coef, 0, key);
        if (e == hipSuccess)
            e = launch_transform_fast(c->stream, d_cells, dtype, du, dxt + P.ngen, P.nfast, P.lds_fast, coef, 0,
                                      key, flags, spos, keep, persistent_grid(c, 0, P.lds_fast));
        // units whose thresh came out < 0 need every coefficient (rare: negative signed max)
        if (e == hipSuccess && flags)
            e = launch_transform_fallback(c->stream, d_cells, dtype, du, (int)P.units.size(), dxt, P.lds_fast, coef,
                                          key, spos, keep);
    }
    c->sparse_staged = flags != nullptr;
    return e == hipSuccess ? WC_OK : hip_fail(c, e, "transform launch");
}

// Second half: K2 threshold + ordered pack of the staged coefficients
// (gthresh: the global-threshold mode's fp32 threshold, or null).  Uses the
// unit keys and the zeroed tickets / look-back granules of the per-call state.
int stage_emit(wc_ctx* c, int n, double keep, const float* gthresh, uint8_t* d_payload, uint64_t* d_offsets,
               uint32_t* d_kept, uint2* d_rows = nullptr) {
    Plan& P = c->plan;
    uint8_t* st = (uint8_t*)c->state.p;
    EmitParams p{};
    p.units = (const UnitDev*)P.d_units.p;
    p.edesc = (const EmitDesc*)P.d_edesc.p;
    p.n = n;
    p.ordered = use_ordered(c) ? (c->opt_reverse ? 2u : 1u) : 0u;
    p.key = (const unsigned long long*)(st + 16);
    p.tickets = (uint32_t*)(st + 16 + 8ull * n);
    p.status = (unsigned long long*)(st + round_up(16 + 20ull * n, 8));
    p.payload = d_payload;
    p.offsets = d_offsets;
    p.kept = d_kept;
    p.err = (uint32_t*)c->errflag.p;
    p.keep = keep;
    if (gthresh) {
        p.use_gthresh = 1;
        p.gthresh = *gthresh;
    }
    p.flags = (c->sparse_staged && !gthresh) ? (const uint8_t*)c->flags.p : nullptr;
    p.rowinfo = d_rows;
    StageTimer t(c, WC_STAGE_EMIT);
    hipError_t e = launch_emit(c->stream, p, (const float*)c->coef.p, P.nedesc_small,
                               (uint32_t)P.edesc.size() - P.nedesc_small);
    if (e != hipSuccess) return hip_fail(c, e, "emit launch");
    return WC_OK;
}

int forward_staged(wc_ctx* c, const void* d_cells, int dtype, int n, double keep, uint8_t* d_payload,
                   uint64_t* d_offsets, uint32_t* d_kept, uint2* d_rows = nullptr) {
    int rc = stage_transform(c, d_cells, dtype, keep, c->opt_sparse);
    return rc ? rc : stage_emit(c, n, keep, nullptr, d_payload, d_offsets, d_kept, d_rows);
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
    // the persistent error word (check_kernel_errors reads and clears it)
    if (ensure(c, c->errflag, 16) != WC_OK || hipMemset(c->errflag.p, 0, 16) != hipSuccess) {
        wc_ctx_destroy(c);
        return WC_ERR_NOMEM;
    }
    *out = c;
    return WC_OK;
}

void wc_ctx_destroy(wc_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (c->aux) (void)hipStreamSynchronize(c->aux);
    DevBuf* bufs[] = {&c->coef,          &c->part,           &c->errflag,        &c->state,
                      &c->flags,         &c->h_cells,        &c->h_payload,      &c->h_packed,
                      &c->h_offsets,     &c->h_poff,         &c->h_kept,         &c->h_out,
                      &c->h_rows,        &c->h_rmse,
                      &c->plan.d_units,  &c->plan.d_xtiles,  &c->plan.d_ftiles,  &c->plan.d_dtiles,
                      &c->plan.d_edesc, &c->plan.d_ixtiles, &c->plan.d_rtiles,
                      &c->plan.d_rdtiles, &c->rowinfo,    &c->istate,        &c->npairs};
    for (DevBuf* b : bufs)
        if (b->p) (void)hipFree(b->p);
    for (Plan& P : c->plan_cache) free_plan(P);
    for (hipEvent_t e : c->hev) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->iev) (void)hipEventDestroy(e);
    if (c->aux) (void)hipStreamDestroy(c->aux);
    if (c->up) (void)hipStreamDestroy(c->up);
    if (c->down) (void)hipStreamDestroy(c->down);
    if (c->pinned) (void)hipHostFree(c->pinned);
    if (c->bounce) (void)hipHostFree(c->bounce);
    for (hipEvent_t e : c->bev) (void)hipEventDestroy(e);
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
    hipStream_t next = s ? (hipStream_t)s : c->own;
    // Kernels queued on the old stream may still read the plan's descriptors
    // and the scratch, which later calls rebuild or reuse in stream order on
    // the new stream: drain the old one first.
    // The switch happens even when the drain fails (a stale handle must not
    // stay the context's stream); the failure is still reported.
    hipError_t e = hipSuccess;
    if (next != c->stream) e = hipStreamSynchronize(c->stream);
    c->stream = next;
    return e == hipSuccess ? WC_OK : hip_fail(c, e, "wc_set_stream: synchronize the previous stream");
}

int wc_set_option(wc_ctx* c, int option, int64_t value) {
    if (!c) return WC_ERR_INVALID;
    switch (option) {
        case WC_OPT_SPARSE:
            c->opt_sparse = value != 0;
            return WC_OK;
        case WC_OPT_RIX_XCD:
            c->opt_rix_xcd = value != 0;
            return WC_OK;
        case WC_OPT_INV_GROUPS:
            if (value < 1 || value > 16) return fail(c, WC_ERR_INVALID, "WC_OPT_INV_GROUPS: 1..16");
            c->opt_inv_groups = (int)value;
            return WC_OK;
        case WC_OPT_ORDERED:
            c->opt_ordered = value != 0;
            return WC_OK;
        case WC_OPT_INVERSE_ROWS:
            c->opt_inv_rows = value != 0;
            return WC_OK;
        case WC_OPT_RIX_LDS:
            if (value < 1024 || value > 16384) return fail(c, WC_ERR_INVALID, "WC_OPT_RIX_LDS: 1024..16384 floats");
            c->opt_rix_lds = (int)value;
            return WC_OK;
        case WC_OPT_RIX_BLOCKED:
            c->opt_rix_blocked = value != 0;
            return WC_OK;
        case WC_OPT_RIX_TX:
            if (value < 0 || value > 5) return fail(c, WC_ERR_INVALID, "WC_OPT_RIX_TX: log2 of 1..32 blocks");
            c->opt_rix_lx = (int)value;
            return WC_OK;
        case WC_OPT_HOST_CHUNK:
            if (value < 0) return fail(c, WC_ERR_INVALID, "WC_OPT_HOST_CHUNK: cells >= 0");
            c->opt_host_chunk = value;
            return WC_OK;
        case WC_OPT_SPIN_LIMIT: {
            if (value < 0 || value > 0xffffffffll) return fail(c, WC_ERR_INVALID, "WC_OPT_SPIN_LIMIT: 0..2^32-1 polls");
            hipError_t e;
            if ((e = hipSetDevice(c->device)) != hipSuccess ||
                (e = hipMemsetD32Async((hipDeviceptr_t)((uint32_t*)c->errflag.p + 1), (int)(uint32_t)value, 1,
                                       c->stream)) != hipSuccess)
                return hip_fail(c, e, "WC_OPT_SPIN_LIMIT");
            c->opt_spin_limit = (uint32_t)value;
            return WC_OK;
        }
        case WC_OPT_TICKETS:
            c->force_tickets = value != 0;
            return WC_OK;
        case WC_OPT_REVERSE_TILES:
            c->opt_reverse = value != 0;
            return WC_OK;
        case WC_OPT_HOST_THREADS:
            if (value < -1 || value > 256) return fail(c, WC_ERR_INVALID, "WC_OPT_HOST_THREADS: -1..256");
            c->opt_host_threads = (int)value;
            return WC_OK;
        case WC_OPT_HOST_THP:
            c->opt_host_thp = value != 0;
            return WC_OK;
        default:
            return fail(c, WC_ERR_INVALID, "unknown option");
    }
}

int wc_get_option(const wc_ctx* c, int option, int64_t* value) {
    if (!c || !value) return WC_ERR_INVALID;
    switch (option) {
        case WC_OPT_SPARSE: *value = c->opt_sparse; return WC_OK;
        case WC_OPT_RIX_XCD: *value = c->opt_rix_xcd; return WC_OK;
        case WC_OPT_INV_GROUPS: *value = c->opt_inv_groups; return WC_OK;
        case WC_OPT_ORDERED: *value = use_ordered(c) ? 1 : 0; return WC_OK;  // the form the next launch takes
        case WC_OPT_INVERSE_ROWS: *value = c->opt_inv_rows; return WC_OK;
        case WC_OPT_RIX_LDS: *value = c->opt_rix_lds; return WC_OK;
        case WC_OPT_RIX_TX: *value = c->opt_rix_lx; return WC_OK;
        case WC_OPT_RIX_BLOCKED: *value = c->opt_rix_blocked; return WC_OK;
        case WC_OPT_HOST_CHUNK: *value = c->opt_host_chunk; return WC_OK;
        case WC_OPT_SPIN_LIMIT: *value = c->opt_spin_limit; return WC_OK;
        case WC_OPT_TICKETS: *value = c->force_tickets ? 1 : 0; return WC_OK;
        case WC_OPT_REVERSE_TILES: *value = c->opt_reverse ? 1 : 0; return WC_OK;
        case WC_OPT_HOST_THREADS:
            *value = c->opt_host_threads < 0 ? host_threads_default() : c->opt_host_threads;
            return WC_OK;
        case WC_OPT_HOST_THP: *value = c->opt_host_thp; return WC_OK;
        default: return WC_ERR_INVALID;
    }
}

int wc_synchronize(wc_ctx* c) {
    if (!c) return WC_ERR_INVALID;
    hipError_t e = hipStreamSynchronize(c->stream);
    // the pipelined inverse's second stream joins c->stream on success; drain it
    // too, so no queued work outlives a synchronize on any path
    if (e == hipSuccess && c->aux) e = hipStreamSynchronize(c->aux);
    if (e != hipSuccess) return hip_fail(c, e, "hipStreamSynchronize");
    return check_kernel_errors(c);
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
    if ((rc = check_aligned(c, d_cells, "cells")) || (rc = check_aligned(c, d_payload, "payload")) ||
        (rc = check_aligned(c, d_offsets, "offsets", 8)) || (rc = check_aligned(c, d_kept, "kept", 4)))
        return rc;
    if ((rc = set_device(c)) || (rc = get_plan(c, units, n))) return rc;
    if ((rc = ensure_scratch(c))) return rc;
    return forward_staged(c, d_cells, dtype, n, keep, d_payload, d_offsets, d_kept);
}

int wc_forward_rows(wc_ctx* c, const void* d_cells, int dtype, const wc_unit* units, int n, double keep,
                    uint8_t* d_payload, uint64_t cap, uint64_t* d_offsets, uint32_t* d_kept, void* d_rowinfo,
                    uint64_t rowinfo_capacity) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (dtype != WC_F32 && dtype != WC_F64) return fail(c, WC_ERR_INVALID, "dtype");
    if (n == 0) return WC_OK;
    if (!d_cells || !d_payload || !d_offsets || !d_kept || !d_rowinfo) return fail(c, WC_ERR_INVALID, "null buffer");
    if (cap < wc_payload_bound(units, n)) return fail(c, WC_ERR_INVALID, "payload_capacity < wc_payload_bound");
    if (rowinfo_capacity < wc_rowindex_bytes(units, n))
        return fail(c, WC_ERR_INVALID, "rowinfo_capacity < wc_rowindex_bytes");
    if ((rc = check_aligned(c, d_cells, "cells")) || (rc = check_aligned(c, d_payload, "payload")) ||
        (rc = check_aligned(c, d_offsets, "offsets", 8)) || (rc = check_aligned(c, d_kept, "kept", 4)) ||
        (rc = check_aligned(c, d_rowinfo, "rowinfo", 8)))
        return rc;
    if ((rc = set_device(c)) || (rc = get_plan(c, units, n))) return rc;
    if (c->plan.rowinfo_entries > 0xffffffffull)  // the emit descriptors keep 32-bit row offsets
        return fail(c, WC_ERR_INVALID, "wc_forward_rows: more than 2^32 row-index entries in one batch");
    if ((rc = ensure_scratch(c))) return rc;
    return forward_staged(c, d_cells, dtype, n, keep, d_payload, d_offsets, d_kept, (uint2*)d_rowinfo);
}

int wc_forward_stage(wc_ctx* c, const void* d_cells, int dtype, const wc_unit* units, int n, uint64_t* d_hist) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (dtype != WC_F32 && dtype != WC_F64) return fail(c, WC_ERR_INVALID, "dtype");
    if (n == 0) return WC_OK;
    if (!d_cells) return fail(c, WC_ERR_INVALID, "null buffer");
    if ((rc = check_aligned(c, d_cells, "cells"))) return rc;
    if ((rc = set_device(c)) || (rc = get_plan(c, units, n))) return rc;
    // dense staging: the histogram and any later threshold need every coefficient
    if ((rc = ensure_scratch(c))) return rc;
    if (!d_hist) {
        if ((rc = stage_transform(c, d_cells, dtype, 0.0, false))) return rc;
        c->staged = true;
        return WC_OK;
    }
    // The fast tiles bin their coefficients as K1 stages them (k_transform_hist:
    // no re-read of the staged coefficients); the generic ones (odd dims, D % 8
    // != 0) stage as usual and k_hist bins those units afterwards.
    Plan& P = c->plan;
    const UnitDev* du = (const UnitDev*)P.d_units.p;
    const XTile* dxt = (const XTile*)P.d_xtiles.p;
    unsigned long long* key = (unsigned long long*)((uint8_t*)c->state.p + 16);
    float* coef = (float*)c->coef.p;
    hipError_t e = hipMemsetAsync(c->state.p, 0, P.state_bytes, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "memset state");
    {
        StageTimer t(c, WC_STAGE_TRANSFORM);
        e = launch_transform(c->stream, d_cells, dtype, du, dxt, P.ngen, P.lds_gen, coef, 0, key);
        if (e == hipSuccess)
            e = launch_transform_hist(c->stream, d_cells, dtype, du, dxt + P.ngen, P.nfast, P.lds_fast, coef, key,
                                      (unsigned long long*)d_hist,
                                      persistent_grid(c, 2, transform_hist_lds_bytes(P.lds_fast)));
        if (e != hipSuccess) return hip_fail(c, e, "transform launch");
    }
    c->sparse_staged = false;
    if (P.ngen) {
        const uint32_t max_blocks = 2048;  // 8 workgroups per CU, 256 CUs
        StageTimer t(c, WC_STAGE_HIST);
        e = launch_hist(c->stream, du, (const FTile*)P.d_ftiles.p, (uint32_t)P.ftiles.size(), coef, max_blocks,
                        (unsigned long long*)d_hist, true);
        if (e != hipSuccess) return hip_fail(c, e, "histogram launch");
    }
    c->staged = true;
    return WC_OK;
}

int wc_hist_threshold(const uint64_t* hist, double quantile, float* thresh, uint64_t* retained) {
    if (!hist || !thresh || !(quantile >= 0.0 && quantile <= 1.0)) return WC_ERR_INVALID;
    uint64_t total = 0;
    for (int b = 0; b < WC_HIST_BINS; ++b) total += hist[b];
    const uint64_t drop = (uint64_t)std::floor(quantile * (double)total);
    const uint64_t target = total - std::min(drop, total);
    uint64_t cum = 0;
    int bstar = -1;  // -1: keep nothing
    if (target > 0)
        for (int b = WC_HIST_BINS - 1; b >= 0; --b) {
            cum += hist[b];
            if (cum >= target) {
                bstar = b;
                break;
            }
        }
    float t;
    if (bstar < 0) {
        t = __builtin_inff();  // |c| > inf never holds
        cum = 0;
    } else if (bstar == 0) {
        t = -1.0f;  // every non-NaN coefficient
    } else {
        const uint32_t bits = ((uint32_t)bstar << WC_HIST_SHIFT) - 1u;
        std::memcpy(&t, &bits, 4);
    }
    *thresh = t;
    if (retained) *retained = cum;
    return WC_OK;
}

int wc_forward_emit(wc_ctx* c, const wc_unit* units, int n, double keep, const float* thresh, uint8_t* d_payload,
                    uint64_t cap, uint64_t* d_offsets, uint32_t* d_kept) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (n == 0) return WC_OK;
    if (!d_payload || !d_offsets || !d_kept) return fail(c, WC_ERR_INVALID, "null buffer");
    if (cap < wc_payload_bound(units, n)) return fail(c, WC_ERR_INVALID, "payload_capacity < wc_payload_bound");
    if ((rc = check_aligned(c, d_payload, "payload")) || (rc = check_aligned(c, d_offsets, "offsets", 8)) ||
        (rc = check_aligned(c, d_kept, "kept", 4)))
        return rc;
    const bool staged = c->staged;
    const uint64_t gen = c->plan_gen;
    if ((rc = set_device(c)) || (rc = get_plan(c, units, n))) return rc;
    // get_plan keeps the cached plan (and so the staged scratch) only for the same units
    if (!staged || gen != c->plan_gen)
        return fail(c, WC_ERR_INVALID, "wc_forward_emit: no staged coefficients for these units (wc_forward_stage)");
    // per-unit tile tickets (tdone) and look-back status words are per call:
    // zero everything after the unit keys
    const Plan& P = c->plan;
    const size_t st_off = 16 + 8ull * n;
    hipError_t e = hipMemsetAsync((uint8_t*)c->state.p + st_off, 0, P.state_bytes - st_off, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "memset status");
    if ((rc = stage_emit(c, n, keep, thresh, d_payload, d_offsets, d_kept))) return rc;
    c->staged = true;  // the coefficients are still there: emit again with another threshold
    return WC_OK;
}

int wc_decompose(wc_ctx* c, const void* d_cells, int dtype, const wc_unit* units, int n, float* d_flat) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (dtype != WC_F32 && dtype != WC_F64) return fail(c, WC_ERR_INVALID, "dtype");
    if (n == 0) return WC_OK;
    if (!d_cells || !d_flat) return fail(c, WC_ERR_INVALID, "null buffer");
    if ((rc = check_aligned(c, d_cells, "cells")) || (rc = check_aligned(c, d_flat, "flat"))) return rc;
    if ((rc = set_device(c)) || (rc = get_plan(c, units, n))) return rc;
    Plan& P = c->plan;
    const UnitDev* du = (const UnitDev*)P.d_units.p;
    const XTile* dxt = (const XTile*)P.d_xtiles.p;
    StageTimer t(c, WC_STAGE_TRANSFORM);
    hipError_t e = launch_transform(c->stream, d_cells, dtype, du, dxt, P.ngen, P.lds_gen, d_flat, 1, nullptr);
    if (e == hipSuccess)
        e = launch_transform_fast(c->stream, d_cells, dtype, du, dxt + P.ngen, P.nfast, P.lds_fast, d_flat, 1,
                                  nullptr, nullptr, nullptr, 0.0, persistent_grid(c, 0, P.lds_fast));
    return e == hipSuccess ? WC_OK : hip_fail(c, e, "transform launch");
}

}  // extern "C"

namespace {

// wc_inverse, and with orig != null also calc_rmse_per_box fused into the
// row-indexed inverse (every unit row-indexed; the caller checks).
// user_rows (wc_inverse_rows): the caller's row index of these payloads, as
// wc_forward_rows wrote it: K6r reads it and the row index kernel does not
// run; units that are not row-indexed still decode densely.
int inverse_impl(wc_ctx* c, const uint8_t* d_payload, const uint64_t* d_offsets, int n, float* d_out,
                 const void* d_orig, int dtype, double* d_rmse, const uint2* user_rows = nullptr) {
    Plan& P = c->plan;
    int rc = WC_OK;
    hipError_t e = hipSuccess;
    // per-call state of the dense decode and of the ticket form: ticket[n] |
    // status[decode tiles] (zeroed).  The row index needs none: its granules
    // carry the call's epoch.  The dense coefficient scratch is fully written
    // by the decode (no memset).
    uint8_t* st = (uint8_t*)c->state.p;
    const bool ord = use_ordered(c);  // once: the clear below and the launch must agree
    if ((!P.dtiles.empty() || !ord) &&
        (e = hipMemsetAsync(st, 0, decode_state_bytes(P), c->stream)) != hipSuccess)
        return hip_fail(c, e, "memset");
    c->epoch = (c->epoch + 1) & kEpochMask;
    if (c->epoch == 0) {  // wrapped: granules of 2^30 calls ago could look current
        if ((e = hipMemsetAsync(c->istate.p, 0, c->istate.bytes, c->stream)) != hipSuccess)
            return hip_fail(c, e, "memset");
        c->epoch = 1;
    }
    const int ng = (int)P.ig_rd.size() - 1;  // row-indexed groups (0: none)
    const bool piped = ng > 1 && !c->prof && !user_rows;  // profiling times each kernel alone
    const uint2* rows_in = user_rows ? user_rows : (const uint2*)c->rowinfo.p;
    if (piped && (rc = inverse_stream(c, 2 * ng + 2))) return rc;
    auto rows = [&](int g, hipStream_t s) {  // K6r over group g's tiles
        const uint32_t t0 = P.ig_rt[g], nt = P.ig_rt[g + 1] - P.ig_rt[g];
        return launch_inverse_rows(s, (const RTile*)P.d_rtiles.p + t0, nt, P.lds_rows,
                                   nt ? persistent_grid(c, 1, P.lds_rows) : 1u, d_payload, d_offsets, rows_in, d_out,
                                   c->opt_rix_blocked ? 1 : 0, d_orig, dtype, (const UnitDev*)P.d_units.p, n,
                                   (double*)c->part.p, d_rmse, g == ng - 1, (const uint32_t*)c->npairs.p);
    };
    auto index = [&](int g, hipStream_t s) {  // K5 over group g's tiles (g = ng: the dense decode)
        const bool dense = g == ng;
        return launch_decode(s, (const UnitDev*)P.d_units.p, (const FTile*)P.d_dtiles.p,
                             dense ? (uint32_t)P.dtiles.size() : 0u, (const FTile*)P.d_rdtiles.p + (dense ? 0 : P.ig_rd[g]),
                             dense ? 0u : P.ig_rd[g + 1] - P.ig_rd[g], (unsigned long long*)c->istate.p, c->epoch,
                             d_payload, d_offsets, (uint32_t*)st, (unsigned long long*)(st + round_up(4ull * n, 8)),
                             (float*)c->coef.p, (uint2*)c->rowinfo.p, (uint32_t*)c->errflag.p, ord ? (c->opt_reverse ? 2 : 1) : 0,
                             (uint32_t*)c->npairs.p);
    };
    if (piped) {
        // K5 of group g + 1 on the context stream beside K6r of group g on the
        // aux stream: the latency-bound row index overlaps the streaming
        // reconstruction; the aux stream joins back before the call returns.
        hipEvent_t* ev = c->iev.data();
        if ((e = hipEventRecord(ev[0], c->stream)) != hipSuccess || (e = hipStreamWaitEvent(c->aux, ev[0], 0)) != hipSuccess)
            return hip_fail(c, e, "inverse pipeline");
        for (int g = 0; g < ng && e == hipSuccess; ++g) {
            e = index(g, c->stream);
            if (e == hipSuccess) e = hipEventRecord(ev[1 + g], c->stream);
            if (e == hipSuccess) e = hipStreamWaitEvent(c->aux, ev[1 + g], 0);
            if (e == hipSuccess) e = rows(g, c->aux);
        }
        if (e == hipSuccess && !P.dtiles.empty()) e = index(ng, c->stream);
        if (e == hipSuccess) e = hipEventRecord(ev[1 + ng], c->aux);
        if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, ev[1 + ng], 0);
        if (e == hipSuccess)
            e = launch_inverse(c->stream, (const float*)c->coef.p, 0, (const UnitDev*)P.d_units.p,
                               (const XTile*)P.d_ixtiles.p, P.ign, P.lds_inverse, P.ifast, P.lds_fast, d_out);
        if (e != hipSuccess) {
            // K6r work already queued on the aux stream still reads the payload
            // and the row index: drain it before the scratch can be reused
            (void)hipStreamSynchronize(c->aux);
            return hip_fail(c, e, "inverse launch");
        }
        c->err_check_pending = true;
        return rc;
    }
    if (ng > 0 && user_rows) {  // the row index is the caller's: check the headers, count the pairs
        StageTimer t(c, WC_STAGE_PAIRS);
        e = launch_pair_counts(c->stream, (const UnitDev*)P.d_units.p, n, d_payload, d_offsets,
                               (uint32_t*)c->npairs.p, (uint32_t*)c->errflag.p);
        if (e != hipSuccess) return hip_fail(c, e, "pair count launch");
    }
    if ((ng > 0 && !user_rows) || !P.dtiles.empty()) {  // a decode stage only when something launches
        StageTimer t(c, WC_STAGE_DECODE);
        for (int g = 0; g <= ng && e == hipSuccess; ++g)
            if ((g < ng && !user_rows) || (g == ng && !P.dtiles.empty())) e = index(g, c->stream);
    }
    if (e != hipSuccess) return hip_fail(c, e, "decode launch");
    {
        StageTimer t(c, WC_STAGE_INVERSE);
        for (int g = 0; g < ng && e == hipSuccess; ++g) e = rows(g, c->stream);
        if (e == hipSuccess && ng == 0 && d_orig)  // every unit empty: the per-unit RMSE (0) only
            e = launch_inverse_rows(c->stream, nullptr, 0, 0, 1u, d_payload, d_offsets, rows_in, d_out, 0, d_orig,
                                    dtype, (const UnitDev*)P.d_units.p, n, (double*)c->part.p, d_rmse, true,
                                    (const uint32_t*)c->npairs.p);
        if (e == hipSuccess)
            e = launch_inverse(c->stream, (const float*)c->coef.p, 0, (const UnitDev*)P.d_units.p,
                               (const XTile*)P.d_ixtiles.p, P.ign, P.lds_inverse, P.ifast, P.lds_fast, d_out);
    }
    if (e != hipSuccess) return hip_fail(c, e, "inverse launch");
    // Malformed payloads surface at the next wc_synchronize (WC_ERR_FORMAT).
    c->err_check_pending = true;
    return rc;
}

}  // namespace

extern "C" {

int wc_inverse(wc_ctx* c, const uint8_t* d_payload, const uint64_t* d_offsets, const wc_unit* units, int n,
               float* d_out) {
    return wc_inverse_rows(c, d_payload, d_offsets, units, n, nullptr, 0, nullptr, WC_F32, d_out, nullptr);
}

int wc_inverse_rmse(wc_ctx* c, const uint8_t* d_payload, const uint64_t* d_offsets, const wc_unit* units, int n,
                    const void* d_orig, int dtype, float* d_out, double* d_rmse) {
    if (!c) return WC_ERR_INVALID;
    if (n > 0 && (!d_orig || !d_rmse)) return fail(c, WC_ERR_INVALID, "null buffer");
    return wc_inverse_rows(c, d_payload, d_offsets, units, n, nullptr, 0, d_orig, dtype, d_out, d_rmse);
}

// wc_inverse / wc_inverse_rmse, and with d_rowinfo the caller's row index in
// place of the row index kernel (wc_forward_rows wrote it for these payloads).
int wc_inverse_rows(wc_ctx* c, const uint8_t* d_payload, const uint64_t* d_offsets, const wc_unit* units, int n,
                    const void* d_rowinfo, uint64_t rowinfo_capacity, const void* d_orig, int dtype, float* d_out,
                    double* d_rmse) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (d_orig && dtype != WC_F32 && dtype != WC_F64) return fail(c, WC_ERR_INVALID, "dtype");
    if (n == 0) return WC_OK;
    if (!d_payload || !d_offsets || !d_out || (!d_orig != !d_rmse)) return fail(c, WC_ERR_INVALID, "null buffer");
    if (d_rowinfo && rowinfo_capacity < wc_rowindex_bytes(units, n))
        return fail(c, WC_ERR_INVALID, "rowinfo_capacity < wc_rowindex_bytes");
    if ((rc = check_aligned(c, d_payload, "payload")) || (rc = check_aligned(c, d_offsets, "offsets", 8)) ||
        (rc = check_aligned(c, d_out, "out")) || (rc = check_aligned(c, d_rowinfo, "rowinfo", 8)) ||
        (rc = check_aligned(c, d_rmse, "rmse", 8)) ||
        (rc = check_aligned(c, d_orig, "orig", dtype == WC_F64 ? 8 : 4)))
        return rc;
    if ((rc = set_device(c)) || (rc = get_plan(c, units, n)) || (rc = ensure_scratch(c))) return rc;
    const uint2* rows = (const uint2*)d_rowinfo;
    if (!d_orig) return inverse_impl(c, d_payload, d_offsets, n, d_out, nullptr, 0, nullptr, rows);
    const Plan& P = c->plan;
    bool all_rix = true;
    for (const UnitDev& d : P.units) all_rix &= d.rix != 0 || d.ncells == 0;
    if (!all_rix) {  // some units decode densely: the two calls, same results
        if ((rc = inverse_impl(c, d_payload, d_offsets, n, d_out, nullptr, 0, nullptr, rows))) return rc;
        return wc_rmse(c, d_orig, dtype, d_out, units, n, d_rmse);
    }
    return inverse_impl(c, d_payload, d_offsets, n, d_out, d_orig, dtype == WC_F64 ? 1 : 0, d_rmse, rows);
}

int wc_inverse_flat(wc_ctx* c, const float* d_flat, const wc_unit* units, int n, float* d_out) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (n == 0) return WC_OK;
    if (!d_flat || !d_out) return fail(c, WC_ERR_INVALID, "null buffer");
    if ((rc = check_aligned(c, d_flat, "flat")) || (rc = check_aligned(c, d_out, "out"))) return rc;
    if ((rc = set_device(c)) || (rc = get_plan(c, units, n))) return rc;
    Plan& P = c->plan;
    StageTimer t(c, WC_STAGE_INVERSE);
    hipError_t e = launch_inverse(c->stream, d_flat, 1, (const UnitDev*)P.d_units.p, (const XTile*)P.d_xtiles.p,
                                  P.ngen, P.lds_inverse, P.nfast, P.lds_fast, d_out);
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

}  // extern "C"

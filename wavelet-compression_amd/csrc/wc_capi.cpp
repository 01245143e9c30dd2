// wc_capi.cpp — the extern "C" boundary (include/wavelet_amd.h).
//
// Owns the per-device context (stream, grow-only scratch in HBM, cached batch
// plans) and turns a batch of units into kernel launches.  No CPU fallback
// exists: every computing entry point launches HIP kernels and fails with
// WC_ERR_HIP if the device or code object is absent.
//
// Forward path per batch (wc_forward), every unit shape: K1 k_transform{,_fast}
// -> flat coefficients in HBM scratch (sparse staging: only the flagged
// segments) + per-unit max keys -> k_transform_fallback (units whose thresh
// is < 0 re-staged densely) -> K2 k_emit (threshold + decoupled look-back +
// ordered pack), writing unit u's serialized bytes at its fixed slot
// offsets[u].  Inverse: K5 k_decode -> dense flat scratch -> K6 k_inverse{,_fast}.
#include "wavelet_amd.h"
#include "wc_internal.h"
#include "wc_hostmem.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>
#include <thread>
#include <condition_variable>

namespace wc {
size_t transform_lds_bytes(int lbx, int lby, int lbz);
size_t transform_fast_lds_bytes(int lbx, int lby, int lbz);
hipError_t launch_transform(hipStream_t, const void*, int, const UnitDev*, const XTile*, uint32_t, size_t,
                            float*, int, unsigned long long*);
hipError_t launch_transform_fast(hipStream_t, const void*, int, const UnitDev*, const XTile*, uint32_t, size_t,
                                 float*, int, unsigned long long*, uint8_t*, uint32_t*, double, uint32_t);
uint32_t transform_pf_grid(size_t lds);
uint32_t inverse_rows_grid(size_t lds);
hipError_t launch_transform_fallback(hipStream_t, const void*, int, const UnitDev*, int, const XTile*, size_t, float*,
                                     const unsigned long long*, const uint32_t*, double);
hipError_t launch_pack(hipStream_t, const UnitDev*, int, const uint32_t*, const uint8_t*, uint64_t*, uint8_t*);
hipError_t launch_decode(hipStream_t, const UnitDev*, const FTile*, uint32_t, const FTile*, uint32_t,
                         unsigned long long*, uint32_t, const uint8_t*, const uint64_t*, uint32_t*,
                         unsigned long long*, float*, uint2*, uint32_t*, int, uint32_t*);
hipError_t launch_pair_counts(hipStream_t, const UnitDev*, int, const uint8_t*, const uint64_t*, uint32_t*, uint32_t*);
hipError_t launch_inverse_rows(hipStream_t, const RTile*, uint32_t, size_t, uint32_t, const uint8_t*,
                               const uint64_t*, const uint2*, float*, int, const void*, int, const UnitDev*, int,
                               double*, double*, bool, const uint32_t*);
hipError_t launch_inverse(hipStream_t, const float*, int, const UnitDev*, const XTile*, uint32_t, size_t, uint32_t,
                          size_t, float*);
hipError_t launch_rmse(hipStream_t, const void*, int, const float*, const UnitDev*, int, const FTile*,
                       uint32_t, double*, double*);
hipError_t launch_emit(hipStream_t, const EmitParams&, const float*, uint32_t, uint32_t);
hipError_t launch_hist(hipStream_t, const UnitDev*, const FTile*, uint32_t, const float*, uint32_t,
                       unsigned long long*);
}  // namespace wc

using namespace wc;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

// A batch plan: unit descriptors and tile lists, mirrored in HBM.
//   xtiles = [generic | fast]   transform tiles, unit-major in each part
//   ixtiles                     the same, fast tiles in reverse unit order (inverse)
//   ftiles                      kFlatTile flat tiles (RMSE, histogram)
//   dtiles                      decode blocks, interleaved by tile index across units
//   edesc                       emit blocks (tile + unit fields), interleaved order
struct Plan {
    std::vector<wc_unit> key;
    std::vector<UnitDev> units;
    std::vector<XTile> xtiles;
    std::vector<XTile> ixtiles;  // dense inverse tiles of the non-row-indexed units: [generic | fast]
    std::vector<RTile> rtiles;   // K6r tiles of the row-indexed units
    std::vector<FTile> ftiles, dtiles, rdtiles;  // dtiles: dense decode, rdtiles: row index (K5)
    int rix_lds = kRixLds;              // WC_OPT_RIX_LDS the plan was built with
    int rix_lx = 4;                     // WC_OPT_RIX_TX the plan was built with
    bool rix_xcd = false;               // WC_OPT_RIX_XCD the plan was built with
    int inv_groups = 1;                 // WC_OPT_INV_GROUPS the plan was built with
    // row-indexed inverse in unit groups (pipelined: K5 of group g + 1 runs
    // beside K6r of group g): group g's row-index tiles are rdtiles
    // [ig_rd[g], ig_rd[g+1]) and its K6r tiles rtiles [ig_rt[g], ig_rt[g+1])
    std::vector<uint32_t> ig_rd, ig_rt;
    std::vector<EmitDesc> edesc;  // [units of kEmitTile tiles | units of kEmitTileBig tiles]
    uint32_t nedesc_small = 0;
    uint32_t ngen = 0, nfast = 0, netiles = 0;
    uint32_t ign = 0, ifast = 0;  // ixtiles split
    bool inv_rows = true;         // WC_OPT_INVERSE_ROWS the plan was built with
    uint64_t rowinfo_entries = 0;
    size_t lds_rows = 0;
    bool any_sparse = false;
    uint64_t coef_extent = 0;  // floats of staged coefficient scratch
    uint64_t flag_bytes = 0;   // bytes of sparse-staging segment flags (UnitDev::flag_off ranges + slack)
    size_t lds_gen = 0, lds_fast = 0, lds_inverse = 0;
    size_t state_bytes = 0;    // forward per-call state: 16 | key[n] | tickets[n] | status[netiles]
    DevBuf d_units, d_xtiles, d_ftiles, d_dtiles, d_edesc, d_ixtiles, d_rtiles, d_rdtiles;
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
    bool opt_ordered = true;  // WC_OPT_ORDERED (see include/wavelet_amd.h)
    bool force_tickets = false;  // WC_OPT_TICKETS: sticky ticket form (set by a look-back timeout)
    uint32_t opt_spin_limit = 0; // WC_OPT_SPIN_LIMIT (0: kSpinLimit), mirrored in errflag[1]
    bool timed_out = false;      // the last error was a look-back wait that timed out
    bool registered = false;     // counted in g_dev_ctx
    bool opt_sparse = true;   // WC_OPT_SPARSE
    bool opt_inv_rows = true; // WC_OPT_INVERSE_ROWS
    int opt_rix_lds = kRixLds; // WC_OPT_RIX_LDS
    int opt_rix_lx = 4;        // WC_OPT_RIX_TX
    bool opt_rix_blocked = false; // WC_OPT_RIX_BLOCKED
    bool opt_rix_xcd = false;     // WC_OPT_RIX_XCD
    int opt_inv_groups = 1;       // WC_OPT_INV_GROUPS
    hipStream_t aux = nullptr;    // second stream of the pipelined inverse
    std::vector<hipEvent_t> iev;  // its events
    // A kernel that may raise error bits ran since the last check.  Kernels
    // atomicOr into ONE persistent error word (errflag, zeroed at creation and
    // after each read), so errors of several async calls accumulate until the
    // next wc_synchronize / _host call reads them.
    bool err_check_pending = false;
    // wc_forward_stage left this plan's coefficients + unit keys in coef/state
    // (cleared by set_device, i.e. by every other compute entry point)
    bool staged = false;
    bool sparse_staged = false;  // the last stage_transform used sparse staging
    uint64_t plan_gen = 0;  // bumped whenever get_plan rebuilds the plan
    // scratch (grow-only)
    DevBuf coef, part, errflag, state, flags, rowinfo, npairs;
    // row index (wc_inverse): epoch-tagged look-back granules, zeroed when
    // allocated and never again (a granule of an earlier call reads as
    // unpublished); epoch: the call counter they are tagged with
    DevBuf istate;
    uint32_t epoch = 0;
    // host-path staging
    DevBuf h_cells, h_payload, h_packed, h_offsets, h_poff, h_kept, h_out;
    // wc_forward_host pipeline: copy streams, per-run events, pinned metadata
    int64_t opt_host_chunk = int64_t(1) << 25;  // WC_OPT_HOST_CHUNK
    hipStream_t up = nullptr, down = nullptr;
    std::vector<hipEvent_t> hev;
    void* pinned = nullptr;
    size_t pinned_bytes = 0;
    // host pages of a copy's destination faulted in ahead of it (wc_hostmem.h)
    int opt_host_threads = -1;    // WC_OPT_HOST_THREADS (-1: not yet resolved from the environment)
    bool opt_host_thp = false;    // WC_OPT_HOST_THP (opt-in: the advice changes the caller's mappings)
    std::unique_ptr<wc::HostPool> hpool;
    // uploads from pageable host memory: copied by upool's threads into pinned
    // bounce slots, each slot's copy to the device ordered by an event
    std::unique_ptr<wc::HostPool> upool;
    void* bounce = nullptr;
    std::vector<hipEvent_t> bev;   // per slot: recorded after the slot's last queued copy
    std::vector<bool> bev_live;    // per slot: bev recorded (wait on it before the slot is rewritten)
    uint32_t bnext = 0;            // next slot (rotates across calls)
    // plans of earlier batches (most recent last), swapped in when a batch recurs
    std::vector<Plan> plan_cache;
    // persistent-grid sizes (resident workgroups for an LDS size) on this device
    std::map<std::pair<int, size_t>, uint32_t> grids;
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

// Device buffers: 16-B aligned (the kernels pick their vector widths from
// element offsets; hipMalloc and torch allocations are 256-B aligned).
int check_aligned(wc_ctx* c, const void* p, const char* what, uintptr_t align = 16) {
    if (((uintptr_t)p & (align - 1)) == 0) return WC_OK;
    return fail(c, WC_ERR_INVALID, std::string(what) + ": device buffer not " + std::to_string(align) + "-byte aligned");
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
    // (64 x 1 x 16 tiles for 128^3 units — whole 512-B fp32 rows — measured
    // slower, round 3: profiles/r03/experiments/gpu_x6.txt.)
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

uint64_t round_up(uint64_t v, uint64_t m) { return (v + m - 1) / m * m; }

// Emit tiles: every unit is split into emit tiles of kEmitTile flat
// coefficients (at least one per unit: an empty unit's tile writes its
// header).  Dispatch order of the emit blocks: interleaved by tile index
// across the units of a group, so that a tile's look-back predecessors (the
// lower tile indices of its unit) have lower block ids and the per-unit
// traffic spreads over the group instead of arriving in one burst.  Groups
// hold >= WC_EMIT_GROUP tiles and >= 128 x the longest unit's tile chain (a
// look-back chain advances one tile per status round trip, so long chains
// need the whole launch to hide in), and run in REVERSE transform order: the
// first emit blocks read the coefficients K1 wrote last, which may still be
// in the Infinity Cache (round 1, 8192-tile groups: 1024 x 64^3 emit 0.346 ->
// 0.327 ms).  Round 3: 65536-tile groups were 3-5 % faster for 8192 x 32^3
// and 32768 x 16^3, equal for 1024 x 64^3, but 7-9 % slower for the full C5
// and C4 batches, where the reverse-order Infinity-Cache reuse matters
// (profiles/r03/experiments/gpu_emit_group.txt): kept at 8192 / 4096.
#ifndef WC_EMIT_GROUP
#define WC_EMIT_GROUP (8192 * 4 / WC_EMIT_EW)  // emit tiles per dispatch group, small-unit launch
#endif
#ifndef WC_EMIT_GROUP_BIG
#define WC_EMIT_GROUP_BIG 4096  // the 8-wave launch (units of >= kEmitBigCells)
#endif
#ifndef WC_EMIT_ILV
#define WC_EMIT_ILV 0  // units interleaved per run of emit blocks within a group (0: every unit of the group)
#endif
void build_etiles(Plan& P, int n) {
    auto big = [](const UnitDev& d) { return d.ncells >= kEmitBigCells; };
    uint32_t total = 0;
    for (int i = 0; i < n; ++i) {
        UnitDev& d = P.units[i];
        const uint64_t tile = big(d) ? kEmitTileBig : kEmitTile;
        d.et_begin = total;
        d.net = (uint32_t)std::max<uint64_t>(1, (d.ncells + tile - 1) / tile);
        total += d.net;
    }
    P.netiles = total;
    // per-call state: 16 (spare) | key[n] (u64) | tickets[n] | spos[n] | spare[n] (u32) |
    // status[tiles] (u64)
    P.state_bytes = round_up(16 + 20ull * n, 8) + 8ull * total;
    P.edesc.clear();
    P.nedesc_small = 0;
    for (int cls = 0; cls < 2; ++cls) {  // one launch per tile size: small units, then big ones
        std::vector<int> us;
        for (int i = 0; i < n; ++i)
            if (big(P.units[i]) == (cls == 1)) us.push_back(i);
        uint32_t maxt = 0;
        for (int i : us) maxt = std::max(maxt, P.units[i].net);
        const uint64_t group_tiles = std::max<uint64_t>(cls ? WC_EMIT_GROUP_BIG : WC_EMIT_GROUP, 128ull * maxt);
        std::vector<std::pair<size_t, size_t>> groups;  // ranges [g0, g1) of us
        for (size_t g0 = 0; g0 < us.size();) {
            uint64_t tiles = 0;
            size_t g1 = g0;
            while (g1 < us.size() && tiles < group_tiles) tiles += P.units[us[g1++]].net;
            groups.emplace_back(g0, g1);
            g0 = g1;
        }
        for (auto g = groups.rbegin(); g != groups.rend(); ++g)
          for (size_t s0 = g->first; s0 < g->second; s0 += (WC_EMIT_ILV ? WC_EMIT_ILV : g->second - g->first)) {
            // interleave by tile index across WC_EMIT_ILV units at a time (0: the whole group)
            const size_t s1 = WC_EMIT_ILV ? std::min<size_t>(g->second, s0 + WC_EMIT_ILV) : g->second;
            uint32_t gmax = 0;
            for (size_t k = s0; k < s1; ++k) gmax = std::max(gmax, P.units[us[k]].net);
            for (uint32_t t = 0; t < gmax; ++t)
                for (size_t k = s0; k < s1; ++k) {
                    const int i = us[k];
                    const UnitDev& d = P.units[i];
                    if (t >= d.net) continue;
                    EmitDesc e{};
                    e.coef_off = d.coef_off;
                    e.pay_off = d.pay_off;
                    e.ncells = d.ncells;
                    e.unit = (uint32_t)i;
                    e.index = t;
                    e.et_begin = d.et_begin;
                    e.net = d.net;
                    e.nx = d.nx;
                    e.ny = d.ny;
                    e.nz = d.nz;
                    e.sparse = d.sparse;
                    e.lbz = d.lbz;
                    e.flag_off = (uint32_t)d.flag_off;
                    P.edesc.push_back(e);
                }
        }
        if (cls == 0) P.nedesc_small = (uint32_t)P.edesc.size();
    }
}

// K6r tiling (wc_inverse.hip k_inverse_rows): TX x TY blocks in (x, y), all of
// z; the tile's LDS is 4 TX ranges of TY*D + 4 floats, at most kRixLds.  TX
// up to 16 blocks (32-cell = 128-B output rows), then TY as large as fits
// (fewer, longer ranges per wave).  Units of
// the fast shape only (even W and H, D % 8 == 0: no odd tails, float4
// sub-band reads); the others decode densely.
size_t rix_lds_bytes(const UnitDev& d) { return sizeof(float) * 4 * (size_t)rix_wr(d.ilbx, d.ilby, d.nz); }

bool set_rix_tiling(UnitDev& d, int budget, int max_lx) {
    d.rix = 0;
    if (!d.fast || d.ncells == 0) return false;
    auto floats = [&](int tx, int ty) { return (int64_t)4 * rix_wr(ceil_log2(tx), ceil_log2(ty), d.nz); };
    int lx = std::min(max_lx, ceil_log2(d.hx));  // 16 blocks: 128-B output rows; the rest of the budget to TY
    while (lx > 0 && floats(1 << lx, 1) > budget) --lx;
    if (floats(1 << lx, 1) > budget) return false;
    int ly = 0;
    while ((1 << ly) < d.hy && floats(1 << lx, 2 << ly) <= budget) ++ly;
    d.ilbx = lx;
    d.ilby = ly;
    d.rix = 1;
    return true;
}

bool plan_matches(const wc_ctx* c, const Plan& P, const wc_unit* units, int n) {
    return P.inv_rows == c->opt_inv_rows && P.rix_lds == c->opt_rix_lds && P.rix_lx == c->opt_rix_lx &&
           P.rix_xcd == c->opt_rix_xcd && P.inv_groups == c->opt_inv_groups &&
           (int)P.key.size() == n && (n == 0 || std::memcmp(P.key.data(), units, sizeof(wc_unit) * n) == 0);
}

void free_plan(Plan& P) {
    DevBuf* bufs[] = {&P.d_units,   &P.d_xtiles, &P.d_ftiles, &P.d_dtiles,
                      &P.d_edesc,   &P.d_ixtiles, &P.d_rtiles, &P.d_rdtiles};
    for (DevBuf* b : bufs) {
        if (b->p) (void)hipFree(b->p);
        *b = DevBuf{};
    }
}

constexpr size_t kPlanCache = 16;  // earlier plans kept (wc_forward_host's unit runs, alternating batches)

// Build (or reuse) the plan for this batch and upload it.  A batch seen
// recently swaps its cached plan back in; a new one pushes the current plan
// into the cache (the oldest cached plan is freed past kPlanCache).
int get_plan(wc_ctx* c, const wc_unit* units, int n) {
    if (c->plan_valid && plan_matches(c, c->plan, units, n)) return WC_OK;
    for (size_t i = 0; i < c->plan_cache.size(); ++i)
        if (plan_matches(c, c->plan_cache[i], units, n)) {
            std::swap(c->plan, c->plan_cache[i]);
            if (!c->plan_valid) {
                free_plan(c->plan_cache[i]);
                c->plan_cache.erase(c->plan_cache.begin() + (std::ptrdiff_t)i);
            }
            c->plan_valid = true;
            ++c->plan_gen;
            return WC_OK;
        }
    if (c->plan_valid) {
        // the new plan is built into the oldest cached plan's buffers (grow-only;
        // the uploads are ordered after every queued kernel on the stream), or
        // into fresh ones while the cache fills
        Plan target{};
        if (c->plan_cache.size() >= kPlanCache) {
            target = std::move(c->plan_cache.front());
            c->plan_cache.erase(c->plan_cache.begin());
        }
        c->plan_cache.push_back(std::move(c->plan));
        c->plan = std::move(target);
    }
    Plan& P = c->plan;
    c->plan_valid = false;
    ++c->plan_gen;
    P.key.assign(units, units + n);
    P.inv_rows = c->opt_inv_rows;
    P.rix_lds = c->opt_rix_lds;
    P.rix_lx = c->opt_rix_lx;
    P.rix_xcd = c->opt_rix_xcd;
    P.inv_groups = c->opt_inv_groups;
    P.units.assign(n, UnitDev{});
    P.xtiles.clear();
    P.ftiles.clear();
    P.ngen = P.nfast = 0;
    P.any_sparse = false;
    P.lds_gen = P.lds_fast = P.lds_inverse = P.lds_rows = 0;
    P.rtiles.clear();
    P.rowinfo_entries = 0;
    std::vector<XTile> gen, fast;
    uint64_t coef_cursor = 0, pay_cursor = 4, flag_cursor = 0;
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
        // row index entries (include/wavelet_amd.h wc_rowindex_bytes): W*H + 1 per unit, every unit
        d.row_off = P.rowinfo_entries;
        P.rowinfo_entries += (uint64_t)u.nx * u.ny + 1;
        d.coef_off = (coef_cursor + 31) & ~uint64_t(31);  // 128 B: sparse-staging segments align
        coef_cursor = d.coef_off + d.ncells;
        if (d.ncells == 0) continue;
        d.fast = (u.nx % 2 == 0) && (u.ny % 2 == 0) && (u.nz % 8 == 0);
        std::vector<XTile>& dst = d.fast ? fast : gen;
        const size_t before = dst.size();
        push_tiles(dst, d, (uint32_t)i);
        d.ntx = (uint32_t)(dst.size() - before);
        // Sparse staging (wc_xform.h xform_fast_p2_sparse): z tiles of >= 16
        // blocks whose flat segments of TZ coefficients each belong to one tile.
        d.sparse = (d.fast && d.lbz >= kSegShift && d.hz % (1 << d.lbz) == 0) ? 1u : 0u;
        if (d.sparse) {  // flag range: whole 2048-coefficient blocks (flag_pos), 8-B aligned
            d.flag_off = flag_cursor;
            flag_cursor += round_up(d.ncells, 2048) >> d.lbz;
            if (flag_cursor >= (uint64_t(1) << 32)) {  // EmitDesc keeps 32 bits: stage densely
                flag_cursor = d.flag_off;                // (and later units may still fit)
                d.sparse = 0;
            }
        }
        P.any_sparse |= d.sparse != 0;
        d.xt_begin = (uint32_t)before;  // rebased below for fast units
        if (d.fast)
            P.lds_fast = std::max(P.lds_fast, transform_fast_lds_bytes(d.lbx, d.lby, d.lbz));
        else
            P.lds_gen = std::max(P.lds_gen, transform_lds_bytes(d.lbx, d.lby, d.lbz));
        P.lds_inverse = std::max(P.lds_inverse, transform_lds_bytes(d.lbx, d.lby, d.lbz));
        if (d.fast) {  // the row-indexable shape: the forward can emit its row index (wc_forward_rows)
            // floor(p / D) = (p * m) >> (31 + l), p < 2^31 (wc_device.h div_rows)
            const int lg = ceil_log2(d.nz);
            const uint64_t m = (uint64_t(1) << (31 + lg)) / (uint64_t)d.nz + 1;
            d.dmagic = m | ((uint64_t)(31 + lg) << 32);
        }
        if (P.inv_rows && set_rix_tiling(d, P.rix_lds, P.rix_lx)) {
            d.rt_begin = (uint32_t)P.rtiles.size();
            for (int by = 0; by < d.hy; by += 1 << d.ilby)
                for (int bx = 0; bx < d.hx; bx += 1 << d.ilbx) {
                    RTile r{};
                    r.row_off = d.row_off;
                    r.cell_off = d.cell_off;
                    r.unit = (uint32_t)i;
                    r.bx0 = bx;
                    r.by0 = by;
                    r.W = d.nx;
                    r.H = d.ny;
                    r.D = d.nz;
                    r.lbx = d.ilbx;
                    r.lby = d.ilby;
                    r.tyv = std::min(1 << d.ilby, d.hy - by);
                    r.nat = (uint32_t)P.rtiles.size();
                    P.rtiles.push_back(r);
                }
            d.nrt = (uint32_t)P.rtiles.size() - d.rt_begin;
            P.lds_rows = std::max(P.lds_rows, rix_lds_bytes(d));
        }
    }
    // K6r tile order, XCD-grouped (WC_OPT_RIX_XCD): workgroups b and b + 8
    // share an XCD (blocks are dealt round-robin over the 8 XCDs; the
    // persistent grid is a multiple of 8), so list position p = 8i + x holds
    // tile start_x + i of a contiguous unit-order run per XCD.  A round of the
    // grid then puts each XCD on a run of whole units: neighbouring tiles of a
    // unit, whose flat-row ranges share payload lines and row entries at their
    // ends, read them through one L2.
    if (P.rix_xcd && P.rtiles.size() > 8) {
        const size_t T = P.rtiles.size();
        std::vector<RTile> perm(T);
        size_t start = 0;
        for (size_t x = 0; x < 8; ++x) {
            const size_t cnt = (T - x + 7) / 8;  // positions p == x (mod 8) below T
            for (size_t i = 0; i < cnt; ++i) perm[8 * i + x] = P.rtiles[start + i];
            start += cnt;
        }
        P.rtiles.swap(perm);
    }
    P.ngen = (uint32_t)gen.size();
    P.nfast = (uint32_t)fast.size();
    for (UnitDev& d : P.units)
        if (d.fast) d.xt_begin += P.ngen;
    P.xtiles = std::move(gen);
    P.xtiles.insert(P.xtiles.end(), fast.begin(), fast.end());
    // Dense inverse tiles of the units that are not row-indexed: generic, then
    // fast in reverse unit order (the first blocks read the coefficients the
    // decode wrote last: Infinity-Cache hits).
    P.ixtiles.clear();
    for (const XTile& x : P.xtiles)
        if (!P.units[x.unit].rix && !P.units[x.unit].fast) P.ixtiles.push_back(x);
    P.ign = (uint32_t)P.ixtiles.size();
    for (auto it = P.xtiles.rbegin(); it != P.xtiles.rend(); ++it)
        if (!P.units[it->unit].rix && P.units[it->unit].fast) P.ixtiles.push_back(*it);
    P.ifast = (uint32_t)P.ixtiles.size() - P.ign;
    for (int i = 0; i < n; ++i) {
        UnitDev& d = P.units[i];
        d.ftile_begin = (uint32_t)P.ftiles.size();
        d.nftiles = (uint32_t)((d.ncells + kFlatTile - 1) / kFlatTile);
        for (uint32_t t = 0; t < d.nftiles; ++t) P.ftiles.push_back(FTile{(uint32_t)i, t});
    }
    // Decode blocks, interleaved by tile index across units: the pair tiles a
    // payload actually has (the low indices) are dispatched first, the blocks
    // past a unit's pairs (which exit at once) last.  A row-indexed unit gets
    // one tile more when kFlatTile divides ncoeff (the virtual pair k = nrle
    // that closes its row index, wc_inverse.hip).
    P.dtiles.clear();
    P.rdtiles.clear();
    {
        uint32_t maxt = 0, total = 0;
        uint64_t rix_cells = 0;
        for (UnitDev& d : P.units) {
            d.ndt = d.rix ? (uint32_t)(d.ncells / kRixTile) + 1 : d.nftiles;
            d.dt_begin = total;
            total += d.ndt;
            maxt = std::max(maxt, d.ndt);
            if (d.rix) rix_cells += d.ncells;
        }
        for (uint32_t t = 0; t < maxt; ++t)
            for (int i = 0; i < n; ++i)
                if (t < P.units[i].ndt && !P.units[i].rix) P.dtiles.push_back(FTile{(uint32_t)i, t});
        // Row-indexed units in up to inv_groups contiguous unit ranges of about
        // equal cells (one group with the XCD-grouped K6r order, which permutes
        // the tiles across units); within a group the row-index tiles are
        // interleaved by tile index across its units (a tile's look-back waits
        // only on lower block ids), and the group's K6r tiles are a contiguous
        // run of the unit-major rtiles.
        const int ng = P.rix_xcd ? 1 : std::max(1, P.inv_groups);
        P.ig_rd.assign(1, 0u);
        P.ig_rt.assign(1, 0u);
        int a = 0;
        for (int g = 0; g < ng && a < n; ++g) {
            const uint64_t target = rix_cells * (uint64_t)(g + 1) / (uint64_t)ng;
            int b = a;
            uint64_t acc = 0;
            for (int i = 0; i < a; ++i) acc += P.units[i].rix ? P.units[i].ncells : 0;
            for (; b < n && (g == ng - 1 || acc < target); ++b)
                if (P.units[b].rix) acc += P.units[b].ncells;
            uint32_t gmax = 0, rt_end = P.ig_rt.back();
            for (int i = a; i < b; ++i)
                if (P.units[i].rix) {
                    gmax = std::max(gmax, P.units[i].ndt);
                    rt_end = P.units[i].rt_begin + P.units[i].nrt;
                }
            for (uint32_t t = 0; t < gmax; ++t)
                for (int i = a; i < b; ++i)
                    if (P.units[i].rix && t < P.units[i].ndt) P.rdtiles.push_back(FTile{(uint32_t)i, t});
            if (P.rdtiles.size() > P.ig_rd.back()) {
                P.ig_rd.push_back((uint32_t)P.rdtiles.size());
                P.ig_rt.push_back(P.rix_xcd ? (uint32_t)P.rtiles.size() : rt_end);
            }
            a = b;
        }
    }
    P.coef_extent = coef_cursor ? coef_cursor + kFlatTile : 0;  // slack: flat tiles read whole float4 groups
    P.flag_bytes = flag_cursor + kEmitTileBig;                  // slack: a partial last tile's flag loads
    build_etiles(P, n);
    int rc;
    if ((rc = upload(c, P.d_units, P.units.data(), sizeof(UnitDev) * P.units.size(), "upload units")) ||
        (rc = upload(c, P.d_xtiles, P.xtiles.data(), sizeof(XTile) * P.xtiles.size(), "upload xtiles")) ||
        (rc = upload(c, P.d_ixtiles, P.ixtiles.data(), sizeof(XTile) * P.ixtiles.size(), "upload ixtiles")) ||
        (rc = upload(c, P.d_ftiles, P.ftiles.data(), sizeof(FTile) * P.ftiles.size(), "upload ftiles")) ||
        (rc = upload(c, P.d_dtiles, P.dtiles.data(), sizeof(FTile) * P.dtiles.size(), "upload dtiles")) ||
        (rc = upload(c, P.d_edesc, P.edesc.data(), sizeof(EmitDesc) * P.edesc.size(), "upload edesc")) ||
        (rc = upload(c, P.d_rtiles, P.rtiles.data(), sizeof(RTile) * P.rtiles.size(), "upload rtiles")) ||
        (rc = upload(c, P.d_rdtiles, P.rdtiles.data(), sizeof(FTile) * P.rdtiles.size(), "upload rdtiles")))
        return rc;
    // The host vectors back the async copies: finish them before returning.
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "plan upload sync");
    c->plan_valid = true;
    return WC_OK;
}

uint64_t decode_tiles(const Plan& P) {
    uint64_t tiles = 0;
    for (const UnitDev& d : P.units) tiles += d.ndt;
    return tiles;
}

// Per-call state of the dense decode: ticket[n] (8-B aligned) | status[decode
// tiles of every unit] (zeroed per call).
size_t decode_state_bytes(const Plan& P) { return round_up(4ull * P.units.size(), 8) + 8ull * decode_tiles(P); }

// Row-index granules: the tiles' sums (at dt_begin).
size_t istate_bytes(const Plan& P) { return 8ull * decode_tiles(P); }

// ensure() for buffers whose contents must start zeroed.
int ensure_zeroed(wc_ctx* c, DevBuf& b, size_t bytes) {
    const void* before = b.p;
    int rc = ensure(c, b, bytes);
    if (rc || b.p == before) return rc;
    hipError_t e = hipMemsetAsync(b.p, 0, b.bytes, c->stream);
    return e == hipSuccess ? WC_OK : hip_fail(c, e, "memset");
}

// Scratch of the staged forward, the inverse and the RMSE (grow-only).
int ensure_scratch(wc_ctx* c) {
    const Plan& P = c->plan;
    const size_t nft = P.ftiles.size();
    int rc;
    if ((rc = ensure(c, c->coef, sizeof(float) * std::max<uint64_t>(P.coef_extent, 1))) ||
        (rc = ensure(c, c->flags, P.flag_bytes)) ||
        (rc = ensure(c, c->part, sizeof(double) * std::max<size_t>(nft, 4 * P.rtiles.size()))) ||
        (rc = ensure(c, c->rowinfo, sizeof(uint32_t) * 2 * std::max<uint64_t>(P.rowinfo_entries, 1))) ||
        (rc = ensure(c, c->npairs, sizeof(uint32_t) * P.units.size())) ||
        (rc = ensure_zeroed(c, c->istate, istate_bytes(P))) ||
        (rc = ensure(c, c->state, std::max(P.state_bytes, decode_state_bytes(P)))))
        return rc;
    return WC_OK;
}

// Resident workgroups of a persistent kernel (which: 0 k_transform_fast_pf,
// 1 k_inverse_rows) for an LDS size, cached per context (one device).
uint32_t persistent_grid(wc_ctx* c, int which, size_t lds) {
    auto key = std::make_pair(which, lds);
    auto it = c->grids.find(key);
    if (it != c->grids.end()) return it->second;
    const uint32_t g = which == 0 ? transform_pf_grid(lds) : inverse_rows_grid(lds);
    c->grids[key] = g;
    return g;
}

// The pipelined inverse's second stream and `nev` events (created once).
int inverse_stream(wc_ctx* c, int nev) {
    hipError_t e;
    if (!c->aux && (e = hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking)) != hipSuccess)
        return hip_fail(c, e, "inverse stream");
    while ((int)c->iev.size() < nev) {
        hipEvent_t ev;
        if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return hip_fail(c, e, "event");
        c->iev.push_back(ev);
    }
    return WC_OK;
}

int set_device(wc_ctx* c) {
    c->staged = false;
    hipError_t e = hipSetDevice(c->device);
    return e == hipSuccess ? WC_OK : hip_fail(c, e, "hipSetDevice");
}

// Live contexts per device, process-wide.  The look-backs' launch-order form
// (WC_OPT_ORDERED 1) assumes the kernel owns the device's dispatch: with two
// contexts' kernels in flight on one device, each can fill an XCD with blocks
// that wait on blocks of its own kernel that the other's occupancy keeps from
// being dispatched.  Contexts sharing a device therefore use the per-unit
// tickets (blocks wait only on tiles that running blocks hold).
std::mutex g_dev_mu;
std::map<int, int> g_dev_ctx;

// WCAMD_SHARED_DEVICE=1 (read once per process): this process shares its GPUs
// with other processes that run look-back kernels, so every context takes the
// ticket form (the launch-order form's dispatch assumption does not hold).
bool shared_device_env() {
    static const bool v = [] {
        const char* e = std::getenv("WCAMD_SHARED_DEVICE");
        return e && *e && std::strcmp(e, "0") != 0;
    }();
    return v;
}

bool use_ordered(const wc_ctx* c) {
    if (!c->opt_ordered || c->force_tickets || shared_device_env()) return false;
    std::lock_guard<std::mutex> lk(g_dev_mu);
    auto it = g_dev_ctx.find(c->device);
    return it == g_dev_ctx.end() || it->second <= 1;
}

// Surface an error bit a kernel raised (malformed payload in the decode, a
// look-back wait that timed out) at the next synchronisation point, and clear
// the word.  The reference exits on a malformed payload
// (src/decompressor.cpp:228-231); here it is WC_ERR_FORMAT.
int check_kernel_errors(wc_ctx* c) {
    if (!c->err_check_pending) return WC_OK;
    c->err_check_pending = false;
    uint32_t flag = 0;
    hipError_t e = hipMemcpyAsync(&flag, c->errflag.p, 4, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess && flag) e = hipMemsetAsync(c->errflag.p, 0, 4, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "error flag readback");
    if (flag & (kErrHeader | kErrNegativeRun)) {
        char buf[128];
        std::snprintf(buf, sizeof buf, "malformed payload (flags 0x%x: 1 header, 2 negative run)", flag);
        return fail(c, WC_ERR_FORMAT, buf);
    }
    if (flag & kErrTimeout) {
        // Sticky: a launch-order look-back that timed out means another
        // kernel holds the dispatch slots its predecessors need (a shared
        // device); every later call of this context takes the ticket form.
        c->timed_out = true;
        c->force_tickets = true;
        return fail(c, WC_ERR_HIP, "a dependency wait between workgroups timed out");
    }
    return WC_OK;
}

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
    p.ordered = use_ordered(c) ? 1u : 0u;
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
    c->err_check_pending = true;  // a look-back wait that timed out surfaces at wc_synchronize
    return WC_OK;
}

int forward_staged(wc_ctx* c, const void* d_cells, int dtype, int n, double keep, uint8_t* d_payload,
                   uint64_t* d_offsets, uint32_t* d_kept, uint2* d_rows = nullptr) {
    int rc = stage_transform(c, d_cells, dtype, keep, c->opt_sparse);
    return rc ? rc : stage_emit(c, n, keep, nullptr, d_payload, d_offsets, d_kept, d_rows);
}

uint64_t cells_extent(const wc_unit* units, int n) {
    uint64_t ext = 0;
    for (int i = 0; i < n; ++i)
        ext = std::max(ext, units[i].cell_offset + (uint64_t)units[i].nx * units[i].ny * units[i].nz);
    return ext;
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
    {
        std::lock_guard<std::mutex> lk(g_dev_mu);
        ++g_dev_ctx[device];
        c->registered = true;
    }
    *out = c;
    return WC_OK;
}

void wc_ctx_destroy(wc_ctx* c) {
    if (!c) return;
    if (c->registered) {
        std::lock_guard<std::mutex> lk(g_dev_mu);
        --g_dev_ctx[c->device];
    }
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (c->aux) (void)hipStreamSynchronize(c->aux);
    DevBuf* bufs[] = {&c->coef,          &c->part,           &c->errflag,        &c->state,
                      &c->flags,         &c->h_cells,        &c->h_payload,      &c->h_packed,
                      &c->h_offsets,     &c->h_poff,         &c->h_kept,         &c->h_out,
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

static int host_threads_default();

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
    if ((rc = check_aligned(c, d_cells, "cells")) || (rc = check_aligned(c, d_payload, "payload")) ||
        (rc = check_aligned(c, d_offsets, "offsets", 8)) || (rc = check_aligned(c, d_kept, "kept", 4)))
        return rc;
    if ((rc = set_device(c)) || (rc = get_plan(c, units, n))) return rc;
    if ((rc = ensure_scratch(c))) return rc;
    return forward_staged(c, d_cells, dtype, n, keep, d_payload, d_offsets, d_kept);
}

uint64_t wc_rowindex_bytes(const wc_unit* units, int n) {
    uint64_t e = 0;
    for (int i = 0; i < n; ++i) e += (uint64_t)units[i].nx * units[i].ny + 1;
    return 8 * e;
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
    if ((rc = ensure_scratch(c)) || (rc = stage_transform(c, d_cells, dtype, 0.0, false))) return rc;
    if (d_hist) {
        const uint32_t max_blocks = 2048;  // 8 workgroups per CU, 256 CUs
        const Plan& P = c->plan;
        StageTimer t(c, WC_STAGE_HIST);
        hipError_t e = launch_hist(c->stream, (const UnitDev*)P.d_units.p, (const FTile*)P.d_ftiles.p,
                                   (uint32_t)P.ftiles.size(), (const float*)c->coef.p, max_blocks,
                                   (unsigned long long*)d_hist);
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
                             (float*)c->coef.p, (uint2*)c->rowinfo.p, (uint32_t*)c->errflag.p, ord ? 1 : 0,
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
    return wc_inverse_rows(c, d_payload, d_offsets, units, n, nullptr, nullptr, WC_F32, d_out, nullptr);
}

int wc_inverse_rmse(wc_ctx* c, const uint8_t* d_payload, const uint64_t* d_offsets, const wc_unit* units, int n,
                    const void* d_orig, int dtype, float* d_out, double* d_rmse) {
    if (!c) return WC_ERR_INVALID;
    if (n > 0 && (!d_orig || !d_rmse)) return fail(c, WC_ERR_INVALID, "null buffer");
    return wc_inverse_rows(c, d_payload, d_offsets, units, n, nullptr, d_orig, dtype, d_out, d_rmse);
}

// wc_inverse / wc_inverse_rmse, and with d_rowinfo the caller's row index in
// place of the row index kernel (wc_forward_rows wrote it for these payloads).
int wc_inverse_rows(wc_ctx* c, const uint8_t* d_payload, const uint64_t* d_offsets, const wc_unit* units, int n,
                    const void* d_rowinfo, const void* d_orig, int dtype, float* d_out, double* d_rmse) {
    if (!c) return WC_ERR_INVALID;
    int rc;
    if ((rc = validate_units(c, units, n))) return rc;
    if (d_orig && dtype != WC_F32 && dtype != WC_F64) return fail(c, WC_ERR_INVALID, "dtype");
    if (n == 0) return WC_OK;
    if (!d_payload || !d_offsets || !d_out || (!d_orig != !d_rmse)) return fail(c, WC_ERR_INVALID, "null buffer");
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
static int host_threads_default() {
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
extern "C++" {
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

static int forward_host_once(wc_ctx* c, const void* cells, int dtype, const wc_unit* units, int n, double keep,
                             uint8_t* payload, uint64_t cap, uint64_t* offsets, uint32_t* kept) {
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
    for (int r = 0; r < nr; ++r) pbase[r + 1] = pbase[r] + wc_payload_bound(units + rb[r], rb[r + 1] - rb[r]);
    const size_t meta_bytes = sizeof(uint64_t) * (size_t)(n + nr) + 4ull * n;
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
            if (hi > lo &&
                (e = host_upload(c, d_cells + esz * lo, (const uint8_t*)cells + esz * lo, esz * (hi - lo), cs)) !=
                    hipSuccess)
                return hip_fail(c, e, "cells upload");
            if (nr > 1 && ((e = hipEventRecord(c->hev[2 * r], c->up)) != hipSuccess ||
                           (e = hipStreamWaitEvent(c->stream, c->hev[2 * r], 0)) != hipSuccess))
                return hip_fail(c, e, "upload event");
            uint8_t* pay = (uint8_t*)c->h_payload.p + pbase[r];
            uint8_t* packed = (uint8_t*)c->h_packed.p + pbase[r];
            uint64_t* doff = (uint64_t*)c->h_offsets.p + (a + r);
            uint64_t* dpoff = (uint64_t*)c->h_poff.p + (a + r);
            uint32_t* dkept = (uint32_t*)c->h_kept.p + a;
            int rc2;
            if ((rc2 = wc_forward(c, c->h_cells.p, dtype, units + a, m, keep, pay, pbase[r + 1] - pbase[r], doff,
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

// The host-buffer entry points own their inputs until they return, so a
// launch-order look-back that timed out (another process's kernels holding the
// dispatch slots its predecessors need, DESIGN.md §Forward progress) is run
// again once with the per-unit tickets, which need no dispatch order.
extern "C++" {
template <class F>
static int with_ticket_retry(wc_ctx* c, F once) {
    c->timed_out = false;
    const bool was_tickets = c->force_tickets;
    int rc = once();
    // check_kernel_errors made the ticket form sticky; run once more with it
    if (rc == WC_ERR_HIP && c->timed_out && !was_tickets) rc = once();
    return rc;
}
}

int wc_forward_host(wc_ctx* c, const void* cells, int dtype, const wc_unit* units, int n, double keep,
                    uint8_t* payload, uint64_t cap, uint64_t* offsets, uint32_t* kept) {
    if (!c) return WC_ERR_INVALID;
    return with_ticket_retry(
        c, [&] { return forward_host_once(c, cells, dtype, units, n, keep, payload, cap, offsets, kept); });
}

int wc_inverse_host(wc_ctx* c, const uint8_t* payload, const uint64_t* offsets, const wc_unit* units, int n,
                    float* out) {
    if (!c) return WC_ERR_INVALID;
    return with_ticket_retry(c, [&] { return inverse_host_once(c, payload, offsets, units, n, out); });
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

// wc_plan.cpp — batch plans of the C-ABI (wc_ctx.h): unit descriptors,
// transform / emit / row-index / K6r tile lists and the row-index layout,
// built once per distinct batch, mirrored in HBM and cached; scratch sizing.
#include "wc_ctx.h"

#include <algorithm>
#include <cstring>

namespace wc {

static void set_tiling(UnitDev& d) {
    // Up to 32 blocks along x (coalesced input rows) and z (contiguous flat
    // rows), the rest along y, at most kMaxTileBlocks blocks per tile.
    // (64 x 1 x 16 tiles for 128^3 units — whole 512-B fp32 rows — measured
    // slower, round 3: profiles/r03/experiments/gpu_x6.txt.)
    d.lbx = std::min(5, ceil_log2(std::max(1, d.nbx)));
    d.lbz = std::min(5, ceil_log2(std::max(1, d.nbz)));
    d.lby = std::min(ceil_log2(std::max(1, d.nby)), 10 - d.lbx - d.lbz);
}

static void push_tiles(std::vector<XTile>& v, const UnitDev& d, uint32_t u) {
    const int TX = 1 << d.lbx, TY = 1 << d.lby, TZ = 1 << d.lbz;
    for (int bz = 0; bz < d.nbz; bz += TZ)
        for (int by = 0; by < d.nby; by += TY)
            for (int bx = 0; bx < d.nbx; bx += TX) v.push_back(XTile{u, (uint32_t)bx, (uint32_t)by, (uint32_t)bz});
}


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
static void build_etiles(Plan& P, int n) {
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
                    e.ncells = (uint32_t)d.ncells;
                    e.unit = (uint32_t)i;
                    e.index = t;
                    e.et_begin = d.et_begin;
                    e.net = d.net;
                    e.nx = d.nx;
                    e.ny = d.ny;
                    e.nz = d.nz;
                    e.mode = (d.sparse ? 1u : 0u) | ((uint32_t)d.lbz << 1) | ((uint32_t)(d.dmagic >> 32) << 8);
                    e.flag_off = (uint32_t)d.flag_off;
                    e.row_off = (uint32_t)d.row_off;
                    e.dmul = (uint32_t)d.dmagic;
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
static size_t rix_lds_bytes(const UnitDev& d) { return sizeof(float) * 4 * (size_t)rix_wr(d.ilbx, d.ilby, d.nz); }

static bool set_rix_tiling(UnitDev& d, int budget, int max_lx) {
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

static bool plan_matches(const wc_ctx* c, const Plan& P, const wc_unit* units, int n) {
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

static constexpr size_t kPlanCache = 16;  // earlier plans kept (wc_forward_host's unit runs, alternating batches)

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
        // row index entries (include/wavelet_amd.h wc_rowindex_bytes): W*H + 1 per unit with
        // cells, none for an empty one (which writes and reads no entry)
        d.row_off = P.rowinfo_entries;
        if (d.ncells) P.rowinfo_entries += (uint64_t)u.nx * u.ny + 1;
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
            // floor(p / D) = (p * m) >> (31 + l), p < 2^31, or p >> l for D = 2^l (wc_device.h div_rows)
            const int lg = ceil_log2(d.nz);
            const uint64_t m = (uint64_t(1) << (31 + lg)) / (uint64_t)d.nz + 1;
            d.dmagic = (d.nz & (d.nz - 1)) == 0 ? (uint64_t)lg << 32 : m | ((uint64_t)(31 + lg) << 32);
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

static uint64_t decode_tiles(const Plan& P) {
    uint64_t tiles = 0;
    for (const UnitDev& d : P.units) tiles += d.ndt;
    return tiles;
}

// Per-call state of the dense decode: ticket[n] (8-B aligned) | status[decode
// tiles of every unit] (zeroed per call).
size_t decode_state_bytes(const Plan& P) { return round_up(4ull * P.units.size(), 8) + 8ull * decode_tiles(P); }

// Row-index granules: the tiles' sums (at dt_begin).
static size_t istate_bytes(const Plan& P) { return 8ull * decode_tiles(P); }

// ensure() for buffers whose contents must start zeroed.
static int ensure_zeroed(wc_ctx* c, DevBuf& b, size_t bytes) {
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
// 1 k_inverse_rows, 2 k_transform_hist) for an LDS size, cached per context
// (one device).
uint32_t persistent_grid(wc_ctx* c, int which, size_t lds) {
    auto key = std::make_pair(which, lds);
    auto it = c->grids.find(key);
    if (it != c->grids.end()) return it->second;
    const uint32_t g = which == 0 ? transform_pf_grid(lds) : which == 1 ? inverse_rows_grid(lds) : transform_hist_grid(lds);
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

}  // namespace wc

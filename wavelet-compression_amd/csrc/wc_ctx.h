// wc_ctx.h — the library context and batch plan, shared by the translation
// units behind the C-ABI (include/wavelet_amd.h).  Internal: not installed.
//
//   wc_common.cpp    errors, device buffers, unit validation, the process-wide
//                    context registry (launch-order vs ticket look-backs), the
//                    kernel error word
//   wc_plan.cpp      batch plans (tile lists, emit descriptors, row-index
//                    layout) mirrored in HBM, scratch sizing
//   wc_capi.cpp      context lifetime, options and the device-pointer entry
//                    points (kernel launches)
//   wc_hostpipe.cpp  the _host entry points: pipelined unit runs over PCIe,
//                    pinned bounce slots, helper threads (no kernels of its
//                    own: it calls the device entry points), also built
//                    against a CPU fake of the HIP runtime for the sanitizer
//                    tests (tests/cpp/test_hostpipe.cpp)
#pragma once

#include "wavelet_amd.h"
#include "wc_hostmem.h"
#include "wc_internal.h"

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace wc {

size_t transform_lds_bytes(int lbx, int lby, int lbz);
size_t transform_fast_lds_bytes(int lbx, int lby, int lbz);
hipError_t launch_transform(hipStream_t, const void*, int, const UnitDev*, const XTile*, uint32_t, size_t,
                            float*, int, unsigned long long*);
hipError_t launch_transform_fast(hipStream_t, const void*, int, const UnitDev*, const XTile*, uint32_t, size_t,
                                 float*, int, unsigned long long*, uint8_t*, uint32_t*, double, uint32_t);
uint32_t transform_pf_grid(size_t lds);
size_t transform_hist_lds_bytes(size_t lds_fast);
uint32_t transform_hist_grid(size_t lds);
hipError_t launch_transform_hist(hipStream_t, const void*, int, const UnitDev*, const XTile*, uint32_t, size_t,
                                 float*, unsigned long long*, unsigned long long*, uint32_t);
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
                       unsigned long long*, bool);

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

inline int ceil_log2(int64_t v) {
    int l = 0;
    while ((int64_t(1) << l) < v) ++l;
    return l;
}

inline uint64_t round_up(uint64_t v, uint64_t m) { return (v + m - 1) / m * m; }

}  // namespace wc

using wc::kRixLds;

struct wc_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    wc::Plan plan;
    bool plan_valid = false;
    bool opt_ordered = true;  // WC_OPT_ORDERED (see include/wavelet_amd.h)
    bool force_tickets = false;  // WC_OPT_TICKETS: the ticket form of the look-backs
    bool opt_reverse = false;    // WC_OPT_REVERSE_TILES (test hook): each unit's look-back tiles in reverse launch order
    uint32_t opt_spin_limit = 0; // WC_OPT_SPIN_LIMIT (0: kSpinSelf), mirrored in errflag[1]
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
    wc::DevBuf coef, part, errflag, state, flags, rowinfo, npairs;
    // row index (wc_inverse): epoch-tagged look-back granules, zeroed when
    // allocated and never again (a granule of an earlier call reads as
    // unpublished); epoch: the call counter they are tagged with
    wc::DevBuf istate;
    uint32_t epoch = 0;
    // host-path staging
    wc::DevBuf h_cells, h_payload, h_packed, h_offsets, h_poff, h_kept, h_out;
    wc::DevBuf h_rows, h_rmse;  // wc_round_trip_host: a run's row index, the per-unit RMSE
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
    std::vector<wc::Plan> plan_cache;
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

namespace wc {

// wc_common.cpp
int fail(wc_ctx* c, int code, const std::string& msg);
int hip_fail(wc_ctx* c, hipError_t e, const char* what);
int ensure(wc_ctx* c, DevBuf& b, size_t bytes);      // grow-only device buffer
int validate_units(wc_ctx* c, const wc_unit* units, int n);
int check_aligned(wc_ctx* c, const void* p, const char* what, uintptr_t align = 16);
hipEvent_t take_event(wc_ctx* c);
int upload(wc_ctx* c, DevBuf& d, const void* h, size_t bytes, const char* what);
int set_device(wc_ctx* c);
bool use_ordered(const wc_ctx* c);
int check_kernel_errors(wc_ctx* c);
uint64_t cells_extent(const wc_unit* units, int n);

// wc_plan.cpp
int get_plan(wc_ctx* c, const wc_unit* units, int n);
void free_plan(Plan& P);
size_t decode_state_bytes(const Plan& P);
int ensure_scratch(wc_ctx* c);
uint32_t persistent_grid(wc_ctx* c, int which, size_t lds);
int inverse_stream(wc_ctx* c, int nev);

// wc_hostpipe.cpp
int host_threads_default();

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

}  // namespace wc

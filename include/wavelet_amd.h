/*
 * wavelet_amd.h — C-ABI of the MI355X (gfx950) wavelet codec.
 *
 * This is the drop-in boundary for the reference's per-box hot path
 * (carsonmw3/wavelet-compression @ 2025-07-04).  The reference calls its codec
 * through C++ functions; the C++ mirror in include/wavelet_amd/ keeps those
 * exact signatures and forwards to the entry points below.  Each entry point
 * names the reference routine(s) it replaces:
 *
 *   wc_forward         compress() minus the xz write      src/compressor.h:9-15,
 *                      = wavelet_decompose + threshold     src/compressor.cpp:192-248
 *                        + rle_encode + serialize          src/compressor.cpp:24-80
 *   wc_decompose       wavelet_decompose                   src/compressor.cpp:85-185
 *   wc_inverse         decompress() minus the xz read      src/decompressor.h:6-10
 *                      = rle_decode + inverse transform    src/decompressor.cpp:14-30,238-255
 *   wc_inverse_flat    inverse_wavelet_decompose           src/decompressor.h:18, .cpp:79-159
 *   wc_rmse            calc_rmse_per_box (one component)   src/calc-loss.h:6-8, .cpp:12-43
 *
 * Conventions
 *   - Plain C types only; every function returns WC_OK (0) or a WC_ERR_* code,
 *     and wc_last_error() describes the last failure on that context.
 *   - A "unit" is one Box3D component (one (time, level, box, component) tuple
 *     of the reference's AMRIterator loop, src/modes.cpp:100-103): W x H x D
 *     cells, x fastest (src/grid.h:15-19).  Batches of units run in one call.
 *   - Functions without a _host suffix take DEVICE pointers (HBM-resident data)
 *     and are asynchronous on the context's stream.  _host variants take host
 *     pointers, copy through pinned staging, and return when results are ready.
 *   - Device buffers of cells, payloads, coefficients and reconstructions must
 *     be 16-byte aligned (hipMalloc and torch allocations are); offsets,
 *     kept counts, row indexes and RMSE outputs need their element alignment;
 *     both inputs of wc_rmse (the original cells and the reconstruction) and
 *     the original cells of the fused calls, any element alignment (wc_rmse
 *     only reads them).  Otherwise WC_ERR_INVALID.
 *   - One context per device per host thread.  The context owns its stream and
 *     its scratch memory; the caller owns every buffer it passes.
 *
 * Payload layout: unit u's serialized bytes, IDENTICAL to the reference's
 * serialize_compressed_wavelet output (src/compressor.cpp:55-80)
 *     int32 W, H, D; int32 ncoeff = W*H*D; int32 nrle; nrle x {int32 run, float32 value}
 * start at payload + offsets[u] and are 20 + 8*kept[u] bytes long.  Every
 * offsets[u] is == 4 (mod 8), so each pair is 8-byte aligned.
 *   - wc_forward (device): offsets[u] is unit u's fixed SLOT, the prefix of the
 *     worst-case sizes 24 + 8*W*H*D of the units before it (starting at 4), so
 *     no unit waits for another's kept count; offsets[n] = end of the last
 *     unit's bytes.  The buffer between units is not written.
 *   - wc_forward_host: the slots are packed densely (each unit 24 + 8*kept[u]
 *     bytes apart) before the copy back; offsets[] describe the packed buffer.
 *   - wc_inverse / wc_inverse_host accept any offsets that are multiples of 4.
 */
#ifndef WAVELET_AMD_H
#define WAVELET_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WC_OK 0
#define WC_ERR_INVALID 1  /* bad argument (null pointer, negative dims, capacity too small) */
#define WC_ERR_HIP 2      /* a HIP runtime call failed */
#define WC_ERR_NOMEM 3    /* device or pinned allocation failed */
#define WC_ERR_FORMAT 4   /* a payload header disagrees with its unit, or a run is negative */

#define WC_F32 0          /* cells are float32 (Box3D, src/box-structs.h:7) */
#define WC_F64 1          /* cells are float64 (plotfile FAB), narrowed in-kernel (src/preprocess.cpp:78) */

typedef struct wc_unit {
    uint64_t cell_offset; /* element offset of the unit's first cell in the cell buffer */
    int32_t nx;           /* Grid3D width  (x, fastest) */
    int32_t ny;           /* Grid3D height (y) */
    int32_t nz;           /* Grid3D depth  (z, slowest) */
    int32_t reserved;     /* must be 0 */
} wc_unit;

typedef struct wc_ctx wc_ctx;

/* Context lifetime.  `device` is a HIP device ordinal. */
int wc_device_count(void);  /* HIP devices visible to this process (0 without a GPU) */
int wc_ctx_create(int device, wc_ctx** out);
void wc_ctx_destroy(wc_ctx* ctx);
const char* wc_last_error(const wc_ctx* ctx);

/* Run on an external hipStream_t (e.g. a torch stream); NULL restores the
 * context's own stream.  Switching drains the previous stream first (kernels
 * queued there may still read the plan and scratch that later calls reuse), so
 * a caller must switch away from its stream BEFORE destroying it.  The switch
 * takes effect even when that drain fails (the error is still returned). */
int wc_set_stream(wc_ctx* ctx, void* hip_stream);
int wc_synchronize(wc_ctx* ctx);  /* also reports (and clears) kernel-side errors of earlier async calls */

/* Tuning switches (wc_set_option).
 * WC_OPT_SPARSE (default 1): the forward's transform stores only the
 *   16/32-coefficient flat segments that hold some |c| > (tile max) * (1 - keep)
 *   and flags them; the emit loads only flagged segments.  Same bytes out;
 *   0 = dense staging of every coefficient.
 * WC_OPT_RIX_XCD (default 0): the row-indexed inverse's tiles dealt to the XCDs
 *   in contiguous runs (neighbouring tiles share payload lines at their range
 *   ends).  Same cells.
 * WC_OPT_INV_GROUPS (default 1): the row-indexed inverse runs in this many
 *   unit groups, pipelined: the row index of group g + 1 (latency-bound) runs
 *   beside the reconstruction of group g on a second stream of the context;
 *   the call stays ordered on the context's stream.  Same cells.  Measured
 *   slower on MI355X (C2: 0.53 ms at 1 group, 0.62 at 2, 0.59 at 4), kept as
 *   an option for workloads whose row index dominates.
 * WC_OPT_ORDERED (default 1): the look-back kernels (forward emit, inverse
 *   row index and decode) take each block's tile index from the launch order
 *   (no atomic per block); 0 takes it from a per-unit ticket atomic instead.
 *   Same bytes out either way, and neither form depends on the order in which
 *   the hardware dispatches workgroups or on other kernels sharing the device:
 *   a block that has waited its bound (WC_OPT_SPIN_LIMIT) for a predecessor
 *   tile to publish derives that tile's count from the tile's own inputs and
 *   goes on (DESIGN.md §Forward progress).  Several contexts or processes may
 *   share a GPU in either form.  wc_get_option(WC_OPT_ORDERED) returns the form
 *   the next launch takes.
 * WC_OPT_TICKETS (default 0): 1 = this context uses the ticket form whatever
 *   WC_OPT_ORDERED says.
 * WC_OPT_SPIN_LIMIT (default 0 = 64 polls, about 0.1 ms): unanswered polls of
 *   an unpublished predecessor before a waiting block derives it itself.  Any
 *   value gives the same bytes; 1 makes nearly every wait take that path
 *   (tests).
 * WC_OPT_REVERSE_TILES (default 0; test hook): the launch-order form with each
 *   unit's tile indices reversed, so that every look-back waits on blocks
 *   dispatched after it (the worst dispatch order).  Same bytes, slower.
 * WC_OPT_INVERSE_ROWS (default 1): the inverse of even-dims units (W, H even,
 *   D % 8 == 0) indexes the payload's pairs by flat row and reconstructs each
 *   tile straight from the payload; 0 decodes every unit into a dense fp32
 *   coefficient scratch first (4 B/cell written and read back).  Same cells.
 * WC_OPT_RIX_LDS (default 9216), WC_OPT_RIX_TX (default 4): tile shape of the
 *   row-indexed inverse: LDS floats per workgroup (1024..16384) and log2 of the
 *   tile's blocks along x (0..5); y takes the rest of the budget.  Same cells.
 * WC_OPT_RIX_BLOCKED (default 0): each workgroup of the row-indexed inverse
 *   runs a contiguous run of tiles (0: tiles b, b + grid, ...).  Same cells.
 * WC_OPT_HOST_CHUNK (default 2^25 cells): wc_forward_host splits a batch of
 *   more than two such chunks into contiguous unit runs of about this many
 *   cells (at most 16 runs) and pipelines them: the cells of run r+1 upload
 *   while run r computes and run r-1's packed payloads download.  Same bytes
 *   and offsets out; 0 = one run.  wc_inverse_host runs the same way (run
 *   r+1's payload bytes upload while run r decodes and run r-1's boxes
 *   download).
 * WC_OPT_HOST_THREADS (default: OMP_NUM_THREADS, else the cores, at most 16):
 *   wc_forward_host / wc_inverse_host make the pages of each destination span
 *   of the caller's host buffer resident (MADV_POPULATE_WRITE, no byte
 *   changed) from this many threads just before the device-to-host copy into
 *   it: a copy into never-touched pageable memory otherwise takes the page
 *   faults on its own thread (C2 payloads: 12-20 GB/s instead of the link's
 *   57).  0 = leave the faults to the copy.  Whole pages inside a span only.
 * WC_OPT_HOST_THP (default 0): 1 = also advise transparent huge pages
 *   (MADV_HUGEPAGE) on the 2-MiB-aligned interior of those spans first.  Off
 *   by default: the advice splits the caller's mappings and changes their
 *   huge-page policy for the life of the mapping (the caller owns its memory).
 */
#define WC_OPT_SPARSE 12
#define WC_OPT_ORDERED 13
#define WC_OPT_INVERSE_ROWS 14
#define WC_OPT_RIX_LDS 15
#define WC_OPT_RIX_TX 16
#define WC_OPT_RIX_BLOCKED 17
#define WC_OPT_HOST_CHUNK 18
#define WC_OPT_SPIN_LIMIT 19
#define WC_OPT_TICKETS 20
#define WC_OPT_REVERSE_TILES 29
#define WC_OPT_RIX_XCD 22
#define WC_OPT_INV_GROUPS 23
/* 24, 25: retired (the round-4 cohort forward, removed: slower than the
 * two-kernel forward in every measured shape) */
#define WC_OPT_HOST_THREADS 27
#define WC_OPT_HOST_THP 28
int wc_set_option(wc_ctx* ctx, int option, int64_t value);
int wc_get_option(const wc_ctx* ctx, int option, int64_t* value);

/* Host-side helpers (no device work). */
uint64_t wc_payload_bound(const wc_unit* units, int n);  /* worst case: every coefficient kept */
uint64_t wc_cell_count(const wc_unit* units, int n);

/* Forward path for a batch: fp64/fp32 cells -> serialized payloads.
 * keep: the reference's `keep` (a float widened to double, src/argparse.h:13).
 * d_offsets: n+1 uint64, d_kept: n uint32 (both device).  payload_capacity must
 * be >= wc_payload_bound(units, n). */
int wc_forward(wc_ctx* ctx, const void* d_cells, int dtype, const wc_unit* units, int n,
               double keep, uint8_t* d_payload, uint64_t payload_capacity,
               uint64_t* d_offsets, uint32_t* d_kept);

int wc_forward_host(wc_ctx* ctx, const void* cells, int dtype, const wc_unit* units, int n,
                    double keep, uint8_t* payload, uint64_t payload_capacity,
                    uint64_t* offsets, uint32_t* kept);

/* wc_forward_host with unit u's W*H*D cells at its own host pointer cells[u]
 * (units[u].cell_offset is ignored): the C++ mirror's compress() hands over
 * the Box3D components it was given (src/compressor.h:9-15) without packing
 * them into one buffer first.  Same payload, offsets and kept counts as
 * wc_forward_host of the packed components. */
int wc_forward_host_units(wc_ctx* ctx, const void* const* cells, int dtype, const wc_unit* units, int n,
                          double keep, uint8_t* payload, uint64_t payload_capacity,
                          uint64_t* offsets, uint32_t* kept);

/* The reference's -estimate round trip on host buffers (src/modes.cpp:236-291:
 * compress the boxes, decompress them again, calc_rmse_per_box against the
 * originals, src/calc-loss.cpp:12-43): wc_forward_host's outputs (packed
 * payloads, offsets, kept counts), plus rmse[u] = the RMSE of unit u's
 * reconstruction against its cells.  The payloads are decoded again on the
 * device with the forward's row index (wc_forward_rows / wc_inverse_rows) and
 * compared there with the cells already uploaded for the forward: the cells
 * cross PCIe once and the reconstruction never does.  RMSE identical to
 * wc_rmse_host of the decoded reconstruction. */
int wc_round_trip_host(wc_ctx* ctx, const void* cells, int dtype, const wc_unit* units, int n, double keep,
                       uint8_t* payload, uint64_t payload_capacity, uint64_t* offsets, uint32_t* kept,
                       double* rmse);

/* Opt-in global-threshold mode (NOT the reference's rule; BASELINE north_star's
 * "keep-percentile histogram + RCCL all-reduce").  The reference thresholds each
 * box at its own max * (1 - keep) (src/compressor.cpp:212-216); this mode picks
 * ONE fp32 threshold for a whole run from the coefficient-magnitude histogram
 * summed over every unit on every rank.  Payload format and decoder unchanged.
 *
 *   wc_forward_stage: transform a batch into the context's coefficient scratch
 *     (the first half of wc_forward) and, when d_hist is not null, ADD the
 *     batch's magnitude histogram to d_hist (WC_HIST_BINS uint64 on the device;
 *     bin = fp32 bits of |c| >> WC_HIST_SHIFT, NaN not counted).  The bins are
 *     counted as the transform stages the coefficients (no second pass over them).
 *   (caller: all-reduce d_hist over ranks, e.g. RCCL sum of 4096 uint64)
 *   wc_hist_threshold: host-only; the fp32 threshold that keeps every
 *     coefficient whose bin is >= the highest bin b at which the count of
 *     coefficients in bins >= b reaches N - floor(quantile * N), N = the total
 *     count (retained >= (1 - quantile) N, by less than one bin's population).
 *     *retained receives that count (may be null).
 *   wc_forward_emit: threshold + pack the staged batch; thresh = NULL applies
 *     the reference per-unit rule with `keep` (so stage + emit == wc_forward),
 *     else every coefficient with |c| > *thresh is kept.  Needs the staged
 *     coefficients of the same units: any other compute call on the context in
 *     between invalidates them (WC_ERR_INVALID). */
#define WC_HIST_BINS 4096
#define WC_HIST_SHIFT 19
int wc_forward_stage(wc_ctx* ctx, const void* d_cells, int dtype, const wc_unit* units, int n,
                     uint64_t* d_hist);
int wc_hist_threshold(const uint64_t* hist, double quantile, float* thresh, uint64_t* retained);
int wc_forward_emit(wc_ctx* ctx, const wc_unit* units, int n, double keep, const float* thresh,
                    uint8_t* d_payload, uint64_t payload_capacity, uint64_t* d_offsets, uint32_t* d_kept);

/* Transform only: cells -> flat fp32 coefficients (x-slowest order), written
 * at the same element offsets as the cells (d_flat has the cell buffer's extent). */
int wc_decompose(wc_ctx* ctx, const void* d_cells, int dtype, const wc_unit* units, int n,
                 float* d_flat);

/* Inverse path for a batch: payloads -> fp32 Box3D cells at units[u].cell_offset.
 * Asynchronous on the context's stream.  Each payload header must match its unit
 * (W,H,D, ncoeff) and no run may be negative, else the next wc_synchronize (or the
 * _host variant itself) returns WC_ERR_FORMAT (the reference exits,
 * src/decompressor.cpp:228-231). */
int wc_inverse(wc_ctx* ctx, const uint8_t* d_payload, const uint64_t* d_offsets,
               const wc_unit* units, int n, float* d_out);

int wc_inverse_host(wc_ctx* ctx, const uint8_t* payload, const uint64_t* offsets,
                    const wc_unit* units, int n, float* out);

/* Inverse transform only: flat coefficients -> fp32 Box3D cells. */
int wc_inverse_flat(wc_ctx* ctx, const float* d_flat, const wc_unit* units, int n, float* d_out);
int wc_inverse_flat_host(wc_ctx* ctx, const float* flat, const wc_unit* units, int n, float* out);

/* Per-unit RMSE between original cells (fp64 narrowed, or fp32) and fp32
 * reconstructions; d_rmse: n doubles (device).  d_orig and d_regen at any
 * element alignment (vector loads where both bases allow them). */
int wc_rmse(wc_ctx* ctx, const void* d_orig, int dtype, const float* d_regen,
            const wc_unit* units, int n, double* d_rmse);
int wc_rmse_host(wc_ctx* ctx, const void* orig, int dtype, const float* regen,
                 const wc_unit* units, int n, double* rmse);

/* wc_inverse then wc_rmse of the reconstruction against d_orig, fused: the
 * row-indexed inverse adds each tile's squared differences right after
 * writing it (the reconstruction is not re-read from HBM).  Same d_out; RMSE
 * equal to wc_rmse's up to the order of the double sum (a batch with a unit
 * on the dense decode path runs the two calls).  Replaces the decompress ->
 * calc_rmse_per_box pair of the reference's -estimate / round-trip
 * (src/modes.cpp:209-327, src/calc-loss.cpp:12-43). */
int wc_inverse_rmse(wc_ctx* ctx, const uint8_t* d_payload, const uint64_t* d_offsets,
                    const wc_unit* units, int n, const void* d_orig, int dtype, float* d_out,
                    double* d_rmse);

/* Round trips in one process (the reference's -estimate: compress, then
 * decompress the same boxes and calc_rmse_per_box, src/modes.cpp:236-291).
 * The forward knows, as it packs the pairs, where every flat row of a unit
 * starts in the payload; wc_forward_rows writes that ROW INDEX beside the
 * payloads, and wc_inverse_rows reads it instead of re-deriving it from the
 * payloads (the row index kernel of wc_inverse, a third of its time).
 *
 *   Row index layout (caller-owned device buffer, wc_rowindex_bytes): unit u
 *   owns W*H + 1 entries of 8 bytes (none when it has no cells), after the
 *   entries of units 0..u-1.  Entry
 *   r < W*H of flat row r = I*H + J (the D coefficients r*D .. r*D + D - 1 of
 *   the reference's flat order, src/compressor.cpp:178-181) is {uint32 k,
 *   uint32 p_k - r*D}: k the first pair whose flat position p_k is >= r*D;
 *   entry W*H and the rows after the last pair hold {nrle, ncoeff - r*D}.
 *   Written for the units of the row-indexed shape (W and H even, D % 8 ==
 *   0, cells > 0); the entries of other units are not written (their inverse
 *   decodes from the payload).
 *
 *   wc_forward_rows: wc_forward (same payloads, offsets, kept counts) that
 *     also writes the row index (rowinfo_capacity >= wc_rowindex_bytes).
 *   wc_inverse_rows: wc_inverse (d_orig = d_rmse = NULL) or wc_inverse_rmse
 *     (both set) of payloads whose row index d_rowinfo came from
 *     wc_forward_rows of the same payloads and units (NULL: derived from the
 *     payloads, = wc_inverse / wc_inverse_rmse; rowinfo_capacity is then
 *     ignored, else it must be >= wc_rowindex_bytes).  Pair indices read from
 *     the row index are clamped to each payload's pair count, so a row index
 *     that belongs to other payloads gives wrong cells but never an access
 *     outside the payloads; headers are checked against the units
 *     (WC_ERR_FORMAT at the next wc_synchronize). */
uint64_t wc_rowindex_bytes(const wc_unit* units, int n);
int wc_forward_rows(wc_ctx* ctx, const void* d_cells, int dtype, const wc_unit* units, int n, double keep,
                    uint8_t* d_payload, uint64_t payload_capacity, uint64_t* d_offsets, uint32_t* d_kept,
                    void* d_rowinfo, uint64_t rowinfo_capacity);
int wc_inverse_rows(wc_ctx* ctx, const uint8_t* d_payload, const uint64_t* d_offsets, const wc_unit* units, int n,
                    const void* d_rowinfo, uint64_t rowinfo_capacity, const void* d_orig, int dtype, float* d_out,
                    double* d_rmse);

/* Transform only, host pointers (the reference's static wavelet_decompose). */
int wc_decompose_host(wc_ctx* ctx, const void* cells, int dtype, const wc_unit* units, int n,
                      float* flat);

/* Per-kernel timing with hipEvents recorded on the context stream around each
 * launch (used by bench.py for the live roofline figure).  Stage ids below;
 * wc_profile_read() returns the summed milliseconds and launch counts since
 * the previous read, then resets. */
#define WC_STAGE_TRANSFORM 0  /* K1  transform (+ dense re-staging fallback) */
#define WC_STAGE_EMIT 1       /* K2  threshold + ordered pack (k_emit) */
#define WC_STAGE_DECODE 2     /* K5  rle_decode */
#define WC_STAGE_INVERSE 3    /* K6  inverse transform */
#define WC_STAGE_RMSE 4       /* K7  */
#define WC_STAGE_HIST 5       /* histogram pass of generic units (wc_forward_stage with d_hist; the fast
                                 units' bins are counted inside the transform stage) */
#define WC_STAGE_PAIRS 6      /* header check + pair counts of wc_inverse_rows with a caller row index */
#define WC_NUM_STAGES 7
int wc_profile_enable(wc_ctx* ctx, int on);
int wc_profile_read(wc_ctx* ctx, double* total_ms, uint32_t* launches, int nstages);

/* Version string of the library build (arch, flags). */
const char* wc_version(void);

#ifdef __cplusplus
}
#endif
#endif /* WAVELET_AMD_H */

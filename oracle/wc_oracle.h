/*
 * wc_oracle.h — CPU restatement of the reference codec's per-box hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (wavelet-compression_amd/)
 * links, loads or calls this code.  It is used by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg, as the checker.
 *
 * Reference: carsonmw3/wavelet-compression @ 2025-07-04 (src/ paths below).
 * The reference itself is not buildable in this image (its codec sources
 * include doctest/doctest.h and spdlog/spdlog.h, which are absent; see
 * DESIGN.md "Oracle"), so this restatement is pinned by the reference's own
 * known-answer tests and data fixtures (tests/test_oracle.py).
 *
 * Layout conventions (same as the reference):
 *   box   : Grid3D<float>, W x H x D, cell (x,y,z) at x + W*(y + H*z)   src/grid.h:15-19
 *   flat  : coefficient (I,J,K) at (I*H + J)*D + K                      src/compressor.cpp:178-181
 */
#ifndef WC_ORACLE_H
#define WC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* fp64 plotfile cell -> fp32 Box3D cell (src/preprocess.cpp:78). */
void wco_narrow_f64(const double* in, float* out, int64_t n);

/* One-level 3-D Haar, Z then Y then X sweeps, flattened x-slowest.
 * src/compressor.cpp:85-185 (wavelet_decompose). */
void wco_wavelet_decompose(const float* box, int W, int H, int D, float* flat);

/* Index of the element std::max_element(..., |a|<|b| in double) returns.
 * src/compressor.cpp:212-215.  n == 0 returns -1. */
int64_t wco_max_index(const float* flat, int64_t n);

/* thresh = (double)flat[max_index] * (1 - keep).  src/compressor.cpp:212-216. */
double wco_threshold(const float* flat, int64_t n, double keep);

/* Mask |c| > thresh (fp64 compare) and RLE-encode as (zeros-before, value)
 * pairs.  src/compressor.cpp:222-238 + rle_encode :24-42.
 * runs/vals must hold n entries.  Returns the number of pairs. */
int64_t wco_threshold_rle(const float* flat, int64_t n, double thresh,
                          int32_t* runs, float* vals);

/* Plain rle_encode over an explicit mask/values (src/compressor.cpp:24-42). */
int64_t wco_rle_encode(const uint8_t* mask, const float* values, int64_t n,
                       int32_t* runs, float* vals);

/* Serialized size: 5 int32 + 8 bytes per pair (src/compressor.cpp:55-80). */
size_t wco_serialized_size(int64_t nrle);

/* Serialize (W,H,D), ncoeff, nrle, pairs; native little-endian.
 * src/compressor.cpp:47-80.  Returns bytes written. */
size_t wco_serialize(int W, int H, int D, int32_t ncoeff, int64_t nrle,
                     const int32_t* runs, const float* vals, uint8_t* out);

/* Whole compress() path for one Box3D component, minus xz:
 * transform -> threshold -> RLE -> serialize.  out must hold
 * wco_serialized_size(W*H*D) bytes.  Returns bytes written; *kept = pairs. */
size_t wco_compress_payload(const float* box, int W, int H, int D, double keep,
                            uint8_t* out, int64_t* kept);

/* Same, starting from fp64 cells (narrowed to fp32 first, preprocess.cpp:78). */
size_t wco_compress_payload_f64(const double* cells, int W, int H, int D,
                                double keep, uint8_t* out, int64_t* kept,
                                float* scratch_box);

/* Parse a serialized payload (src/decompressor.cpp:35-74).  Returns 0 on
 * success, -1 if the buffer is too short for the header or the pairs. */
int wco_parse_header(const uint8_t* data, size_t len, int32_t* W, int32_t* H,
                     int32_t* D, int32_t* ncoeff, int32_t* nrle);

/* rle_decode (src/decompressor.cpp:14-30): zero array of `total`, pairs
 * placed at idx += run; if (idx < total) out[idx++] = val. */
void wco_rle_decode(const int32_t* runs, const float* vals, int64_t nrle,
                    int64_t total, float* out);

/* Decode a serialized payload straight to flat coefficients (total = ncoeff). */
int wco_payload_to_flat(const uint8_t* data, size_t len, float* flat, int64_t cap);

/* inverse_wavelet_decompose (src/decompressor.cpp:79-159): X, Y, Z sweeps in
 * double, stored as float; odd tails become 0. */
void wco_inverse_wavelet_decompose(const float* flat, int W, int H, int D, float* box);

/* calc_rmse_per_box for one component (src/calc-loss.cpp:12-43). */
double wco_rmse(const float* actual, const float* pred, int W, int H, int D);

/* Synthetic AMR box generator:
 *   v = 300 + 50 sin(0.1 gx) cos(0.07 gy) + 0.01 gz + sigma N(0,1)
 * g = lo + local; N(0,1) from splitmix64 + Box-Muller, seed per unit. */
void wco_synth_box_f64(uint64_t seed, int lox, int loy, int loz, int W, int H,
                       int D, double sigma, double* out);

uint64_t wco_unit_seed(int t, int lev, int box, int comp);

#ifdef __cplusplus
}
#endif
#endif

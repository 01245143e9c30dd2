/*
 * wc_oracle.c — CPU restatement of the reference's per-box codec.
 *
 * TEST INFRASTRUCTURE ONLY (see wc_oracle.h).  Written from the reference's
 * documented behaviour, one function per reference routine, each citing the
 * file:line it restates.  Arithmetic deliberately follows the reference's own
 * operation order and widths (float adds, "/ 2.0" in double, fp64 compares),
 * so results are bit-identical, including the quirks listed in SURVEY.md §0.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math).
 */
#include "wc_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* src/preprocess.cpp:78 — `float value = mfdata(i,j,k,comp)` (fp64 -> fp32 RNE) */
void wco_narrow_f64(const double* in, float* out, int64_t n) {
    for (int64_t i = 0; i < n; ++i) out[i] = (float)in[i];
}

/* ------------------------------------------------------------------ */
/* One Haar analysis step on a strided line of n floats, in place.
 * Pairs (2m, 2m+1) -> low at m, high at n/2 + m; an odd last element stays.
 * Each output is `(a + b) / 2.0`: float add, double divide, float store
 * (src/compressor.cpp:107-111, :135-139, :160-164). */
static void analysis_line(float* p, int64_t stride, int n, float* scratch) {
    const int half = n / 2;
    for (int m = 0; m < half; ++m) {
        const float a = p[(int64_t)(2 * m) * stride];
        const float b = p[(int64_t)(2 * m + 1) * stride];
        const float s = a + b;
        const float d = a - b;
        scratch[m] = (float)((double)s / 2.0);
        scratch[half + m] = (float)((double)d / 2.0);
    }
    for (int m = 0; m < 2 * half; ++m) p[(int64_t)m * stride] = scratch[m];
}

/* src/compressor.cpp:85-185 — wavelet_decompose. */
void wco_wavelet_decompose(const float* box, int W, int H, int D, float* flat) {
    const int64_t sx = 1, sy = W, sz = (int64_t)W * H;
    const int64_t n = (int64_t)W * H * D;
    if (n == 0) return;
    float* t = (float*)malloc(sizeof(float) * (size_t)n);
    int longest = W > H ? W : H;
    if (D > longest) longest = D;
    float* scratch = (float*)malloc(sizeof(float) * (size_t)(longest + 1));
    memcpy(t, box, sizeof(float) * (size_t)n);

    /* Z sweep (:98-125): one line per (x, y). */
    for (int x = 0; x < W; ++x)
        for (int y = 0; y < H; ++y) analysis_line(t + x * sx + y * sy, sz, D, scratch);
    /* Y sweep (:128-150): one line per (x, z). */
    for (int x = 0; x < W; ++x)
        for (int z = 0; z < D; ++z) analysis_line(t + x * sx + z * sz, sy, H, scratch);
    /* X sweep (:153-175): one line per (y, z). */
    for (int y = 0; y < H; ++y)
        for (int z = 0; z < D; ++z) analysis_line(t + y * sy + z * sz, sx, W, scratch);

    /* Flatten x-slowest, z-fastest (:178-181). */
    int64_t f = 0;
    for (int x = 0; x < W; ++x)
        for (int y = 0; y < H; ++y)
            for (int z = 0; z < D; ++z) flat[f++] = t[x * sx + y * sy + z * sz];

    free(scratch);
    free(t);
}

/* ------------------------------------------------------------------ */
/* src/compressor.cpp:212-215 — std::max_element with comp |a| < |b| on doubles:
 * keep the current best unless a strictly larger magnitude follows.  So the
 * FIRST index of the largest magnitude wins, and a NaN only "wins" when it is
 * element 0 (every comparison against NaN is false). */
int64_t wco_max_index(const float* flat, int64_t n) {
    if (n <= 0) return -1;
    int64_t best = 0;
    for (int64_t i = 1; i < n; ++i) {
        if (fabs((double)flat[best]) < fabs((double)flat[i])) best = i;
    }
    return best;
}

/* src/compressor.cpp:216 — thresh = max_val * (1 - keep), max_val signed. */
double wco_threshold(const float* flat, int64_t n, double keep) {
    const int64_t i = wco_max_index(flat, n);
    if (i < 0) return 0.0;
    const double max_val = (double)flat[i];
    return max_val * (1 - keep);
}

/* src/compressor.cpp:24-42 — rle_encode: (falses since last true, value). */
int64_t wco_rle_encode(const uint8_t* mask, const float* values, int64_t n,
                       int32_t* runs, float* vals) {
    int64_t np = 0, vi = 0;
    int32_t gap = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (mask[i]) {
            runs[np] = gap;
            vals[np] = values[vi++];
            ++np;
            gap = 0;
        } else {
            ++gap;
        }
    }
    return np;
}

/* src/compressor.cpp:222-238 — mask `std::abs(val) > thresh` with val the
 * coefficient widened to double, kept values narrowed back (exact), then RLE. */
int64_t wco_threshold_rle(const float* flat, int64_t n, double thresh,
                          int32_t* runs, float* vals) {
    int64_t np = 0;
    int32_t gap = 0;
    for (int64_t i = 0; i < n; ++i) {
        const double v = (double)flat[i];
        if (fabs(v) > thresh) {
            runs[np] = gap;
            vals[np] = (float)v;
            ++np;
            gap = 0;
        } else {
            ++gap;
        }
    }
    return np;
}

/* ------------------------------------------------------------------ */
/* src/compressor.cpp:47-80 — 3 dims, coeff count, pair count, pairs. */
size_t wco_serialized_size(int64_t nrle) { return 5 * sizeof(int32_t) + (size_t)nrle * 8; }

static void put_i32(uint8_t* p, int32_t v) { memcpy(p, &v, 4); }
static void put_f32(uint8_t* p, float v) { memcpy(p, &v, 4); }

size_t wco_serialize(int W, int H, int D, int32_t ncoeff, int64_t nrle,
                     const int32_t* runs, const float* vals, uint8_t* out) {
    uint8_t* p = out;
    put_i32(p, W); p += 4;
    put_i32(p, H); p += 4;
    put_i32(p, D); p += 4;
    put_i32(p, ncoeff); p += 4;
    put_i32(p, (int32_t)nrle); p += 4;
    for (int64_t i = 0; i < nrle; ++i) {
        put_i32(p, runs[i]); p += 4;
        put_f32(p, vals[i]); p += 4;
    }
    return (size_t)(p - out);
}

/* src/compressor.cpp:192-297 minus the xz stage (:250-291). */
size_t wco_compress_payload(const float* box, int W, int H, int D, double keep,
                            uint8_t* out, int64_t* kept) {
    const int64_t n = (int64_t)W * H * D;
    float* flat = (float*)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    int32_t* runs = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    float* vals = (float*)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    wco_wavelet_decompose(box, W, H, D, flat);
    const double thresh = wco_threshold(flat, n, keep);
    const int64_t np = n > 0 ? wco_threshold_rle(flat, n, thresh, runs, vals) : 0;
    const size_t bytes = wco_serialize(W, H, D, (int32_t)n, np, runs, vals, out);
    if (kept) *kept = np;
    free(vals);
    free(runs);
    free(flat);
    return bytes;
}

size_t wco_compress_payload_f64(const double* cells, int W, int H, int D,
                                double keep, uint8_t* out, int64_t* kept,
                                float* scratch_box) {
    const int64_t n = (int64_t)W * H * D;
    wco_narrow_f64(cells, scratch_box, n);
    return wco_compress_payload(scratch_box, W, H, D, keep, out, kept);
}

/* ------------------------------------------------------------------ */
/* src/decompressor.cpp:35-74 — header is 5 native int32. */
int wco_parse_header(const uint8_t* data, size_t len, int32_t* W, int32_t* H,
                     int32_t* D, int32_t* ncoeff, int32_t* nrle) {
    if (len < 20) return -1;
    memcpy(W, data + 0, 4);
    memcpy(H, data + 4, 4);
    memcpy(D, data + 8, 4);
    memcpy(ncoeff, data + 12, 4);
    memcpy(nrle, data + 16, 4);
    if (*nrle < 0 || len < 20 + (size_t)(*nrle) * 8) return -1;
    return 0;
}

/* src/decompressor.cpp:14-30 — rle_decode. */
void wco_rle_decode(const int32_t* runs, const float* vals, int64_t nrle,
                    int64_t total, float* out) {
    for (int64_t i = 0; i < total; ++i) out[i] = 0.0f;
    int64_t idx = 0;
    for (int64_t i = 0; i < nrle; ++i) {
        idx += runs[i];
        if (idx < total) {
            out[idx] = vals[i];
            ++idx;
        }
    }
}

int wco_payload_to_flat(const uint8_t* data, size_t len, float* flat, int64_t cap) {
    int32_t W, H, D, nc, nr;
    if (wco_parse_header(data, len, &W, &H, &D, &nc, &nr) != 0) return -1;
    if (nc < 0 || nc > cap) return -1;
    for (int64_t i = 0; i < nc; ++i) flat[i] = 0.0f;
    int64_t idx = 0;
    const uint8_t* p = data + 20;
    for (int32_t i = 0; i < nr; ++i, p += 8) {
        int32_t run;
        float v;
        memcpy(&run, p, 4);
        memcpy(&v, p + 4, 4);
        idx += run;
        if (idx >= 0 && idx < nc) {
            flat[idx] = v;
            ++idx;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* One Haar synthesis step on a strided line: avg at m, diff at n/2 + m ->
 * (avg + diff, avg - diff) computed in double and stored as float; the
 * buffer is zero-initialised so an odd tail comes back as 0
 * (src/decompressor.cpp:94-112, :119-133, :140-154). */
static void synthesis_line(float* p, int64_t stride, int n, double* scratch) {
    const int half = n / 2;
    for (int m = 0; m < n; ++m) scratch[m] = 0.0;
    for (int m = 0; m < half; ++m) {
        const double avg = p[(int64_t)m * stride];
        const double diff = p[(int64_t)(half + m) * stride];
        scratch[2 * m] = avg + diff;
        scratch[2 * m + 1] = avg - diff;
    }
    for (int m = 0; m < n; ++m) p[(int64_t)m * stride] = (float)scratch[m];
}

/* src/decompressor.cpp:79-159 — inverse_wavelet_decompose. */
void wco_inverse_wavelet_decompose(const float* flat, int W, int H, int D, float* box) {
    const int64_t sx = 1, sy = W, sz = (int64_t)W * H;
    const int64_t n = (int64_t)W * H * D;
    if (n == 0) return;
    int longest = W > H ? W : H;
    if (D > longest) longest = D;
    double* scratch = (double*)malloc(sizeof(double) * (size_t)(longest + 1));

    /* Reshape flat (x-slowest) into the x-fastest box (:82-87). */
    int64_t f = 0;
    for (int x = 0; x < W; ++x)
        for (int y = 0; y < H; ++y)
            for (int z = 0; z < D; ++z) box[x * sx + y * sy + z * sz] = flat[f++];

    /* X (:89-114), then Y (:116-135), then Z (:137-156). */
    for (int y = 0; y < H; ++y)
        for (int z = 0; z < D; ++z) synthesis_line(box + y * sy + z * sz, sx, W, scratch);
    for (int x = 0; x < W; ++x)
        for (int z = 0; z < D; ++z) synthesis_line(box + x * sx + z * sz, sy, H, scratch);
    for (int x = 0; x < W; ++x)
        for (int y = 0; y < H; ++y) synthesis_line(box + x * sx + y * sy, sz, D, scratch);
    free(scratch);
}

/* ------------------------------------------------------------------ */
/* src/calc-loss.cpp:12-43 — float difference, widened, squared and summed in
 * double in z, y, x loop order; sqrt(sum / (W*H*D)). */
double wco_rmse(const float* actual, const float* pred, int W, int H, int D) {
    double sum = 0.0;
    for (int z = 0; z < D; ++z)
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                const int64_t i = x + (int64_t)W * (y + (int64_t)H * z);
                const float fd = actual[i] - pred[i];
                const double d = fd;
                sum += d * d;
            }
    return sqrt(sum / (W * H * D));
}

/* ------------------------------------------------------------------ */
/* Synthetic generator; portable: splitmix64 + Box-Muller. */
static uint64_t splitmix64(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t wco_unit_seed(int t, int lev, int box, int comp) {
    uint64_t s = 1234;
    uint64_t h = ((uint64_t)(uint32_t)t << 48) ^ ((uint64_t)(uint32_t)lev << 40) ^
                 ((uint64_t)(uint32_t)comp << 32) ^ (uint64_t)(uint32_t)box;
    s ^= h;
    return splitmix64(&s);
}

void wco_synth_box_f64(uint64_t seed, int lox, int loy, int loz, int W, int H,
                       int D, double sigma, double* out) {
    uint64_t s = seed;
    const double two_pi = 6.283185307179586476925286766559;
    const int64_t n = (int64_t)W * H * D;
    double spare = 0.0;
    int have_spare = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int x = (int)(i % W);
        const int y = (int)((i / W) % H);
        const int z = (int)(i / ((int64_t)W * H));
        double g;
        if (have_spare) {
            g = spare;
            have_spare = 0;
        } else {
            /* u1 in (0,1], u2 in [0,1) from the top 53 bits. */
            const double u1 = ((double)(splitmix64(&s) >> 11) + 1.0) * (1.0 / 9007199254740992.0);
            const double u2 = (double)(splitmix64(&s) >> 11) * (1.0 / 9007199254740992.0);
            const double r = sqrt(-2.0 * log(u1));
            g = r * cos(two_pi * u2);
            spare = r * sin(two_pi * u2);
            have_spare = 1;
        }
        const double gx = lox + x, gy = loy + y, gz = loz + z;
        out[i] = 300.0 + 50.0 * sin(0.1 * gx) * cos(0.07 * gy) + 0.01 * gz + sigma * g;
    }
}

// nan_probe.hip — NaN results of fp32 add / sub on the GPU against the x86 float and double
// paths of the reference (src/decompressor.cpp:89-156 computes avg +/- diff in double, stored as
// float), for NaN (quiet, signalling, both signs, payloads), +/-inf and 1.0 operand pairs.
// Prints one line per pair, DIFF where the GPU bits differ from the reference path.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdint>
__global__ void k(const float* a, const float* b, float* add, float* sub, int n) {
    int i = threadIdx.x;
    if (i < n) { add[i] = a[i] + b[i]; sub[i] = a[i] - b[i]; }
}
static float fb(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t bf(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
int main() {
    const uint32_t vals[] = {0x7fc00000u, 0xffc00000u, 0x7fc12345u, 0xffc54321u, 0x7f800000u, 0xff800000u, 0x3f800000u, 0x7fa00000u};
    const int nv = 8;
    float ha[64], hb[64];
    int n = 0;
    for (int i = 0; i < nv; ++i) for (int j = 0; j < nv; ++j) { ha[n] = fb(vals[i]); hb[n] = fb(vals[j]); ++n; }
    float *da, *db, *dadd, *dsub;
    hipMalloc(&da, 256); hipMalloc(&db, 256); hipMalloc(&dadd, 256); hipMalloc(&dsub, 256);
    hipMemcpy(da, ha, 256, hipMemcpyHostToDevice); hipMemcpy(db, hb, 256, hipMemcpyHostToDevice);
    k<<<1, 64>>>(da, db, dadd, dsub, n);
    float gadd[64], gsub[64];
    hipMemcpy(gadd, dadd, 256, hipMemcpyDeviceToHost); hipMemcpy(gsub, dsub, 256, hipMemcpyDeviceToHost);
    int diff = 0;
    for (int i = 0; i < n; ++i) {
        volatile float a = ha[i], b = hb[i];
        float cadd = a + b, csub = a - b;  // host x86 SSE
        volatile double da2 = (double)ha[i], db2 = (double)hb[i];
        float dadd2 = (float)(da2 + db2), dsub2 = (float)(da2 - db2);  // the reference's double path
        const bool same = bf(gadd[i]) == bf(dadd2) && bf(gsub[i]) == bf(dsub2);
        if (!same) ++diff;
        printf("%08x %08x | gpu add %08x sub %08x | x86 f32 add %08x sub %08x | x86 f64 add %08x sub %08x %s\n",
               bf(ha[i]), bf(hb[i]), bf(gadd[i]), bf(gsub[i]), bf(cadd), bf(csub), bf(dadd2), bf(dsub2), same ? "" : "DIFF");
    }
    printf("%d of %d differ from the reference's double path\n", diff, n);
    return 0;
}

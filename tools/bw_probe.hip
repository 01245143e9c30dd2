// bw_probe.hip — the HBM ceiling for a kernel's read:write mix.
//
// The kernel table in DESIGN.md prices every kernel against 8 TB/s.  What a
// streaming kernel can actually reach depends on how much of its traffic is
// writes (round 4's mall_probe: 4 GiB written alone ran at 5.2 TB/s).  This
// probe streams bytes in and out in ONE launch at a fixed read:write ratio
// P:Q, mixed evenly (every wave reads P and writes Q blocks of 1 KiB per
// group, four groups in flight), the way K1 / the emit / K6r mix them, and
// prints the rate.  Nothing it writes is checked; the reads feed the written
// values so they cannot be dropped.
//
// usage: bw_probe P Q [total_MB=4096] [ntload=0|1] [ntstore=0|1] [reps=10]
//        P:Q in {1:0, 0:1, 1:1, 2:1, 5:1, 1:2}; prints one JSON line
//        (best and median of reps, (read + written bytes) / time)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            std::exit(2);                                                          \
        }                                                                          \
    } while (0)

using f32x4 = float __attribute__((ext_vector_type(4)));
constexpr int kWaves = 4;              // waves per workgroup
constexpr int kGroups = 4;             // groups per wave iteration, loads in flight together
constexpr long long kBlock = 64 * 16;  // bytes of one wave access (16 B per lane)

template <int P, int Q, bool NTL, bool NTS>
__global__ __launch_bounds__(64 * kWaves) void k_mix(const f32x4* __restrict__ in, f32x4* __restrict__ out,
                                                     long long G) {
    const int lane = threadIdx.x & 63;
    const long long wave =
        (long long)blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const long long nwaves = (long long)gridDim.x * kWaves;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (long long g0 = wave * kGroups; g0 < G; g0 += nwaves * kGroups) {
        f32x4 v[kGroups][P > 0 ? P : 1];
#pragma unroll
        for (int j = 0; j < kGroups; ++j)
#pragma unroll
            for (int i = 0; i < P; ++i) {
                v[j][i] = acc;
                if (g0 + j < G) {
                    const f32x4* p = in + ((g0 + j) * P + i) * 64 + lane;
                    if constexpr (NTL)
                        v[j][i] = __builtin_nontemporal_load(p);
                    else
                        v[j][i] = *p;
                }
            }
#pragma unroll
        for (int j = 0; j < kGroups; ++j) {
            f32x4 s = acc;
#pragma unroll
            for (int i = 0; i < P; ++i) s += v[j][i];
            acc = s;
#pragma unroll
            for (int i = 0; i < Q; ++i)
                if (g0 + j < G) {
                    f32x4* p = out + ((g0 + j) * Q + i) * 64 + lane;
                    const f32x4 x = s + (float)i;
                    if constexpr (NTS)
                        __builtin_nontemporal_store(x, p);
                    else
                        *p = x;
                }
        }
    }
    if (acc.x == 1.2345e-30f) out[lane] = acc;  // keeps the reads live
}

template <int P, int Q>
void launch_pq(int grid, const f32x4* in, f32x4* out, long long G, int ntl, int nts) {
    if (ntl && nts)
        k_mix<P, Q, true, true><<<grid, 64 * kWaves>>>(in, out, G);
    else if (ntl)
        k_mix<P, Q, true, false><<<grid, 64 * kWaves>>>(in, out, G);
    else if (nts)
        k_mix<P, Q, false, true><<<grid, 64 * kWaves>>>(in, out, G);
    else
        k_mix<P, Q, false, false><<<grid, 64 * kWaves>>>(in, out, G);
}

int main(int argc, char** argv) {
    const int P = argc > 1 ? atoi(argv[1]) : 1, Q = argc > 2 ? atoi(argv[2]) : 1;
    const long long tmb = argc > 3 ? atoll(argv[3]) : 4096;
    const int ntl = argc > 4 ? atoi(argv[4]) : 0, nts = argc > 5 ? atoi(argv[5]) : 0;
    const int reps = argc > 6 ? atoi(argv[6]) : 10;
    const long long G = tmb * (1LL << 20) / kBlock / (P + Q);
    const long long rbytes = G * P * kBlock, wbytes = G * Q * kBlock;
    void (*fn)(int, const f32x4*, f32x4*, long long, int, int) = nullptr;
    if (P == 1 && Q == 0) fn = launch_pq<1, 0>;
    if (P == 0 && Q == 1) fn = launch_pq<0, 1>;
    if (P == 1 && Q == 1) fn = launch_pq<1, 1>;
    if (P == 2 && Q == 1) fn = launch_pq<2, 1>;
    if (P == 5 && Q == 1) fn = launch_pq<5, 1>;
    if (P == 1 && Q == 2) fn = launch_pq<1, 2>;
    if (!fn || G <= 0 || reps <= 0) {
        std::fprintf(stderr, "usage: bw_probe P Q [total_MB] [ntload] [ntstore] [reps]; P:Q in 1:0 0:1 1:1 2:1 5:1 1:2\n");
        return 2;
    }
    f32x4 *in = nullptr, *out = nullptr;
    CK(hipMalloc(&in, std::max(rbytes, kBlock)));
    CK(hipMalloc(&out, std::max(wbytes, kBlock)));
    CK(hipMemset(in, 0, std::max(rbytes, kBlock)));
    CK(hipMemset(out, 0, std::max(wbytes, kBlock)));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int grid = prop.multiProcessorCount * 8;  // 8 workgroups of 4 waves per CU
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    fn(grid, in, out, G, ntl, nts);
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a));
        fn(grid, in, out, G, ntl, nts);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float m = 0;
        CK(hipEventElapsedTime(&m, a, b));
        ms.push_back(m);
    }
    CK(hipGetLastError());
    std::sort(ms.begin(), ms.end());
    const double bytes = (double)(rbytes + wbytes);
    std::printf("{\"p\": %d, \"q\": %d, \"read_gb\": %.3f, \"write_gb\": %.3f, \"write_share\": %.3f, \"ntload\": %d, "
                "\"ntstore\": %d, \"ms_best\": %.4f, \"ms_median\": %.4f, \"tb_s_best\": %.3f, \"tb_s_median\": %.3f}\n",
                P, Q, rbytes * 1e-9, wbytes * 1e-9, (double)Q / (P + Q), ntl, nts, ms.front(), ms[ms.size() / 2],
                bytes / ms.front() * 1e-9, bytes / ms[ms.size() / 2] * 1e-9);
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
}

// wc_compact.hip — host-path packing of the forward payload: the slots of
// wc_forward (fixed worst-case offsets) are packed densely before the copy
// back (wc_forward_host).  The forward compaction itself is k_emit
// (wc_emit.hip).
#include "wc_device.h"

namespace wc {

// Host-path compaction: packed offsets (== 4 mod 8) from kept counts ...
__global__ __launch_bounds__(1024) void k_pack_offsets(int n, const uint32_t* __restrict__ kept,
                                                     uint64_t* __restrict__ packed) {
    __shared__ uint64_t s_w[16];
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t carry = 4;
    for (int c0 = 0; c0 < n; c0 += 1024) {
        const int u = c0 + threadIdx.x;
        const bool ok = u < n;
        const uint64_t k = ok ? kept[u] : 0;
        const uint64_t sz = ok ? 24 + 8 * k : 0;
        uint64_t incl = sz;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            uint64_t t = __shfl_up(incl, o);
            if (l >= o) incl += t;
        }
        if (l == 63) s_w[w] = incl;
        __syncthreads();
        uint64_t wb = 0, tot = 0;
        for (int i = 0; i < 16; ++i) {
            if (i < w) wb += s_w[i];
            tot += s_w[i];
        }
        __syncthreads();
        if (ok) {
            const uint64_t off = carry + wb + incl - sz;
            packed[u] = off;
            if (u == n - 1) packed[n] = off + 20 + 8 * k;
        }
        carry += tot;
    }
}

// ... and the copy of each unit's bytes from its slot to its packed offset.
__global__ __launch_bounds__(256) void k_pack_copy(const UnitDev* __restrict__ units,
                                                 const uint32_t* __restrict__ kept,
                                                 const uint8_t* __restrict__ src, const uint64_t* __restrict__ packed,
                                                 uint8_t* __restrict__ dst) {
    const int u = blockIdx.x;
    const UnitDev& U = units[u];
    const uint64_t words = (20 + 8ull * kept[u]) / 4;
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src + U.pay_off);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst + packed[u]);
    for (uint64_t i = threadIdx.x; i < words; i += blockDim.x) d[i] = s[i];
}

// ---------------------------------------------------------------------------
hipError_t launch_pack(hipStream_t st, const UnitDev* units, int n, const uint32_t* kept, const uint8_t* src,
                       uint64_t* packed, uint8_t* dst) {
    k_pack_offsets<<<1, 1024, 0, st>>>(n, kept, packed);
    k_pack_copy<<<n, 256, 0, st>>>(units, kept, src, packed, dst);
    return hipGetLastError();
}

}  // namespace wc

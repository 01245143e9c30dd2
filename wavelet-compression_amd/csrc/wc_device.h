// wc_device.h — device helpers shared by the codec kernels (wave64 reductions,
// block scans, x-pair loads, the Haar butterfly halves).
#pragma once

#include "wc_internal.h"

namespace wc {

__device__ __forceinline__ float haar_lo(float a, float b) { return (a + b) * 0.5f; }
__device__ __forceinline__ float haar_hi(float a, float b) { return (a - b) * 0.5f; }

// The reference keeps |c| iff (double)|c| > thresh (src/compressor.cpp:225-226).
// With tf = thresh rounded toward -inf to float, that is exactly |c| > tf for
// every float |c|: no float lies strictly between tf and thresh; NaN and
// +-inf thresholds map to themselves.
__device__ __forceinline__ float thresh_as_float(double thresh) { return __double2float_rd(thresh); }

__device__ __forceinline__ int lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0));
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}

// Load the x-pair (x, x+1) of a row as fp32 (fp64 cells narrowed RNE,
// src/preprocess.cpp:78).  `vec`: both elements in one aligned vector load.
template <typename T>
__device__ __forceinline__ void load_xpair(const T* __restrict__ p, bool two, bool vec,
                                           float& a, float& b) {
    if (two) {
        if (vec) {
            if constexpr (sizeof(T) == 8) {
                const double2 d = *reinterpret_cast<const double2*>(p);
                a = (float)d.x;
                b = (float)d.y;
            } else {
                const float2 d = *reinterpret_cast<const float2*>(p);
                a = d.x;
                b = d.y;
            }
        } else {
            a = (float)p[0];
            b = (float)p[1];
        }
    } else {
        a = (float)p[0];
        b = 0.0f;
    }
}

// Flat position of output index s (0 = low, 1 = high) of block b on an axis
// with h pairs and n cells: low -> b, high -> h + b, tail block (b == h) -> n - 1.
__device__ __forceinline__ int out_index(int b, int s, int h, int n) {
    return b < h ? b + s * h : n - 1;
}


// Block-wide (256 threads) exclusive sum + exclusive max, with carry-in.
struct ScanOut {
    uint64_t excl_sum, total_sum;
    uint32_t excl_max, total_max;
};

template <typename S>
__device__ __forceinline__ ScanOut block_scan_sum_max(S v, uint32_t m, S* s_sum, uint32_t* s_max) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    S incl = v;
    uint32_t im = m;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        S t = __shfl_up(incl, o);
        uint32_t tm = __shfl_up(im, o);
        if (l >= o) {
            incl += t;
            im = tm > im ? tm : im;
        }
    }
    if (l == 63) {
        s_sum[w] = incl;
        s_max[w] = im;
    }
    __syncthreads();
    S wbase = 0, tot = 0;
    uint32_t wmax = 0, totm = 0;
    for (int i = 0; i < 4; ++i) {
        if (i < w) {
            wbase += s_sum[i];
            wmax = s_max[i] > wmax ? s_max[i] : wmax;
        }
        tot += s_sum[i];
        totm = s_max[i] > totm ? s_max[i] : totm;
    }
    __syncthreads();
    ScanOut r;
    r.excl_sum = (uint64_t)(wbase + incl - v);
    // exclusive max: max over lanes < l in this wave and all earlier waves
    uint32_t em = __shfl_up(im, 1);
    if (l == 0) em = 0;
    r.excl_max = em > wmax ? em : wmax;
    r.total_sum = (uint64_t)tot;
    r.total_max = totm;
    return r;
}


}  // namespace wc

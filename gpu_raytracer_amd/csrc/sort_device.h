// sort_device.h -- device helpers of the stable 10-bit bucket ranking shared
// by the sort kernels (sort_kernels.hip) and the tile-bucketing Morton kernel
// (build_kernels.hip, k_morton_tb).  SURVEY.md §8(a) a4/a5, §9.4.
#pragma once

#include "rt_device.h"

namespace rt {

__device__ __forceinline__ uint32_t sort_count_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Stable rank of each item among the equal 10-bit digits of its wave, in
// (item, lane) order, on top of the wave's running digit counters s_wc[w]:
// a wave64 match-any by 10 ballots (no LDS atomics, so the order among equal
// digits is the index order by construction).
template <int P>
__device__ __forceinline__ void rank10(const uint32_t (&dg)[P], const bool (&ok)[P],
                                       uint32_t (*s_wc)[kMsbBuckets], uint32_t (&r)[P]) {
    const uint32_t w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < P; ++i) {
        const uint32_t d = dg[i];
        uint64_t peers = __ballot(ok[i]);
        if (!peers) continue;  // wave-uniform: no item of this group (a bucket's tail)
#pragma unroll
        for (int b = 0; b < 10; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bal = __ballot(ok[i] && bit);
            peers &= bit ? bal : ~bal;
        }
        const uint32_t below = sort_count_below(peers);
        const uint32_t cur = s_wc[w][d];
        r[i] = cur + below;
        if (ok[i] && below == 0) s_wc[w][d] = cur + (uint32_t)__popcll(peers);
    }
}

// s_wc[w][d] -> exclusive prefix over the waves, with 16-B LDS accesses (4
// digits per thread and wave row); s_cnt[d] = the digit's total.  s_wc rows
// and s_cnt 16-B aligned.
template <int NW, int NT>
__device__ __forceinline__ void wave_prefix4(uint32_t (*s_wc)[kMsbBuckets], uint32_t* s_cnt) {
    for (uint32_t q = threadIdx.x; q < kMsbBuckets / 4; q += NT) {
        uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            uint4* row = reinterpret_cast<uint4*>(s_wc[w]);
            const uint4 c = row[q];
            row[q] = acc;
            acc.x += c.x; acc.y += c.y; acc.z += c.z; acc.w += c.w;
        }
        reinterpret_cast<uint4*>(s_cnt)[q] = acc;
    }
}

// In-place exclusive scan of a[1024] in LDS by NT threads (a written before a
// barrier); thread t owns a[t * PER .. t * PER + PER).  Ends with a barrier.
template <int NT>
__device__ __forceinline__ void scan1024(uint32_t* a, uint32_t* s_sw /* [NT / 64] */) {
    constexpr int PER = (int)kMsbBuckets / NT;
    const uint32_t t = threadIdx.x, l = t & 63, w = t >> 6;
    uint32_t v[PER], sum = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        v[j] = a[t * PER + j];
        sum += v[j];
    }
    uint32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (l >= (uint32_t)o) x += y;
    }
    if (l == 63) s_sw[w] = x;
    __syncthreads();
    uint32_t pre = x - sum;
    for (uint32_t k = 0; k < w; ++k) pre += s_sw[k];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        a[t * PER + j] = pre;
        pre += v[j];
    }
    __syncthreads();
}

}  // namespace rt

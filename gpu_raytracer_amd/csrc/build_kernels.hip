// build_kernels.hip -- BVH build hot path for gfx950.
//
//   K0 k_bounds      centroid bounds (grid-stride, LDS-staged float4 loads of
//                    the AoS soup) + last-block reduction -> BuildParams;
//                    also zeroes the per-build control words (sort status,
//                    tile tickets, digit histograms, crossing-list counter).
//   K1 k_morton      Morton codes (§9.3) + the 4 global 8-bit digit histograms
//                    (LDS histograms, one global atomic per non-empty bin).
//   K2/K3 k_onesweep stable LSB radix sort, one launch per 8-bit digit:
//                    wave64 ballot match-any ranking into LDS buckets, decoupled
//                    look-back over per-tile digit counts (single 32-bit
//                    {flag,count} words, relaxed agent-scope atomics: the data is
//                    the flag), LDS-staged coalesced scatter.
//   K4 k_karras      Karras 2012 topology (§9.5) + closed-form escape links
//                    (§9.6) + parent pointers.
//   K5/K6 k_refit_local  block-local bottom-up refit in LDS (leaf AABBs gathered
//                    from the soup; LDS arrival counters; no inter-workgroup
//                    traffic) + per-block prefix/suffix/total AABBs.
//   K6 k_refit_cross nodes whose leaf range crosses a refit-block boundary:
//                    union(suffix, middle blocks, prefix) -- exact, order-free.
//
// No kernel waits on another workgroup except the onesweep look-back (dynamic
// tile ids make it deadlock-free) and K0's last-block hand-off (Guideline 16
// recipe: release fence + ticket, acquire in the last block).
#include "rt_device.h"
#include "rt_launch.h"

#include <algorithm>

namespace rt {

// ---------------------------------------------------------------- helpers
__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

__device__ __forceinline__ uint32_t count_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Stage `cnt` (<=256) AoS triangles starting at tri `base` into LDS.
__device__ __forceinline__ void stage_tris(const float* __restrict__ tris, uint32_t base, uint32_t cnt, float4* stage) {
    const float* src = tris + (uint64_t)base * 9;
    if (cnt == 256) {  // 9216 B, 16-B aligned (base % 256 == 0)
        const float4* s4 = reinterpret_cast<const float4*>(src);
        for (int j = threadIdx.x; j < 576; j += 256) stage[j] = s4[j];
    } else {
        float* sf = reinterpret_cast<float*>(stage);
        for (uint32_t j = threadIdx.x; j < cnt * 9; j += 256) sf[j] = src[j];
    }
}

// ---------------------------------------------------------------- K0
__global__ __launch_bounds__(256) void k_bounds(const float* __restrict__ tris, uint32_t n,
                                                float* __restrict__ partials, uint32_t* ticket,
                                                BuildParams* __restrict__ params,
                                                uint32_t* __restrict__ zero_words, uint32_t nzero) {
    __shared__ float4 stage[576];
    __shared__ float red[4][6];
    __shared__ uint32_t s_last;
    // zero the per-build control words (visible to K1.. after this launch)
    for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < nzero; j += gridDim.x * 256) zero_words[j] = 0u;

    float lo[3], hi[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) { lo[c] = __builtin_inff(); hi[c] = -__builtin_inff(); }
    for (uint32_t base = blockIdx.x * 256u; base < n; base += gridDim.x * 256u) {
        const uint32_t rem = n - base;
        const uint32_t cnt = rem < 256u ? rem : 256u;
        stage_tris(tris, base, cnt, stage);
        __syncthreads();
        if (threadIdx.x < cnt) {
            const float* t = reinterpret_cast<const float*>(stage) + threadIdx.x * 9;
            float bmin[3], bmax[3];
            tri_bounds(t, bmin, bmax);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float cc = (bmin[c] + bmax[c]) * 0.5f;
                lo[c] = fminf(lo[c], cc);
                hi[c] = fmaxf(hi[c], cc);
            }
        }
        __syncthreads();
    }
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
    for (int c = 0; c < 3; ++c) { lo[c] = wave_min(lo[c]); hi[c] = wave_max(hi[c]); }
    if (l == 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) { red[w][c] = lo[c]; red[w][3 + c] = hi[c]; }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float r[6];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            r[c] = fminf(fminf(red[0][c], red[1][c]), fminf(red[2][c], red[3][c]));
            r[3 + c] = fmaxf(fmaxf(red[0][3 + c], red[1][3 + c]), fmaxf(red[2][3 + c], red[3][3 + c]));
        }
#pragma unroll
        for (int c = 0; c < 6; ++c) partials[blockIdx.x * 6 + c] = r[c];
        // Guideline 16 producer: release (write back L2), explicit wait, ticket.
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (t == gridDim.x - 1) ? 1u : 0u;
    }
    __syncthreads();
    if (!s_last) return;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 3; ++c) { lo[c] = __builtin_inff(); hi[c] = -__builtin_inff(); }
    for (uint32_t b = threadIdx.x; b < gridDim.x; b += 256) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            lo[c] = fminf(lo[c], partials[b * 6 + c]);
            hi[c] = fmaxf(hi[c], partials[b * 6 + 3 + c]);
        }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) { lo[c] = wave_min(lo[c]); hi[c] = wave_max(hi[c]); }
    __syncthreads();
    if (l == 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) { red[w][c] = lo[c]; red[w][3 + c] = hi[c]; }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        BuildParams p;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            p.lo[c] = fminf(fminf(red[0][c], red[1][c]), fminf(red[2][c], red[3][c]));
            p.hi[c] = fmaxf(fmaxf(red[0][3 + c], red[1][3 + c]), fmaxf(red[2][3 + c], red[3][3 + c]));
            // §9.2: inv = (hi>lo) ? 1/(hi-lo) : 0 -- correctly rounded fp32 division
            p.inv[c] = (p.hi[c] > p.lo[c]) ? 1.0f / (p.hi[c] - p.lo[c]) : 0.0f;
        }
#pragma unroll
        for (int c = 0; c < 7; ++c) p.pad[c] = 0u;
        *params = p;
        *ticket = 0u;  // re-arm for the next build (also memset at allocation)
    }
}

// ---------------------------------------------------------------- K1
__device__ __forceinline__ uint32_t quant(float c, float lo, float inv) {
    const float x = ((c - lo) * inv) * 1024.0f;
    return (uint32_t)fminf(fmaxf(x, 0.0f), 1023.0f);
}

__global__ __launch_bounds__(256) void k_morton(const float* __restrict__ tris, uint32_t n,
                                                const BuildParams* __restrict__ params,
                                                uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                uint32_t* __restrict__ ghist /* [4][256] */) {
    __shared__ float4 stage[576];
    __shared__ uint32_t hist[4 * 256];
    for (int j = threadIdx.x; j < 1024; j += 256) hist[j] = 0u;
    const BuildParams p = *params;
    for (uint32_t base = blockIdx.x * 256u; base < n; base += gridDim.x * 256u) {
        const uint32_t rem = n - base;
        const uint32_t cnt = rem < 256u ? rem : 256u;
        stage_tris(tris, base, cnt, stage);
        __syncthreads();
        if (threadIdx.x < cnt) {
            const float* t = reinterpret_cast<const float*>(stage) + threadIdx.x * 9;
            float bmin[3], bmax[3];
            tri_bounds(t, bmin, bmax);
            uint32_t q[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) q[c] = quant((bmin[c] + bmax[c]) * 0.5f, p.lo[c], p.inv[c]);
            const uint32_t key = expand10(q[0]) * 4u + expand10(q[1]) * 2u + expand10(q[2]);
            const uint32_t i = base + threadIdx.x;
            keys[i] = key;
            vals[i] = i;
#pragma unroll
            for (int d = 0; d < 4; ++d) atomicAdd(&hist[d * 256 + ((key >> (8 * d)) & 0xFFu)], 1u);
        }
        __syncthreads();
    }
    for (int j = threadIdx.x; j < 1024; j += 256) {
        const uint32_t v = hist[j];
        if (v) atomicAdd(&ghist[j], v);
    }
}

// ---------------------------------------------------------------- K2/K3 onesweep
// 256-thread exclusive scan (4 waves); returns exclusive prefix, *total = sum.
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* sw /* [4] */, uint32_t* total) {
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (l >= (uint32_t)o) x += y;
    }
    if (l == 63) sw[w] = x;
    __syncthreads();
    uint32_t pre = 0;
    for (uint32_t k = 0; k < w; ++k) pre += sw[k];
    *total = sw[0] + sw[1] + sw[2] + sw[3];
    __syncthreads();
    return pre + x - v;
}

template <int SHIFT>
__global__ __launch_bounds__(kSortThreads) void k_onesweep(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                           uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                           uint32_t n, const uint32_t* __restrict__ ghist /* this digit's 256 bins */,
                                                           uint32_t* status /* [256][ntiles] */, uint32_t ntiles,
                                                           uint32_t* tile_ctr, uint32_t* err) {
    constexpr int W = kSortThreads / 64;
    __shared__ uint32_t s_wc[W][256];
    __shared__ uint32_t s_key[kSortTile];
    __shared__ uint32_t s_val[kSortTile];
    __shared__ uint32_t s_lstart[256];
    __shared__ uint32_t s_gofs[256];
    __shared__ uint32_t s_sw[4];
    __shared__ uint32_t s_tile;

    const uint32_t tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(tile_ctr, 1u);
    for (uint32_t j = tid; j < W * 256; j += kSortThreads) (&s_wc[0][0])[j] = 0u;
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint32_t base = tile * (uint32_t)kSortTile;

    uint32_t k[kSortItems], v[kSortItems], r[kSortItems];
#pragma unroll
    for (int i = 0; i < kSortItems; ++i) {
        const uint32_t idx = base + w * (64u * kSortItems) + i * 64u + l;
        const bool ok = idx < n;
        k[i] = ok ? kin[idx] : 0u;
        v[i] = ok ? vin[idx] : 0u;
    }
    // ---- stable per-wave ranking: order (i, lane) == original index order
#pragma unroll
    for (int i = 0; i < kSortItems; ++i) {
        const uint32_t idx = base + w * (64u * kSortItems) + i * 64u + l;
        const bool ok = idx < n;
        const uint32_t d = (k[i] >> SHIFT) & 0xFFu;
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bal = __ballot(ok && bit);
            peers &= bit ? bal : ~bal;
        }
        const uint32_t below = count_below(peers);
        const uint32_t cur = s_wc[w][d];
        r[i] = cur + below;
        if (ok && below == 0) s_wc[w][d] = cur + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // ---- per-digit tile count, per-wave exclusive prefix (in place)
    const uint32_t d = tid;  // kSortThreads == 256: one digit per thread
    uint32_t cnt = 0;
#pragma unroll
    for (int ww = 0; ww < W; ++ww) {
        const uint32_t c = s_wc[ww][d];
        s_wc[ww][d] = cnt;
        cnt += c;
    }
    // publish this tile's aggregate as early as possible
    uint32_t* st = status + (uint64_t)d * ntiles;
    __hip_atomic_store(st + tile, (tile == 0 ? kFlagInc : kFlagAgg) | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t tot;
    const uint32_t lstart = block_excl_scan256(cnt, s_sw, &tot);
    s_lstart[d] = lstart;
    const uint32_t dbase = block_excl_scan256(ghist[d], s_sw, &tot);
    // ---- decoupled look-back for digit d
    uint32_t excl = 0;
    if (tile > 0) {
        int64_t kk = (int64_t)tile - 1;
        uint32_t spins = 0;
        while (kk >= 0) {
            const uint32_t s = __hip_atomic_load(st + kk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t flag = s & ~kCountMask;
            if (flag == 0u) {
                if (++spins > (1u << 22)) { atomicOr(err, 1u); break; }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            excl += s & kCountMask;
            if (flag == kFlagInc) break;
            --kk;
        }
        __hip_atomic_store(st + tile, kFlagInc | (excl + cnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_gofs[d] = dbase + excl;
    __syncthreads();
    // ---- local scatter into LDS buckets
#pragma unroll
    for (int i = 0; i < kSortItems; ++i) {
        const uint32_t idx = base + w * (64u * kSortItems) + i * 64u + l;
        if (idx < n) {
            const uint32_t dd = (k[i] >> SHIFT) & 0xFFu;
            const uint32_t pos = s_lstart[dd] + s_wc[w][dd] + r[i];
            s_key[pos] = k[i];
            s_val[pos] = v[i];
        }
    }
    __syncthreads();
    const uint32_t trem = n - base;
    const uint32_t tcount = trem < (uint32_t)kSortTile ? trem : (uint32_t)kSortTile;
#pragma unroll
    for (int m = 0; m < kSortItems; ++m) {
        const uint32_t pidx = tid + m * kSortThreads;
        if (pidx < tcount) {
            const uint32_t key = s_key[pidx];
            const uint32_t dd = (key >> SHIFT) & 0xFFu;
            const uint32_t o = s_gofs[dd] + (pidx - s_lstart[dd]);
            kout[o] = key;
            vout[o] = s_val[pidx];
        }
    }
}

// ---------------------------------------------------------------- K4 Karras
__device__ __forceinline__ int kdelta(const uint32_t* __restrict__ keys, int64_t n, int64_t i, uint32_t ki, int64_t j) {
    if (j < 0 || j >= n) return -1;
    const uint32_t kj = keys[j];
    if (ki == kj) return 32 + __clz((int)((uint32_t)i ^ (uint32_t)j));
    return __clz((int)(ki ^ kj));
}

__device__ __forceinline__ int kdir(const uint32_t* __restrict__ keys, int64_t n, int64_t i) {
    const uint32_t ki = keys[i];
    return (kdelta(keys, n, i, ki, i + 1) - kdelta(keys, n, i, ki, i - 1)) > 0 ? 1 : -1;
}

__global__ __launch_bounds__(256) void k_karras(const uint32_t* __restrict__ keys, uint32_t n,
                                                uint4* __restrict__ topo, uint32_t* __restrict__ parent,
                                                uint32_t* __restrict__ lesc) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t N = n;
    if (i >= N - 1) return;
    const uint32_t L0 = n - 1;
    const uint32_t ki = keys[i];
    const int d = (kdelta(keys, N, i, ki, i + 1) - kdelta(keys, N, i, ki, i - 1)) > 0 ? 1 : -1;
    const int dmin = kdelta(keys, N, i, ki, i - d);
    int64_t lmax = 2;
    while (kdelta(keys, N, i, ki, i + lmax * d) > dmin) lmax <<= 1;
    int64_t l = 0;
    for (int64_t t = lmax >> 1; t >= 1; t >>= 1)
        if (kdelta(keys, N, i, ki, i + (l + t) * d) > dmin) l += t;
    const int64_t j = i + l * d;
    const int dnode = kdelta(keys, N, i, ki, j);
    int64_t s = 0, t = l;
    do {
        t = (t + 1) >> 1;
        if (kdelta(keys, N, i, ki, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int64_t g = i + s * d + (d < 0 ? d : 0);
    const int64_t mn = d > 0 ? i : j, mx = d > 0 ? j : i;
    const uint32_t left = (mn == g) ? (uint32_t)(L0 + g) : (uint32_t)g;
    const uint32_t right = (mx == g + 1) ? (uint32_t)(L0 + g + 1) : (uint32_t)(g + 1);
    // §9.6 closed form: esc(node with range end r) = r == n-1 ? SENT
    //   : (r+1 <= n-2 && dir(r+1) == +1) ? internal r+1 : leaf r+1
    uint32_t esc;
    if (mx == N - 1) esc = RT_SENT;
    else if (mx + 1 <= N - 2 && kdir(keys, N, mx + 1) > 0) esc = (uint32_t)(mx + 1);
    else esc = (uint32_t)(L0 + mx + 1);
    topo[i] = make_uint4(left, esc, (uint32_t)mn, (uint32_t)mx);
    parent[left] = (uint32_t)i;
    parent[right] = (uint32_t)i;
    if (i == 0) parent[0] = RT_SENT;
    // leaf i-1 escapes to the right child of split i-1 == internal i iff dir(i) == +1
    if (i >= 1) lesc[i - 1] = d > 0 ? (uint32_t)i : (uint32_t)(L0 + i);
    if (i == N - 2) { lesc[N - 2] = L0 + (uint32_t)(N - 1); lesc[N - 1] = RT_SENT; }
}

// ---------------------------------------------------------------- K5/K6 refit
__device__ __forceinline__ void shfl_up_aabb(Aabb& a, int o) {
    Aabb b;
#pragma unroll
    for (int c = 0; c < 3; ++c) { b.lo[c] = __shfl_up(a.lo[c], o, 64); b.hi[c] = __shfl_up(a.hi[c], o, 64); }
    if ((int)(threadIdx.x & 63) >= o) aabb_union(a, b);
}
__device__ __forceinline__ void shfl_down_aabb(Aabb& a, int o) {
    Aabb b;
#pragma unroll
    for (int c = 0; c < 3; ++c) { b.lo[c] = __shfl_down(a.lo[c], o, 64); b.hi[c] = __shfl_down(a.hi[c], o, 64); }
    if ((int)(threadIdx.x & 63) + o < 64) aabb_union(a, b);
}

__device__ __forceinline__ void store_node(void* nodes, uint32_t idx, const Aabb& b, uint32_t a, uint32_t esc) {
    float4* p = reinterpret_cast<float4*>(reinterpret_cast<char*>(nodes) + (uint64_t)idx * 32);
    p[0] = make_float4(b.lo[0], b.lo[1], b.lo[2], b.hi[0]);
    p[1] = make_float4(b.hi[1], b.hi[2], __uint_as_float(a), __uint_as_float(esc));
}

__device__ __forceinline__ void store_aabb(float* buf, uint64_t idx, const Aabb& b) {
    float* p = buf + idx * 6;
#pragma unroll
    for (int c = 0; c < 3; ++c) { p[c] = b.lo[c]; p[3 + c] = b.hi[c]; }
}
__device__ __forceinline__ Aabb load_aabb(const float* buf, uint64_t idx) {
    const float* p = buf + idx * 6;
    Aabb b;
#pragma unroll
    for (int c = 0; c < 3; ++c) { b.lo[c] = p[c]; b.hi[c] = p[3 + c]; }
    return b;
}

// One block = kRefitT consecutive sorted leaves [B0, B1), one thread per leaf.
__global__ __launch_bounds__(kRefitT) void k_refit_local(const float* __restrict__ tris, uint32_t n,
                                                         const uint32_t* __restrict__ svals,
                                                         const uint4* __restrict__ topo,
                                                         const uint32_t* __restrict__ parent,
                                                         const uint32_t* __restrict__ lesc,
                                                         void* __restrict__ nodes,
                                                         float* __restrict__ prebuf, float* __restrict__ sufbuf,
                                                         float* __restrict__ totals,
                                                         uint32_t* __restrict__ cross, uint32_t* cross_ctr) {
    constexpr int T = kRefitT, NW = T / 64;
    __shared__ Aabb s_box[2 * T];      // [0,T) leaves, [T,2T) internal nodes of the block
    __shared__ uint4 s_topo[T];
    __shared__ uint32_t s_par[2 * T];
    __shared__ uint32_t s_cnt[T];
    __shared__ Aabb s_wpre[NW], s_wsuf[NW];

    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t L0 = n - 1;
    // 32-bit index math throughout (n <= 2^30): a 64-bit min() here was
    // miscompiled by hipcc 7.2 (v_cmp_*_u64 + s_cselect on a stale SCC).
    const uint32_t B0 = blockIdx.x * (uint32_t)T;
    const uint32_t B1 = (n - B0) < (uint32_t)T ? n : B0 + (uint32_t)T;
    const uint32_t k = B0 + tid;
    const bool valid = k < B1;

    Aabb box = aabb_empty();
    uint4 tp = make_uint4(0, 0, 0, 0);
    if (valid) {
        const uint32_t prim = svals[k];
        float t[9];
        const float* src = tris + (uint64_t)prim * 9;
#pragma unroll
        for (int c = 0; c < 9; ++c) t[c] = src[c];
        tri_bounds(t, box.lo, box.hi);
        const uint32_t e = (k == n - 1) ? RT_SENT : lesc[k];
        store_node(nodes, L0 + (uint32_t)k, box, prim, e);
        s_box[tid] = box;
        s_par[tid] = (n > 1) ? parent[L0 + k] : RT_SENT;
        if (k + 1 < n) {  // internal node k exists
            tp = topo[k];
            s_topo[tid] = tp;
            s_par[T + tid] = parent[k];
        }
    }
    s_cnt[tid] = 0u;
    // ---- block prefix / suffix scans of leaf AABBs (exact min/max)
    Aabb pre = box, suf = box;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) { shfl_up_aabb(pre, o); shfl_down_aabb(suf, o); }
    if (lane == 63) s_wpre[wv] = pre;
    if (lane == 0) s_wsuf[wv] = suf;
    __syncthreads();
    for (uint32_t q = 0; q < wv; ++q) aabb_union(pre, s_wpre[q]);
    for (uint32_t q = wv + 1; q < NW; ++q) aabb_union(suf, s_wsuf[q]);
    if (valid) {
        // crossing ends (see DESIGN.md "refit"): the topmost node starting at
        // leaf k is internal k iff its range starts at k; the topmost node
        // ending at k is internal k iff its range ends at k; the root ends at n-1.
        const bool has_int = k + 1 < n;
        const bool need_suf = has_int && tp.z == k && tp.w >= B1;
        const bool need_pre = (has_int && tp.w == k && tp.z < B0) || (k == n - 1 && B0 > 0);
        if (need_suf) store_aabb(sufbuf, k, suf);
        if (need_pre) store_aabb(prebuf, k, pre);
        if (k == B1 - 1) store_aabb(totals, blockIdx.x, pre);
        if (has_int && (tp.z < B0 || tp.w >= B1)) {
            const uint32_t slot = atomicAdd(cross_ctr, 1u);
            cross[slot] = (uint32_t)k;
        }
    }
    __syncthreads();
    if (!valid || n == 1) return;
    // ---- bottom-up climb inside the block (LDS arrival counters)
    uint32_t node = L0 + (uint32_t)k;
    uint32_t slot = tid;
    for (uint32_t depth = 0; depth < (uint32_t)T; ++depth) {  // local depth < T
        const uint32_t p = s_par[slot];
        if (p == RT_SENT || p < B0 || p >= B1) break;
        const uint4 pt = s_topo[p - B0];
        if (pt.z < B0 || pt.w >= B1) break;  // p crosses the block: K6t's job
        const uint32_t old = __hip_atomic_fetch_add(&s_cnt[p - B0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (old == 0u) break;  // first arrival: the sibling finishes p
        const uint32_t left = pt.x;
        const uint32_t g = left >= L0 ? left - L0 : left;
        const uint32_t right = (pt.w == g + 1) ? L0 + g + 1 : g + 1;
        const uint32_t sib = (left == node) ? right : left;
        const uint32_t sslot = sib >= L0 ? (sib - L0 - (uint32_t)B0) : (T + sib - (uint32_t)B0);
        aabb_union(box, s_box[sslot]);
        slot = T + (p - (uint32_t)B0);
        s_box[slot] = box;
        store_node(nodes, p, box, pt.x, pt.y);
        node = p;
    }
}

// LDS segment tree over the M per-block totals (M <= kLdsTreeMaxBlocks) or a
// global sparse table (levels built by k_sparse_level) for larger M.
__global__ __launch_bounds__(256) void k_sparse_level(const float* __restrict__ src, float* __restrict__ dst, uint32_t m, uint32_t half) {
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b >= m) return;
    Aabb a = load_aabb(src, b);
    if (b + half < m) aabb_union(a, load_aabb(src, b + half));
    store_aabb(dst, b, a);
}

template <bool LDS_TREE>
__global__ __launch_bounds__(256) void k_refit_cross(const uint4* __restrict__ topo,
                                                     const float* __restrict__ prebuf, const float* __restrict__ sufbuf,
                                                     const float* __restrict__ table /* totals, or sparse levels */,
                                                     uint32_t m, const uint32_t* __restrict__ cross,
                                                     const uint32_t* __restrict__ cross_ctr, void* __restrict__ nodes,
                                                     uint32_t n) {
    constexpr uint32_t T = kRefitT;
    extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
    Aabb* tree = reinterpret_cast<Aabb*>(s_raw);
    uint32_t P = 1;
    while (P < m) P <<= 1;
    if (LDS_TREE) {
        for (uint32_t j = threadIdx.x; j < P; j += 256) tree[P + j] = j < m ? load_aabb(table, j) : aabb_empty();
        __syncthreads();
        for (uint32_t len = P >> 1; len >= 1; len >>= 1) {
            for (uint32_t j = threadIdx.x; j < len; j += 256) {
                Aabb a = tree[2 * (len + j)];
                aabb_union(a, tree[2 * (len + j) + 1]);
                tree[len + j] = a;
            }
            __syncthreads();
        }
    }
    const uint32_t count = *cross_ctr;
    for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q < count; q += gridDim.x * 256) {
        const uint32_t i = cross[q];
        const uint4 tp = topo[i];
        const uint32_t l = tp.z, r = tp.w;
        if (l >= n || r >= n || l > r) continue;  // malformed topology: never read out of bounds
        Aabb box = load_aabb(sufbuf, l);
        aabb_union(box, load_aabb(prebuf, r));
        const uint32_t bl = l / T + 1, br = r / T;  // middle blocks [bl, br)
        if (bl < br) {
            if (LDS_TREE) {
                uint32_t a = bl + P, b = br + P;
                while (a < b) {
                    if (a & 1) aabb_union(box, tree[a++]);
                    if (b & 1) aabb_union(box, tree[--b]);
                    a >>= 1;
                    b >>= 1;
                }
            } else {
                const uint32_t len = br - bl;
                const uint32_t s = 31 - __clz((int)len);
                const float* lvl = table + (uint64_t)s * m * 6;
                aabb_union(box, load_aabb(lvl, bl));
                aabb_union(box, load_aabb(lvl, br - (1u << s)));
            }
        }
        store_node(nodes, i, box, tp.x, tp.y);
    }
}

template __global__ void k_onesweep<0>(const uint32_t*, const uint32_t*, uint32_t*, uint32_t*, uint32_t, const uint32_t*, uint32_t*, uint32_t, uint32_t*, uint32_t*);
template __global__ void k_onesweep<8>(const uint32_t*, const uint32_t*, uint32_t*, uint32_t*, uint32_t, const uint32_t*, uint32_t*, uint32_t, uint32_t*, uint32_t*);
template __global__ void k_onesweep<16>(const uint32_t*, const uint32_t*, uint32_t*, uint32_t*, uint32_t, const uint32_t*, uint32_t*, uint32_t, uint32_t*, uint32_t*);
template __global__ void k_onesweep<24>(const uint32_t*, const uint32_t*, uint32_t*, uint32_t*, uint32_t, const uint32_t*, uint32_t*, uint32_t, uint32_t*, uint32_t*);
template __global__ void k_refit_cross<true>(const uint4*, const float*, const float*, const float*, uint32_t, const uint32_t*, const uint32_t*, void*, uint32_t);
template __global__ void k_refit_cross<false>(const uint4*, const float*, const float*, const float*, uint32_t, const uint32_t*, const uint32_t*, void*, uint32_t);

// Stand-alone digit histogram (rt_stage_sort on caller keys; the build fuses
// this into K1).
__global__ __launch_bounds__(256) void k_digit_hist(const uint32_t* __restrict__ keys, uint32_t n, uint32_t* __restrict__ ghist) {
    __shared__ uint32_t hist[4 * 256];
    for (int j = threadIdx.x; j < 1024; j += 256) hist[j] = 0u;
    __syncthreads();
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        const uint32_t key = keys[i];
#pragma unroll
        for (int d = 0; d < 4; ++d) atomicAdd(&hist[d * 256 + ((key >> (8 * d)) & 0xFFu)], 1u);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < 1024; j += 256) {
        const uint32_t v = hist[j];
        if (v) atomicAdd(&ghist[j], v);
    }
}

// ================================================================ launchers
static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

uint32_t sort_tiles(uint32_t n) { return n ? cdiv(n, kSortTile) : 0u; }

static uint32_t sparse_levels(uint32_t m) {
    uint32_t L = 1;
    while ((1ull << L) < m) ++L;
    return L;
}

hipError_t alloc_build(BuildBufs& b, uint32_t n) {
    free_build(b);
    const uint64_t N = n ? n : 1;
    b.cap_n = n;
    b.ntiles = sort_tiles((uint32_t)N);
    b.m_blocks = cdiv(N, kRefitT);
    b.levels = sparse_levels(b.m_blocks);
    b.nzero = kZStatus + 4u * 256u * b.ntiles;
    hipError_t e;
#define RT_ALLOC(ptr, bytes) \
    if ((e = hipMalloc((void**)&(ptr), (bytes))) != hipSuccess) { free_build(b); return e; }
    RT_ALLOC(b.tris, N * 36);
    RT_ALLOC(b.keys[0], N * 4);
    RT_ALLOC(b.keys[1], N * 4);
    RT_ALLOC(b.vals[0], N * 4);
    RT_ALLOC(b.vals[1], N * 4);
    RT_ALLOC(b.nodes, (2 * N - 1) * 32);
    RT_ALLOC(b.parent, (2 * N - 1) * 4);
    RT_ALLOC(b.topo, N * 16);
    RT_ALLOC(b.lesc, N * 4);
    RT_ALLOC(b.prebuf, N * 24);
    RT_ALLOC(b.sufbuf, N * 24);
    RT_ALLOC(b.table, (uint64_t)b.levels * b.m_blocks * 24);
    RT_ALLOC(b.cross, N * 4);
    RT_ALLOC(b.partials, kBoundsGrid * 24);
    RT_ALLOC(b.ticket, 256);
    RT_ALLOC(b.params, sizeof(BuildParams));
    RT_ALLOC(b.zero, (uint64_t)b.nzero * 4);
#undef RT_ALLOC
    if ((e = hipMemset(b.ticket, 0, 256)) != hipSuccess) { free_build(b); return e; }
    if ((e = hipMemset(b.zero, 0, (uint64_t)b.nzero * 4)) != hipSuccess) { free_build(b); return e; }
    return hipSuccess;
}

void free_build(BuildBufs& b) {
    void* ps[] = {b.tris, b.keys[0], b.keys[1], b.vals[0], b.vals[1], b.nodes, b.parent, b.topo, b.lesc,
                  b.prebuf, b.sufbuf, b.table, b.cross, b.partials, b.ticket, b.params, b.zero};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    b = BuildBufs{};
}

hipError_t launch_bounds_only(const float* tris, uint32_t n, float* partials, uint32_t* ticket,
                              BuildParams* params, hipStream_t s) {
    const uint32_t g = std::max(1u, std::min<uint32_t>(kBoundsGrid, cdiv(n, 256)));
    hipLaunchKernelGGL(k_bounds, dim3(g), dim3(256), 0, s, tris, n, partials, ticket, params, (uint32_t*)nullptr, 0u);
    return hipGetLastError();
}

hipError_t launch_morton(const float* tris, uint32_t n, const BuildParams* params, uint32_t* keys,
                         uint32_t* vals, uint32_t* ghist, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint32_t g = std::min<uint32_t>(512, cdiv(n, 256));
    hipLaunchKernelGGL(k_morton, dim3(g), dim3(256), 0, s, tris, n, params, keys, vals, ghist);
    return hipGetLastError();
}

hipError_t launch_digit_hist(const uint32_t* keys, uint32_t n, uint32_t* ghist, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint32_t g = std::min<uint32_t>(512, cdiv(n, 256));
    hipLaunchKernelGGL(k_digit_hist, dim3(g), dim3(256), 0, s, keys, n, ghist);
    return hipGetLastError();
}

// 4 onesweep passes, ping-pong 0->1->0->1->0; zero = control words (zeroed).
hipError_t launch_sort(uint32_t* keys[2], uint32_t* vals[2], uint32_t n, uint32_t* zero, hipStream_t s) {
    if (n <= 1) return hipSuccess;
    const uint32_t nt = sort_tiles(n);
    uint32_t* hist = zero + kZHist;
    uint32_t* st = zero + kZStatus;
    const uint64_t sstride = 256ull * nt;
    hipLaunchKernelGGL(k_onesweep<0>, dim3(nt), dim3(kSortThreads), 0, s, keys[0], vals[0], keys[1], vals[1], n,
                       hist + 0, st + 0 * sstride, nt, zero + kZTileCtr + 0, zero + kZErr);
    hipLaunchKernelGGL(k_onesweep<8>, dim3(nt), dim3(kSortThreads), 0, s, keys[1], vals[1], keys[0], vals[0], n,
                       hist + 256, st + 1 * sstride, nt, zero + kZTileCtr + 1, zero + kZErr);
    hipLaunchKernelGGL(k_onesweep<16>, dim3(nt), dim3(kSortThreads), 0, s, keys[0], vals[0], keys[1], vals[1], n,
                       hist + 512, st + 2 * sstride, nt, zero + kZTileCtr + 2, zero + kZErr);
    hipLaunchKernelGGL(k_onesweep<24>, dim3(nt), dim3(kSortThreads), 0, s, keys[1], vals[1], keys[0], vals[0], n,
                       hist + 768, st + 3 * sstride, nt, zero + kZTileCtr + 3, zero + kZErr);
    return hipGetLastError();
}

hipError_t launch_karras(const uint32_t* keys, uint32_t n, uint4* topo, uint32_t* parent, uint32_t* lesc,
                         hipStream_t s) {
    if (n < 2) return hipSuccess;
    hipLaunchKernelGGL(k_karras, dim3(cdiv(n - 1, 256)), dim3(256), 0, s, keys, n, topo, parent, lesc);
    return hipGetLastError();
}

static hipError_t launch_refit(const BuildBufs& b, uint32_t n, hipStream_t s) {
    const uint32_t m = cdiv(n, kRefitT);
    hipLaunchKernelGGL(k_refit_local, dim3(m), dim3(kRefitT), 0, s, b.tris, n, b.vals[0], b.topo, b.parent, b.lesc,
                       b.nodes, b.prebuf, b.sufbuf, b.table, b.cross, b.zero + kZCrossCtr);
    if (m <= 1) return hipGetLastError();
    if (m <= (uint32_t)kLdsTreeMaxBlocks) {
        uint32_t P = 1;
        while (P < m) P <<= 1;
        const size_t lds = 2ull * P * sizeof(Aabb);
        static bool attr_set = false;
        if (!attr_set) {
            hipError_t e = hipFuncSetAttribute((const void*)k_refit_cross<true>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               2 * kLdsTreeMaxBlocks * (int)sizeof(Aabb));
            if (e != hipSuccess) return e;
            attr_set = true;
        }
        hipLaunchKernelGGL(k_refit_cross<true>, dim3(64), dim3(256), lds, s, b.topo, b.prebuf, b.sufbuf, b.table, m,
                           b.cross, b.zero + kZCrossCtr, b.nodes, n);
    } else {
        const uint32_t L = sparse_levels(m);
        for (uint32_t lv = 1; lv < L; ++lv) {
            hipLaunchKernelGGL(k_sparse_level, dim3(cdiv(m, 256)), dim3(256), 0, s, b.table + (uint64_t)(lv - 1) * m * 6,
                               b.table + (uint64_t)lv * m * 6, m, 1u << (lv - 1));
        }
        hipLaunchKernelGGL(k_refit_cross<false>, dim3(256), dim3(256), 0, s, b.topo, b.prebuf, b.sufbuf, b.table, m,
                           b.cross, b.zero + kZCrossCtr, b.nodes, n);
    }
    return hipGetLastError();
}

hipError_t launch_build(const BuildBufs& b, uint32_t n, hipStream_t s, BuildEvents* ev) {
    hipError_t e;
    auto rec = [&](int i) -> hipError_t { return ev ? hipEventRecord(ev->e[i], s) : hipSuccess; };
    if ((e = rec(0)) != hipSuccess) return e;
    const uint32_t g = std::max(1u, std::min<uint32_t>(kBoundsGrid, cdiv(n, 256)));
    hipLaunchKernelGGL(k_bounds, dim3(g), dim3(256), 0, s, b.tris, n, b.partials, b.ticket, b.params, b.zero,
                       kZStatus + 4u * 256u * sort_tiles(n));
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = rec(1)) != hipSuccess) return e;
    if ((e = launch_morton(b.tris, n, b.params, b.keys[0], b.vals[0], b.zero + kZHist, s)) != hipSuccess) return e;
    if ((e = rec(2)) != hipSuccess) return e;
    uint32_t* K[2] = {b.keys[0], b.keys[1]};
    uint32_t* V[2] = {b.vals[0], b.vals[1]};
    if ((e = launch_sort(K, V, n, b.zero, s)) != hipSuccess) return e;
    if ((e = rec(3)) != hipSuccess) return e;
    if ((e = launch_karras(b.keys[0], n, b.topo, b.parent, b.lesc, s)) != hipSuccess) return e;
    // n == 1: no internal node, K4 is not launched; the root is leaf 0.
    if (n == 1 && (e = hipMemsetAsync(b.parent, 0xFF, 4, s)) != hipSuccess) return e;
    if ((e = rec(4)) != hipSuccess) return e;
    if (n && (e = launch_refit(b, n, s)) != hipSuccess) return e;
    if ((e = rec(5)) != hipSuccess) return e;
    return hipSuccess;
}

}  // namespace rt

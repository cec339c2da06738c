// sort_kernels.hip -- stable 32-bit LSB radix sort (4 x 8-bit digits) of
// Morton key / prim-index pairs for gfx950 (§9.4).
//
// Per digit pass, two launches and no intra-launch inter-workgroup traffic:
//   k_tile_hist<S>  per-tile (4096 keys) digit counts -> counts[tile][256]
//                   (pass 0's counts come from K1, whose block is one tile)
//   k_scatter<S>    ranks the tile's keys stably (wave64 ballot match-any,
//                   per-wave LDS digit counters), buckets them in LDS, then
//                   writes each digit run coalesced to
//                   digit_base[d] + sum_{tiles i < t} counts[i][d] + local.
// digit_base comes from the 4 global histograms K1 builds once (exact
// totals for every pass).  The cross-tile prefix is summed inside the
// scatter kernel from plain loads of the previous launch's counts (<= 256
// tiles, i.e. <= 1M keys); above that k_scan_tiles turns counts into
// exclusive offsets first.  Why not single-pass decoupled look-back: every
// poll of another CU's status word is a device-scope (L2-bypassing) load, and
// the measured chain cost ~2.5 us per hop on MI355X (tools/diag_stamps.py).
#include "rt_device.h"
#include "rt_launch.h"
#include "sort_device.h"

#include <algorithm>
#include <cmath>
#include <mutex>

namespace rt {

#ifdef RT_STAMPS
hipError_t read_stamps_sort(void* out, size_t bytes) { return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rt_stamps), bytes); }
#endif

// exclusive scan of one value per thread over threads [0,256) of a block of
// kSortThreads (others pass 0); returns the prefix for threads < 256.
__device__ __forceinline__ uint32_t scan256(uint32_t v, uint32_t* sw /* [4] */) {
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (l >= (uint32_t)o) x += y;
    }
    if (l == 63 && w < 4) sw[w] = x;
    __syncthreads();
    uint32_t pre = 0;
    for (uint32_t k = 0; k < w && k < 4; ++k) pre += sw[k];
    __syncthreads();
    return pre + x - v;
}

// ---------------------------------------------------------------- histogram
template <int SHIFT>
__global__ __launch_bounds__(kSortThreads) void k_tile_hist(const uint32_t* __restrict__ keys, uint32_t n,
                                                            uint32_t* __restrict__ counts /* [tile][256] */,
                                                            Gate gate = Gate{}) {
    if (gated_off(gate)) return;
    __shared__ uint32_t h[256];
    if (threadIdx.x < 256) h[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t base = blockIdx.x * (uint32_t)kSortTile + threadIdx.x * (uint32_t)kSortItems;
    if (base + kSortItems <= n) {
        const uint4* p = reinterpret_cast<const uint4*>(keys + base);
        const uint4 a = p[0], b = p[1];
        const uint32_t k[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) atomicAdd(&h[(k[i] >> SHIFT) & 0xFFu], 1u);
    } else {
#pragma unroll
        for (uint32_t i = 0; i < (uint32_t)kSortItems; ++i)
            if (base + i < n) atomicAdd(&h[(keys[base + i] >> SHIFT) & 0xFFu], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 256) counts[(uint64_t)blockIdx.x * 256 + threadIdx.x] = h[threadIdx.x];
}

// In-place exclusive scan of counts[tile][d] over tiles, one workgroup per
// digit (used when tiles > kPrefixInKernelMaxTiles).
__global__ __launch_bounds__(256) void k_scan_tiles(uint32_t* __restrict__ counts, uint32_t ntiles,
                                                    Gate gate = Gate{}) {
    if (gated_off(gate)) return;
    __shared__ uint32_t sw[4];
    __shared__ uint32_t s_carry;
    const uint32_t d = blockIdx.x;
    if (threadIdx.x == 0) s_carry = 0u;
    __syncthreads();
    for (uint32_t c0 = 0; c0 < ntiles; c0 += 256 * 8) {
        uint32_t v[8], sum = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t i = c0 + threadIdx.x * 8 + j;
            v[j] = i < ntiles ? counts[(uint64_t)i * 256 + d] : 0u;
            sum += v[j];
        }
        const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
        uint32_t x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (l >= (uint32_t)o) x += y;
        }
        if (l == 63) sw[w] = x;
        __syncthreads();
        uint32_t pre = s_carry;
        for (uint32_t k = 0; k < w; ++k) pre += sw[k];
        pre += x - sum;
        const uint32_t total = sw[0] + sw[1] + sw[2] + sw[3];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t i = c0 + threadIdx.x * 8 + j;
            if (i < ntiles) counts[(uint64_t)i * 256 + d] = pre;
            pre += v[j];
        }
        __syncthreads();
        if (threadIdx.x == 0) s_carry += total;
        __syncthreads();
    }
}

// ---------------------------------------------------------------- scatter
template <int SHIFT, bool PREFIX_IN_KERNEL>
__global__ __launch_bounds__(kSortThreads) void k_scatter(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                          uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                          uint32_t n, const uint32_t* __restrict__ ghist /* this digit's 256 */,
                                                          const uint32_t* __restrict__ counts /* [tile][256] counts or offsets */,
                                                          Gate gate = Gate{}) {
    if (gated_off(gate)) return;
    constexpr int W = kSortThreads / 64;  // 8 waves
    __shared__ uint32_t s_wc[W][256];
    __shared__ uint32_t s_key[kSortTile];
    __shared__ uint32_t s_val[kSortTile];
    __shared__ uint32_t s_lstart[256];
    __shared__ uint32_t s_gofs[256];
    __shared__ uint32_t s_part[8][256];
    __shared__ uint32_t s_sw[4];

    const uint32_t tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const uint32_t tile = blockIdx.x;
    const uint32_t base = tile * (uint32_t)kSortTile;
    RT_STAMP(0);
    for (uint32_t j = tid; j < W * 256; j += kSortThreads) (&s_wc[0][0])[j] = 0u;

    // ---- cross-tile prefix of this tile's digit offsets (independent of the
    // ranking below: issue it first so its loads overlap the key loads)
    uint4 part = make_uint4(0, 0, 0, 0);
    if (PREFIX_IN_KERNEL) {
        // thread t: digits 4q..4q+3 (q = t & 63), tiles i = p (mod 8) (p = t >> 6)
        const uint32_t q = tid & 63, p = tid >> 6;
        const uint4* c4 = reinterpret_cast<const uint4*>(counts);
        for (uint32_t i = p; i < tile; i += 8 * 4) {
            uint4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t ii = i + 8 * u;
                v[u] = ii < tile ? c4[(uint64_t)ii * 64 + q] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) { part.x += v[u].x; part.y += v[u].y; part.z += v[u].z; part.w += v[u].w; }
        }
    }

    uint32_t k[kSortItems], v[kSortItems], r[kSortItems];
#pragma unroll
    for (int i = 0; i < kSortItems; ++i) {
        const uint32_t idx = base + w * (64u * kSortItems) + i * 64u + l;
        const bool ok = idx < n;
        k[i] = ok ? kin[idx] : 0u;
        v[i] = ok ? vin[idx] : 0u;
    }
    if (PREFIX_IN_KERNEL) {
        const uint32_t q = tid & 63, p = tid >> 6;
        s_part[p][4 * q] = part.x; s_part[p][4 * q + 1] = part.y;
        s_part[p][4 * q + 2] = part.z; s_part[p][4 * q + 3] = part.w;
    }
    __syncthreads();
    RT_STAMP(1);
    // ---- stable per-wave ranking: order (wave, item, lane) == index order
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
        const uint32_t below = sort_count_below(peers);
        const uint32_t cur = s_wc[w][d];
        r[i] = cur + below;
        if (ok && below == 0) s_wc[w][d] = cur + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    RT_STAMP(2);
    // ---- per-digit tile count, per-wave exclusive prefix (in place)
    uint32_t cnt = 0;
    if (tid < 256) {
#pragma unroll
        for (int ww = 0; ww < W; ++ww) {
            const uint32_t c = s_wc[ww][tid];
            s_wc[ww][tid] = cnt;
            cnt += c;
        }
    }
    const uint32_t lstart = scan256(tid < 256 ? cnt : 0u, s_sw);
    const uint32_t dbase = scan256(tid < 256 ? ghist[tid & 255] : 0u, s_sw);
    if (tid < 256) {
        s_lstart[tid] = lstart;
        uint32_t pre;
        if (PREFIX_IN_KERNEL) {
            pre = 0;
#pragma unroll
            for (int p = 0; p < 8; ++p) pre += s_part[p][tid];
        } else {
            pre = counts[(uint64_t)tile * 256 + tid];  // exclusive offsets from k_scan_tiles
        }
        s_gofs[tid] = dbase + pre;
    }
    __syncthreads();
    RT_STAMP(3);
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
    RT_STAMP(4);
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
    RT_STAMP(5);
}

// Stand-alone 4-digit global histogram (rt_stage_sort on caller keys; the
// build gets it from K1).
__global__ __launch_bounds__(256) void k_digit_hist(const uint32_t* __restrict__ keys, uint32_t n, uint32_t* __restrict__ ghist,
                                                    Gate gate = Gate{}) {
    if (gated_off(gate)) return;
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

// ================================================================ MSB bucket sort
// The build's sort for 2 <= n <= kMsbMaxN 30-bit Morton keys: one global
// scatter by the top 10 key bits, then every bucket sorted on its own in LDS
// -- two scatter levels instead of four LSB passes.
//   K1 (k_morton<true>)  per-tile counts of bucket d = key >> 20 and the
//                        global bucket histogram (one LDS atomic per key);
//   k_msb_scan           counts -> exclusive destinations offs[tile][d] =
//                        bucket start + earlier tiles' counts; bucket starts;
//   k_msb_scatter        one 4096-key tile per block: stable 10-bit ballot
//                        ranking, LDS bucketing, runs -> keys[1]/vals[1];
//   k_bucket_sort        one bucket per block: stable LSB sort of the bucket by
//                        the low 20 key bits (2 x 10-bit passes) in LDS ->
//                        keys[0]/vals[0]; a bucket over kBucketCap keys runs
//                        the same passes chunk by chunk through global memory.
// The first level is stable, so a bucket arrives in index order, and the
// second is stable: the result is §9.4's unique (key, index) order, the LSB
// sort's (tests/test_parity_gpu.py compares the two).
constexpr int kBucketThreads = 256;
constexpr int kBucketWaves = kBucketThreads / 64;
constexpr uint32_t kBucketCap = kBucketThreads * kSortItems;  // keys per LDS sort

// counts[t][d] (t < nt <= 512) -> exclusive destinations bucket start +
// sum_{t' < t} counts[t'][d], in place; bstart[0..1024] = bucket starts.
// 16 blocks x 1024 threads: block b owns buckets [64b, 64b + 64), a thread
// one bucket and a chunk of <= 32 tiles.
// dense (optional): 1 when a bucket holds more than cap keys (a probe build's
// verdict: the gated MSB kernels below stand down and the LSB sort runs), else 0
__global__ __launch_bounds__(1024) void k_msb_scan(uint32_t* __restrict__ offs, uint32_t nt,
                                                   const uint32_t* __restrict__ ghist, uint32_t* __restrict__ bstart,
                                                   uint32_t cap = 0, uint32_t* __restrict__ dense = nullptr) {
    __shared__ uint32_t s_base[kMsbBuckets];
    __shared__ uint32_t s_sw[16];
    __shared__ uint32_t s_csum[16][64];
    const uint32_t t = threadIdx.x;
    const uint32_t g = ghist[t];
    s_base[t] = g;
    __syncthreads();
    scan1024<1024>(s_base, s_sw);
    if (blockIdx.x == 0) {
        bstart[t] = s_base[t];
        if (t == kMsbBuckets - 1) bstart[kMsbBuckets] = s_base[t] + g;
        if (dense) {  // block-uniform branch: every thread of block 0 reaches the barrier
            const int big = __syncthreads_or(g > cap);
            if (t == 0) dense[0] = big ? 1u : 0u;
        }
    }
    const uint32_t dl = t & 63, c = t >> 6, d = blockIdx.x * 64 + dl;
    const uint32_t C = (nt + 15) / 16;
    uint32_t v[32], sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < 32; ++j) {
        const uint32_t tt = c * C + j;
        v[j] = (j < C && tt < nt) ? offs[(uint64_t)tt * kMsbBuckets + d] : 0u;
        sum += v[j];
    }
    s_csum[c][dl] = sum;
    __syncthreads();
    uint32_t run = s_base[d];
    for (uint32_t k = 0; k < c; ++k) run += s_csum[k][dl];
#pragma unroll
    for (uint32_t j = 0; j < 32; ++j) {
        const uint32_t tt = c * C + j;
        if (j < C && tt < nt) {
            offs[(uint64_t)tt * kMsbBuckets + d] = run;
            run += v[j];
        }
    }
}

// First level: one tile of NT * P keys per block (kSortTile = 4096 for
// n <= kMsbMaxN; 4 sort tiles = 16384 keys per 1024-thread block above, so a
// bucket's run from one block is ~16 keys instead of ~4 -- the 10M path's
// output writes), bucket d = key >> 20.  offs = the exclusive destinations
// of the block's first sort tile.
template <int NT, int P>
__device__ __forceinline__ void msb_scatter_tile(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                 uint32_t* __restrict__ kout, uint32_t* __restrict__ vout, uint32_t n,
                                                 const uint32_t* __restrict__ offs, uint32_t* s_buf,
                                                 uint32_t* s_start, uint32_t* s_gofs, uint32_t* s_sw) {
    constexpr int W = NT / 64;
    constexpr uint32_t TILE = (uint32_t)NT * P;
    // s_buf holds max(W * 1024 counters, the bucketed tile's 2 * TILE words)
    uint32_t(*s_wc)[kMsbBuckets] = reinterpret_cast<uint32_t(*)[kMsbBuckets]>(s_buf);
    uint32_t* s_key = s_buf;
    uint32_t* s_val = s_buf + TILE;
    const uint32_t tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const uint32_t base = blockIdx.x * TILE;
    for (uint32_t j = tid; j < W * kMsbBuckets / 4; j += NT) reinterpret_cast<uint4*>(s_buf)[j] = make_uint4(0, 0, 0, 0);
    const uint64_t orow = (uint64_t)blockIdx.x * (TILE / kSortTile) * kMsbBuckets;
    for (uint32_t j = tid; j < kMsbBuckets; j += NT) s_gofs[j] = offs[orow + j];
    uint32_t k[P], v[P], dg[P], r[P];
    bool ok[P];
#pragma unroll
    for (int i = 0; i < P; ++i) {
        const uint32_t idx = base + w * (64u * P) + i * 64u + l;
        ok[i] = idx < n;
        k[i] = ok[i] ? kin[idx] : 0u;
        v[i] = ok[i] ? vin[idx] : 0u;
        dg[i] = (k[i] >> kMsbShift) & (kMsbBuckets - 1);
    }
    __syncthreads();
    rank10<P>(dg, ok, s_wc, r);
    __syncthreads();
    wave_prefix4<W, NT>(s_wc, s_start);
    __syncthreads();
    scan1024<NT>(s_start, s_sw);
    uint32_t pos[P];
#pragma unroll
    for (int i = 0; i < P; ++i) pos[i] = s_start[dg[i]] + s_wc[w][dg[i]] + r[i];
    __syncthreads();  // the counters are dead: the buffer becomes the bucketed tile
#pragma unroll
    for (int i = 0; i < P; ++i)
        if (ok[i]) {
            s_key[pos[i]] = k[i];
            s_val[pos[i]] = v[i];
        }
    __syncthreads();
    const uint32_t trem = n - base;
    const uint32_t tcount = trem < TILE ? trem : TILE;
#pragma unroll
    for (int m = 0; m < P; ++m) {
        const uint32_t q = tid + m * NT;
        if (q < tcount) {
            const uint32_t key = s_key[q];
            const uint32_t d = (key >> kMsbShift) & (kMsbBuckets - 1);
            const uint32_t o = s_gofs[d] + (q - s_start[d]);
            kout[o] = key;
            vout[o] = s_val[q];
        }
    }
}

#ifndef RT_MSB_SCATTER_NT
#define RT_MSB_SCATTER_NT 512
#endif
constexpr int kMsbScatterNT = RT_MSB_SCATTER_NT;  // threads per 4096-key tile
static_assert(kSortTile % kMsbScatterNT == 0, "a tile is whole items per thread");
constexpr uint32_t kMsbScatterBuf = (kMsbScatterNT / 64) * kMsbBuckets > 2 * kSortTile
                                        ? (kMsbScatterNT / 64) * kMsbBuckets : 2 * kSortTile;
__global__ __launch_bounds__(kMsbScatterNT) void k_msb_scatter(const uint32_t* __restrict__ kin,
                                                              const uint32_t* __restrict__ vin,
                                                              uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                              uint32_t n, const uint32_t* __restrict__ offs, Gate gate = Gate{}) {
    if (gated_off(gate)) return;
    __shared__ __attribute__((aligned(16))) uint32_t s_buf[kMsbScatterBuf];  // ranking counters s_wc[W][1024], then the bucketed tile
    __shared__ __attribute__((aligned(16))) uint32_t s_start[kMsbBuckets];
    __shared__ uint32_t s_gofs[kMsbBuckets];
    __shared__ uint32_t s_sw[kMsbScatterNT / 64];
    msb_scatter_tile<kMsbScatterNT, kSortTile / kMsbScatterNT>(kin, vin, kout, vout, n, offs, s_buf, s_start, s_gofs, s_sw);
}

constexpr int kScatterBigItems = 16;
constexpr uint32_t kScatterBigTile = 1024u * kScatterBigItems;  // 4 sort tiles
constexpr size_t kScatterBigLds = (size_t)2 * kScatterBigTile * 4 + (size_t)kMsbBuckets * 4 * 2 + 64;
static_assert(16 * kMsbBuckets <= 2 * (int)kScatterBigTile, "the big scatter's counters fit its tile buffer");
__global__ __launch_bounds__(1024) void k_msb_scatter_big(const uint32_t* __restrict__ kin,
                                                          const uint32_t* __restrict__ vin,
                                                          uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                          uint32_t n, const uint32_t* __restrict__ offs, Gate gate = Gate{}) {
    if (gated_off(gate)) return;
    extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
    uint32_t* s_buf = s_dyn;
    uint32_t* s_start = s_dyn + 2 * kScatterBigTile;
    uint32_t* s_gofs = s_start + kMsbBuckets;
    uint32_t* s_sw = s_gofs + kMsbBuckets;
    msb_scatter_tile<1024, kScatterBigItems>(kin, vin, kout, vout, n, offs, s_buf, s_start, s_gofs, s_sw);
}

// Ranks one chunk (<= kBucketCap items in registers, item j = w*64*per +
// i*64 + lane, wave-major) by the 10-bit digit at `shift`: r[i] = the item's position among its
// digit's items of the chunk (earlier waves first, then item order); s_cnt =
// the chunk's digit counts.  Callers barrier before reusing s_wc.
template <int NT = kBucketThreads, int P = kSortItems>
__device__ __forceinline__ void bucket_rank(const uint32_t (&k)[P], const bool (&ok)[P],
                                            uint32_t shift, uint32_t (*s_wc)[kMsbBuckets], uint32_t* s_cnt,
                                            uint32_t (&dg)[P], uint32_t (&r)[P]) {
    constexpr int NW = NT / 64;
    {  // 16-B stores
        uint4* z = reinterpret_cast<uint4*>(&s_wc[0][0]);
        for (uint32_t j = threadIdx.x; j < NW * kMsbBuckets / 4; j += NT) z[j] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < P; ++i) dg[i] = (k[i] >> shift) & (kMsbBuckets - 1);
    rank10<P>(dg, ok, s_wc, r);
    __syncthreads();
    wave_prefix4<NW, NT>(s_wc, s_cnt);
    __syncthreads();
    const uint32_t w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < P; ++i) r[i] += s_wc[w][dg[i]];
}

// Second level: one bucket [bstart[b], bstart[b+1]) per block, sorted stably by
// key bits 0..19 (the bucket shares bits 20..29).
__global__ __launch_bounds__(kBucketThreads) void k_bucket_sort(uint32_t* __restrict__ kin, uint32_t* __restrict__ vin,
                                                                uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                                const uint32_t* __restrict__ bstart, Gate gate = Gate{}) {
    if (gated_off(gate)) return;
    static_assert(kBucketWaves * kMsbBuckets == 2 * kBucketCap, "counters and sorted chunk share one buffer");
    __shared__ __attribute__((aligned(16))) uint32_t s_wc[kBucketWaves][kMsbBuckets];  // ranking counters; fast path: then the sorted chunk
    __shared__ __attribute__((aligned(16))) uint32_t s_cnt[kMsbBuckets];
    __shared__ uint32_t s_run[kMsbBuckets];
    __shared__ uint32_t s_sw[kBucketWaves];
    const uint32_t s = bstart[blockIdx.x], m = bstart[blockIdx.x + 1] - s;
    if (m == 0) return;
    const uint32_t tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    uint32_t k[kSortItems], v[kSortItems], dg[kSortItems], r[kSortItems];
    bool ok[kSortItems];
    if (m <= kBucketCap) {
        uint32_t* s_key = &s_wc[0][0];
        uint32_t* s_val = s_key + kBucketCap;
        // per items per lane (<= kSortItems): wave w holds [64 per w, 64 per (w+1)),
        // so all four waves rank a partly filled bucket (index order is
        // wave-major, then item, then lane, as the ranking counts it)
        const uint32_t per = (m + kBucketThreads - 1) / kBucketThreads;
        RT_STAMP(0);
#pragma unroll
        for (int i = 0; i < kSortItems; ++i) {
            const uint32_t j = w * (64u * per) + i * 64u + l;
            ok[i] = (uint32_t)i < per && j < m;
            k[i] = ok[i] ? kin[s + j] : 0u;
            v[i] = ok[i] ? vin[s + j] : 0u;
        }
        for (uint32_t shift = 0; shift < kMsbShift; shift += 10) {
            RT_STAMP(1 + shift / 5);  // 1, 3: before the ranking
            bucket_rank(k, ok, shift, s_wc, s_cnt, dg, r);
            RT_STAMP(2 + shift / 5);  // 2, 4: ranked
            scan1024<kBucketThreads>(s_cnt, s_sw);  // its barriers also end every counter read
#pragma unroll
            for (int i = 0; i < kSortItems; ++i)
                if (ok[i]) {
                    const uint32_t p = s_cnt[dg[i]] + r[i];
                    s_key[p] = k[i];
                    s_val[p] = v[i];
                }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < kSortItems; ++i) {
                const uint32_t j = w * (64u * per) + i * 64u + l;
                if (ok[i]) {
                    k[i] = s_key[j];
                    v[i] = s_val[j];
                }
            }
            __syncthreads();
        }
        RT_STAMP(5);
#pragma unroll
        for (int i = 0; i < kSortItems; ++i) {
            const uint32_t j = w * (64u * per) + i * 64u + l;
            if (ok[i]) {
                kout[s + j] = k[i];
                vout[s + j] = v[i];
            }
        }
        RT_STAMP(6);
        return;
    }
    // A bucket beyond one LDS sort (clustered or degenerate scenes): the same
    // two passes chunk by chunk through global memory -- kin -> kout (digit 0),
    // kout -> kin (digit 1) -- then a copy kin -> kout.  The block owns
    // [s, s + m) of all four arrays.
    uint32_t *sk = kin, *sv = vin, *dk = kout, *dv = vout;
    for (uint32_t shift = 0; shift < kMsbShift; shift += 10) {
        for (uint32_t j = tid; j < kMsbBuckets; j += kBucketThreads) s_run[j] = 0u;
        __syncthreads();
        for (uint32_t j = tid; j < m; j += kBucketThreads) atomicAdd(&s_run[(sk[s + j] >> shift) & (kMsbBuckets - 1)], 1u);
        __syncthreads();
        scan1024<kBucketThreads>(s_run, s_sw);
        for (uint32_t c0 = 0; c0 < m; c0 += kBucketCap) {
#pragma unroll
            for (int i = 0; i < kSortItems; ++i) {
                const uint32_t j = c0 + w * (64u * kSortItems) + i * 64u + l;
                ok[i] = j < m;
                k[i] = ok[i] ? sk[s + j] : 0u;
                v[i] = ok[i] ? sv[s + j] : 0u;
            }
            bucket_rank(k, ok, shift, s_wc, s_cnt, dg, r);
#pragma unroll
            for (int i = 0; i < kSortItems; ++i)
                if (ok[i]) {
                    const uint32_t o = s_run[dg[i]] + r[i];
                    dk[s + o] = k[i];
                    dv[s + o] = v[i];
                }
            __syncthreads();  // s_run and s_wc reads done
            for (uint32_t d = tid; d < kMsbBuckets; d += kBucketThreads) s_run[d] += s_cnt[d];
            __syncthreads();
        }
        // this pass's stores before the next pass's loads by the block's other waves
        // (one CU, one L1: a workgroup-scope fence; __threadfence would also write
        // back the XCD's L2, ~60 us, profiles/calib_barrier_r03.log)
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __syncthreads();
        uint32_t* t0 = sk;
        sk = dk;
        dk = t0;
        t0 = sv;
        sv = dv;
        dv = t0;
    }
    for (uint32_t j = tid; j < m; j += kBucketThreads) {  // the result is in kin/vin
        kout[s + j] = kin[s + j];
        vout[s + j] = vin[s + j];
    }
}

// ---- large n (kMsbMaxN < n <= kMsbBigMaxN, the 10M path): the same two
// levels with more tiles and bigger buckets (~n/1024 keys each).
//   k_msb_chunk_sum, k_msb_scan, k_msb_chunk_apply: the tile-count prefix for
//     any number of tiles, over chunks of kMsbChunk tiles (per-chunk column
//     sums, their exclusive scan from the bucket starts by k_msb_scan on the
//     [chunk][1024] sums, then each chunk's tiles) instead of one 16-block
//     k_msb_scan whose threads would walk ~150 tiles each;
//   k_msb_scatter_big: the first level over 16384-key blocks;
//   k_bucket_sort_big: one bucket per 1024-thread block, the same two stable
//     10-bit passes in LDS (capacity kBigCap keys: 12 per thread), the
//     counters (16 waves x 1024) sharing the tile buffer; a bucket beyond
//     kBigCap runs the passes chunk by chunk through global memory.
uint32_t msb_bucket_cap(uint32_t n) { return n <= kMsbMaxN ? kBucketCap : (uint32_t)(1024 * 12); }

constexpr uint32_t kMsbChunk = 32;
constexpr int kBigThreads = 1024;
constexpr int kBigWaves = kBigThreads / 64;
constexpr int kBigItems = 12;
constexpr uint32_t kBigCap = kBigThreads * kBigItems;  // 12288 keys
constexpr size_t kBigLds = (size_t)2 * kBigCap * 4 + (size_t)kMsbBuckets * 4 * 2 + 64;  // tile + s_cnt + s_run + s_sw
static_assert(kBigWaves * kMsbBuckets <= 2 * (int)kBigCap, "the counters fit the tile buffer");

__global__ __launch_bounds__(1024) void k_msb_chunk_sum(const uint32_t* __restrict__ counts, uint32_t nt,
                                                         uint32_t* __restrict__ csum) {
    const uint32_t c = blockIdx.x, d = threadIdx.x, t0 = c * kMsbChunk;
    const uint32_t t1 = t0 + kMsbChunk < nt ? t0 + kMsbChunk : nt;
    uint32_t v[kMsbChunk], sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < kMsbChunk; ++j) v[j] = t0 + j < t1 ? counts[(uint64_t)(t0 + j) * kMsbBuckets + d] : 0u;
#pragma unroll
    for (uint32_t j = 0; j < kMsbChunk; ++j) sum += v[j];
    csum[(uint64_t)c * kMsbBuckets + d] = sum;
}

__global__ __launch_bounds__(1024) void k_msb_chunk_apply(uint32_t* __restrict__ counts, uint32_t nt,
                                                           const uint32_t* __restrict__ csum) {
    const uint32_t c = blockIdx.x, d = threadIdx.x, t0 = c * kMsbChunk;
    const uint32_t t1 = t0 + kMsbChunk < nt ? t0 + kMsbChunk : nt;
    uint32_t v[kMsbChunk];
#pragma unroll
    for (uint32_t j = 0; j < kMsbChunk; ++j) v[j] = t0 + j < t1 ? counts[(uint64_t)(t0 + j) * kMsbBuckets + d] : 0u;
    uint32_t run = csum[(uint64_t)c * kMsbBuckets + d];
#pragma unroll
    for (uint32_t j = 0; j < kMsbChunk; ++j)
        if (t0 + j < t1) {
            counts[(uint64_t)(t0 + j) * kMsbBuckets + d] = run;
            run += v[j];
        }
}

__global__ __launch_bounds__(kBigThreads) void k_bucket_sort_big(uint32_t* __restrict__ kin, uint32_t* __restrict__ vin,
                                                                 uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                                 const uint32_t* __restrict__ bstart, Gate gate = Gate{}) {
    if (gated_off(gate)) return;
    extern __shared__ __attribute__((aligned(16))) uint32_t s_big[];
    uint32_t(*s_wc)[kMsbBuckets] = reinterpret_cast<uint32_t(*)[kMsbBuckets]>(s_big);  // counters, then the tile
    uint32_t* s_key = s_big;
    uint32_t* s_val = s_big + kBigCap;
    uint32_t* s_cnt = s_big + 2 * kBigCap;
    uint32_t* s_run = s_cnt + kMsbBuckets;
    uint32_t* s_sw = s_run + kMsbBuckets;
    const uint32_t s = bstart[blockIdx.x], m = bstart[blockIdx.x + 1] - s;
    if (m == 0) return;
    const uint32_t tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    uint32_t k[kBigItems], v[kBigItems], dg[kBigItems], r[kBigItems];
    bool ok[kBigItems];
    if (m <= kBigCap) {
        // per items per lane: wave w holds [64 per w, 64 per (w + 1)) (index
        // order = wave, item, lane -- the ranking's order)
        const uint32_t per = (m + kBigThreads - 1) / kBigThreads;
#pragma unroll
        for (int i = 0; i < kBigItems; ++i) {
            const uint32_t j = w * (64u * per) + i * 64u + l;
            ok[i] = (uint32_t)i < per && j < m;
            k[i] = ok[i] ? kin[s + j] : 0u;
            v[i] = ok[i] ? vin[s + j] : 0u;
        }
        for (uint32_t shift = 0; shift < kMsbShift; shift += 10) {
            bucket_rank<kBigThreads, kBigItems>(k, ok, shift, s_wc, s_cnt, dg, r);
            scan1024<kBigThreads>(s_cnt, s_sw);  // its barriers also end every counter read
#pragma unroll
            for (int i = 0; i < kBigItems; ++i)
                if (ok[i]) {
                    const uint32_t p = s_cnt[dg[i]] + r[i];
                    s_key[p] = k[i];
                    s_val[p] = v[i];
                }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < kBigItems; ++i) {
                const uint32_t j = w * (64u * per) + i * 64u + l;
                if (ok[i]) {
                    k[i] = s_key[j];
                    v[i] = s_val[j];
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (int i = 0; i < kBigItems; ++i) {
            const uint32_t j = w * (64u * per) + i * 64u + l;
            if (ok[i]) {
                kout[s + j] = k[i];
                vout[s + j] = v[i];
            }
        }
        return;
    }
    // beyond one LDS sort: k_bucket_sort's chunked global passes with this
    // block's width (kin -> kout, kout -> kin, then the copy kin -> kout)
    uint32_t *sk = kin, *sv = vin, *dk = kout, *dv = vout;
    for (uint32_t shift = 0; shift < kMsbShift; shift += 10) {
        for (uint32_t j = tid; j < kMsbBuckets; j += kBigThreads) s_run[j] = 0u;
        __syncthreads();
        for (uint32_t j = tid; j < m; j += kBigThreads) atomicAdd(&s_run[(sk[s + j] >> shift) & (kMsbBuckets - 1)], 1u);
        __syncthreads();
        scan1024<kBigThreads>(s_run, s_sw);
        for (uint32_t c0 = 0; c0 < m; c0 += kBigCap) {
#pragma unroll
            for (int i = 0; i < kBigItems; ++i) {
                const uint32_t j = c0 + w * (64u * kBigItems) + i * 64u + l;
                ok[i] = j < m;
                k[i] = ok[i] ? sk[s + j] : 0u;
                v[i] = ok[i] ? sv[s + j] : 0u;
            }
            bucket_rank<kBigThreads, kBigItems>(k, ok, shift, s_wc, s_cnt, dg, r);
#pragma unroll
            for (int i = 0; i < kBigItems; ++i)
                if (ok[i]) {
                    const uint32_t o = s_run[dg[i]] + r[i];
                    dk[s + o] = k[i];
                    dv[s + o] = v[i];
                }
            __syncthreads();  // s_run and s_wc reads done
            for (uint32_t d = tid; d < kMsbBuckets; d += kBigThreads) s_run[d] += s_cnt[d];
            __syncthreads();
        }
        // this pass's stores before the next pass's loads by the block's other waves
        // (one CU, one L1: a workgroup-scope fence; __threadfence would also write
        // back the XCD's L2, ~60 us, profiles/calib_barrier_r03.log)
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __syncthreads();
        uint32_t* t0 = sk;
        sk = dk;
        dk = t0;
        t0 = sv;
        sv = dv;
        dv = t0;
    }
    for (uint32_t j = tid; j < m; j += kBigThreads) {  // the result is in kin/vin
        kout[s + j] = kin[s + j];
        vout[s + j] = vin[s + j];
    }
}

// ================================================================ tile-bucketed gather sort (r04)
// The build's MSB sort without a global prefix, a first-level scatter launch
// or any stability requirement.  K1 (k_morton_tb, build_kernels.hip) groups
// each 4096-key tile by bucket d = key >> 20 and writes it bucket by bucket,
// one word per key (key bits 0..19 << 12 | the key's index in its tile),
// with tb[tile][d] = run start | run length << 16.  k_bucket_gather then
// owns bucket d:
//   1. its runs = column d of the table, their offsets a block scan over
//      the tiles; its size = the sum of the run lengths and its start = the
//      sum of the runs' tile-local starts (no global histogram);
//   2. each run marks its first bucket position and a max-scan gives every
//      position its run, so element j is read by lane j (consecutive lanes
//      read consecutive words of one run), and decoded to (key, index);
//   3. the bucket is grouped by bin b = key bits 10..19 (LDS atomics: one
//      histogram pass, a scan, one scatter pass -- again in any order);
//   4. each element's rank in its bin is the number of bin elements whose
//      (key, index) pair is smaller: the sorted position is bin start +
//      rank, i.e. §9.4's unique (key, index) order by construction, whatever
//      order the atomics left -- so neither level needs a stable ranking;
//   5. the bin-sorted bucket is written back coalesced.
// A uniform soup's bins hold n / 2^20 keys on average, so step 4 is a short
// loop.  A block with a bin beyond kGatherHot keys (clustered geometry: the
// bunny and Sponza substitutes' 75- and 32-key bins) sorts its bucket by two
// stable 10-bit radix passes instead (gather_radix_sort, r06); only a run of
// more than kGatherBinFast identical keys (degenerate, duplicated geometry)
// flags the scene (*slow) so its later builds use the MSB sort.  A bucket beyond the block's LDS (a probe
// build's verdict normally prevents this) flags *overflow and is left
// unsorted: the host then rebuilds with the LSB sort.
// Blocks are dealt to buckets XCD by XCD (dispatch order is round-robin over
// the 8 XCDs, so block b runs on XCD b mod 8): XCD x owns buckets
// [128x, 128x + 128), i.e. one contiguous eighth of every tile's runs and of
// every table row, which its own L2 then serves to its 128 blocks.
constexpr uint32_t kGatherMaxTilesPerThread = 4;  // runs (tiles) per thread in step 1
#ifndef RT_GATHER_SKEW
#define RT_GATHER_SKEW 0  // k_bucket_dense's skew verdict: largest bucket > this x the mean (0: off)
#endif
#ifndef RT_GATHER_BIN_FAST
#define RT_GATHER_BIN_FAST 64
#endif
constexpr uint32_t kGatherBinFast = RT_GATHER_BIN_FAST;  // identical-key runs above this flag the scene as clustered
#ifndef RT_GATHER_HOT
#define RT_GATHER_HOT 16
#endif
constexpr uint32_t kGatherHot = RT_GATHER_HOT;  // a bin above this many keys: the block takes the radix path (r06)
// the radix path's shapes: P = 8 items per thread in bucket_rank's wave-major
// order, NT <= 512 (its W x 1024 counters fit next to the bucket)
constexpr bool gather_radix(int nt, int p) { return p == 8 && nt <= 512; }

// tiles (runs per bucket) the block's LDS holds: NT * 4, less for the
// 12- and 16-key-per-thread shapes, whose buckets take 96 / 128 KB (n <= 12.05M)
constexpr uint32_t gather_max_tiles(int nt, int p) { return p >= 12 ? 2944u : (uint32_t)nt * kGatherMaxTilesPerThread; }
// bin width by shape: key bits [20 - BB, 20), so a uniform soup's bins hold
// ~1-2 keys (1M: 977 keys per bucket over 1024 bins; 10M: 9766 over 4096)
constexpr int gather_bin_bits(int nt, int p) { return nt * p >= 12288 && p < 16 ? 12 : nt * p >= 4096 && p < 16 ? 11 : 10; }
// LDS words of k_bucket_gather<NT, P>: the bucket as (key, index) pairs
// (2 x NT*P; first the run marks), the bin starts and cursors (2 x (2^BB +
// 1)), the run offsets and entries (2 x tiles + 1), two [16] reduction rows
// (radix path: the bucket as keys and values, then W x 1024 counters, 1024
// digit starts and a [16] row in the same buffer)
constexpr size_t gather_lds_words(int nt, int p) {
    return (size_t)2 * nt * p + 2 * ((1u << gather_bin_bits(nt, p)) + 1) + 2 * (size_t)gather_max_tiles(nt, p) + 1 + 32;
}
constexpr size_t gather_radix_words(int nt, int p) {
    return gather_radix(nt, p) ? (size_t)2 * nt * p + (size_t)(nt / 64 + 1) * kMsbBuckets + 16 : 0;
}
constexpr size_t gather_lds_bytes(int nt, int p) {
    return (gather_lds_words(nt, p) > gather_radix_words(nt, p) ? gather_lds_words(nt, p) : gather_radix_words(nt, p)) * 4;
}

// In-place exclusive scan of a[N] in LDS by NT threads (N a multiple of NT;
// a written before a barrier); thread t owns a[t * N/NT ..].  Ends with a barrier.
template <int NT, int N>
__device__ __forceinline__ void scan_lds(uint32_t* a, uint32_t* s_sw /* [NT / 64] */) {
    constexpr int PER = N / NT;
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

// k_bucket_gather's path for a bucket with a hot bin (r06): the m (key,
// index) pairs in registers (element j = tid + i*NT) sorted by two stable
// 10-bit passes (key bits 0..9, then 10..19; bucket_rank's wave-major order),
// then each identical-key run ordered by index -- the gather left the pairs
// in atomic order, so equal keys are the only unsorted part.  O(m) plus
// O(run^2) per run; a run beyond kGatherBinFast keys (degenerate geometry)
// flags the scene (*slow) so its later builds leave the gather sort.
template <int NT, int P>
__device__ __forceinline__ void gather_radix_sort(const uint32_t (&key)[P], const uint32_t (&val)[P],
                                                            uint32_t m, uint32_t s, uint32_t* __restrict__ kout,
                                                            uint32_t* __restrict__ vout, uint32_t* __restrict__ flags,
                                                            uint32_t* s_dyn) {
    constexpr int NW = NT / 64;
    constexpr uint32_t CAP = (uint32_t)NT * P;
    uint32_t* s_rk = s_dyn;       // [CAP] keys
    uint32_t* s_rv = s_dyn + CAP;  // [CAP] indices
    uint32_t(*s_wc)[kMsbBuckets] = reinterpret_cast<uint32_t(*)[kMsbBuckets]>(s_dyn + 2 * CAP);
    uint32_t* s_cnt = s_dyn + 2 * CAP + NW * kMsbBuckets;
    uint32_t* s_sw = s_cnt + kMsbBuckets;
    const uint32_t tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const uint32_t per = __builtin_amdgcn_readfirstlane((m + NT - 1) / NT);
    uint32_t k[P], v[P], dg[P], r[P];
    bool ok[P];
#pragma unroll
    for (int i = 0; i < P; ++i) {  // pass 1's order is free: the pairs as gathered
        ok[i] = tid + (uint32_t)i * NT < m;
        k[i] = key[i];
        v[i] = val[i];
    }
    for (uint32_t shift = 0; shift < kMsbShift; shift += 10) {
        bucket_rank<NT, P>(k, ok, shift, s_wc, s_cnt, dg, r);  // (its first barrier orders the reads below)
        scan1024<NT>(s_cnt, s_sw);
#pragma unroll
        for (int i = 0; i < P; ++i)
            if (ok[i]) {
                const uint32_t p = s_cnt[dg[i]] + r[i];
                s_rk[p] = k[i];
                s_rv[p] = v[i];
            }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < P; ++i) {  // the next pass reads in ranking order
            // q < CAP for every item (per <= P): unconditional reads, all in
            // flight together (a read under `if (ok)` waited item by item)
            const uint32_t q = w * (64u * per) + (uint32_t)i * 64u + l;
            ok[i] = (uint32_t)i < per && q < m;
            k[i] = s_rk[q];
            v[i] = s_rv[q];
        }
#ifdef RT_GDIAG
        if (shift) RT_STAMP(4);  // diagnostic: both passes, then the tie loop, then the barrier
#else
        RT_STAMP(4 + shift / 10);  // diagnostic builds only
#endif
    }
    // sorted by key; each element's place in its identical-key run by index.
    // Both neighbours first (all 2P reads in flight): a lone key stays put
    bool tie[P];
    uint32_t c[P];
#pragma unroll
    for (int i = 0; i < P; ++i) {
        const uint32_t q = w * (64u * per) + (uint32_t)i * 64u + l;
        const uint32_t pv = s_rk[q ? q - 1 : 0u];
        const uint32_t nx = s_rk[q + 1 < CAP ? q + 1 : q];
        tie[i] = ok[i] && ((q > 0 && pv == k[i]) || (q + 1 < m && nx == k[i]));
        c[i] = q;
    }
    bool longrun = false;
#pragma unroll
    for (int i = 0; i < P; ++i)
        if (tie[i]) {
            const uint32_t q = c[i];
            // a run within TW positions on either side is read in one round
            // of (clamped) loads and ranked from registers; a longer run
            // takes the scans below
            constexpr int TW = 4;  // (2: Sponza -1.8 us, bunny +1.4; 4: both -1 to -1.4; profiles/gather_radix_r06.log)
            uint32_t wk[2 * TW], wv[2 * TW];
#pragma unroll
            for (int o = 0; o < 2 * TW; ++o) {
                const int off = o < TW ? o - TW : o - TW + 1;  // -TW..-1, 1..TW
                const int x = (int)q + off;
                const uint32_t xc = x < 0 ? 0u : (uint32_t)x >= m ? m - 1u : (uint32_t)x;
                wk[o] = s_rk[xc];
                wv[o] = s_rv[xc];
            }
            bool inl = true, inr = true;  // still inside the run going left / right
            uint32_t r = 0, na = 0;  // smaller indices in the run; run members left of q
#pragma unroll
            for (int o = TW - 1; o >= 0; --o) {  // left: q-1, q-2, ...
                const int x = (int)q - (TW - o);
                inl = inl && x >= 0 && wk[o] == k[i];
                na += inl ? 1u : 0u;
                r += (inl && wv[o] < v[i]) ? 1u : 0u;
            }
#pragma unroll
            for (int o = TW; o < 2 * TW; ++o) {  // right: q+1, q+2, ...
                const uint32_t x = q + (uint32_t)(o - TW + 1);
                inr = inr && x < m && wk[o] == k[i];
                r += (inr && wv[o] < v[i]) ? 1u : 0u;
            }
            if (!inl && !inr) {
                c[i] = q - na + r;
                continue;
            }
            uint32_t a = q, e = q + 1;
            while (a > 0 && s_rk[a - 1] == k[i]) --a;
            while (e < m && s_rk[e] == k[i]) ++e;
            uint32_t r2 = a;
            for (uint32_t x = a; x < e; ++x) r2 += s_rv[x] < v[i] ? 1u : 0u;
            c[i] = r2;
            longrun |= e - a > kGatherBinFast;
        }
#pragma unroll
    for (int i = 0; i < P; ++i)
        if (ok[i]) {
            const uint32_t q = w * (64u * per) + (uint32_t)i * 64u + l;
            kout[s + q] = k[i];
            vout[s + c[i]] = v[i];
        }
#ifdef RT_GDIAG
    RT_STAMP(5);
#endif
    if (__syncthreads_or(longrun) && tid == 0) atomicOr(flags, 1u);
    RT_STAMP(6);
}

template <int NT, int P>
__global__ __launch_bounds__(NT) void k_bucket_gather(const uint32_t* __restrict__ words_tb,
                                                      const uint32_t* __restrict__ tb, uint32_t nt,
                                                      uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                      uint32_t* __restrict__ flags /* [0] slow, [1] overflow */,
                                                      uint32_t* __restrict__ bstart /* [1025] bucket starts */,
                                                      Gate gate = Gate{}) {
    if (gated_off(gate)) return;
    constexpr int NW = NT / 64;
    constexpr uint32_t CAP = (uint32_t)NT * P;
    constexpr uint32_t TMAX = gather_max_tiles(NT, P);
    constexpr int BB = gather_bin_bits(NT, P);
    constexpr uint32_t NB = 1u << BB;
    constexpr uint32_t BSH = kMsbShift - BB;  // bin = key bits [BSH, 20)
    extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
    uint2* s_kv = reinterpret_cast<uint2*>(s_dyn);              // [CAP] (key, index); first the run marks
    uint32_t* s_mark = s_dyn;                                   // [CAP] run index of each bucket position
    uint32_t* s_bin = s_dyn + 2 * CAP;                          // [NB + 1] bin counts, then starts
    uint32_t* s_cur = s_bin + NB + 1;                           // [NB + 1] bin cursors
    uint32_t* s_off = s_cur + NB + 1;                           // [TMAX + 1] run offsets in the bucket
    uint32_t* s_ent = s_off + TMAX + 1;                         // [TMAX] run entries start | len << 16
    uint32_t* s_sw = s_ent + TMAX;                              // [16]
    uint32_t* s_sw2 = s_sw + 16;                                // [16]
    const uint32_t tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const uint32_t b = blockIdx.x;
    const uint32_t d = (b & 7u) * (kMsbBuckets / 8) + (b >> 3);  // XCD x: buckets [128x, 128x + 128)
    RT_STAMP(0);  // diagnostic builds only (tools/diag_gather.py)
    for (uint32_t j = tid; j <= NB; j += NT) s_bin[j] = 0u;
    // 1. this bucket's run in every tile: thread tid owns tiles [tid*K, tid*K + K).
    // The bucket's size m is the sum of its runs, and its start the sum of
    // the runs' tile-local starts (a run starts after its tile's keys of the
    // lower buckets): no global histogram is needed
    const uint32_t K = (nt + NT - 1) / NT;
    uint32_t e[kGatherMaxTilesPerThread], csum = 0, gs = 0;
#pragma unroll
    for (uint32_t k = 0; k < kGatherMaxTilesPerThread; ++k) {
        const uint32_t t = tid * K + k;
        e[k] = (k < K && t < nt) ? tb[(uint64_t)t * kMsbBuckets + d] : 0u;
        csum += e[k] >> 16;
        gs += e[k] & 0xFFFFu;
    }
    uint32_t x = csum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (l >= (uint32_t)o) x += y;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) gs += __shfl_xor(gs, o, 64);
    if (l == 63) s_sw[w] = x;
    if (l == 0) s_sw2[w] = gs;
    __syncthreads();
    uint32_t off = x - csum, s = 0, m = 0;
    for (uint32_t q = 0; q < (uint32_t)NW; ++q) {
        if (q < w) off += s_sw[q];
        s += s_sw2[q];
        m += s_sw[q];
    }
    if (tid == 0) {  // the bucket starts, for k_topo_refit's long-range nodes
        bstart[d] = s;
        if (d == kMsbBuckets - 1) bstart[kMsbBuckets] = s + m;
    }
    RT_STAMP_VAL(7, m);
    RT_STAMP(1);
    if (m == 0) return;  // block-uniform
    if (m > CAP) {       // block-uniform: beyond one LDS sort
        if (tid == 0) atomicOr(flags + 1, 1u);
        // the host discards this build (and rebuilds with the LSB sort), but
        // the stages after it still gather through this bucket's range:
        // in-range indices there, never stale or uninitialised words
        for (uint32_t j = tid; j < m; j += NT) {
            kout[s + j] = 0u;
            vout[s + j] = s + j;
        }
        return;
    }
    // 2. run index of every bucket position: each non-empty run marks its
    // first position with its tile, then an inclusive max-scan fills the
    // rest (tiles increase along the bucket); thread tid scans the
    // contiguous positions [tid*per, tid*per + per)
    const uint32_t per = (m + NT - 1) / NT;
    for (uint32_t j = tid; j < m; j += NT) s_mark[j] = 0u;
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kGatherMaxTilesPerThread; ++k) {
        const uint32_t t = tid * K + k;
        if (k < K && t < nt) {
            s_off[t] = off;
            s_ent[t] = e[k];
            if (e[k] >> 16) s_mark[off] = t;
            off += e[k] >> 16;
        }
    }
    __syncthreads();
    {
        uint32_t run = 0;
        for (uint32_t i = 0; i < per; ++i) {
            const uint32_t j = tid * per + i;
            if (j < m) run = max(run, s_mark[j]);
        }
        uint32_t y = run;  // inclusive max-scan over the threads' chunks
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t z = __shfl_up(y, o, 64);
            if (l >= (uint32_t)o) y = max(y, z);
        }
        if (l == 63) s_sw2[w] = y;
        __syncthreads();
        uint32_t carry = __shfl_up(y, 1, 64);
        carry = l ? carry : 0u;
        for (uint32_t q = 0; q < w; ++q) carry = max(carry, s_sw2[q]);
        for (uint32_t i = 0; i < per; ++i) {
            const uint32_t j = tid * per + i;
            if (j < m) {
                carry = max(carry, s_mark[j]);
                s_mark[j] = carry;
            }
        }
    }
    __syncthreads();
    RT_STAMP(2);
    // 3. gather: element j = tid + i*NT (consecutive lanes read consecutive
    // words of a run) and decode (key, index)
    uint32_t key[P], val[P], bin[P];
#pragma unroll
    for (int i = 0; i < P; ++i) {
        const uint32_t j = tid + (uint32_t)i * NT;
        if (j < m) {
            const uint32_t t = s_mark[j], en = s_ent[t];
            const uint32_t wd = words_tb[t * (uint32_t)kSortTile + (en & 0xFFFFu) + (j - s_off[t])];
            key[i] = (d << kMsbShift) | (wd >> 12);
            val[i] = t * (uint32_t)kSortTile + (wd & 0xFFFu);
            bin[i] = (key[i] >> BSH) & (NB - 1);
        }
    }
#pragma unroll
    for (int i = 0; i < P; ++i)
        if (tid + (uint32_t)i * NT < m) atomicAdd(&s_bin[bin[i]], 1u);
    __syncthreads();
    RT_STAMP(3);
    // 4. bin starts (s_bin[NB] = m) and cursors, then the bin grouping (the
    // marks are dead: s_kv takes their words).  A bin beyond kGatherHot keys
    // (clustered geometry) would make step 5 a long loop: the block sorts by
    // radix instead (block-uniform)
    {
        uint32_t mx = 0;
        for (uint32_t j = tid; j < NB; j += NT) mx = max(mx, s_bin[j]);
        if (__syncthreads_or(mx > kGatherHot)) {
            if constexpr (gather_radix(NT, P)) {
                gather_radix_sort<NT, P>(key, val, m, s, kout, vout, flags, s_dyn);
                return;
            } else if (tid == 0 && mx > kGatherBinFast) {
                atomicOr(flags, 1u);
            }
        }
    }
    scan_lds<NT, (int)NB>(s_bin, s_sw);  // ends with a barrier
    for (uint32_t j = tid; j < NB; j += NT) s_cur[j] = s_bin[j];
    if (tid == 0) s_bin[NB] = m;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < P; ++i)
        if (tid + (uint32_t)i * NT < m) s_kv[atomicAdd(&s_cur[bin[i]], 1u)] = make_uint2(key[i], val[i]);
    __syncthreads();
    RT_STAMP(4);
    // 5. rank in the bin by the (key, index) pair; item-interleaved, so the
    // thread's P bin reads of one step are in flight together
    uint32_t pos[P], len[P], kmax = 0;
#pragma unroll
    for (int i = 0; i < P; ++i) {
        pos[i] = 0;
        len[i] = 0;
        if (tid + (uint32_t)i * NT < m) {
            pos[i] = s_bin[bin[i]];
            len[i] = s_bin[bin[i] + 1] - pos[i];
            kmax = max(kmax, len[i]);
        }
    }
    uint32_t r[P];
#pragma unroll
    for (int i = 0; i < P; ++i) r[i] = 0;
    for (uint32_t k = 0; k < kmax; ++k) {
        if constexpr (NT <= 512) {
            // rows i < per (scalar branch), clamped reads in every lane: a
            // step's reads in flight together (r06; the 10M shapes' 10-16 rows
            // of ~2-key bins keep the exact reads, whose LDS traffic is lower)
            const uint32_t perU = __builtin_amdgcn_readfirstlane(per);
#pragma unroll
            for (int i = 0; i < P; ++i)
                if ((uint32_t)i < perU) {
                    const uint32_t x = pos[i] + k;
                    const uint2 o = s_kv[x < CAP ? x : CAP - 1u];
                    r[i] += (k < len[i] && (o.x < key[i] || (o.x == key[i] && o.y < val[i]))) ? 1u : 0u;
                }
        } else {
#pragma unroll
            for (int i = 0; i < P; ++i)
                if (k < len[i]) {
                    const uint2 o = s_kv[pos[i] + k];
                    r[i] += (o.x < key[i] || (o.x == key[i] && o.y < val[i])) ? 1u : 0u;
                }
        }
    }
#pragma unroll
    for (int i = 0; i < P; ++i) pos[i] += r[i];
    __syncthreads();  // every bin read
    RT_STAMP(5);
#pragma unroll
    for (int i = 0; i < P; ++i)
        if (tid + (uint32_t)i * NT < m) s_kv[pos[i]] = make_uint2(key[i], val[i]);
    __syncthreads();
    // 6. the sorted bucket, coalesced
    for (uint32_t j = tid; j < m; j += NT) {
        const uint2 o = s_kv[j];
        kout[s + j] = o.x;
        vout[s + j] = o.y;
    }
    RT_STAMP(6);
}

// A probe build's verdict for the gather sort: 1 when some bucket holds more
// than cap keys (the LSB sort then runs), else 0.
// dense[0]: a bucket beyond the gather block's LDS (the LSB leg runs);
// dense[3]: skewed -- the largest bucket holds more than 4x the mean (and
// over 256 keys), so one block sorts it while the others idle: the host
// moves the scene to the MSB sort (BuildBufs::gather_off), which spreads it
__global__ __launch_bounds__(1024) void k_bucket_dense(const uint32_t* __restrict__ ghist, uint32_t cap, uint32_t n,
                                                       uint32_t* __restrict__ dense) {
    __shared__ uint32_t s_max;
    if (threadIdx.x == 0) s_max = 0u;
    const uint32_t v = ghist[threadIdx.x];
    const int big = __syncthreads_or(v > cap);  // (also orders s_max's init)
    atomicMax(&s_max, v);
    __syncthreads();
    if (threadIdx.x == 0) {
        dense[0] = big ? 1u : 0u;
        dense[3] = RT_GATHER_SKEW && !big && s_max > 256u && (uint64_t)s_max * kMsbBuckets > (uint64_t)RT_GATHER_SKEW * n ? 1u : 0u;
    }
}

// ================================================================ launchers
static inline uint32_t sdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

uint32_t sort_tiles(uint32_t n) { return n ? sdiv(n, kSortTile) : 0u; }

static hipError_t digit_hist(const uint32_t* keys, uint32_t n, uint32_t* ghist, hipStream_t s, Gate g = Gate{}) {
    if (!n) return hipSuccess;
    RT_KLAUNCH(k_digit_hist, dim3(std::min<uint32_t>(512, sdiv(n, 256))), dim3(256), 0, s, keys, n, ghist, g);
    return hipGetLastError();
}

static hipError_t tile_hist0(const uint32_t* keys, uint32_t n, uint32_t* counts, hipStream_t s, Gate g = Gate{}) {
    if (!n) return hipSuccess;
    RT_KLAUNCH(k_tile_hist<0>, dim3(sort_tiles(n)), dim3(kSortThreads), 0, s, keys, n, counts, g);
    return hipGetLastError();
}

hipError_t launch_digit_hist(const uint32_t* keys, uint32_t n, uint32_t* ghist, hipStream_t s) {
    return digit_hist(keys, n, ghist, s);
}

hipError_t launch_tile_hist0(const uint32_t* keys, uint32_t n, uint32_t* counts, hipStream_t s) {
    return tile_hist0(keys, n, counts, s);
}

template <int SHIFT>
static void scatter_pass(const uint32_t* ki, const uint32_t* vi, uint32_t* ko, uint32_t* vo, uint32_t n,
                         const uint32_t* gh, uint32_t* counts, hipStream_t s, Gate g = Gate{}) {
    const uint32_t nt = sort_tiles(n);
    if (nt <= kPrefixInKernelMaxTiles) {
        RT_KLAUNCH((k_scatter<SHIFT, true>), dim3(nt), dim3(kSortThreads), 0, s, ki, vi, ko, vo, n, gh, counts, g);
    } else {
        RT_KLAUNCH(k_scan_tiles, dim3(256), dim3(256), 0, s, counts, nt, g);
        RT_KLAUNCH((k_scatter<SHIFT, false>), dim3(nt), dim3(kSortThreads), 0, s, ki, vi, ko, vo, n, gh, counts, g);
    }
}

static hipError_t sort_lsb(uint32_t* keys[2], uint32_t* vals[2], uint32_t n, const uint32_t* ghist,
                           uint32_t* counts[4], hipStream_t s, Gate g = Gate{}) {
    if (n <= 1) return hipSuccess;
    const uint32_t nt = sort_tiles(n);
    scatter_pass<0>(keys[0], vals[0], keys[1], vals[1], n, ghist + 0, counts[0], s, g);
    RT_KLAUNCH(k_tile_hist<8>, dim3(nt), dim3(kSortThreads), 0, s, keys[1], n, counts[1], g);
    scatter_pass<8>(keys[1], vals[1], keys[0], vals[0], n, ghist + 256, counts[1], s, g);
    RT_KLAUNCH(k_tile_hist<16>, dim3(nt), dim3(kSortThreads), 0, s, keys[0], n, counts[2], g);
    scatter_pass<16>(keys[0], vals[0], keys[1], vals[1], n, ghist + 512, counts[2], s, g);
    RT_KLAUNCH(k_tile_hist<24>, dim3(nt), dim3(kSortThreads), 0, s, keys[1], n, counts[3], g);
    scatter_pass<24>(keys[1], vals[1], keys[0], vals[0], n, ghist + 768, counts[3], s, g);
    return hipGetLastError();
}

// 4 passes, ping-pong 0->1->0->1->0.  Needs: ghist [4][256] (all digits) and
// counts0 = pass-0 tile counts; counts[1..3] are scratch of ntiles*256 words.
hipError_t launch_sort(uint32_t* keys[2], uint32_t* vals[2], uint32_t n, const uint32_t* ghist, uint32_t* counts[4],
                       hipStream_t s) {
    return sort_lsb(keys, vals, n, ghist, counts, s);
}

static hipError_t ensure_big_attr() {
    static std::once_flag once;
    static hipError_t err = hipSuccess;
    std::call_once(once, [] {
        err = hipFuncSetAttribute(reinterpret_cast<const void*>(k_bucket_sort_big),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBigLds);
        if (err == hipSuccess)
            err = hipFuncSetAttribute(reinterpret_cast<const void*>(k_msb_scatter_big),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)kScatterBigLds);
    });
    return err;
}

hipError_t launch_sort_msb(uint32_t* keys[2], uint32_t* vals[2], uint32_t n, const uint32_t* ghist, uint32_t* counts,
                           uint32_t* bstart, uint32_t* scratch, hipStream_t s, uint32_t* dense) {
    if (n <= 1) return hipSuccess;
    const uint32_t nt = sort_tiles(n);
    if (n > kMsbBigMaxN) return hipErrorInvalidValue;
    const uint32_t cap = msb_bucket_cap(n);
    const Gate g{dense, 0u};  // with dense: the MSB kernels run only when no bucket outgrew cap
    if (n <= kMsbMaxN) {
        RT_KLAUNCH(k_msb_scan, dim3(kMsbBuckets / 64), dim3(1024), 0, s, counts, nt, ghist, bstart, cap, dense);
    } else {
        if (!scratch) return hipErrorInvalidValue;
        const uint32_t nch = sdiv(nt, kMsbChunk);
        RT_KLAUNCH(k_msb_chunk_sum, dim3(nch), dim3(1024), 0, s, counts, nt, scratch);
        // the chunk sums' exclusive scan from the bucket starts is k_msb_scan's
        // job on a [chunk][1024] table (nch <= 512: n <= 67M)
        RT_KLAUNCH(k_msb_scan, dim3(kMsbBuckets / 64), dim3(1024), 0, s, scratch, nch, ghist, bstart, cap, dense);
        RT_KLAUNCH(k_msb_chunk_apply, dim3(nch), dim3(1024), 0, s, counts, nt, scratch);
    }
    if (n <= kMsbMaxN) {
        RT_KLAUNCH(k_msb_scatter, dim3(nt), dim3(kMsbScatterNT), 0, s, keys[0], vals[0], keys[1], vals[1], n, counts,
                   g);
        RT_KLAUNCH(k_bucket_sort, dim3(kMsbBuckets), dim3(kBucketThreads), 0, s, keys[1], vals[1], keys[0], vals[0],
                   bstart, g);
    } else {
        const hipError_t e = ensure_big_attr();
        if (e != hipSuccess) return e;
        RT_KLAUNCH(k_msb_scatter_big, dim3(sdiv(n, kScatterBigTile)), dim3(1024), kScatterBigLds, s, keys[0], vals[0],
                   keys[1], vals[1], n, counts, g);
        RT_KLAUNCH(k_bucket_sort_big, dim3(kMsbBuckets), dim3(kBigThreads), kBigLds, s, keys[1], vals[1], keys[0],
                   vals[0], bstart, g);
    }
    return hipGetLastError();
}

hipError_t launch_sort_probe(uint32_t* keys[2], uint32_t* vals[2], uint32_t n, const uint32_t* ghist,
                             uint32_t* counts, uint32_t* bstart, uint32_t* scratch, uint32_t* ghist4,
                             uint32_t* dense, hipStream_t s) {
    if (n <= 1) return hipSuccess;
    hipError_t e = launch_sort_msb(keys, vals, n, ghist, counts, bstart, scratch, s, dense);
    if (e != hipSuccess) return e;
    // dense: keys[0]/vals[0] are still K1's; the MSB counts are spent, so the
    // LSB passes reuse their words ([4][tile][256] = [tile][1024])
    const Gate g{dense, 1u};
    const uint64_t cs = (uint64_t)sort_tiles(n) * 256;
    uint32_t* c4[4] = {counts, counts + cs, counts + 2 * cs, counts + 3 * cs};
    if ((e = digit_hist(keys[0], n, ghist4, s, g)) != hipSuccess) return e;
    if ((e = tile_hist0(keys[0], n, c4[0], s, g)) != hipSuccess) return e;
    return sort_lsb(keys, vals, n, ghist4, c4, s, g);
}

// ---- the gather sort's launchers.  Block shape by n: the smallest bucket
// block whose LDS holds a uniform soup's n/1024 keys with a wide margin
// (mean + 16 sigma + 64), so a uniform scene never overflows one (ADVICE r03:
// a fixed 2048-key cap up to 2^21 sent uniform 2M soups to the LSB sort for
// good).
struct GatherShape { int nt, p; };
static GatherShape gather_shape(uint32_t n) {
    const double mean = (double)n / kMsbBuckets;
    const double need = mean + 16.0 * std::sqrt(mean) + 64.0;
#ifndef RT_GATHER_SMALL_NT
#define RT_GATHER_SMALL_NT 256  // the n <= ~1.9M shape: 256 x 8 keys (512 x 4 measured in r04)
#endif
    if (need <= 256 * 8) return {RT_GATHER_SMALL_NT, 2048 / RT_GATHER_SMALL_NT};
    if (need <= 512 * 8) return {512, 8};
    if (need <= 1024 * 12) return {1024, 12};
    return {1024, 16};
}
uint32_t gather_bucket_cap(uint32_t n) {
    const GatherShape g = gather_shape(n);
    return (uint32_t)(g.nt * g.p);
}
bool gather_sort_fits(uint32_t n) {  // every run of a bucket in its block's LDS
    const GatherShape g = gather_shape(n);
    return n >= 2 && sort_tiles(n) <= gather_max_tiles(g.nt, g.p);
}

template <int NT, int P>
static hipError_t gather_launch(const uint32_t* words, const uint32_t* tb, uint32_t nt, uint32_t* ko, uint32_t* vo,
                                uint32_t* flags, uint32_t* bstart, hipStream_t s, Gate g) {
    static std::once_flag once[kMaxDevices];
    static hipError_t err[kMaxDevices];
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
    constexpr size_t lds = gather_lds_bytes(NT, P);
    static_assert(lds <= 160 * 1024, "one block's LDS");
    std::call_once(once[dev], [dev] {
        err[dev] = hipFuncSetAttribute(reinterpret_cast<const void*>(k_bucket_gather<NT, P>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    });
    if (err[dev] != hipSuccess) return err[dev];
    RT_KLAUNCH((k_bucket_gather<NT, P>), dim3(kMsbBuckets), dim3(NT), lds, s, words, tb, nt, ko, vo, flags, bstart, g);
    return hipGetLastError();
}

hipError_t launch_sort_gather(const uint32_t* words, const uint32_t* tb, uint32_t n, const uint32_t* ghist,
                              uint32_t* kout, uint32_t* vout, uint32_t* flags, uint32_t* bstart, uint32_t* dense,
                              hipStream_t s) {
    if (n <= 1) return hipSuccess;
    if (!gather_sort_fits(n)) return hipErrorInvalidValue;
    const uint32_t nt = sort_tiles(n);
    const GatherShape gs = gather_shape(n);
    if (dense) RT_KLAUNCH(k_bucket_dense, dim3(1), dim3(kMsbBuckets), 0, s, ghist, (uint32_t)(gs.nt * gs.p), n, dense);
    const Gate g{dense, 0u};
    if (gs.nt * gs.p == 2048 && gs.nt == 256) return gather_launch<256, 8>(words, tb, nt, kout, vout, flags, bstart, s, g);
#if RT_GATHER_SMALL_NT == 512
    if (gs.nt * gs.p == 2048) return gather_launch<512, 4>(words, tb, nt, kout, vout, flags, bstart, s, g);
#endif
    if (gs.nt == 512) return gather_launch<512, 8>(words, tb, nt, kout, vout, flags, bstart, s, g);
    if (gs.p == 12) return gather_launch<1024, 12>(words, tb, nt, kout, vout, flags, bstart, s, g);
    return gather_launch<1024, 16>(words, tb, nt, kout, vout, flags, bstart, s, g);
}

// The probe build's LSB leg when the verdict is dense (*dense == 1): K1 again
// in index order (k_morton<false>: the keys, their 4 digit histograms and
// pass 0's tile counts) and the 4-pass LSB sort, every launch gated.
hipError_t launch_sort_lsb_gated(uint32_t* keys[2], uint32_t* vals[2], uint32_t n, const uint32_t* ghist4,
                                 uint32_t* counts, const uint32_t* dense, hipStream_t s) {
    if (n <= 1) return hipSuccess;
    const uint64_t cs = (uint64_t)sort_tiles(n) * 256;
    uint32_t* c4[4] = {counts, counts + cs, counts + 2 * cs, counts + 3 * cs};
    return sort_lsb(keys, vals, n, ghist4, c4, s, Gate{dense, 1u});
}

hipError_t launch_sort_top(uint32_t* keys[2], uint32_t* vals[2], uint32_t n, const uint32_t* ghist, uint32_t* counts,
                           uint32_t digits, uint32_t* out_buf, hipStream_t s) {
    *out_buf = 0;
    if (n <= 1 || !digits) return hipSuccess;
    if (digits > 4) digits = 4;
    const uint32_t nt = sort_tiles(n);
    uint32_t src = 0;
    for (uint32_t dgt = 4 - digits; dgt < 4; ++dgt, src ^= 1u) {
        const uint32_t dst = src ^ 1u;
        switch (dgt) {
#define RT_SORT_PASS(SH)                                                                                            \
    RT_KLAUNCH(k_tile_hist<SH>, dim3(nt), dim3(kSortThreads), 0, s, keys[src], n, counts);                 \
    scatter_pass<SH>(keys[src], vals[src], keys[dst], vals[dst], n, ghist + 256 * (SH / 8), counts, s);          \
    break
            case 0: RT_SORT_PASS(0);
            case 1: RT_SORT_PASS(8);
            case 2: RT_SORT_PASS(16);
            default: RT_SORT_PASS(24);
#undef RT_SORT_PASS
        }
    }
    *out_buf = src;
    return hipGetLastError();
}

}  // namespace rt

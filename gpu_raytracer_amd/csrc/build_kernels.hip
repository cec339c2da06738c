// build_kernels.hip -- BVH build hot path for gfx950.
//
//   K0 k_bounds         centroid bounds: 8 AoS triangles per thread as 18
//                       independent 16-B loads, wave/LDS min-max -> one
//                       partial box per block (the second level runs inside
//                       every K1 block -> BuildParams {lo, hi, inv}).  Also
//                       zeroes the per-build control words (digit
//                       histograms, crossing counters).
//   K1 k_morton         Morton codes (§9.3); one block = one 4096-key sort tile,
//                       so it also writes the tile's pass-0 digit counts and
//                       adds the 4 global digit histograms (sort_kernels.hip).
//   K2/K3               radix sort, sort_kernels.hip.
//   K4 k_karras_leaves  Karras 2012 topology (§9.5) + closed-form escape links
//                       (§9.6) + parent pointers for internal node i, and, in the
//                       same thread, leaf i: gather of its triangle (independent
//                       loads that overlap the binary-search latency), leaf node
//                       {AABB, prim, esc} and the leaf-ordered {v0,e1,e2} record
//                       the trace kernel reads.
//   K6 k_refit_local    per 1024-leaf block: bottom-up refit of every internal
//                       node whose leaf range lies in the block, in LDS only
//                       (LDS arrival counters), plus block prefix/suffix/total
//                       AABBs for the crossing nodes.
//   K6 k_refit_cross    nodes whose range crosses a block boundary:
//                       union(suffix, middle blocks, prefix) -- exact min/max,
//                       so the result is independent of evaluation order.
#include "rt_device.h"
#include "rt_launch.h"
#include "sort_device.h"

#include <mutex>

#include <algorithm>

namespace rt {

#ifdef RT_STAMPS
hipError_t read_stamps_build(void* out, size_t bytes) { return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rt_stamps), bytes); }
#endif

// ---------------------------------------------------------------- helpers
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

// 8 triangles per thread, lane-interleaved: lane l of a wave whose span
// starts at triangle `base` takes triangles base + 64q + l (q < 8), each as
// three 12-B vertex loads.  Lanes are 36 B apart, so one wave-instruction
// covers 2304 contiguous bytes (18 lines) and the wave's 24 instructions read
// its 18-KB span with no LDS.  The r02 form (8 consecutive triangles per
// thread as 18 x 16-B loads) put lanes 288 B apart -- 64 lines per
// instruction -- and streamed at 3.8 TB/s against 6.1 TB/s for this one
// (tools/bench_stream.hip, profiles/bench_stream_r03.log).
// All index math is 32-bit (n <= 2^30): a 64-bit min() of the tail size was
// miscompiled by hipcc 7.2 (v_cmp_*_u64 feeding an s_cselect on a stale SCC).
constexpr uint32_t kTrisPerThread = 8;
struct Vtx { float x, y, z; };

// t[q] = triangle base + 64q + lane (zeros past n); returns the valid mask
__device__ __forceinline__ uint32_t load_tri_lanes(const float* __restrict__ tris, uint32_t n, uint32_t base,
                                                   float (&t)[kTrisPerThread][9]) {
    const uint32_t lane = threadIdx.x & 63;
    const Vtx* p = reinterpret_cast<const Vtx*>(tris);
    uint32_t mask = 0;
#pragma unroll
    for (uint32_t q = 0; q < kTrisPerThread; ++q) {
        const uint32_t k = base + q * 64u + lane;
        const bool ok = k < n;
        mask |= (ok ? 1u : 0u) << q;
#pragma unroll
        for (uint32_t j = 0; j < 3; ++j) {
            const Vtx v = ok ? p[(uint64_t)k * 3 + j] : Vtx{0.0f, 0.0f, 0.0f};
            t[q][3 * j] = v.x;
            t[q][3 * j + 1] = v.y;
            t[q][3 * j + 2] = v.z;
        }
    }
    return mask;
}

// the same for triangles q0 .. q0 + Q - 1 of the lane's 8 (t[q - q0])
template <uint32_t Q>
__device__ __forceinline__ uint32_t load_tri_lanes_part(const float* __restrict__ tris, uint32_t n, uint32_t base,
                                                        uint32_t q0, float (&t)[Q][9]) {
    const uint32_t lane = threadIdx.x & 63;
    const Vtx* p = reinterpret_cast<const Vtx*>(tris);
    uint32_t mask = 0;
#pragma unroll
    for (uint32_t q = 0; q < Q; ++q) {
        const uint32_t k = base + (q0 + q) * 64u + lane;
        const bool ok = k < n;
        mask |= (ok ? 1u : 0u) << (q0 + q);
#pragma unroll
        for (uint32_t j = 0; j < 3; ++j) {
            const Vtx v = ok ? p[(uint64_t)k * 3 + j] : Vtx{0.0f, 0.0f, 0.0f};
            t[q][3 * j] = v.x;
            t[q][3 * j + 1] = v.y;
            t[q][3 * j + 2] = v.z;
        }
    }
    return mask;
}

// ---------------------------------------------------------------- K0
#ifndef RT_K0_WAVES
#define RT_K0_WAVES 1  // min waves per SIMD K0 is compiled for (1: the compiler's choice, 84 VGPRs / 5)
#endif
#ifndef RT_K0_HALVES
#define RT_K0_HALVES 0  // 1: 4 + 4 triangles per lane (47 VGPRs, 8 waves): no faster at 10M (r04)
#endif
__global__ __launch_bounds__(256, RT_K0_WAVES) void k_bounds(const float* __restrict__ tris, uint32_t n,
                                                float* __restrict__ partials,
                                                uint32_t* __restrict__ zero_words, uint32_t nzero) {
    __shared__ float red[4][6];
    for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < nzero; j += gridDim.x * 256u) zero_words[j] = 0u;

    float lo[3], hi[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) { lo[c] = __builtin_inff(); hi[c] = -__builtin_inff(); }
    {
        // RT_K0_HALVES: the lane's 8 triangles in batches of QB (36 instead of
        // 72 triangle registers at QB = 4), for more resident waves
        constexpr uint32_t QB = RT_K0_HALVES ? kTrisPerThread / 2 : kTrisPerThread;
        const uint32_t base = (blockIdx.x * 4u + (threadIdx.x >> 6)) * 64u * kTrisPerThread;
#pragma unroll
        for (uint32_t h = 0; h < kTrisPerThread / QB; ++h) {
            float t[QB][9];
            const uint32_t ok = load_tri_lanes_part<QB>(tris, n, base, h * QB, t);
#pragma unroll
            for (uint32_t qi = 0; qi < QB; ++qi) {
                if ((ok >> (h * QB + qi)) & 1u) {
                    float bmin[3], bmax[3];
                    tri_bounds(t[qi], bmin, bmax);
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        const float cc = (bmin[c] + bmax[c]) * 0.5f;
                        lo[c] = fminf(lo[c], cc);
                        hi[c] = fmaxf(hi[c], cc);
                    }
                }
            }
        }
    }
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
    for (int c = 0; c < 3; ++c) { lo[c] = wave_min(lo[c]); hi[c] = wave_max(hi[c]); }
    if (l == 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) { red[w][c] = lo[c]; red[w][3 + c] = hi[c]; }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int c = threadIdx.x;
        partials[blockIdx.x * 6 + c] = c < 3 ? fminf(fminf(red[0][c], red[1][c]), fminf(red[2][c], red[3][c]))
                                             : fmaxf(fmaxf(red[0][c], red[1][c]), fmaxf(red[2][c], red[3][c]));
    }
}

// Second level of K0, run by every block of its consumer (K1) instead of a
// last-block ticket: the nb partial boxes (a few KB, L2-resident) reduced by
// the whole block -- exact min/max, so every block gets the same result --
// then §9.2 inv.  No device-scope fence or atomic on the critical path.
template <int NT>
__device__ __forceinline__ BuildParams bounds_final(const float* __restrict__ partials, uint32_t nb, float (*red)[6]) {
    float lo[3], hi[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) { lo[c] = __builtin_inff(); hi[c] = -__builtin_inff(); }
    for (uint32_t b = threadIdx.x; b < nb; b += NT) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            lo[c] = fminf(lo[c], partials[b * 6 + c]);
            hi[c] = fmaxf(hi[c], partials[b * 6 + 3 + c]);
        }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) { lo[c] = wave_min(lo[c]); hi[c] = wave_max(hi[c]); }
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) { red[w][c] = lo[c]; red[w][3 + c] = hi[c]; }
    }
    __syncthreads();
    BuildParams p;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float a = red[0][c], b = red[0][3 + c];
#pragma unroll
        for (int k = 1; k < NT / 64; ++k) { a = fminf(a, red[k][c]); b = fmaxf(b, red[k][3 + c]); }
        p.lo[c] = a;
        p.hi[c] = b;
        // §9.2: inv = (hi>lo) ? 1/(hi-lo) : 0 -- correctly rounded fp32 division
        p.inv[c] = (b > a) ? 1.0f / (b - a) : 0.0f;
    }
#pragma unroll
    for (int c = 0; c < 7; ++c) p.pad[c] = 0u;
    return p;
}

// stage entry point (rt_stage_bounds): the second level on its own
__global__ __launch_bounds__(256) void k_bounds_final(const float* __restrict__ partials, uint32_t nb,
                                                      BuildParams* __restrict__ params) {
    __shared__ float red[4][6];
    const BuildParams p = bounds_final<256>(partials, nb, red);
    if (threadIdx.x == 0) *params = p;
}

// ---------------------------------------------------------------- K1
__device__ __forceinline__ uint32_t quant(float c, float lo, float inv) {
    const float x = ((c - lo) * inv) * 1024.0f;
    return (uint32_t)fminf(fmaxf(x, 0.0f), 1023.0f);
}

// one block = one radix-sort tile: kSortThreads x kTrisPerThread = 4096 prims
static_assert(kSortThreads * kTrisPerThread == kSortTile, "K1 block must be one sort tile");

// MSB: the histograms are of the bucket digit key >> kMsbShift ([tile][1024]
// counts + [1024] totals, for launch_sort_msb) instead of the four bytes.
template <bool MSB>
__global__ __launch_bounds__(kSortThreads) void k_morton(const float* __restrict__ tris, uint32_t n,
                                                         BuildParams* __restrict__ params,
                                                         const float* __restrict__ partials, uint32_t nb,
                                                         uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                         uint32_t* __restrict__ ghist /* [4][256] */,
                                                         uint32_t* __restrict__ counts0 /* [tile][256] */,
                                                         uint32_t vbase = 0 /* vals = vbase + index */,
                                                         Gate gate = Gate{}) {
    if (gated_off(gate)) return;
    __shared__ uint32_t hist[4 * 256];
    __shared__ float red[kSortThreads / 64][6];
    for (uint32_t j = threadIdx.x; j < 1024; j += kSortThreads) hist[j] = 0u;
    // wave w of the tile: triangles tile*4096 + 512w + 64q + lane
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wbase = blockIdx.x * (uint32_t)kSortTile + (threadIdx.x >> 6) * 64u * kTrisPerThread;
    float t[kTrisPerThread][9];
    const uint32_t ok = load_tri_lanes(tris, n, wbase, t);  // in flight while the bounds are reduced
    BuildParams p;
    if (partials) {
        p = bounds_final<kSortThreads>(partials, nb, red);
        if (blockIdx.x == 0 && threadIdx.x == 0) *params = p;  // for the later stages / readback
    } else {
        p = *params;
    }
    uint32_t k8[kTrisPerThread];
#pragma unroll
    for (uint32_t q = 0; q < kTrisPerThread; ++q) {
        float bmin[3], bmax[3];
        tri_bounds(t[q], bmin, bmax);
        uint32_t qq[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) qq[c] = quant((bmin[c] + bmax[c]) * 0.5f, p.lo[c], p.inv[c]);
        k8[q] = expand10(qq[0]) * 4u + expand10(qq[1]) * 2u + expand10(qq[2]);
    }
#pragma unroll
    for (uint32_t q = 0; q < kTrisPerThread; ++q)  // 256 contiguous bytes per wave-instruction
        if ((ok >> q) & 1u) {
            const uint32_t k = wbase + q * 64u + lane;
            keys[k] = k8[q];
            vals[k] = vbase + k;
        }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kTrisPerThread; ++q)
        if ((ok >> q) & 1u) {
            if (MSB) {
                atomicAdd(&hist[k8[q] >> kMsbShift], 1u);  // 30-bit keys: < 1024
            } else {
#pragma unroll
                for (int d = 0; d < 4; ++d) atomicAdd(&hist[d * 256 + ((k8[q] >> (8 * d)) & 0xFFu)], 1u);
            }
        }
    __syncthreads();
    if (MSB) {
        for (uint32_t j = threadIdx.x; j < kMsbBuckets; j += kSortThreads)
            counts0[(uint64_t)blockIdx.x * kMsbBuckets + j] = hist[j];
    } else if (threadIdx.x < 256) {
        counts0[(uint64_t)blockIdx.x * 256 + threadIdx.x] = hist[threadIdx.x];
    }
    for (uint32_t j = threadIdx.x; j < 1024; j += kSortThreads) {
        const uint32_t v = hist[j];
        if (v) atomicAdd(&ghist[j], v);
    }
}

// A grid-wide barrier of co-resident blocks (the fused K0 + K1 below; the
// pattern of tools/calib_barrier.hip, 2.4 us on MI355X): the data handed over
// is stored with agent-scope relaxed atomic stores (write-through, no L2
// writeback), the block drains them (workgroup release = s_waitcnt) and
// arrives on one agent-scope counter, and readers use agent-scope atomic
// loads.  The counter holds generation << 16 | arrivals, so it resets itself
// for the next build: the last arrival bumps the generation and zeroes the
// count, the others wait for the generation to change.  A wait gives up
// after ~100 ms (s_memrealtime) and sets *err -- a grid that is not
// co-resident must not hang the GPU (the host reads *err after the build).
// It is split for a last-arriver step: grid_arrive_last counts the block in
// and tells it (block-uniform) whether it is the last; the last block does
// its step and then grid_open bumps the generation (and resets the count);
// the others grid_wait for that.  The arrival's old value stays in LDS for
// grid_wait.
// Publication order: a workgroup-scope release emits no vmcnt
// wait outside tgsplit mode, so the write-through stores a wave has handed
// over could still be in flight when thread 0's arrival (or the opening
// RMW) reaches L2 -- the last arriver on another XCD would then reduce a
// stale partial box.  Every wave therefore drains its own vector memory
// counter (s_waitcnt vmcnt(0): on gfx9 stores count there too, and a
// write-through store is acknowledged once it is visible device-wide) before
// the block's s_barrier; thread 0's RMW follows that barrier.  An agent-scope
// release RMW would also write back the XCD's whole L2 (buffer_wbl2), which
// is what made the fenced barrier cost ~59 us.  tests/test_isa.py checks the
// emitted order in librtamd.so.
__device__ __forceinline__ void drain_vm_stores() {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // gfx9 encoding: vmcnt(0), expcnt/lgkmcnt untouched (max)
}
__device__ __forceinline__ uint32_t* grid_old_slot() {
    __shared__ uint32_t s_old;
    return &s_old;
}
__device__ __forceinline__ bool grid_arrive_last(uint32_t* bar, uint32_t nblocks) {
    uint32_t* s_old = grid_old_slot();
    drain_vm_stores();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (threadIdx.x == 0) *s_old = __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    return (*s_old & 0xFFFFu) == nblocks - 1;
}
__device__ __forceinline__ void grid_open(uint32_t* bar, uint32_t nblocks) {
    drain_vm_stores();  // the published box is acknowledged before the generation moves
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(bar, 0x10000u - nblocks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void grid_wait(uint32_t* bar, uint32_t* err) {
    const uint32_t old = *grid_old_slot();
    if (threadIdx.x == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while ((__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 16) == (old >> 16)) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 10000000ull) {
                __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
}


// K1 + the first level of the gather sort (r04, sort_kernels.hip "tile-bucketed
// gather sort"): the block's 4096 Morton keys are also grouped by bucket
// d = key >> 20 inside the tile (LDS atomics: the order inside a bucket is
// free, since the second level orders by the whole (key, index) pair) and
// written bucket by bucket as ONE word per key, key bits 0..19 << 12 | the
// key's index inside the tile (the bucket is the run's, the tile the
// table row's), with tb[tile][d] = run start | run length << 16 (the
// bucket's total and start are sums over the table's column); ghist
// (nullable: a scene's first build only, for its verdict) gets the global
// bucket totals.  No global prefix over tiles exists:
// each bucket's block gathers its runs from every tile.
// FUSED (the grid must be co-resident, launch_build
// checks): K0 in the same launch -- the block's triangles, loaded once, give
// its partial centroid box (published for the grid barrier) and then its
// keys; the zero words K0 clears are cleared here before the barrier.  One
// soup read and one launch instead of two.
struct FuseArgs {
    uint32_t* zero = nullptr;  // per-build control words (K0's)
    uint32_t nzero = 0;
    uint32_t* bar = nullptr;   // grid barrier counter (never zeroed: self-resetting)
    uint32_t* err = nullptr;   // set on a barrier timeout
    float* box = nullptr;      // [6] the global centroid box, from the barrier's last block
};
static_assert(kSortTile <= 4096, "tile-local indices are 12 bits");
#ifndef RT_K1_REVERSE
#define RT_K1_REVERSE 1
#endif
#ifndef RT_K1_AGG
#define RT_K1_AGG 1  // r06: wave-aggregated bucket atomics for the first lane's bucket (clustered tiles)
#endif
#ifndef RT_K1TB_HALVES
#define RT_K1TB_HALVES 1  // 10M: K1 157 -> 126 us (66 instead of 106 VGPRs); 1M (fused) unchanged
#endif
// NT threads per 4096-key tile (NT x kSortTile / NT triangles; the block shape
// is RT_K1F_NT / RT_K1U_NT below)
#ifndef RT_K1U_WAVES
#define RT_K1U_WAVES 8  // the unfused K1-TB at 8 waves per SIMD (62 VGPRs, no spills): 10M K1 80 -> 76 us (r04)
#endif
template <bool FUSED, int NT = kSortThreads>
__global__ __launch_bounds__(NT, FUSED ? 1 : RT_K1U_WAVES) void k_morton_tb(const float* __restrict__ tris, uint32_t n,
                                                            BuildParams* __restrict__ params,
                                                            float* __restrict__ partials, uint32_t nb,
                                                            uint32_t* __restrict__ words_tb,
                                                            uint32_t* __restrict__ ghist /* [1024] */,
                                                            uint32_t* __restrict__ tb /* [tile][1024] */,
                                                            FuseArgs fu = FuseArgs{}) {
    constexpr int W = NT / 64;
    constexpr uint32_t TPT = kSortTile / NT;  // triangles per thread
    static_assert(TPT * NT == kSortTile && TPT <= 32 && (TPT % 2) == 0, "tile shape");
    __shared__ uint32_t s_word[kSortTile];  // the bucketed tile
    __shared__ __attribute__((aligned(16))) uint32_t s_start[kMsbBuckets];
    __shared__ float red[W][6];
    __shared__ uint32_t s_sw[W];
    for (uint32_t j = threadIdx.x; j < kMsbBuckets; j += NT) s_start[j] = 0u;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // the unfused kernel walks the tiles from the soup's end: K0 has just
    // streamed the soup front to back, so its last ~256 MB are what the
    // Infinity Cache still holds (the 10M soup is 360 MB)
    const uint32_t tile = (FUSED || !RT_K1_REVERSE) ? blockIdx.x : gridDim.x - 1 - blockIdx.x;
    const uint32_t tbase = tile * (uint32_t)kSortTile;
    const uint32_t wbase = tbase + w * 64u * TPT;
    // HALVES (the unfused kernel): the lane's 8 triangles in two batches of 4,
    // so it holds 36 instead of 72 triangle registers -- more resident blocks
    // per CU to overlap one block's LDS phases with the others' loads
    constexpr bool HALVES = !FUSED && RT_K1TB_HALVES;
    constexpr uint32_t QL = HALVES ? TPT / 2 : TPT;
    float t[QL][9];
    if (FUSED) RT_STAMP_HI(0);
    uint32_t okm = load_tri_lanes_part<QL>(tris, n, wbase, 0u, t);
    BuildParams p;
    if constexpr (FUSED) {
        // K0: the zero words, then this tile's partial centroid box, published
        for (uint32_t j = tile * NT + threadIdx.x; j < fu.nzero; j += gridDim.x * NT)
            __hip_atomic_store(fu.zero + j, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        float lo[3], hi[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) { lo[c] = __builtin_inff(); hi[c] = -__builtin_inff(); }
#pragma unroll
        for (uint32_t q = 0; q < TPT; ++q) {
            if ((okm >> q) & 1u) {
                float bmin[3], bmax[3];
                tri_bounds(t[q], bmin, bmax);
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float cc = (bmin[c] + bmax[c]) * 0.5f;
                    lo[c] = fminf(lo[c], cc);
                    hi[c] = fmaxf(hi[c], cc);
                }
            }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) { lo[c] = wave_min(lo[c]); hi[c] = wave_max(hi[c]); }
        if (lane == 0) {
#pragma unroll
            for (int c = 0; c < 3; ++c) { red[w][c] = lo[c]; red[w][3 + c] = hi[c]; }
        }
        __syncthreads();
        if (threadIdx.x < 6) {
            const int c = threadIdx.x;
            float v = red[0][c];
#pragma unroll
            for (int k = 1; k < W; ++k) v = c < 3 ? fminf(v, red[k][c]) : fmaxf(v, red[k][c]);
            __hip_atomic_store(partials + tile * 6 + c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // The second level, as bounds_final (exact min/max: the same box as K0
        // + K1 give), done ONCE: by the block that arrives last at the grid
        // barrier -- every partial is published by then -- which stores the
        // box and only then opens the barrier; the others read its 6 words.
        // (Every block reducing all partials itself put tiles x 1470 coherent
        // loads on the same few lines.)
        RT_STAMP_HI(1);  // triangles loaded, partial box published
        if (grid_arrive_last(fu.bar, gridDim.x)) {  // block-uniform
#pragma unroll
            for (int c = 0; c < 3; ++c) { lo[c] = __builtin_inff(); hi[c] = -__builtin_inff(); }
            for (uint32_t b = threadIdx.x; b < gridDim.x; b += NT) {
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    lo[c] = fminf(lo[c], __hip_atomic_load(partials + b * 6 + c, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT));
                    hi[c] = fmaxf(hi[c], __hip_atomic_load(partials + b * 6 + 3 + c, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT));
                }
            }
#pragma unroll
            for (int c = 0; c < 3; ++c) { lo[c] = wave_min(lo[c]); hi[c] = wave_max(hi[c]); }
            __syncthreads();  // red[] reads of the partial box done
            if (lane == 0) {
#pragma unroll
                for (int c = 0; c < 3; ++c) { red[w][c] = lo[c]; red[w][3 + c] = hi[c]; }
            }
            __syncthreads();
            if (threadIdx.x < 6) {
                const int c = threadIdx.x;
                float v = red[0][c];
#pragma unroll
                for (int k = 1; k < W; ++k) v = c < 3 ? fminf(v, red[k][c]) : fmaxf(v, red[k][c]);
                __hip_atomic_store(fu.box + c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            grid_open(fu.bar, gridDim.x);
        } else {
            grid_wait(fu.bar, fu.err);
        }
        __syncthreads();  // red[] free again
        RT_STAMP_HI(2);  // through the barrier
        if (threadIdx.x < 6)
            red[0][threadIdx.x] = __hip_atomic_load(fu.box + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float a = red[0][c], b = red[0][3 + c];
            p.lo[c] = a;
            p.hi[c] = b;
            p.inv[c] = (b > a) ? 1.0f / (b - a) : 0.0f;  // §9.2, correctly rounded
        }
#pragma unroll
        for (int c = 0; c < 7; ++c) p.pad[c] = 0u;
    } else {
        p = bounds_final<NT>(partials, nb, red);  // ends with a barrier
    }
    if (tile == 0 && threadIdx.x == 0) *params = p;
    if (FUSED) RT_STAMP_HI(3);  // box read
    uint32_t k8[TPT];
#pragma unroll
    for (uint32_t h = 0; h < TPT / QL; ++h) {
        if (h > 0) okm |= load_tri_lanes_part<QL>(tris, n, wbase, h * QL, t);
#pragma unroll
        for (uint32_t qi = 0; qi < QL; ++qi) {
            const uint32_t q = h * QL + qi;
            float bmin[3], bmax[3];
            tri_bounds(t[qi], bmin, bmax);
            uint32_t qq[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) qq[c] = quant((bmin[c] + bmax[c]) * 0.5f, p.lo[c], p.inv[c]);
            k8[q] = expand10(qq[0]) * 4u + expand10(qq[1]) * 2u + expand10(qq[2]);
#if RT_K1_AGG
            {  // the lanes sharing the first lane's bucket count once (one LDS atomic)
                const bool ok = (okm >> q) & 1u;
                const uint32_t bk = k8[q] >> kMsbShift;  // 30-bit keys: bucket < 1024
                const uint32_t b0 = __builtin_amdgcn_readfirstlane(bk);
                const uint64_t peers = __ballot(ok && bk == b0);
                if (ok && bk != b0) atomicAdd(&s_start[bk], 1u);
                else if (peers && lane == (uint32_t)__ffsll((long long)peers) - 1)
                    atomicAdd(&s_start[b0], (uint32_t)__popcll(peers));
            }
#else
            if ((okm >> q) & 1u) atomicAdd(&s_start[k8[q] >> kMsbShift], 1u);  // 30-bit keys: bucket < 1024
#endif
        }
    }
    __syncthreads();
    if (FUSED) RT_STAMP_HI(4);  // keys + LDS histogram
    constexpr int PER = kMsbBuckets / NT;  // buckets per thread in scan1024's layout
    uint32_t cnt[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) cnt[j] = s_start[threadIdx.x * PER + j];
    scan1024<NT>(s_start, s_sw);  // exclusive starts; ends with a barrier
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const uint32_t d = threadIdx.x * PER + j;
        tb[(uint64_t)tile * kMsbBuckets + d] = s_start[d] | (cnt[j] << 16);
        if (ghist && cnt[j]) atomicAdd(&ghist[d], cnt[j]);  // a probe build's verdict needs the totals
    }
    __syncthreads();  // every start read: the starts become the bucket cursors
    if (FUSED) RT_STAMP_HI(5);  // scan + table
#pragma unroll
    for (uint32_t q = 0; q < TPT; ++q) {
#if RT_K1_AGG
        // clustered geometry puts a wave's 64 consecutive triangles in few
        // buckets, and same-address LDS atomics serialise: the lanes sharing
        // the first lane's bucket take one cursor range (any order within a
        // bucket is fine: k_bucket_gather sorts by (key, index))
        const bool ok = (okm >> q) & 1u;
        const uint32_t bk = k8[q] >> kMsbShift;
        const uint32_t b0 = __builtin_amdgcn_readfirstlane(bk);
        const uint64_t peers = __ballot(ok && bk == b0);
        const uint32_t lead = peers ? (uint32_t)__ffsll((long long)peers) - 1 : 0u;
        uint32_t pos = 0;
        if (ok && bk != b0) pos = atomicAdd(&s_start[bk], 1u);
        else if (peers && lane == lead) pos = atomicAdd(&s_start[b0], (uint32_t)__popcll(peers));
        const uint32_t base = (uint32_t)__shfl((int)pos, (int)lead, 64);
        if (ok && bk == b0) pos = base + sort_count_below(peers);
        if (ok) s_word[pos] = (k8[q] << 12) | (w * 64u * TPT + q * 64u + lane);  // key bits 0..19, index
#else
        if ((okm >> q) & 1u) {
            const uint32_t pos = atomicAdd(&s_start[k8[q] >> kMsbShift], 1u);
            s_word[pos] = (k8[q] << 12) | (w * 64u * TPT + q * 64u + lane);  // key bits 0..19, index
        }
#endif
    }
    __syncthreads();
    if (FUSED) RT_STAMP_HI(6);  // LDS scatter
    const uint32_t trem = n - tbase;
    const uint32_t tcount = trem < (uint32_t)kSortTile ? trem : (uint32_t)kSortTile;
#pragma unroll
    for (uint32_t m = 0; m < TPT; ++m) {
        const uint32_t q = threadIdx.x + m * NT;
        if (q < tcount) words_tb[tbase + q] = s_word[q];
    }
#ifdef RT_STAMPS
    if (FUSED) {
        __builtin_amdgcn_s_waitcnt(0x0F70);  // the stamp after the stores land
        RT_STAMP_HI(7);
    }
#endif
}

// ---------------------------------------------------------------- K4 (+K5)
__device__ __forceinline__ int kdelta(const uint32_t* __restrict__ keys, int64_t n, int64_t i, uint32_t ki, int64_t j) {
    if (j < 0 || j >= n) return -1;
    const uint32_t kj = keys[j];
    if (ki == kj) return 32 + __clz((int)((uint32_t)i ^ (uint32_t)j));
    return __clz((int)(ki ^ kj));
}

// Sorted keys seen through an LDS window [lo, hi) staged by the block, with
// global loads outside it: K4's delta searches mostly probe near i (most
// ranges are short), so most of their dependent loads become LDS reads.
struct KeyWin {
    const uint32_t* __restrict__ g;
    const uint32_t* s;
    int64_t lo, hi;
    __device__ __forceinline__ uint32_t operator[](int64_t j) const { return (j >= lo && j < hi) ? s[j - lo] : g[j]; }
};

__device__ __forceinline__ int kdelta(const KeyWin& keys, int64_t n, int64_t i, uint32_t ki, int64_t j) {
    if (j < 0 || j >= n) return -1;
    const uint32_t kj = keys[j];
    if (ki == kj) return 32 + __clz((int)((uint32_t)i ^ (uint32_t)j));
    return __clz((int)(ki ^ kj));
}

// 32-bit forms for the per-thread searches (n <= 2^30 at the ABI): an
// index j = i + m*d is formed modulo 2^32, so a position before 0 wraps
// above n and both out-of-range cases are the one test j >= n.
__device__ __forceinline__ uint32_t kkey32(const KeyWin& keys, uint32_t j) {
    const uint32_t r = j - (uint32_t)keys.lo;
    return r < (uint32_t)(keys.hi - keys.lo) ? keys.s[r] : keys.g[j];
}
__device__ __forceinline__ int kdelta32(const KeyWin& keys, uint32_t n, uint32_t i, uint32_t ki, uint32_t j) {
    if (j >= n) return -1;
    const uint32_t kj = kkey32(keys, j);
    if (ki == kj) return 32 + __clz((int)(i ^ j));
    return __clz((int)(ki ^ kj));
}

__device__ __forceinline__ int kdir(const KeyWin& keys, int64_t n, int64_t i) {
    const uint32_t ki = keys[i];
    return (kdelta(keys, n, i, ki, i + 1) - kdelta(keys, n, i, ki, i - 1)) > 0 ? 1 : -1;
}

__device__ __forceinline__ int kdir(const uint32_t* __restrict__ keys, int64_t n, int64_t i) {
    const uint32_t ki = keys[i];
    return (kdelta(keys, n, i, ki, i + 1) - kdelta(keys, n, i, ki, i - 1)) > 0 ? 1 : -1;
}

__device__ __forceinline__ void store_node(void* nodes, uint32_t idx, const Aabb& b, uint32_t a, uint32_t esc) {
    float4* p = reinterpret_cast<float4*>(reinterpret_cast<char*>(nodes) + (uint64_t)idx * 32);
    p[0] = make_float4(b.lo[0], b.lo[1], b.lo[2], b.hi[0]);
    p[1] = make_float4(b.hi[1], b.hi[2], __uint_as_float(a), __uint_as_float(esc));
}

// Leaf-ordered triangle record for the trace kernels: {v0, v1, v2, prim} in
// three aligned 16-B words.  The trace recomputes the leaf box (tri_bounds)
// and the Moller-Trumbore edges from the exact vertices, with the same fp32
// operations K4 and §9.7 use.
// Leaf-ordered triangle record k (48 B): {v0, v1, v2, prim, esc, 0}.  esc is
// leaf k's escape link: with the prim and the box (tri_bounds of the
// vertices) the record holds the whole binary leaf node, so the build does
// not write leaf nodes (rt_bvh_read derives them: k_leaf_nodes).
__device__ __forceinline__ void store_leaf_tri(float4* __restrict__ tri_s, uint32_t k, const float* t, uint32_t prim,
                                               uint32_t esc) {
    float4* o = tri_s + (uint64_t)k * 3;
    o[0] = make_float4(t[0], t[1], t[2], t[3]);
    o[1] = make_float4(t[4], t[5], t[6], t[7]);
    o[2] = make_float4(t[8], __uint_as_float(prim), __uint_as_float(esc), 0.0f);
}

// leaf k's box from its triangle record (§9.2, as the leaf node holds it)
__device__ __forceinline__ Aabb leaf_box(const float4* __restrict__ tri_s, uint32_t k) {
    const float4* p = tri_s + (uint64_t)k * 3;
    const float4 A = p[0], B = p[1], C = p[2];
    const float t[9] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w, C.x};
    Aabb b;
    tri_bounds(t, b.lo, b.hi);
    return b;
}

// Stage the sorted keys [B - KW, B + NT + KW) of a block of NT threads.
template <int NT, int KW>
__device__ __forceinline__ KeyWin stage_keys(const uint32_t* __restrict__ keys_g, uint32_t n, uint32_t* s_keys,
                                             uint32_t block = blockIdx.x) {
    const int64_t B = (int64_t)block * NT;
    const int64_t wlo = B - KW < 0 ? 0 : B - KW;
    const int64_t whi = B + NT + KW > (int64_t)n ? (int64_t)n : B + NT + KW;
    for (int64_t j = wlo + threadIdx.x; j < whi; j += NT) s_keys[j - wlo] = keys_g[j];
    __syncthreads();
    return KeyWin{keys_g, s_keys, wlo, whi};
}

// Karras topology word of internal node i from its direction d, dmin and the
// range length l, plus the two parent pointers and the
// §9.6 closed-form escape link.  lsplit: the split offset s.
__device__ __forceinline__ uint4 karras_finish(const KeyWin& keys, int64_t N, int64_t i, int d, int64_t l, int64_t s,
                                               uint4* __restrict__ topo, uint32_t* __restrict__ parent) {
    const uint32_t L0 = (uint32_t)N - 1;
    const int64_t j = i + l * d;
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
    const uint4 tp = make_uint4(left, esc, (uint32_t)mn, (uint32_t)mx);
    if (topo) topo[i] = tp;  // k_topo_refit stores the crossing nodes' words only
    if (parent) {
        parent[left] = (uint32_t)i;
        parent[right] = (uint32_t)i;
    }
    return tp;
}

// Thread i: internal node i (i < n-1) and leaf i (i < n).  Writes topo[i],
// the two parent pointers, leaf node L0+i and tri_s[i]; returns the
// topology word (zero when node i does not exist) and the leaf box.  With
// allow_defer, a node whose exponential search would leave the staged key
// window (a range longer than the window margin: the top ~log2(n/KW) levels,
// about one node per block) is not searched here -- `deferred` is set and
// its wave searches it cooperatively (karras_wave_search): the serial
// search would be ~40 dependent global loads and hold the whole block.
// Leaf i's triangle, gathered through the sorted index (issued early by the
// callers so its latency overlaps the key staging and the searches).
struct LeafTri { float v[9]; uint32_t prim; };
__device__ __forceinline__ LeafTri gather_leaf(uint32_t prim, const float* __restrict__ tris) {
    LeafTri t;
    t.prim = prim;
    const Vtx* src = reinterpret_cast<const Vtx*>(tris) + (uint64_t)t.prim * 3;  // three 12-B loads
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const Vtx v = src[j];
        t.v[3 * j] = v.x;
        t.v[3 * j + 1] = v.y;
        t.v[3 * j + 2] = v.z;
    }
    return t;
}

// The end, in direction d, of the run of sorted positions whose keys share
// their top L bits with key ki (ki's bucket bid = ki >> 20), when L <= 12:
// such a prefix covers only bucket bits (bits 31..30 of a 30-bit key are 0),
// so the run is a range of whole buckets and its ends are bucket starts
// (bstart[1025]).  This answers §9.5's searches for the long ranges of the
// top tree levels -- whose keys differ in the bucket bits -- with two loads
// instead of a wave-wide search through global memory.
__device__ __forceinline__ uint32_t bucket_run_end(const uint32_t* __restrict__ bstart, uint32_t ki, int L, int d,
                                                   uint32_t n) {
    const int shift = 12 - L;  // bucket bits below the prefix
    if (shift >= 10) return d > 0 ? n - 1 : 0u;
    const uint32_t g = (ki >> kMsbShift) >> shift;
    return d > 0 ? bstart[(g + 1) << shift] - 1 : bstart[g << shift];
}

__device__ __forceinline__ void karras_node_leaf(const KeyWin& keys, const LeafTri& lt, uint32_t n, uint32_t i32,
                                                 uint4* __restrict__ topo, uint32_t* __restrict__ parent,
                                                 void* __restrict__ nodes, float4* __restrict__ tri_s, uint4& tp_out,
                                                 Aabb& box, bool allow_defer, bool& deferred, bool leaf_node = false,
                                                 const uint32_t* __restrict__ bstart = nullptr) {
    const int64_t i = i32, N = n;
    const uint32_t L0 = n - 1;
    if (i32 == 0 && parent) parent[0] = RT_SENT;  // root: internal 0, or leaf 0 when n == 1
    uint32_t lesc;
    tp_out = make_uint4(0, 0, 0, 0);
    deferred = false;
    if (i < N - 1) {
        // §9.5 searches in 32-bit index arithmetic (kdelta32); m*d as
        // (d > 0 ? m : -m) modulo 2^32
        const uint32_t ki = kkey32(keys, i32);
        const int d = (kdelta32(keys, n, i32, ki, i32 + 1) - kdelta32(keys, n, i32, ki, i32 - 1)) > 0 ? 1 : -1;
        const uint32_t ud = (uint32_t)d;  // +1 or 0xFFFFFFFF
        const int dmin = kdelta32(keys, n, i32, ki, i32 - ud);
        uint32_t lmax = 2;
        for (;;) {
            const uint32_t q = i32 + lmax * ud;
            if (allow_defer && q < n && (q - (uint32_t)keys.lo) >= (uint32_t)(keys.hi - keys.lo)) {
                deferred = true;
                break;
            }
            if (!(kdelta32(keys, n, i32, ki, q) > dmin)) break;
            lmax <<= 1;
        }
        if (deferred && bstart && dmin <= 11) {
            // the range leaves the key window: its end is a bucket boundary
            // (dmin + 1 <= 12 prefix bits); so is the split when the range's
            // ends differ in their bucket (dnode <= 11)
            const uint32_t j = bucket_run_end(bstart, ki, dmin + 1, d, n);
            const int dnode = kdelta32(keys, n, i32, ki, j);
            if (dnode <= 11) {
                const uint32_t l = d > 0 ? j - i32 : i32 - j;
                const uint32_t g = bucket_run_end(bstart, ki, dnode + 1, d, n);
                const uint32_t sp = d > 0 ? g - i32 : i32 - g;
                tp_out = karras_finish(keys, N, i, d, (int64_t)l, (int64_t)sp, topo, parent);
                deferred = false;
            } else {
                tp_out = make_uint4(0, 0, d > 0 ? i32 : 0u, d > 0 ? RT_SENT - 1 : i32);
            }
        } else if (!deferred) {
            uint32_t l = 0;
            for (uint32_t t = lmax >> 1; t >= 1; t >>= 1)
                if (kdelta32(keys, n, i32, ki, i32 + (l + t) * ud) > dmin) l += t;
            const int dnode = kdelta32(keys, n, i32, ki, i32 + l * ud);
            uint32_t s = 0, t = l;
            do {
                t = (t + 1) >> 1;
                if (kdelta32(keys, n, i32, ki, i32 + (s + t) * ud) > dnode) s += t;
            } while (t > 1);
            tp_out = karras_finish(keys, N, i, d, (int64_t)l, (int64_t)s, topo, parent);
        } else {
            // the crossing flags only need which end of the range i is
            tp_out = make_uint4(0, 0, d > 0 ? i32 : 0u, d > 0 ? RT_SENT - 1 : i32);
        }
        // leaf i's range ends at i: same closed form with r = i
        lesc = (i + 1 <= N - 2 && kdir(keys, N, i + 1) > 0) ? (uint32_t)(i + 1) : (uint32_t)(L0 + i + 1);
    } else {
        lesc = RT_SENT;  // leaf n-1
    }
    tri_bounds(lt.v, box.lo, box.hi);
    if (leaf_node) store_node(nodes, L0 + i32, box, lt.prim, lesc);  // the stage entry point's full node array
    store_leaf_tri(tri_s, i32, lt.v, lt.prim, lesc);
}

// Largest t in [0, R) with delta(i, i + t d) > thr, all 64 lanes probing at
// once (63-ary search; the predicate is monotone in t and true at t = 0).
__device__ __forceinline__ int64_t wave_max_true(const KeyWin& keys, int64_t N, int64_t i, uint32_t ki, int d, int thr,
                                                 int64_t R) {
    const uint32_t lane = threadIdx.x & 63;
    int64_t base = 0, span = R;  // answer in [base, base + span)
    while (span > 1) {
        const int64_t step = (span + 62) / 63;
        const int64_t t = base + (int64_t)(lane + 1) * step;
        const bool p = lane < 63 && t < base + span && kdelta(keys, N, i, ki, i + t * d) > thr;
        const uint32_t c = (uint32_t)__popcll(__ballot(p));  // monotone: lanes [0, c) true
        const int64_t nb = base + (int64_t)c * step;
        const int64_t end = base + span;
        base = nb;
        span = (nb + step < end ? nb + step : end) - nb;
    }
    return base;
}

// The wave's deferred nodes, one at a time, every lane probing: exponential
// search in one round (lanes p = 1..31 test 2^p), then the range and split
// searches 63-ary.  Same monotone predicates and answers as the serial code.
__device__ __forceinline__ void karras_wave_search(const KeyWin& keys, uint32_t n, uint32_t i32, bool deferred,
                                                   uint4* __restrict__ topo, uint32_t* __restrict__ parent,
                                                   uint4& tp) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t dm = __ballot(deferred);
    const int64_t N = n;
    while (dm) {
        const uint32_t src = (uint32_t)__ffsll((long long)dm) - 1;
        dm &= dm - 1;
        const int64_t i = (int64_t)(uint32_t)__shfl((int)i32, (int)src, 64);
        const uint32_t ki = keys[i];
        const int d = (kdelta(keys, N, i, ki, i + 1) - kdelta(keys, N, i, ki, i - 1)) > 0 ? 1 : -1;
        const int dmin = kdelta(keys, N, i, ki, i - d);
        const bool pe = lane >= 1 && lane <= 31 && kdelta(keys, N, i, ki, i + ((int64_t)1 << lane) * d) > dmin;
        const uint32_t pstar = 1u + (uint32_t)__popcll(__ballot(pe));
        const int64_t lmax = (int64_t)1 << pstar;
        const int64_t l = wave_max_true(keys, N, i, ki, d, dmin, lmax);
        const int dnode = kdelta(keys, N, i, ki, i + l * d);
        const int64_t s = wave_max_true(keys, N, i, ki, d, dnode, l);
        if (lane == src) tp = karras_finish(keys, N, i, d, l, s, topo, parent);
    }
}

// K4 alone (rt_stage_topology).
__global__ __launch_bounds__(256) void k_karras_leaves(const uint32_t* __restrict__ keys_g, const uint32_t* __restrict__ svals,
                                                       const float* __restrict__ tris, uint32_t n,
                                                       uint4* __restrict__ topo, uint32_t* __restrict__ parent,
                                                       void* __restrict__ nodes, float4* __restrict__ tri_s) {
    __shared__ uint32_t s_keys[256 + 2 * 1024];
    const uint32_t i32 = blockIdx.x * 256u + threadIdx.x;
    const uint32_t prim = i32 < n ? svals[i32] : 0u;
    const KeyWin keys = stage_keys<256, 1024>(keys_g, n, s_keys);
    if (i32 >= n) return;
    const LeafTri lt = gather_leaf(prim, tris);
    uint4 tp;
    Aabb box;
    bool deferred;
    karras_node_leaf(keys, lt, n, i32, topo, parent, nodes, tri_s, tp, box, false, deferred, true);
}

// Stand-alone leaf-triangle pass (rt_stage_trace on caller nodes).
__global__ __launch_bounds__(256) void k_leaf_tris(const void* __restrict__ nodes, const float* __restrict__ tris,
                                                   uint32_t n, float4* __restrict__ tri_s) {
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= n) return;
    const uint32_t* leaf = reinterpret_cast<const uint32_t*>(nodes) + ((uint64_t)(n - 1) + k) * 8;
    const uint32_t prim = leaf[6];
    float t[9];
#pragma unroll
    for (int c = 0; c < 9; ++c) t[c] = tris[(uint64_t)prim * 9 + c];
    store_leaf_tri(tri_s, k, t, prim, leaf[7]);
}

// The binary leaf nodes L0 + k, derived from the triangle records
// (rt_bvh_read / rt_bvh_save / rt_stage_refit: the build writes internal
// nodes only).
__global__ __launch_bounds__(256) void k_leaf_nodes(const float4* __restrict__ tri_s, uint32_t n,
                                                    void* __restrict__ nodes) {
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= n) return;
    const float4 C = tri_s[(uint64_t)k * 3 + 2];
    store_node(nodes, n - 1 + k, leaf_box(tri_s, k), __float_as_uint(C.y), __float_as_uint(C.z));
}

// ---------------------------------------------------------------- K6 refit
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

// ---------------------------------------------------------------- K7w wide tree (the trace-layout pack of SURVEY.md §8(a) a9)
__device__ __forceinline__ Aabb load_aabb_node(const void* nodes, uint32_t i) {
    const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(nodes) + (uint64_t)i * 32);
    const float4 A = p[0], B = p[1];
    Aabb b;
    b.lo[0] = A.x; b.lo[1] = A.y; b.lo[2] = A.z;
    b.hi[0] = A.w; b.hi[1] = B.x; b.hi[2] = B.y;
    return b;
}

// Children of internal node X from its topology word {left, esc, lo, hi}:
// the split g is the left child's index (internal g or leaf L0+g); the right
// child is internal g+1, or leaf L0+g+1 when the range ends at g+1.
// The topology word of internal node i rebuilt from its node record {box,
// left, esc}: kids_of needs the left child and the range end mx, and the
// escape link is §9.6's closed form of mx (SENT: mx = n-1; leaf L0+mx+1;
// internal mx+1), so mx follows from it.  The range start is not needed.
__device__ __forceinline__ uint4 topo_of_node(const void* nodes, uint32_t i, uint32_t L0) {
    const float4 B = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(nodes) + (uint64_t)i * 32)[1];
    const uint32_t left = __float_as_uint(B.z), esc = __float_as_uint(B.w);
    const uint32_t mx = esc == RT_SENT ? L0 : esc >= L0 ? esc - L0 - 1 : esc - 1;
    return make_uint4(left, esc, 0u, mx);
}

__device__ __forceinline__ void kids_of(const uint4& tp, uint32_t L0, uint32_t& l, uint32_t& r) {
    l = tp.x;
    const uint32_t g = l < L0 ? l : l - L0;
    r = tp.w == g + 1 ? L0 + g + 1 : g + 1;
}

// One axis of one record: grid step 2^e with 255 * 2^e >= extent, then for
// each valid child the outward-rounded planes.  false: not representable
// (non-finite values, exponent > 119, or origin + 255 * 2^e rounding below
// hi) -- the record goes wild.  Fixed 4 slots, fully unrolled (no dynamic
// register indexing -> no scratch).
//
// Why one correction step and no clamps suffice (planes are checked with
// wide_plane, the trace kernel's own arithmetic):
//  * every slot's planes lie in [olo, ohi] (X's box is the exact union of its
//    entries' boxes; unused slots carry X's box), so c = fl(x - olo) * 2^-e is
//    in [0, fl(ohi - olo) * 2^-e] subset [0, 255] by the choice of e: floor
//    and ceil need no clamp;
//  * lo side: f = floor(c) gives a real plane olo + f 2^e <= lo + u|lo - olo|;
//    if its rounding lands above lo, f - 1 is a full step 2^e >= ext/255 >>
//    u|lo - olo| lower, so its real value is < lo and its rounding is <= lo
//    (lo is a float).  f = 0 never needs the step (olo <= lo);
//  * hi side, symmetric: ceil, and one step up when the plane rounds below
//    hi.  The step would leave the byte only if origin + 255 * 2^e rounds
//    below hi <= ohi, which the per-axis check `top` rejects (wild).
// A NaN/inf anywhere makes the slot sum non-finite (so does an overflowing
// sum of finite values: wild, which is only conservative).
template <int W>
__device__ __forceinline__ bool quant_axis(float olo, float ohi, const float (&clo)[W], const float (&chi)[W],
                                           uint32_t valid, uint32_t (&qlo_w)[W / 4], uint32_t (&qhi_w)[W / 4],
                                           int& e_out) {
    const float ext = ohi - olo;
    // callers pass X's own box in unused slots (inside [olo, ohi]); their
    // bytes are written as 0
    const float(&lo)[W] = clo;
    const float(&hi)[W] = chi;
    float chk = ext;
#pragma unroll
    for (int i = 0; i < W; i += 4)
        chk = chk + (((lo[i] + lo[i + 1]) + (lo[i + 2] + lo[i + 3])) + ((hi[i] + hi[i + 1]) + (hi[i + 2] + hi[i + 3])));
    if (!isfinite(chk) || !(ext >= 0.0f)) return false;
    const uint32_t be = (__float_as_uint(ext) >> 23) & 0xFF;  // ext normal: 2^(be-127) <= ext
    int e = (ext > 0.0f && be) ? (int)be - 134 : -126;
    e = e < -126 ? -126 : e;
    e += (ldexpf(255.0f, e) < ext) ? 1 : 0;
    if (e > 119) return false;
    const float sc = wide_scale(e);
    const bool top = !(wide_plane(olo, 255u, sc) < ohi);
#pragma unroll
    for (int wd = 0; wd < W / 4; ++wd) {
        uint32_t lw = 0, hw = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = 4 * wd + j;
            float fl = floorf(ldexpf(lo[i] - olo, -e));
            fl = fmaf(fl, sc, olo) > lo[i] ? fl - 1.0f : fl;
            float fh = ceilf(ldexpf(hi[i] - olo, -e));
            fh = fmaf(fh, sc, olo) < hi[i] ? fh + 1.0f : fh;
            const bool v = (valid >> i) & 1u;
            lw = __builtin_amdgcn_cvt_pk_u8_f32(v ? fl : 0.0f, (uint32_t)j, lw);
            hw = __builtin_amdgcn_cvt_pk_u8_f32(v ? fh : 0.0f, (uint32_t)j, hw);
        }
        qlo_w[wd] = lw;
        qhi_w[wd] = hw;
    }
    e_out = e;
    return top;
}

// Quantize and store the wide record of internal node X from its box and the
// boxes of its 2-W cut entries (node[] binary indices in preorder, RT_SENT in
// unused slots); box_of(slot) fetches an entry's box (LDS in K6, global in
// k_wide_cross).  Layouts: rt_device.h (K7w for W = 4, K7w8 for W = 8).  A
// wild record (a plane not representable) gets exponent bytes 255 and zero
// planes: the trace then takes every valid child.
template <int W, typename BoxOf>
__device__ __forceinline__ void store_wide(uint4* __restrict__ wnodes, uint32_t X, const Aabb& bx,
                                           const uint32_t (&node)[W], BoxOf box_of, uint32_t L0) {
    constexpr int QW = W / 4;
    uint32_t valid = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) valid |= (node[i] != RT_SENT ? 1u : 0u) << i;
    float bl[3][W], bh[3][W];  // static indices only: no scratch
#pragma unroll
    for (int i = 0; i < W; ++i) {
        const Aabb b = box_of(i);
#pragma unroll
        for (int c = 0; c < 3; ++c) { bl[c][i] = b.lo[c]; bh[c][i] = b.hi[c]; }
    }
    uint32_t ql[3][QW], qh[3][QW];
    int e[3] = {0, 0, 0};
    bool wild = false;
#pragma unroll
    for (int c = 0; c < 3; ++c)
        if (!quant_axis<W>(bx.lo[c], bx.hi[c], bl[c], bh[c], valid, ql[c], qh[c], e[c])) wild = true;
    uint32_t eb = (uint32_t)(e[0] + 127) | ((uint32_t)(e[1] + 127) << 8) | ((uint32_t)(e[2] + 127) << 16);
    if (wild) {
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int k = 0; k < QW; ++k) ql[c][k] = qh[c][k] = 0u;
        eb = kWideWildExp | (kWideWildExp << 8) | (kWideWildExp << 16);
    }
    uint32_t ref[W];
#pragma unroll
    for (int i = 0; i < W; ++i)
        ref[i] = node[i] == RT_SENT ? RT_SENT : node[i] < L0 ? node[i] : (kWideLeaf | (node[i] - L0));
    uint4* o = wnodes + (uint64_t)X * WideFmt<W>::words;
    if constexpr (W == 4) {
        const uint32_t meta = eb | ((valid << 4 | (wild ? kWideWild : 0u)) << 24);
        o[0] = make_uint4(__float_as_uint(bx.lo[0]), __float_as_uint(bx.lo[1]), __float_as_uint(bx.lo[2]), meta);
        o[1] = make_uint4(ql[0][0], ql[1][0], ql[2][0], qh[0][0]);
        o[2] = make_uint4(qh[1][0], qh[2][0], ref[0], ref[1]);
        o[3] = make_uint4(ref[2], ref[3], 0u, 0u);
    } else {
        const uint32_t meta = eb | (valid << 24);
        o[0] = make_uint4(__float_as_uint(bx.lo[0]), __float_as_uint(bx.lo[1]), __float_as_uint(bx.lo[2]), meta);
        o[1] = make_uint4(ql[0][0], ql[0][QW - 1], ql[1][0], ql[1][QW - 1]);
        o[2] = make_uint4(ql[2][0], ql[2][QW - 1], qh[0][0], qh[0][QW - 1]);
        o[3] = make_uint4(qh[1][0], qh[1][QW - 1], qh[2][0], qh[2][QW - 1]);
        o[4] = make_uint4(ref[0], ref[1], ref[2], ref[3]);
        o[5] = make_uint4(ref[4], ref[5], ref[6], ref[7]);
    }
}

// The record's entries (W slots, RT_SENT-padded); topo_of(i) gives internal
// node i's topology word, box_of_node(i) its box.  The greedy cut (r01; the
// fixed two-level cut, build.wide_collapse = 0, was removed in r06 --
// profiles/ab_collapse_r01.log, profiles/rejected_knobs_r06.patch): starting
// from {left, right}, W - 2 times replace the internal entry with the largest box
// surface (first in preorder on ties) by its two children.  Any such set is
// a preorder cut of X's subtree (each entry a descendant, their subtrees
// partitioning X's leaves, listed in preorder), which is all the trace's
// exactness argument uses; the greedy cut fills the slots a leaf child
// leaves empty in the fixed one and descends where the big boxes are.
__device__ __forceinline__ float half_area(const Aabb& b) {
    const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
    return (dx * dy + dy * dz) + dz * dx;
}

template <int W, typename TopoOf, typename BoxOfNode>
__device__ __forceinline__ void wide_entries(const uint4& tx, uint32_t L0, TopoOf topo_of, BoxOfNode box_of_node,
                                             uint32_t (&node)[W]) {
    uint32_t l, r;
    kids_of(tx, L0, l, r);
    {
        // W - 2 greedy replacements; ar[] caches the entries' surfaces
        // (internal entries only; leaves and empty slots are never picked)
        float ar[W];
        node[0] = l; node[1] = r;
#pragma unroll
        for (int i = 2; i < W; ++i) node[i] = RT_SENT;
        ar[0] = l < L0 ? half_area(box_of_node(l)) : 0.0f;
        ar[1] = r < L0 ? half_area(box_of_node(r)) : 0.0f;
#pragma unroll
        for (int i = 2; i < W; ++i) ar[i] = 0.0f;
#pragma unroll
        for (int step = 0; step < W - 2; ++step) {
            int best = -1;
            float ba = 0.0f;
#pragma unroll
            for (int i = 0; i < step + 2; ++i) {  // slots past step + 1 are still empty
                if (node[i] < L0) {               // internal (RT_SENT and leaves are >= L0)
                    if (best < 0 || ar[i] > ba) { best = i; ba = ar[i]; }
                }
            }
            if (best < 0) break;
            uint32_t pick = node[0];
#pragma unroll
            for (int i = 1; i < step + 2; ++i) pick = best == i ? node[i] : pick;
            uint32_t c0, c1;
            kids_of(topo_of(pick), L0, c0, c1);
            const float a0 = c0 < L0 ? half_area(box_of_node(c0)) : 0.0f;
            const float a1 = c1 < L0 ? half_area(box_of_node(c1)) : 0.0f;
            uint32_t nn[W];
            float na[W];
#pragma unroll
            for (int i = 0; i < W; ++i) {
                nn[i] = i < best ? node[i] : i == best ? c0 : i == best + 1 ? c1 : node[i - 1 < 0 ? 0 : i - 1];
                na[i] = i < best ? ar[i] : i == best ? a0 : i == best + 1 ? a1 : ar[i - 1 < 0 ? 0 : i - 1];
            }
#pragma unroll
            for (int i = 0; i < W; ++i) { node[i] = nn[i]; ar[i] = na[i]; }
        }
    }
}

// K4 + K6 local + K7w local, fused.  One block = kRefitT consecutive sorted
// leaves [B0, B1) and the internal nodes with the same indices, one thread
// per leaf/node:
//   1. Karras topology of internal node i and leaf i (karras_node_leaf; the
//      topology words stay in LDS for step 4);
//   2. block prefix/suffix scans of the leaf boxes for the crossing nodes
//      (K6t: k_refit_cross) and the crossing list;
//   3. the box of every LOCAL internal node (range inside the block) as a
//      range union over its leaves: a sparse table over the block's leaf
//      boxes, built level by level in LDS, and box[l, r] = T_k[l] U
//      T_k[r - 2^k + 1] (k = floor(log2(r - l + 1))).  min/max are exact and
//      order-free, so this is bit-identical to the bottom-up union of
//      children -- without the serial climb (the old K6 spent ~6 us per
//      block in its atomic-arrival loop) and without re-reading the
//      topology and parent arrays K4 used to write for it;
//   4. coalesced stores of the local internal nodes and their K7w records.
// keys staged on each side of a refit block (its nodes' delta searches run in
// LDS inside this window; a search that would leave it runs wave-wide in
// global memory)
#ifndef RT_REFIT_KEY_MARGIN
#define RT_REFIT_KEY_MARGIN (RT_REFIT_T >= 512 ? 1024 : 512)  // the window must fit the T-entry table buffer
#endif
template <int W>
__global__ __launch_bounds__(kRefitT) void k_topo_refit(const uint32_t* __restrict__ keys_g,
                                                        const uint32_t* __restrict__ svals,
                                                        const float* __restrict__ tris, uint32_t n,
                                                        uint4* __restrict__ topo, uint32_t* __restrict__ parent,
                                                        void* __restrict__ nodes, float4* __restrict__ tri_s,
                                                        float* __restrict__ prebuf, float* __restrict__ sufbuf,
                                                        float* __restrict__ totals, uint32_t* __restrict__ cross,
                                                        uint32_t* cross_ctr, uint32_t cross_cap,
                                                        uint4* __restrict__ wnodes,
                                                        uint32_t block0 = 0,
                                                        const uint32_t* __restrict__ flags_src = nullptr,
                                                        uint32_t* __restrict__ flags_dst = nullptr,
                                                        const uint32_t* __restrict__ bstart = nullptr) {
    constexpr int T = kRefitT, NW = T / 64, KW = RT_REFIT_KEY_MARGIN;
    // the build's verdict words (zero[kZDense ..]), final once the sort
    // kernels have run, to the host's mapped pinned copy: no copy launch
    if (flags_dst && blockIdx.x == 0 && threadIdx.x < 8) flags_dst[threadIdx.x] = flags_src[threadIdx.x];
    static_assert((T + 2 * KW) * 4 <= T * (int)sizeof(Aabb), "key window must fit the table buffer");
    static_assert(sizeof(uint4) <= sizeof(Aabb), "topology words must fit the table buffer");
    __shared__ Aabb s_tab[T];          // key window first (uint32), then the odd sparse-table levels
    __shared__ Aabb s_box[2 * T];      // [0,T) leaves; [T,2T) the even levels, then local internal nodes
    __shared__ Aabb s_wpre[NW], s_wsuf[NW];
    __shared__ uint32_t s_ncross, s_cbase;

    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t L0 = n - 1;
    const uint32_t gb = blockIdx.x + block0;  // global refit block (a rank's share starts at block0)
    const uint32_t B0 = gb * (uint32_t)T;
    const uint32_t B1 = (n - B0) < (uint32_t)T ? n : B0 + (uint32_t)T;
    const uint32_t k = B0 + tid;
    const bool valid = k < B1;
    const bool has_int = k + 1 < n;
    if (tid == 0) s_ncross = 0u;
    RT_STAMP(0);
    // ---- 1. topology + leaf
    uint4 tp = make_uint4(0, 0, 0, 0);
    Aabb box = aabb_empty();
    {
        // the gather is issued after the key staging: before it, the staging's
        // wait (vmcnt is in order) would also wait for the random gather
        const uint32_t prim = valid ? svals[k] : 0u;  // coalesced, with the window loads
        const KeyWin keys = stage_keys<T, KW>(keys_g, n, reinterpret_cast<uint32_t*>(s_tab), gb);
        RT_STAMP(1);
        LeafTri lt;
#ifdef RT_EXP_GATHER_SEQ
        // traffic attribution only (tools/topo_traffic.sh, wrong output): leaf k's
        // triangle read coalesced from tris[k] instead of gathered from tris[prim]
        if (valid) { lt = gather_leaf(k, tris); lt.prim = prim; }
#else
        if (valid) lt = gather_leaf(prim, tris);
#endif
        bool deferred = false;
        // topology words stay in registers/LDS: only the crossing nodes' go to
        // global memory (step 2), for k_refit_cross / k_wide_cross
        if (valid) karras_node_leaf(keys, lt, n, k, nullptr, parent, nodes, tri_s, tp, box, true, deferred, false, bstart);
        RT_STAMP(6);  // diagnostic builds: the own node and leaf done (the wave searches follow)
        karras_wave_search(keys, n, k, deferred, nullptr, parent, tp);
    }
    s_box[tid] = box;
    RT_STAMP(2);
    // ---- 2. block prefix / suffix scans of leaf AABBs (exact min/max)
    Aabb pre = box, suf = box;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) { shfl_up_aabb(pre, o); shfl_down_aabb(suf, o); }
    if (lane == 63) s_wpre[wv] = pre;
    if (lane == 0) s_wsuf[wv] = suf;
    __syncthreads();  // also: s_box leaves complete; the key window is dead
    for (uint32_t q = 0; q < wv; ++q) aabb_union(pre, s_wpre[q]);
    for (uint32_t q = wv + 1; q < NW; ++q) aabb_union(suf, s_wsuf[q]);
    uint32_t cslot = RT_SENT;
    if (valid) {
        // crossing ends (DESIGN.md "refit"): the topmost node starting at leaf
        // k is internal k iff its range starts at k; the topmost node ending at
        // k is internal k iff its range ends at k; the root ends at n-1.
        const bool need_suf = has_int && tp.z == k && tp.w >= B1;
        const bool need_pre = (has_int && tp.w == k && tp.z < B0) || (k == n - 1 && B0 > 0);
        if (need_suf) store_aabb(sufbuf, k, suf);
        if (need_pre) store_aabb(prebuf, k, pre);
        if (k == B1 - 1) store_aabb(totals, gb, pre);
        if (has_int && (tp.z < B0 || tp.w >= B1)) {
            cslot = atomicAdd(&s_ncross, 1u);  // LDS
            topo[k] = tp;
        }
    }
    __syncthreads();
    RT_STAMP(3);
    // one aggregated reservation per block on one of kCrossShards counters
    // (a single global counter hit by every wave serialises at ~90 ops/us);
    // issued here, consumed after the sweep, so its latency overlaps it
    uint32_t cbase = 0;
    if (tid == 0 && s_ncross)
        cbase = (gb % kCrossShards) * cross_cap + atomicAdd(&cross_ctr[gb % kCrossShards], s_ncross);
    // ---- 3. sparse-table sweep: level kk holds T_kk[j] = U leaves [j, j + 2^kk),
    // odd levels in s_tab, even ones in s_box[T, 2T) (ping-pong: one barrier
    // per level); a node's box waits in registers until the sweep is over
    const bool local = valid && has_int && tp.z >= B0 && tp.w < B1;
    uint32_t need = 0, qa = 0, qb = 0;
    if (local) {
        const uint32_t len = tp.w - tp.z + 1;  // >= 2
        need = 31u - (uint32_t)__clz((int)len);
        qa = tp.z - B0;
        qb = tp.w - B0 + 1 - (1u << need);
    }
    const uint32_t cnt = B1 - B0;
    Aabb nbox = aabb_empty();
    for (uint32_t kk = 1; (1u << kk) <= cnt; ++kk) {
        const uint32_t h = 1u << (kk - 1);
        const Aabb* src = kk == 1 ? s_box : (kk & 1) ? s_box + T : s_tab;
        Aabb* dst = (kk & 1) ? s_tab : s_box + T;
        if (tid + 2 * h <= cnt) {  // window [tid, tid + 2^kk) inside the block
            Aabb v = src[tid];
            aabb_union(v, src[tid + h]);
            dst[tid] = v;
        }
        __syncthreads();
        if (need == kk) {
            nbox = dst[qa];
            aabb_union(nbox, dst[qb]);
        }
    }
    __syncthreads();  // the even-level buffer becomes the internal-node boxes; s_tab the topology words
    uint4* s_topo = reinterpret_cast<uint4*>(s_tab);
    if (local) s_box[T + tid] = nbox;
    s_topo[tid] = tp;
    if (tid == 0) s_cbase = cbase;
    __syncthreads();
    RT_STAMP(4);
    if (cslot != RT_SENT) cross[s_cbase + cslot] = k;
    // ---- 4. coalesced store of this block's local internal nodes and their
    // K7w wide records (every box they need is in LDS)
    if (local) {
        const Aabb bx = s_box[T + tid];
        store_node(nodes, k, bx, tp.x, tp.y);
        uint32_t node[W];
        // every descendant of a local node is local: topology and boxes in LDS
        wide_entries<W>(tp, L0, [&](uint32_t i) { return s_topo[i - B0]; },
                        [&](uint32_t i) { return s_box[T + i - B0]; }, node);
        uint32_t slot[W];
#pragma unroll
        for (int i = 0; i < W; ++i)
            slot[i] = node[i] == RT_SENT ? T + tid : node[i] >= L0 ? node[i] - L0 - B0 : T + node[i] - B0;
        store_wide<W>(wnodes, k, bx, node, [&](int i) { return s_box[slot[i]]; }, L0);
    }
    RT_STAMP(5);
}

// Global sparse table over the m per-block totals (more than
// kLdsTreeMaxBlocks blocks, the 10M path): level k entry b = U totals
// [b, min(b + 2^k, m)), table + k*m*6.  Two launches instead of one per
// level (14 at 10M, ~4.6 us each, almost all of it launch and drain):
//   k_sparse_near: levels 1..kSparseNear, each block doubling a window of
//     512 totals in LDS for its 256 entries;
//   k_sparse_far: levels above, each entry the union of level kSparseNear
//     entries 256 apart (<= 2^(L-1-kSparseNear) L2-resident loads).
// min/max are exact, so every entry is the same union as the level-by-level
// doubling's.
constexpr uint32_t kSparseNear = 8;
__global__ __launch_bounds__(256) void k_sparse_near(float* __restrict__ table, uint32_t m, uint32_t levels) {
    __shared__ Aabb s_w[512];
    const uint32_t c0 = blockIdx.x * 256u, t = threadIdx.x;
    s_w[t] = c0 + t < m ? load_aabb(table, c0 + t) : aabb_empty();
    s_w[t + 256] = c0 + t + 256 < m ? load_aabb(table, c0 + t + 256) : aabb_empty();
    __syncthreads();
    for (uint32_t lv = 1; lv < levels && lv <= kSparseNear; ++lv) {
        const uint32_t h = 1u << (lv - 1);
        Aabb a = s_w[t], b = s_w[t + 256];
        aabb_union(a, s_w[t + h]);
        if (t + 256 + h < 512) aabb_union(b, s_w[t + 256 + h]);
        __syncthreads();
        s_w[t] = a;
        s_w[t + 256] = b;
        __syncthreads();
        if (c0 + t < m) store_aabb(table + (uint64_t)lv * m * 6, c0 + t, a);
    }
}
__global__ __launch_bounds__(256) void k_sparse_far(float* __restrict__ table, uint32_t m, uint32_t levels) {
    const uint32_t b = blockIdx.x * 256u + threadIdx.x;
    if (b >= m) return;
    const float* near = table + (uint64_t)kSparseNear * m * 6;
    Aabb a = load_aabb(near, b);
    uint32_t have = 1;  // level-kSparseNear entries folded in: b, b + 256, ...
    for (uint32_t lv = kSparseNear + 1; lv < levels; ++lv) {
        const uint32_t want = 1u << (lv - kSparseNear);
        for (; have < want; ++have) {
            const uint64_t j = (uint64_t)b + (uint64_t)have * (1u << kSparseNear);
            if (j < m) aabb_union(a, load_aabb(near, j));
        }
        store_aabb(table + (uint64_t)lv * m * 6, b, a);
    }
}

// Group tables (r05, the default crossing path up to kLdsTreeMaxBlocks
// groups): the m per-block totals (table level 0, written by k_topo_refit)
// in groups of kGroupBlocks = 64 blocks, one wave per group:
//   levels 1..5  U totals [b, b + 2^k) inside the group (range queries of
//                fewer than 64 blocks: two entries of one level),
//   level  6     U totals [group start, b]  (in-group prefix),
//   level  7     U totals [b, group end]    (in-group suffix),
//   level  8     the group totals ([ng] entries),
// at table + k * m * 6.  A middle-block range [bl, br) that crosses groups is
// then gsuf[bl] U (groups strictly between, an LDS segment tree over <= 2048
// group totals in each k_refit_cross block) U gpre[br - 1].  This replaces the
// global sparse table (k_sparse_near + k_sparse_far, whose top levels loop
// over up to 2^(L-9) entries each: 21 us at 10M with 512-leaf blocks, ~4x
// that with 256) and the per-block LDS tree over up to 2048 block totals
// (98 KB of LDS in each of the crossing kernel's blocks) with one wave per 64
// blocks.  min/max are exact, so every box is the same union.  (Folding
// this into k_topo_refit -- the last block of each group computing its
// tables behind write-through totals and an arrival counter -- cost the
// refit kernel what it saved in launches, whether the blocks arrived at
// their end (1M build 139.5 -> 140.7 us, 10M 1123.7 -> 1122.7 us) or right
// after publishing their totals (1M 140.6 -> 140.0 / 141.3 us, 10M 1126.9 ->
// 1145.5 us; the folded kernel also needs 58 VGPRs instead of 52);
// profiles/ab_group_fold_r05.log.  Not kept.)
constexpr uint32_t kGroupBlocks = 64;
__global__ __launch_bounds__(64) void k_group_tables(float* __restrict__ table, uint32_t m) {
    const uint32_t g = blockIdx.x, l = threadIdx.x, b = g * kGroupBlocks + l;
    const bool ok = b < m;
    const Aabb t = ok ? load_aabb(table, b) : aabb_empty();
    Aabb pre = t, suf = t;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) { shfl_up_aabb(pre, o); shfl_down_aabb(suf, o); }
    if (ok) {
        store_aabb(table + 6ull * m * 6, b, pre);
        store_aabb(table + 7ull * m * 6, b, suf);
    }
    if (l == 0) store_aabb(table + 8ull * m * 6, g, suf);  // lane 0's suffix = the whole group
    Aabb v = t;
#pragma unroll
    for (int k = 1; k <= 5; ++k) {
        const int h = 1 << (k - 1);
        Aabb u;
#pragma unroll
        for (int c = 0; c < 3; ++c) { u.lo[c] = __shfl_down(v.lo[c], h, 64); u.hi[c] = __shfl_down(v.hi[c], h, 64); }
        if ((int)l + h < 64) aabb_union(v, u);  // entries past the group end are never queried
        if (ok) store_aabb(table + (uint64_t)k * m * 6, b, v);
    }
}

// K6 for the crossing nodes: box = suffix(l) U middle block totals U
// prefix(r).  MODE 1: the group tables above (ng <= kLdsTreeMaxBlocks);
// MODE 0: the global sparse table (levels built by k_sparse_near /
// k_sparse_far) for larger m; MODE 2 (m <= kSmallTreeBlocks: n <= 262K at
// 256-leaf blocks): each block's LDS segment tree over all m block totals
// (<= 48 KB), so no group-table launch -- the small scenes' crossing stage
// is three launches of a few us each, mostly latency.
template <int MODE>
__global__ __launch_bounds__(256) void k_refit_cross(const uint4* __restrict__ topo,
                                                     const float* __restrict__ prebuf, const float* __restrict__ sufbuf,
                                                     const float* __restrict__ table /* totals, or sparse levels */,
                                                     uint32_t m, const uint32_t* __restrict__ cross,
                                                     const uint32_t* __restrict__ cross_ctr, uint32_t cross_cap,
                                                     void* __restrict__ nodes, uint32_t n) {
    constexpr uint32_t T = kRefitT;
    extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
    Aabb* tree = reinterpret_cast<Aabb*>(s_raw);
    uint32_t pre[kCrossShards + 1];
    pre[0] = 0;
#pragma unroll
    for (uint32_t sh = 0; sh < kCrossShards; ++sh) pre[sh + 1] = pre[sh] + cross_ctr[sh];
    const uint32_t count = pre[kCrossShards];
    auto node_of = [&](uint32_t q) {
        uint32_t sh = 0;
#pragma unroll
        for (uint32_t j = 1; j < kCrossShards; ++j) sh += (q >= pre[j]) ? 1u : 0u;
        return cross[sh * cross_cap + (q - pre[sh])];
    };
    // a thread's first node is usually its only one (~20K crossing nodes at
    // 1M): its list entry and topology word are loaded while the block builds
    // its LDS tree, which does not depend on them (two dependent round trips
    // off the critical path)
    const uint32_t q0 = blockIdx.x * 256 + threadIdx.x;
    uint32_t i0 = q0 < count ? node_of(q0) : 0u;
    const uint32_t ng = MODE == 2 ? m : (m + kGroupBlocks - 1) / kGroupBlocks;  // the tree's leaves
    uint32_t P = 1;
    while (P < ng) P <<= 1;
    const float* gtot = MODE == 2 ? table : table + 8ull * m * 6;  // block totals / group totals
    if (MODE >= 1) {
        for (uint32_t j = threadIdx.x; j < P; j += 256) tree[P + j] = j < ng ? load_aabb(gtot, j) : aabb_empty();
    }
    uint4 tp0 = q0 < count ? topo[i0] : make_uint4(0u, 0u, 0u, 0u);
    if (MODE >= 1) {
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
    for (uint32_t q = q0; q < count; q += gridDim.x * 256) {
        const uint32_t i = q == q0 ? i0 : node_of(q);
        const uint4 tp = q == q0 ? tp0 : topo[i];
        const uint32_t l = tp.z, r = tp.w;
        if (l >= n || r >= n || l > r) continue;  // malformed topology: never read out of bounds
        Aabb box = load_aabb(sufbuf, l);
        aabb_union(box, load_aabb(prebuf, r));
        const uint32_t bl = l / T + 1, br = r / T;  // middle blocks [bl, br)
        if (bl < br) {
            if (MODE == 2) {
                uint32_t a = bl + P, b = br + P;  // blocks [bl, br)
                while (a < b) {
                    if (a & 1) aabb_union(box, tree[a++]);
                    if (b & 1) aabb_union(box, tree[--b]);
                    a >>= 1;
                    b >>= 1;
                }
            } else if (MODE == 1) {
                const uint32_t gl = bl / kGroupBlocks, gr = (br - 1) / kGroupBlocks;
                // inside one group and shorter than it: two entries of one in-group level (0..5); a
                // whole group (64 blocks) takes the other branch, as its suffix U prefix
                if (gl == gr && br - bl < kGroupBlocks) {
                    const uint32_t len = br - bl;
                    const uint32_t s = 31 - __clz((int)len);
                    const float* lvl = table + (uint64_t)s * m * 6;
                    aabb_union(box, load_aabb(lvl, bl));
                    aabb_union(box, load_aabb(lvl, br - (1u << s)));
                } else {
                    aabb_union(box, load_aabb(table + 7ull * m * 6, bl));      // in-group suffix
                    aabb_union(box, load_aabb(table + 6ull * m * 6, br - 1));  // in-group prefix
                    uint32_t a = gl + 1 + P, b = gr + P;                       // groups strictly between
                    while (a < b) {
                        if (a & 1) aabb_union(box, tree[a++]);
                        if (b & 1) aabb_union(box, tree[--b]);
                        a >>= 1;
                        b >>= 1;
                    }
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

// The greedy cut of wide_entries for a record built from
// global memory (k_wide_cross), with each entry's box and topology cached
// from ONE load of its record -- an internal entry's 32-B node record holds
// both (topo_of_node), a leaf entry's triangle record gives its box -- so the
// chain is X's topology word, its children's records, then one round of
// records per replacement: 4 dependent rounds instead of 7 (the generic form
// loads a picked entry's topology again after choosing it, and every final
// entry's box once more for the record).  Same entries, same boxes, so the
// same record bytes (tests: build parity compares every K7w record's
// containment and the BVH digests).
struct WEnt {
    Aabb box;
    uint32_t left, mx;  // topology (internal entries): left child, range end
};
// BF (r06, scenes up to kWentBfMaxN): branch-free, three 16-B loads from the
// entry's record -- an internal node's 32 B (its second word read twice) or a
// triangle record's 48 B -- so a round's two entries issue all their loads
// together instead of each waiting inside its own lane-divergent branch
// (the crossing stage -1 to -1.2 us from 70K to 1M); at 10M the stage is
// bound by its random lines, and the extra leaf-path loads cost 4 us
// (profiles/ab_went_bf_r06.log)
constexpr uint32_t kWentBfMaxN = 1u << 22;
template <bool BF>
__device__ __forceinline__ WEnt went_load(const void* nodes, const float4* tri_s, uint32_t i, uint32_t L0) {
    WEnt e;
    if constexpr (BF) {
        const bool in = i < L0;
        const float4* p = in ? reinterpret_cast<const float4*>(reinterpret_cast<const char*>(nodes) + (uint64_t)i * 32)
                             : tri_s + (uint64_t)(i - L0) * 3;
        const float4 A = p[0], B = p[1], C = p[in ? 1 : 2];
        const float t[9] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w, C.x};
        float lo[3], hi[3];
        tri_bounds(t, lo, hi);
        e.box.lo[0] = in ? A.x : lo[0]; e.box.lo[1] = in ? A.y : lo[1]; e.box.lo[2] = in ? A.z : lo[2];
        e.box.hi[0] = in ? A.w : hi[0]; e.box.hi[1] = in ? B.x : hi[1]; e.box.hi[2] = in ? B.y : hi[2];
        const uint32_t esc = __float_as_uint(B.w);
        e.left = in ? __float_as_uint(B.z) : 0u;
        e.mx = !in ? 0u : esc == RT_SENT ? L0 : esc >= L0 ? esc - L0 - 1 : esc - 1;
        return e;
    }
    if (i < L0) {
        const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(nodes) + (uint64_t)i * 32);
        const float4 A = p[0], B = p[1];
        e.box.lo[0] = A.x; e.box.lo[1] = A.y; e.box.lo[2] = A.z;
        e.box.hi[0] = A.w; e.box.hi[1] = B.x; e.box.hi[2] = B.y;
        const uint32_t esc = __float_as_uint(B.w);
        e.left = __float_as_uint(B.z);
        e.mx = esc == RT_SENT ? L0 : esc >= L0 ? esc - L0 - 1 : esc - 1;
    } else {
        e.box = leaf_box(tri_s, i - L0);
        e.left = 0u;
        e.mx = 0u;
    }
    return e;
}

template <int W, bool BF>
__device__ __forceinline__ void wide_record_g(uint32_t X, const uint4& tx, const Aabb& bx, uint32_t L0,
                                              const void* __restrict__ nodes, const float4* __restrict__ tri_s,
                                              uint4* __restrict__ wnodes) {
    // per entry: node index, box (6 floats), left child, range end, surface --
    // scalar arrays with static indices only (selects of whole structs went
    // through scratch)
    uint32_t node[W], el[W], em[W];
    float bb[6][W], ar[W];
    auto put = [&](int i, uint32_t nd, const WEnt& e) {
        node[i] = nd;
        el[i] = e.left;
        em[i] = e.mx;
#pragma unroll
        for (int c = 0; c < 3; ++c) { bb[c][i] = e.box.lo[c]; bb[3 + c][i] = e.box.hi[c]; }
        ar[i] = nd < L0 ? half_area(e.box) : 0.0f;
    };
    uint32_t l, r;
    kids_of(tx, L0, l, r);
    put(0, l, went_load<BF>(nodes, tri_s, l, L0));
    put(1, r, went_load<BF>(nodes, tri_s, r, L0));
#pragma unroll
    for (int i = 2; i < W; ++i) {
        node[i] = RT_SENT; el[i] = 0u; em[i] = 0u; ar[i] = 0.0f;
#pragma unroll
        for (int c = 0; c < 3; ++c) { bb[c][i] = bx.lo[c]; bb[3 + c][i] = bx.hi[c]; }
    }
#pragma unroll
    for (int step = 0; step < W - 2; ++step) {
        int best = -1;
        float ba = 0.0f;
#pragma unroll
        for (int i = 0; i < step + 2; ++i) {
            if (node[i] < L0) {
                if (best < 0 || ar[i] > ba) { best = i; ba = ar[i]; }
            }
        }
        if (best < 0) continue;  // no internal entry left (nor in the later steps)
        uint32_t pl = el[0], pm = em[0];
#pragma unroll
        for (int i = 1; i < step + 2; ++i) {
            pl = best == i ? el[i] : pl;
            pm = best == i ? em[i] : pm;
        }
        uint32_t c0, c1;
        kids_of(make_uint4(pl, 0u, 0u, pm), L0, c0, c1);
        const WEnt e0 = went_load<BF>(nodes, tri_s, c0, L0), e1 = went_load<BF>(nodes, tri_s, c1, L0);
        // shift the entries after `best` one slot right, then put the two children at best, best + 1
#pragma unroll
        for (int i = W - 1; i >= 1; --i) {
            if (i > best + 1) {
                node[i] = node[i - 1]; el[i] = el[i - 1]; em[i] = em[i - 1]; ar[i] = ar[i - 1];
#pragma unroll
                for (int c = 0; c < 6; ++c) bb[c][i] = bb[c][i - 1];
            }
        }
#pragma unroll
        for (int i = 0; i < W; ++i) {
            if (i == best) put(i, c0, e0);
            if (i == best + 1) put(i, c1, e1);
        }
    }
    store_wide<W>(wnodes, X, bx, node, [&](int i) {
        Aabb b;
#pragma unroll
        for (int c = 0; c < 3; ++c) { b.lo[c] = bb[c][i]; b.hi[c] = bb[3 + c][i]; }
        return b;
    }, L0);
}

// K7w records of the crossing internal nodes, once K6t has written their
// boxes (every box such a record needs is then final in `nodes`).
template <int W, bool BF>
__global__ __launch_bounds__(256) void k_wide_cross(const uint4* __restrict__ topo, const uint32_t* __restrict__ cross,
                                                    const uint32_t* __restrict__ cross_ctr, uint32_t cross_cap,
                                                    const void* __restrict__ nodes, const float4* __restrict__ tri_s,
                                                    uint32_t n, uint4* __restrict__ wnodes) {
    uint32_t pre[kCrossShards + 1];
    pre[0] = 0;
#pragma unroll
    for (uint32_t sh = 0; sh < kCrossShards; ++sh) pre[sh + 1] = pre[sh] + cross_ctr[sh];
    const uint32_t count = pre[kCrossShards];
    const uint32_t L0 = n - 1;
    for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q < count; q += gridDim.x * 256) {
        uint32_t sh = 0;
#pragma unroll
        for (uint32_t j = 1; j < kCrossShards; ++j) sh += (q >= pre[j]) ? 1u : 0u;
        const uint32_t X = cross[sh * cross_cap + (q - pre[sh])];
        if (X >= L0) continue;
        // the greedy cut, one record load per entry
        wide_record_g<W, BF>(X, topo[X], load_aabb_node(nodes, X), L0, nodes, tri_s, wnodes);
    }
}

template __global__ void k_refit_cross<1>(const uint4*, const float*, const float*, const float*, uint32_t, const uint32_t*, const uint32_t*, uint32_t, void*, uint32_t);
template __global__ void k_refit_cross<0>(const uint4*, const float*, const float*, const float*, uint32_t, const uint32_t*, const uint32_t*, uint32_t, void*, uint32_t);
template __global__ void k_refit_cross<2>(const uint4*, const float*, const float*, const float*, uint32_t, const uint32_t*, const uint32_t*, uint32_t, void*, uint32_t);

// ================================================================ launchers
static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

uint32_t bounds_grid(uint32_t n) { return n ? cdiv(n, 256 * kTrisPerThread) : 1u; }

// crossing-list shard capacity: blocks b = s (mod S) each own <= kRefitT entries
static uint32_t cross_cap(uint32_t m) { return cdiv(m, kCrossShards) * (uint32_t)kRefitT; }

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
    b.levels = std::max<uint32_t>(sparse_levels(b.m_blocks), 9u);  // group tables: levels 0..8
    b.nzero = kZEnd;
    hipError_t e;
#define RT_ALLOC(ptr, bytes) \
    if ((e = dev_alloc(&(ptr), (bytes))) != hipSuccess) { free_build(b); return e; }
    RT_ALLOC(b.tris, N * 36);
    RT_ALLOC(b.keys[0], N * 4);
    RT_ALLOC(b.keys[1], N * 4);
    RT_ALLOC(b.vals[0], N * 4);
    RT_ALLOC(b.vals[1], N * 4);
    RT_ALLOC(b.nodes, (2 * N - 1) * 32);
    RT_ALLOC(b.tri_s, N * 48);
    RT_ALLOC(b.parent, (2 * N - 1) * 4);
    RT_ALLOC(b.topo, N * 16);
    RT_ALLOC(b.wnodes, N * kWideRecMaxBytes);  // either arity (build.wide_arity)
    RT_ALLOC(b.prebuf, N * 24);
    RT_ALLOC(b.sufbuf, N * 24);
    RT_ALLOC(b.table, (uint64_t)b.levels * b.m_blocks * 24);
    RT_ALLOC(b.cross, (uint64_t)cross_cap(b.m_blocks) * kCrossShards * 4);
    RT_ALLOC(b.counts, (uint64_t)4 * b.ntiles * 256 * 4);
    RT_ALLOC(b.bstart, (kMsbBuckets + 4) * 4);
    RT_ALLOC(b.partials, (uint64_t)bounds_grid((uint32_t)N) * 24);
    RT_ALLOC(b.params, sizeof(BuildParams));
    RT_ALLOC(b.zero, (uint64_t)kZAlloc * 4);
#undef RT_ALLOC
    if ((e = hipMemset(b.zero, 0, (uint64_t)kZAlloc * 4)) != hipSuccess) { free_build(b); return e; }
    return hipSuccess;
}

void free_build(BuildBufs& b) {
    void* ps[] = {b.tris, b.keys[0], b.keys[1], b.vals[0], b.vals[1], b.nodes, b.tri_s, b.parent, b.topo, b.wnodes,
                  b.prebuf, b.sufbuf, b.table, b.cross, b.counts, b.bstart, b.partials, b.params, b.zero};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    b = BuildBufs{};
}

hipError_t launch_bounds_only(const float* tris, uint32_t n, float* partials, BuildParams* params, hipStream_t s) {
    RT_KLAUNCH(k_bounds, dim3(bounds_grid(n)), dim3(256), 0, s, tris, n, partials, (uint32_t*)nullptr, 0u);
    RT_KLAUNCH(k_bounds_final, dim3(1), dim3(256), 0, s, partials, bounds_grid(n), params);
    return hipGetLastError();
}

static hipError_t launch_morton_impl(const float* tris, uint32_t n, BuildParams* params, const float* partials,
                                     uint32_t nb, uint32_t* keys, uint32_t* vals, uint32_t* ghist, uint32_t* counts0,
                                     hipStream_t s, bool msb = false) {
    if (!n) return hipSuccess;
    if (msb)
        RT_KLAUNCH(k_morton<true>, dim3(sort_tiles(n)), dim3(kSortThreads), 0, s, tris, n, params, partials, nb,
                           keys, vals, ghist, counts0);
    else
        RT_KLAUNCH(k_morton<false>, dim3(sort_tiles(n)), dim3(kSortThreads), 0, s, tris, n, params, partials,
                           nb, keys, vals, ghist, counts0);
    return hipGetLastError();
}

hipError_t launch_morton(const float* tris, uint32_t n, const BuildParams* params, uint32_t* keys,
                         uint32_t* vals, uint32_t* ghist, uint32_t* counts0, hipStream_t s) {
    return launch_morton_impl(tris, n, const_cast<BuildParams*>(params), nullptr, 0, keys, vals, ghist, counts0, s);
}

hipError_t launch_leaf_nodes(const float4* tri_s, uint32_t n, void* nodes, hipStream_t s) {
    if (!n) return hipSuccess;
    RT_KLAUNCH(k_leaf_nodes, dim3(cdiv(n, 256)), dim3(256), 0, s, tri_s, n, nodes);
    return hipGetLastError();
}

hipError_t launch_leaf_tris(const void* nodes, const float* tris, uint32_t n, float4* tri_s, hipStream_t s) {
    if (!n) return hipSuccess;
    RT_KLAUNCH(k_leaf_tris, dim3(cdiv(n, 256)), dim3(256), 0, s, nodes, tris, n, tri_s);
    return hipGetLastError();
}

hipError_t launch_karras(const uint32_t* keys, const uint32_t* svals, const float* tris, uint32_t n, uint4* topo,
                         uint32_t* parent, void* nodes, float4* tri_s, hipStream_t s) {
    if (!n) return hipSuccess;
    RT_KLAUNCH(k_karras_leaves, dim3(cdiv(n, 256)), dim3(256), 0, s, keys, svals, tris, n, topo, parent, nodes,
                       tri_s);
    return hipGetLastError();
}

// K6t + K7w for the nodes whose range crosses a refit block (after k_topo_refit).
// k_refit_cross<true>'s dynamic LDS above 64 KB needs the attribute once per
// device (a process may drive several devices from several threads).
static hipError_t ensure_cross_attr() {
    static std::once_flag once[kMaxDevices];
    static hipError_t err[kMaxDevices];
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
    std::call_once(once[dev], [dev] {
        err[dev] = hipFuncSetAttribute((const void*)k_refit_cross<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       2 * kLdsTreeMaxBlocks * (int)sizeof(Aabb));
    });
    return err[dev];
}

// grids of the crossing stage: a crossing node is a short chain of dependent
// global loads, so more threads in flight beat each block's LDS segment-tree
// setup (profiles/ab_cross_grid_r02.log: 64/64 blocks 28.3 us, 128/256 20.0 us)
#ifndef RT_CROSS_GRID
#define RT_CROSS_GRID 128
#endif
#ifndef RT_WCROSS_GRID
#define RT_WCROSS_GRID 256
#endif
// Crossing nodes are short chains of dependent loads, one node per thread
// at a time: a grid that gives every node its own thread (about 11 per refit
// block: ~2 above the block level and ~log2(kRefitT) straddling each block
// boundary) instead of looping over them.
#ifndef RT_XGRID_PER_BLOCK
#define RT_XGRID_PER_BLOCK 12
#endif
// MODE 2 of k_refit_cross up to this many refit blocks (2 x 1024 x 24 B = 48 KB of LDS per block)
constexpr uint32_t kSmallTreeBlocks = 1024;
static uint32_t cross_grid(uint32_t m, uint32_t floor_blocks) {
    return std::min<uint32_t>(4096u, std::max<uint32_t>(floor_blocks, cdiv(RT_XGRID_PER_BLOCK * m, 256)));
}

static hipError_t launch_cross(const BuildBufs& b, uint32_t n, uint32_t arity, hipStream_t s) {
    const uint32_t m = cdiv(n, kRefitT);
    if (m <= 1) return hipGetLastError();
    const uint32_t ng = cdiv(m, kGroupBlocks);
    // up to kSmallTreeBlocks refit blocks: every block total in each block's LDS tree, no group tables
    // (r05: bunny/Sponza substitutes' crossing stage 18.1-19.2 -> 15.2-17.2 us, profiles/ab_cross_small_r05.log)
    if (m <= kSmallTreeBlocks) {
        uint32_t P = 1;
        while (P < m) P <<= 1;
        RT_KLAUNCH(k_refit_cross<2>, dim3(cross_grid(m, RT_CROSS_GRID)), dim3(256), 2ull * P * sizeof(Aabb), s, b.topo,
                   b.prebuf, b.sufbuf, b.table, m, b.cross, b.zero + kZCrossCtr, cross_cap(m), b.nodes, n);
    } else if (ng <= (uint32_t)kLdsTreeMaxBlocks) {
        uint32_t P = 1;
        while (P < ng) P <<= 1;
        const size_t lds = 2ull * P * sizeof(Aabb);
        const hipError_t e = ensure_cross_attr();
        if (e != hipSuccess) return e;
        RT_KLAUNCH(k_group_tables, dim3(ng), dim3(kGroupBlocks), 0, s, b.table, m);
        RT_KLAUNCH(k_refit_cross<1>, dim3(cross_grid(m, RT_CROSS_GRID)), dim3(256), lds, s, b.topo, b.prebuf, b.sufbuf,
                   b.table, m, b.cross, b.zero + kZCrossCtr, cross_cap(m), b.nodes, n);
    } else {
        const uint32_t L = sparse_levels(m);
        RT_KLAUNCH(k_sparse_near, dim3(cdiv(m, 256)), dim3(256), 0, s, b.table, m, L);
        if (L > kSparseNear + 1) RT_KLAUNCH(k_sparse_far, dim3(cdiv(m, 256)), dim3(256), 0, s, b.table, m, L);
        RT_KLAUNCH(k_refit_cross<0>, dim3(cross_grid(m, 256)), dim3(256), 0, s, b.topo, b.prebuf, b.sufbuf, b.table, m,
                           b.cross, b.zero + kZCrossCtr, cross_cap(m), b.nodes, n);
    }
#define RT_WCROSS(W, BF)                                                                                       \
    RT_KLAUNCH((k_wide_cross<W, BF>), dim3(cross_grid(m, RT_WCROSS_GRID)), dim3(256), 0, s, b.topo, b.cross,      \
               b.zero + kZCrossCtr, cross_cap(m), b.nodes, b.tri_s, n, b.wnodes)
    const bool bf = n <= kWentBfMaxN;
    if (arity == 8 && bf) RT_WCROSS(8, true);
    else if (arity == 8) RT_WCROSS(8, false);
    else if (bf) RT_WCROSS(4, true);
    else RT_WCROSS(4, false);
#undef RT_WCROSS
    return hipGetLastError();
}

// K4 + K5 + K6-local + K7w-local (k_topo_refit) over sorted keys/vals in
// keys[0]/vals[0]; expects the crossing-list counters zeroed (K0 does it).
static hipError_t launch_topo_blocks(const BuildBufs& b, uint32_t n, uint32_t arity,
                                     uint32_t block0, uint32_t nblocks, hipStream_t s,
                                     uint32_t* host_flags = nullptr, const uint32_t* bstart = nullptr) {
    const uint32_t* fsrc = host_flags ? b.zero + kZDense : nullptr;
    const uint32_t m = cdiv(n, kRefitT);
    if (arity == 8)
        RT_KLAUNCH(k_topo_refit<8>, dim3(nblocks), dim3(kRefitT), 0, s, b.keys[0], b.vals[0], b.tris, n,
                           b.topo, (uint32_t*)nullptr, b.nodes, b.tri_s, b.prebuf, b.sufbuf, b.table, b.cross,
                           b.zero + kZCrossCtr, cross_cap(m), b.wnodes, block0, fsrc, host_flags, bstart);
    else
        RT_KLAUNCH(k_topo_refit<4>, dim3(nblocks), dim3(kRefitT), 0, s, b.keys[0], b.vals[0], b.tris, n,
                           b.topo, (uint32_t*)nullptr, b.nodes, b.tri_s, b.prebuf, b.sufbuf, b.table, b.cross,
                           b.zero + kZCrossCtr, cross_cap(m), b.wnodes, block0, fsrc, host_flags, bstart);
    return hipGetLastError();
}

// bstart (nullable): the [1025] bucket starts of the keys' top 10 bits (an
// MSB or gather sort wrote them), for the long-range nodes' closed form
static hipError_t launch_topo_local(const BuildBufs& b, uint32_t n, uint32_t arity,
                                    hipStream_t s, uint32_t* host_flags = nullptr, const uint32_t* bstart = nullptr) {
    if (!n) return hipSuccess;
    return launch_topo_blocks(b, n, arity, 0u, cdiv(n, kRefitT), s, host_flags, bstart);
}

hipError_t launch_refit_stage(const BuildBufs& b, uint32_t n, hipStream_t s) {
    hipError_t e = hipMemsetAsync(b.zero + kZCrossCtr, 0, kCrossShards * 4, s);
    if (e != hipSuccess) return e;
    if ((e = launch_topo_local(b, n, b.warity, s)) != hipSuccess) return e;
    return n ? launch_cross(b, n, b.warity, s) : hipSuccess;
}

// ------------------------------------------- distributed build
// The per-rank device phases of rt_dbuild_* (DESIGN.md "Distributed build");
// the exchanges between them are the caller's.  Every phase runs the build's
// own kernels on a slice or a block range, so each value it produces is the
// one the single-GPU build computes.

// centroid bounds of tris[lo, lo + cnt) -> b.params (lo, hi; inv of the slice)
hipError_t launch_dbuild_bounds(const BuildBufs& b, uint32_t lo, uint32_t cnt, hipStream_t s) {
    RT_KLAUNCH(k_bounds, dim3(bounds_grid(cnt)), dim3(256), 0, s, b.tris + (uint64_t)lo * 9, cnt, b.partials,
                       (uint32_t*)nullptr, 0u);
    RT_KLAUNCH(k_bounds_final, dim3(1), dim3(256), 0, s, b.partials, bounds_grid(cnt), b.params);
    return hipGetLastError();
}

// Morton codes of tris[lo, lo + cnt) against the global bounds reduced from
// every rank's box (boxes: nboxes x {lo[3], hi[3]}, device) into
// keys[1]/vals[1] (vals = global indices), and the [1024] top-10-bit bucket
// histogram into ghist (the caller then sorts the slice: launch_dbuild_sort).
hipError_t launch_dbuild_keys(const BuildBufs& b, uint32_t lo, uint32_t cnt, const float* boxes, uint32_t nboxes,
                              hipStream_t s) {
    uint32_t* ghist = b.zero + kZHist;
    hipError_t e = hipMemsetAsync(ghist, 0, 1024 * 4, s);
    if (e != hipSuccess) return e;
    // block 0 also stores the global lo/hi/inv into params (rt_bvh_read)
    RT_KLAUNCH(k_morton<true>, dim3(std::max(1u, sort_tiles(cnt))), dim3(kSortThreads), 0, s,
                       b.tris + (uint64_t)lo * 9, cnt, b.params, boxes, nboxes, b.keys[1], b.vals[1], ghist, b.counts,
                       lo);
    return hipGetLastError();
}

// stable LSB sort of keys[0]/vals[0][0, cnt) (scratch keys[1]/vals[1]); the
// digit histograms go to ghist/counts (their previous contents are dead)
hipError_t launch_dbuild_sort(uint32_t* keys[2], uint32_t* vals[2], uint32_t cnt, const BuildBufs& b, hipStream_t s) {
    if (cnt <= 1) return hipSuccess;
    uint32_t* ghist = b.zero + kZHist;
    hipError_t e = hipMemsetAsync(ghist, 0, 1024 * 4, s);
    if (e != hipSuccess) return e;
    const uint64_t cs = (uint64_t)sort_tiles(b.cap_n ? b.cap_n : 1) * 256;
    uint32_t* counts[4] = {b.counts, b.counts + cs, b.counts + 2 * cs, b.counts + 3 * cs};
    if ((e = launch_digit_hist(keys[0], cnt, ghist, s)) != hipSuccess) return e;
    if ((e = launch_tile_hist0(keys[0], cnt, counts[0], s)) != hipSuccess) return e;
    return launch_sort(keys, vals, cnt, ghist, counts, s);
}

// K4 + K5 + K6-local + K7w-local over refit blocks [block0, block0 + nblocks)
// of the full sorted keys/vals in keys[0]/vals[0]
hipError_t launch_dbuild_subtrees(const BuildBufs& b, uint32_t n, uint32_t block0, uint32_t nblocks, hipStream_t s) {
    hipError_t e = hipMemsetAsync(b.zero + kZCrossCtr, 0, kCrossShards * 4, s);
    if (e != hipSuccess || !n || !nblocks) return e;
    return launch_topo_blocks(b, n, b.warity, block0, nblocks, s);
}

uint32_t dbuild_cross_cap(uint32_t n) { return cross_cap(cdiv(n ? n : 1, kRefitT)); }
uint32_t refit_blocks(uint32_t n) { return n ? cdiv(n, kRefitT) : 0u; }

// K6t + K7w of every crossing node, with the crossing list and counters
// (b.cross / zero + kZCrossCtr) and every share's blocks in place
hipError_t launch_dbuild_merge(const BuildBufs& b, uint32_t n, hipStream_t s) {
    return n ? launch_cross(b, n, b.warity, s) : hipSuccess;
}

// The build's sort for this n and config: 0 = the 4-pass LSB sort, 1 = the
// MSB scatter + bucket sort, 2 = the tile-bucketed gather sort (the default).
// A scene whose first MSB/gather build found a bucket beyond one block's LDS
// sort (sort_mode 2 for that sort) keeps the LSB sort; one whose gather probe
// found clustered bins only (gather_off) moves on to the MSB sort.
uint32_t build_sort_kind(const BuildBufs& b, uint32_t n, const TraceConfig& cfg) {
    if (n < 2 || n > kMsbBigMaxN || cfg.sort_msb == 0) return 0;
    if (cfg.sort_msb == 2 && !gather_sort_fits(n)) return 0;
    const uint32_t want = cfg.sort_msb == 2 && b.gather_off ? 1u : cfg.sort_msb;  // clustered bins: MSB
    if (b.sort_mode == 2 && b.sort_mode_of == want) return 0;
    return want;
}

// block shapes of K1-TB (a 4096-key tile on 512 threads x 8 triangles, or
// 1024 x 4 / 256 x 16): fused (FUSED = one block per CU at 1M) and unfused
#ifndef RT_K1F_NT
#define RT_K1F_NT 512
#endif
#ifndef RT_K1U_NT
#define RT_K1U_NT 512
#endif
std::mutex& fused_gate(int device) {
    static std::mutex m[kMaxDevices];
    return m[device >= 0 && device < kMaxDevices ? device : 0];
}

// Co-residency of k_morton_tb<true>'s grid (one block per sort tile): the
// occupancy API's blocks per CU, less one (MI355X_MICROARCH.md: the API can
// be one block per CU high), times the CUs, must hold every tile -- the grid
// barrier would otherwise wait for blocks that cannot start (it gives up
// after ~100 ms and flags it rather than hang).
bool fused_k01_fits(uint32_t n) {
    static std::once_flag once[kMaxDevices];
    static uint32_t cap[kMaxDevices];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return false;
    std::call_once(once[dev], [dev] {
        int per_cu = 0, cus = 0;
        cap[dev] = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu,
                                                         reinterpret_cast<const void*>(k_morton_tb<true, RT_K1F_NT>),
                                                         RT_K1F_NT, 0) != hipSuccess)
            return;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return;
        cap[dev] = per_cu > 1 ? (uint32_t)(per_cu - 1) * (uint32_t)cus : 0u;
    });
    return n >= 2 && sort_tiles(n) <= cap[dev];
}

hipError_t launch_build(const BuildBufs& b, uint32_t n, hipStream_t s, BuildEvents* ev, bool stages,
                        const TraceConfig& cfg, uint32_t* probed, bool allow_fused, bool* fused_out,
                        uint32_t* host_flags) {
    hipError_t e;
    if (probed) *probed = 0;
    if (fused_out) *fused_out = false;
    auto rec = [&](int i) -> hipError_t {
        return (ev && (stages || i == 0 || i == 6)) ? hipEventRecord(ev->e[i], s) : hipSuccess;
    };
    const uint32_t kind = build_sort_kind(b, n, cfg);
    // fuse_k01 == 2 (tests): fused even when the grid cannot be co-resident
    const bool fused = kind == 2 && allow_fused && cfg.fuse_k01 && (cfg.fuse_k01 == 2 || fused_k01_fits(n));
    if ((e = rec(0)) != hipSuccess) return e;
    if (!fused) {
        RT_KLAUNCH(k_bounds, dim3(bounds_grid(n)), dim3(256), 0, s, b.tris, n, b.partials, b.zero, kZEnd);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if ((e = rec(1)) != hipSuccess) return e;
    const uint64_t cs = (uint64_t)sort_tiles(n) * 256;
    uint32_t* counts[4] = {b.counts, b.counts + cs, b.counts + 2 * cs, b.counts + 3 * cs};
    if (!n) RT_KLAUNCH(k_bounds_final, dim3(1), dim3(256), 0, s, b.partials, 1u, b.params);
    // the scene's first build with this sort: the verdict on its bucket sizes
    // decides its later builds' sort (the host reads kZDense afterwards)
    const bool probe = kind != 0 && !(b.sort_mode != 0 && b.sort_mode_of == kind);
    if (kind == 2 && fused) {
        const FuseArgs fu{b.zero, kZEnd, b.zero + kZBar, b.zero + kZFuseErr,
                          reinterpret_cast<float*>(b.zero + kZBox)};
        RT_KLAUNCH((k_morton_tb<true, RT_K1F_NT>), dim3(sort_tiles(n)), dim3(RT_K1F_NT), 0, s, b.tris, n, b.params, b.partials,
                   sort_tiles(n), b.keys[1], probe ? b.zero + kZHist : nullptr, b.counts, fu);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (fused_out) *fused_out = true;
    } else if (kind == 2) {
        if (n) RT_KLAUNCH((k_morton_tb<false, RT_K1U_NT>), dim3(sort_tiles(n)), dim3(RT_K1U_NT), 0, s, b.tris, n, b.params,
                          b.partials, bounds_grid(n), b.keys[1], probe ? b.zero + kZHist : nullptr, b.counts,
                          FuseArgs{});
        if ((e = hipGetLastError()) != hipSuccess) return e;
    } else if ((e = launch_morton_impl(b.tris, n, b.params, b.partials, bounds_grid(n), b.keys[0], b.vals[0],
                                       b.zero + kZHist, counts[0], s, kind == 1)) != hipSuccess) {
        return e;
    }
    if ((e = rec(2)) != hipSuccess) return e;
    uint32_t* K[2] = {b.keys[0], b.keys[1]};
    uint32_t* V[2] = {b.vals[0], b.vals[1]};
    if (kind == 2) {
        // keys[1] = K1's tile-bucketed words -> keys[0]/vals[0]
        uint32_t* dense = probe ? b.zero + kZDense : nullptr;
        e = launch_sort_gather(b.keys[1], b.counts, n, b.zero + kZHist, b.keys[0], b.vals[0], b.zero + kZGatherFlags,
                               b.bstart, dense, s);
        if (e == hipSuccess && dense) {  // the LSB leg of a dense probe build: K1 again, in index order
            RT_KLAUNCH(k_morton<false>, dim3(sort_tiles(n)), dim3(kSortThreads), 0, s, b.tris, n, b.params,
                       (const float*)nullptr, 0u, b.keys[0], b.vals[0], b.zero + kZHist4, counts[0], 0u,
                       Gate{dense, 1u});
            if ((e = hipGetLastError()) == hipSuccess)
                e = launch_sort_lsb_gated(K, V, n, b.zero + kZHist4, b.counts, dense, s);
        }
    } else if (kind == 1 && probe) {  // both sorts, gated on the bucket totals
        // scratch for the chunked tile scan (n > kMsbMaxN): the parent array,
        // which the build does not write (ceil(tiles/32) x 1024 words <= 2n - 1)
        e = launch_sort_probe(K, V, n, b.zero + kZHist, b.counts, b.bstart, b.parent, b.zero + kZHist4,
                              b.zero + kZDense, s);
    } else if (kind == 1) {
        e = launch_sort_msb(K, V, n, b.zero + kZHist, b.counts, b.bstart, b.parent, s);
    } else {
        e = launch_sort(K, V, n, b.zero + kZHist, counts, s);
    }
    if (e != hipSuccess) return e;
    if (probe && probed) *probed = kind;
    if ((e = rec(3)) != hipSuccess) return e;
    // bucket starts: written by the MSB/gather sort (a dense probe build's LSB
    // leg leaves them stale: that build searches as before)
    const uint32_t* bst = (kind != 0 && !probe) ? b.bstart : nullptr;
    if ((e = launch_topo_local(b, n, b.warity, s, host_flags, bst)) != hipSuccess) return e;
    if ((e = rec(4)) != hipSuccess) return e;
    if (n && (e = launch_cross(b, n, b.warity, s)) != hipSuccess) return e;
    if ((e = rec(5)) != hipSuccess) return e;
    if ((e = rec(6)) != hipSuccess) return e;  // K7w is fused into K4/K6 (records written with the boxes)
    return hipSuccess;
}

}  // namespace rt

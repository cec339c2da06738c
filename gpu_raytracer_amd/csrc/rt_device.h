// rt_device.h -- shared device-side definitions for the gfx950 hot path.
//
// Numeric contract: SURVEY.md §9.1.  Everything here is compiled with
// -ffp-contract=off (no FMA contraction) and HIP's default correctly rounded
// fp32 division; fminf/fmaxf lower to v_min_f32/v_max_f32 (v_min3/v_max3),
// whose NaN-ignoring, -0 < +0 semantics the CPU oracle restates (oracle
// rt_oracle.c orc_fmin/orc_fmax; probed on hardware by rt_stage_minmax).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define RT_SENT 0xFFFFFFFFu

namespace rt {

struct Tri9 { float v[9]; };

struct Aabb { float lo[3], hi[3]; };

__device__ __forceinline__ void aabb_union(Aabb& a, const Aabb& b) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        a.lo[c] = fminf(a.lo[c], b.lo[c]);
        a.hi[c] = fmaxf(a.hi[c], b.hi[c]);
    }
}

__device__ __forceinline__ Aabb aabb_empty() {
    Aabb a;
#pragma unroll
    for (int c = 0; c < 3; ++c) { a.lo[c] = __builtin_inff(); a.hi[c] = -__builtin_inff(); }
    return a;
}

// §9.2: bmin = fmin(fmin(v0,v1),v2) per component, likewise bmax
__device__ __forceinline__ void tri_bounds(const float* t, float* bmin, float* bmax) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        bmin[c] = fminf(fminf(t[c], t[3 + c]), t[6 + c]);
        bmax[c] = fmaxf(fmaxf(t[c], t[3 + c]), t[6 + c]);
    }
}

// §9.3
__device__ __forceinline__ uint32_t expand10(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

// §9.7
__device__ __forceinline__ uint32_t pcg_hash(uint32_t x) {
    uint32_t st = x * 747796405u + 2891336453u;
    uint32_t w = ((st >> ((st >> 28u) + 4u)) ^ st) * 277803737u;
    return (w >> 22u) ^ w;
}

// Build-time scalar parameters written by K0 (bounds) for K1 (Morton).
// A kernel's run condition on a device word written by an earlier kernel of
// the same stream (the first build of a scene runs both sorts, each gated on
// the MSB scan's verdict, launch_build): p = nullptr runs unconditionally.
struct Gate {
    const uint32_t* p = nullptr;
    uint32_t want = 0;
};
__device__ __forceinline__ bool gated_off(const Gate& g) { return g.p && *g.p != g.want; }

struct BuildParams {
    float lo[3], hi[3], inv[3];
    uint32_t pad[7];
};

// Morton/sort geometry shared by host and device.
constexpr int kSortThreads = 512;
constexpr int kSortItems = 8;
constexpr int kSortTile = kSortThreads * kSortItems;   // 4096 keys / tile
constexpr uint32_t kPrefixInKernelMaxTiles = 256;      // <= 1M keys: cross-tile prefix inside k_scatter
// MSB bucket sort (sort_kernels.hip): bucket = key >> kMsbShift of the 30-bit
// Morton keys, used by the build for 2 <= n <= kMsbBigMaxN
constexpr uint32_t kMsbShift = 20;
constexpr uint32_t kMsbBuckets = 1024;
constexpr uint32_t kMsbMaxN = 512u * kSortTile;
// above kMsbMaxN (the 10M path) the same two levels with a chunked tile scan
// and 1024-thread bucket sorts of up to 12288 keys (sort_kernels.hip); a
// uniform soup's buckets hold n/1024 +- a few sigma keys
constexpr uint32_t kMsbBigMaxN = 12u * 1000u * 1000u;
// leaves per k_topo_refit block: 256 since r05 (with the group-table crossing
// stage, 10M build 1123.7 -> 1103.2 us, 1M 139.5 -> 138.7 us;
// profiles/ab_refit_t256_r05.log); 512 = the r04 layout (tools/build_exp.sh)
#ifndef RT_REFIT_T
#define RT_REFIT_T 256
#endif
constexpr int kRefitT = RT_REFIT_T;                     // leaves per refit block
constexpr int kLdsTreeMaxBlocks = 2048;                // K6t LDS segment-tree capacity

// ---- K7w wide (4-ary) trace tree, derived from the binary tree after K6.
// Record X (one per binary internal node X, 64 B) holds X's children with
// every internal child replaced by its two children: 2-4 entries in §9.7
// preorder.  Child boxes are quantized to 8 bits per plane on a power-of-two
// grid anchored at X.lo, rounded OUTWARD and verified at build time with the
// trace kernel's own arithmetic (wide_plane), so every quantized box
// contains the exact box.
//   w0 = {origin.x, origin.y, origin.z, meta}  meta: e+127 per axis in bytes
//        0..2; byte 3 = valid-child mask << 4 | wild (non-finite: every
//        valid child counts as hit)
//   w1 = {qlo.x[4], qlo.y[4], qlo.z[4], qhi.x[4]}  (byte i = child i)
//   w2 = {qhi.y[4], qhi.z[4], ref0, ref1}
//   w3 = {ref2, ref3, 0, 0}        ref = internal X, or kWideLeaf | k
constexpr uint32_t kWideLeaf = 0x80000000u;
constexpr uint32_t kWideWild = 1u;
// A wild record (build.wide_arity 4 and 8) also carries exponent bytes 255:
// its grid step is +inf, so the trace's slack is infinite and every valid
// child counts as hit whatever the planes say (record_test).
constexpr uint32_t kWideWildExp = 255u;
// per-ray LDS stack entries (+1 spare slot, 6 B each, x 256 threads = 22.5 KB
// per workgroup: 7 workgroups per CU fit the 160 KB of LDS);
// overflow -> exact binary traversal from the overflowing record
#ifndef RT_WIDE_STACK
#define RT_WIDE_STACK 14
#endif
constexpr int kWideStack = RT_WIDE_STACK;

// ---- K7w8: the 8-ary form (build.wide_arity = 8, SURVEY.md §8(f) row 1's
// "4/8-wide").  Record X holds up to 8 entries of X's greedy
// largest-surface cut (2-8 entries in §9.7 preorder), 96 B:
//   w0 = {origin.x, origin.y, origin.z, meta}  meta: e+127 per axis in bytes
//        0..2 (255 on every axis: wild); byte 3 = valid-child mask
//   w1 = {qlo.x[0..3], qlo.x[4..7], qlo.y[0..3], qlo.y[4..7]}
//   w2 = {qlo.z[0..3], qlo.z[4..7], qhi.x[0..3], qhi.x[4..7]}
//   w3 = {qhi.y[0..3], qhi.y[4..7], qhi.z[0..3], qhi.z[4..7]}
//   w4 = {ref0..ref3}, w5 = {ref4..ref7}
// A traversal step over it replaces up to three binary levels (two for the
// 4-ary form): the heaviest rays' dependent fetch chains are ~25 % shorter
// (tests/tools/wide_sim.py).  Its per-ray stacks hold 18 entries (a record pushes
// up to 7).
template <int W> struct WideFmt;
template <> struct WideFmt<4> {
    static constexpr uint32_t words = 4, bytes = 64;
    static constexpr int stack = kWideStack;
};
template <> struct WideFmt<8> {
    static constexpr uint32_t words = 6, bytes = 96;
    static constexpr int stack = 18;
};
// 4-ary stacks of 64-thread blocks (one rank's tiles of a multi-GPU frame):
// 16 entries.  A ray whose stack overflows finishes in the binary traversal,
// uncapped by the heavy-ray queue, and one such ray sets its rank's time: on
// the bench's orbit a few frames hold overflowing rays, and the rank that owns
// their tiles took 0.19-0.25 ms against 0.12 for the others
// (profiles/ab_stack_depth_r04.log: 20 entries fixed it).  16 entries fix it
// as well and leave the 1-spp tile kernel (77 VGPRs) its 6 waves per SIMD:
// 6.4 KB per block, 24 blocks per CU (profiles/ab_tile_spp1_stack16_r04.log).
// The 256-thread full-frame kernels keep 14 (16-24 entries cost them a block
// per CU or more, and overflows are rare in a full frame's throughput).
#ifndef RT_WIDE_STACK64
#define RT_WIDE_STACK64 16
#endif
template <int W, int NT> struct StackOf {
    static constexpr int v = (W == 4 && NT == 64) ? RT_WIDE_STACK64 : WideFmt<W>::stack;
};
constexpr int kWideStackMax = (RT_WIDE_STACK64 > 18 && RT_WIDE_STACK64 > kWideStack) ? RT_WIDE_STACK64
                              : (kWideStack > 18 ? kWideStack : 18);
constexpr uint32_t kWideRecMaxBytes = 96;  // wnodes is allocated for either arity

// plane = origin + q * 2^e, rounded once: q * 2^e is exact (q < 2^8 and
// -126 <= e <= 119, so no overflow and an exact denormal at worst), hence
// the fma equals the separately rounded add.  scale = 2^e as a float.
__device__ __forceinline__ float wide_plane(float origin, uint32_t q, float scale) {
    return fmaf((float)q, scale, origin);
}
__device__ __forceinline__ float wide_scale(int e) { return __uint_as_float((uint32_t)(e + 127) << 23); }


}  // namespace rt

// ---- diagnostic phase stamps (separate -DRT_STAMPS build only; the shipped
// library executes none).  Thread 0 of each block writes s_memrealtime
// (100 MHz, chip-wide clock) into slot s of its 8-word record.
#ifdef RT_STAMPS
// one stamp array per translation unit (no relocatable device code)
static __device__ unsigned long long g_rt_stamps[1u << 20];
#define RT_STAMP(s)                                                          \
    do {                                                                     \
        if (threadIdx.x == 0) {                                              \
            __builtin_amdgcn_sched_barrier(0);                               \
            g_rt_stamps[(uint64_t)blockIdx.x * 8 + (s)] = __builtin_amdgcn_s_memrealtime(); \
            __builtin_amdgcn_sched_barrier(0);                               \
        }                                                                    \
    } while (0)
#define RT_STAMP_VAL(s, v)                                                   \
    do {                                                                     \
        if (threadIdx.x == 0) g_rt_stamps[(uint64_t)blockIdx.x * 8 + (s)] = (v); \
    } while (0)
// a second record set from block 65536 on (a kernel that runs before another
// stamped kernel of the same translation unit)
#define RT_STAMP_HI(s)                                                       \
    do {                                                                     \
        if (threadIdx.x == 0) {                                              \
            __builtin_amdgcn_sched_barrier(0);                               \
            g_rt_stamps[(65536ull + blockIdx.x) * 8 + (s)] = __builtin_amdgcn_s_memrealtime(); \
            __builtin_amdgcn_sched_barrier(0);                               \
        }                                                                    \
    } while (0)
#else
#define RT_STAMP_HI(s) do {} while (0)
#define RT_STAMP(s) do {} while (0)
#define RT_STAMP_VAL(s, v) do {} while (0)
#endif

// trace_kernels.hip -- K8 trace + K9 shade for gfx950.
//
// One thread per pixel; a 256-thread workgroup owns one 16x16-pixel image
// tile and each wave64 an 8x8 sub-tile, so the 64 rays that share an
// instruction stream are spatially coherent.  Per sample: raygen (§9.7),
// stackless escape-link traversal over 32-B nodes (two 16-B loads per node),
// Moller-Trumbore on the leaf's triangle, closest hit with strict '<'.
// K9 is fused: the thread averages its pixel's samples in order and writes
// RGBA8.  Tiles are dealt round-robin to ranks (tile t -> rank t mod P); with
// PACKED the rank writes its tiles compactly for the RCCL gather.
#include "rt_device.h"
#include "rt_launch.h"

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>

namespace rt {

#ifdef RT_STAMPS
hipError_t read_stamps_trace(void* out, size_t bytes) { return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rt_stamps), bytes); }
#endif

struct Cam { float eye[3], w00[3], du[3], dv[3]; };

// The image tile of one rank's slot: round-robin, tile t = rank + slot * P
// (the costly and cheap image bands spread over every rank).  The
// RT_EXP_TILE_BANDS diagnostic build (tools/build_exp.sh; wrong gathers,
// timing only) gives each rank a contiguous band of as many tiles instead,
// to price the round-robin deal's loss of locality (DESIGN.md, r06:
// profiles/bands_r06.log -- no per-ray gain, and the bands unbalance the ranks).
__device__ __forceinline__ uint32_t rank_tile(uint32_t rank, uint32_t slot, uint32_t nranks, uint32_t tilesX, uint32_t H) {
#ifdef RT_EXP_TILE_BANDS
    const uint32_t ntl = tilesX * ((H + 15) / 16);
    return rank * (ntl / nranks) + min(rank, ntl % nranks) + slot;
#else
    (void)tilesX;
    (void)H;
    return rank + slot * nranks;
#endif
}


__device__ __forceinline__ float dot3(const float* a, const float* b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
__device__ __forceinline__ void cross3(const float* a, const float* b, float* o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

// §9.7 Moller-Trumbore, two-sided, no epsilon, on precomputed edges
// e1 = v1-v0, e2 = v2-v0; writes t/u/v on a closer hit.
__device__ __forceinline__ bool intersect_e(const float* o, const float* d, const float* v0, const float* e1,
                                            const float* e2, float tb, float& tout, float& uout, float& vout) {
    float p[3], s[3], q[3];
    cross3(d, e2, p);
    const float det = dot3(e1, p);
    if (det == 0.0f) return false;
    const float inv = 1.0f / det;
#pragma unroll
    for (int c = 0; c < 3; ++c) s[c] = o[c] - v0[c];
    const float u = dot3(s, p) * inv;
    if (u < 0.0f || u > 1.0f) return false;
    cross3(s, e1, q);
    const float v = dot3(d, q) * inv;
    if (v < 0.0f || u + v > 1.0f) return false;
    const float t = dot3(e2, q) * inv;
    if (t <= 0.0f) return false;
    if (!(t < tb)) return false;
    tout = t; uout = u; vout = v;
    return true;
}

__device__ __forceinline__ bool intersect_tri(const float* o, const float* d, const float* tri, float tb,
                                              float& tout, float& uout, float& vout) {
    float e1[3], e2[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) { e1[c] = tri[3 + c] - tri[c]; e2[c] = tri[6 + c] - tri[c]; }
    return intersect_e(o, d, tri, e1, e2, tb, tout, uout, vout);
}

// §9.7 stackless escape-link traversal of one ray: an internal node is its
// 32-B record (two 16-B loads), a leaf its 48-B triangle record (box from the
// vertices, prim and escape link in the record's spare words), so a leaf
// costs one memory round trip for the box test and the Moller-Trumbore test
// together -- the §9.7 order, hence the same tests with the same operands.
// (Until r02 the build also wrote 32-B leaf nodes and a leaf's triangle test
// was deferred one step to share the escape node's round trip.)  A
// well-formed tree visits each node once; the guard and index checks only
// keep a malformed one from faulting.
//
// trace_ray_from resumes that loop at node `start` with the caller's
// tb/hu/hv/hp: exact whenever every leaf before `start` in preorder has been
// tested with §9.7's outcome (the wide traversal's overflow hand-off); a
// start below a culled ancestor only adds box tests that miss.
template <bool COUNT, bool ANY = false>
__device__ __forceinline__ void trace_ray_from(const char* __restrict__ nodes, const float4* __restrict__ tri_s,
                                               uint32_t n, const float* o, const float* d, uint32_t start, float& tb,
                                               float& hu, float& hv, uint32_t& hp, uint32_t& cn, uint32_t& ct,
                                               bool any = ANY) {
    float invd[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) invd[c] = 1.0f / d[c];
    const uint32_t L0 = n ? n - 1 : 0;
    const uint32_t total = n ? 2 * n - 1 : 0;
    uint32_t idx = start;
    // A leaf is read from its triangle record {v0, v1, v2, prim, esc}: its box
    // is tri_bounds of the vertices (the build writes no leaf nodes), and the
    // Moller-Trumbore test uses the same loads.
    for (uint32_t guard = 0; idx < total && guard <= total; ++guard) {
        if (COUNT) ++cn;
        float lo[3], hi[3], tv[9];
        uint32_t na, esc;
        const bool leaf = idx >= L0;
        if (leaf) {
            const float4* tp = tri_s + (uint64_t)(idx - L0) * 3;
            const float4 T0 = tp[0], T1 = tp[1], T2 = tp[2];
            tv[0] = T0.x; tv[1] = T0.y; tv[2] = T0.z; tv[3] = T0.w; tv[4] = T1.x;
            tv[5] = T1.y; tv[6] = T1.z; tv[7] = T1.w; tv[8] = T2.x;
            tri_bounds(tv, lo, hi);
            na = __float_as_uint(T2.y);
            esc = __float_as_uint(T2.z);
        } else {
            const float4* np = reinterpret_cast<const float4*>(nodes + (uint64_t)idx * 32);
            const float4 A = np[0], B = np[1];
            lo[0] = A.x; lo[1] = A.y; lo[2] = A.z; hi[0] = A.w; hi[1] = B.x; hi[2] = B.y;
            na = __float_as_uint(B.z);
            esc = __float_as_uint(B.w);
        }
        const float t0x = (lo[0] - o[0]) * invd[0], t1x = (hi[0] - o[0]) * invd[0];
        const float t0y = (lo[1] - o[1]) * invd[1], t1y = (hi[1] - o[1]) * invd[1];
        const float t0z = (lo[2] - o[2]) * invd[2], t1z = (hi[2] - o[2]) * invd[2];
        const float tn = fmaxf(fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z)), 0.0f);
        const float tf = fminf(fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z)), tb);
        const bool hit = tn <= tf;
        if (hit && leaf) {
            if (COUNT) ++ct;
            float t, u, v;
            if (intersect_tri(o, d, tv, tb, t, u, v)) {
                tb = t; hu = u; hv = v; hp = na;
                if (any) return;  // any-hit (shadow ray): the first hit ends the search
            }
        }
        idx = (hit && !leaf) ? na : esc;
    }
}

template <bool COUNT>
__device__ __forceinline__ void trace_ray(const char* __restrict__ nodes, const float4* __restrict__ tri_s,
                                          uint32_t n, const float* o, const float* d, float& tb, float& hu,
                                          float& hv, uint32_t& hp, uint32_t& cn, uint32_t& ct) {
    tb = __builtin_inff(); hu = 0.0f; hv = 0.0f; hp = RT_SENT;
    trace_ray_from<COUNT>(nodes, tri_s, n, o, d, n ? 0u : RT_SENT, tb, hu, hv, hp, cn, ct);
}

// §9.7 slab test of the box lo/hi against [0, tb]; tn out.
__device__ __forceinline__ bool slab_hit(const float* lo, const float* hi, const float* o, const float* invd, float tb,
                                         float& tn) {
    const float t0x = (lo[0] - o[0]) * invd[0], t1x = (hi[0] - o[0]) * invd[0];
    const float t0y = (lo[1] - o[1]) * invd[1], t1y = (hi[1] - o[1]) * invd[1];
    const float t0z = (lo[2] - o[2]) * invd[2], t1z = (hi[2] - o[2]) * invd[2];
    tn = fmaxf(fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z)), 0.0f);
    const float tf = fminf(fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z)), tb);
    return tn <= tf;
}

// Wide (4-ary) traversal over the K7w records, same hits as trace_ray.
//
// Why the result is identical, not just close: for a ray whose 1/d is
// finite on every axis the slab interval is monotone in the box, so a box
// that contains another never misses where the inner one hits (and a larger
// tb never turns a hit into a miss).  The quantized child boxes contain the
// exact ones, so every triangle §9.7 reaches is reached here, in the same
// preorder; the leaf itself is tested with its EXACT box (recomputed from
// the vertices with tri_bounds) against the current tb before
// Moller-Trumbore.  By induction over the preorder, each leaf sees the same
// tb as in §9.7, so the exact leaf test admits exactly the triangles §9.7
// tests and nothing else; extra subtrees entered through the looser
// quantized boxes contain only leaves whose exact test fails.  Rays with an
// infinite 1/d component (d exactly 0 on an axis, where NaN slabs break
// monotonicity) are traced by trace_ray; a ray whose stack would overflow
// at record X hands over to trace_ray_from(X) with its current tb -- every
// leaf before X in preorder is done and everything after X (the pending
// stack included) is X's subtree or lies on X's escape chain.
//
// One wide_step fetches at most one record (cur) and one triangle
// (pend, the leaf that precedes cur in preorder) with all loads in flight
// together, tests the triangle first and the record's four children second,
// so a step costs one memory round trip.  The children are tested without
// branches; hit children after the first are pushed (in reverse) with
// unconditional LDS writes into a spare slot and a predicated stack-pointer
// increment.  Stack entries carry the child's entry distance tn; an entry
// whose tn exceeds the (since shrunken) tb is skipped -- exactly the miss
// its re-test would give, since tn <= tf held when it was pushed.
//
// The stack lives in LDS, entry-major ([entry][thread], conflict-free):
// ref (4 B) + tn truncated to its upper 16 bits (2 B; tn >= +0, so the
// truncation rounds down and the skip test stays conservative).  Slot `cap`
// is the spare that takes the writes of children that are not pushed.
struct WRay {
    float d[3], invd[3], kn[3], kf[3];  // kn/kf: the record test's per-ray offsets (record_test)
    float tb, hu, hv, ctn;
    uint32_t hp, cur, pend, sp, steps;
    bool fin;  // 1/d finite on every axis: the wide traversal applies
#ifdef RT_STEPSTAMPS
    unsigned long long t1, t2;  // diagnostic: s_memtime after the pop and once the step's loads are back
#endif
};

#ifdef RT_STEPSTAMPS
// Diagnostic build only (tools/diag_steps.py): the shader clock at a point
// of the wide step, with every LDS read before it complete (MI355X guide
// "In-kernel stamps": one asm statement, the wait inside it).
#define RT_TSTAMP(v)                                                                        \
    do {                                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : : "memory");        \
        __builtin_amdgcn_sched_barrier(0);                                                  \
    } while (0)
#endif

// The scene box (the binary root's, internal node 0, for n >= 2): every
// record's origin and grid lie inside it, which bounds the record test's
// rounding per ray instead of per record (record_test).
struct SceneBox { float lo[3], hi[3]; };
__device__ __forceinline__ float uniform_f(float x) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}
__device__ __forceinline__ SceneBox scene_box(const void* nodes) {
    const float4* p = reinterpret_cast<const float4*>(nodes);
    const float4 a = p[0], b = p[1];  // the same address in every lane: kept in SGPRs
    return SceneBox{{uniform_f(a.x), uniform_f(a.y), uniform_f(a.z)}, {uniform_f(a.w), uniform_f(b.x), uniform_f(b.y)}};
}

// R.fin: 1/d finite on every axis and the record-test slack finite and
// small -- the wide traversal applies (else the binary one from the root).
__device__ __forceinline__ void wray_init(const float* o, const float* d, WRay& R, const SceneBox& sb) {
    bool ok = true;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        R.d[c] = d[c];
        const float inv = 1.0f / d[c];
        R.invd[c] = inv;
        const float ai = fabsf(inv);
        const float oi = o[c] * inv;
        // |a| = |(org - o) / d| for any record origin org in the scene box,
        // and 256 |B| = 256 * 2^e / |d| <= 4 * extent / |d| (quant_axis picks
        // 2^e <= extent / 64 unless 2^e = 2^-126)
        const float M = fmaxf(fabsf(sb.lo[c] - o[c]), fabsf(sb.hi[c] - o[c])) * ai;
        const float B256 = fmaxf((sb.hi[c] - sb.lo[c]) * 4.0f, 0x1p-118f) * ai;
        const float dl = fmaf((M + B256) + fabsf(oi), 0x1p-19f, 0x1p-125f);
        ok = ok && isfinite(inv) && dl < 0x1p90f;  // false for NaN and infinities too
        R.kn[c] = -oi - dl;
        R.kf[c] = -oi + dl;
    }
    R.fin = ok;
    R.tb = __builtin_inff(); R.hu = 0.0f; R.hv = 0.0f; R.hp = RT_SENT;
    R.cur = 0; R.pend = RT_SENT; R.ctn = 0.0f; R.sp = 0; R.steps = 0;
}

// §9.7 raygen of sample s of pixel (x, y)
__device__ __forceinline__ void ray_dir(const Cam& cam, uint32_t x, uint32_t y, uint32_t W, uint32_t spp, uint32_t s,
                                        float* d) {
    const uint32_t sidx = (y * W + x) * spp + s;
    float jx = 0.5f, jy = 0.5f;
    if (s > 0) {
        const uint32_t h = pcg_hash(sidx);
        jx = (float)(h >> 8) * 0x1p-24f;
        jy = (float)(pcg_hash(h) >> 8) * 0x1p-24f;
    }
    const float px = (float)x + jx, py = (float)y + jy;
#pragma unroll
    for (int c = 0; c < 3; ++c) d[c] = (cam.w00[c] + px * cam.du[c]) + py * cam.dv[c];
}

__device__ __forceinline__ void wray_setup(const Cam& cam, uint32_t x, uint32_t y, uint32_t W, uint32_t spp,
                                           uint32_t s, WRay& R, const SceneBox& sb) {
    float d[3];
    ray_dir(cam, x, y, W, spp, s, d);
    wray_init(cam.eye, d, R, sb);
}

__device__ __forceinline__ uint32_t bin_of(uint32_t ref, uint32_t L0) {
    return (ref & kWideLeaf) ? L0 + (ref & ~kWideLeaf) : ref;
}

// Conservative slab test of a record's quantized child boxes, in about a
// third of the VALU of the §9.7 formula (this is the traversal's inner loop,
// and the kernel is VALU-issue bound).  Child plane p = org + q*2^e, so §9.7's
// (p - o)*invd is computed as fma(q, B, A') with B = 2^e*invd and, per record
// and axis, A' = fma(org, invd, K) = (org - o)*invd -/+ dl (K = -o*invd -/+ dl
// per ray, R.kn / R.kf); each axis's near/far plane is picked once per record
// by the sign of invd (q_lo <= q_hi for every valid child).
//
// Exactness.  The internal-node tests only prune; the traversal stays exact
// as long as a child is entered whenever §9.7's test of the child's EXACT box
// b would hit (see the wide_step comment).  With a = (org - o)*invd (real),
// u = 2^-24: A' differs from a -/+ dl by <= u(|a| + 2|o*invd| + 2dl) (the
// roundings of o*invd, K and the fma); the child fma adds u|t| (|t| <= |a| +
// 255|B| + dl); §9.7's own two roundings 2u|t|; and the real plane org + q*2^e
// differs from its rounded value, which the build compared with b, by <=
// u(|a| + |o*invd| + 256|B|).  In total less than u(5|a| + 3|o*invd| +
// 1021|B| + 3dl) + denormal terms.  wray_init takes
//     dl = 2^-19 (M + 256 Bmax + |o*invd|) + 2^-125
// with M >= |a| and Bmax >= |B| for every record of the scene (its origin and
// grid lie in the scene box), 32x the bound's |a|, |o*invd| and 8x its |B|
// weight: tn_fast <= tn_97 and tf_fast >= tf_97, so a child §9.7 enters is
// always entered and the stack entry distance stays a lower bound of §9.7's.
// (The r01 form computed dl per record from the record's own A and B: 15
// more VALU per record for a slack ~2^-19 of the scene size narrower.)  A
// wild record (rt_device.h) has exponent bytes 255 and zero planes: B = +-inf,
// fma(0, inf, A') = NaN on every axis, and the NaN-ignoring min/max give
// tn = 0 <= tf = tb: every valid child is hit with entry distance 0.
//
// W = 8 (K7w8, rt_device.h): the same test over 8 children whose plane
// bytes sit in two words per plane.
template <int W>
__device__ __forceinline__ void record_test(const WRay& R, const uint4 (&w)[WideFmt<W>::words], bool (&hit)[W],
                                            float (&tn)[W]) {
    constexpr int QW = W / 4;
    const uint4 w0 = w[0];
    const float org[3] = {__uint_as_float(w0.x), __uint_as_float(w0.y), __uint_as_float(w0.z)};
    uint32_t qlo[3][QW], qhi[3][QW];
    if constexpr (W == 4) {
        qlo[0][0] = w[1].x; qlo[1][0] = w[1].y; qlo[2][0] = w[1].z;
        qhi[0][0] = w[1].w; qhi[1][0] = w[2].x; qhi[2][0] = w[2].y;
    } else {
        qlo[0][0] = w[1].x; qlo[0][QW - 1] = w[1].y; qlo[1][0] = w[1].z; qlo[1][QW - 1] = w[1].w;
        qlo[2][0] = w[2].x; qlo[2][QW - 1] = w[2].y; qhi[0][0] = w[2].z; qhi[0][QW - 1] = w[2].w;
        qhi[1][0] = w[3].x; qhi[1][QW - 1] = w[3].y; qhi[2][0] = w[3].z; qhi[2][QW - 1] = w[3].w;
    }
    float An[3], Af[3], B[3];
    uint32_t qn[3][QW], qf[3][QW];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float scl = __uint_as_float(((w0.w >> (8 * c)) & 0xFFu) << 23);  // 2^e
        B[c] = scl * R.invd[c];
        An[c] = fmaf(org[c], R.invd[c], R.kn[c]);
        Af[c] = fmaf(org[c], R.invd[c], R.kf[c]);
        const bool neg = R.invd[c] < 0.0f;
#pragma unroll
        for (int k = 0; k < QW; ++k) {
            qn[c][k] = neg ? qhi[c][k] : qlo[c][k];
            qf[c][k] = neg ? qlo[c][k] : qhi[c][k];
        }
    }
#pragma unroll
    for (int i = 0; i < W; ++i) {
        float tnear[3], tfar[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            tnear[c] = fmaf((float)((qn[c][i >> 2] >> (8 * (i & 3))) & 0xFFu), B[c], An[c]);
            tfar[c] = fmaf((float)((qf[c][i >> 2] >> (8 * (i & 3))) & 0xFFu), B[c], Af[c]);
        }
        tn[i] = fmaxf(fmaxf(fmaxf(tnear[0], tnear[1]), tnear[2]), 0.0f);
        const float tf = fminf(fminf(fminf(tfar[0], tfar[1]), tfar[2]), R.tb);
        hit[i] = tn[i] <= tf;
    }
}

// valid-child mask and child refs of a record (layouts: rt_device.h)
template <int W>
__device__ __forceinline__ uint32_t rec_mask(const uint4 (&w)[WideFmt<W>::words]) {
    return W == 4 ? (w[0].w >> 28) & 0xFu : w[0].w >> 24;
}
template <int W>
__device__ __forceinline__ uint32_t rec_ref(const uint4 (&w)[WideFmt<W>::words], int i) {
    if constexpr (W == 4) {
        return i == 0 ? w[2].z : i == 1 ? w[2].w : i == 2 ? w[3].x : w[3].y;
    } else {
        const uint4 v = w[4 + (i >> 2)];
        return (i & 3) == 0 ? v.x : (i & 3) == 1 ? v.y : (i & 3) == 2 ? v.z : v.w;
    }
}

template <int NT>
__device__ __forceinline__ void wide_pop(WRay& R, const uint32_t* sref, const uint16_t* stn) {
    if (R.sp == 0) { R.cur = RT_SENT; return; }
    --R.sp;
    R.cur = sref[R.sp * NT];
    R.ctn = __uint_as_float((uint32_t)stn[R.sp * NT] << 16);
}

// Returns 0 = more steps, 1 = done, 2 = finish with
// trace_ray_from(bin_of(R.cur)) (stack overflow at record R.cur, or the step
// guard of a malformed tree).
//
// MTF: Moller-Trumbore before the leaf-box test -- fewer instructions per
// step, more registers (84 vs 72 VGPRs: 5 waves per SIMD instead of 7).
// Used where waves run latency-bound (a rank's tiles, shadow rays:
// 4-6 % faster); the full-frame primary kernel, issue-bound at high
// occupancy, and path mode (3 % slower with it) keep the box test first
// (profiles/ab_mtfirst_r01.log).
// Buffer views of the wide records and the leaf triangle records (BUF
// steps): a step loads its record and its triangle with buffer loads whose
// offset is out of range -- zero returned, no memory access -- for a lane
// that needs neither, instead of branching around flat loads.  Without the
// branches the compiler has no phi copies of half-arrived registers to make
// and issues both loads before waiting for either: one round trip per step
// where the flat form (a copy of the triangle's registers before the record
// loads are issued) took two.  32-bit offsets: (n - 1) * 96 and n * 48 bytes
// must fit (n <= 2^26; the launcher uses the flat form above that).
struct WideMem {
    __amdgpu_buffer_rsrc_t wr, tr;
    uint32_t wbytes, tbytes;
};
constexpr uint32_t kBufMaxN = 1u << 26;

template <int W = 4>
__device__ __forceinline__ WideMem wide_mem(const uint4* wnodes, const float4* tri_s, uint32_t n) {
    WideMem m;
    m.wbytes = n >= 2 ? (n - 1) * WideFmt<W>::bytes : 0u;
    m.tbytes = n * 48u;
    m.wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(wnodes), 0, (int)m.wbytes, 0x00020000);
    m.tr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(tri_s), 0, (int)m.tbytes, 0x00020000);
    return m;
}
__device__ __forceinline__ uint4 bload_u4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ float4 bload_f4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ uint2 bload_u2(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
// the third word of a triangle record {v2.z, prim, esc, 0}: a step needs its
// first two only (8 B, two VGPRs in flight instead of four)
__device__ __forceinline__ float4 bload_tri2(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    const uint2 v = bload_u2(r, off);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), 0.0f, 0.0f);
}
// record word k of a W-ary record; a 4-ary record's last word {ref2, ref3, 0, 0}
// is loaded as 8 B
template <int W>
__device__ __forceinline__ uint4 bload_rec(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t k) {
    if (W == 4 && k == WideFmt<4>::words - 1) {
        const uint2 v = bload_u2(r, off);
        return make_uint4(v.x, v.y, 0u, 0u);
    }
    return bload_u4(r, off);
}

template <bool COUNT, int NT, bool ANY = false, bool MTF = false, bool BUF = false, int W = 4>
__device__ __forceinline__ int wide_step(WRay& R, const uint4* __restrict__ wnodes, const float4* __restrict__ tri_s,
                                         const float* o, uint32_t cap, uint32_t limit, uint32_t* sref, uint16_t* stn,
                                         uint32_t& cn, uint32_t& ct, bool any = ANY, const WideMem* M = nullptr) {
#ifdef RT_STEPSTAMPS
    R.t1 = R.t2 = 0ull;
#endif
    if (++R.steps > limit) return 2;
    if (R.pend == RT_SENT) {
        if (R.cur == RT_SENT) wide_pop<NT>(R, sref, stn);
        if (R.cur != RT_SENT && (R.cur & kWideLeaf)) {
            R.pend = R.cur;
            wide_pop<NT>(R, sref, stn);
        }
    }
    if (R.pend == RT_SENT && R.cur == RT_SENT) return 1;
    const bool node = R.cur != RT_SENT && !(R.cur & kWideLeaf);
    const bool leaf = R.pend != RT_SENT;
    // both addresses before any load: with a load in flight, a register
    // the compiler reuses for the second address would force a wait for the
    // first load, and the triangle and the record would cost two round trips
    constexpr uint32_t NW = WideFmt<W>::words;
    const uint4* wp = wnodes + (uint64_t)(node ? R.cur : 0u) * NW;
    const float4* tp = tri_s + (uint64_t)(leaf ? (R.pend & ~kWideLeaf) : 0u) * 3;
    const uint32_t to = BUF ? (leaf ? (R.pend & ~kWideLeaf) * 48u : M->tbytes) : 0u;
    uint4 wr[NW];
    float4 T0, T1, T2;
#ifdef RT_STEPSTAMPS
    RT_TSTAMP(R.t1);
#endif
    if (BUF) {
        const uint32_t wo = node ? R.cur * WideFmt<W>::bytes : M->wbytes;
        T0 = bload_f4(M->tr, to); T1 = bload_f4(M->tr, to + 16); T2 = bload_tri2(M->tr, to + 32);
#pragma unroll
        for (uint32_t k = 0; k < NW; ++k) wr[k] = bload_rec<W>(M->wr, wo + 16 * k, k);
#ifdef RT_STEPSTAMPS
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
        RT_TSTAMP(R.t2);
#endif
    } else {
        if (leaf) { T0 = tp[0]; T1 = tp[1]; T2 = tp[2]; }
        if (node) {
#pragma unroll
            for (uint32_t k = 0; k < NW; ++k) wr[k] = wp[k];
        }
    }
    if (leaf) {
        if (COUNT) ++ct;
        const float tv[9] = {T0.x, T0.y, T0.z, T0.w, T1.x, T1.y, T1.z, T1.w, T2.x};
        if (MTF) {
            // §9.7 takes the triangle iff its exact leaf box passes the slab
            // test and Moller-Trumbore hits closer, both against the same tb:
            // MT first, the box test only for lanes with a closer MT hit (the
            // wave skips it when it has none), on vertices loaded again
            // (L1-hot) rather than kept live across MT.
            float t, u, v;
            if (intersect_tri(o, R.d, tv, R.tb, t, u, v)) {
                __asm__ volatile("" ::: "memory");  // reload below instead of keeping tv live
                const float4 U0 = BUF ? bload_f4(M->tr, to) : tp[0], U1 = BUF ? bload_f4(M->tr, to + 16) : tp[1],
                             U2 = BUF ? bload_tri2(M->tr, to + 32) : tp[2];
                const float uv[9] = {U0.x, U0.y, U0.z, U0.w, U1.x, U1.y, U1.z, U1.w, U2.x};
                float lo[3], hi[3], tn;
                tri_bounds(uv, lo, hi);
                if (slab_hit(lo, hi, o, R.invd, R.tb, tn)) {
                    R.tb = t; R.hu = u; R.hv = v; R.hp = __float_as_uint(U2.y);
                    if (any) { R.pend = RT_SENT; return 1; }  // any-hit: done
                }
            }
        } else {
            float lo[3], hi[3], tn;
            tri_bounds(tv, lo, hi);
            if (slab_hit(lo, hi, o, R.invd, R.tb, tn)) {
                float t, u, v;
                if (intersect_tri(o, R.d, tv, R.tb, t, u, v)) {
                    R.tb = t; R.hu = u; R.hv = v; R.hp = __float_as_uint(T2.y);
                    if (any) { R.pend = RT_SENT; return 1; }  // any-hit: done
                }
            }
        }
        R.pend = RT_SENT;
    }
    if (!node) return 0;
    if (R.ctn > R.tb) { R.cur = RT_SENT; return 0; }
    if (COUNT) ++cn;
    const uint32_t valid = rec_mask<W>(wr);
    bool hit[W];
    float tn[W];
    record_test<W>(R, wr, hit, tn);
#pragma unroll
    for (int i = 0; i < W; ++i) hit[i] = ((valid >> i) & 1u) && hit[i];
    bool earlier[W];
    earlier[0] = false;
#pragma unroll
    for (int i = 1; i < W; ++i) earlier[i] = earlier[i - 1] || hit[i - 1];
    bool over = false;
#pragma unroll
    for (int i = W - 1; i >= 1; --i) {
        const bool push = hit[i] && earlier[i];
        const uint32_t slot = R.sp < cap ? R.sp : cap;
        sref[slot * NT] = rec_ref<W>(wr, i);
        stn[slot * NT] = (uint16_t)(__float_as_uint(tn[i]) >> 16);
        over = over || (push && R.sp >= cap);
        R.sp += (push && R.sp < cap) ? 1u : 0u;
    }
    if (over) return 2;
    uint32_t cur = RT_SENT;
    float ctn = tn[W - 1];
#pragma unroll
    for (int i = W - 1; i >= 0; --i) {
        cur = hit[i] ? rec_ref<W>(wr, i) : cur;
        ctn = hit[i] ? tn[i] : ctn;
    }
    R.cur = cur;
    R.ctn = ctn;
    return 0;
}

// One ray from o along d over (0, tmax): the wide traversal when it applies
// (finite 1/d, K7w records present), with the binary hand-off on overflow;
// the binary traversal from the root otherwise.  any: the first hit ends it.
template <bool COUNT, int NT, bool MTF = false, int W = 4>
__device__ __forceinline__ void trace_gen(const char* __restrict__ nodes, const uint4* __restrict__ wnodes,
                                          uint32_t wcap, const float4* __restrict__ tri_s, uint32_t n, const float* o,
                                          const float* d, float tmax, bool any, uint32_t* sref, uint16_t* stn,
                                          float& tb, float& hu, float& hv, uint32_t& hp, uint32_t& cn, uint32_t& ct) {
    WRay R;
    wray_init(o, d, R, scene_box(nodes));
    R.tb = tmax;
    const bool wide = R.fin && wnodes && n >= 2;
    int st = wide ? 0 : 2;
    if (W == 8 || n <= kBufMaxN) {  // buffer loads (WideMem): record and triangle in one round trip
        const WideMem M = wide_mem<W>(wnodes, tri_s, n);
        while (st == 0)
            st = wide_step<COUNT, NT, false, MTF, true, W>(R, wnodes, tri_s, o, wcap, 4 * n + 16, sref, stn, cn, ct,
                                                           any, &M);
    } else {
        while (st == 0)
            st = wide_step<COUNT, NT, false, MTF>(R, wnodes, tri_s, o, wcap, 4 * n + 16, sref, stn, cn, ct, any);
    }
    if (st == 2) {
        const uint32_t start = !wide ? (n ? 0u : RT_SENT) : (R.cur == RT_SENT ? RT_SENT : bin_of(R.cur, n - 1));
        trace_ray_from<COUNT>(nodes, tri_s, n, o, R.d, start, R.tb, R.hu, R.hv, R.hp, cn, ct, any);
    }
    tb = R.tb; hu = R.hu; hv = R.hv; hp = R.hp;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// A hit record store.  nt: nontemporal (primary frames, launch_trace) -- a frame's hit
// records (530 MB at 4Kx4 or 1080p x 16, 33 MB at 1080p1) stream to HBM while the
// trace, which uses a few % of HBM bandwidth, runs, instead of staying dirty
// in L2 / the MALL until the next build's soup read evicts them (DESIGN.md
// "(d)", the 10M K0 read floor).
typedef float rt_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_hit(float4* p, float4 v, uint32_t nt) {
    if (nt) {
        const rt_f4 x = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(x, reinterpret_cast<rt_f4*>(p));
    } else {
        *p = v;
    }
}

__device__ __forceinline__ uint32_t q8(float x) { return (uint32_t)fminf(fmaxf(x * 255.0f + 0.5f, 0.0f), 255.0f); }

// Shading frame of a hit (shadow and path modes): P = o + t d,
// unit geometric normal N flipped to face the incoming ray, S = P + 1e-4 N,
// D = light - S, cosl = N.D/|D|.  Operation order as the oracle's.
struct Surf { float N[3], S[3], D[3], cosl; };

__device__ __forceinline__ void surface(const float* __restrict__ tris, uint32_t prim, const float* o, const float* d,
                                        float t, const float* lp, Surf& f) {
    const float* tri = tris + (uint64_t)prim * 9;
    float P[3], e1[3], e2[3], nrm[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        P[a] = o[a] + t * d[a];
        e1[a] = tri[3 + a] - tri[a];
        e2[a] = tri[6 + a] - tri[a];
    }
    cross3(e1, e2, nrm);
    const float nl = sqrtf(dot3(nrm, nrm));
#pragma unroll
    for (int a = 0; a < 3; ++a) f.N[a] = nl > 0.0f ? nrm[a] / nl : 0.0f;
    if (dot3(f.N, d) > 0.0f) {
#pragma unroll
        for (int a = 0; a < 3; ++a) f.N[a] = -f.N[a];
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        f.S[a] = P[a] + f.N[a] * 1e-4f;
        f.D[a] = lp[a] - f.S[a];
    }
    const float dl = sqrtf(dot3(f.D, f.D));
    f.cosl = dl > 0.0f ? dot3(f.N, f.D) / dl : 0.0f;
}

// Shadow mode [SPEC, DESIGN.md "Shadow mode"]: the lighting factor f of a
// primary hit -- one any-hit shadow ray from the hit (offset 1e-4 along the
// viewer-facing geometric normal) toward the point light over t in (0, 1),
// Lambert term, ambient floor.  Operation order as orc_render_shadow.
struct Light { float p[3]; float ambient; };

template <bool COUNT, int NT, int W = 4>
__device__ __forceinline__ float shadow_factor(const char* __restrict__ nodes, const uint4* __restrict__ wnodes,
                                               uint32_t wcap, const float4* __restrict__ tri_s,
                                               const float* __restrict__ tris, uint32_t n, const float* o,
                                               const float* d, float t, uint32_t prim, const Light& lt,
                                               uint32_t* sref, uint16_t* stn, uint32_t& cn, uint32_t& ct) {
    Surf f;
    surface(tris, prim, o, d, t, lt.p, f);
    float tb, hu, hv;
    uint32_t hp;
    trace_gen<COUNT, NT, true, W>(nodes, wnodes, wcap, tri_s, n, f.S, f.D, 1.0f, true, sref, stn, tb, hu, hv, hp, cn,
                                  ct);
    const float lit = hp != RT_SENT ? 0.0f : fmaxf(f.cosl, 0.0f);
    return lt.ambient + (1.0f - lt.ambient) * lit;
}

// trace.px_sort: a 256-thread block deals its tile's 256 pixels to its four
// waves costliest first by the previous frame's per-pixel step counts
// (px_prev, written by k_trace), computed at block start (no extra launch).
// Only the wave a pixel lands in matters, so a 16-bucket key (two per octave
// of the step count) is enough; the ranking is atomic-free -- per wave one
// ballot per bucket, then position = pixels in costlier buckets + same-bucket
// pixels of earlier waves + the lane's rank in its own ballot -- so it is a
// permutation whatever the costs.  Returns the local pixel (ly * 16 + lx) of
// thread tid.  Called by all 256 threads.
__device__ __forceinline__ uint32_t px_bucket(uint32_t c) {
    if (c < 4) return 0u;
    const uint32_t e = 31u - (uint32_t)__clz((int)c);  // c in [2^e, 2^(e+1)), e >= 2
    return min(15u, 2u * (e - 2u) + ((c >> (e - 1u)) & 1u));
}

// lds: >= 144 words of the caller's LDS, free until this returns (k_trace
// passes its stack array: the ranking's 576 B would otherwise take the block
// past 160 KB / 7, i.e. cost a block per CU).  Ends with a barrier, so the
// caller may overwrite them at once.
__device__ __forceinline__ uint32_t tile_pixel_order(const uint16_t* __restrict__ px_prev, uint32_t tid,
                                                     uint32_t* lds) {
    uint32_t (*s_cnt)[16] = reinterpret_cast<uint32_t (*)[16]>(lds);  // [wave][bucket] pixel counts
    uint32_t* s_pre = lds + 64;                                        // pixels in costlier buckets
    uint8_t* s_perm = reinterpret_cast<uint8_t*>(lds + 80);
    const uint32_t lane = tid & 63, wv = tid >> 6;
    const uint32_t b = 15u - px_bucket(px_prev[tid]);  // 0 = costliest
    uint32_t rank = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
        const uint64_t m = __ballot(b == k);
        if (b == k) rank = lanes_below(m);
        if (lane == k) s_cnt[wv][k] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (tid < 64) {  // exclusive scan of the 16 bucket totals in wave 0
        const uint32_t tot = tid < 16 ? s_cnt[0][tid] + s_cnt[1][tid] + s_cnt[2][tid] + s_cnt[3][tid] : 0u;
        uint32_t x = tot;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= (uint32_t)o) x += y;
        }
        if (tid < 16) s_pre[tid] = x - tot;
    }
    __syncthreads();
    uint32_t pos = s_pre[b] + rank;
    for (uint32_t q = 0; q < wv; ++q) pos += s_cnt[q][b];
    s_perm[pos] = (uint8_t)tid;
    __syncthreads();
    const uint32_t li = s_perm[tid];
    __syncthreads();
    return li;
}

// Heavy-ray queue (trace.coop_cap, DESIGN.md "Cooperative heavy rays"): a
// primary ray still traversing after coop_cap wide steps stops, and its
// pixel -- from that sample on, with the colour sums of the samples before
// it -- is queued for k_trace_coop, which traces it with a whole wave.
// Entries of kCoopEntry x 16 B: {x, y, deferred sample, output pixel index}
// {r, g, b sums of the earlier samples, best prim} {tb, hu, hv, nst} and
// the deferred sample's traversal state -- its nst <= the stack depth + 1 pending
// entries {ref, tn} bottom to top (the lane's stack, then its current entry):
// k_trace_coop resumes the ray there instead of restarting it at the root.
// They live in kCoopShards shards of `cap` entries, each with its own reservation counter
// (wave gw reserves in shard gw mod kCoopShards): tens of thousands of
// returning atomics on ONE device-scope counter serialise (~10 ns each, a
// full-frame pass 1 went 0.33 -> 0.42 ms), spread over 64 they do not.  A
// counter may pass `cap`: lanes that find their shard full go on tracing.
// minimum waves per SIMD the trace kernels are compiled for (the register
// budget): the shadow kernel (primary + shadow traversal in one loop nest)
// at 5, whose 107 VGPRs would leave 4 (0.764 -> 0.72 ms per frame); the
// primary kernels at the compiler's choice (forcing 6 waves spills and is
// slower, profiles/ab_slack_r02.log)
#ifndef RT_KTRACE_WAVES
#define RT_KTRACE_WAVES 1
#endif
#ifndef RT_KSHADOW_WAVES
#define RT_KSHADOW_WAVES 5
#endif
#ifndef RT_KTILES_WAVES
#define RT_KTILES_WAVES 5
#endif
constexpr uint32_t kCoopShards = 64;
constexpr uint32_t kCoopFrontier = kWideStackMax + 1;        // pending entries a deferred ray can have (either arity)
constexpr uint32_t kCoopEntry = 3 + (kCoopFrontier + 1) / 2;  // uint4 per queue entry
static_assert(kCoopEntry * 16 == kCoopEntryBytes, "rt_launch.h sizes the queue (deeper stacks: raise kCoopEntryBytes)");
struct CoopQ {
    uint4* q = nullptr;
    uint32_t* ctr = nullptr;       // [kCoopShards] this frame's reservation counters
    uint32_t* ctr_next = nullptr;  // [kCoopShards] the next frame's, zeroed by k_trace_coop
    uint32_t cap = 0;              // entries per shard
};

// Called by the lanes that reach the step cap in this step (divergent): one
// atomic per wave reserves their entries.  Returns 3 (deferred) with the
// entry index, or 0 (shard full: keep tracing).
// The deferring lane's entry: pixel, colour sums, best hit and its pending
// subtrees in preorder from the bottom of its LDS stack (stack entries carry
// their tn truncated to 16 bits: a lower bound, as in wide_step).
template <int NT>
__device__ __forceinline__ void coop_store(const CoopQ& cq, uint32_t qslot, uint32_t x, uint32_t y, uint32_t s,
                                           uint32_t pi, float r, float g, float b, const WRay& R,
                                           const uint32_t* sref, const uint16_t* stn) {
    uint4* e = cq.q + (uint64_t)qslot * kCoopEntry;
    const uint32_t nst = R.sp + (R.cur != RT_SENT ? 1u : 0u);
    e[0] = make_uint4(x, y, s, pi);
    e[1] = make_uint4(__float_as_uint(r), __float_as_uint(g), __float_as_uint(b), R.hp);
    e[2] = make_uint4(__float_as_uint(R.tb), __float_as_uint(R.hu), __float_as_uint(R.hv), nst);
    for (uint32_t j = 0; j < nst; j += 2) {
        uint32_t rf[2], tn[2];
#pragma unroll
        for (uint32_t k = 0; k < 2; ++k) {
            const uint32_t i = j + k;
            rf[k] = i < R.sp ? sref[i * NT] : R.cur;
            tn[k] = i < R.sp ? (uint32_t)stn[i * NT] << 16 : __float_as_uint(R.ctn);
        }
        e[3 + j / 2] = make_uint4(rf[0], tn[0], rf[1], tn[1]);
    }
}

__device__ __forceinline__ int coop_defer(const CoopQ& cq, uint32_t gw, uint32_t& qslot) {
    const uint64_t mm = __ballot(1);
    const uint32_t leader = (uint32_t)__builtin_ctzll(mm);
    const uint32_t sh = gw & (kCoopShards - 1);
    uint32_t base = 0;
    if (__lane_id() == leader) base = atomicAdd(cq.ctr + sh, (uint32_t)__popcll(mm));
    base = __builtin_amdgcn_readlane(base, leader);
    const uint32_t p = base + lanes_below(mm);
    if (p < cq.cap) {
        qslot = sh * cq.cap + p;
        return 3;
    }
    return 0;
}

// ---------------------------------------------------------------- tile order
// DESIGN.md "Tile order".  A frame's time is set by its longest waves (~1 us
// per dependent record fetch, up to ~200 fetches for rays grazing the soup):
// dispatched in row-major order they start late and the GPU idles behind
// them.  Each wave of k_trace records its duration into cost[slot]
// (atomicMax over the tile's waves); the next frame of the same size
// dispatches its tiles longest-first from that map.  The order only decides
// which block renders which tile, never a pixel's result.
//
// Counting sort, costliest first, on a log-scale key: 8 buckets per octave
// of the duration (10-ns clock ticks).  Order within a bucket is free.
__device__ __forceinline__ uint32_t cost_bucket(uint32_t d) {
    if (d < 8) return d;
    const uint32_t e = 31u - (uint32_t)__clz((int)d);  // d in [2^e, 2^(e+1)), e >= 3
    return min(255u, (e - 2) * 8 + ((d >> (e - 3)) & 7u));
}

constexpr uint32_t kOrderPerThread = 32;  // k_tile_order: up to 32768 tiles per rank (4K frames)

// It also clears the map it consumed: after the host's swap that buffer is
// the one the next frame writes, so no memset is needed per frame.
// The counting sort of one block of NTH threads, PER costs per thread (nb <=
// NTH * PER): k_tile_order (1024 threads, its own launch) or block 0 of the
// previous frame's k_trace_coop (256 threads, nb <= 4096: one rank's tiles),
// whose order the next frame then finds ready (TileSched::order_ready).
// The sort key is not the last frame's cost but a running mean m = (m + c)/2
// over the frames of this shape (`ema`, kept beside the maps): a tile's cost
// is its slowest wave, set by one costly ray that a small camera move makes
// or breaks, and the mean ranks the tiles that keep holding such rays (the
// bench's orbit: 0.363 -> 0.353 ms, profiles/ab_order_ema_r02.log).
template <int NTH, int PER>
__device__ __forceinline__ void tile_order_block(uint32_t* __restrict__ cost, uint32_t nb,
                                                 uint32_t* __restrict__ order, uint32_t* s_hist, uint32_t* s_sum,
                                                 uint32_t* __restrict__ ema) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (uint32_t j = tid; j < 256; j += NTH) s_hist[j] = 0u;
    __syncthreads();
    // each cost is read once: both passes see the same buckets, so `order`
    // is a permutation even if the map were being rewritten meanwhile
    uint8_t bk[PER];
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        const uint32_t i = tid + j * NTH;
        bk[j] = 0;
        if (i < nb) {
            uint32_t c = cost[i];
            if (ema) {  // the key: a running mean over this shape's frames (m = (m + c) / 2)
                c = (uint32_t)(((uint64_t)ema[i] + c) >> 1);
                ema[i] = c;
            }
            bk[j] = (uint8_t)(255u - cost_bucket(c));
            atomicAdd(&s_hist[bk[j]], 1u);
            cost[i] = 0u;
        }
    }
    __syncthreads();
    if (tid < 256) {  // exclusive scan of 256 buckets: 4 waves of 64
        const uint32_t v = s_hist[tid];
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= (uint32_t)o) x += y;
        }
        if (lane == 63) s_sum[wv] = x;
    }
    __syncthreads();
    if (tid < 256) {
        uint32_t pre = 0;
        for (uint32_t k = 0; k < wv; ++k) pre += s_sum[k];
        const uint32_t v = s_hist[tid];
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= (uint32_t)o) x += y;
        }
        s_hist[tid] = pre + x - v;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        const uint32_t i = tid + j * NTH;
        if (i < nb) order[atomicAdd(&s_hist[bk[j]], 1u)] = i;
    }
}

// The same counting sort for any nb (no per-thread bucket registers): pass 1
// folds the running mean and builds the histogram, pass 2 re-derives each
// tile's bucket from the mean it stored (ema[i], or the cost itself without
// one: the map read is not written while this runs) and clears the cost.
// Used by the samples-in-lanes full frames (4K: 32400 tiles), loads batched
// by UNR per thread so a pass is nb / (NTH * UNR) memory round trips.
template <int NTH, int UNR>
__device__ __forceinline__ void tile_order_loop(uint32_t* __restrict__ cost, uint32_t nb,
                                                uint32_t* __restrict__ order, uint32_t* s_hist, uint32_t* s_sum,
                                                uint32_t* __restrict__ ema) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (uint32_t j = tid; j < 256; j += NTH) s_hist[j] = 0u;
    __syncthreads();
    for (uint32_t i0 = tid; i0 < nb; i0 += NTH * UNR) {
        uint32_t c[UNR], m[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const uint32_t i = i0 + u * NTH;
            c[u] = i < nb ? cost[i] : 0u;
            m[u] = i < nb && ema ? ema[i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const uint32_t i = i0 + u * NTH;
            if (i < nb) {
                uint32_t k = c[u];
                if (ema) {
                    k = (uint32_t)(((uint64_t)m[u] + k) >> 1);
                    ema[i] = k;
                }
                atomicAdd(&s_hist[255u - cost_bucket(k)], 1u);
            }
        }
    }
    __syncthreads();
    // exclusive scan of 256 buckets: 4 waves of 64 (as tile_order_block), or
    // one wave of 64 with 4 consecutive buckets per lane (64-thread blocks)
    static_assert(NTH == 64 || NTH >= 256, "one wave or >= one thread per bucket");
    if constexpr (NTH == 64) {
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[j] = s_hist[4 * tid + j]; sum += v[j]; }
        uint32_t x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= (uint32_t)o) x += y;
        }
        uint32_t run = x - sum;
#pragma unroll
        for (int j = 0; j < 4; ++j) { s_hist[4 * tid + j] = run; run += v[j]; }
    } else {
        const uint32_t hv = tid < 256 ? s_hist[tid] : 0u;
        uint32_t hx = hv;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(hx, o, 64);
            if (lane >= (uint32_t)o) hx += y;
        }
        if (tid < 256 && lane == 63) s_sum[wv] = hx;
        __syncthreads();
        if (tid < 256) {
            uint32_t pre = 0;
            for (uint32_t k = 0; k < wv; ++k) pre += s_sum[k];
            s_hist[tid] = pre + hx - hv;
        }
    }
    __syncthreads();
    for (uint32_t i0 = tid; i0 < nb; i0 += NTH * UNR) {
        uint32_t k[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const uint32_t i = i0 + u * NTH;
            k[u] = i < nb ? (ema ? ema[i] : cost[i]) : 0u;
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const uint32_t i = i0 + u * NTH;
            if (i < nb) {
                order[atomicAdd(&s_hist[255u - cost_bucket(k[u])], 1u)] = i;
                cost[i] = 0u;
            }
        }
    }
}

// Full frames: the next frame's tile order sorted by one extra block of
// this frame's k_trace (the grid's last block, dispatched when the frame's
// tail is already running) from the previous frame's costs folded into the
// running mean, instead of a k_tile_order launch at the head of the next
// frame.  The order is then one frame older, which the running mean makes
// cheap.
struct OrderFold {
    uint32_t* cost = nullptr;  // the previous frame's cost map (read and cleared)
    uint32_t* out = nullptr;   // the next frame's order
    uint32_t* ema = nullptr;   // the running mean
    uint32_t nb = 0;
};
constexpr uint32_t kFoldPerThread = 32;  // 256 threads: up to 8192 tiles (a 1080p frame has 8160)
#ifndef RT_ORDER_FOLD
#define RT_ORDER_FOLD 1  // 0: k_tile_order at the head of every frame (A/B)
#endif

// CQ: compiled with the heavy-ray queue (trace.coop_cap*).  Without it the
// queue's state (entry writes, the deferring lane's stack copy) drops out of
// the loop: the full-frame primary kernel goes from 89 to 80 VGPRs, i.e. from
// 5 to 6 waves per SIMD.
// SPPC: the sample count as a compile-time constant (1: the colour sums and
// the sample loop are not live across the traversal), 0 = the argument.
template <bool COUNT, bool PACKED, bool WIDE, int NT, bool SHADOW = false, bool BUF = false, int WA = 4, bool CQ = true,
          int SPPC = 0>
__global__ __launch_bounds__(NT, (SHADOW && WA == 4) ? RT_KSHADOW_WAVES : (PACKED && WA == 4) ? RT_KTILES_WAVES : RT_KTRACE_WAVES)
void k_trace(const void* __restrict__ nodes, const uint4* __restrict__ wnodes,
                                               uint32_t wcap, const float4* __restrict__ tri_s, uint32_t n,
                                               Cam cam, uint32_t W, uint32_t H, uint32_t spp_in,
                                               uint32_t rank, uint32_t nranks, uint32_t tilesX,
                                               float4* __restrict__ hits, uint32_t* __restrict__ rgba,
                                               unsigned long long* __restrict__ counters,
                                               const float* __restrict__ tris = nullptr, Light lt = Light{},
                                               const uint32_t* __restrict__ order = nullptr,
                                               uint32_t* __restrict__ cost_out = nullptr,
                                               const uint16_t* __restrict__ px_prev = nullptr,
                                               uint16_t* __restrict__ px_cost = nullptr,
                                               uint32_t coop_cap = 0, CoopQ cq = CoopQ{},
                                               OrderFold fold = OrderFold{}, uint32_t nt_hits = 0) {
    // PX: the per-pixel order (below); its ranking borrows s_ref, so the
    // binary instance (no stack) still sizes s_ref for tile_pixel_order
    constexpr bool PX = !SHADOW && !COUNT && NT == 256;
    constexpr uint32_t kStackWords = (WIDE || SHADOW) ? (StackOf<WA, NT>::v + 1) * NT : 1u;
    constexpr uint32_t kRefWords = (PX && kStackWords < 144u) ? 144u : kStackWords;
    __shared__ uint32_t s_ref[kRefWords];
    __shared__ uint16_t s_tn[kStackWords];
    const uint32_t spp = SPPC ? (uint32_t)SPPC : spp_in;
    if constexpr (!PACKED && !SHADOW && !COUNT && NT == 256 && (WIDE || SHADOW)) {
        if (fold.out && blockIdx.x == gridDim.x - 1) {  // uniform: the extra block sorts and leaves
            static_assert(sizeof(s_ref) >= (256 + 16) * sizeof(uint32_t), "tile_order_block's LDS");
            tile_order_block<256, kFoldPerThread>(fold.cost, fold.nb, fold.out, s_ref, s_ref + 256, fold.ema);
            return;
        }
    }
    // tile slot from the block id: consecutive tiles go to different XCDs
    // under the round-robin dispatch, which balances the image's cheap and
    // costly bands over the 8 XCDs (an XCD-banded remap measured 1.2x
    // slower).  NT = 256: one 16x16 tile per block, wave w = quadrant w;
    // NT = 64: one quadrant (8x8) per block, so a finished wave frees its
    // slot and LDS at once instead of waiting for the tile's slowest wave.
    constexpr uint32_t WPB = NT / 64;
    const uint32_t gw = blockIdx.x * WPB + (threadIdx.x >> 6);  // global wave id
    const uint32_t slot = order ? order[gw >> 2] : gw >> 2;  // dispatch order -> tile slot
    const uint32_t t = rank_tile(rank, slot, nranks, tilesX, H);
    const uint32_t tx = t % tilesX, ty = t / tilesX;
    const uint32_t l = threadIdx.x & 63, w = gw & 3;
    // pixel of this lane: the 8x8 quadrant w of the tile, or (trace.px_sort,
    // 256-thread blocks, from the 2nd frame of a shape on) the tile's pixels
    // dealt to waves costliest first by the previous frame's per-pixel step
    // counts, so the tile's expensive rays share a wave instead of
    // stretching all four.  Primary-ray full frames only: compiled out of the
    // shadow, counting and 64-thread variants, whose registers it would cost.
    uint32_t lx = (w & 1) * 8 + (l & 7), ly = (w >> 1) * 8 + (l >> 3);
    if (PX && px_prev) {  // uniform: the whole block
        static_assert(!PX || sizeof(s_ref) >= 144 * sizeof(uint32_t), "tile_pixel_order's LDS");
        const uint32_t li = tile_pixel_order(px_prev + (uint64_t)slot * 256, threadIdx.x, s_ref);
        lx = li & 15;
        ly = li >> 4;
    }
    const uint32_t x = tx * 16 + lx, y = ty * 16 + ly;
    const bool valid = x < W && y < H;
    const SceneBox sb = scene_box(nodes);
    // uniform: with the queue off (full frames by default) the per-step cap
    // test, and its kernel-argument reload, drop out of the loop
    const bool coop_on = CQ && !SHADOW && coop_cap != 0;
    uint32_t cn = 0, ct = 0, steps = 0;
    uint32_t qslot = 0, dsamp = RT_SENT;  // heavy-ray queue entry, deferred sample
    const unsigned long long wt0 = cost_out ? __builtin_amdgcn_s_memrealtime() : 0ull;
#ifdef RT_STAMPS
    const unsigned long long st0 = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef RT_STEPSTAMPS
    unsigned long long ss_pop = 0, ss_wait = 0, ss_exec = 0, mt0;
    uint32_t ss_n = 0;
    RT_TSTAMP(mt0);
#endif
    if (valid) {
        float r = 0.0f, g = 0.0f, b = 0.0f;
        for (uint32_t s = 0; s < spp; ++s) {
            const uint32_t sidx = (y * W + x) * spp + s;
            float jx = 0.5f, jy = 0.5f;
            if (s > 0) {
                const uint32_t h = pcg_hash(sidx);
                jx = (float)(h >> 8) * 0x1p-24f;
                jy = (float)(pcg_hash(h) >> 8) * 0x1p-24f;
            }
            const float px = (float)x + jx, py = (float)y + jy;
            float d[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) d[c] = (cam.w00[c] + px * cam.du[c]) + py * cam.dv[c];
            float tb = 0.0f, hu = 0.0f, hv = 0.0f;
            uint32_t hp = RT_SENT;
            if (WIDE) {
                WRay R;
                wray_init(cam.eye, d, R, sb);
                int st = R.fin ? 0 : 2;
                const char* nd = reinterpret_cast<const char*>(nodes);
                const WideMem M = wide_mem<WA>(wnodes, tri_s, n);
                while (st == 0) {
#ifdef RT_STEPSTAMPS
                    unsigned long long t0, t3;
                    RT_TSTAMP(t0);
#endif
                    st = wide_step<COUNT, NT, false, PACKED || SHADOW, BUF, WA>(
                        R, wnodes, tri_s, cam.eye, wcap, 4 * n + 16, s_ref + threadIdx.x, s_tn + threadIdx.x, cn, ct,
                        false, &M);
#ifdef RT_STEPSTAMPS
                    RT_TSTAMP(t3);
                    if (R.t2) {  // a step that fetched: pop + address, the loads, the rest
                        ss_pop += R.t1 - t0;
                        ss_wait += R.t2 - R.t1;
                        ss_exec += t3 - R.t2;
                        ++ss_n;
                    }
#endif
                    if (coop_on && st == 0 && R.steps == coop_cap) st = coop_defer(cq, gw, qslot);
                }
                if (PX) steps += R.steps;
                if (st == 3) {  // heavy: k_trace_coop finishes this pixel from here on
                    coop_store<NT>(cq, qslot, x, y, s, PACKED ? slot * 256 + ly * 16 + lx : y * W + x, r, g, b, R,
                                   s_ref + threadIdx.x, s_tn + threadIdx.x);
                    dsamp = s;
                    break;
                }
                if (st == 2) {
                    if (!R.fin) { R.cur = 0; R.tb = __builtin_inff(); R.hu = R.hv = 0.0f; R.hp = RT_SENT; }
                    trace_ray_from<COUNT>(nd, tri_s, n, cam.eye, d, R.cur == RT_SENT ? RT_SENT : bin_of(R.cur, n - 1),
                                          R.tb, R.hu, R.hv, R.hp, cn, ct);
                }
                tb = R.tb; hu = R.hu; hv = R.hv; hp = R.hp;
                if (PX && st == 2) steps += 64u;  // a binary finish: a nominal charge
            } else {
                trace_ray<COUNT>(reinterpret_cast<const char*>(nodes), tri_s, n, cam.eye, d, tb, hu, hv, hp, cn, ct);
            }
            if (hits) {
                const uint64_t hi = PACKED ? ((uint64_t)slot * 256 + ly * 16 + lx) * spp + s : (uint64_t)sidx;
                store_hit(hits + hi, make_float4(tb, hu, hv, __uint_as_float(hp)), nt_hits);
            }
            if (SHADOW) {
                float f = 0.0f;
                if (hp != RT_SENT)
                    f = shadow_factor<COUNT, NT, WA>(reinterpret_cast<const char*>(nodes), WIDE ? wnodes : nullptr, wcap,
                                                 tri_s, tris, n, cam.eye, d, tb, hp, lt, s_ref + threadIdx.x,
                                                 s_tn + threadIdx.x, cn, ct);
                if (hp != RT_SENT) {
                    r = r + hu * f;
                    g = g + hv * f;
                    b = b + ((1.0f - hu) - hv) * f;
                } else {
                    r = r + 0.0f; g = g + 0.0f; b = b + 0.0f;
                }
            } else if (hp != RT_SENT) {
                r = r + hu;
                g = g + hv;
                b = b + ((1.0f - hu) - hv);
            } else {
                r = r + 0.0f; g = g + 0.0f; b = b + 0.0f;
            }
        }
        const uint32_t pi = PACKED ? slot * 256 + ly * 16 + lx : y * W + x;
        if (dsamp == RT_SENT && rgba) {
            const float sc = 1.0f / (float)spp;
            const uint32_t px = q8(r * sc) | (q8(g * sc) << 8) | (q8(b * sc) << 16) | (255u << 24);
            rgba[pi] = px;
        }
    }
#ifdef RT_STEPSTAMPS
    // per-wave {start, end (100 MHz), HW_ID | XCC_ID << 32, steps of the lane with the most fetching steps,
    // its pop / wait / rest shader cycles, the wave's shader cycles} (tools/diag_steps.py)
    {
        uint32_t best = ss_n;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) best = max(best, (uint32_t)__shfl_xor(best, o, 64));
        const uint64_t mine = __ballot(ss_n == best);
        const int src = __builtin_ctzll(mine);
        const unsigned long long p = __shfl(ss_pop, src, 64), wq = __shfl(ss_wait, src, 64),
                                 ex = __shfl(ss_exec, src, 64);
        unsigned long long mt1;
        RT_TSTAMP(mt1);
        if (l == 0) {
            const uint64_t wslot = (uint64_t)gw * 8;
            g_rt_stamps[wslot + 0] = st0;
            g_rt_stamps[wslot + 1] = __builtin_amdgcn_s_memrealtime();
            g_rt_stamps[wslot + 2] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                                     ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
            g_rt_stamps[wslot + 3] = best;
            g_rt_stamps[wslot + 4] = p;
            g_rt_stamps[wslot + 5] = wq;
            g_rt_stamps[wslot + 6] = ex;
            g_rt_stamps[wslot + 7] = mt1 - mt0;
        }
    }
#elif defined(RT_STAMPS)
    // per-wave {start, end, HW_ID | XCC_ID << 32, max lane nodes | wave nodes << 32}
    // (tools/diag_trace.py; node counts only in the COUNT variant)
    {
        uint32_t mx = cn, sm = cn;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            mx = max(mx, (uint32_t)__shfl_xor(mx, o, 64));
            sm += __shfl_xor(sm, o, 64);
        }
        if (l == 0) {
            const uint64_t wslot = (uint64_t)gw * 4;
            g_rt_stamps[wslot + 0] = st0;
            g_rt_stamps[wslot + 1] = __builtin_amdgcn_s_memrealtime();
            g_rt_stamps[wslot + 2] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                                     ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
            g_rt_stamps[wslot + 3] = (uint64_t)mx | ((uint64_t)sm << 32);
        }
    }
#endif
    if (COUNT) {
        unsigned long long a = cn, bsum = ct;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            a += __shfl_xor(a, o, 64);
            bsum += __shfl_xor(bsum, o, 64);
        }
        if (l == 0) {
            atomicAdd(&counters[0], a);
            atomicAdd(&counters[1], bsum);
        }
    }
    if (PX && px_cost) px_cost[(uint64_t)slot * 256 + ly * 16 + lx] = (uint16_t)min(steps, 65535u);
    if (cost_out && l == 0) {  // this wave's duration (10-ns ticks) -> the tile's cost map entry
        const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - wt0;
        atomicMax(&cost_out[slot], (uint32_t)min(dt, 0xFFFFFFFFull));
    }
}

__global__ __launch_bounds__(1024) void k_tile_order(uint32_t* __restrict__ cost, uint32_t nb,
                                                     uint32_t* __restrict__ order, uint32_t* __restrict__ ema) {
    __shared__ uint32_t s_hist[256];
    __shared__ uint32_t s_sum[16];
    tile_order_block<1024, kOrderPerThread>(cost, nb, order, s_hist, s_sum, ema);
}

// ------------------------------------------------------- samples in lanes
// trace.spp_lanes (r05, DESIGN.md (e) "Samples in lanes for one rank's
// tiles"): a multi-spp frame whose S = spp samples per pixel (a power of two,
// 2..16) are traced by S adjacent lanes at once -- one ray per lane, and a
// wave (a unit) holds the S samples of 64/S pixels of a compact block of its
// tile (8x4 pixels at 2 spp, 4x4 at 4, 4x2 at 8, 2x2 at 16).  A tile is 4S units.  The loop kernel (k_trace, a lane runs its
// pixel's samples one after the other) makes the costliest pixel's S
// dependent traversals one lane's chain: a rank of an 8-GPU 10M 4Kx4 frame
// ran 1.2-1.3 ms against a 0.6-ms share (r05: max-rank efficiency 0.45 with
// the queue off, 0.30 with it).  Here the longest chain is one ray, capped by
// the heavy-ray queue like a 1-spp frame's.  The colour is the same ordered
// sum as the loop's, r = ((0 + c_0) + c_1) + ..., taken over the pixel's
// lanes with shuffles, then q8(r * (1/spp)): bit-identical images and hits.
// A sample that the queue takes is finished by k_trace_coop (one ray:
// kCoopOne) and its pixel's colour by k_coop_resolve from the hits of all
// its samples; the rest of the wave never waits for it.
constexpr uint32_t kCoopOne = 0x80000000u;  // queue entry's sample word: this sample only (samples in lanes)

template <int S>
struct SlShape {
    // (32 / 64 samples would spill in the colour sum's shuffles: the loop kernel keeps them)
    static_assert(S >= 2 && S <= 16 && (S & (S - 1)) == 0, "2..16 samples, a power of two");
    static constexpr uint32_t PW = 64 / S;                                          // pixels per unit
    static constexpr uint32_t TW = S == 2 ? 8 : S <= 8 ? 4 : 2;                    // block width
    static constexpr uint32_t TH = PW / TW, TPR = 16 / TW, UPT = 256 / PW;          // rows, blocks per row, units per tile
};

// MTF: Moller-Trumbore first (wide_step) -- one rank's tiles by default
// (trace.sl_mtf), the box test first for full frames
template <bool PACKED, int NT, int S, bool MTF = PACKED>
__global__ __launch_bounds__(NT, RT_KTILES_WAVES) void k_trace_sl(const void* __restrict__ nodes,
                                                                 const uint4* __restrict__ wnodes, uint32_t wcap,
                                                                 const float4* __restrict__ tri_s, uint32_t n,
                                                                 Cam cam, uint32_t W, uint32_t H, uint32_t rank,
                                                                 uint32_t nranks, uint32_t tilesX,
                                                                 float4* __restrict__ hits, uint32_t* __restrict__ rgba,
                                                                 const uint32_t* __restrict__ order,
                                                                 uint32_t* __restrict__ cost_out, uint32_t coop_cap,
                                                                 CoopQ cq, uint32_t nt_hits,
                                                                 OrderFold fold = OrderFold{}) {
    using SH = SlShape<S>;
    constexpr uint32_t kStackWords = (StackOf<4, NT>::v + 1) * NT;
    __shared__ uint32_t s_ref[kStackWords];
    __shared__ uint16_t s_tn[kStackWords];
    // block 0 sorts the next frame's tile order (OrderFold; full frames and
    // one rank's tiles) and the units start at block 1.  The first block
    // rather than the last: a 4K map takes this block tens of us, hidden
    // under the frame's bulk, not added to its tail.
    uint32_t bid = blockIdx.x;
    if (fold.out) {
        if (bid == 0) {  // uniform: the whole block sorts and leaves
            static_assert(kStackWords >= 256 + 16, "tile_order_loop's LDS");
            tile_order_loop<NT, 8>(fold.cost, fold.nb, fold.out, s_ref, s_ref + 256, fold.ema);
            return;
        }
        --bid;
    }
    const uint32_t gw = bid * (NT / 64) + (threadIdx.x >> 6);  // global unit (wave) id
    const uint32_t ti = gw / SH::UPT, q = gw % SH::UPT;
    const uint32_t slot = order ? order[ti] : ti;
    const uint32_t t = rank_tile(rank, slot, nranks, tilesX, H);
    const uint32_t tx = t % tilesX, ty = t / tilesX;
    const uint32_t l = threadIdx.x & 63, p = l / S, smp = l % S;
    const uint32_t lx = (q % SH::TPR) * SH::TW + p % SH::TW, ly = (q / SH::TPR) * SH::TH + p / SH::TW;
    const uint32_t x = tx * 16 + lx, y = ty * 16 + ly;
    const bool valid = x < W && y < H;
    const uint32_t pi = PACKED ? slot * 256 + ly * 16 + lx : y * W + x;
    const unsigned long long wt0 = cost_out ? __builtin_amdgcn_s_memrealtime() : 0ull;
    float cr = 0.0f, cg = 0.0f, cb = 0.0f;
    bool deferred = false;
    if (valid) {
        const uint32_t sidx = (y * W + x) * S + smp;
        float jx = 0.5f, jy = 0.5f;
        if (smp > 0) {
            const uint32_t h = pcg_hash(sidx);
            jx = (float)(h >> 8) * 0x1p-24f;
            jy = (float)(pcg_hash(h) >> 8) * 0x1p-24f;
        }
        const float px = (float)x + jx, py = (float)y + jy;
        float d[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) d[c] = (cam.w00[c] + px * cam.du[c]) + py * cam.dv[c];
        WRay R;
        wray_init(cam.eye, d, R, scene_box(nodes));
        int st = R.fin ? 0 : 2;
        uint32_t cn = 0, ct = 0, qslot = 0;
        const WideMem M = wide_mem<4>(wnodes, tri_s, n);
        while (st == 0) {
            st = wide_step<false, NT, false, MTF, true, 4>(R, wnodes, tri_s, cam.eye, wcap, 4 * n + 16,
                                                            s_ref + threadIdx.x, s_tn + threadIdx.x, cn, ct, false, &M);
            if (coop_cap != 0 && st == 0 && R.steps == coop_cap) st = coop_defer(cq, gw, qslot);
        }
        if (st == 3) {  // heavy: k_trace_coop finishes this sample, k_coop_resolve its pixel
            coop_store<NT>(cq, qslot, x, y, smp | kCoopOne, pi, 0.0f, 0.0f, 0.0f, R, s_ref + threadIdx.x,
                           s_tn + threadIdx.x);
            deferred = true;
        } else {
            if (st == 2) {
                if (!R.fin) { R.cur = 0; R.tb = __builtin_inff(); R.hu = R.hv = 0.0f; R.hp = RT_SENT; }
                trace_ray_from<false>(reinterpret_cast<const char*>(nodes), tri_s, n, cam.eye, d,
                                      R.cur == RT_SENT ? RT_SENT : bin_of(R.cur, n - 1), R.tb, R.hu, R.hv, R.hp, cn,
                                      ct);
            }
            if (hits) store_hit(hits + (uint64_t)pi * S + smp, make_float4(R.tb, R.hu, R.hv, __uint_as_float(R.hp)), nt_hits);
            if (R.hp != RT_SENT) {
                cr = R.hu;
                cg = R.hv;
                cb = (1.0f - R.hu) - R.hv;
            }
        }
    }
    // the pixel's colour: the loop's ordered sum over its S lanes (every lane
    // of the wave takes part in the shuffles)
    const uint64_t dm = __ballot(deferred);
    const uint32_t base = p * S;
    float r = 0.0f, g = 0.0f, b = 0.0f;
#pragma unroll
    for (int k = 0; k < S; ++k) {
        r = r + __uint_as_float((uint32_t)__shfl((int)__float_as_uint(cr), (int)(base + k), 64));
        g = g + __uint_as_float((uint32_t)__shfl((int)__float_as_uint(cg), (int)(base + k), 64));
        b = b + __uint_as_float((uint32_t)__shfl((int)__float_as_uint(cb), (int)(base + k), 64));
    }
    const uint64_t pm = (S == 64 ? ~0ull : ((1ull << S) - 1ull)) << base;
    if (valid && smp == 0 && !(dm & pm) && rgba) {
        const float sc = 1.0f / (float)S;
        const uint32_t px = q8(r * sc) | (q8(g * sc) << 8) | (q8(b * sc) << 16) | (255u << 24);
        rgba[pi] = px;
    }
    if (cost_out && l == 0) {  // this unit's duration -> its tile's cost map entry (the tile order's key)
        const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - wt0;
        atomicMax(&cost_out[slot], (uint32_t)min(dt, 0xFFFFFFFFull));
    }
}

// ------------------------------------------------------ cooperative heavy rays
// DESIGN.md "Cooperative heavy rays".  A group of G lanes (16, 32 or 64:
// trace.coop_lanes) traces one queued ray: a frame's (or one rank's
// share's) duration is set by its slowest waves, and those hold rays that
// need 100-250 dependent record fetches (rays grazing the soup, whose §9.7
// preorder enters far subtrees while tb is still infinite).  Here the ray's
// pending subtrees form a frontier list in preorder (an LDS stack per group,
// head on top), and each step the group takes the first m <= G entries at
// once: a record entry is fetched and its children tested against the
// current tb (pushed in order), a leaf entry's triangle is fetched and tested
// (exact leaf box + Moller-Trumbore) and becomes a "resolved" entry carrying
// (tn, t, u, v).  Resolved entries are folded into (tb, hit) only when they
// reach the head, i.e. in preorder, by §9.7's leaf rule: accept iff
// tn <= tb && t < tb, then tb = t.
//
// Why this is exactly §9.7.  §9.7's result is the fold over all leaves in
// preorder of that leaf rule (a box test on an ancestor passes whenever it
// passes on the contained leaf box: the monotonicity argument of wide_step),
// and the rule is monotone in tb: a leaf it rejects at some tb it rejects at
// every smaller tb.  Our tb at any moment is the fold over a preorder prefix
// of the leaves before every pending entry, so it is >= §9.7's tb at that
// entry's position: culling records (conservative quantized tn > tb) and
// dropping leaves that fail the rule at our tb only removes leaves §9.7
// rejects too, and every leaf §9.7 might accept is folded in preorder with
// §9.7's own tb.  A frontier that would overflow hands over to the binary
// traversal from its head entry with the current tb (every leaf before the
// head in preorder is folded: the hand-off of wide_step).
//
// Groups narrower than a wave run side by side in it: every group-level
// value (sp, m, j, tb, ...) is held identically by the group's lanes, the
// ballots are cut to the group's bits and lane reads go through ds_bpermute
// (__shfl) from the group's own lanes.  A finished group's lanes idle until
// the wave's other groups are done.
constexpr uint32_t kCoopRes = 0x40000000u;  // frontier entry: resolved leaf (kWideLeaf | kCoopRes | k)
constexpr uint32_t kCoopGrid = 2048;        // persistent 256-thread blocks (replaced by the resident capacity)

// frontier entries per group: a step takes m <= G entries and a record
// entry adds at most 3, so the list needs room for the growth of a few steps
template <int G, int W = 4>
struct CoopCfg {
    static constexpr uint32_t cap = (G == 64 ? 256u : G == 32 ? 192u : 112u) * (W == 8 ? 2u : 1u);
    static constexpr uint32_t groups = 256u / G;  // per 256-thread block
};

template <int G, int W = 4>
struct CoopLds {
    uint32_t ref[CoopCfg<G, W>::cap];
    float tn[CoopCfg<G, W>::cap], t[CoopCfg<G, W>::cap], u[CoopCfg<G, W>::cap], v[CoopCfg<G, W>::cap];
};

// this group's bits of a wave-wide ballot, shifted to bit 0
template <int G>
__device__ __forceinline__ uint64_t gballot(bool p, uint32_t gbase) {
    const uint64_t b = __ballot(p);
    if constexpr (G == 64) return b;
    else return (b >> gbase) & ((1ull << G) - 1ull);
}

__device__ __forceinline__ float gread_f(float x, uint32_t src) {
    return __uint_as_float((uint32_t)__shfl((int)__float_as_uint(x), (int)src, 64));
}
__device__ __forceinline__ uint32_t gread_u(uint32_t x, uint32_t src) {
    return (uint32_t)__shfl((int)x, (int)src, 64);
}

// One group, one ray (o, d the same in all its lanes), 1/d finite on every
// axis.  hp = prim.
// resume (nullable): a queue entry -- start from its best hit and pending
// entries (pass 1's state) instead of the root.
template <bool COUNT, int G, int W = 4>
__device__ __forceinline__ void coop_trace(const char* __restrict__ nodes, const uint4* __restrict__ wnodes,
                                           const float4* __restrict__ tri_s, uint32_t n, const float* o,
                                           const float* d, CoopLds<G, W>& L, const uint4* __restrict__ resume,
                                           float& tb_out, float& hu_out, float& hv_out, uint32_t& hp_out,
                                           uint32_t& cn, uint32_t& ct) {
    constexpr uint32_t CAP = CoopCfg<G, W>::cap;
    constexpr uint32_t NW = WideFmt<W>::words;
    static_assert(CAP >= kCoopFrontier + (W - 1), "room for a resumed frontier and one record's children");
    const uint32_t lane = __lane_id();
    const uint32_t gl = lane & (G - 1), gbase = lane & ~(uint32_t)(G - 1);
    WRay R;
    wray_init(o, d, R, scene_box(nodes));
    const WideMem M = wide_mem<W>(wnodes, tri_s, n);  // n <= kBufMaxN (the launcher's condition)
    float tb = __builtin_inff(), hu = 0.0f, hv = 0.0f;
    uint32_t hk = RT_SENT;   // tri_s slot of a best hit found here (its prim is read at the end)
    uint32_t hp0 = RT_SENT;  // the best hit's prim when resumed
    uint32_t sp = 1;
    if (resume) {
        const uint4 h1 = resume[1], h2 = resume[2];
        hp0 = h1.w;
        tb = __uint_as_float(h2.x); hu = __uint_as_float(h2.y); hv = __uint_as_float(h2.z);
        sp = h2.w;
        for (uint32_t i = gl; i < sp; i += G) {
            const uint4 pr = resume[3 + i / 2];
            L.ref[i] = (i & 1) ? pr.z : pr.x;
            L.tn[i] = __uint_as_float((i & 1) ? pr.w : pr.y);
        }
    } else if (gl == 0) {
        L.ref[0] = 0u;  // the root record
        L.tn[0] = 0.0f;
    }
    __builtin_amdgcn_wave_barrier();
    __asm__ volatile("" ::: "memory");
    const uint32_t limit = 4 * n + 16;
    bool handoff = false;
    for (uint32_t guard = 0; sp > 0; ++guard) {
        uint32_t m = min((uint32_t)G, sp);
        if (sp + (W - 1) * m > CAP) m = (CAP - sp) / (W - 1);  // a record adds at most W - 1 entries
        if (m == 0 || guard > limit) {
            handoff = true;
            break;
        }
        const bool act = gl < m;
        uint32_t ref = 0u;
        float etn = 0.0f, et = 0.0f, eu = 0.0f, ev = 0.0f;
        if (act) {
            const uint32_t pos = sp - 1 - gl;
            ref = L.ref[pos]; etn = L.tn[pos]; et = L.t[pos]; eu = L.u[pos]; ev = L.v[pos];
        }
        __builtin_amdgcn_wave_barrier();
        __asm__ volatile("" ::: "memory");
        const bool res = (ref & kCoopRes) != 0u;
        // 0. every entry that may expand issues its loads now, before the
        // fold (whose t_best only culls more): a triangle or a record, both
        // as buffer loads with an out-of-range offset for the other one --
        // no branches, so a step costs one memory round trip whatever mix
        // of leaves and records the group holds
        const bool pre_leaf = act && !res && (ref & kWideLeaf) && etn <= tb;
        const bool pre_rec = act && !res && !(ref & kWideLeaf) && etn <= tb;
        const uint32_t to = pre_leaf ? (ref & ~kWideLeaf) * 48u : M.tbytes;
        const uint32_t wo = pre_rec ? ref * WideFmt<W>::bytes : M.wbytes;
        const float4 T0 = bload_f4(M.tr, to), T1 = bload_f4(M.tr, to + 16), T2 = bload_f4(M.tr, to + 32);
        uint4 wr[NW];
#pragma unroll
        for (uint32_t k = 0; k < NW; ++k) wr[k] = bload_u4(M.wr, wo + 16 * k);
        // 1. fold the head run of resolved leaves, in preorder
        const uint64_t nonres = gballot<G>(act && !res, gbase);
        const uint32_t j = nonres ? (uint32_t)__builtin_ctzll(nonres) : m;
        int last = -1;
        for (;;) {
            const uint64_t cm = gballot<G>((int)gl > last && gl < j && tb >= etn && tb > et, gbase);
            if (!cm) break;
            last = (int)__builtin_ctzll(cm);
            const uint32_t src = gbase + (uint32_t)last;
            tb = gread_f(et, src);
            hu = gread_f(eu, src);
            hv = gread_f(ev, src);
            hk = gread_u(ref, src) & ~(kWideLeaf | kCoopRes);
        }
        // 2. expand entries j..m-1 against the folded tb
        R.tb = tb;
        bool h[W];
        uint32_t cref[W];
        float ctn[W];
#pragma unroll
        for (int i = 0; i < W; ++i) { h[i] = false; cref[i] = i == 0 ? ref : 0u; ctn[i] = i == 0 ? etn : 0.0f; }
        if (act && gl >= j && etn <= tb) {
            if (res) {
                h[0] = true;  // not at the head yet: stays pending
            } else if (ref & kWideLeaf) {
                if (COUNT) ++ct;
                const float tv[9] = {T0.x, T0.y, T0.z, T0.w, T1.x, T1.y, T1.z, T1.w, T2.x};
                float lo[3], hi[3], tn;
                tri_bounds(tv, lo, hi);
                float t, u, v;
                if (slab_hit(lo, hi, o, R.invd, tb, tn) && intersect_tri(o, d, tv, tb, t, u, v)) {
                    h[0] = true;
                    cref[0] = ref | kCoopRes;
                    ctn[0] = tn;
                    et = t; eu = u; ev = v;
                }
            } else {
                if (COUNT) ++cn;
                float tn[W];
                record_test<W>(R, wr, h, tn);
                const uint32_t valid = rec_mask<W>(wr);
#pragma unroll
                for (int i = 0; i < W; ++i) {
                    cref[i] = rec_ref<W>(wr, i);
                    h[i] = ((valid >> i) & 1u) && h[i];
                    ctn[i] = tn[i];
                }
            }
        }
        // 3. the outputs in preorder (lane order, then child order) replace
        // the m entries taken: output g lands at spn - 1 - g
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < W; ++i) c += (uint32_t)h[i];
        // each lane's output count c <= W, summed over the group bit by bit
        constexpr int CB = W == 8 ? 4 : 3;
        const uint64_t below = (1ull << gl) - 1ull;
        uint32_t pre = 0, total = 0;
#pragma unroll
        for (int bit = 0; bit < CB; ++bit) {
            const uint64_t bb = gballot<G>((c >> bit) & 1u, gbase);
            pre += (uint32_t)__popcll(bb & below) << bit;
            total += (uint32_t)__popcll(bb) << bit;
        }
        const uint32_t spn = sp - m + total;
        uint32_t g = pre;
#pragma unroll
        for (int i = 0; i < W; ++i) {
            if (h[i]) {
                const uint32_t p = spn - 1 - g;
                L.ref[p] = cref[i];
                L.tn[p] = ctn[i];
                if (i == 0) { L.t[p] = et; L.u[p] = eu; L.v[p] = ev; }
                ++g;
            }
        }
        __builtin_amdgcn_wave_barrier();
        __asm__ volatile("" ::: "memory");
        sp = spn;
    }
    uint32_t hp = hk == RT_SENT ? hp0 : __float_as_uint(tri_s[(uint64_t)hk * 3 + 2].y);
    if (handoff) {
        if (gl == 0) {
            const uint32_t head = sp ? L.ref[sp - 1] & ~kCoopRes : RT_SENT;
            trace_ray_from<COUNT>(nodes, tri_s, n, o, d, head == RT_SENT ? RT_SENT : bin_of(head, n - 1), tb, hu,
                                  hv, hp, cn, ct);
        }
        tb = gread_f(tb, gbase); hu = gread_f(hu, gbase); hv = gread_f(hv, gbase);
        hp = gread_u(hp, gbase);
    }
    tb_out = tb; hu_out = hu; hv_out = hv; hp_out = hp;
}

// Pass 2 of a primary frame with trace.coop_cap*: the queued heavy pixels,
// one group of G lanes each (a persistent grid striding over the queue), from
// the queued sample on; writes their hits and RGBA exactly as k_trace would.
// Block 0 zeroes the next frame's queue counters.  With ord_out (one rank's
// tiles, nb <= kOrderInCoop) block 0 instead sorts the cost map this frame's
// k_trace just wrote into the next frame's tile order -- the k_tile_order
// launch (8-11 us, all of it latency) leaves the next frame's critical path
// -- and leaves the queue to the other blocks.
constexpr uint32_t kOrderInCoop = 256 * 32;  // up to 8192 tiles: a 1080p full frame has 8160
// trace.coop_skip: the bunny substitute queues 0-5 rays a frame at the 96-step
// cap, the 1M soup 4500-6500 (profiles/ab_coop_skip_r05.log)
constexpr uint32_t kQueueSkip = 64;
constexpr uint32_t kQueueProbe = 16;
template <bool COUNT, bool PACKED, int G, int WA = 4>
__global__ __launch_bounds__(256) void k_trace_coop(const void* __restrict__ nodes, const uint4* __restrict__ wnodes,
                                                    const float4* __restrict__ tri_s, uint32_t n, Cam cam,
                                                    uint32_t W, uint32_t spp, CoopQ cq, float4* __restrict__ hits,
                                                    uint32_t* __restrict__ rgba,
                                                    unsigned long long* __restrict__ counters,
                                                    uint32_t* __restrict__ ord_cost = nullptr, uint32_t ord_nb = 0,
                                                    uint32_t* __restrict__ ord_out = nullptr,
                                                    uint32_t* __restrict__ ord_ema = nullptr,
                                                    uint32_t* __restrict__ q_count = nullptr) {
    constexpr uint32_t NG = CoopCfg<G, WA>::groups;
    __shared__ CoopLds<G, WA> s_l[NG];
    static_assert(kCoopShards == 64, "one shard per lane");
    if (blockIdx.x == 0 && threadIdx.x < kCoopShards) cq.ctr_next[threadIdx.x] = 0u;
    static_assert(sizeof(CoopLds<G, WA>) >= (256 + 16) * sizeof(uint32_t), "tile_order_block's LDS");
    const bool order_block = ord_out && gridDim.x > 1;  // uniform
    if (order_block && blockIdx.x == 0) {
        tile_order_block<256, kOrderInCoop / 256>(ord_cost, ord_nb, ord_out, reinterpret_cast<uint32_t*>(&s_l[0]),
                                  reinterpret_cast<uint32_t*>(&s_l[0]) + 256, ord_ema);
        return;
    }
    const uint32_t b0 = order_block ? 1u : 0u;  // queue work over blocks [b0, gridDim.x)
    const uint32_t lane = threadIdx.x & 63, grp = threadIdx.x / G, gl = threadIdx.x & (G - 1);
    // the shards' filled lengths and their exclusive prefix, lane k = shard k
    const uint32_t len = min(cq.ctr[lane], cq.cap);
    uint32_t incl = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= (uint32_t)o) incl += y;
    }
    // the shard table goes through LDS: inside the divergent loop below the
    // lanes of finished groups are inactive, and a lane read (readlane or a
    // shuffle) of a value the compiler computes there would see stale lanes
    __shared__ uint32_t s_excl[kCoopShards], s_len[kCoopShards];
    if (threadIdx.x < 64) {
        s_excl[lane] = incl - len;
        s_len[lane] = len;
    }
    __syncthreads();
    const uint32_t cnt = __builtin_amdgcn_readlane(incl, 63);
    // this frame's queue length to the host's mapped word (trace.coop_skip): the last block
    if (q_count && blockIdx.x == gridDim.x - 1 && threadIdx.x < 1) q_count[threadIdx.x] = cnt;
    uint32_t cn = 0, ct = 0;
    for (uint32_t e = (blockIdx.x - b0) * NG + grp; e < cnt; e += (gridDim.x - b0) * NG) {
        // queued ray e lives in the last non-empty shard whose prefix is <= e
        uint32_t sh = 0, sbase = 0;
        for (uint32_t k = 0; k < 64; ++k) {
            const uint32_t ek = s_excl[k];
            if (s_len[k] > 0 && ek <= e) { sh = k; sbase = ek; }
        }
        const uint32_t slot = sh * cq.cap + (e - sbase);
        const uint4* ent = cq.q + (uint64_t)slot * kCoopEntry;
        const uint4 a = ent[0], b = ent[1];
        const uint32_t x = a.x, y = a.y, pi = a.w;
        // kCoopOne (samples in lanes): this sample only; its pixel's colour is
        // k_coop_resolve's.  Else the pixel from this sample on.
        const bool one = (a.z & kCoopOne) != 0u;
        const uint32_t s0 = a.z & ~kCoopOne, s1 = one ? s0 + 1 : spp;
        float r = __uint_as_float(b.x), g = __uint_as_float(b.y), bl = __uint_as_float(b.z);
        for (uint32_t s = s0; s < s1; ++s) {
            const uint32_t sidx = (y * W + x) * spp + s;
            float jx = 0.5f, jy = 0.5f;
            if (s > 0) {
                const uint32_t hh = pcg_hash(sidx);
                jx = (float)(hh >> 8) * 0x1p-24f;
                jy = (float)(pcg_hash(hh) >> 8) * 0x1p-24f;
            }
            const float px = (float)x + jx, py = (float)y + jy;
            float d[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) d[c] = (cam.w00[c] + px * cam.du[c]) + py * cam.dv[c];
            float tb, hu, hv;
            uint32_t hp;
            coop_trace<COUNT, G, WA>(reinterpret_cast<const char*>(nodes), wnodes, tri_s, n, cam.eye, d, s_l[grp],
                                 s == s0 ? ent : nullptr, tb, hu, hv, hp, cn, ct);
            if (hits && gl == 0) hits[(uint64_t)pi * spp + s] = make_float4(tb, hu, hv, __uint_as_float(hp));
            if (hp != RT_SENT) {
                r = r + hu;
                g = g + hv;
                bl = bl + ((1.0f - hu) - hv);
            } else {
                r = r + 0.0f; g = g + 0.0f; bl = bl + 0.0f;
            }
        }
        if (rgba && gl == 0 && !one) {
            const float sc = 1.0f / (float)spp;
            rgba[pi] = q8(r * sc) | (q8(g * sc) << 8) | (q8(bl * sc) << 16) | (255u << 24);
        }
    }
    if (COUNT) {
        unsigned long long a = cn, bs = ct;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            a += __shfl_xor(a, o, 64);
            bs += __shfl_xor(bs, o, 64);
        }
        if (lane == 0 && (a || bs)) {
            atomicAdd(&counters[0], a);
            atomicAdd(&counters[1], bs);
        }
    }
}

// Samples in lanes: the colour of every pixel with a queued sample, from the
// hits of all its samples (k_trace_sl wrote the others, k_trace_coop the
// queued ones), as the loop's ordered sum.  One thread per queue entry; a
// pixel with several queued samples is written once per entry, with the same
// value.  After k_trace_coop on the same stream, so every hit is in place.
__global__ __launch_bounds__(256) void k_coop_resolve(CoopQ cq, uint32_t spp, const float4* __restrict__ hits,
                                                      uint32_t* __restrict__ rgba) {
    __shared__ uint32_t s_excl[kCoopShards], s_len[kCoopShards];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t len = min(cq.ctr[lane], cq.cap);
    uint32_t incl = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= (uint32_t)o) incl += y;
    }
    if (threadIdx.x < 64) {
        s_excl[lane] = incl - len;
        s_len[lane] = len;
    }
    __syncthreads();
    const uint32_t cnt = s_excl[63] + s_len[63];
    for (uint32_t e = blockIdx.x * 256 + threadIdx.x; e < cnt; e += gridDim.x * 256) {
        uint32_t sh = 0, sbase = 0;
        for (uint32_t k = 0; k < 64; ++k) {
            const uint32_t ek = s_excl[k];
            if (s_len[k] > 0 && ek <= e) { sh = k; sbase = ek; }
        }
        const uint4 a = cq.q[(uint64_t)(sh * cq.cap + (e - sbase)) * kCoopEntry];
        if (!(a.z & kCoopOne)) continue;
        const uint32_t pi = a.w;
        float r = 0.0f, g = 0.0f, b = 0.0f;
        for (uint32_t s = 0; s < spp; ++s) {
            const float4 h = hits[(uint64_t)pi * spp + s];
            if (__float_as_uint(h.w) != RT_SENT) {
                r = r + h.y;
                g = g + h.z;
                b = b + ((1.0f - h.y) - h.z);
            } else {
                r = r + 0.0f; g = g + 0.0f; b = b + 0.0f;
            }
        }
        const float sc = 1.0f / (float)spp;
        rgba[pi] = q8(r * sc) | (q8(g * sc) << 8) | (q8(b * sc) << 16) | (255u << 24);
    }
}

// ---------------------------------------------------------------- path mode
// Path mode [SPEC, DESIGN.md "Path mode"; SURVEY.md §8(f) row 3]: per
// sample a diffuse path of up to 1 + max_depth segments; at every hit a
// shadow ray toward the point light when it is above the surface (next-event
// estimation) and, below max_depth, a cosine-weighted bounce.  Operation
// order as orc_render_path.
//
// Megakernel with ONE trace call site: each lane runs a small state machine
// (segment / shadow ray / next sample) around a single trace_gen, so lanes
// whose next ray is a shadow ray and lanes whose next ray is a bounce share
// the same traversal loop instead of running two divergent loops in turn.
__device__ __forceinline__ uint32_t path_next(uint32_t& st) { st = pcg_hash(st); return st; }
__device__ __forceinline__ float path_u01(uint32_t& st) { return (float)(path_next(st) >> 8) * 0x1p-24f; }

struct PathCfg { float light[3]; float sky; uint32_t max_depth; };

template <bool COUNT, int NT, int WA = 4>
__global__ __launch_bounds__(NT) void k_path(const void* __restrict__ nodes, const uint4* __restrict__ wnodes,
                                              uint32_t wcap, const float4* __restrict__ tri_s,
                                              const float* __restrict__ tris, uint32_t n, Cam cam, uint32_t W,
                                              uint32_t H, uint32_t spp, uint32_t tilesX, PathCfg pc,
                                              float4* __restrict__ hits, uint32_t* __restrict__ rgba,
                                              unsigned long long* __restrict__ counters) {
    __shared__ uint32_t s_ref[(StackOf<WA, NT>::v + 1) * NT];
    __shared__ uint16_t s_tn[(StackOf<WA, NT>::v + 1) * NT];
    constexpr uint32_t WPB = NT / 64;
    const uint32_t gw = blockIdx.x * WPB + (threadIdx.x >> 6);
    const uint32_t t = gw >> 2;
    const uint32_t l = threadIdx.x & 63, w = gw & 3;
    const uint32_t x = (t % tilesX) * 16 + (w & 1) * 8 + (l & 7), y = (t / tilesX) * 16 + (w >> 1) * 8 + (l >> 3);
    const char* nd = reinterpret_cast<const char*>(nodes);
    uint32_t cn = 0, ct = 0, crays = 0;
    if (x < W && y < H) {
        float r = 0.0f, g = 0.0f, b = 0.0f;
        float o[3], d[3], L[3], beta[3], alb[3], N[3], S[3], cosl = 0.0f, tmax = 0.0f;
        uint32_t s = 0, depth = 0, st = 0, sidx = 0;
        bool shadow = false;
        auto start_sample = [&]() {
            sidx = (y * W + x) * spp + s;
            ray_dir(cam, x, y, W, spp, s, d);
#pragma unroll
            for (int a = 0; a < 3; ++a) { o[a] = cam.eye[a]; L[a] = 0.0f; beta[a] = 1.0f; }
            st = pcg_hash(sidx ^ 0x5bd1e995u);
            depth = 0; shadow = false; tmax = __builtin_inff();
        };
        start_sample();
        for (;;) {
            float tb, hu, hv;
            uint32_t hp;
            trace_gen<COUNT, NT, false, WA>(nd, wnodes, wcap, tri_s, n, o, d, tmax, shadow, s_ref + threadIdx.x,
                                 s_tn + threadIdx.x, tb, hu, hv, hp, cn, ct);
            ++crays;
            bool bounce = false, done = false;
            if (!shadow) {
                if (depth == 0 && hits) hits[sidx] = make_float4(tb, hu, hv, __uint_as_float(hp));
                if (hp == RT_SENT) {
                    if (depth > 0) {
#pragma unroll
                        for (int a = 0; a < 3; ++a) L[a] = L[a] + beta[a] * pc.sky;
                    }
                    done = true;
                } else {
                    Surf f;
                    surface(tris, hp, o, d, tb, pc.light, f);
                    const uint32_t ha = pcg_hash(hp ^ 0x27d4eb2fu);
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        N[a] = f.N[a];
                        S[a] = f.S[a];
                        alb[a] = 0.25f + (float)((ha >> (8 * a)) & 0xFFu) * 0x1p-9f;
                    }
                    cosl = f.cosl;
                    if (cosl > 0.0f) {  // next: the shadow ray
                        shadow = true;
                        tmax = 1.0f;
#pragma unroll
                        for (int a = 0; a < 3; ++a) { o[a] = S[a]; d[a] = f.D[a]; }
                    } else {
                        bounce = true;
                    }
                }
            } else {
                if (hp == RT_SENT) {
#pragma unroll
                    for (int a = 0; a < 3; ++a) L[a] = L[a] + (beta[a] * alb[a]) * cosl;
                }
                bounce = true;
            }
            if (bounce) {
                if (depth == pc.max_depth) {
                    done = true;
                } else {
#pragma unroll
                    for (int a = 0; a < 3; ++a) beta[a] = beta[a] * alb[a];
                    float px = 0.0f, py = 0.0f, r2 = 0.0f;
                    for (int k = 0; k < 16; ++k) {
                        const float qx = path_u01(st) * 2.0f - 1.0f;
                        const float qy = path_u01(st) * 2.0f - 1.0f;
                        const float q2 = qx * qx + qy * qy;
                        if (q2 < 1.0f) { px = qx; py = qy; r2 = q2; break; }
                    }
                    const float z = sqrtf(1.0f - r2);
                    const float sg = N[2] >= 0.0f ? 1.0f : -1.0f;
                    const float ia = -1.0f / (sg + N[2]);
                    const float ib = (N[0] * N[1]) * ia;
                    const float T[3] = {1.0f + ((sg * N[0]) * N[0]) * ia, sg * ib, -(sg * N[0])};
                    const float B[3] = {ib, sg + (N[1] * N[1]) * ia, -N[1]};
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        d[a] = (px * T[a] + py * B[a]) + z * N[a];
                        o[a] = S[a];
                    }
                    shadow = false;
                    tmax = __builtin_inff();
                    ++depth;
                }
            }
            if (done) {
                r = r + L[0];
                g = g + L[1];
                b = b + L[2];
                if (++s == spp) break;
                start_sample();
            }
        }
        if (rgba) {
            const float sc = 1.0f / (float)spp;
            rgba[(uint64_t)y * W + x] = q8(r * sc) | (q8(g * sc) << 8) | (q8(b * sc) << 16) | (255u << 24);
        }
    }
    if (COUNT) {
        unsigned long long a = cn, bsum = ct, c = crays;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            a += __shfl_xor(a, off, 64);
            bsum += __shfl_xor(bsum, off, 64);
            c += __shfl_xor(c, off, 64);
        }
        if (l == 0) {
            atomicAdd(&counters[0], a);
            atomicAdd(&counters[1], bsum);
            atomicAdd(&counters[2], c);
        }
    }
}

// ------------------------------------------------------ path mode, wavefront
// The same paths as k_path, advanced depth by depth over all paths of a batch
// ("ray reordering"): k_pw_primary traces the
// primary rays tile by tile; k_pw_shade turns every path's pending results
// into its next rays (shadow ray and/or bounce), appended to a queue with one
// atomic per 1024-thread block; the queue is sorted by a coherence key (ray
// kind, direction octant, Morton code of the origin in the scene's centroid
// box); k_pw_trace traces the sorted queue, one ray per lane, so a wave's
// rays start close together and head the same way.  Each path's arithmetic
// is k_path's in the same order -- shadow result of depth k before the
// segment of depth k+1 -- so the image is bit-identical whatever the queue
// order (the numpy restatement in oracle/oracle_np.py is this schedule).
enum : uint32_t { kPfO = 0, kPfD = 3, kPfL = 6, kPfB = 9, kPfW = 12, kPfT = 15, kPathF = 16 };
enum : uint32_t { kPuSt = 0, kPuFl = 1, kPuPrim = 2, kPuVis = 3, kPathU = 4 };
enum : uint32_t { kFlShadow = 1, kFlSeg = 2 };

__device__ __forceinline__ uint32_t ray_key(const float* o, const float* d, bool shadow, const BuildParams& bp) {
    uint32_t q[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) q[a] = (uint32_t)fminf(fmaxf((o[a] - bp.lo[a]) * bp.inv[a] * 512.0f, 0.0f), 511.0f);
    const uint32_t m = (expand10(q[0]) << 2) | (expand10(q[1]) << 1) | expand10(q[2]);
    const uint32_t oct = (d[0] < 0.0f ? 1u : 0u) | (d[1] < 0.0f ? 2u : 0u) | (d[2] < 0.0f ? 4u : 0u);
    return (shadow ? 1u << 30 : 0u) | (oct << 27) | m;
}

template <bool COUNT, int WA = 4>
__global__ __launch_bounds__(256) void k_pw_primary(const void* __restrict__ nodes, const uint4* __restrict__ wnodes,
                                                     uint32_t wcap, const float4* __restrict__ tri_s, uint32_t n,
                                                     Cam cam, uint32_t W, uint32_t H, uint32_t spp, uint32_t tilesX,
                                                     uint32_t t0, float* __restrict__ pf, uint32_t* __restrict__ pu,
                                                     uint32_t cap, float4* __restrict__ hits,
                                                     unsigned long long* __restrict__ counters) {
    __shared__ uint32_t s_ref[(WideFmt<WA>::stack + 1) * 256];
    __shared__ uint16_t s_tn[(WideFmt<WA>::stack + 1) * 256];
    const uint32_t t = t0 + blockIdx.x;
    const uint32_t l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t lx = (wv & 1) * 8 + (l & 7), ly = (wv >> 1) * 8 + (l >> 3);
    const uint32_t x = (t % tilesX) * 16 + lx, y = (t / tilesX) * 16 + ly;
    const uint32_t pbase = (blockIdx.x * 256 + ly * 16 + lx) * spp;
    uint32_t cn = 0, ct = 0;
    const bool valid = x < W && y < H;
    for (uint32_t s = 0; s < spp; ++s) {
        const uint32_t pid = pbase + s;
        if (!valid) { pu[kPuFl * cap + pid] = 0u; continue; }
        const uint32_t sidx = (y * W + x) * spp + s;
        float d[3], tb, hu, hv;
        uint32_t hp;
        ray_dir(cam, x, y, W, spp, s, d);
        trace_gen<COUNT, 256, false, WA>(reinterpret_cast<const char*>(nodes), wnodes, wcap, tri_s, n, cam.eye, d,
                              __builtin_inff(), false, s_ref + threadIdx.x, s_tn + threadIdx.x, tb, hu, hv, hp, cn, ct);
        if (hits) hits[sidx] = make_float4(tb, hu, hv, __uint_as_float(hp));
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            pf[(kPfO + a) * cap + pid] = cam.eye[a];
            pf[(kPfD + a) * cap + pid] = d[a];
            pf[(kPfL + a) * cap + pid] = 0.0f;
            pf[(kPfB + a) * cap + pid] = 1.0f;
        }
        pf[kPfT * cap + pid] = tb;
        pu[kPuSt * cap + pid] = pcg_hash(sidx ^ 0x5bd1e995u);
        pu[kPuFl * cap + pid] = kFlSeg;
        pu[kPuPrim * cap + pid] = hp;
    }
    if (COUNT) {
        unsigned long long a = cn, bsum = ct, c = valid ? spp : 0u;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            a += __shfl_xor(a, off, 64);
            bsum += __shfl_xor(bsum, off, 64);
            c += __shfl_xor(c, off, 64);
        }
        if (l == 0) {
            atomicAdd(&counters[0], a);
            atomicAdd(&counters[1], bsum);
            atomicAdd(&counters[2], c);
        }
    }
}

// One path's step at `depth`: the pending shadow result of depth-1, then the
// pending segment of depth; emits the path's next rays into the queue.
__global__ __launch_bounds__(1024) void k_pw_shade(float* __restrict__ pf, uint32_t* __restrict__ pu, uint32_t cap,
                                                   uint32_t np, uint32_t depth, PathCfg pc,
                                                   const float* __restrict__ tris,
                                                   const BuildParams* __restrict__ params,
                                                   float4* __restrict__ rays, uint32_t* __restrict__ keys,
                                                   uint32_t* __restrict__ vals, uint32_t* __restrict__ qcount) {
    __shared__ uint32_t s_wave[16];
    __shared__ uint32_t s_base;
    const uint32_t pid = blockIdx.x * 1024 + threadIdx.x;
    const uint32_t l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t fl = pid < np ? pu[kPuFl * cap + pid] : 0u;
    bool emit_sh = false, emit_bo = false;
    float S[3], D[3], nd[3];
    if (fl) {
        float L[3], beta[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) { L[a] = pf[(kPfL + a) * cap + pid]; beta[a] = pf[(kPfB + a) * cap + pid]; }
        if ((fl & kFlShadow) && pu[kPuVis * cap + pid]) {
#pragma unroll
            for (int a = 0; a < 3; ++a) L[a] = L[a] + pf[(kPfW + a) * cap + pid];
        }
        if (fl & kFlSeg) {
            const uint32_t prim = pu[kPuPrim * cap + pid];
            if (prim == RT_SENT) {
                if (depth > 0) {
#pragma unroll
                    for (int a = 0; a < 3; ++a) L[a] = L[a] + beta[a] * pc.sky;
                }
            } else {
                float o[3], d[3], alb[3];
#pragma unroll
                for (int a = 0; a < 3; ++a) { o[a] = pf[(kPfO + a) * cap + pid]; d[a] = pf[(kPfD + a) * cap + pid]; }
                Surf f;
                surface(tris, prim, o, d, pf[kPfT * cap + pid], pc.light, f);
                const uint32_t ha = pcg_hash(prim ^ 0x27d4eb2fu);
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    alb[a] = 0.25f + (float)((ha >> (8 * a)) & 0xFFu) * 0x1p-9f;
                    S[a] = f.S[a];
                    D[a] = f.D[a];
                }
                if (f.cosl > 0.0f) {
                    emit_sh = true;
#pragma unroll
                    for (int a = 0; a < 3; ++a) pf[(kPfW + a) * cap + pid] = (beta[a] * alb[a]) * f.cosl;
                }
                if (depth < pc.max_depth) {
                    emit_bo = true;
#pragma unroll
                    for (int a = 0; a < 3; ++a) beta[a] = beta[a] * alb[a];
                    uint32_t st = pu[kPuSt * cap + pid];
                    float px = 0.0f, py = 0.0f, r2 = 0.0f;
                    for (int k = 0; k < 16; ++k) {
                        const float qx = path_u01(st) * 2.0f - 1.0f;
                        const float qy = path_u01(st) * 2.0f - 1.0f;
                        const float q2 = qx * qx + qy * qy;
                        if (q2 < 1.0f) { px = qx; py = qy; r2 = q2; break; }
                    }
                    pu[kPuSt * cap + pid] = st;
                    const float* N = f.N;
                    const float z = sqrtf(1.0f - r2);
                    const float sg = N[2] >= 0.0f ? 1.0f : -1.0f;
                    const float ia = -1.0f / (sg + N[2]);
                    const float ib = (N[0] * N[1]) * ia;
                    const float T[3] = {1.0f + ((sg * N[0]) * N[0]) * ia, sg * ib, -(sg * N[0])};
                    const float B[3] = {ib, sg + (N[1] * N[1]) * ia, -N[1]};
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        nd[a] = (px * T[a] + py * B[a]) + z * N[a];
                        pf[(kPfO + a) * cap + pid] = S[a];
                        pf[(kPfD + a) * cap + pid] = nd[a];
                        pf[(kPfB + a) * cap + pid] = beta[a];
                    }
                }
            }
        }
#pragma unroll
        for (int a = 0; a < 3; ++a) pf[(kPfL + a) * cap + pid] = L[a];
        pu[kPuFl * cap + pid] = (emit_sh ? kFlShadow : 0u) | (emit_bo ? kFlSeg : 0u);
    }
    // queue slots: wave ballots, a block scan over the 16 waves, one atomic
    const uint64_t bs = __ballot(emit_sh), bb = __ballot(emit_bo);
    const uint32_t nsh = (uint32_t)__popcll(bs), nw = nsh + (uint32_t)__popcll(bb);
    if (l == 0) s_wave[wv] = nw;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int k = 0; k < 16; ++k) { const uint32_t c = s_wave[k]; s_wave[k] = tot; tot += c; }
        s_base = tot ? atomicAdd(qcount, tot) : 0u;
    }
    __syncthreads();
    const uint32_t wbase = s_base + s_wave[wv];
    const BuildParams bp = *params;
    if (emit_sh) {
        const uint32_t slot = wbase + lanes_below(bs);
        rays[2 * (uint64_t)slot] = make_float4(S[0], S[1], S[2], 1.0f);
        rays[2 * (uint64_t)slot + 1] = make_float4(D[0], D[1], D[2], __uint_as_float(pid | 0x80000000u));
        keys[slot] = ray_key(S, D, true, bp);
        vals[slot] = slot;
    }
    if (emit_bo) {
        const uint32_t slot = wbase + nsh + lanes_below(bb);
        rays[2 * (uint64_t)slot] = make_float4(S[0], S[1], S[2], __builtin_inff());
        rays[2 * (uint64_t)slot + 1] = make_float4(nd[0], nd[1], nd[2], __uint_as_float(pid));
        keys[slot] = ray_key(S, nd, false, bp);
        vals[slot] = slot;
    }
}

template <bool COUNT, int WA = 4>
__global__ __launch_bounds__(256) void k_pw_trace(const void* __restrict__ nodes, const uint4* __restrict__ wnodes,
                                                   uint32_t wcap, const float4* __restrict__ tri_s, uint32_t n,
                                                   const float4* __restrict__ rays, const uint32_t* __restrict__ order,
                                                   uint32_t count, const uint32_t* __restrict__ count_dev,
                                                   float* __restrict__ pf, uint32_t* __restrict__ pu,
                                                   uint32_t cap, unsigned long long* __restrict__ counters) {
    __shared__ uint32_t s_ref[(WideFmt<WA>::stack + 1) * 256];
    __shared__ uint16_t s_tn[(WideFmt<WA>::stack + 1) * 256];
    if (count_dev) count = *count_dev;  // grid sized for the bound, queue length read here
    if (blockIdx.x * 256 >= count) return;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint32_t cn = 0, ct = 0;
    if (i < count) {
        const uint32_t r = order ? order[i] : i;
        const float4 A = rays[2 * (uint64_t)r], B = rays[2 * (uint64_t)r + 1];
        const float o[3] = {A.x, A.y, A.z}, d[3] = {B.x, B.y, B.z};
        const uint32_t tag = __float_as_uint(B.w), pid = tag & 0x7FFFFFFFu;
        const bool shadow = tag >> 31;
        float tb, hu, hv;
        uint32_t hp;
        trace_gen<COUNT, 256, false, WA>(reinterpret_cast<const char*>(nodes), wnodes, wcap, tri_s, n, o, d, A.w, shadow,
                              s_ref + threadIdx.x, s_tn + threadIdx.x, tb, hu, hv, hp, cn, ct);
        if (shadow) {
            pu[kPuVis * cap + pid] = hp == RT_SENT ? 1u : 0u;
        } else {
            pf[kPfT * cap + pid] = tb;
            pu[kPuPrim * cap + pid] = hp;
        }
    }
    if (COUNT) {
        unsigned long long a = cn, bsum = ct, c = i < count ? 1u : 0u;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            a += __shfl_xor(a, off, 64);
            bsum += __shfl_xor(bsum, off, 64);
            c += __shfl_xor(c, off, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&counters[0], a);
            atomicAdd(&counters[1], bsum);
            atomicAdd(&counters[2], c);
        }
    }
}

__global__ __launch_bounds__(256) void k_pw_finish(const float* __restrict__ pf, uint32_t cap, uint32_t W, uint32_t H,
                                                   uint32_t spp, uint32_t tilesX, uint32_t t0,
                                                   uint32_t* __restrict__ rgba) {
    const uint32_t t = t0 + blockIdx.x;
    const uint32_t l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t lx = (wv & 1) * 8 + (l & 7), ly = (wv >> 1) * 8 + (l >> 3);
    const uint32_t x = (t % tilesX) * 16 + lx, y = (t / tilesX) * 16 + ly;
    if (x >= W || y >= H) return;
    const uint32_t pbase = (blockIdx.x * 256 + ly * 16 + lx) * spp;
    float r = 0.0f, g = 0.0f, b = 0.0f;
    for (uint32_t s = 0; s < spp; ++s) {
        r = r + pf[(kPfL + 0) * cap + pbase + s];
        g = g + pf[(kPfL + 1) * cap + pbase + s];
        b = b + pf[(kPfL + 2) * cap + pbase + s];
    }
    const float sc = 1.0f / (float)spp;
    rgba[(uint64_t)y * W + x] = q8(r * sc) | (q8(g * sc) << 8) | (q8(b * sc) << 16) | (255u << 24);
}

// Gathered slabs [rank][tile][256 px] -> W x H image.
__global__ __launch_bounds__(256) void k_unpack(const uint32_t* __restrict__ slabs, uint32_t tiles_per_slab, uint32_t W,
                                                uint32_t H, uint32_t nranks, uint32_t tilesX, uint32_t ntiles,
                                                uint32_t* __restrict__ img) {
    const uint32_t rk = blockIdx.x / tiles_per_slab, b = blockIdx.x % tiles_per_slab;
    const uint32_t t = rk + b * nranks;
    if (t >= ntiles) return;
    const uint32_t tx = t % tilesX, ty = t / tilesX;
    const uint32_t lx = threadIdx.x & 15, ly = threadIdx.x >> 4;
    const uint32_t x = tx * 16 + lx, y = ty * 16 + ly;
    if (x < W && y < H) img[(uint64_t)y * W + x] = slabs[(uint64_t)blockIdx.x * 256 + threadIdx.x];
}

// Gathered hit slabs [rank][tile][256 px][spp] -> hits[(y*W+x)*spp + s].
__global__ __launch_bounds__(256) void k_unpack_hits(const float4* __restrict__ slabs, uint32_t tiles_per_slab,
                                                     uint32_t W, uint32_t H, uint32_t spp, uint32_t nranks,
                                                     uint32_t tilesX, uint32_t ntiles, float4* __restrict__ hits) {
    const uint32_t rk = blockIdx.x / tiles_per_slab, b = blockIdx.x % tiles_per_slab;
    const uint32_t t = rk + b * nranks;
    if (t >= ntiles) return;
    const uint32_t tx = t % tilesX, ty = t / tilesX;
    const uint32_t lx = threadIdx.x & 15, ly = threadIdx.x >> 4;
    const uint32_t x = tx * 16 + lx, y = ty * 16 + ly;
    if (x >= W || y >= H) return;
    const uint64_t src = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * spp, dst = ((uint64_t)y * W + x) * spp;
    for (uint32_t s = 0; s < spp; ++s) hits[dst + s] = slabs[src + s];
}

// KAT entry point: Moller-Trumbore per (o, d, tri, t_best).
__global__ void k_intersect(uint32_t count, const float* __restrict__ o, const float* __restrict__ d,
                            const float* __restrict__ tri, const float* __restrict__ tbest,
                            uint32_t* __restrict__ hit, float* __restrict__ tuv) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    float t = 0.0f, u = 0.0f, v = 0.0f;
    float oo[3] = {o[3 * i], o[3 * i + 1], o[3 * i + 2]};
    float dd[3] = {d[3 * i], d[3 * i + 1], d[3 * i + 2]};
    float tt[9];
#pragma unroll
    for (int c = 0; c < 9; ++c) tt[c] = tri[9 * i + c];
    const bool h = intersect_tri(oo, dd, tt, tbest[i], t, u, v);
    hit[i] = h ? 1u : 0u;
    tuv[3 * i] = t; tuv[3 * i + 1] = u; tuv[3 * i + 2] = v;
}

// Semantics probe of the device min/max the whole contract relies on.
__global__ void k_minmax(uint32_t count, const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    out[2 * i] = fminf(a[i], b[i]);
    out[2 * i + 1] = fmaxf(a[i], b[i]);
}


// ================================================================ launchers
uint32_t tiles_for_rank(uint32_t w, uint32_t h, uint32_t rank, uint32_t nranks) {
    const uint32_t nt = ((w + 15) / 16) * ((h + 15) / 16);
    if (!nranks || rank >= nranks || rank >= nt) return 0;
    return (nt - rank + nranks - 1) / nranks;
}

namespace {
TraceConfig initial_config() {
    TraceConfig c;
    const char* p = std::getenv("RT_DEBUG_POISON");
    const char* l = std::getenv("RT_DEBUG_LDS_SCRIBBLE");
    c.poison = (p && std::strcmp(p, "1") == 0) ? 1u : 0u;
    c.lds_scribble = (l && std::strcmp(l, "1") == 0) ? 1u : 0u;
    return c;
}
TraceConfig g_trace_config = initial_config();
std::mutex g_config_mu;
std::atomic<uint32_t> g_lds_scribble{g_trace_config.lds_scribble};
std::atomic<uint32_t> g_scribble_seed{0x9E3779B9u};
}  // namespace

// debug.lds_scribble: fill as much of every CU's 160 KB LDS as the
// dispatcher gives us (4 blocks x 40 KB per CU requested) with a pattern
// that changes every launch.  The dummy global store keeps the LDS writes
// alive; it never fires (no block reads the pattern it is looking for).
constexpr uint32_t kScribbleBytes = 40 * 1024;
__global__ __launch_bounds__(256) void k_lds_scribble(uint32_t seed, uint32_t* __restrict__ never) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_scr[];
    uint32_t h = pcg_hash(seed ^ (blockIdx.x * 0x85EBCA6Bu) ^ threadIdx.x);
    for (uint32_t i = threadIdx.x; i < kScribbleBytes / 4; i += 256) {
        h = pcg_hash(h + i);
        s_scr[i] = h;
    }
    __syncthreads();
    if (s_scr[(threadIdx.x * 7u) % (kScribbleBytes / 4)] == seed && seed == 0u) never[0] = 1u;
}

void lds_scribble_if(hipStream_t s) {
    if (!g_lds_scribble.load(std::memory_order_relaxed)) return;
    static std::once_flag once;
    std::call_once(once, [] {
        (void)hipFuncSetAttribute((const void*)k_lds_scribble, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)kScribbleBytes);
    });
    const uint32_t seed = g_scribble_seed.fetch_add(0x6D2B79F5u, std::memory_order_relaxed) | 1u;
    hipLaunchKernelGGL(k_lds_scribble, dim3(1024), dim3(256), kScribbleBytes, s, seed, (uint32_t*)nullptr);
}

TraceConfig config_snapshot() {
    std::lock_guard<std::mutex> lk(g_config_mu);
    return g_trace_config;
}

bool config_apply(bool (*f)(TraceConfig&, const char*, int64_t), const char* key, int64_t value) {
    std::lock_guard<std::mutex> lk(g_config_mu);
    TraceConfig c = g_trace_config;
    if (!f(c, key, value)) return false;
    g_trace_config = c;
    g_lds_scribble.store(c.lds_scribble, std::memory_order_relaxed);
    return true;
}

hipError_t dev_alloc(void** p, size_t bytes) {
    *p = nullptr;
    hipError_t e = hipMalloc(p, bytes ? bytes : 16);
    if (e != hipSuccess || !config_snapshot().poison) return e;
    // debug.poison: 0xFF in every byte (a NaN float, RT_SENT index, 255 plane),
    // finished before any stream can use the buffer.  The fill runs on a
    // private non-blocking stream of the current device and only that stream
    // is waited for (a device-wide synchronize here would also
    // wait for -- and hide the ordering of -- other scenes' in-flight work).
    static std::once_flag once[kMaxDevices];
    static hipStream_t fill[kMaxDevices];
    int dev = 0;
    if ((e = hipGetDevice(&dev)) == hipSuccess && (dev < 0 || dev >= kMaxDevices)) e = hipErrorInvalidDevice;
    if (e == hipSuccess) {
        std::call_once(once[dev], [dev] { (void)hipStreamCreateWithFlags(&fill[dev], hipStreamNonBlocking); });
        e = fill[dev] ? hipMemsetAsync(*p, 0xFF, bytes ? bytes : 16, fill[dev]) : hipErrorInvalidResourceHandle;
    }
    if (e == hipSuccess) e = hipStreamSynchronize(fill[dev]);
    if (e != hipSuccess) {
        (void)hipFree(*p);
        *p = nullptr;
    }
    return e;
}

// the wide stack entries a launch of NT-thread blocks uses: trace.stack_cap
// (tests force overflows with small values), at most the kernel's stack
// (StackOf: arity and block size); 0 = all of it
static uint32_t stack_cap_for(const TraceConfig& cfg, uint32_t warity, uint32_t nt) {
    const uint32_t full = warity == 8   ? (uint32_t)StackOf<8, 256>::v
                          : nt == 64    ? (uint32_t)StackOf<4, 64>::v
                                        : (uint32_t)StackOf<4, 256>::v;
    return cfg.stack_cap ? min(cfg.stack_cap, full) : full;
}

// k_trace with the record arity and load form chosen at run time (the
// binary kernel, WI = false, has one form)
#ifndef RT_SPP1
#define RT_SPP1 1  // 0: 1-spp full frames run the generic kernel (A/B)
#endif
// One rank's 1-spp tiles run the 1-spp instance too (r04): 77 VGPRs, 6 waves
// per SIMD with the 16-entry tile stacks (RT_WIDE_STACK64).  No faster at
// P = 4 / 8, where a rank's waves are resident at once; at P = 2 (1.6
// rounds of waves) the orbit's max over ranks 0.2247 -> 0.2099 ms
// (profiles/ab_tile_spp1_stack16_r04.log).  0: the generic kernel (A/B).
#ifndef RT_SPP1_TILES
#define RT_SPP1_TILES 1
#endif
template <bool C, bool P, bool WI, int NT, typename... A>
static void k_trace_go(bool buf, uint32_t warity, bool cq, bool spp1, uint32_t grid, hipStream_t s, A... a) {
    if constexpr (WI) {
        if (warity == 8) {
            if (cq) RT_KLAUNCH((k_trace<C, P, true, NT, false, true, 8, true>), dim3(grid), dim3(NT), 0, s, a...);
            else RT_KLAUNCH((k_trace<C, P, true, NT, false, true, 8, false>), dim3(grid), dim3(NT), 0, s, a...);
            return;
        }
        if (buf) {
            // (one rank's tiles: the 1-spp instance since r04, RT_SPP1_TILES; r03 measured it
            // no faster per rank on the static camera, profiles/ab_occupancy_r03.log)
            if (cq && RT_SPP1 && !C && (RT_SPP1_TILES ? true : !P && NT == 256) && spp1)  // full frames with the queue (trace.coop_cap)
                RT_KLAUNCH((k_trace<C, P, true, NT, false, true, 4, true, 1>), dim3(grid), dim3(NT), 0, s, a...);
            else if (cq) RT_KLAUNCH((k_trace<C, P, true, NT, false, true, 4, true>), dim3(grid), dim3(NT), 0, s, a...);
            else if (RT_SPP1 && !C && !P && NT == 256 && spp1)  // the headline kernel: 1 spp full frames
                RT_KLAUNCH((k_trace<C, P, true, NT, false, true, 4, false, 1>), dim3(grid), dim3(NT), 0, s, a...);
            else RT_KLAUNCH((k_trace<C, P, true, NT, false, true, 4, false>), dim3(grid), dim3(NT), 0, s, a...);
            return;
        }
    }
    RT_KLAUNCH((k_trace<C, P, WI, NT, false, false, 4>), dim3(grid), dim3(NT), 0, s, a...);
}

hipError_t launch_trace(const void* nodes, const uint4* wnodes, uint32_t warity, const float4* tris, uint32_t n,
                        const CamF& c, uint32_t w, uint32_t h, uint32_t spp, uint32_t rank, uint32_t nranks,
                        bool packed, void* hits, void* rgba, unsigned long long* counters, bool binary_counts,
                        TileSched* sched, hipStream_t s) {
    const TraceConfig cfg = config_snapshot();
    const uint32_t nb = tiles_for_rank(w, h, rank, nranks);
    if (!nb) return hipSuccess;
    Cam cam;
    for (int i = 0; i < 3; ++i) {
        cam.eye[i] = c.eye[i]; cam.w00[i] = c.w00[i]; cam.du[i] = c.du[i]; cam.dv[i] = c.dv[i];
    }
    const uint32_t tilesX = (w + 15) / 16;
    float4* H = reinterpret_cast<float4*>(hits);
    uint32_t* R = reinterpret_cast<uint32_t*>(rgba);
    if (warity != 4 && warity != 8) return hipErrorInvalidValue;
    if (warity == 8 && n > kWide8MaxN) return hipErrorInvalidValue;  // the build keeps 8-ary records to n <= kWide8MaxN
    // wide (4-ary) traversal unless asked for the binary one: variant 2, no
    // K7w records (stage entry points), n < 2, or binary work counters
    const bool wide = wnodes && n >= 2 && cfg.variant != 2 && !binary_counts;
    const bool small = (nranks > 1 ? cfg.wg_tiles : cfg.wg) == 64;
    // costliest tiles first from the previous frame's map (DESIGN.md "Tile order")
    const uint32_t* order = nullptr;
    uint32_t* cost_out = nullptr;
    // full frames on 256-thread wide kernels (no queue, no counters): the
    // next frame's order is sorted by an extra block of this launch
    // (OrderFold) instead of a k_tile_order launch ahead of it
    // heavy rays to k_trace_coop (DESIGN.md "Cooperative heavy rays")
    uint32_t coop_cap0 =
        wide && sched && sched->coop_q && n <= kBufMaxN
            ? (nranks > 1 ? coop_cap_for_tiles(cfg.coop_cap_tiles, nranks) : coop_cap_for_frame(cfg.coop_cap, spp, small))
            : 0u;
    // queue skip: with the automatic cap, a frame shape whose last queue-on frame queued fewer than
    // kQueueSkip rays runs without the queue (its pass would be all launch and order sort), re-probing
    // every kQueueProbe-th frame (an explicit cap always runs the queue).  Best effort: q_host may be a
    // few frames old (TileSched::q_host); it picks the schedule, never a result.
    const bool cap_auto = (nranks > 1 ? cfg.coop_cap_tiles : cfg.coop_cap) == kCoopCapAuto;
    if (coop_cap0 && cap_auto && sched->q_host) {
        if (__atomic_load_n(sched->q_host, __ATOMIC_RELAXED) < kQueueSkip && sched->q_frames + 1 < kQueueProbe) {
            coop_cap0 = 0u;
            ++sched->q_frames;
        } else {
            sched->q_frames = 0;
        }
    }
    // samples in lanes (k_trace_sl): multi-spp tiles and full frames (trace.spp_lanes = 2, the default;
    // 1 = tiles only)
    const bool sl = spp >= 2 && spp <= 16 && (spp & (spp - 1)) == 0 && wide && warity == 4 && !counters &&
                    n <= kBufMaxN &&
                    (cfg.spp_lanes == 2 || (cfg.spp_lanes == 1 && (packed || nranks > 1)));
    // its queue needs the hits of every sample (k_coop_resolve), so no queue without a hits buffer
    const uint32_t sl_cap = !sl || !hits || !sched || !sched->coop_q ? 0u
                            : coop_cap_for_sl(nranks > 1 ? cfg.coop_cap_tiles : cfg.coop_cap);
    const uint32_t coop_cap = sl ? sl_cap : coop_cap0;
    // (k_trace's extra block holds its costs in registers: nb <= 8192, full frames; k_trace_sl's block 0
    // loops, any nb, full frames and one rank's tiles)
    // (with the heavy-ray queue on, k_trace_coop's block 0 sorts this frame's costs instead)
    const bool can_fold = RT_ORDER_FOLD && sched && wide && !counters && !cfg.order_override && coop_cap == 0 &&
                          (sl || (nranks == 1 && !packed && !small && nb <= 256 * kFoldPerThread));
    OrderFold fold;
    if (sched && cfg.tile_order && nb <= 1024 * kOrderPerThread) {
        if (sched->fresh) {  // new maps: clear both once (k_tile_order clears the one it reads)
            hipError_t me = hipMemsetAsync(sched->cost_prev, 0, (size_t)nb * 4, s);
            if (me == hipSuccess) me = hipMemsetAsync(sched->cost_cur, 0, (size_t)nb * 4, s);
            if (me == hipSuccess) me = hipMemsetAsync(sched->cost_ema, 0, (size_t)nb * 4, s);
            if (me != hipSuccess) return me;
            sched->fresh = false;
        }
        if (sched->have_prev) {
            // computed already by the previous frame (its k_trace_coop for one rank's tiles, its
            // k_trace's extra block for full frames), else here -- except that the first frame
            // that folds runs in row-major order
            if (sched->order_ready) {
                order = sched->order;
            } else if (!can_fold) {
                RT_KLAUNCH(k_tile_order, dim3(1), dim3(1024), 0, s, sched->cost_prev, nb, sched->order,
                                   sched->cost_ema);
                order = sched->order;
            }
            if (can_fold) {
                fold.cost = sched->cost_prev;
                fold.out = sched->order_next;
                fold.ema = sched->cost_ema;
                fold.nb = nb;
            }
        }
        sched->order_ready = false;
        cost_out = sched->cost_cur;
    }
    if (cfg.order_override) order = cfg.order_override;
    const uint16_t* px_prev = nullptr;
    uint16_t* px_cost = nullptr;
    // full frames only by default: a frame is issue-bound and the sort cuts the
    // instructions its costly tiles issue; one rank's share of a multi-GPU
    // frame is bound by its slowest wave, which a wave of 64 costly rays
    // (more lanes in both branches of every step) only lengthens
    // (DESIGN.md "Pixel order").  256-thread blocks only (the ranking is per
    // block).
    //
    // The previous frame's per-pixel costs describe this frame's pixels only
    // when the camera has not moved: with the bench's orbit (0.25 deg per
    // frame, a few pixels of image motion) the stale order put lanes of
    // different cost together and cost 3 % (0.372 vs 0.383 ms,
    // profiles/ab_moving_r02.log), so after a camera change the frame keeps
    // the quadrant layout and only records its costs for the next one.
    if (cost_out && !small && !sl && sched->px_cur &&
        (cfg.px_sort == 2 || (cfg.px_sort == 1 && nranks == 1))) {
        const bool same_cam = sched->prev_cam_valid && std::memcmp(&sched->prev_cam, &c, sizeof(CamF)) == 0;
        if (sched->have_prev && same_cam) px_prev = sched->px_prev;
        px_cost = sched->px_cur;
    }
    if (sched) {
        sched->prev_cam = c;
        sched->prev_cam_valid = true;
    }
    CoopQ cq;
    if (coop_cap) {
        if (sched->coop_fresh) {
            hipError_t me = hipMemsetAsync(sched->coop_ctr, 0, 2 * kCoopShards * sizeof(uint32_t), s);
            if (me != hipSuccess) return me;
            sched->coop_fresh = false;
        }
        cq.q = sched->coop_q;
        cq.ctr = sched->coop_ctr + sched->coop_par * kCoopShards;
        cq.ctr_next = sched->coop_ctr + (sched->coop_par ^ 1u) * kCoopShards;
        cq.cap = sched->coop_qcap / kCoopShards;
    }
    // buffer loads for the wide step whenever the offsets fit 32 bits (WideMem)
    const bool buf = n <= kBufMaxN;
    // nontemporal hit records, every frame (r05: 10M K0 after a 4Kx4 frame 104.5 -> 82.8 us, the 1M build
    // after a 1080p1 frame 140.3 -> 137.7 us, frames unchanged; profiles/ab_nt_hits_1spp_r05.log)
    const uint32_t nt_hits = 1u;
#define RT_TRACE_NT(C, P, WI, NT)                                                                                    \
    k_trace_go<C, P, WI, NT>(buf, warity, coop_cap != 0, spp == 1, nb * (256 / NT) + (fold.out ? 1u : 0u), s, nodes, \
                             wnodes, stack_cap_for(cfg, warity, NT), tris, n,                                            \
                             cam, w, h, spp, rank, nranks, tilesX, H, R, counters, (const float*)nullptr, Light{},      \
                             order, cost_out, px_prev, px_cost, coop_cap, cq, fold, nt_hits)
#define RT_TRACE(C, P, WI) \
    if (small) RT_TRACE_NT(C, P, WI, 64); else RT_TRACE_NT(C, P, WI, 256)
#define RT_TRACE_W(C, P)           \
    if (wide) {                    \
        RT_TRACE(C, P, true);      \
    } else {                       \
        RT_TRACE(C, P, false);     \
    }
    if (sl) {
        const uint32_t nt = small ? 64u : 256u;
        const uint32_t grid = (uint32_t)((uint64_t)nb * 4 * spp / (nt / 64)) + (fold.out ? 1u : 0u);
        const uint32_t wc = stack_cap_for(cfg, 4, nt);
#define RT_SL(P, NT, S_)                                                                                             \
    RT_KLAUNCH((k_trace_sl<P, NT, S_>), dim3(grid), dim3(NT), 0, s, nodes, wnodes, wc, tris, n, cam, w, h, rank, \
               nranks, tilesX, H, R, order, cost_out, coop_cap, cq, nt_hits, fold)
#define RT_SL_S(P, NT)                  \
    switch (spp) {                      \
        case 2: RT_SL(P, NT, 2); break;   \
        case 4: RT_SL(P, NT, 4); break;   \
        case 8: RT_SL(P, NT, 8); break;   \
        default: RT_SL(P, NT, 16); break; \
    }
        if (packed) {
            if (small) { RT_SL_S(true, 64); } else { RT_SL_S(true, 256); }
        } else {
            if (small) { RT_SL_S(false, 64); } else { RT_SL_S(false, 256); }
        }
#undef RT_SL_S
#undef RT_SL
    } else if (counters) {
        if (packed) { RT_TRACE_W(true, true); } else { RT_TRACE_W(true, false); }
    } else {
        if (packed) { RT_TRACE_W(false, true); } else { RT_TRACE_W(false, false); }
    }
#undef RT_TRACE_W
#undef RT_TRACE
#undef RT_TRACE_NT
    if (fold.out) {  // the order this launch sorts is the next frame's
        std::swap(sched->order, sched->order_next);
        sched->order_ready = true;
    }
    if (coop_cap) {
        hipError_t le = hipGetLastError();
        if (le != hipSuccess) return le;
        uint32_t cgrid = kCoopGrid;
        {  // persistent grid = the resident capacity (per device and group width, computed once)
            static std::atomic<uint32_t> resident[kMaxDevices][3][2];
            int dev = 0;
            hipError_t e = hipGetDevice(&dev);
            if (e != hipSuccess) return e;
            if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
            const int gi = cfg.coop_lanes == 16 ? 0 : cfg.coop_lanes == 32 ? 1 : 2;
            const int ai = warity == 8 ? 1 : 0;
            uint32_t r = resident[dev][gi][ai].load(std::memory_order_relaxed);
            if (!r) {
                int per_cu = 0, cus = 0;
                const void* kf =
                    ai ? (gi == 0   ? reinterpret_cast<const void*>(k_trace_coop<false, false, 16, 8>)
                          : gi == 1 ? reinterpret_cast<const void*>(k_trace_coop<false, false, 32, 8>)
                                    : reinterpret_cast<const void*>(k_trace_coop<false, false, 64, 8>))
                       : (gi == 0   ? reinterpret_cast<const void*>(k_trace_coop<false, false, 16>)
                          : gi == 1 ? reinterpret_cast<const void*>(k_trace_coop<false, false, 32>)
                                    : reinterpret_cast<const void*>(k_trace_coop<false, false, 64>));
                if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kf, 256, 0)) != hipSuccess) return e;
                if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess)
                    return e;
                r = (uint32_t)(per_cu > 0 ? per_cu : 1) * (uint32_t)(cus > 0 ? cus : 1);
                resident[dev][gi][ai].store(r, std::memory_order_relaxed);
            }
            cgrid = r;
        }
        // block 0 sorts this frame's cost map into the next frame's tile order
        const bool ord = !fold.out && cost_out && !cfg.order_override && nb <= kOrderInCoop && cgrid > 1;
        uint32_t* ord_cost = ord ? cost_out : nullptr;
        uint32_t* ord_out = ord ? sched->order : nullptr;
        uint32_t* ord_ema = ord ? sched->cost_ema : nullptr;
#define RT_COOP_G(C, P, G)                                                                                        \
    if (warity == 8)                                                                                               \
        RT_KLAUNCH((k_trace_coop<C, P, G, 8>), dim3(cgrid), dim3(256), 0, s, nodes, wnodes, tris, n, cam, w, \
                           spp, cq, H, R, counters, ord_cost, nb, ord_out, ord_ema, sched->q_dev);                \
    else                                                                                                           \
        RT_KLAUNCH((k_trace_coop<C, P, G, 4>), dim3(cgrid), dim3(256), 0, s, nodes, wnodes, tris, n, cam, w, \
                           spp, cq, H, R, counters, ord_cost, nb, ord_out, ord_ema, sched->q_dev)
#define RT_COOP(C, P)                  \
    if (cfg.coop_lanes == 16) {        \
        RT_COOP_G(C, P, 16);           \
    } else if (cfg.coop_lanes == 32) { \
        RT_COOP_G(C, P, 32);           \
    } else {                           \
        RT_COOP_G(C, P, 64);           \
    }
        if (counters) {
            if (packed) { RT_COOP(true, true); } else { RT_COOP(true, false); }
        } else {
            if (packed) { RT_COOP(false, true); } else { RT_COOP(false, false); }
        }
#undef RT_COOP
#undef RT_COOP_G
        if (sl) {  // the colours of the pixels with a queued sample
            hipError_t le2 = hipGetLastError();
            if (le2 != hipSuccess) return le2;
            RT_KLAUNCH(k_coop_resolve, dim3(64), dim3(256), 0, s, cq, spp, H, R);
        }
        sched->coop_par ^= 1u;
        if (ord) sched->order_ready = true;
    }
    return hipGetLastError();
}

hipError_t launch_trace_shadow(const void* nodes, const uint4* wnodes, uint32_t warity, const float4* tri_s,
                               const float* tris, uint32_t n, const CamF& c, uint32_t w, uint32_t h, uint32_t spp,
                               const float light[3], float ambient, void* hits, void* rgba,
                               unsigned long long* counters, hipStream_t s) {
    const TraceConfig cfg = config_snapshot();
    const uint32_t nb = tiles_for_rank(w, h, 0, 1);
    if (!nb) return hipSuccess;
    Cam cam;
    for (int i = 0; i < 3; ++i) {
        cam.eye[i] = c.eye[i]; cam.w00[i] = c.w00[i]; cam.du[i] = c.du[i]; cam.dv[i] = c.dv[i];
    }
    Light lt;
    for (int i = 0; i < 3; ++i) lt.p[i] = light[i];
    lt.ambient = ambient;
    const uint32_t tilesX = (w + 15) / 16;
    float4* H = reinterpret_cast<float4*>(hits);
    uint32_t* R = reinterpret_cast<uint32_t*>(rgba);
    if (warity != 4 && warity != 8) return hipErrorInvalidValue;
    const bool wide = wnodes && n >= 2 && cfg.variant != 2;
    const uint32_t cap = stack_cap_for(cfg, warity, 256);
#define RT_SHADOW(C, WI, WW)                                                                                       \
    RT_KLAUNCH((k_trace<C, false, WI, 256, true, false, WW>), dim3(nb), dim3(256), 0, s, nodes, wnodes, cap, \
                       tri_s, n, cam, w, h, spp, 0u, 1u, tilesX, H, R, counters, tris, lt)
    if (counters) {
        if (wide && warity == 8) RT_SHADOW(true, true, 8);
        else if (wide) RT_SHADOW(true, true, 4);
        else RT_SHADOW(true, false, 4);
    } else {
        if (wide && warity == 8) RT_SHADOW(false, true, 8);
        else if (wide) RT_SHADOW(false, true, 4);
        else RT_SHADOW(false, false, 4);
    }
#undef RT_SHADOW
    return hipGetLastError();
}

hipError_t launch_trace_path(const void* nodes, const uint4* wnodes, uint32_t warity, const float4* tri_s,
                             const float* tris, uint32_t n, const CamF& c, uint32_t w, uint32_t h, uint32_t spp,
                             const float light[3], float sky, uint32_t max_depth, void* hits, void* rgba,
                             unsigned long long* counters, hipStream_t s) {
    const TraceConfig cfg = config_snapshot();
    const uint32_t nb = tiles_for_rank(w, h, 0, 1);
    if (!nb) return hipSuccess;
    Cam cam;
    for (int i = 0; i < 3; ++i) {
        cam.eye[i] = c.eye[i]; cam.w00[i] = c.w00[i]; cam.du[i] = c.du[i]; cam.dv[i] = c.dv[i];
    }
    PathCfg pc;
    for (int i = 0; i < 3; ++i) pc.light[i] = light[i];
    pc.sky = sky;
    pc.max_depth = max_depth;
    const uint32_t tilesX = (w + 15) / 16;
    float4* H = reinterpret_cast<float4*>(hits);
    uint32_t* R = reinterpret_cast<uint32_t*>(rgba);
    // K7w records unless the binary traversal is asked for (variant 2)
    const uint4* wn = (cfg.variant != 2) ? wnodes : nullptr;
    if (warity != 4 && warity != 8) return hipErrorInvalidValue;
    const bool small = cfg.path_wg == 64;
    const uint32_t cap = stack_cap_for(cfg, warity, small ? 64 : 256);
#define RT_PATH(C, NT)                                                                                                 \
    if (warity == 8)                                                                                                 \
        RT_KLAUNCH((k_path<C, NT, 8>), dim3(nb * (256 / NT)), dim3(NT), 0, s, nodes, wn, cap, tri_s, tris, n, \
                           cam, w, h, spp, tilesX, pc, H, R, counters);                                              \
    else                                                                                                             \
        RT_KLAUNCH((k_path<C, NT, 4>), dim3(nb * (256 / NT)), dim3(NT), 0, s, nodes, wn, cap, tri_s, tris, n, \
                           cam, w, h, spp, tilesX, pc, H, R, counters)
    if (counters) {
        if (small) { RT_PATH(true, 64); } else { RT_PATH(true, 256); }
    } else {
        if (small) { RT_PATH(false, 64); } else { RT_PATH(false, 256); }
    }
#undef RT_PATH
    return hipGetLastError();
}

hipError_t alloc_path(PathBufs& b, uint32_t cap) {
    free_path(b);
    const uint64_t q = 2ull * cap;
    hipError_t e;
    if ((e = dev_alloc(&b.f, (uint64_t)kPathF * cap * 4)) != hipSuccess) return e;
    if ((e = dev_alloc(&b.u, (uint64_t)kPathU * cap * 4)) != hipSuccess) return e;
    if ((e = dev_alloc(&b.rays, q * 32)) != hipSuccess) return e;
    for (int i = 0; i < 2; ++i) {
        if ((e = dev_alloc(&b.keys[i], q * 4)) != hipSuccess) return e;
        if ((e = dev_alloc(&b.vals[i], q * 4)) != hipSuccess) return e;
    }
    if ((e = dev_alloc(&b.counts, (uint64_t)sort_tiles((uint32_t)q) * 256 * 4 + 1024)) != hipSuccess) return e;
    if ((e = dev_alloc(&b.ghist, 4096 + 256)) != hipSuccess) return e;
    b.qcount = b.ghist + 1024;
    if ((e = hipHostMalloc((void**)&b.hq, 256, hipHostMallocDefault)) != hipSuccess) return e;
    b.cap = cap;
    return hipSuccess;
}

void free_path(PathBufs& b) {
    (void)hipFree(b.f);
    (void)hipFree(b.u);
    (void)hipFree(b.rays);
    for (int i = 0; i < 2; ++i) { (void)hipFree(b.keys[i]); (void)hipFree(b.vals[i]); }
    (void)hipFree(b.counts);
    (void)hipFree(b.ghist);
    if (b.hq) (void)hipHostFree(b.hq);
    b = PathBufs{};
}

hipError_t launch_path_wavefront(const void* nodes, const uint4* wnodes, uint32_t warity, const float4* tri_s,
                                 const float* tris, const BuildParams* params, uint32_t n, const CamF& c, uint32_t w,
                                 uint32_t h,
                                 uint32_t spp, const float light[3], float sky, uint32_t max_depth, void* hits,
                                 void* rgba, unsigned long long* counters, PathBufs& pb, uint32_t sort_digits,
                                 hipStream_t s) {
    const TraceConfig cfg = config_snapshot();
    const uint32_t nt = tiles_for_rank(w, h, 0, 1);
    if (!nt) return hipSuccess;
    const uint32_t per_tile = 256 * spp;
    if (pb.cap < per_tile) return hipErrorInvalidValue;
    Cam cam;
    for (int i = 0; i < 3; ++i) {
        cam.eye[i] = c.eye[i]; cam.w00[i] = c.w00[i]; cam.du[i] = c.du[i]; cam.dv[i] = c.dv[i];
    }
    PathCfg pc;
    for (int i = 0; i < 3; ++i) pc.light[i] = light[i];
    pc.sky = sky;
    pc.max_depth = max_depth;
    const uint32_t tilesX = (w + 15) / 16;
    const uint4* wn = (cfg.variant != 2) ? wnodes : nullptr;
    if (warity != 4 && warity != 8) return hipErrorInvalidValue;
    const uint32_t wcap = stack_cap_for(cfg, warity, 256);
    const bool w8 = warity == 8;
    const uint32_t batch = pb.cap / per_tile;
    float4* H = reinterpret_cast<float4*>(hits);
    hipError_t e;
    for (uint32_t t0 = 0; t0 < nt; t0 += batch) {
        const uint32_t nb = min(batch, nt - t0);
        const uint32_t np = nb * per_tile;
#define RT_PW_PRIMARY(C, WW)                                                                                  \
    RT_KLAUNCH((k_pw_primary<C, WW>), dim3(nb), dim3(256), 0, s, nodes, wn, wcap, tri_s, n, cam, w, h, spp, \
                       tilesX, t0, pb.f, pb.u, pb.cap, H, counters)
        if (counters) {
            if (w8) RT_PW_PRIMARY(true, 8); else RT_PW_PRIMARY(true, 4);
        } else {
            if (w8) RT_PW_PRIMARY(false, 8); else RT_PW_PRIMARY(false, 4);
        }
#undef RT_PW_PRIMARY
        for (uint32_t depth = 0; depth <= max_depth + 1; ++depth) {
            if ((e = hipMemsetAsync(pb.qcount, 0, 4, s)) != hipSuccess) return e;
            RT_KLAUNCH(k_pw_shade, dim3((np + 1023) / 1024), dim3(1024), 0, s, pb.f, pb.u, pb.cap, np, depth,
                               pc, tris, params, pb.rays, pb.keys[0], pb.vals[0], pb.qcount);
            if (depth == max_depth + 1) break;  // only the last shadow results were left to apply
            uint32_t count = 0, grid = 0;
            const uint32_t* order = nullptr;
            const uint32_t* count_dev = nullptr;
            if (sort_digits) {  // the sort needs the queue length on the host
                if ((e = hipMemcpyAsync(pb.hq, pb.qcount, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
                if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
                count = *pb.hq;
                if (!count) break;  // every path has ended
                grid = (count + 255) / 256;
                if (count > 1) {
                    if ((e = hipMemsetAsync(pb.ghist, 0, 4096, s)) != hipSuccess) return e;
                    if ((e = launch_digit_hist(pb.keys[0], count, pb.ghist, s)) != hipSuccess) return e;
                    uint32_t ob = 0;
                    if ((e = launch_sort_top(pb.keys, pb.vals, count, pb.ghist, pb.counts, sort_digits, &ob, s)) !=
                        hipSuccess)
                        return e;
                    order = pb.vals[ob];
                }
            } else {  // no host round trip: blocks past the queue length exit at once
                count_dev = pb.qcount;
                grid = (2 * np + 255) / 256;
            }
#define RT_PW_TRACE(C, WW)                                                                                     \
    RT_KLAUNCH((k_pw_trace<C, WW>), dim3(grid), dim3(256), 0, s, nodes, wn, wcap, tri_s, n, pb.rays, order, \
                       count, count_dev, pb.f, pb.u, pb.cap, counters)
            if (counters) {
                if (w8) RT_PW_TRACE(true, 8); else RT_PW_TRACE(true, 4);
            } else {
                if (w8) RT_PW_TRACE(false, 8); else RT_PW_TRACE(false, 4);
            }
#undef RT_PW_TRACE
        }
        if (rgba)
            RT_KLAUNCH(k_pw_finish, dim3(nb), dim3(256), 0, s, pb.f, pb.cap, w, h, spp, tilesX, t0,
                               reinterpret_cast<uint32_t*>(rgba));
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipGetLastError();
}

hipError_t launch_unpack(const void* slabs, uint32_t tiles_per_slab, uint32_t w, uint32_t h, uint32_t nranks,
                         void* img, hipStream_t s) {
    if (!tiles_per_slab || !nranks) return hipSuccess;
    const uint32_t tilesX = (w + 15) / 16, nt = tilesX * ((h + 15) / 16);
    RT_KLAUNCH(k_unpack, dim3(tiles_per_slab * nranks), dim3(256), 0, s, (const uint32_t*)slabs, tiles_per_slab,
                       w, h, nranks, tilesX, nt, (uint32_t*)img);
    return hipGetLastError();
}

hipError_t launch_unpack_hits(const void* slabs, uint32_t tiles_per_slab, uint32_t w, uint32_t h, uint32_t spp,
                              uint32_t nranks, void* hits, hipStream_t s) {
    if (!tiles_per_slab || !nranks) return hipSuccess;
    const uint32_t tilesX = (w + 15) / 16, nt = tilesX * ((h + 15) / 16);
    RT_KLAUNCH(k_unpack_hits, dim3(tiles_per_slab * nranks), dim3(256), 0, s, (const float4*)slabs,
                       tiles_per_slab, w, h, spp, nranks, tilesX, nt, (float4*)hits);
    return hipGetLastError();
}

hipError_t launch_intersect(uint32_t count, const float* o, const float* d, const float* tri, const float* tb,
                            uint32_t* hit, float* tuv, hipStream_t s) {
    if (!count) return hipSuccess;
    RT_KLAUNCH(k_intersect, dim3((count + 255) / 256), dim3(256), 0, s, count, o, d, tri, tb, hit, tuv);
    return hipGetLastError();
}

hipError_t launch_minmax(uint32_t count, const float* a, const float* b, float* out, hipStream_t s) {
    if (!count) return hipSuccess;
    RT_KLAUNCH(k_minmax, dim3((count + 255) / 256), dim3(256), 0, s, count, a, b, out);
    return hipGetLastError();
}

}  // namespace rt

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

namespace rt {

#ifdef RT_STAMPS
hipError_t read_stamps_trace(void* out, size_t bytes) { return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rt_stamps), bytes); }
#endif

struct Cam { float eye[3], w00[3], du[3], dv[3]; };

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

// §9.7 stackless escape-link traversal of one ray over the 32-B nodes (two
// 16-B loads per node), with the leaf's triangle test deferred by one step:
// after a leaf's box hits, the next node is always its escape, which the
// leaf record already names, so the next step issues the escape node's
// loads AND the leaf's triangle loads together, tests the triangle first (it
// may shrink tb) and the node box second -- the §9.7 order, hence the same
// tests with the same operands.  A wave step then costs one memory round
// trip instead of two whenever some lane is at a leaf (+2-4 %,
// profiles/ab_trace_r01_variants.log).  A well-formed tree visits each node
// once; the guard and index checks only keep a malformed one from faulting.
template <bool COUNT>
__device__ __forceinline__ void trace_ray(const char* __restrict__ nodes, const float4* __restrict__ tri_s,
                                                uint32_t n, const float* o, const float* d, float& tb, float& hu,
                                                float& hv, uint32_t& hp, uint32_t& cn, uint32_t& ct) {
    float invd[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) invd[c] = 1.0f / d[c];
    tb = __builtin_inff(); hu = 0.0f; hv = 0.0f; hp = RT_SENT;
    const uint32_t L0 = n ? n - 1 : 0;
    const uint32_t total = n ? 2 * n - 1 : 0;
    uint32_t idx = n ? 0u : RT_SENT;
    uint32_t pend = RT_SENT, pprim = 0;  // leaf whose triangle test is due
    for (uint32_t guard = 0; (idx < total || pend != RT_SENT) && guard <= total; ++guard) {
        float4 A, B;
        const bool node = idx < total;
        if (node) {
            const float4* np = reinterpret_cast<const float4*>(nodes + (uint64_t)idx * 32);
            A = np[0]; B = np[1];
        }
        if (pend != RT_SENT) {
            if (COUNT) ++ct;
            const float4* tp = tri_s + (uint64_t)pend * 3;
            const float4 T0 = tp[0], T1 = tp[1], T2 = tp[2];
            const float v0[3] = {T0.x, T0.y, T0.z};
            const float e1[3] = {T0.w, T1.x, T1.y};
            const float e2[3] = {T1.z, T1.w, T2.x};
            float t, u, v;
            if (intersect_e(o, d, v0, e1, e2, tb, t, u, v)) { tb = t; hu = u; hv = v; hp = pprim; }
            pend = RT_SENT;
        }
        if (!node) break;
        if (COUNT) ++cn;
        const float t0x = (A.x - o[0]) * invd[0], t1x = (A.w - o[0]) * invd[0];
        const float t0y = (A.y - o[1]) * invd[1], t1y = (B.x - o[1]) * invd[1];
        const float t0z = (A.z - o[2]) * invd[2], t1z = (B.y - o[2]) * invd[2];
        const float tn = fmaxf(fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z)), 0.0f);
        const float tf = fminf(fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z)), tb);
        const uint32_t na = __float_as_uint(B.z), esc = __float_as_uint(B.w);
        const bool hit = tn <= tf;
        if (hit && idx >= L0) { pend = idx - L0; pprim = na; }
        idx = (hit && idx < L0) ? na : esc;
    }
}

__device__ __forceinline__ uint32_t q8(float x) { return (uint32_t)fminf(fmaxf(x * 255.0f + 0.5f, 0.0f), 255.0f); }

template <bool COUNT, bool PACKED>
__global__ __launch_bounds__(256) void k_trace(const void* __restrict__ nodes, const float4* __restrict__ tri_s, uint32_t n,
                                               Cam cam, uint32_t W, uint32_t H, uint32_t spp,
                                               uint32_t rank, uint32_t nranks, uint32_t tilesX,
                                               float4* __restrict__ hits, uint32_t* __restrict__ rgba,
                                               unsigned long long* __restrict__ counters) {
    // tile slot = block id: consecutive tiles go to different XCDs under the
    // round-robin dispatch, which balances the image's cheap and costly
    // bands over the 8 XCDs (an XCD-banded remap measured 1.2x slower)
    const uint32_t slot = blockIdx.x;
    const uint32_t t = rank + slot * nranks;
    const uint32_t tx = t % tilesX, ty = t / tilesX;
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t lx = (w & 1) * 8 + (l & 7), ly = (w >> 1) * 8 + (l >> 3);
    const uint32_t x = tx * 16 + lx, y = ty * 16 + ly;
    const bool valid = x < W && y < H;
    uint32_t cn = 0, ct = 0;
#ifdef RT_STAMPS
    const unsigned long long st0 = __builtin_amdgcn_s_memrealtime();
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
            float tb, hu, hv;
            uint32_t hp;
            trace_ray<COUNT>(reinterpret_cast<const char*>(nodes), tri_s, n, cam.eye, d, tb, hu, hv, hp, cn, ct);
            if (hits) {
                const uint64_t hi = PACKED ? ((uint64_t)slot * 256 + ly * 16 + lx) * spp + s : (uint64_t)sidx;
                hits[hi] = make_float4(tb, hu, hv, __uint_as_float(hp));
            }
            if (hp != RT_SENT) {
                r = r + hu;
                g = g + hv;
                b = b + ((1.0f - hu) - hv);
            } else {
                r = r + 0.0f; g = g + 0.0f; b = b + 0.0f;
            }
        }
        if (rgba) {
            const float sc = 1.0f / (float)spp;
            const uint32_t px = q8(r * sc) | (q8(g * sc) << 8) | (q8(b * sc) << 16) | (255u << 24);
            const uint64_t pi = PACKED ? (uint64_t)slot * 256 + ly * 16 + lx : (uint64_t)y * W + x;
            rgba[pi] = px;
        }
    }
#ifdef RT_STAMPS
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
            const uint64_t wslot = ((uint64_t)blockIdx.x * 4 + w) * 4;
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
}

// ---------------------------------------------------------------- persistent
// Persistent wave-level work distribution with per-lane refill.  Each wave
// pulls units -- 8x8 quarters of this rank's 16x16 tiles (t = rank +
// b*nranks) -- from a work counter; lanes whose pixel is finished take the
// next pixel of the current unit (in lane order), so a wave no longer idles
// behind its slowest ray.  A lane owns a whole pixel (its spp samples in order), which
// keeps the per-pixel sample average of §9.7 sequential.  The traversal step
// is the exact §9.7 escape-link loop body: results are bit-identical.
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

struct RayState {
    float d[3], invd[3];
    float tb, hu, hv;
    uint32_t hp, idx, guard;
};

__device__ __forceinline__ void ray_setup(const Cam& cam, uint32_t x, uint32_t y, uint32_t W, uint32_t spp, uint32_t s,
                                          uint32_t n, RayState& R) {
    const uint32_t sidx = (y * W + x) * spp + s;
    float jx = 0.5f, jy = 0.5f;
    if (s > 0) {
        const uint32_t h = pcg_hash(sidx);
        jx = (float)(h >> 8) * 0x1p-24f;
        jy = (float)(pcg_hash(h) >> 8) * 0x1p-24f;
    }
    const float px = (float)x + jx, py = (float)y + jy;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        R.d[c] = (cam.w00[c] + px * cam.du[c]) + py * cam.dv[c];
        R.invd[c] = 1.0f / R.d[c];
    }
    R.tb = __builtin_inff(); R.hu = 0.0f; R.hv = 0.0f; R.hp = RT_SENT;
    R.idx = n ? 0u : RT_SENT;
    R.guard = 0;
}

template <bool COUNT, bool PACKED>
__global__ __launch_bounds__(256) void k_trace_persist(const void* __restrict__ nodes_, const float4* __restrict__ tri_s,
                                                       uint32_t n, Cam cam, uint32_t W, uint32_t H, uint32_t spp,
                                                       uint32_t rank, uint32_t nranks, uint32_t tilesX,
                                                       uint32_t ntiles_rank, uint32_t refill_min,
                                                       float4* __restrict__ hits, uint32_t* __restrict__ rgba,
                                                       unsigned long long* __restrict__ counters,
                                                       uint32_t* __restrict__ work) {
    const char* __restrict__ nodes = reinterpret_cast<const char*>(nodes_);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t L0 = n ? n - 1 : 0;
    const uint32_t total = n ? 2 * n - 1 : 0;
    // lane state
    bool active = false;
    uint32_t x = 0, y = 0, lp = 0, tb_idx = 0, s = 0;
    float cr = 0.0f, cg = 0.0f, cb = 0.0f;
    RayState R;
    R.idx = RT_SENT;
    // wave-uniform tile cursor
    uint32_t cur_unit = 0, next = 64;
    bool more = true;
    uint32_t cn = 0, ct = 0;
    const float o[3] = {cam.eye[0], cam.eye[1], cam.eye[2]};

    for (;;) {
        // ---- refill idle lanes (wave-uniform control flow)
        uint64_t idle = __ballot(!active);
        if (more && (uint32_t)__popcll(idle) >= refill_min) {
            while (idle && more) {
                if (next >= 64) {
                    uint32_t u = 0;
                    if (lane == 0) u = atomicAdd(work, 1u);
                    u = __shfl(u, 0, 64);
                    if (u >= ntiles_rank * 4) { more = false; break; }
                    cur_unit = u;
                    next = 0;
                }
                const uint32_t pos = lanes_below(idle);
                const uint32_t nidle = (uint32_t)__popcll(idle);
                const uint32_t take = nidle < 64 - next ? nidle : 64 - next;
                if (!active && pos < take) {
                    // unit = one 8x8 quarter of a 16x16 tile
                    const uint32_t p = next + pos, sub = cur_unit & 3;
                    lp = ((sub >> 1) * 8 + (p >> 3)) * 16 + (sub & 1) * 8 + (p & 7);
                    tb_idx = cur_unit >> 2;
                    const uint32_t t = rank + tb_idx * nranks;
                    x = (t % tilesX) * 16 + (lp & 15);
                    y = (t / tilesX) * 16 + (lp >> 4);
                    if (x < W && y < H) {
                        active = true;
                        s = 0;
                        cr = cg = cb = 0.0f;
                        ray_setup(cam, x, y, W, spp, 0, n, R);
                    }
                }
                next += take;
                idle = __ballot(!active);
            }
        }
        if (__ballot(active) == 0) break;  // every lane idle and no work left
        // ---- one escape-link traversal step (§9.7)
        if (active) {
            if (R.idx < total && R.guard < total) {
                ++R.guard;
                const float4* np = reinterpret_cast<const float4*>(nodes + (uint64_t)R.idx * 32);
                const float4 A = np[0], B = np[1];
                if (COUNT) ++cn;
                const float t0x = (A.x - o[0]) * R.invd[0], t1x = (A.w - o[0]) * R.invd[0];
                const float t0y = (A.y - o[1]) * R.invd[1], t1y = (B.x - o[1]) * R.invd[1];
                const float t0z = (A.z - o[2]) * R.invd[2], t1z = (B.y - o[2]) * R.invd[2];
                const float tn = fmaxf(fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z)), 0.0f);
                const float tf = fminf(fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z)), R.tb);
                const uint32_t na = __float_as_uint(B.z), esc = __float_as_uint(B.w);
                if (!(tn <= tf)) {
                    R.idx = esc;
                } else if (R.idx >= L0) {
                    if (COUNT) ++ct;
                    const float4* tp = tri_s + (uint64_t)(R.idx - L0) * 3;
                    const float4 T0 = tp[0], T1 = tp[1], T2 = tp[2];
                    const float v0[3] = {T0.x, T0.y, T0.z};
                    const float e1[3] = {T0.w, T1.x, T1.y};
                    const float e2[3] = {T1.z, T1.w, T2.x};
                    float t, u, v;
                    if (intersect_e(o, R.d, v0, e1, e2, R.tb, t, u, v)) { R.tb = t; R.hu = u; R.hv = v; R.hp = na; }
                    R.idx = esc;
                } else {
                    R.idx = na;
                }
            } else {
                // sample finished
                if (hits) {
                    const uint64_t hi = PACKED ? ((uint64_t)tb_idx * 256 + lp) * spp + s
                                               : (uint64_t)((y * W + x) * spp + s);
                    hits[hi] = make_float4(R.tb, R.hu, R.hv, __uint_as_float(R.hp));
                }
                if (R.hp != RT_SENT) {
                    cr = cr + R.hu;
                    cg = cg + R.hv;
                    cb = cb + ((1.0f - R.hu) - R.hv);
                } else {
                    cr = cr + 0.0f; cg = cg + 0.0f; cb = cb + 0.0f;
                }
                if (++s < spp) {
                    ray_setup(cam, x, y, W, spp, s, n, R);
                } else {
                    if (rgba) {
                        const float sc = 1.0f / (float)spp;
                        const uint32_t px = q8(cr * sc) | (q8(cg * sc) << 8) | (q8(cb * sc) << 16) | (255u << 24);
                        const uint64_t pi = PACKED ? (uint64_t)tb_idx * 256 + lp : (uint64_t)y * W + x;
                        rgba[pi] = px;
                    }
                    active = false;
                }
            }
        }
    }
    if (COUNT) {
        unsigned long long a = cn, bsum = ct;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            a += __shfl_xor(a, off, 64);
            bsum += __shfl_xor(bsum, off, 64);
        }
        if (lane == 0) {
            atomicAdd(&counters[0], a);
            atomicAdd(&counters[1], bsum);
        }
    }
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

TraceConfig g_trace_config;

hipError_t launch_trace(const void* nodes, const float4* tris, uint32_t n, const CamF& c, uint32_t w, uint32_t h,
                        uint32_t spp, uint32_t rank, uint32_t nranks, bool packed, void* hits, void* rgba,
                        unsigned long long* counters, uint32_t* work, hipStream_t s) {
    const uint32_t nb = tiles_for_rank(w, h, rank, nranks);
    if (!nb) return hipSuccess;
    Cam cam;
    for (int i = 0; i < 3; ++i) {
        cam.eye[i] = c.eye[i]; cam.w00[i] = c.w00[i]; cam.du[i] = c.du[i]; cam.dv[i] = c.dv[i];
    }
    const uint32_t tilesX = (w + 15) / 16;
    float4* H = reinterpret_cast<float4*>(hits);
    uint32_t* R = reinterpret_cast<uint32_t*>(rgba);
    if (g_trace_config.variant == 1 && work) {
        hipError_t e = hipMemsetAsync(work, 0, 4, s);
        if (e != hipSuccess) return e;
        const uint32_t waves = g_trace_config.blocks * 4;
        const uint32_t grid = nb * 4 < waves ? nb : g_trace_config.blocks;  // 4 units (8x8) per tile
        const uint32_t rmin = g_trace_config.refill_min;
#define RT_PERSIST(C, P)                                                                                          \
    hipLaunchKernelGGL((k_trace_persist<C, P>), dim3(grid), dim3(256), 0, s, nodes, tris, n, cam, w, h, spp, rank, \
                       nranks, tilesX, nb, rmin, H, R, counters, work)
        if (counters) {
            if (packed) RT_PERSIST(true, true); else RT_PERSIST(true, false);
        } else {
            if (packed) RT_PERSIST(false, true); else RT_PERSIST(false, false);
        }
#undef RT_PERSIST
        return hipGetLastError();
    }
    if (counters) {
        if (packed) hipLaunchKernelGGL((k_trace<true, true>), dim3(nb), dim3(256), 0, s, nodes, tris, n, cam, w, h, spp, rank, nranks, tilesX, H, R, counters);
        else hipLaunchKernelGGL((k_trace<true, false>), dim3(nb), dim3(256), 0, s, nodes, tris, n, cam, w, h, spp, rank, nranks, tilesX, H, R, counters);
    } else {
        if (packed) hipLaunchKernelGGL((k_trace<false, true>), dim3(nb), dim3(256), 0, s, nodes, tris, n, cam, w, h, spp, rank, nranks, tilesX, H, R, counters);
        else hipLaunchKernelGGL((k_trace<false, false>), dim3(nb), dim3(256), 0, s, nodes, tris, n, cam, w, h, spp, rank, nranks, tilesX, H, R, counters);
    }
    return hipGetLastError();
}

hipError_t launch_unpack(const void* slabs, uint32_t tiles_per_slab, uint32_t w, uint32_t h, uint32_t nranks,
                         void* img, hipStream_t s) {
    if (!tiles_per_slab || !nranks) return hipSuccess;
    const uint32_t tilesX = (w + 15) / 16, nt = tilesX * ((h + 15) / 16);
    hipLaunchKernelGGL(k_unpack, dim3(tiles_per_slab * nranks), dim3(256), 0, s, (const uint32_t*)slabs, tiles_per_slab,
                       w, h, nranks, tilesX, nt, (uint32_t*)img);
    return hipGetLastError();
}

hipError_t launch_intersect(uint32_t count, const float* o, const float* d, const float* tri, const float* tb,
                            uint32_t* hit, float* tuv, hipStream_t s) {
    if (!count) return hipSuccess;
    hipLaunchKernelGGL(k_intersect, dim3((count + 255) / 256), dim3(256), 0, s, count, o, d, tri, tb, hit, tuv);
    return hipGetLastError();
}

hipError_t launch_minmax(uint32_t count, const float* a, const float* b, float* out, hipStream_t s) {
    if (!count) return hipSuccess;
    hipLaunchKernelGGL(k_minmax, dim3((count + 255) / 256), dim3(256), 0, s, count, a, b, out);
    return hipGetLastError();
}

}  // namespace rt

/*
 * rt_oracle.c -- scalar CPU restatement of the hot-path contract
 * (SURVEY.md §9).  TEST INFRASTRUCTURE ONLY -- see rt_oracle.h for who may
 * use it and for the parity-pinning status ("parity unpinned" vs upstream).
 *
 * Build: oracle/Makefile (gcc -O3 -ffp-contract=off, never -ffast-math, no
 * FTZ/DAZ) -> oracle/build/liboracle.so.  The flags matter: §9.1 fixes the
 * rounding of every fp32 operation (no contraction to FMA).
 */
#include "rt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- §9.1 ---
 * Min/max with the semantics the device's v_min_f32/v_max_f32 implement
 * (IEEE-754 minimumNumber/maximumNumber): a NaN operand yields the other
 * operand, and -0 orders below +0.  glibc's fminf() returns an
 * operand-order-dependent zero for (+0,-0), so it is not used. */
float orc_fmin(float a, float b) {
    if (a != a) return b;
    if (b != b) return a;
    if (a < b) return a;
    if (b < a) return b;
    return signbit(a) ? a : b; /* equal: prefer -0 */
}
float orc_fmax(float a, float b) {
    if (a != a) return b;
    if (b != b) return a;
    if (a > b) return a;
    if (b > a) return b;
    return signbit(a) ? b : a; /* equal: prefer +0 */
}
#define FMIN orc_fmin
#define FMAX orc_fmax

/* §9.1 operation order */
static inline float dot3(const float a[3], const float b[3]) {
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}
static inline void cross3(const float a[3], const float b[3], float o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

/* ---------------------------------------------------------------- §9.9 --- */
uint64_t orc_splitmix64(uint64_t* s) {
    *s += 0x9E3779B97F4A7C15ull;
    uint64_t z = *s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline float u01(uint64_t* s) { return (float)(orc_splitmix64(s) >> 40) * 0x1p-24f; }

void orc_soup_generate(uint32_t n, uint64_t seed, float* tris) {
    uint64_t s = seed;
    /* r = (float)(1/cbrt(N)), SURVEY.md §8(d) */
    const float r = n ? (float)(1.0 / cbrt((double)n)) : 0.0f;
    for (uint32_t i = 0; i < n; ++i) {
        float c[3];
        c[0] = u01(&s);
        c[1] = u01(&s);
        c[2] = u01(&s);
        for (int v = 0; v < 3; ++v)
            for (int a = 0; a < 3; ++a) tris[(size_t)i * 9 + v * 3 + a] = c[a] + (2.0f * u01(&s) - 1.0f) * r;
    }
}

/* ---------------------------------------------------------------- §9.7 ---
 * forward f = normalize(at-eye); right r = normalize(f x up); true up
 * u = r x f (right-handed); w00 = f + u*tan(vfov/2) - r*tan(vfov/2)*aspect;
 * du = r*(2 tan aspect / W); dv = -u*(2 tan / H); aspect = W/H. */
static void dnorm(double v[3]) {
    double l = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    v[0] /= l; v[1] /= l; v[2] /= l;
}
static void dcross(const double a[3], const double b[3], double o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
void orc_camera_look_at(const double eye[3], const double at[3], const double up[3],
                        double vfov_deg, uint32_t w, uint32_t h, orc_camera* out) {
    double f[3] = {at[0] - eye[0], at[1] - eye[1], at[2] - eye[2]};
    dnorm(f);
    double r[3], u[3];
    dcross(f, up, r);
    dnorm(r);
    dcross(r, f, u);
    const double th = tan(vfov_deg * 3.14159265358979323846 / 360.0);
    const double aspect = (double)w / (double)h;
    for (int a = 0; a < 3; ++a) {
        out->eye[a] = (float)eye[a];
        out->w00[a] = (float)(f[a] + u[a] * th - r[a] * th * aspect);
        out->du[a] = (float)(r[a] * (2.0 * th * aspect / (double)w));
        out->dv[a] = (float)(-u[a] * (2.0 * th / (double)h));
    }
}

/* ---------------------------------------------------------------- §9.2 --- */
static inline void tri_bounds(const float* t, float bmin[3], float bmax[3]) {
    for (int a = 0; a < 3; ++a) {
        bmin[a] = FMIN(FMIN(t[a], t[3 + a]), t[6 + a]);
        bmax[a] = FMAX(FMAX(t[a], t[3 + a]), t[6 + a]);
    }
}
void orc_centroid_bounds(const float* tris, uint32_t n, float lo[3], float hi[3], float inv[3]) {
    for (int a = 0; a < 3; ++a) { lo[a] = INFINITY; hi[a] = -INFINITY; }
    for (uint32_t i = 0; i < n; ++i) {
        float bmin[3], bmax[3];
        tri_bounds(tris + (size_t)i * 9, bmin, bmax);
        for (int a = 0; a < 3; ++a) {
            float c = (bmin[a] + bmax[a]) * 0.5f;
            lo[a] = FMIN(lo[a], c);
            hi[a] = FMAX(hi[a], c);
        }
    }
    for (int a = 0; a < 3; ++a) inv[a] = (hi[a] > lo[a]) ? 1.0f / (hi[a] - lo[a]) : 0.0f;
}

/* ---------------------------------------------------------------- §9.3 --- */
uint32_t orc_expand10(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
uint32_t orc_morton3(uint32_t qx, uint32_t qy, uint32_t qz) {
    return orc_expand10(qx) * 4u + orc_expand10(qy) * 2u + orc_expand10(qz);
}
static inline uint32_t quant(float c, float lo, float inv) {
    float x = (c - lo) * inv * 1024.0f;
    return (uint32_t)FMIN(FMAX(x, 0.0f), 1023.0f);
}
void orc_morton(const float* tris, uint32_t n, const float lo[3], const float inv[3],
                uint32_t* keys, uint32_t* vals) {
    for (uint32_t i = 0; i < n; ++i) {
        float bmin[3], bmax[3];
        tri_bounds(tris + (size_t)i * 9, bmin, bmax);
        uint32_t q[3];
        for (int a = 0; a < 3; ++a) q[a] = quant((bmin[a] + bmax[a]) * 0.5f, lo[a], inv[a]);
        keys[i] = orc_morton3(q[0], q[1], q[2]);
        vals[i] = i;
    }
}

/* ---------------------------------------------------------------- §9.4 --- */
void orc_radix_sort(uint32_t* keys, uint32_t* vals, uint32_t n, uint32_t* tk, uint32_t* tv) {
    uint32_t *sk = keys, *sv = vals, *dk = tk, *dv = tv;
    for (int p = 0; p < 4; ++p) {
        uint32_t cnt[257];
        memset(cnt, 0, sizeof cnt);
        const int sh = 8 * p;
        for (uint32_t i = 0; i < n; ++i) cnt[((sk[i] >> sh) & 0xFFu) + 1]++;
        for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
        for (uint32_t i = 0; i < n; ++i) {
            uint32_t pos = cnt[(sk[i] >> sh) & 0xFFu]++;
            dk[pos] = sk[i];
            dv[pos] = sv[i];
        }
        uint32_t* t;
        t = sk; sk = dk; dk = t;
        t = sv; sv = dv; dv = t;
    }
    /* 4 passes: result is back in keys/vals */
}

/* ---------------------------------------------------------------- §9.5 --- */
static inline int clz32(uint32_t x) { return x ? __builtin_clz(x) : 32; }
int orc_delta(const uint32_t* keys, uint32_t n, int64_t i, int64_t j) {
    if (j < 0 || j > (int64_t)n - 1) return -1;
    uint32_t ki = keys[i], kj = keys[j];
    if (ki == kj) return 32 + clz32((uint32_t)i ^ (uint32_t)j);
    return clz32(ki ^ kj);
}
void orc_karras(const uint32_t* keys, uint32_t n, uint32_t* left, uint32_t* right,
                uint32_t* range_lo, uint32_t* range_hi, uint32_t* parent) {
    if (n == 0) return;
    const uint32_t L0 = n - 1; /* leaf k -> unified n-1+k */
    parent[0] = ORC_SENTINEL;  /* root: internal 0, or leaf 0 when n == 1 */
    for (int64_t i = 0; i < (int64_t)n - 1; ++i) {
        const int d = (orc_delta(keys, n, i, i + 1) - orc_delta(keys, n, i, i - 1)) > 0 ? 1 : -1;
        const int dmin = orc_delta(keys, n, i, i - d);
        int64_t lmax = 2;
        while (orc_delta(keys, n, i, i + lmax * d) > dmin) lmax *= 2;
        int64_t l = 0;
        for (int64_t t = lmax / 2; t >= 1; t /= 2)
            if (orc_delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
        const int64_t j = i + l * d;
        const int dnode = orc_delta(keys, n, i, j);
        int64_t s = 0, t = l;
        do {
            t = (t + 1) >> 1;
            if (orc_delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
        } while (t > 1);
        const int64_t g = i + s * d + (d < 0 ? d : 0);
        const int64_t mn = i < j ? i : j, mx = i < j ? j : i;
        left[i] = (mn == g) ? (uint32_t)(L0 + g) : (uint32_t)g;
        right[i] = (mx == g + 1) ? (uint32_t)(L0 + g + 1) : (uint32_t)(g + 1);
        range_lo[i] = (uint32_t)mn;
        range_hi[i] = (uint32_t)mx;
        parent[left[i]] = (uint32_t)i;
        parent[right[i]] = (uint32_t)i;
    }
}

/* ---------------------------------------------------------------- §9.6 --- */
void orc_escape(uint32_t n, const uint32_t* left, const uint32_t* right,
                const uint32_t* parent, uint32_t* esc) {
    if (n == 0) return;
    const uint32_t total = 2 * n - 1;
    for (uint32_t m0 = 0; m0 < total; ++m0) {
        uint32_t m = m0, e = ORC_SENTINEL;
        while (parent[m] != ORC_SENTINEL) {
            const uint32_t p = parent[m];
            if (left[p] == m) { e = right[p]; break; }
            m = p;
        }
        esc[m0] = e;
    }
}

void orc_refit_pack(const float* tris, uint32_t n, const uint32_t* sorted_vals,
                    const uint32_t* left, const uint32_t* right, const uint32_t* esc,
                    orc_node* nodes) {
    if (n == 0) return;
    const uint32_t L0 = n - 1;
    for (uint32_t k = 0; k < n; ++k) {
        orc_node* nd = &nodes[L0 + k];
        tri_bounds(tris + (size_t)sorted_vals[k] * 9, nd->lo, nd->hi);
        nd->a = sorted_vals[k];
        nd->esc = esc[L0 + k];
    }
    if (n == 1) return;
    /* iterative post-order from the root (internal 0) */
    uint32_t* stack = (uint32_t*)malloc(sizeof(uint32_t) * 2 * (size_t)n);
    uint8_t* seen = (uint8_t*)calloc(n, 1);
    size_t sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const uint32_t i = stack[sp - 1];
        if (!seen[i]) {
            seen[i] = 1;
            if (right[i] < L0) stack[sp++] = right[i];
            if (left[i] < L0) stack[sp++] = left[i];
            continue;
        }
        --sp;
        const orc_node *A = &nodes[left[i]], *B = &nodes[right[i]];
        orc_node* nd = &nodes[i];
        for (int a = 0; a < 3; ++a) {
            nd->lo[a] = FMIN(A->lo[a], B->lo[a]);
            nd->hi[a] = FMAX(A->hi[a], B->hi[a]);
        }
        nd->a = left[i];
        nd->esc = esc[i];
    }
    free(stack);
    free(seen);
}

int orc_build(const float* tris, uint32_t n, orc_node* nodes, uint32_t* sorted_keys,
              uint32_t* sorted_vals, uint32_t* parent_out, orc_bounds* bounds_out) {
    orc_bounds b;
    orc_centroid_bounds(tris, n, b.lo, b.hi, b.inv);
    if (bounds_out) *bounds_out = b;
    if (n == 0) return 0;
    const size_t N = n, T = 2 * N - 1;
    uint32_t* keys = (uint32_t*)malloc(4 * N);
    uint32_t* vals = (uint32_t*)malloc(4 * N);
    uint32_t* tk = (uint32_t*)malloc(4 * N);
    uint32_t* tv = (uint32_t*)malloc(4 * N);
    uint32_t* left = (uint32_t*)malloc(4 * N);
    uint32_t* right = (uint32_t*)malloc(4 * N);
    uint32_t* rlo = (uint32_t*)malloc(4 * N);
    uint32_t* rhi = (uint32_t*)malloc(4 * N);
    uint32_t* parent = (uint32_t*)malloc(4 * T);
    uint32_t* esc = (uint32_t*)malloc(4 * T);
    int rc = 0;
    if (!keys || !vals || !tk || !tv || !left || !right || !rlo || !rhi || !parent || !esc) {
        rc = -2;
        goto out;
    }
    orc_morton(tris, n, b.lo, b.inv, keys, vals);
    orc_radix_sort(keys, vals, n, tk, tv);
    orc_karras(keys, n, left, right, rlo, rhi, parent);
    orc_escape(n, left, right, parent, esc);
    orc_refit_pack(tris, n, vals, left, right, esc, nodes);
    if (sorted_keys) memcpy(sorted_keys, keys, 4 * N);
    if (sorted_vals) memcpy(sorted_vals, vals, 4 * N);
    if (parent_out) memcpy(parent_out, parent, 4 * T);
out:
    free(keys); free(vals); free(tk); free(tv); free(left); free(right);
    free(rlo); free(rhi); free(parent); free(esc);
    return rc;
}

/* ---------------------------------------------------------------- §9.7 --- */
uint32_t orc_pcg_hash(uint32_t x) {
    uint32_t st = x * 747796405u + 2891336453u;
    uint32_t w = ((st >> ((st >> 28u) + 4u)) ^ st) * 277803737u;
    return (w >> 22u) ^ w;
}

/* Moller-Trumbore, two-sided, no epsilon.  Returns 1 and writes t/u/v when
 * the triangle is hit with t < t_best. */
int orc_intersect_tri(const float o[3], const float d[3], const float* tri, float t_best,
                      float* tout, float* uout, float* vout) {
    const float* v0 = tri;
    float e1[3], e2[3], p[3], s[3], q[3];
    for (int a = 0; a < 3; ++a) { e1[a] = tri[3 + a] - v0[a]; e2[a] = tri[6 + a] - v0[a]; }
    cross3(d, e2, p);
    const float det = dot3(e1, p);
    if (det == 0.0f) return 0;
    const float inv = 1.0f / det;
    for (int a = 0; a < 3; ++a) s[a] = o[a] - v0[a];
    const float u = dot3(s, p) * inv;
    if (u < 0.0f || u > 1.0f) return 0;
    cross3(s, e1, q);
    const float v = dot3(d, q) * inv;
    if (v < 0.0f || u + v > 1.0f) return 0;
    const float t = dot3(e2, q) * inv;
    if (t <= 0.0f) return 0;
    if (!(t < t_best)) return 0;
    *tout = t; *uout = u; *vout = v;
    return 1;
}

/* tmax: INFINITY for the §9.7 closest hit; 1.0f with any_hit for the
 * shadow ray of the shadow mode (the first hit with 0 < t < 1 ends it). */
static void trace_ray_t(const orc_node* nodes, uint32_t n, const float* tris, const float o[3],
                        const float d[3], float tmax, int any_hit, orc_hit* hit, uint64_t* cn, uint64_t* ct) {
    float invd[3];
    for (int a = 0; a < 3; ++a) invd[a] = 1.0f / d[a];
    float tb = tmax, hu = 0.0f, hv = 0.0f;
    uint32_t hp = ORC_SENTINEL;
    uint32_t idx = n ? 0u : ORC_SENTINEL;
    const uint32_t L0 = n ? n - 1 : 0;
    uint64_t nn = 0, nt = 0;
    while (idx != ORC_SENTINEL) {
        const orc_node* nd = &nodes[idx];
        ++nn;
        float t0[3], t1[3];
        for (int a = 0; a < 3; ++a) {
            t0[a] = (nd->lo[a] - o[a]) * invd[a];
            t1[a] = (nd->hi[a] - o[a]) * invd[a];
        }
        const float tn = FMAX(FMAX(FMAX(FMIN(t0[0], t1[0]), FMIN(t0[1], t1[1])), FMIN(t0[2], t1[2])), 0.0f);
        const float tf = FMIN(FMIN(FMIN(FMAX(t0[0], t1[0]), FMAX(t0[1], t1[1])), FMAX(t0[2], t1[2])), tb);
        if (!(tn <= tf)) { idx = nd->esc; continue; }
        if (idx >= L0) {
            ++nt;
            float t, u, v;
            if (orc_intersect_tri(o, d, tris + (size_t)nd->a * 9, tb, &t, &u, &v)) {
                tb = t; hu = u; hv = v; hp = nd->a;
                if (any_hit) break;
            }
            idx = nd->esc;
        } else {
            idx = nd->a;
        }
    }
    hit->t = tb; hit->u = hu; hit->v = hv; hit->prim = hp;
    *cn += nn;
    *ct += nt;
}

static void trace_ray(const orc_node* nodes, uint32_t n, const float* tris, const float o[3],
                      const float d[3], orc_hit* hit, uint64_t* cn, uint64_t* ct) {
    trace_ray_t(nodes, n, tris, o, d, INFINITY, 0, hit, cn, ct);
}

/* Worker threads.  A thread that cannot be created (EAGAIN under a task
 * limit: the GPU box caps a job's processes and threads) must not lose its
 * share: the trace's shared cursor is drained by the calling thread, and a
 * path job whose thread did not start runs on the caller.  (Until r03 the
 * return value was ignored and glibc's pthread_join of the never-set id
 * returns ESRCH without waiting: had every creation failed, the expected
 * hits would have stayed at their "miss" initial values -- a wrong oracle,
 * not a wrong GPU result.)  orc_debug_fail_spawn(1) makes every creation
 * fail, for the CPU test of that path. */
static atomic_int g_fail_spawn;
void orc_debug_fail_spawn(int on) { atomic_store(&g_fail_spawn, on); }
static unsigned char spawn(pthread_t* t, void* (*fn)(void*), void* arg) {
    if (atomic_load(&g_fail_spawn)) return 0;
    return pthread_create(t, NULL, fn, arg) == 0;
}

typedef struct {
    const orc_node* nodes; uint32_t n; const float* tris; const orc_camera* cam;
    uint32_t w, h, spp, row0, row_step; orc_hit* hits;
    atomic_uint_fast64_t* next;  /* shared work cursor: 64-pixel row segments */
    uint64_t cn, ct;
} trace_job;

/* Work is dealt dynamically in 64-pixel row segments (the rows the camera
 * sees differ ~100x in cost), and each thread keeps its counters in locals:
 * per-ray updates of adjacent job structs would false-share a cache line.
 * Every ray's result lands at its own index, so the output and the counter
 * sums are the same for any thread count and schedule. */
static void* trace_worker(void* arg) {
    trace_job* j = (trace_job*)arg;
    const orc_camera* c = j->cam;
    const uint64_t rows = j->row0 < j->h ? (j->h - j->row0 + j->row_step - 1) / j->row_step : 0;
    const uint64_t segs_per_row = (j->w + 63) / 64, units = rows * segs_per_row;
    uint64_t cn = 0, ct = 0;
    for (;;) {
        const uint64_t u = atomic_fetch_add_explicit(j->next, 1, memory_order_relaxed);
        if (u >= units) break;
        const uint64_t y = j->row0 + (u / segs_per_row) * j->row_step;
        const uint32_t x0 = (uint32_t)(u % segs_per_row) * 64u, x1 = x0 + 64u < j->w ? x0 + 64u : j->w;
        for (uint32_t x = x0; x < x1; ++x) {
            for (uint32_t s = 0; s < j->spp; ++s) {
                const uint32_t sidx = (uint32_t)((y * j->w + x) * j->spp + s);
                float jx = 0.5f, jy = 0.5f;
                if (s > 0) {
                    const uint32_t hh = orc_pcg_hash(sidx);
                    jx = (float)(hh >> 8) * 0x1p-24f;
                    jy = (float)(orc_pcg_hash(hh) >> 8) * 0x1p-24f;
                }
                const float px = (float)x + jx, py = (float)y + jy;
                float d[3];
                for (int a = 0; a < 3; ++a) d[a] = (c->w00[a] + px * c->du[a]) + py * c->dv[a];
                trace_ray(j->nodes, j->n, j->tris, c->eye, d, &j->hits[sidx], &cn, &ct);
            }
        }
    }
    j->cn = cn;
    j->ct = ct;
    return NULL;
}

void orc_trace(const orc_node* nodes, uint32_t n, const float* tris, const orc_camera* cam,
               uint32_t w, uint32_t h, uint32_t spp, uint32_t row0, uint32_t row_step,
               orc_hit* hits, uint64_t counters[2], int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (row_step < 1) row_step = 1;
    trace_job* jobs = (trace_job*)calloc((size_t)nthreads, sizeof(trace_job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    unsigned char* live = (unsigned char*)calloc((size_t)nthreads, 1);
    atomic_uint_fast64_t next;
    atomic_init(&next, 0);
    for (int t = 0; t < nthreads; ++t) {
        trace_job jb = {nodes, n, tris, cam, w, h, spp, row0, row_step, hits, &next, 0, 0};
        jobs[t] = jb;
    }
    for (int t = 1; t < nthreads; ++t) live[t] = spawn(&th[t], trace_worker, &jobs[t]);
    trace_worker(&jobs[0]);  /* the caller is worker 0: the shared cursor is drained even if no thread starts */
    for (int t = 1; t < nthreads; ++t)
        if (live[t]) pthread_join(th[t], NULL);
    free(live);
    if (counters) {
        counters[0] = counters[1] = 0;
        for (int t = 0; t < nthreads; ++t) { counters[0] += jobs[t].cn; counters[1] += jobs[t].ct; }
    }
    free(jobs);
    free(th);
}

/* shading, §9.7: hit -> (u, v, 1-u-v), miss -> 0; sequential mean; u8 quantise */
static inline uint8_t q8(float x) { return (uint8_t)FMIN(FMAX(x * 255.0f + 0.5f, 0.0f), 255.0f); }
void orc_shade(const orc_hit* hits, uint32_t w, uint32_t h, uint32_t spp, uint8_t* rgba) {
    const float sc = 1.0f / (float)spp;
    for (uint64_t p = 0; p < (uint64_t)w * h; ++p) {
        float r = 0.0f, g = 0.0f, b = 0.0f;
        for (uint32_t s = 0; s < spp; ++s) {
            const orc_hit* ht = &hits[p * spp + s];
            if (ht->prim != ORC_SENTINEL) {
                r = r + ht->u;
                g = g + ht->v;
                b = b + ((1.0f - ht->u) - ht->v);
            } else {
                r = r + 0.0f; g = g + 0.0f; b = b + 0.0f;
            }
        }
        rgba[p * 4 + 0] = q8(r * sc);
        rgba[p * 4 + 1] = q8(g * sc);
        rgba[p * 4 + 2] = q8(b * sc);
        rgba[p * 4 + 3] = 255;
    }
}

/* ------------------------------------------------------ shadow mode [SPEC] */
/* DESIGN.md "Shadow mode": one shadow ray per primary hit toward the point
 * light L, any-hit over (0, 1) of S -> L, Lambert term, ambient floor.
 * Writes the primary hits and the shaded RGBA8 image. */
static void shade_sample(const orc_node* nodes, uint32_t n, const float* tris, const float o[3],
                         const float d[3], const orc_hit* h, const float L[3], float ambient,
                         float rgb[3], uint64_t* cn, uint64_t* ct) {
    if (h->prim == ORC_SENTINEL) { rgb[0] = rgb[1] = rgb[2] = 0.0f; return; }
    const float* tri = tris + (size_t)h->prim * 9;
    float P[3], e1[3], e2[3], nrm[3], N[3], S[3], D[3];
    for (int a = 0; a < 3; ++a) {
        P[a] = o[a] + h->t * d[a];
        e1[a] = tri[3 + a] - tri[a];
        e2[a] = tri[6 + a] - tri[a];
    }
    cross3(e1, e2, nrm);
    const float nl = sqrtf(dot3(nrm, nrm));
    for (int a = 0; a < 3; ++a) N[a] = nl > 0.0f ? nrm[a] / nl : 0.0f;
    if (dot3(N, d) > 0.0f)
        for (int a = 0; a < 3; ++a) N[a] = -N[a];
    for (int a = 0; a < 3; ++a) {
        S[a] = P[a] + N[a] * 1e-4f;
        D[a] = L[a] - S[a];
    }
    orc_hit sh;
    trace_ray_t(nodes, n, tris, S, D, 1.0f, 1, &sh, cn, ct);
    const float dl = sqrtf(dot3(D, D));
    const float cosl = dl > 0.0f ? dot3(N, D) / dl : 0.0f;
    const float lit = sh.prim != ORC_SENTINEL ? 0.0f : FMAX(cosl, 0.0f);
    const float f = ambient + (1.0f - ambient) * lit;
    rgb[0] = h->u * f;
    rgb[1] = h->v * f;
    rgb[2] = ((1.0f - h->u) - h->v) * f;
}

void orc_render_shadow(const orc_node* nodes, uint32_t n, const float* tris, const orc_camera* cam,
                       uint32_t w, uint32_t h, uint32_t spp, const float light[3], float ambient,
                       orc_hit* hits, uint8_t* rgba, uint64_t counters[2], int nthreads) {
    uint64_t c2[2] = {0, 0};
    orc_trace(nodes, n, tris, cam, w, h, spp, 0, 1, hits, c2, nthreads);
    uint64_t cn = 0, ct = 0;
    const float sc = 1.0f / (float)spp;
    for (uint64_t y = 0; y < h; ++y)
        for (uint32_t x = 0; x < w; ++x) {
            float r = 0.0f, g = 0.0f, b = 0.0f;
            for (uint32_t s = 0; s < spp; ++s) {
                const uint32_t sidx = (uint32_t)((y * w + x) * spp + s);
                float jx = 0.5f, jy = 0.5f;
                if (s > 0) {
                    const uint32_t hh = orc_pcg_hash(sidx);
                    jx = (float)(hh >> 8) * 0x1p-24f;
                    jy = (float)(orc_pcg_hash(hh) >> 8) * 0x1p-24f;
                }
                const float px = (float)x + jx, py = (float)y + jy;
                float d[3], rgb[3];
                for (int a = 0; a < 3; ++a) d[a] = (cam->w00[a] + px * cam->du[a]) + py * cam->dv[a];
                shade_sample(nodes, n, tris, cam->eye, d, &hits[sidx], light, ambient, rgb, &cn, &ct);
                r = r + rgb[0];
                g = g + rgb[1];
                b = b + rgb[2];
            }
            const uint64_t p = y * w + x;
            rgba[p * 4 + 0] = q8(r * sc);
            rgba[p * 4 + 1] = q8(g * sc);
            rgba[p * 4 + 2] = q8(b * sc);
            rgba[p * 4 + 3] = 255;
        }
    if (counters) { counters[0] = cn; counters[1] = ct; }
}

/* ------------------------------------------------------- path mode [SPEC] */
/* DESIGN.md "Path mode" ("simple path tracing"):
 * per sample, a diffuse path of up to 1 + max_depth closest-hit segments.
 * At every hit: next-event estimation toward the point light (one any-hit
 * shadow ray over (0, 1), traced only when the light is above the surface),
 * then -- below max_depth -- a cosine-weighted bounce about the
 * viewer-facing geometric normal.  Escaped bounce rays add the constant sky
 * radiance; an escaped primary ray is black.  Albedo per triangle from
 * pcg_hash(prim).  Every operation is IEEE fp32 (+, -, *, /, sqrtf) in the
 * order written, so the GPU result is bit-identical. */
static inline uint32_t path_next(uint32_t* st) { *st = orc_pcg_hash(*st); return *st; }
static inline float path_u01(uint32_t* st) { return (float)(path_next(st) >> 8) * 0x1p-24f; }

static void path_sample(const orc_node* nodes, uint32_t n, const float* tris, const float eye[3],
                        const float d0[3], uint32_t sidx, const float Lp[3], float sky, uint32_t max_depth,
                        orc_hit* primary, float Lo[3], uint64_t cnt[3]) {
    float o[3] = {eye[0], eye[1], eye[2]}, d[3] = {d0[0], d0[1], d0[2]};
    float L[3] = {0.0f, 0.0f, 0.0f}, beta[3] = {1.0f, 1.0f, 1.0f};
    uint32_t st = orc_pcg_hash(sidx ^ 0x5bd1e995u);
    for (uint32_t depth = 0;; ++depth) {
        orc_hit h;
        trace_ray_t(nodes, n, tris, o, d, INFINITY, 0, &h, &cnt[0], &cnt[1]);
        ++cnt[2];
        if (depth == 0 && primary) *primary = h;
        if (h.prim == ORC_SENTINEL) {
            if (depth > 0)
                for (int a = 0; a < 3; ++a) L[a] = L[a] + beta[a] * sky;
            break;
        }
        const float* tri = tris + (size_t)h.prim * 9;
        float P[3], e1[3], e2[3], nrm[3], N[3], S[3], D[3], alb[3];
        for (int a = 0; a < 3; ++a) {
            P[a] = o[a] + h.t * d[a];
            e1[a] = tri[3 + a] - tri[a];
            e2[a] = tri[6 + a] - tri[a];
        }
        cross3(e1, e2, nrm);
        const float nl = sqrtf(dot3(nrm, nrm));
        for (int a = 0; a < 3; ++a) N[a] = nl > 0.0f ? nrm[a] / nl : 0.0f;
        if (dot3(N, d) > 0.0f)
            for (int a = 0; a < 3; ++a) N[a] = -N[a];
        const uint32_t ha = orc_pcg_hash(h.prim ^ 0x27d4eb2fu);
        for (int a = 0; a < 3; ++a) {
            S[a] = P[a] + N[a] * 1e-4f;
            D[a] = Lp[a] - S[a];
            alb[a] = 0.25f + (float)((ha >> (8 * a)) & 0xFFu) * 0x1p-9f;
        }
        const float dl = sqrtf(dot3(D, D));
        const float cosl = dl > 0.0f ? dot3(N, D) / dl : 0.0f;
        if (cosl > 0.0f) {
            orc_hit sh;
            trace_ray_t(nodes, n, tris, S, D, 1.0f, 1, &sh, &cnt[0], &cnt[1]);
            ++cnt[2];
            if (sh.prim == ORC_SENTINEL)
                for (int a = 0; a < 3; ++a) L[a] = L[a] + (beta[a] * alb[a]) * cosl;
        }
        if (depth == max_depth) break;
        for (int a = 0; a < 3; ++a) beta[a] = beta[a] * alb[a];
        /* cosine-weighted direction: a point of the unit disk by rejection
         * (16 tries, then the centre), lifted to the hemisphere about N */
        float px = 0.0f, py = 0.0f, r2 = 0.0f;
        for (int k = 0; k < 16; ++k) {
            const float qx = path_u01(&st) * 2.0f - 1.0f;
            const float qy = path_u01(&st) * 2.0f - 1.0f;
            const float q2 = qx * qx + qy * qy;
            if (q2 < 1.0f) { px = qx; py = qy; r2 = q2; break; }
        }
        const float z = sqrtf(1.0f - r2);
        const float sg = N[2] >= 0.0f ? 1.0f : -1.0f;
        const float ia = -1.0f / (sg + N[2]);
        const float ib = (N[0] * N[1]) * ia;
        const float T[3] = {1.0f + ((sg * N[0]) * N[0]) * ia, sg * ib, -(sg * N[0])};
        const float B[3] = {ib, sg + (N[1] * N[1]) * ia, -N[1]};
        for (int a = 0; a < 3; ++a) {
            d[a] = (px * T[a] + py * B[a]) + z * N[a];
            o[a] = S[a];
        }
    }
    for (int a = 0; a < 3; ++a) Lo[a] = L[a];
}

typedef struct {
    const orc_node* nodes; uint32_t n; const float* tris; const orc_camera* cam;
    uint32_t w, h, spp, max_depth; const float* light; float sky;
    orc_hit* hits; uint8_t* rgba; int tid, nthreads; uint64_t cnt[3];
} path_job;

static void* path_worker(void* arg) {
    path_job* j = (path_job*)arg;
    const orc_camera* c = j->cam;
    const float sc = 1.0f / (float)j->spp;
    for (uint64_t y = (uint64_t)j->tid; y < j->h; y += (uint64_t)j->nthreads)
        for (uint32_t x = 0; x < j->w; ++x) {
            float r = 0.0f, g = 0.0f, b = 0.0f;
            for (uint32_t s = 0; s < j->spp; ++s) {
                const uint32_t sidx = (uint32_t)((y * j->w + x) * j->spp + s);
                float jx = 0.5f, jy = 0.5f;
                if (s > 0) {
                    const uint32_t hh = orc_pcg_hash(sidx);
                    jx = (float)(hh >> 8) * 0x1p-24f;
                    jy = (float)(orc_pcg_hash(hh) >> 8) * 0x1p-24f;
                }
                const float px = (float)x + jx, py = (float)y + jy;
                float d[3], rgb[3];
                for (int a = 0; a < 3; ++a) d[a] = (c->w00[a] + px * c->du[a]) + py * c->dv[a];
                path_sample(j->nodes, j->n, j->tris, c->eye, d, sidx, j->light, j->sky, j->max_depth,
                            j->hits ? &j->hits[sidx] : NULL, rgb, j->cnt);
                r = r + rgb[0];
                g = g + rgb[1];
                b = b + rgb[2];
            }
            const uint64_t p = y * j->w + x;
            j->rgba[p * 4 + 0] = q8(r * sc);
            j->rgba[p * 4 + 1] = q8(g * sc);
            j->rgba[p * 4 + 2] = q8(b * sc);
            j->rgba[p * 4 + 3] = 255;
        }
    return NULL;
}

void orc_render_path(const orc_node* nodes, uint32_t n, const float* tris, const orc_camera* cam,
                     uint32_t w, uint32_t h, uint32_t spp, const float light[3], float sky, uint32_t max_depth,
                     orc_hit* hits, uint8_t* rgba, uint64_t counters[3], int nthreads) {
    if (nthreads < 1) nthreads = 1;
    path_job* jobs = (path_job*)calloc((size_t)nthreads, sizeof(path_job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    unsigned char* live = (unsigned char*)calloc((size_t)nthreads, 1);
    for (int t = 0; t < nthreads; ++t) {
        path_job jb = {nodes, n, tris, cam, w, h, spp, max_depth, light, sky, hits, rgba, t, nthreads, {0, 0, 0}};
        jobs[t] = jb;
    }
    for (int t = 1; t < nthreads; ++t) live[t] = spawn(&th[t], path_worker, &jobs[t]);
    path_worker(&jobs[0]);
    for (int t = 1; t < nthreads; ++t) {  /* a thread that did not start: its rows on the caller */
        if (live[t]) pthread_join(th[t], NULL);
        else path_worker(&jobs[t]);
    }
    free(live);
    if (counters) {
        counters[0] = counters[1] = counters[2] = 0;
        for (int t = 0; t < nthreads; ++t)
            for (int k = 0; k < 3; ++k) counters[k] += jobs[t].cnt[k];
    }
    free(jobs);
    free(th);
}

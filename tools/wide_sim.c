/* wide_sim.c -- CPU model of the wide traversal's step counts for K-ary
 * greedy cuts of the binary tree (design experiment, not test or product code).
 *
 * Record X = X's cut with up to K entries: start from X's two children and
 * repeatedly replace the internal entry with the largest box surface by its
 * two children (K = 4 is build.wide_collapse = 1).  A step (wide_step in
 * trace_kernels.hip) processes at most one record and one leaf.  Boxes are
 * the exact binary boxes (the GPU's quantized boxes only add entries).
 *
 * Build: gcc -O2 -shared -fPIC -o /tmp/libwsim.so tools/wide_sim.c -L oracle/build -loracle -lm
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float lo[3], hi[3]; uint32_t a, esc; } node_t;
typedef struct { float eye[3], w00[3], du[3], dv[3]; } cam_t;
int orc_intersect_tri(const float o[3], const float d[3], const float* tri, float t_best, float* t, float* u, float* v);
float orc_fmin(float, float);
float orc_fmax(float, float);

static float area(const node_t* b) {
    float e0 = b->hi[0] - b->lo[0], e1 = b->hi[1] - b->lo[1], e2 = b->hi[2] - b->lo[2];
    return e0 * e1 + e1 * e2 + e2 * e0;
}

/* cut[X*K + i]: entry i of record X (unified node index), SENT past the end */
void wsim_cut(const node_t* nodes, uint32_t n, uint32_t K, uint32_t* cut) {
    const uint32_t L0 = n - 1;
    for (uint32_t x = 0; x + 1 < n; ++x) {
        uint32_t e[16], m = 2;
        e[0] = nodes[x].a;
        e[1] = nodes[e[0]].esc;
        while (m < K) {
            int best = -1;
            float ba = -1.0f;
            for (uint32_t i = 0; i < m; ++i)
                if (e[i] < L0 && area(&nodes[e[i]]) > ba) { ba = area(&nodes[e[i]]); best = (int)i; }
            if (best < 0) break;
            const uint32_t l = nodes[e[best]].a, r = nodes[l].esc;
            memmove(&e[best + 2], &e[best + 1], sizeof(uint32_t) * (m - best - 1));
            e[best] = l;
            e[best + 1] = r;
            ++m;
        }
        for (uint32_t i = 0; i < K; ++i) cut[(size_t)x * K + i] = i < m ? e[i] : 0xFFFFFFFFu;
    }
}

static int slab(const node_t* b, const float* o, const float* invd, float tb, float* tn_out) {
    float t0[3], t1[3];
    for (int a = 0; a < 3; ++a) { t0[a] = (b->lo[a] - o[a]) * invd[a]; t1[a] = (b->hi[a] - o[a]) * invd[a]; }
    const float tn = orc_fmax(orc_fmax(orc_fmax(orc_fmin(t0[0], t1[0]), orc_fmin(t0[1], t1[1])), orc_fmin(t0[2], t1[2])), 0.0f);
    const float tf = orc_fmin(orc_fmin(orc_fmin(orc_fmax(t0[0], t1[0]), orc_fmax(t0[1], t1[1])), orc_fmax(t0[2], t1[2])), tb);
    *tn_out = tn;
    return tn <= tf;
}

/* steps[pixel], recs[pixel], leaves[pixel]; returns prim of the hit in hitp */
void wsim_trace(const node_t* nodes, uint32_t n, const float* tris, const uint32_t* cut, uint32_t K,
                const cam_t* c, uint32_t w, uint32_t h, uint32_t y0, uint32_t y1, uint16_t* steps, uint16_t* recs,
                uint16_t* leaves, uint32_t* hitp, uint8_t* maxsp) {
    const uint32_t L0 = n - 1;
    uint32_t stk[512];
    float stn[512];
    for (uint32_t y = y0; y < y1; ++y)
        for (uint32_t x = 0; x < w; ++x) {
            const float px = (float)x + 0.5f, py = (float)y + 0.5f;
            float d[3], invd[3];
            for (int a = 0; a < 3; ++a) {
                d[a] = (c->w00[a] + px * c->du[a]) + py * c->dv[a];
                invd[a] = 1.0f / d[a];
            }
            float tb = INFINITY;
            uint32_t hp = 0xFFFFFFFFu, sp = 0, cur = 0, pend = 0xFFFFFFFFu, ns = 0, nr = 0, nl = 0, msp = 0;
            float ctn = 0.0f;
            for (;;) {
                if (pend == 0xFFFFFFFFu) {
                    if (cur == 0xFFFFFFFFu) { if (sp) { --sp; cur = stk[sp]; ctn = stn[sp]; } }
                    if (cur != 0xFFFFFFFFu && cur >= L0) {
                        pend = cur;
                        cur = 0xFFFFFFFFu;
                        if (sp) { --sp; cur = stk[sp]; ctn = stn[sp]; }
                    }
                }
                if (pend == 0xFFFFFFFFu && cur == 0xFFFFFFFFu) break;
                ++ns;
                if (pend != 0xFFFFFFFFu) {
                    ++nl;
                    float tn, t, u, v;
                    const node_t* lf = &nodes[pend];
                    if (slab(lf, c->eye, invd, tb, &tn) &&
                        orc_intersect_tri(c->eye, d, tris + (size_t)lf->a * 9, tb, &t, &u, &v)) {
                        tb = t;
                        hp = lf->a;
                    }
                    pend = 0xFFFFFFFFu;
                }
                if (cur == 0xFFFFFFFFu || cur >= L0) continue;  /* a second popped leaf waits for the next step */
                if (ctn > tb) { cur = 0xFFFFFFFFu; continue; }
                ++nr;
                const uint32_t* e = cut + (size_t)cur * K;
                uint32_t hit[16], m = 0;
                float htn[16];
                for (uint32_t i = 0; i < K && e[i] != 0xFFFFFFFFu; ++i) {
                    float tn;
                    if (slab(&nodes[e[i]], c->eye, invd, tb, &tn)) { hit[m] = e[i]; htn[m] = tn; ++m; }
                }
                cur = 0xFFFFFFFFu;
                if (m) {
                    for (uint32_t i = m - 1; i >= 1; --i) { stk[sp] = hit[i]; stn[sp] = htn[i]; ++sp; }
                    if (sp > msp) msp = sp;
                    cur = hit[0];
                    ctn = htn[0];
                }
            }
            const size_t p = (size_t)y * w + x;
            steps[p] = (uint16_t)(ns > 65535 ? 65535 : ns);
            recs[p] = (uint16_t)(nr > 65535 ? 65535 : nr);
            leaves[p] = (uint16_t)(nl > 65535 ? 65535 : nl);
            hitp[p] = hp;
            maxsp[p] = (uint8_t)(msp > 255 ? 255 : msp);
        }
}

/* wide_sim.c -- CPU model of the wide traversal's step counts for K-ary
 * greedy cuts of the binary tree (design experiment, not test or product code).
 *
 * Record X = X's cut with up to K entries: start from X's two children and
 * repeatedly replace the internal entry with the largest box surface by its
 * two children (K = 4 is build.wide_collapse = 1).  A step (wide_step in
 * trace_kernels.hip) processes at most one record and one leaf.  Boxes are
 * the exact binary boxes (the GPU's quantized boxes only add entries).
 *
 * Build: gcc -O2 -shared -fPIC -o /tmp/libwsim.so tests/tools/wide_sim.c -L oracle/build -loracle -lm
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

/* ---- wave model: the 64 lanes of each 8x8 quadrant step together; a step
 * runs the leaf block when any lane tests a leaf and the record block when
 * any lane tests a record.  policy 0 = today's (a popped leaf is tested in
 * the next step); policy F > 0 = a per-lane FIFO of up to F popped leaves,
 * served (one per lane) only when some lane cannot go on without it (FIFO
 * full, or no record left) or at least T lanes hold one.  Leaves are folded
 * in preorder either way (exact); records are tested with the current tb.
 * out[0] wave-steps, out[1] leaf blocks run, out[2] record blocks run,
 * out[3] lane-leaf tests, out[4] lane-record tests, out[5] sum over waves of
 * the VALU cost model (40 + 116*leafblock + 136*recblock per step). */
typedef struct {
    uint32_t stk[48]; float stn[48]; uint32_t sp, cur; float ctn, tb; uint32_t hp, pix;
    uint32_t fifo[16]; uint32_t fc; int done; float d[3], invd[3];
} lane_t;

static int leaf_test(const node_t* nodes, const float* tris, const float* o, lane_t* L, uint32_t leaf) {
    float tn, t, u, v;
    const node_t* lf = &nodes[leaf];
    if (slab(lf, o, L->invd, L->tb, &tn) && orc_intersect_tri(o, L->d, tris + (size_t)lf->a * 9, L->tb, &t, &u, &v)) {
        L->tb = t;
        L->hp = lf->a;
        return 1;
    }
    return 0;
}

void wsim_waves(const node_t* nodes, uint32_t n, const float* tris, const uint32_t* cut, uint32_t K, const cam_t* c,
                uint32_t w, uint32_t h, uint32_t qy0, uint32_t qy1, uint32_t F, uint32_t T, double* out,
                uint32_t* hitp) {
    const uint32_t L0 = n - 1;
    static __thread lane_t lanes[64];
    for (uint32_t qy = qy0; qy < qy1; ++qy)
        for (uint32_t qx = 0; qx < w / 8; ++qx) {
            for (int l = 0; l < 64; ++l) {
                lane_t* L = &lanes[l];
                const uint32_t x = qx * 8 + (l & 7), y = qy * 8 + (l >> 3);
                const float px = (float)x + 0.5f, py = (float)y + 0.5f;
                for (int a = 0; a < 3; ++a) {
                    L->d[a] = (c->w00[a] + px * c->du[a]) + py * c->dv[a];
                    L->invd[a] = 1.0f / L->d[a];
                }
                L->tb = INFINITY; L->hp = 0xFFFFFFFFu; L->sp = 0; L->cur = 0; L->ctn = 0.0f; L->fc = 0; L->done = 0;
            }
            uint32_t pend[64];
            for (int l = 0; l < 64; ++l) pend[l] = 0xFFFFFFFFu;
            for (;;) {
                int any = 0;
                /* gather phase: pops */
                int want = 0, have = 0;
                for (int l = 0; l < 64; ++l) {
                    lane_t* L = &lanes[l];
                    if (L->done) continue;
                    if (F == 0) {
                        if (pend[l] == 0xFFFFFFFFu) {
                            if (L->cur == 0xFFFFFFFFu && L->sp) { --L->sp; L->cur = L->stk[L->sp]; L->ctn = L->stn[L->sp]; }
                            if (L->cur != 0xFFFFFFFFu && L->cur >= L0) {
                                pend[l] = L->cur; L->cur = 0xFFFFFFFFu;
                                if (L->sp) { --L->sp; L->cur = L->stk[L->sp]; L->ctn = L->stn[L->sp]; }
                            }
                        }
                        if (pend[l] == 0xFFFFFFFFu && L->cur == 0xFFFFFFFFu) { L->done = 1; continue; }
                    } else {
                        for (;;) {
                            if (L->cur == 0xFFFFFFFFu && L->sp) { --L->sp; L->cur = L->stk[L->sp]; L->ctn = L->stn[L->sp]; }
                            if (L->cur != 0xFFFFFFFFu && L->cur >= L0 && L->fc < F) { L->fifo[L->fc++] = L->cur; L->cur = 0xFFFFFFFFu; continue; }
                            break;
                        }
                        if (L->fc == 0 && L->cur == 0xFFFFFFFFu) { L->done = 1; continue; }
                        if (L->fc && (L->fc == F || L->cur == 0xFFFFFFFFu || L->cur >= L0)) want = 1;
                        if (L->fc) ++have;
                    }
                    any = 1;
                }
                if (!any) break;
                const int serve = F == 0 ? 1 : (want || have >= (int)T);
                int lb = 0, rb = 0;
                for (int l = 0; l < 64; ++l) {
                    lane_t* L = &lanes[l];
                    if (L->done) continue;
                    if (F == 0) {
                        if (pend[l] != 0xFFFFFFFFu) { lb = 1; out[3] += 1; leaf_test(nodes, tris, c->eye, L, pend[l]); pend[l] = 0xFFFFFFFFu; }
                    } else if (serve && L->fc) {
                        lb = 1; out[3] += 1;
                        leaf_test(nodes, tris, c->eye, L, L->fifo[0]);
                        memmove(&L->fifo[0], &L->fifo[1], sizeof(uint32_t) * (L->fc - 1));
                        --L->fc;
                    }
                    if (L->cur == 0xFFFFFFFFu || L->cur >= L0) continue;
                    if (L->ctn > L->tb) { L->cur = 0xFFFFFFFFu; continue; }
                    rb = 1; out[4] += 1;
                    const uint32_t* e = cut + (size_t)L->cur * K;
                    uint32_t hit[16], m = 0;
                    float htn[16];
                    for (uint32_t i = 0; i < K && e[i] != 0xFFFFFFFFu; ++i) {
                        float tn;
                        if (slab(&nodes[e[i]], c->eye, L->invd, L->tb, &tn)) { hit[m] = e[i]; htn[m] = tn; ++m; }
                    }
                    L->cur = 0xFFFFFFFFu;
                    if (m) {
                        for (uint32_t i = m - 1; i >= 1; --i) { L->stk[L->sp] = hit[i]; L->stn[L->sp] = htn[i]; ++L->sp; }
                        L->cur = hit[0]; L->ctn = htn[0];
                    }
                }
                out[0] += 1; out[1] += lb; out[2] += rb;
                out[5] += 40.0 + 116.0 * lb + 136.0 * rb;
            }
            for (int l = 0; l < 64; ++l) hitp[(size_t)(qy * 8 + (l >> 3)) * w + qx * 8 + (l & 7)] = lanes[l].hp;
        }
}

/* ---- wave compaction model: pass 1 runs each 8x8-quadrant wave (policy 0
 * steps) until fewer than A of its lanes are still tracing (after at least
 * S steps); those rays are queued with their state and pass 2 runs the queue
 * packed 64 rays per wave, in queue order, to completion.  out as
 * wsim_waves (pass 1 + pass 2), out[6] = rays queued. */
static void run_wave(const node_t* nodes, uint32_t n, const float* tris, const uint32_t* cut, uint32_t K,
                     const float* o, lane_t* lanes, int nl, uint32_t A, uint32_t S, double* out, lane_t* q,
                     size_t* nq) {
    const uint32_t L0 = n - 1;
    uint32_t pend[64];
    for (int l = 0; l < 64; ++l) pend[l] = 0xFFFFFFFFu;
    for (uint32_t step = 0;; ++step) {
        int act = 0;
        for (int l = 0; l < nl; ++l) {
            lane_t* L = &lanes[l];
            if (L->done) continue;
            if (pend[l] == 0xFFFFFFFFu) {
                if (L->cur == 0xFFFFFFFFu && L->sp) { --L->sp; L->cur = L->stk[L->sp]; L->ctn = L->stn[L->sp]; }
                if (L->cur != 0xFFFFFFFFu && L->cur >= L0) {
                    pend[l] = L->cur; L->cur = 0xFFFFFFFFu;
                    if (L->sp) { --L->sp; L->cur = L->stk[L->sp]; L->ctn = L->stn[L->sp]; }
                }
            }
            if (pend[l] == 0xFFFFFFFFu && L->cur == 0xFFFFFFFFu) { L->done = 1; continue; }
            ++act;
        }
        if (!act) break;
        if (q && step >= S && (uint32_t)act < A) {  /* compact: queue the live rays (pending leaf back on top) */
            for (int l = 0; l < nl; ++l) {
                lane_t* L = &lanes[l];
                if (L->done) continue;
                if (pend[l] != 0xFFFFFFFFu) {  /* order: pend, cur, stack */
                    if (L->cur != 0xFFFFFFFFu) { L->stk[L->sp] = L->cur; L->stn[L->sp] = L->ctn; ++L->sp; }
                    L->cur = pend[l]; L->ctn = 0.0f;
                }
                q[(*nq)++] = *L;
                L->done = 1;
            }
            out[6] += act;
            break;
        }
        int lb = 0, rb = 0;
        for (int l = 0; l < nl; ++l) {
            lane_t* L = &lanes[l];
            if (L->done) continue;
            if (pend[l] != 0xFFFFFFFFu) { lb = 1; out[3] += 1; leaf_test(nodes, tris, o, L, pend[l]); pend[l] = 0xFFFFFFFFu; }
            if (L->cur == 0xFFFFFFFFu || L->cur >= L0) continue;
            if (L->ctn > L->tb) { L->cur = 0xFFFFFFFFu; continue; }
            rb = 1; out[4] += 1;
            const uint32_t* e = cut + (size_t)L->cur * K;
            uint32_t hit[16], m = 0;
            float htn[16];
            for (uint32_t i = 0; i < K && e[i] != 0xFFFFFFFFu; ++i) {
                float tn;
                if (slab(&nodes[e[i]], o, L->invd, L->tb, &tn)) { hit[m] = e[i]; htn[m] = tn; ++m; }
            }
            L->cur = 0xFFFFFFFFu;
            if (m) {
                for (uint32_t i = m - 1; i >= 1; --i) { L->stk[L->sp] = hit[i]; L->stn[L->sp] = htn[i]; ++L->sp; }
                L->cur = hit[0]; L->ctn = htn[0];
            }
        }
        out[0] += 1; out[1] += lb; out[2] += rb;
        out[5] += 40.0 + 116.0 * lb + 136.0 * rb;
    }
}

void wsim_compact(const node_t* nodes, uint32_t n, const float* tris, const uint32_t* cut, uint32_t K, const cam_t* c,
                  uint32_t w, uint32_t h, uint32_t qy0, uint32_t qy1, uint32_t A, uint32_t S, double* out,
                  uint32_t* hitp) {
    lane_t lanes[64];
    const size_t cap = (size_t)(qy1 - qy0) * (w / 8) * 64;
    lane_t* q = (lane_t*)malloc(sizeof(lane_t) * cap);
    size_t nq = 0;
    for (uint32_t qy = qy0; qy < qy1; ++qy)
        for (uint32_t qx = 0; qx < w / 8; ++qx) {
            for (int l = 0; l < 64; ++l) {
                lane_t* L = &lanes[l];
                const uint32_t x = qx * 8 + (l & 7), y = qy * 8 + (l >> 3);
                const float px = (float)x + 0.5f, py = (float)y + 0.5f;
                for (int a = 0; a < 3; ++a) {
                    L->d[a] = (c->w00[a] + px * c->du[a]) + py * c->dv[a];
                    L->invd[a] = 1.0f / L->d[a];
                }
                L->tb = INFINITY; L->hp = 0xFFFFFFFFu; L->sp = 0; L->cur = 0; L->ctn = 0.0f; L->fc = 0; L->done = 0;
                L->pix = y * w + x;
            }
            run_wave(nodes, n, tris, cut, K, c->eye, lanes, 64, A, S, out, q, &nq);
            for (int l = 0; l < 64; ++l) if (lanes[l].hp != 0xFFFFFFFFu || 1) hitp[lanes[l].pix] = lanes[l].hp;
        }
    /* pass 2: the queue, 64 rays per wave; a queued ray's hit is written at the end */
    for (size_t b = 0; b < nq; b += 64) {
        const int nl = (int)(nq - b < 64 ? nq - b : 64);
        for (int l = 0; l < nl; ++l) { lanes[l] = q[b + l]; lanes[l].done = 0; }
        run_wave(nodes, n, tris, cut, K, c->eye, lanes, nl, 0, 0, out, NULL, NULL);
        for (int l = 0; l < nl; ++l) hitp[lanes[l].pix] = lanes[l].hp;
    }
    free(q);
}

/* Top-of-stack prefetch model (design experiment): the lane keeps the record
 * (or leaf) on top of its stack loaded, re-issuing the load whenever the top
 * changes.  A step needs no memory wait when everything it processes came off
 * the stack as a top established at least two steps earlier (its load was in
 * flight for a whole step); entries reached by descent, or a second entry
 * popped in one step, still wait.  ready[pixel] = such steps. */
void wsim_chain(const node_t* nodes, uint32_t n, const float* tris, const uint32_t* cut, uint32_t K,
                const cam_t* c, uint32_t w, uint32_t h, uint32_t y0, uint32_t y1, uint16_t* steps, uint16_t* ready,
                uint32_t* hitp) {
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
            uint32_t hp = 0xFFFFFFFFu, sp = 0, cur = 0, pend = 0xFFFFFFFFu, ns = 0, nready = 0;
            int top_step = -1000;            /* step whose end established the current top */
            int cur_ok = 0, pend_ok = 0;     /* data already present for cur / pend */
            float ctn = 0.0f;
            for (;;) {
                const int s = (int)ns;
                if (pend == 0xFFFFFFFFu) {
                    int popped = 0;
                    if (cur == 0xFFFFFFFFu && sp) {
                        --sp; cur = stk[sp]; ctn = stn[sp];
                        cur_ok = (s - top_step >= 2);
                        top_step = s - 1;
                        popped = 1;
                    }
                    if (cur != 0xFFFFFFFFu && cur >= L0) {
                        pend = cur;
                        pend_ok = cur_ok;
                        cur = 0xFFFFFFFFu;
                        if (sp) {
                            --sp; cur = stk[sp]; ctn = stn[sp];
                            cur_ok = popped ? 0 : (s - top_step >= 2);  /* a second pop in one step waits */
                            top_step = s - 1;
                        }
                    }
                }
                if (pend == 0xFFFFFFFFu && cur == 0xFFFFFFFFu) break;
                ++ns;
                int ok = 1;
                if (pend != 0xFFFFFFFFu) {
                    ok &= pend_ok;
                    float tn, t, u, v;
                    const node_t* lf = &nodes[pend];
                    if (slab(lf, c->eye, invd, tb, &tn) &&
                        orc_intersect_tri(c->eye, d, tris + (size_t)lf->a * 9, tb, &t, &u, &v)) {
                        tb = t;
                        hp = lf->a;
                    }
                    pend = 0xFFFFFFFFu;
                }
                if (cur == 0xFFFFFFFFu || cur >= L0) { nready += ok; continue; }
                if (ctn > tb) { nready += ok; cur = 0xFFFFFFFFu; continue; }
                ok &= cur_ok;
                nready += ok;
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
                    if (m > 1) top_step = s;  /* pushed at the end of this step */
                    cur = hit[0];
                    ctn = htn[0];
                    cur_ok = 0;              /* reached by descent: fetched next step */
                }
            }
            const size_t p = (size_t)y * w + x;
            steps[p] = (uint16_t)(ns > 65535 ? 65535 : ns);
            ready[p] = (uint16_t)(nready > 65535 ? 65535 : nready);
            hitp[p] = hp;
        }
}

/* ---- SAH-optimal K-ary cut (r03 design experiment).  C(x) = ci*SA(x) +
 * min over cuts of x's subtree with <= K entries of sum(cost(e)), cost(leaf)
 * = cl*SA(leaf), cost(internal e) = C(e): a post-order DP with B(y, j) = the
 * cheapest cover of y's subtree by <= j entries.  Entries in preorder. */
#define SAH_KMAX 8
static float* g_B;      /* [node][j], j = 1..K (index j-1), unified index */
static uint8_t* g_ch;   /* split choice: 0 = y itself, else j1 for the left child */
static uint32_t g_K;
static void sah_emit(const node_t* nodes, uint32_t L0, uint32_t y, uint32_t j, uint32_t* e, uint32_t* m) {
    const uint8_t c = (y < L0) ? g_ch[(size_t)y * SAH_KMAX + (j - 1)] : 0;
    if (c == 0) { e[(*m)++] = y; return; }
    const uint32_t l = nodes[y].a, r = nodes[l].esc;
    sah_emit(nodes, L0, l, c, e, m);
    sah_emit(nodes, L0, r, j - c, e, m);
}
void wsim_cut_sah(const node_t* nodes, uint32_t n, uint32_t K, float ci, float cl, uint32_t* cut) {
    const uint32_t L0 = n - 1, NN = 2 * n - 1;
    g_K = K;
    g_B = (float*)malloc(sizeof(float) * (size_t)NN * SAH_KMAX);
    g_ch = (uint8_t*)calloc((size_t)NN * SAH_KMAX, 1);
    uint8_t* top = (uint8_t*)calloc((size_t)n, 1); /* best split for the record of x (j1 for left) */
    for (uint32_t k = 0; k < n; ++k)
        for (uint32_t j = 0; j < SAH_KMAX; ++j) g_B[(size_t)(L0 + k) * SAH_KMAX + j] = cl * area(&nodes[L0 + k]);
    /* iterative post-order over internal nodes */
    uint32_t* st = (uint32_t*)malloc(sizeof(uint32_t) * 2 * n);
    uint8_t* vis = (uint8_t*)calloc(n, 1);
    uint32_t sp = 0;
    st[sp++] = 0;
    while (sp) {
        const uint32_t y = st[sp - 1];
        const uint32_t l = nodes[y].a, r = nodes[l].esc;
        if (!vis[y]) {
            vis[y] = 1;
            if (r < L0) st[sp++] = r;
            if (l < L0) st[sp++] = l;
            continue;
        }
        --sp;
        const float* Bl = &g_B[(size_t)l * SAH_KMAX];
        const float* Br = &g_B[(size_t)r * SAH_KMAX];
        float best = INFINITY;
        uint8_t bj = 1;
        for (uint32_t j1 = 1; j1 < K; ++j1)
            for (uint32_t j2 = 1; j1 + j2 <= K; ++j2) {
                const float c = Bl[j1 - 1] + Br[j2 - 1];
                if (c < best) { best = c; bj = (uint8_t)j1; top[y] = (uint8_t)j1; top[y] |= (uint8_t)(j2 << 4); }
            }
        (void)bj;
        const float C = ci * area(&nodes[y]) + best;
        float* By = &g_B[(size_t)y * SAH_KMAX];
        uint8_t* cy = &g_ch[(size_t)y * SAH_KMAX];
        for (uint32_t j = 1; j <= K; ++j) {
            float b = C;
            uint8_t c = 0;
            for (uint32_t j1 = 1; j1 < j; ++j1) {
                const float v = Bl[j1 - 1] + Br[j - j1 - 1];
                if (v < b) { b = v; c = (uint8_t)j1; }
            }
            By[j - 1] = b;
            cy[j - 1] = c;
        }
    }
    for (uint32_t x = 0; x + 1 < n; ++x) {
        uint32_t e[SAH_KMAX], m = 0;
        const uint32_t l = nodes[x].a, r = nodes[l].esc;
        sah_emit(nodes, L0, l, top[x] & 15u, e, &m);
        sah_emit(nodes, L0, r, top[x] >> 4, e, &m);
        for (uint32_t i = 0; i < K; ++i) cut[(size_t)x * K + i] = i < m ? e[i] : 0xFFFFFFFFu;
    }
    free(st); free(vis); free(top); free(g_B); free(g_ch);
}

/* ---- In-block wave merging model (r03 design experiment).  One 16x16 tile =
 * four 8x8 quadrant waves stepping in lockstep rounds.  From round S on, a
 * wave with fewer than A live lanes hands its live rays to the block's pool
 * and exits, provided another wave of the block is still live; every round a
 * live wave first fills its finished lanes from the pool.  out[0] wave-steps,
 * out[1] leaf blocks, out[2] record blocks, out[3] VALU model, out[4] sum of
 * tile durations (rounds), out[5] rays moved, out[6] max tile rounds. */
typedef struct { lane_t L; uint32_t pend; } mray_t;
static int mlane_gather(uint32_t L0, lane_t* L, uint32_t* pend) {
    if (L->done) return 0;
    if (*pend == 0xFFFFFFFFu) {
        if (L->cur == 0xFFFFFFFFu && L->sp) { --L->sp; L->cur = L->stk[L->sp]; L->ctn = L->stn[L->sp]; }
        if (L->cur != 0xFFFFFFFFu && L->cur >= L0) {
            *pend = L->cur; L->cur = 0xFFFFFFFFu;
            if (L->sp) { --L->sp; L->cur = L->stk[L->sp]; L->ctn = L->stn[L->sp]; }
        }
    }
    if (*pend == 0xFFFFFFFFu && L->cur == 0xFFFFFFFFu) { L->done = 1; return 0; }
    return 1;
}
static void mlane_step(const node_t* nodes, uint32_t L0, const float* tris, const uint32_t* cut, uint32_t K,
                       const float* o, lane_t* L, uint32_t* pend, int* lb, int* rb) {
    if (*pend != 0xFFFFFFFFu) { *lb = 1; leaf_test(nodes, tris, o, L, *pend); *pend = 0xFFFFFFFFu; }
    if (L->cur == 0xFFFFFFFFu || L->cur >= L0) return;
    if (L->ctn > L->tb) { L->cur = 0xFFFFFFFFu; return; }
    *rb = 1;
    const uint32_t* e = cut + (size_t)L->cur * K;
    uint32_t hit[16], m = 0;
    float htn[16];
    for (uint32_t i = 0; i < K && e[i] != 0xFFFFFFFFu; ++i) {
        float tn;
        if (slab(&nodes[e[i]], o, L->invd, L->tb, &tn)) { hit[m] = e[i]; htn[m] = tn; ++m; }
    }
    L->cur = 0xFFFFFFFFu;
    if (m) {
        for (uint32_t i = m - 1; i >= 1; --i) { L->stk[L->sp] = hit[i]; L->stn[L->sp] = htn[i]; ++L->sp; }
        L->cur = hit[0]; L->ctn = htn[0];
    }
}
void wsim_merge(const node_t* nodes, uint32_t n, const float* tris, const uint32_t* cut, uint32_t K, const cam_t* c,
                uint32_t w, uint32_t h, uint32_t ty0, uint32_t ty1, uint32_t A, uint32_t S, double* out,
                uint32_t* hitp) {
    const uint32_t L0 = n - 1;
    static __thread lane_t lanes[4][64];
    static __thread uint32_t pend[4][64];
    static __thread mray_t pool[256];
    for (uint32_t ty = ty0; ty < ty1; ++ty)
        for (uint32_t tx = 0; tx < w / 16; ++tx) {
            int wlive[4] = {1, 1, 1, 1};
            uint32_t np = 0;
            for (int wv = 0; wv < 4; ++wv)
                for (int l = 0; l < 64; ++l) {
                    lane_t* L = &lanes[wv][l];
                    const uint32_t x = tx * 16 + (wv & 1) * 8 + (l & 7), y = ty * 16 + (wv >> 1) * 8 + (l >> 3);
                    const float px = (float)x + 0.5f, py = (float)y + 0.5f;
                    for (int a = 0; a < 3; ++a) {
                        L->d[a] = (c->w00[a] + px * c->du[a]) + py * c->dv[a];
                        L->invd[a] = 1.0f / L->d[a];
                    }
                    L->tb = INFINITY; L->hp = 0xFFFFFFFFu; L->sp = 0; L->cur = 0; L->ctn = 0.0f; L->done = 0;
                    L->pix = y * w + x;
                    pend[wv][l] = 0xFFFFFFFFu;
                }
            uint32_t round = 0;
            for (;; ++round) {
                int any = 0;
                for (int wv = 0; wv < 4; ++wv) {
                    if (!wlive[wv]) continue;
                    int act = 0;
                    for (int l = 0; l < 64; ++l) {
                        lane_t* L = &lanes[wv][l];
                        if (!L->done) { act += mlane_gather(L0, L, &pend[wv][l]); }
                        if (L->done && np && (A & 0x10000u) == 0) {  /* refill a finished lane from the pool */
                            hitp[L->pix] = L->hp;
                            --np; *L = pool[np].L; pend[wv][l] = pool[np].pend; L->done = 0;
                            act += mlane_gather(L0, L, &pend[wv][l]);
                        }
                    }
                    if (!act && np && (A & 0x10000u)) {  /* empty-only refill: a whole wave of pool rays */
                        for (int l = 0; l < 64; ++l) {
                            lane_t* L = &lanes[wv][l];
                            hitp[L->pix] = L->hp;
                            if (np) { --np; *L = pool[np].L; pend[wv][l] = pool[np].pend; L->done = 0;
                                      act += mlane_gather(L0, L, &pend[wv][l]); }
                        }
                    }
                    if (!act) {
                        for (int l = 0; l < 64; ++l) hitp[lanes[wv][l].pix] = lanes[wv][l].hp;
                        wlive[wv] = 0;
                        continue;
                    }
                    int others = 0;
                    for (int k = 0; k < 4; ++k) others += (k != wv) && wlive[k];
                    if (round >= S && (uint32_t)act < (A & 0xFFFFu) && others) {  /* donate and exit */
                        for (int l = 0; l < 64; ++l) {
                            lane_t* L = &lanes[wv][l];
                            if (L->done) { hitp[L->pix] = L->hp; continue; }
                            pool[np].L = *L; pool[np].pend = pend[wv][l]; ++np;
                            out[5] += 1;
                            L->done = 1;
                        }
                        wlive[wv] = 0;
                        continue;
                    }
                    int lb = 0, rb = 0;
                    for (int l = 0; l < 64; ++l) {
                        lane_t* L = &lanes[wv][l];
                        if (L->done) continue;
                        mlane_step(nodes, L0, tris, cut, K, c->eye, L, &pend[wv][l], &lb, &rb);
                    }
                    out[0] += 1; out[1] += lb; out[2] += rb;
                    out[3] += 40.0 + 116.0 * lb + 136.0 * rb;
                    any = 1;
                }
                if (!any && np == 0) break;
                if (!any && np) {  /* every wave exited with rays pooled: cannot happen (donation needs a live wave) */
                    out[6] = -1e9;
                    break;
                }
            }
            out[4] += round;
            if (round > out[6]) out[6] = round;
        }
}

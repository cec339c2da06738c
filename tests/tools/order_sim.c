/* order_sim.c -- design experiment (CPU model, not product code): node fetches
 * per ray of §9.7's fixed preorder traversal against a nearest-first stack
 * traversal over the same binary BVH, and how often the nearest-first answer
 * (the smallest (t, leaf index) among "self-consistent" candidates, those
 * whose Moller-Trumbore t is not below their own leaf box's slab entry tn)
 * differs from §9.7's.  Built and driven by tests/tools/order_sim.py. */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../oracle/rt_oracle.h"

#define SENT 0xFFFFFFFFu
#define FMIN orc_fmin
#define FMAX orc_fmax

static void slab(const orc_node* nd, const float* o, const float* invd, float* tn, float* tf) {
    float t0[3], t1[3];
    for (int a = 0; a < 3; ++a) {
        t0[a] = (nd->lo[a] - o[a]) * invd[a];
        t1[a] = (nd->hi[a] - o[a]) * invd[a];
    }
    *tn = FMAX(FMAX(FMAX(FMIN(t0[0], t1[0]), FMIN(t0[1], t1[1])), FMIN(t0[2], t1[2])), 0.0f);
    *tf = FMIN(FMIN(FMAX(t0[0], t1[0]), FMAX(t0[1], t1[1])), FMAX(t0[2], t1[2]));
}

/* §9.7 preorder: returns fetches, writes prim/t */
static uint32_t pre(const orc_node* nodes, uint32_t n, const float* tris, const float* o, const float* d,
                    const float* invd, uint32_t* prim, float* tout) {
    float tb = INFINITY;
    uint32_t hp = SENT, idx = 0, L0 = n - 1, cnt = 0;
    while (idx != SENT) {
        const orc_node* nd = &nodes[idx];
        ++cnt;
        float tn, tf;
        slab(nd, o, invd, &tn, &tf);
        tf = FMIN(tf, tb);
        if (!(tn <= tf)) { idx = nd->esc; continue; }
        if (idx >= L0) {
            float t, u, v;
            if (orc_intersect_tri(o, d, tris + (size_t)nd->a * 9, tb, &t, &u, &v)) { tb = t; hp = nd->a; }
            idx = nd->esc;
        } else idx = nd->a;
    }
    *prim = hp;
    *tout = tb;
    return cnt;
}

/* nearest-first: flags bit0 = a non-self-consistent candidate with (t, k) <=
 * the answer was seen (would need the preorder fallback) */
static uint32_t nf(const orc_node* nodes, uint32_t n, const float* tris, const float* o, const float* d,
                   const float* invd, uint32_t* prim, float* tout, uint32_t* flags, uint32_t* maxsp) {
    uint32_t stk[256];
    float stn[256];
    uint32_t sp = 0, cnt = 0, L0 = n - 1, fl = 0;
    float bt = INFINITY, nsc_t = INFINITY;
    uint32_t bk = SENT, bp = SENT, nsc_k = SENT;
    float rtn, rtf;
    slab(&nodes[0], o, invd, &rtn, &rtf);
    uint32_t cur = (rtn <= rtf) ? 0u : SENT;
    float ctn = rtn;
    *maxsp = 0;
    for (;;) {
        if (cur == SENT) {
            if (!sp) break;
            --sp;
            cur = stk[sp];
            ctn = stn[sp];
        }
        if (ctn > bt) { cur = SENT; continue; }
        const orc_node* nd = &nodes[cur];
        ++cnt;
        if (cur >= L0) {
            float tn, tf, t, u, v;
            slab(nd, o, invd, &tn, &tf);
            const uint32_t k = cur - L0;
            if (tn <= tf && orc_intersect_tri(o, d, tris + (size_t)nd->a * 9, INFINITY, &t, &u, &v)) {
                if (tn <= t) {
                    if (t < bt || (t == bt && k < bk)) { bt = t; bk = k; bp = nd->a; }
                } else if (t < nsc_t || (t == nsc_t && k < nsc_k)) {
                    nsc_t = t; nsc_k = k;
                }
            }
            cur = SENT;
            continue;
        }
        const uint32_t l = nd->a, r = nodes[l].esc;
        float ln, lf, rn, rf;
        slab(&nodes[l], o, invd, &ln, &lf);
        slab(&nodes[r], o, invd, &rn, &rf);
        const int lh = ln <= FMIN(lf, bt), rh = rn <= FMIN(rf, bt);
        if (lh && rh) {
            const int lfirst = ln <= rn;
            stk[sp] = lfirst ? r : l;
            stn[sp] = lfirst ? rn : ln;
            ++sp;
            if (sp > *maxsp) *maxsp = sp;
            cur = lfirst ? l : r;
            ctn = lfirst ? ln : rn;
        } else if (lh) { cur = l; ctn = ln; }
        else if (rh) { cur = r; ctn = rn; }
        else cur = SENT;
    }
    if (nsc_t < bt || (nsc_t == bt && nsc_k < bk)) fl |= 1u;
    *prim = bp;
    *tout = bt;
    *flags = fl;
    return cnt;
}

/* rows [y0, y1) of a w x h x 1 frame */
void osim_trace(const orc_node* nodes, uint32_t n, const float* tris, const orc_camera* c, uint32_t w,
                uint32_t h, uint32_t y0, uint32_t y1, uint16_t* pre_steps, uint16_t* nf_steps, uint8_t* flags,
                uint8_t* stackmax) {
    (void)h;
    for (uint32_t y = y0; y < y1; ++y)
        for (uint32_t x = 0; x < w; ++x) {
            const float px = (float)x + 0.5f, py = (float)y + 0.5f;
            float d[3], invd[3];
            for (int a = 0; a < 3; ++a) {
                d[a] = (c->w00[a] + px * c->du[a]) + py * c->dv[a];
                invd[a] = 1.0f / d[a];
            }
            uint32_t p1, p2, fl, ms;
            float t1, t2;
            const uint64_t i = (uint64_t)y * w + x;
            const uint32_t a = pre(nodes, n, tris, c->eye, d, invd, &p1, &t1);
            const uint32_t b = nf(nodes, n, tris, c->eye, d, invd, &p2, &t2, &fl, &ms);
            pre_steps[i] = (uint16_t)(a > 65535 ? 65535 : a);
            nf_steps[i] = (uint16_t)(b > 65535 ? 65535 : b);
            /* bit1: answers differ although no flag was raised (theory wrong) */
            if (p1 != p2 && !(fl & 1u)) fl |= 2u;
            if (p1 != p2) fl |= 4u;
            flags[i] = (uint8_t)fl;
            stackmax[i] = (uint8_t)(ms > 255 ? 255 : ms);
        }
}

/* VERDICT r04 item 6 (certified nearest-first, the stop rule): per ray, the
 * subtrees the nearest-first pass culls ONLY because their entry tn exceeds
 * the best self-consistent t found so far (tn <= tf: the float slab test
 * passes, so §9.7 -- whose tb can be larger there -- may enter them).  A
 * sound certificate must show that no triangle inside such a subtree has a
 * Moller-Trumbore t below the answer, i.e. bound MT's forward error for every
 * triangle in it; that error grows like 1/|d.n| (the ray nearly in the
 * triangle's plane), so the bound needs the subtree's normal cone, and a cone
 * over more than a few random triangles spans the sphere.  Reported per ray:
 * the number of such subtrees and the largest one's leaf count (range length
 * from rlo/rhi; a leaf counts 1).  nf_hz_count[i], nf_hz_max[i]. */
static uint32_t nf_hazards(const orc_node* nodes, uint32_t n, const float* tris, const float* o, const float* d,
                           const float* invd, const uint32_t* rlo, const uint32_t* rhi, uint32_t* hz_count,
                           uint32_t* hz_max) {
    uint32_t stk[256];
    float stn[256];
    uint32_t sp = 0, cnt = 0, L0 = n - 1, hc = 0, hm = 0;
    float bt = INFINITY;
    float rtn, rtf;
    slab(&nodes[0], o, invd, &rtn, &rtf);
    uint32_t cur = (rtn <= rtf) ? 0u : SENT;
    float ctn = rtn;
#define HZ(node_)                                                                          \
    do {                                                                                   \
        const uint32_t s_ = (node_) >= L0 ? 1u : rhi[(node_)] - rlo[(node_)] + 1u;       \
        ++hc;                                                                              \
        if (s_ > hm) hm = s_;                                                              \
    } while (0)
    for (;;) {
        if (cur == SENT) {
            if (!sp) break;
            --sp;
            cur = stk[sp];
            ctn = stn[sp];
        }
        if (ctn > bt) { HZ(cur); cur = SENT; continue; }  /* popped after bt shrank below its entry */
        const orc_node* nd = &nodes[cur];
        ++cnt;
        if (cur >= L0) {
            float tn, tf, t, u, v;
            slab(nd, o, invd, &tn, &tf);
            if (tn <= tf && orc_intersect_tri(o, d, tris + (size_t)nd->a * 9, INFINITY, &t, &u, &v) && tn <= t &&
                t < bt)
                bt = t;
            cur = SENT;
            continue;
        }
        const uint32_t l = nd->a, r = nodes[l].esc;
        float ln, lf, rn, rf;
        slab(&nodes[l], o, invd, &ln, &lf);
        slab(&nodes[r], o, invd, &rn, &rf);
        const int lg = ln <= lf, rg = rn <= rf;  /* geometric hits (tb-independent) */
        const int lh = lg && ln <= bt, rh = rg && rn <= bt;
        if (lg && !lh) HZ(l);
        if (rg && !rh) HZ(r);
        if (lh && rh) {
            const int lfirst = ln <= rn;
            stk[sp] = lfirst ? r : l;
            stn[sp] = lfirst ? rn : ln;
            ++sp;
            cur = lfirst ? l : r;
            ctn = lfirst ? ln : rn;
        } else if (lh) { cur = l; ctn = ln; }
        else if (rh) { cur = r; ctn = rn; }
        else cur = SENT;
    }
#undef HZ
    *hz_count = hc;
    *hz_max = hm;
    return cnt;
}

void osim_hazards(const orc_node* nodes, uint32_t n, const float* tris, const orc_camera* c, uint32_t w,
                  uint32_t y0, uint32_t y1, const uint32_t* rlo, const uint32_t* rhi, uint16_t* pre_steps,
                  uint32_t* hz_count, uint32_t* hz_max) {
    for (uint32_t y = y0; y < y1; ++y)
        for (uint32_t x = 0; x < w; ++x) {
            const float px = (float)x + 0.5f, py = (float)y + 0.5f;
            float d[3], invd[3];
            for (int a = 0; a < 3; ++a) {
                d[a] = (c->w00[a] + px * c->du[a]) + py * c->dv[a];
                invd[a] = 1.0f / d[a];
            }
            uint32_t p1;
            float t1;
            const uint64_t i = (uint64_t)y * w + x;
            const uint32_t a = pre(nodes, n, tris, c->eye, d, invd, &p1, &t1);
            pre_steps[i] = (uint16_t)(a > 65535 ? 65535 : a);
            nf_hazards(nodes, n, tris, c->eye, d, invd, rlo, rhi, &hz_count[i], &hz_max[i]);
        }
}

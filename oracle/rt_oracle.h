/*
 * rt_oracle.h -- CPU ORACLE for the BVH-build + ray-trace hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load or execute anything under oracle/.
 * The product (gpu_raytracer_amd/, librtamd.so) never links or calls it.
 *
 * Parity status: UNPINNED against upstream SoslanGM/gpu_raytracer.  The
 * mounted reference (/root/reference @ v0) is a stub: README.md:1-2 (title +
 * one sentence) and test.txt:1 ("This is an update") -- no code, no tests, no
 * golden vectors.  This oracle is a scalar restatement of the
 * semantic contract in SURVEY.md §9 (Appendix A), which the survey derived
 * from BASELINE.json:5.  It is pinned by
 *   - the known-answer tests of SURVEY.md §4 / §9.8 (Morton, Karras Fig. 4
 *     topology + escape links, Moller-Trumbore),
 *   - std::stable_sort-equivalence of the radix sort (tests/),
 *   - an independent numpy restatement (oracle/oracle_np.py) that must
 *     reproduce the committed fixtures under tests/golden/ bit-for-bit.
 *
 * Every function cites the SURVEY.md section it follows (the reference has no
 * file:line to cite for code).
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_SENTINEL 0xFFFFFFFFu

typedef struct { float eye[3], w00[3], du[3], dv[3]; } orc_camera;   /* §9.7 */
typedef struct { float t, u, v; uint32_t prim; } orc_hit;            /* §9.1, 16 B */
typedef struct { float lo[3], hi[3]; uint32_t a, esc; } orc_node;    /* §9.1, 32 B */

/* §9.9 scene generators */
uint64_t orc_splitmix64(uint64_t* state);
void orc_soup_generate(uint32_t n, uint64_t seed, float* tris /* n*9 */);

/* §9.7 camera: host double math rounded to float */
void orc_camera_look_at(const double eye[3], const double at[3], const double up[3],
                        double vfov_deg, uint32_t w, uint32_t h, orc_camera* out);

/* §9.2 centroid bounds; inv = (hi>lo) ? 1/(hi-lo) : 0 per axis */
void orc_centroid_bounds(const float* tris, uint32_t n, float lo[3], float hi[3], float inv[3]);

/* §9.3 Morton */
uint32_t orc_expand10(uint32_t v);
uint32_t orc_morton3(uint32_t qx, uint32_t qy, uint32_t qz);
void orc_morton(const float* tris, uint32_t n, const float lo[3], const float inv[3],
                uint32_t* keys, uint32_t* vals);

/* §9.4 stable LSB radix sort, 4 x 8-bit digits, in place (tmp: n words each) */
void orc_radix_sort(uint32_t* keys, uint32_t* vals, uint32_t n, uint32_t* tmpk, uint32_t* tmpv);

/* §9.5 Karras 2012 topology.  left/right/range_lo/range_hi: n-1 entries;
 * parent: 2n-1 entries over the unified index space. */
int orc_delta(const uint32_t* keys, uint32_t n, int64_t i, int64_t j);
void orc_karras(const uint32_t* keys, uint32_t n, uint32_t* left, uint32_t* right,
                uint32_t* range_lo, uint32_t* range_hi, uint32_t* parent);

/* §9.6 escape links by the DEFINITION (walk to the nearest ancestor-or-self
 * that is a left child, take its right sibling).  esc: 2n-1 entries. */
void orc_escape(uint32_t n, const uint32_t* left, const uint32_t* right,
                const uint32_t* parent, uint32_t* esc);

/* §9.6 refit (post-order union of children) + node pack (§9.1). */
void orc_refit_pack(const float* tris, uint32_t n, const uint32_t* sorted_vals,
                    const uint32_t* left, const uint32_t* right, const uint32_t* esc,
                    orc_node* nodes /* 2n-1 */);

/* Whole build: bounds -> morton -> sort -> karras -> escape -> refit/pack.
 * Optional outputs may be NULL.  Returns 0 on success, -2 on OOM. */
typedef struct {
    float lo[3], hi[3], inv[3];
} orc_bounds;
int orc_build(const float* tris, uint32_t n, orc_node* nodes /* 2n-1 (n>=1) */,
              uint32_t* sorted_keys, uint32_t* sorted_vals, uint32_t* parent,
              orc_bounds* bounds_out);

/* §9.7 helpers exposed for KATs */
uint32_t orc_pcg_hash(uint32_t x);
float orc_fmin(float a, float b);
float orc_fmax(float a, float b);
int orc_intersect_tri(const float o[3], const float d[3], const float* tri,
                      float t_best, float* t, float* u, float* v);

/* §9.7 trace: hits[(y*w+x)*spp+s]; counters (nullable): [0]=nodes fetched,
 * [1]=tris tested, summed over all traced rays.  Rows traced: y = row0,
 * row0+row_step, ... (row_step>=1) -- lets the CPU baseline time a bounded
 * sample.  nthreads>=1: 64-pixel row segments dealt to the calling thread
 * and nthreads-1 POSIX threads from a shared cursor. */
void orc_trace(const orc_node* nodes, uint32_t n, const float* tris, const orc_camera* cam,
               uint32_t w, uint32_t h, uint32_t spp, uint32_t row0, uint32_t row_step,
               orc_hit* hits, uint64_t counters[2], int nthreads);

/* §9.7 shading: rgba[(y*w+x)*4] from hits of that pixel's spp samples. */
void orc_shade(const orc_hit* hits, uint32_t w, uint32_t h, uint32_t spp, uint8_t* rgba);

/* Shadow mode [SPEC, DESIGN.md "Shadow mode"; SURVEY.md §8(f) row 3]: the
 * §9.7 primary hits, then one any-hit shadow ray per hit toward the point
 * light; rgba = Lambert-lit (u, v, 1-u-v) with an ambient floor.  counters
 * (nullable): shadow-ray nodes fetched / tris tested. */
void orc_render_shadow(const orc_node* nodes, uint32_t n, const float* tris, const orc_camera* cam,
                       uint32_t w, uint32_t h, uint32_t spp, const float light[3], float ambient,
                       orc_hit* hits, uint8_t* rgba, uint64_t counters[2], int nthreads);

/* Path mode [SPEC, DESIGN.md "Path mode"; SURVEY.md §8(f) row 3]: diffuse
 * paths of 1 + max_depth segments with next-event estimation toward the point
 * light and sky radiance `sky` for escaped bounce rays.  hits (nullable): the
 * primary hits.  counters (nullable): [0] nodes fetched, [1] tris tested,
 * [2] rays traced (primary + bounce + shadow).  Rows interleaved over
 * nthreads POSIX threads. */
void orc_render_path(const orc_node* nodes, uint32_t n, const float* tris, const orc_camera* cam,
                     uint32_t w, uint32_t h, uint32_t spp, const float light[3], float sky, uint32_t max_depth,
                     orc_hit* hits, uint8_t* rgba, uint64_t counters[3], int nthreads);

/* Test hook: on != 0 makes every worker-thread creation fail, so the CPU
 * suite checks that the traces still cover every pixel on the calling
 * thread (tests/test_oracle.py). */
void orc_debug_fail_spawn(int on);

#ifdef __cplusplus
}
#endif
#endif

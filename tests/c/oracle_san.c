/* oracle_san.c -- the CPU oracle (oracle/rt_oracle.c, TEST INFRASTRUCTURE)
 * under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5
 * "sanitizers"; `make -C tests/c sanitize`; run by tests/test_sanitizers.py).
 * Drives every oracle function over small and degenerate inputs -- n = 1, 2,
 * identical triangles, a flat scene, a 3000-triangle soup -- through build,
 * trace (1 and 3 threads), shade, shadow and path modes.  The sanitizers abort
 * on the first error; exit 0 = clean. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/rt_oracle.h"

static void frame(const float* tris, uint32_t n, uint32_t w, uint32_t h, uint32_t spp) {
    orc_node* nodes = (orc_node*)malloc((size_t)(2 * n - 1) * sizeof(orc_node));
    uint32_t* keys = (uint32_t*)malloc((size_t)n * 4);
    uint32_t* vals = (uint32_t*)malloc((size_t)n * 4);
    uint32_t* parent = (uint32_t*)malloc((size_t)(2 * n - 1) * 4);
    orc_bounds b;
    if (orc_build(tris, n, nodes, keys, vals, parent, &b) != 0) { fprintf(stderr, "build failed\n"); exit(1); }
    const double eye[3] = {0.5, 0.5, -1.5}, at[3] = {0.5, 0.5, 0.5}, up[3] = {0, 1, 0};
    orc_camera cam;
    orc_camera_look_at(eye, at, up, 45.0, w, h, &cam);
    const size_t nh = (size_t)w * h * spp;
    orc_hit* hits = (orc_hit*)malloc(nh * sizeof(orc_hit));
    orc_hit* hits3 = (orc_hit*)malloc(nh * sizeof(orc_hit));
    uint8_t* rgba = (uint8_t*)malloc((size_t)w * h * 4);
    uint64_t c1[2] = {0, 0}, c3[2] = {0, 0}, c[3] = {0, 0, 0};
    orc_trace(nodes, n, tris, &cam, w, h, spp, 0, 1, hits, c1, 1);
    orc_trace(nodes, n, tris, &cam, w, h, spp, 0, 1, hits3, c3, 3);
    if (memcmp(hits, hits3, nh * sizeof(orc_hit)) != 0 || c1[0] != c3[0] || c1[1] != c3[1]) {
        fprintf(stderr, "threaded trace differs\n");
        exit(1);
    }
    orc_shade(hits, w, h, spp, rgba);
    const float light[3] = {2.0f, 3.0f, -2.0f};
    orc_render_shadow(nodes, n, tris, &cam, w, h, spp, light, 0.2f, hits, rgba, c, 2);
    orc_render_path(nodes, n, tris, &cam, w, h, spp, light, 0.3f, 3, hits, rgba, c, 2);
    free(nodes); free(keys); free(vals); free(parent); free(hits); free(hits3); free(rgba);
}

int main(void) {
    /* KATs of the small helpers */
    if (orc_morton3(1023, 1023, 1023) != 0x3FFFFFFFu) { fprintf(stderr, "morton KAT\n"); return 1; }
    const float o[3] = {0.25f, 0.25f, -1.0f}, d[3] = {0, 0, 1}, tri[9] = {0, 0, 0, 1, 0, 0, 0, 1, 0};
    float t, u, v;
    if (!orc_intersect_tri(o, d, tri, 1e30f, &t, &u, &v) || t != 1.0f) { fprintf(stderr, "MT KAT\n"); return 1; }
    (void)orc_fmin(-0.0f, 0.0f);
    (void)orc_pcg_hash(12345u);

    const uint32_t n = 3000;
    float* soup = (float*)malloc((size_t)n * 9 * sizeof(float));
    orc_soup_generate(n, 3, soup);
    frame(soup, n, 48, 32, 2);
    frame(soup, 1, 17, 9, 1);
    frame(soup, 2, 16, 16, 1);
    /* identical triangles (all keys equal) and a flat scene (zero extent axis) */
    float* same = (float*)malloc(64 * 9 * sizeof(float));
    for (int i = 0; i < 64; ++i) memcpy(same + 9 * i, soup, 9 * sizeof(float));
    frame(same, 64, 24, 24, 1);
    for (int i = 0; i < 64; ++i) same[9 * i + 2] = same[9 * i + 5] = same[9 * i + 8] = 0.5f;
    frame(same, 64, 24, 24, 1);
    /* the radix sort alone, adversarial keys */
    uint32_t keys[1000], vals[1000], tk[1000], tv[1000];
    for (uint32_t i = 0; i < 1000; ++i) { keys[i] = (i * 2654435761u) & 0x3FFFFFFFu; vals[i] = i; }
    orc_radix_sort(keys, vals, 1000, tk, tv);
    for (uint32_t i = 1; i < 1000; ++i)
        if (keys[i - 1] > keys[i]) { fprintf(stderr, "sort order\n"); return 1; }
    free(soup);
    free(same);
    printf("oracle_san OK\n");
    return 0;
}

/* rt_host.c -- a plain C host of librtamd, the binding INTEGRATION.md shows:
 * ingest -> rt_bvh_build -> rt_render -> dumps, through the C-ABI only
 * (include/gpu_raytracer_amd.h).  Built by __graft_entry__.build() /
 * `make -C tests/c`; run by tests/test_c_host_gpu.py, which compares its
 * outputs with the CPU oracle byte for byte.
 *
 * usage: rt_host <n_tris> <seed> <w> <h> <spp> <ngpus> <out.rgba> <out.hits>
 * Renders the SURVEY.md §9.9 soup from the §8(d) soup-1M camera; writes the
 * raw w*h*4 RGBA bytes and the w*h*spp 16-B hit records.  Exit status: 0 ok,
 * 2 usage, 3 library error (message on stderr, status code on stdout). */
#include <stdio.h>
#include <stdlib.h>

#include "../../include/gpu_raytracer_amd.h"

static int die(const char* what, rt_status st) {
    printf("%d\n", (int)st);
    fprintf(stderr, "%s: status %d: %s\n", what, (int)st, rt_last_error());
    return 3;
}

int main(int argc, char** argv) {
    if (argc != 9) {
        fprintf(stderr, "usage: %s n seed w h spp ngpus out.rgba out.hits\n", argv[0]);
        return 2;
    }
    const uint32_t n = (uint32_t)strtoul(argv[1], NULL, 10);
    const uint64_t seed = strtoull(argv[2], NULL, 10);
    const uint32_t w = (uint32_t)strtoul(argv[3], NULL, 10), h = (uint32_t)strtoul(argv[4], NULL, 10);
    const uint32_t spp = (uint32_t)strtoul(argv[5], NULL, 10), ngpus = (uint32_t)strtoul(argv[6], NULL, 10);
    rt_scene* s = NULL;
    rt_status st = rt_scene_generate_soup(n, seed, &s);
    if (st != RT_OK) return die("rt_scene_generate_soup", st);
    double ms = 0.0;
    if ((st = rt_bvh_build(s, RT_BACKEND_HIP, 0u, &ms)) != RT_OK) return die("rt_bvh_build", st);
    const double eye[3] = {0.5, 0.5, -1.5}, at[3] = {0.5, 0.5, 0.5}, up[3] = {0.0, 1.0, 0.0};
    rt_camera cam;
    if ((st = rt_camera_look_at(eye, at, up, 45.0, w, h, &cam)) != RT_OK) return die("rt_camera_look_at", st);
    uint8_t* rgba = (uint8_t*)malloc((size_t)w * h * 4);
    rt_hit* hits = (rt_hit*)malloc((size_t)w * h * spp * sizeof(rt_hit));
    if (!rgba || !hits) return 3;
    /* SURVEY.md §8(b)'s rt_render; rt_render_timed (NULL outputs) then times the same frame */
    if ((st = rt_render(s, &cam, w, h, spp, ngpus, hits, rgba)) != RT_OK) return die("rt_render", st);
    double frame_ms = 0.0;
    if ((st = rt_render_timed(s, &cam, w, h, spp, ngpus, NULL, NULL, &frame_ms)) != RT_OK)
        return die("rt_render_timed", st);
    FILE* f = fopen(argv[7], "wb");
    if (!f || fwrite(rgba, 1, (size_t)w * h * 4, f) != (size_t)w * h * 4) return 3;
    fclose(f);
    if ((st = rt_hits_dump(hits, (size_t)w * h * spp, argv[8])) != RT_OK) return die("rt_hits_dump", st);
    printf("0\nbuild %.4f ms, frame %.4f ms\n", ms, frame_ms);
    free(rgba);
    free(hits);
    rt_scene_free(s);
    return 0;
}

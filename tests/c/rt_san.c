/* rt_san.c -- host-side exercise of librtamd built with AddressSanitizer +
 * UndefinedBehaviorSanitizer on its HOST code (SURVEY.md §5 "sanitizers";
 * `make -C tests/c sanitize`; run by tests/test_sanitizers.py on the CPU).
 *
 * Covers every entry point that does host work before (or instead of) device
 * work: scene ingest (soup, generator, OBJ with continuations / fans /
 * negative indices / CRLF / malformed lines, RTSOUP1 save/load and corrupt
 * files), camera, config knobs, dumps, argument validation, and -- without a
 * GPU -- the RT_EDEVICE refusals of every compute entry point (no CPU
 * fallback).  Exit status 0 = every expectation held; the sanitizers abort
 * the process on the first memory / UB error.
 *
 * usage: rt_san <scratch dir> */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/gpu_raytracer_amd.h"

static int g_fail = 0;
#define EXPECT(cond)                                                               \
    do {                                                                           \
        if (!(cond)) {                                                             \
            fprintf(stderr, "%s:%d: expectation failed: %s (%s)\n", __FILE__, __LINE__, #cond, \
                    rt_last_error());                                              \
            g_fail = 1;                                                            \
        }                                                                          \
    } while (0)

static char g_dir[512];
static const char* path_of(const char* name) {
    static char buf[1024];
    snprintf(buf, sizeof(buf), "%s/%s", g_dir, name);
    return buf;
}

static void write_file(const char* name, const char* text, size_t len) {
    FILE* f = fopen(path_of(name), "wb");
    if (!f) { perror("fopen"); exit(2); }
    fwrite(text, 1, len, f);
    fclose(f);
}

static uint32_t obj_tris(const char* name, const char* text, rt_status* st_out) {
    write_file(name, text, strlen(text));
    rt_scene* s = NULL;
    rt_status st = rt_scene_load_obj(path_of(name), &s);
    if (st_out) *st_out = st;
    uint32_t n = 0xFFFFFFFFu;
    if (st == RT_OK) {
        EXPECT(rt_scene_num_tris(s, &n) == RT_OK);
        if (n) {
            float* t = (float*)malloc((size_t)n * 9 * sizeof(float));
            EXPECT(rt_scene_get_tris(s, t) == RT_OK);
            free(t);
        }
        rt_scene_free(s);
    }
    return n;
}

static void test_obj(void) {
    rt_status st;
    EXPECT(obj_tris("quad.obj", "v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nf 1 2 3 4\n", &st) == 2);
    EXPECT(obj_tris("neg.obj", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf -3 -2 -1\n", &st) == 1);
    EXPECT(obj_tris("crlf.obj", "v 0 0 0\r\nv 1 0 0\r\nv 0 1 0\r\nf 1/1/1 2/2/2 3//3\r\n", &st) == 1);
    EXPECT(obj_tris("cont.obj", "# c\nv 0 0 \\\n 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\nvt 0 0\ng x\ns off\nf 1 \\\n2 3\n", &st) == 1);
    /* a 5-gon fan and a very long line (> any fixed buffer) */
    {
        size_t cap = 200000, len = 0;
        char* big = (char*)malloc(cap);
        len += (size_t)snprintf(big + len, cap - len, "v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nv 0 2 0\n# ");
        while (len < cap - 64) big[len++] = 'x';
        len += (size_t)snprintf(big + len, cap - len, "\nf 1 2 3 4 5\n");
        EXPECT(obj_tris("fan.obj", big, &st) == 3);
        free(big);
    }
    /* malformed: index out of range, zero index, too few vertices, garbage */
    obj_tris("bad1.obj", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 9\n", &st);
    EXPECT(st == RT_EINVAL || st == RT_EIO);
    obj_tris("bad2.obj", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 0 1 2\n", &st);
    EXPECT(st == RT_EINVAL || st == RT_EIO);
    obj_tris("bad3.obj", "v 0 0 0\nv 1 0 0\nf 1 2\n", &st);
    EXPECT(st == RT_EINVAL || st == RT_EIO);
    obj_tris("bad4.obj", "v 0 zero 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n", &st);
    EXPECT(st == RT_EINVAL || st == RT_EIO);
    obj_tris("bad5.obj", "f -7 1 2\n", &st);
    EXPECT(st == RT_EINVAL || st == RT_EIO);
    EXPECT(obj_tris("empty.obj", "", &st) == 0 || st != RT_OK);
    rt_scene* s = NULL;
    EXPECT(rt_scene_load_obj(path_of("does_not_exist.obj"), &s) == RT_EIO);
    EXPECT(s == NULL);
}

static void test_soup_io(void) {
    rt_scene* s = NULL;
    EXPECT(rt_scene_generate_soup(1000, 7, &s) == RT_OK);
    uint32_t n = 0;
    EXPECT(rt_scene_num_tris(s, &n) == RT_OK && n == 1000);
    float* a = (float*)malloc(9000 * sizeof(float));
    float* b = (float*)malloc(9000 * sizeof(float));
    EXPECT(rt_scene_get_tris(s, a) == RT_OK);
    EXPECT(rt_scene_save_soup(s, path_of("s.rtsoup")) == RT_OK);
    rt_scene_free(s);
    s = NULL;
    EXPECT(rt_scene_load_soup(path_of("s.rtsoup"), &s) == RT_OK);
    EXPECT(rt_scene_get_tris(s, b) == RT_OK);
    EXPECT(memcmp(a, b, 9000 * sizeof(float)) == 0);
    rt_scene_free(s);
    /* from_soup copies; the caller's buffer may go away */
    s = NULL;
    EXPECT(rt_scene_from_soup(a, 1000, &s) == RT_OK);
    memset(a, 0, 9000 * sizeof(float));
    EXPECT(rt_scene_get_tris(s, a) == RT_OK && memcmp(a, b, 9000 * sizeof(float)) == 0);
    rt_scene_free(s);
    /* truncated and foreign files */
    FILE* f = fopen(path_of("s.rtsoup"), "rb");
    char head[64];
    size_t got = fread(head, 1, sizeof(head), f);
    fclose(f);
    write_file("trunc.rtsoup", head, got);
    s = NULL;
    EXPECT(rt_scene_load_soup(path_of("trunc.rtsoup"), &s) == RT_EIO && s == NULL);
    write_file("foreign.rtsoup", "NOTASOUP\0\0\0\0\0\0\0\0", 16);
    EXPECT(rt_scene_load_soup(path_of("foreign.rtsoup"), &s) == RT_EIO && s == NULL);
    free(a);
    free(b);
    /* empty scenes and argument checks */
    s = NULL;
    EXPECT(rt_scene_from_soup(NULL, 0, &s) == RT_OK || s == NULL);
    rt_scene_free(s);
    EXPECT(rt_scene_from_soup(NULL, 5, &s) == RT_EINVAL);
    EXPECT(rt_scene_num_tris(NULL, &n) == RT_EINVAL);
    rt_scene_free(NULL);
}

static void test_camera_config_dumps(void) {
    const double eye[3] = {0.5, 0.5, -1.5}, at[3] = {0.5, 0.5, 0.5}, up[3] = {0, 1, 0};
    rt_camera cam;
    EXPECT(rt_camera_look_at(eye, at, up, 45.0, 64, 48, &cam) == RT_OK);
    EXPECT(isfinite(cam.w00[0]) && isfinite(cam.du[0]) && isfinite(cam.dv[1]));
    EXPECT(rt_camera_look_at(eye, eye, up, 45.0, 64, 48, &cam) == RT_EINVAL);  /* degenerate */
    EXPECT(rt_camera_look_at(eye, at, up, 45.0, 0, 48, &cam) == RT_EINVAL);
    EXPECT(rt_config_set("trace.variant", 2) == RT_OK);
    EXPECT(rt_config_set("trace.variant", 0) == RT_OK);
    EXPECT(rt_config_set("trace.variant", 99) == RT_EINVAL);
    EXPECT(rt_config_set("no.such.knob", 1) == RT_EINVAL);
    EXPECT(rt_config_set(NULL, 1) == RT_EINVAL);
    uint8_t rgba[16 * 8 * 4];
    for (size_t i = 0; i < sizeof(rgba); ++i) rgba[i] = (uint8_t)i;
    EXPECT(rt_framebuffer_dump_ppm(rgba, 16, 8, path_of("f.ppm")) == RT_OK);
    EXPECT(rt_framebuffer_dump_ppm(rgba, 16, 8, path_of("no_dir/f.ppm")) == RT_EIO);
    rt_hit hits[7];
    for (int i = 0; i < 7; ++i) { hits[i].t = (float)i; hits[i].u = hits[i].v = 0.25f; hits[i].prim = (uint32_t)i; }
    EXPECT(rt_hits_dump(hits, 7, path_of("h.bin")) == RT_OK);
    EXPECT(rt_tiles_for_rank(1920, 1080, 0, 8) + rt_tiles_for_rank(1920, 1080, 7, 8) > 0);
    EXPECT(rt_version() != NULL && rt_last_error() != NULL);
}

/* no GPU: every compute entry point refuses with RT_EDEVICE, none falls back */
static void test_no_device(void) {
    if (rt_device_count() > 0) return;
    rt_scene* s = NULL;
    EXPECT(rt_scene_generate_soup(300, 1, &s) == RT_OK);
    double ms = 0;
    EXPECT(rt_bvh_build(s, RT_BACKEND_CPU, 0, &ms) == RT_EINVAL);
    EXPECT(rt_bvh_build(s, RT_BACKEND_HIP, 0, &ms) == RT_EDEVICE);
    const double eye[3] = {0.5, 0.5, -1.5}, at[3] = {0.5, 0.5, 0.5}, up[3] = {0, 1, 0};
    rt_camera cam;
    EXPECT(rt_camera_look_at(eye, at, up, 45.0, 32, 32, &cam) == RT_OK);
    rt_hit* hits = (rt_hit*)malloc(32 * 32 * sizeof(rt_hit));
    uint8_t* rgba = (uint8_t*)malloc(32 * 32 * 4);
    EXPECT(rt_render(s, &cam, 32, 32, 1, 1, hits, rgba) != RT_OK);
    EXPECT(rt_render_timed(s, &cam, 32, 32, 1, 1, hits, rgba, &ms) != RT_OK);
    EXPECT(rt_render_timed(s, &cam, 32, 32, 1, 4, hits, rgba, &ms) != RT_OK);
    EXPECT(rt_bvh_save(s, path_of("x.rtbvh")) != RT_OK);
    EXPECT(rt_bvh_load(s, path_of("x.rtbvh")) != RT_OK);
    float b9[9];
    float tris[9] = {0, 0, 0, 1, 0, 0, 0, 1, 0};
    EXPECT(rt_stage_bounds(0, tris, 1, b9) == RT_EDEVICE);
    free(hits);
    free(rgba);
    rt_scene_free(s);
}

int main(int argc, char** argv) {
    if (argc != 2) {
        fprintf(stderr, "usage: %s scratch_dir\n", argv[0]);
        return 2;
    }
    snprintf(g_dir, sizeof(g_dir), "%s", argv[1]);
    test_obj();
    test_soup_io();
    test_camera_config_dumps();
    test_no_device();
    if (g_fail) return 1;
    printf("rt_san OK\n");
    return 0;
}

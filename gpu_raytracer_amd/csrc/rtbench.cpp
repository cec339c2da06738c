// rtbench -- the C++ command-line driver of SURVEY.md §1.2 L6 / §3(i):
//
//   rtbench --scene soup --n 1000000 --res 1920x1080 --spp 1 --gpus 1
//
// Everything goes through the C-ABI (include/gpu_raytracer_amd.h), exactly as
// a reference-side host would: scene ingest (synthetic soup, the §9.9
// substitutes, an OBJ or an RTSOUP1 file), rt_bvh_build, `frames` renders
// with rt_render (ngpus > 1: the in-library multi-GPU path of §3(iii) --
// replicas, tile deal, RCCL gather), optional framebuffer/hit dumps.  One
// JSON line on stdout: the scene, the build time and Mprims/s, the median
// and best event-timed frame and Mrays/s.  Errors: one JSON line with the
// rt_status and rt_last_error(), exit code 1.
//
// Scenes: soup (rt_scene_generate_soup, splitmix64), cornell,
// bunny, sponza (the §9.9 generators, restated here in C++ double math like
// gpu_raytracer_amd/scenes.py), obj:PATH, rtsoup:PATH.  --config 1..5 selects
// a BASELINE.json config's scene, resolution and spp.  --orbit DEG turns the
// camera about the vertical axis through the look-at point per frame (the
// bench's moving camera, 0.25 deg).
#include "gpu_raytracer_amd.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

struct View {
    double eye[3], at[3], up[3], vfov;
};

// scenes.py: CORNELL_VIEW, SOUP_VIEW, BUNNY_VIEW, SPONZA_VIEW
const View kCornellView{{278.0, 273.0, -800.0}, {278.0, 273.0, 0.0}, {0.0, 1.0, 0.0}, 39.3077};
const View kSoupView{{0.5, 0.5, -1.5}, {0.5, 0.5, 0.5}, {0.0, 1.0, 0.0}, 45.0};
const View kBunnyView{{0.0, 0.3, -3.2}, {0.0, 0.0, 0.0}, {0.0, 1.0, 0.0}, 45.0};
const View kSponzaView{{128.0, 22.0, -24.0}, {128.0, 8.0, 300.0}, {0.0, 1.0, 0.0}, 60.0};

using Tris = std::vector<float>;

void push_tri(Tris& t, const double* a, const double* b, const double* c) {
    for (const double* v : {a, b, c})
        for (int k = 0; k < 3; ++k) t.push_back((float)v[k]);
}
void push_quad(Tris& t, const double* a, const double* b, const double* c, const double* d) {
    push_tri(t, a, b, c);
    push_tri(t, a, c, d);
}

// scenes.py cornell_tris: 5 walls + light + 2 blocks, 2 triangles per quad
Tris cornell() {
    const double X = 556.0, Y = 548.8, Z = 559.2;
    Tris t;
    auto q = [&](std::initializer_list<double> a, std::initializer_list<double> b, std::initializer_list<double> c,
                 std::initializer_list<double> d) { push_quad(t, a.begin(), b.begin(), c.begin(), d.begin()); };
    q({0, 0, 0}, {X, 0, 0}, {X, 0, Z}, {0, 0, Z});
    q({0, Y, 0}, {0, Y, Z}, {X, Y, Z}, {X, Y, 0});
    q({0, 0, Z}, {X, 0, Z}, {X, Y, Z}, {0, Y, Z});
    q({X, 0, 0}, {X, Y, 0}, {X, Y, Z}, {X, 0, Z});
    q({0, 0, 0}, {0, 0, Z}, {0, Y, Z}, {0, Y, 0});
    q({213, Y - 0.1, 227}, {343, Y - 0.1, 227}, {343, Y - 0.1, 332}, {213, Y - 0.1, 332});
    auto block = [&](double x0, double x1, double z0, double z1, double h) {
        q({x0, h, z0}, {x1, h, z0}, {x1, h, z1}, {x0, h, z1});
        q({x0, 0, z0}, {x1, 0, z0}, {x1, h, z0}, {x0, h, z0});
        q({x1, 0, z0}, {x1, 0, z1}, {x1, h, z1}, {x1, h, z0});
        q({x0, 0, z1}, {x0, 0, z0}, {x0, h, z0}, {x0, h, z1});
        q({x1, 0, z1}, {x0, 0, z1}, {x0, h, z1}, {x1, h, z1});
    };
    block(82.0, 240.0, 65.0, 225.0, 165.0);
    block(265.0, 430.0, 272.0, 440.0, 330.0);
    return t;
}

// scenes.py bunny_substitute_tris: closed lat-long sphere, 2*M*(L-1) tris,
// radius 1 + 0.1*sin(5 theta)*cos(7 phi)
Tris bunny(int M = 200, int L = 176) {
    const double pi = 3.14159265358979323846;
    std::vector<double> ring((size_t)(L - 1) * M * 3);
    for (int i = 0; i < L - 1; ++i) {
        const double th = pi * (i + 1) / L;
        for (int j = 0; j < M; ++j) {
            const double ph = 2.0 * pi * j / M;
            const double r = 1.0 + 0.1 * std::sin(5.0 * th) * std::cos(7.0 * ph);
            double* v = &ring[((size_t)i * M + j) * 3];
            v[0] = r * std::sin(th) * std::cos(ph);
            v[1] = r * std::cos(th);
            v[2] = r * std::sin(th) * std::sin(ph);
        }
    }
    auto R = [&](int i, int j) { return &ring[((size_t)i * M + j) * 3]; };
    const double top[3] = {0.0, 1.0, 0.0}, bot[3] = {0.0, -1.0, 0.0};
    Tris t;
    t.reserve((size_t)2 * M * (L - 1) * 9);
    for (int j = 0; j < M; ++j) push_tri(t, top, R(0, (j + 1) % M), R(0, j));
    for (int i = 0; i < L - 2; ++i) {
        for (int j = 0; j < M; ++j) push_tri(t, R(i, j), R(i, (j + 1) % M), R(i + 1, (j + 1) % M));
        for (int j = 0; j < M; ++j) push_tri(t, R(i, j), R(i + 1, (j + 1) % M), R(i + 1, j));
    }
    for (int j = 0; j < M; ++j) push_tri(t, bot, R(L - 2, j), R(L - 2, (j + 1) % M));
    return t;
}

// scenes.py sponza_substitute_tris: heightfield "canyon" of nx*nz quads
Tris sponza(int nx = 256, int nz = 512) {
    auto V = [&](int i, int k, double* v) {
        const double x = i, z = k;
        const double a = std::min(std::max(std::fabs(x - nx / 2.0) / (nx / 2.0), 0.0), 1.0);
        const double wall = 60.0 * std::pow(a, 4.0);
        const double ripple = 2.0 * std::sin(0.11 * z) * std::cos(0.17 * x) + 1.5 * std::sin(0.031 * z + 0.05 * x);
        v[0] = x;
        v[1] = wall + ripple;
        v[2] = z;
    };
    Tris t((size_t)2 * nx * nz * 9);
    const size_t half = (size_t)nx * nz;
    for (int i = 0; i < nx; ++i)
        for (int k = 0; k < nz; ++k) {
            double a[3], b[3], c[3], d[3];
            V(i, k, a);
            V(i + 1, k, b);
            V(i + 1, k + 1, c);
            V(i, k + 1, d);
            const size_t q = (size_t)i * nz + k;
            const double* first[3] = {a, b, c};
            const double* second[3] = {a, c, d};
            for (int v = 0; v < 3; ++v)
                for (int e = 0; e < 3; ++e) {
                    t[q * 9 + v * 3 + e] = (float)first[v][e];
                    t[(half + q) * 9 + v * 3 + e] = (float)second[v][e];
                }
        }
    return t;
}

struct Args {
    std::string scene = "soup", mode = "primary", dump, hits, save_soup;
    uint32_t n = 1000000, w = 1920, h = 1080, spp = 1, gpus = 1, frames = 10, warmup = 2, depth = 2, builds = 5;
    uint64_t seed = 1;
    double orbit = 0.0, sky = 0.3;
    std::vector<std::pair<std::string, long long>> sets;
};

[[noreturn]] void usage(int code) {
    std::fprintf(code ? stderr : stdout,
                 "usage: rtbench [--config 1..5] [--scene soup|cornell|bunny|sponza|obj:PATH|rtsoup:PATH]\n"
                 "               [--n N] [--seed S] [--res WxH] [--spp S] [--gpus P] [--frames K] [--warmup W]\n"
                 "               [--builds B]\n"
                 "               [--orbit DEG] [--mode primary|shadow|path] [--depth D] [--sky F]\n"
                 "               [--set key=value]... [--dump out.ppm] [--hits out.bin] [--save-soup out.rtsoup]\n");
    std::exit(code);
}

int fail(rt_status st, const char* what) {
    std::string msg = rt_last_error() ? rt_last_error() : "";
    for (char& c : msg)
        if (c == '"' || c == '\\' || c < 32) c = ' ';
    std::printf("{\"tool\": \"rtbench\", \"status\": \"error\", \"code\": %d, \"call\": \"%s\", \"message\": \"%s\"}\n",
                (int)st, what, msg.c_str());
    return 1;
}

#define RT_OR_FAIL(call)                          \
    do {                                          \
        const rt_status st_ = (call);             \
        if (st_ != RT_OK) return fail(st_, #call); \
    } while (0)

const View& view_for(const std::string& scene) {
    if (scene == "cornell") return kCornellView;
    if (scene == "bunny") return kBunnyView;
    if (scene == "sponza") return kSponzaView;
    return kSoupView;
}

// scenes.py LIGHTS
void light_for(const std::string& scene, float* l) {
    const float c[3] = {278.0f, 540.0f, 279.5f}, s[3] = {2.0f, 3.0f, -2.0f}, b[3] = {2.0f, 3.0f, -3.0f},
                p[3] = {128.0f, 120.0f, 150.0f};
    const float* src = scene == "cornell" ? c : scene == "bunny" ? b : scene == "sponza" ? p : s;
    std::memcpy(l, src, 3 * sizeof(float));
}

}  // namespace

int main(int argc, char** argv) {
    Args a;
    for (int i = 1; i < argc; ++i) {
        const std::string k = argv[i];
        auto val = [&]() -> std::string {
            if (i + 1 >= argc) usage(2);
            return argv[++i];
        };
        if (k == "-h" || k == "--help") usage(0);
        else if (k == "--config") {
            const int c = std::atoi(val().c_str());
            // BASELINE.json configs (scenes.py CONFIGS)
            switch (c) {
                case 1: a.scene = "cornell"; a.w = 256; a.h = 256; a.spp = 1; break;
                case 2: a.scene = "bunny"; a.w = 1920; a.h = 1080; a.spp = 1; break;
                case 3: a.scene = "soup"; a.n = 1000000; a.w = 1920; a.h = 1080; a.spp = 1; break;
                case 4: a.scene = "sponza"; a.w = 1920; a.h = 1080; a.spp = 16; break;
                case 5: a.scene = "soup"; a.n = 10000000; a.w = 3840; a.h = 2160; a.spp = 4; break;
                default: usage(2);
            }
        } else if (k == "--scene") a.scene = val();
        else if (k == "--n") a.n = (uint32_t)std::strtoul(val().c_str(), nullptr, 10);
        else if (k == "--seed") a.seed = std::strtoull(val().c_str(), nullptr, 10);
        else if (k == "--res") {
            const std::string r = val();
            if (std::sscanf(r.c_str(), "%ux%u", &a.w, &a.h) != 2) usage(2);
        } else if (k == "--spp") a.spp = (uint32_t)std::atoi(val().c_str());
        else if (k == "--gpus") a.gpus = (uint32_t)std::atoi(val().c_str());
        else if (k == "--frames") a.frames = (uint32_t)std::atoi(val().c_str());
        else if (k == "--warmup") a.warmup = (uint32_t)std::atoi(val().c_str());
        else if (k == "--builds") a.builds = (uint32_t)std::atoi(val().c_str());
        else if (k == "--orbit") a.orbit = std::atof(val().c_str());
        else if (k == "--mode") a.mode = val();
        else if (k == "--depth") a.depth = (uint32_t)std::atoi(val().c_str());
        else if (k == "--sky") a.sky = std::atof(val().c_str());
        else if (k == "--dump") a.dump = val();
        else if (k == "--hits") a.hits = val();
        else if (k == "--save-soup") a.save_soup = val();
        else if (k == "--set") {
            const std::string kv = val();
            const size_t eq = kv.find('=');
            if (eq == std::string::npos) usage(2);
            a.sets.emplace_back(kv.substr(0, eq), std::atoll(kv.c_str() + eq + 1));
        } else usage(2);
    }
    if (a.mode != "primary" && a.mode != "shadow" && a.mode != "path") usage(2);
    if (!a.frames) a.frames = 1;

    for (const auto& kv : a.sets) RT_OR_FAIL(rt_config_set(kv.first.c_str(), kv.second));

    // ---- scene
    rt_scene* s = nullptr;
    std::string base = a.scene;
    if (a.scene == "soup") {
        RT_OR_FAIL(rt_scene_generate_soup(a.n, a.seed, &s));
    } else if (a.scene.rfind("obj:", 0) == 0) {
        RT_OR_FAIL(rt_scene_load_obj(a.scene.c_str() + 4, &s));
        base = "obj";
    } else if (a.scene.rfind("rtsoup:", 0) == 0) {
        RT_OR_FAIL(rt_scene_load_soup(a.scene.c_str() + 7, &s));
        base = "rtsoup";
    } else if (a.scene == "cornell" || a.scene == "bunny" || a.scene == "sponza") {
        const Tris t = a.scene == "cornell" ? cornell() : a.scene == "bunny" ? bunny() : sponza();
        RT_OR_FAIL(rt_scene_from_soup(t.data(), (uint32_t)(t.size() / 9), &s));
    } else {
        usage(2);
    }
    uint32_t n = 0;
    RT_OR_FAIL(rt_scene_num_tris(s, &n));
    if (!a.save_soup.empty()) RT_OR_FAIL(rt_scene_save_soup(s, a.save_soup.c_str()));

    // ---- build (the frame's BVH; H2D upload outside the timed region): the
    // first build (allocations, first launches) and the median of the next
    // `builds` (the steady state a frame loop sees)
    double cold_ms = 0.0;
    RT_OR_FAIL(rt_bvh_build(s, RT_BACKEND_HIP, 0u, &cold_ms));
    std::vector<double> bms;
    for (uint32_t b = 0; b < a.builds; ++b) {
        double t = 0.0;
        RT_OR_FAIL(rt_bvh_build(s, RT_BACKEND_HIP, 0u, &t));
        bms.push_back(t);
    }
    std::sort(bms.begin(), bms.end());
    const double build_ms = bms.empty() ? cold_ms : bms[bms.size() / 2];

    // ---- frames
    const View& v = view_for(base);
    const double pi = 3.14159265358979323846;
    std::vector<uint8_t> rgba((size_t)a.w * a.h * 4);
    std::vector<rt_hit> hits(a.hits.empty() ? 0 : (size_t)a.w * a.h * a.spp);
    float light[3];
    light_for(base, light);
    std::vector<double> ms;
    for (uint32_t f = 0; f < a.warmup + a.frames; ++f) {
        const double ang = a.orbit * pi / 180.0 * f;
        const double ex = v.eye[0] - v.at[0], ey = v.eye[1] - v.at[1], ez = v.eye[2] - v.at[2];
        const double eye[3] = {v.at[0] + ex * std::cos(ang) + ez * std::sin(ang), v.at[1] + ey,
                               v.at[2] - ex * std::sin(ang) + ez * std::cos(ang)};
        rt_camera cam;
        RT_OR_FAIL(rt_camera_look_at(eye, v.at, v.up, v.vfov, a.w, a.h, &cam));
        const bool last = f + 1 == a.warmup + a.frames;
        rt_hit* ho = last && !hits.empty() ? hits.data() : nullptr;
        uint8_t* ro = last && !a.dump.empty() ? rgba.data() : nullptr;
        double t = 0.0;
        if (a.mode == "primary")
            RT_OR_FAIL(rt_render_timed(s, &cam, a.w, a.h, a.spp, a.gpus, ho, ro, &t));
        else if (a.mode == "shadow")
            RT_OR_FAIL(rt_render_shadow(s, &cam, light, 0.2f, a.w, a.h, a.spp, ho, ro ? ro : rgba.data(), &t));
        else
            RT_OR_FAIL(rt_render_path(s, &cam, light, (float)a.sky, a.depth, a.w, a.h, a.spp, ho,
                                      ro ? ro : rgba.data(), &t));
        if (f >= a.warmup) ms.push_back(t);
    }
    if (!a.dump.empty()) RT_OR_FAIL(rt_framebuffer_dump_ppm(rgba.data(), a.w, a.h, a.dump.c_str()));
    if (!a.hits.empty()) RT_OR_FAIL(rt_hits_dump(hits.data(), hits.size(), a.hits.c_str()));
    std::vector<double> sorted = ms;
    std::sort(sorted.begin(), sorted.end());
    const double med = sorted[sorted.size() / 2], best = sorted.front();
    const double rays = (double)a.w * a.h * a.spp;
    std::printf("{\"tool\": \"rtbench\", \"status\": \"ok\", \"scene\": \"%s\", \"n_tris\": %u, \"res\": [%u, %u], "
                "\"spp\": %u, \"gpus\": %u, \"mode\": \"%s\", \"orbit_deg\": %g, \"frames\": %u, \"warmup\": %u, "
                "\"build_ms\": %.4f, \"build_ms_first\": %.4f, \"build_mprims_per_s\": %.1f, \"frame_ms_median\": %.4f, "
                "\"frame_ms_best\": %.4f, "
                "\"mrays_per_s\": %.1f, \"version\": \"%s\"}\n",
                a.scene.c_str(), n, a.w, a.h, a.spp, a.gpus, a.mode.c_str(), a.orbit, a.frames, a.warmup, build_ms, cold_ms,
                build_ms > 0 ? n / (build_ms * 1e3) : 0.0, med, best, rays / (med * 1e3), rt_version());
    rt_scene_free(s);
    return 0;
}

// scene_io.cpp -- scene ingest for librtamd.
//
//   load_obj       Wavefront OBJ -> triangle soup: 'v x y z [w]' and
//                  'f a b c ...' with v, v/vt, v//vn, v/vt/vn forms, negative
//                  (relative) indices and polygon fan triangulation
//                  (a,b,c),(a,c,d),...; every other statement is ignored.
//   soup_generate  the synthetic random-triangle soup of SURVEY.md §9.9
//                  (splitmix64, centroids U[0,1)^3, offsets U[-r,r)^3,
//                  r = (float)(1/cbrt(N))).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace rtio {

static inline uint64_t splitmix64(uint64_t& s) {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void soup_generate(uint32_t n, uint64_t seed, float* tris) {
    uint64_t s = seed;
    const float r = n ? (float)(1.0 / std::cbrt((double)n)) : 0.0f;
    auto u01 = [&s]() { return (float)(splitmix64(s) >> 40) * 0x1p-24f; };
    for (uint32_t i = 0; i < n; ++i) {
        float c[3];
        c[0] = u01();
        c[1] = u01();
        c[2] = u01();
        float* t = tris + (size_t)i * 9;
        for (int v = 0; v < 3; ++v)
            for (int a = 0; a < 3; ++a) {
                const float u = u01();
                t[v * 3 + a] = c[a] + (2.0f * u - 1.0f) * r;
            }
    }
}

static bool parse_index(const char* tok, long nverts, long& out) {
    char* end = nullptr;
    long v = std::strtol(tok, &end, 10);
    if (end == tok) return false;
    if (v > 0) out = v - 1;
    else if (v < 0) out = nverts + v;
    else return false;
    return out >= 0 && out < nverts;
}

bool load_obj(const char* path, std::vector<float>& tris, std::string& err) {
    FILE* f = std::fopen(path, "rb");
    if (!f) {
        err = std::string("cannot open ") + path;
        return false;
    }
    std::vector<float> verts;
    std::vector<long> face;
    char line[4096];
    long lineno = 0;
    bool ok = true;
    while (std::fgets(line, sizeof line, f)) {
        ++lineno;
        char* p = line;
        while (*p == ' ' || *p == '\t') ++p;
        if (p[0] == 'v' && (p[1] == ' ' || p[1] == '\t')) {
            float x, y, z;
            if (std::sscanf(p + 2, "%f %f %f", &x, &y, &z) != 3) {
                err = "bad vertex at line " + std::to_string(lineno);
                ok = false;
                break;
            }
            verts.push_back(x);
            verts.push_back(y);
            verts.push_back(z);
        } else if (p[0] == 'f' && (p[1] == ' ' || p[1] == '\t')) {
            face.clear();
            const long nv = (long)(verts.size() / 3);
            char* save = nullptr;
            for (char* tok = strtok_r(p + 2, " \t\r\n", &save); tok; tok = strtok_r(nullptr, " \t\r\n", &save)) {
                long idx;
                if (!parse_index(tok, nv, idx)) {
                    err = "bad face index at line " + std::to_string(lineno);
                    ok = false;
                    break;
                }
                face.push_back(idx);
            }
            if (!ok) break;
            for (size_t k = 1; k + 1 < face.size(); ++k) {
                const long ids[3] = {face[0], face[k], face[k + 1]};
                for (long id : ids)
                    for (int a = 0; a < 3; ++a) tris.push_back(verts[(size_t)id * 3 + a]);
            }
        }
    }
    std::fclose(f);
    if (ok && tris.size() / 9 > (1u << 30)) {
        err = "too many triangles";
        ok = false;
    }
    return ok;
}

}  // namespace rtio

// scene_io.cpp -- scene ingest for librtamd.
//
//   load_obj       Wavefront OBJ -> triangle soup (see load_obj below)
//   load_soup /    RTSOUP1 binary triangle soup
//   save_soup
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

static bool parse_index(const char* tok, size_t len, long nverts, long& out) {
    // "v", "v/vt", "v//vn", "v/vt/vn": only the vertex index counts
    char buf[32];
    size_t k = 0;
    while (k < len && tok[k] != '/' && k + 1 < sizeof buf) { buf[k] = tok[k]; ++k; }
    buf[k] = 0;
    char* end = nullptr;
    const long v = std::strtol(buf, &end, 10);
    if (end == buf || *end) return false;
    if (v > 0) out = v - 1;
    else if (v < 0) out = nverts + v;   // relative index
    else return false;
    return out >= 0 && out < nverts;
}

static bool read_file(const char* path, std::string& data, std::string& err) {
    FILE* f = std::fopen(path, "rb");
    if (!f) {
        err = std::string("cannot open ") + path;
        return false;
    }
    char buf[1 << 16];
    size_t got;
    while ((got = std::fread(buf, 1, sizeof buf, f)) > 0) data.append(buf, got);
    const bool bad = std::ferror(f) != 0;
    std::fclose(f);
    if (bad) err = std::string("read error on ") + path;
    return !bad;
}

// Wavefront OBJ: lines of any length, LF or CRLF, '#' comments, '\'
// continuation lines; 'v x y z [w]' and 'f' with 3+ corners in any of the
// four index forms; everything else (vt, vn, o, g, s, mtllib, usemtl, l, p,
// curves) is ignored.  Faces are fan-triangulated (a,b,c), (a,c,d), ...
bool load_obj(const char* path, std::vector<float>& tris, std::string& err) {
    std::string data;
    if (!read_file(path, data, err)) return false;
    std::vector<float> verts;
    std::vector<long> face;
    std::string line;
    size_t pos = 0;
    long lineno = 0;
    while (pos < data.size()) {
        // gather one logical line (joining backslash continuations)
        line.clear();
        for (;;) {
            size_t eol = data.find('\n', pos);
            if (eol == std::string::npos) eol = data.size();
            size_t end = eol;
            if (end > pos && data[end - 1] == '\r') --end;
            ++lineno;
            const bool cont = end > pos && data[end - 1] == '\\';
            line.append(data, pos, (cont ? end - 1 : end) - pos);
            pos = eol < data.size() ? eol + 1 : eol;
            if (!cont || pos >= data.size()) break;
            line.push_back(' ');
        }
        const size_t hash = line.find('#');
        if (hash != std::string::npos) line.resize(hash);
        const char* p = line.c_str();
        while (*p == ' ' || *p == '\t') ++p;
        if (p[0] == 'v' && (p[1] == ' ' || p[1] == '\t')) {
            char* q = const_cast<char*>(p + 2);
            float xyz[3];
            for (int a = 0; a < 3; ++a) {
                char* e = nullptr;
                xyz[a] = std::strtof(q, &e);
                if (e == q) {
                    err = "bad vertex at line " + std::to_string(lineno);
                    return false;
                }
                q = e;
            }
            verts.insert(verts.end(), xyz, xyz + 3);
        } else if (p[0] == 'f' && (p[1] == ' ' || p[1] == '\t')) {
            face.clear();
            const long nv = (long)(verts.size() / 3);
            const char* q = p + 2;
            for (;;) {
                while (*q == ' ' || *q == '\t') ++q;
                if (!*q) break;
                const char* t = q;
                while (*q && *q != ' ' && *q != '\t') ++q;
                long idx;
                if (!parse_index(t, (size_t)(q - t), nv, idx)) {
                    err = "bad face index at line " + std::to_string(lineno);
                    return false;
                }
                face.push_back(idx);
            }
            if (face.size() < 3) {
                err = "face with fewer than 3 vertices at line " + std::to_string(lineno);
                return false;
            }
            for (size_t k = 1; k + 1 < face.size(); ++k) {
                const long ids[3] = {face[0], face[k], face[k + 1]};
                for (long id : ids)
                    for (int a = 0; a < 3; ++a) tris.push_back(verts[(size_t)id * 3 + a]);
            }
        }
        if (tris.size() / 9 > (1u << 30)) {
            err = "too many triangles";
            return false;
        }
    }
    return true;
}

// RTSOUP1 binary soup: "RTSOUP1\0", u32 version = 1, u32 0, u64 n, then
// n x 9 little-endian float32 (the rt_scene_from_soup layout).
static const char kSoupMagic[8] = {'R', 'T', 'S', 'O', 'U', 'P', '1', 0};

bool load_soup(const char* path, std::vector<float>& tris, std::string& err) {
    std::string data;
    if (!read_file(path, data, err)) return false;
    if (data.size() < 24 || std::memcmp(data.data(), kSoupMagic, 8) != 0) {
        err = std::string(path) + ": not an RTSOUP1 file";
        return false;
    }
    uint32_t ver;
    uint64_t n;
    std::memcpy(&ver, data.data() + 8, 4);
    std::memcpy(&n, data.data() + 16, 8);
    if (ver != 1) {
        err = std::string(path) + ": unsupported RTSOUP version " + std::to_string(ver);
        return false;
    }
    if (n > (1ull << 30) || data.size() != 24 + n * 36) {
        err = std::string(path) + ": size does not match the triangle count";
        return false;
    }
    tris.resize((size_t)n * 9);
    if (n) std::memcpy(tris.data(), data.data() + 24, (size_t)n * 36);
    return true;
}

bool save_soup(const char* path, const float* tris, uint64_t n, std::string& err) {
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        err = std::string("cannot create ") + path;
        return false;
    }
    const uint32_t hdr[2] = {1u, 0u};
    bool ok = std::fwrite(kSoupMagic, 1, 8, f) == 8 && std::fwrite(hdr, 4, 2, f) == 2 &&
              std::fwrite(&n, 8, 1, f) == 1 && (n == 0 || std::fwrite(tris, 36, n, f) == n);
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) err = std::string("write error on ") + path;
    return ok;
}

}  // namespace rtio

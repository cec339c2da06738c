// rt_abi.cpp -- extern "C" boundary of librtamd.so (include/gpu_raytracer_amd.h).
//
// Host C++ around the gfx950 kernels: scene objects, device buffers kept
// resident per scene, one HIP stream per scene, hipEvent timing, error
// mapping (HIP -> RT_EDEVICE) and a thread-local error message.  There is no
// CPU compute path here: without a gfx950 device every compute entry point
// returns RT_EDEVICE.
#include "../../include/gpu_raytracer_amd.h"
#include "rt_device.h"
#include "rt_launch.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

namespace rtio {
bool load_obj(const char* path, std::vector<float>& tris, std::string& err);
bool load_soup(const char* path, std::vector<float>& tris, std::string& err);
bool save_soup(const char* path, const float* tris, uint64_t n, std::string& err);
void soup_generate(uint32_t n, uint64_t seed, float* tris);
}  // namespace rtio

struct rt_scene {
    std::vector<float> tris;  // host copy, n*9
    uint32_t n = 0;
    int device = 0;
    hipStream_t stream = nullptr;
    rt::BuildBufs bufs;
    bool uploaded = false, built = false;
    rt::BuildEvents ev;
    rt_build_times times{};
    // render scratch (grown on demand)
    void* d_hits = nullptr;
    size_t hits_cap = 0;
    void* d_rgba = nullptr;
    size_t rgba_cap = 0;
    unsigned long long* d_ctr = nullptr;
    uint32_t* d_work = nullptr;  // pool-trace unit counters
    void* d_order = nullptr;     // tile-order state: [order][cost A][cost B] per tile slot
    size_t order_cap = 0;
    rt::TileSched sched;
    uint32_t sched_key[5] = {0, 0, 0, 0, 0};  // w, h, spp, rank, nranks of the cost map
    rt::PathBufs path;           // wavefront path-mode state (grown on demand)
    hipEvent_t r0 = nullptr, r1 = nullptr;
};

namespace {

thread_local std::string g_err;

rt_status fail(rt_status s, const std::string& m) {
    g_err = m;
    return s;
}
rt_status hip_fail(hipError_t e, const char* where) {
    return fail(RT_EDEVICE, std::string(where) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")");
}

#define HIPR(expr)                                          \
    do {                                                    \
        hipError_t _e = (expr);                             \
        if (_e != hipSuccess) return hip_fail(_e, #expr);   \
    } while (0)

rt_status ensure_device(int dev) {
    int cnt = 0;
    hipError_t e = hipGetDeviceCount(&cnt);
    if (e != hipSuccess || cnt == 0)
        return fail(RT_EDEVICE, "no HIP device available (librtamd has no CPU path)");
    if (dev < 0 || dev >= cnt) return fail(RT_EINVAL, "device index out of range");
    HIPR(hipSetDevice(dev));
    return RT_OK;
}

rt_status ensure_stream(rt_scene* s) {
    rt_status st = ensure_device(s->device);
    if (st) return st;
    if (!s->stream) {
        HIPR(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        // timing-only events: no system-scope fence (L2 writeback + invalidate)
        // at each record, which would add ~4.7 us per event to the GPU
        // timeline between the kernels being timed.  Every host read of
        // results goes through a stream synchronize or a blocking copy.
        const unsigned fl = rt::g_trace_config.event_fence ? hipEventDefault : hipEventDisableSystemFence;
        for (auto& e : s->ev.e) HIPR(hipEventCreateWithFlags(&e, fl));
        s->ev.valid = true;
        HIPR(hipEventCreateWithFlags(&s->r0, fl));
        HIPR(hipEventCreateWithFlags(&s->r1, fl));
        HIPR(hipMalloc((void**)&s->d_work, 4096));  // kPoolCounters x 128 B
    }
    return RT_OK;
}

rt_status upload(rt_scene* s) {
    rt_status st = ensure_stream(s);
    if (st) return st;
    if (s->uploaded) return RT_OK;
    if (s->bufs.cap_n != s->n || !s->bufs.tris) {
        hipError_t e = rt::alloc_build(s->bufs, s->n);
        if (e == hipErrorOutOfMemory) return fail(RT_ENOMEM, "device allocation failed");
        if (e != hipSuccess) return hip_fail(e, "alloc_build");
    }
    if (s->n) HIPR(hipMemcpyAsync(s->bufs.tris, s->tris.data(), (size_t)s->n * 36, hipMemcpyHostToDevice, s->stream));
    HIPR(hipStreamSynchronize(s->stream));
    s->uploaded = true;
    return RT_OK;
}

rt_status grow(void** p, size_t* cap, size_t need) {
    if (*cap >= need && *p) return RT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc(p, need ? need : 16);
    if (e == hipErrorOutOfMemory) return fail(RT_ENOMEM, "device allocation failed");
    if (e != hipSuccess) return hip_fail(e, "hipMalloc");
    *cap = need;
    return RT_OK;
}

// Tile-order state for a frame of this shape (DESIGN.md "Tile order"): the
// cost map of the previous frame with the same w, h, spp, rank, nranks
// drives this frame's dispatch order (nullptr: row-major, no map).
rt::TileSched* sched_for(rt_scene* s, uint32_t w, uint32_t h, uint32_t spp, uint32_t rank, uint32_t nranks) {
    const uint32_t nb = rt::tiles_for_rank(w, h, rank, nranks);
    const uint32_t key[5] = {w, h, spp, rank, nranks};
    const bool same = std::memcmp(key, s->sched_key, sizeof(key)) == 0;
    // [order][cost A][cost B] u32, [px A][px B] u16 x 256 per tile slot
    const size_t need = 3ull * nb * 4 + 2ull * nb * 512;
    if (!same || s->order_cap < need) {
        if (grow(&s->d_order, &s->order_cap, need)) return nullptr;
        uint32_t* b = static_cast<uint32_t*>(s->d_order);
        s->sched.order = b;
        s->sched.cost_prev = b + nb;
        s->sched.cost_cur = b + 2 * nb;
        s->sched.px_prev = reinterpret_cast<uint16_t*>(b + 3 * nb);
        s->sched.px_cur = s->sched.px_prev + (size_t)nb * 256;
        s->sched.have_prev = false;
        s->sched.fresh = true;
        std::memcpy(s->sched_key, key, sizeof(key));
    }
    return &s->sched;
}

// after a launch that used sched_for: this frame's map becomes the previous one
void sched_done(rt_scene* s) {
    if (!rt::g_trace_config.tile_order) return;
    std::swap(s->sched.cost_prev, s->sched.cost_cur);
    std::swap(s->sched.px_prev, s->sched.px_cur);
    s->sched.have_prev = true;
}

rt::CamF camf(const rt_camera* c) {
    rt::CamF f;
    std::memcpy(&f, c, sizeof(f));
    return f;
}

// RAII device scratch for the stage entry points
struct DevBuf {
    void* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes ? bytes : 16); }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

}  // namespace

extern "C" {

const char* rt_last_error(void) { return g_err.c_str(); }
const char* rt_version(void) { return "gpu_raytracer_amd 0.1 (gfx950)"; }

rt_status rt_config_set(const char* key, int64_t value) {
    if (!key) return fail(RT_EINVAL, "null key");
    const std::string k(key);
    if (k == "trace.variant" && value >= 0 && value <= 2) rt::g_trace_config.variant = (uint32_t)value;
    else if (k == "trace.stack_cap" && value >= 1 && value <= 14) rt::g_trace_config.stack_cap = (uint32_t)value;
    else if (k == "trace.wg" && (value == 64 || value == 256)) rt::g_trace_config.wg = (uint32_t)value;
    else if (k == "trace.wg_tiles" && (value == 64 || value == 256)) rt::g_trace_config.wg_tiles = (uint32_t)value;
    else if (k == "trace.tile_order" && (value == 0 || value == 1)) rt::g_trace_config.tile_order = (uint32_t)value;
    else if (k == "trace.px_sort" && value >= 0 && value <= 2) rt::g_trace_config.px_sort = (uint32_t)value;
    else if (k == "trace.blocks" && value >= 0 && value <= (1 << 20)) rt::g_trace_config.blocks = (uint32_t)value;
    else if (k == "build.sort" && (value == 0 || value == 1)) rt::g_trace_config.sort_msb = (uint32_t)value;
    else if (k == "build.wide_collapse" && (value == 0 || value == 1)) rt::g_trace_config.wide_collapse = (uint32_t)value;
    else if (k == "build.stage_events" && (value == 0 || value == 1)) rt::g_trace_config.stage_events = (uint32_t)value;
    else if (k == "timing.event_fence" && (value == 0 || value == 1)) rt::g_trace_config.event_fence = (uint32_t)value;
    else if (k == "path.wavefront" && (value == 0 || value == 1)) rt::g_trace_config.path_wave = (uint32_t)value;
    else if (k == "path.wg" && (value == 64 || value == 256)) rt::g_trace_config.path_wg = (uint32_t)value;
    else if (k == "path.sort" && value >= 0 && value <= 4) rt::g_trace_config.path_sort = (uint32_t)value;
    else if (k == "path.batch" && value >= 0 && value <= (1 << 28)) rt::g_trace_config.path_batch = (uint32_t)value;
    else return fail(RT_EINVAL, "unknown config key or value out of range: " + k);
    return RT_OK;
}

int rt_device_count(void) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c;
}

// ------------------------------------------------------------------ scenes
rt_status rt_scene_from_soup(const float* tris, uint32_t n, rt_scene** out) {
    if (!out || (n && !tris)) return fail(RT_EINVAL, "null argument");
    if (n > (1u << 30)) return fail(RT_EINVAL, "n exceeds 2^30 triangles");
    std::unique_ptr<rt_scene> s(new (std::nothrow) rt_scene);
    if (!s) return fail(RT_ENOMEM, "host allocation failed");
    try {
        s->tris.assign(tris, tris + (size_t)n * 9);
    } catch (...) {
        return fail(RT_ENOMEM, "host allocation failed");
    }
    s->n = n;
    *out = s.release();
    return RT_OK;
}

rt_status rt_scene_load_obj(const char* path, rt_scene** out) {
    if (!path || !out) return fail(RT_EINVAL, "null argument");
    std::vector<float> t;
    std::string err;
    if (!rtio::load_obj(path, t, err)) return fail(RT_EIO, err);
    return rt_scene_from_soup(t.data(), (uint32_t)(t.size() / 9), out);
}

rt_status rt_scene_load_soup(const char* path, rt_scene** out) {
    if (!path || !out) return fail(RT_EINVAL, "null argument");
    std::vector<float> t;
    std::string err;
    if (!rtio::load_soup(path, t, err)) return fail(RT_EIO, err);
    return rt_scene_from_soup(t.data(), (uint32_t)(t.size() / 9), out);
}

rt_status rt_scene_save_soup(const rt_scene* s, const char* path) {
    if (!s || !path) return fail(RT_EINVAL, "null argument");
    std::string err;
    if (!rtio::save_soup(path, s->tris.data(), s->n, err)) return fail(RT_EIO, err);
    return RT_OK;
}

rt_status rt_scene_generate_soup(uint32_t n, uint64_t seed, rt_scene** out) {
    if (!out) return fail(RT_EINVAL, "null argument");
    if (n > (1u << 30)) return fail(RT_EINVAL, "n exceeds 2^30 triangles");
    std::unique_ptr<rt_scene> s(new (std::nothrow) rt_scene);
    if (!s) return fail(RT_ENOMEM, "host allocation failed");
    try {
        s->tris.resize((size_t)n * 9);
    } catch (...) {
        return fail(RT_ENOMEM, "host allocation failed");
    }
    rtio::soup_generate(n, seed, s->tris.data());
    s->n = n;
    *out = s.release();
    return RT_OK;
}

rt_status rt_scene_num_tris(const rt_scene* s, uint32_t* n_out) {
    if (!s || !n_out) return fail(RT_EINVAL, "null argument");
    *n_out = s->n;
    return RT_OK;
}

rt_status rt_scene_get_tris(const rt_scene* s, float* out) {
    if (!s || !out) return fail(RT_EINVAL, "null argument");
    std::memcpy(out, s->tris.data(), s->tris.size() * sizeof(float));
    return RT_OK;
}

rt_status rt_scene_set_device(rt_scene* s, int device) {
    if (!s) return fail(RT_EINVAL, "null argument");
    if (s->stream) return fail(RT_EINVAL, "device must be set before the first build");
    s->device = device;
    return RT_OK;
}

void rt_scene_free(rt_scene* s) {
    if (!s) return;
    if (s->stream) {
        (void)hipSetDevice(s->device);
        (void)hipStreamSynchronize(s->stream);
        rt::free_build(s->bufs);
        rt::free_path(s->path);
        if (s->d_hits) (void)hipFree(s->d_hits);
        if (s->d_rgba) (void)hipFree(s->d_rgba);
        if (s->d_ctr) (void)hipFree(s->d_ctr);
        if (s->d_work) (void)hipFree(s->d_work);
        if (s->d_order) (void)hipFree(s->d_order);
        for (auto& e : s->ev.e) (void)hipEventDestroy(e);
        (void)hipEventDestroy(s->r0);
        (void)hipEventDestroy(s->r1);
        (void)hipStreamDestroy(s->stream);
    }
    delete s;
}

rt_status rt_scene_stream(rt_scene* s, void** stream_out) {
    if (!s || !stream_out) return fail(RT_EINVAL, "null argument");
    rt_status st = ensure_stream(s);
    if (st) return st;
    *stream_out = (void*)s->stream;
    return RT_OK;
}

rt_status rt_scene_sync(rt_scene* s) {
    if (!s) return fail(RT_EINVAL, "null argument");
    if (!s->stream) return RT_OK;
    HIPR(hipSetDevice(s->device));
    HIPR(hipStreamSynchronize(s->stream));
    return RT_OK;
}

// ------------------------------------------------------------------ camera
// f = normalize(at-eye), r = normalize(f x up), u = r x f;
// w00 = f + u*tan - r*tan*aspect; du = r*(2 tan aspect/W); dv = -u*(2 tan/H).
rt_status rt_camera_look_at(const double eye[3], const double at[3], const double up[3], double vfov_deg,
                            uint32_t w, uint32_t h, rt_camera* out) {
    if (!eye || !at || !up || !out || !w || !h) return fail(RT_EINVAL, "bad camera arguments");
    double f[3] = {at[0] - eye[0], at[1] - eye[1], at[2] - eye[2]};
    auto norm = [](double* v) {
        const double l = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        v[0] /= l; v[1] /= l; v[2] /= l;
    };
    auto cross = [](const double* a, const double* b, double* o) {
        o[0] = a[1] * b[2] - a[2] * b[1];
        o[1] = a[2] * b[0] - a[0] * b[2];
        o[2] = a[0] * b[1] - a[1] * b[0];
    };
    norm(f);
    double r[3], u[3];
    cross(f, up, r);
    norm(r);
    cross(r, f, u);
    const double th = std::tan(vfov_deg * 3.14159265358979323846 / 360.0);
    const double aspect = (double)w / (double)h;
    for (int a = 0; a < 3; ++a) {
        out->eye[a] = (float)eye[a];
        out->w00[a] = (float)(f[a] + u[a] * th - r[a] * th * aspect);
        out->du[a] = (float)(r[a] * (2.0 * th * aspect / (double)w));
        out->dv[a] = (float)(-u[a] * (2.0 * th / (double)h));
    }
    return RT_OK;
}

// ------------------------------------------------------------------ build
rt_status rt_bvh_build(rt_scene* s, double* ms_out) {
    if (!s) return fail(RT_EINVAL, "null scene");
    rt_status st = upload(s);
    if (st) return st;
    const bool stages = rt::g_trace_config.stage_events != 0;
    hipError_t e = rt::launch_build(s->bufs, s->n, s->stream, &s->ev, stages);
    if (e != hipSuccess) return hip_fail(e, "launch_build");
    HIPR(hipStreamSynchronize(s->stream));
    float t[6] = {0, 0, 0, 0, 0, 0};
    if (stages)
        for (int i = 0; i < 6; ++i) HIPR(hipEventElapsedTime(&t[i], s->ev.e[i], s->ev.e[i + 1]));
    s->times.bounds = t[0];
    s->times.morton = t[1];
    s->times.sort = t[2];
    s->times.topology = t[3];
    s->times.refit = t[4];
    s->times.wide = t[5];
    float tot = 0;
    HIPR(hipEventElapsedTime(&tot, s->ev.e[0], s->ev.e[6]));
    s->times.total = tot;
    if (ms_out) *ms_out = tot;
    s->built = true;
    return RT_OK;
}

rt_status rt_bvh_build_times(const rt_scene* s, rt_build_times* out) {
    if (!s || !out) return fail(RT_EINVAL, "null argument");
    if (!s->built) return fail(RT_EINVAL, "scene not built");
    *out = s->times;
    return RT_OK;
}

rt_status rt_bvh_read(const rt_scene* s, rt_node* nodes, uint32_t* keys, uint32_t* vals, uint32_t* parent,
                      float* bounds9) {
    if (!s) return fail(RT_EINVAL, "null scene");
    if (!s->built) return fail(RT_EINVAL, "scene not built");
    HIPR(hipSetDevice(s->device));
    HIPR(hipStreamSynchronize(s->stream));
    const size_t n = s->n, tot = n ? 2 * n - 1 : 0;
    if (nodes && tot) HIPR(hipMemcpy(nodes, s->bufs.nodes, tot * 32, hipMemcpyDeviceToHost));
    if (keys && n) HIPR(hipMemcpy(keys, s->bufs.keys[0], n * 4, hipMemcpyDeviceToHost));
    if (vals && n) HIPR(hipMemcpy(vals, s->bufs.vals[0], n * 4, hipMemcpyDeviceToHost));
    if (parent && tot) HIPR(hipMemcpy(parent, s->bufs.parent, tot * 4, hipMemcpyDeviceToHost));
    if (bounds9) HIPR(hipMemcpy(bounds9, s->bufs.params, 9 * 4, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_bvh_read_wide(const rt_scene* s, void* records) {
    if (!s || !records) return fail(RT_EINVAL, "null argument");
    if (!s->built) return fail(RT_EINVAL, "scene not built");
    HIPR(hipSetDevice(s->device));
    HIPR(hipStreamSynchronize(s->stream));
    if (s->n >= 2) HIPR(hipMemcpy(records, s->bufs.wnodes, (size_t)(s->n - 1) * 64, hipMemcpyDeviceToHost));
    return RT_OK;
}

// ------------------------------------------------------------------ BVH cache
// RTBVH1: "RTBVH1\0\0", u32 version, u32 n, u64 FNV-1a hash of the n*36
// triangle bytes, u64 layout tag, then the device buffers the trace and
// rt_bvh_read use, in order: BuildParams (64 B), sorted keys and vals (n x 4),
// nodes ((2n-1) x 32), parent ((2n-1) x 4), tri_s (n x 48), wide records
// ((n-1) x 64).  The tag changes whenever one of those layouts does.
extern "C++" {
namespace {
const char kBvhMagic[8] = {'R', 'T', 'B', 'V', 'H', '1', 0, 0};
constexpr uint32_t kBvhVersion = 1;
constexpr uint64_t kBvhLayout = 0x7274616d64000001ull;  // "rtamd" + layout revision 1

uint64_t fnv1a(const void* p, size_t bytes) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < bytes; ++i) {
        h ^= b[i];
        h *= 0x100000001b3ull;
    }
    return h;
}

struct BvhSection {
    void* dev;
    size_t bytes;
};

std::vector<BvhSection> bvh_sections(const rt_scene* s) {
    const size_t n = s->n, tot = n ? 2 * n - 1 : 0;
    static_assert(sizeof(rt::BuildParams) == 64, "RTBVH1 stores a 64-B BuildParams");
    return {{s->bufs.params, sizeof(rt::BuildParams)},
            {s->bufs.keys[0], n * 4},
            {s->bufs.vals[0], n * 4},
            {s->bufs.nodes, tot * 32},
            {s->bufs.parent, tot * 4},
            {s->bufs.tri_s, n * 48},
            {s->bufs.wnodes, n >= 2 ? (n - 1) * 64 : 0}};
}
}  // namespace
}  // extern "C++"

rt_status rt_bvh_save(const rt_scene* s, const char* path) {
    if (!s || !path) return fail(RT_EINVAL, "null argument");
    if (!s->built) return fail(RT_EINVAL, "scene not built");
    HIPR(hipSetDevice(s->device));
    HIPR(hipStreamSynchronize(s->stream));
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(RT_EIO, std::string("cannot create ") + path);
    const uint32_t hv[2] = {kBvhVersion, s->n};
    const uint64_t hh[2] = {fnv1a(s->tris.data(), s->tris.size() * sizeof(float)), kBvhLayout};
    bool ok = std::fwrite(kBvhMagic, 1, 8, f) == 8 && std::fwrite(hv, 4, 2, f) == 2 && std::fwrite(hh, 8, 2, f) == 2;
    std::vector<unsigned char> host;
    for (const BvhSection& sec : bvh_sections(s)) {
        if (!ok || !sec.bytes) continue;
        host.resize(sec.bytes);
        if (hipMemcpy(host.data(), sec.dev, sec.bytes, hipMemcpyDeviceToHost) != hipSuccess) {
            std::fclose(f);
            return fail(RT_EDEVICE, "device read of the BVH failed");
        }
        ok = std::fwrite(host.data(), 1, sec.bytes, f) == sec.bytes;
    }
    ok = (std::fclose(f) == 0) && ok;
    return ok ? RT_OK : fail(RT_EIO, std::string("write error on ") + path);
}

rt_status rt_bvh_load(rt_scene* s, const char* path) {
    if (!s || !path) return fail(RT_EINVAL, "null argument");
    FILE* f = std::fopen(path, "rb");
    if (!f) return fail(RT_EIO, std::string("cannot open ") + path);
    char magic[8];
    uint32_t hv[2] = {0, 0};
    uint64_t hh[2] = {0, 0};
    const bool hdr = std::fread(magic, 1, 8, f) == 8 && std::fread(hv, 4, 2, f) == 2 && std::fread(hh, 8, 2, f) == 2;
    if (!hdr || std::memcmp(magic, kBvhMagic, 8) != 0) {
        std::fclose(f);
        return fail(RT_EIO, std::string(path) + ": not an RTBVH1 file");
    }
    if (hv[0] != kBvhVersion || hh[1] != kBvhLayout) {
        std::fclose(f);
        return fail(RT_EIO, std::string(path) + ": BVH cache from another library layout");
    }
    if (hv[1] != s->n || hh[0] != fnv1a(s->tris.data(), s->tris.size() * sizeof(float))) {
        std::fclose(f);
        return fail(RT_EINVAL, std::string(path) + ": BVH cache was built for different triangles");
    }
    rt_status st = upload(s);
    if (st) {
        std::fclose(f);
        return st;
    }
    std::vector<unsigned char> host;
    for (const BvhSection& sec : bvh_sections(s)) {
        if (!sec.bytes) continue;
        host.resize(sec.bytes);
        if (std::fread(host.data(), 1, sec.bytes, f) != sec.bytes) {
            std::fclose(f);
            s->built = false;
            return fail(RT_EIO, std::string(path) + ": truncated BVH cache");
        }
        HIPR(hipMemcpy(sec.dev, host.data(), sec.bytes, hipMemcpyHostToDevice));
    }
    const bool extra = std::fgetc(f) != EOF;
    std::fclose(f);
    if (extra) {
        s->built = false;
        return fail(RT_EIO, std::string(path) + ": trailing bytes in BVH cache");
    }
    s->times = rt_build_times{};
    s->built = true;
    return RT_OK;
}

// Device-resident BVH exchange (SURVEY.md §8(e) "rank 0 builds and then
// broadcasts"): the same sections as the RTBVH1 file, as device pointers.
rt_status rt_bvh_prepare(rt_scene* s) {
    if (!s) return fail(RT_EINVAL, "null scene");
    return upload(s);
}

rt_status rt_bvh_device_sections(rt_scene* s, uint32_t max, void** ptrs, uint64_t* bytes, uint32_t* count_out) {
    if (!s || !count_out || (max && (!ptrs || !bytes))) return fail(RT_EINVAL, "null argument");
    if (!s->uploaded) return fail(RT_EINVAL, "scene not prepared (rt_bvh_prepare or rt_bvh_build)");
    const std::vector<BvhSection> secs = bvh_sections(s);
    *count_out = (uint32_t)secs.size();
    for (uint32_t i = 0; i < max && i < secs.size(); ++i) {
        ptrs[i] = secs[i].dev;
        bytes[i] = secs[i].bytes;
    }
    return RT_OK;
}

rt_status rt_bvh_mark_built(rt_scene* s) {
    if (!s) return fail(RT_EINVAL, "null scene");
    if (!s->uploaded) return fail(RT_EINVAL, "scene not prepared (rt_bvh_prepare)");
    HIPR(hipSetDevice(s->device));
    HIPR(hipDeviceSynchronize());  // the caller's writes (any stream) land before the first render
    s->times = rt_build_times{};
    s->built = true;
    return RT_OK;
}

// ------------------------------------------------------------------ render
rt_status rt_render(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp, rt_hit* hits_out,
                    uint8_t* rgba_out, double* ms_out) {
    if (!s || !cam || !w || !h || !spp) return fail(RT_EINVAL, "bad render arguments");
    if (!s->built) return fail(RT_EINVAL, "scene not built (call rt_bvh_build)");
    if ((uint64_t)w * h * spp > 0xFFFFFFFFull) return fail(RT_EINVAL, "w*h*spp exceeds 2^32 samples");
    rt_status st = ensure_stream(s);
    if (st) return st;
    const size_t nh = (size_t)w * h * spp;
    if (hits_out && (st = grow(&s->d_hits, &s->hits_cap, nh * 16))) return st;
    if ((st = grow(&s->d_rgba, &s->rgba_cap, (size_t)w * h * 4))) return st;
    HIPR(hipEventRecord(s->r0, s->stream));
    hipError_t e = rt::launch_trace(s->bufs.nodes, s->bufs.wnodes, s->bufs.tri_s, s->n, camf(cam), w, h, spp, 0, 1,
                                    false, hits_out ? s->d_hits : nullptr, s->d_rgba, nullptr, false, s->d_work,
                                    sched_for(s, w, h, spp, 0, 1), s->stream);
    if (e != hipSuccess) return hip_fail(e, "launch_trace");
    sched_done(s);
    HIPR(hipEventRecord(s->r1, s->stream));
    HIPR(hipStreamSynchronize(s->stream));
    float ms = 0;
    HIPR(hipEventElapsedTime(&ms, s->r0, s->r1));
    if (ms_out) *ms_out = ms;
    if (hits_out) HIPR(hipMemcpy(hits_out, s->d_hits, nh * 16, hipMemcpyDeviceToHost));
    if (rgba_out) HIPR(hipMemcpy(rgba_out, s->d_rgba, (size_t)w * h * 4, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_render_shadow_device(rt_scene* s, const rt_camera* cam, const float light[3], float ambient,
                                  uint32_t w, uint32_t h, uint32_t spp, void* d_hits, void* d_rgba, void* stream,
                                  double* ms_out) {
    if (!s || !cam || !light || !w || !h || !spp) return fail(RT_EINVAL, "bad render arguments");
    if (!s->built) return fail(RT_EINVAL, "scene not built (call rt_bvh_build)");
    if ((uint64_t)w * h * spp > 0xFFFFFFFFull) return fail(RT_EINVAL, "w*h*spp exceeds 2^32 samples");
    rt_status st = ensure_stream(s);
    if (st) return st;
    hipStream_t hs = stream ? (hipStream_t)stream : s->stream;
    if (ms_out) HIPR(hipEventRecord(s->r0, hs));
    hipError_t e = rt::launch_trace_shadow(s->bufs.nodes, s->bufs.wnodes, s->bufs.tri_s, s->bufs.tris, s->n, camf(cam),
                                           w, h, spp, light, ambient, d_hits, d_rgba, nullptr, hs);
    if (e != hipSuccess) return hip_fail(e, "launch_trace_shadow");
    if (ms_out) {
        HIPR(hipEventRecord(s->r1, hs));
        HIPR(hipEventSynchronize(s->r1));
        float ms = 0;
        HIPR(hipEventElapsedTime(&ms, s->r0, s->r1));
        *ms_out = ms;
    }
    return RT_OK;
}

rt_status rt_render_shadow(rt_scene* s, const rt_camera* cam, const float light[3], float ambient, uint32_t w,
                           uint32_t h, uint32_t spp, rt_hit* hits_out, uint8_t* rgba_out, double* ms_out) {
    if (!s || !cam || !light || !w || !h || !spp) return fail(RT_EINVAL, "bad render arguments");
    if (!s->built) return fail(RT_EINVAL, "scene not built (call rt_bvh_build)");
    if ((uint64_t)w * h * spp > 0xFFFFFFFFull) return fail(RT_EINVAL, "w*h*spp exceeds 2^32 samples");
    rt_status st = ensure_stream(s);
    if (st) return st;
    const size_t nh = (size_t)w * h * spp;
    if (hits_out && (st = grow(&s->d_hits, &s->hits_cap, nh * 16))) return st;
    if ((st = grow(&s->d_rgba, &s->rgba_cap, (size_t)w * h * 4))) return st;
    st = rt_render_shadow_device(s, cam, light, ambient, w, h, spp, hits_out ? s->d_hits : nullptr, s->d_rgba,
                                 nullptr, ms_out);
    if (st) return st;
    HIPR(hipStreamSynchronize(s->stream));
    if (hits_out) HIPR(hipMemcpy(hits_out, s->d_hits, nh * 16, hipMemcpyDeviceToHost));
    if (rgba_out) HIPR(hipMemcpy(rgba_out, s->d_rgba, (size_t)w * h * 4, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_render_shadow_work(rt_scene* s, const rt_camera* cam, const float light[3], float ambient, uint32_t w,
                                uint32_t h, uint32_t spp, uint64_t counters_out[2]) {
    if (!s || !cam || !light || !counters_out || !w || !h || !spp) return fail(RT_EINVAL, "bad arguments");
    if (!s->built) return fail(RT_EINVAL, "scene not built (call rt_bvh_build)");
    rt_status st = ensure_stream(s);
    if (st) return st;
    if (!s->d_ctr) HIPR(hipMalloc((void**)&s->d_ctr, 32));
    HIPR(hipMemsetAsync(s->d_ctr, 0, 16, s->stream));
    hipError_t e = rt::launch_trace_shadow(s->bufs.nodes, s->bufs.wnodes, s->bufs.tri_s, s->bufs.tris, s->n, camf(cam),
                                           w, h, spp, light, ambient, nullptr, nullptr, s->d_ctr, s->stream);
    if (e != hipSuccess) return hip_fail(e, "launch_trace_shadow");
    HIPR(hipStreamSynchronize(s->stream));
    HIPR(hipMemcpy(counters_out, s->d_ctr, 16, hipMemcpyDeviceToHost));
    return RT_OK;
}

// Path mode: the megakernel, or the wavefront schedule with ray reordering
// (config path.wavefront); the wavefront reads each depth's queue length back
// to the host, so it synchronizes the stream between depths.
static rt_status path_launch(rt_scene* s, const rt_camera* cam, const float light[3], float sky, uint32_t max_depth,
                             uint32_t w, uint32_t h, uint32_t spp, void* d_hits, void* d_rgba,
                             unsigned long long* ctr, hipStream_t hs) {
    hipError_t e;
    if (rt::g_trace_config.path_wave) {
        const uint64_t per_tile = 256ull * spp;
        const uint64_t tiles = rt::tiles_for_rank(w, h, 0, 1);
        const uint64_t want = rt::g_trace_config.path_batch ? rt::g_trace_config.path_batch : (1u << 22);
        uint64_t cap = std::min<uint64_t>(tiles * per_tile, std::max<uint64_t>(per_tile, want / per_tile * per_tile));
        if (cap > (1u << 30)) return fail(RT_EINVAL, "path batch exceeds 2^30 paths (lower spp or path.batch)");
        if (s->path.cap < cap) {
            if ((e = rt::alloc_path(s->path, (uint32_t)cap)) != hipSuccess) {
                rt::free_path(s->path);
                return hip_fail(e, "alloc_path");
            }
        }
        e = rt::launch_path_wavefront(s->bufs.nodes, s->bufs.wnodes, s->bufs.tri_s, s->bufs.tris, s->bufs.params, s->n,
                                      camf(cam), w, h, spp, light, sky, max_depth, d_hits, d_rgba, ctr, s->path,
                                      rt::g_trace_config.path_sort, hs);
        if (e != hipSuccess) return hip_fail(e, "launch_path_wavefront");
        return RT_OK;
    }
    e = rt::launch_trace_path(s->bufs.nodes, s->bufs.wnodes, s->bufs.tri_s, s->bufs.tris, s->n, camf(cam), w, h, spp,
                              light, sky, max_depth, d_hits, d_rgba, ctr, hs);
    if (e != hipSuccess) return hip_fail(e, "launch_trace_path");
    return RT_OK;
}

rt_status rt_render_path_device(rt_scene* s, const rt_camera* cam, const float light[3], float sky,
                                uint32_t max_depth, uint32_t w, uint32_t h, uint32_t spp, void* d_hits, void* d_rgba,
                                void* stream, double* ms_out) {
    if (!s || !cam || !light || !w || !h || !spp) return fail(RT_EINVAL, "bad render arguments");
    if (max_depth > 64) return fail(RT_EINVAL, "max_depth exceeds 64");
    if (!s->built) return fail(RT_EINVAL, "scene not built (call rt_bvh_build)");
    if ((uint64_t)w * h * spp > 0xFFFFFFFFull) return fail(RT_EINVAL, "w*h*spp exceeds 2^32 samples");
    rt_status st = ensure_stream(s);
    if (st) return st;
    hipStream_t hs = stream ? (hipStream_t)stream : s->stream;
    if (ms_out) HIPR(hipEventRecord(s->r0, hs));
    if ((st = path_launch(s, cam, light, sky, max_depth, w, h, spp, d_hits, d_rgba, nullptr, hs))) return st;
    if (ms_out) {
        HIPR(hipEventRecord(s->r1, hs));
        HIPR(hipEventSynchronize(s->r1));
        float ms = 0;
        HIPR(hipEventElapsedTime(&ms, s->r0, s->r1));
        *ms_out = ms;
    }
    return RT_OK;
}

rt_status rt_render_path(rt_scene* s, const rt_camera* cam, const float light[3], float sky, uint32_t max_depth,
                         uint32_t w, uint32_t h, uint32_t spp, rt_hit* hits_out, uint8_t* rgba_out, double* ms_out) {
    if (!s || !cam || !light || !w || !h || !spp) return fail(RT_EINVAL, "bad render arguments");
    if (!s->built) return fail(RT_EINVAL, "scene not built (call rt_bvh_build)");
    if ((uint64_t)w * h * spp > 0xFFFFFFFFull) return fail(RT_EINVAL, "w*h*spp exceeds 2^32 samples");
    rt_status st = ensure_stream(s);
    if (st) return st;
    const size_t nh = (size_t)w * h * spp;
    if (hits_out && (st = grow(&s->d_hits, &s->hits_cap, nh * 16))) return st;
    if ((st = grow(&s->d_rgba, &s->rgba_cap, (size_t)w * h * 4))) return st;
    st = rt_render_path_device(s, cam, light, sky, max_depth, w, h, spp, hits_out ? s->d_hits : nullptr, s->d_rgba,
                               nullptr, ms_out);
    if (st) return st;
    HIPR(hipStreamSynchronize(s->stream));
    if (hits_out) HIPR(hipMemcpy(hits_out, s->d_hits, nh * 16, hipMemcpyDeviceToHost));
    if (rgba_out) HIPR(hipMemcpy(rgba_out, s->d_rgba, (size_t)w * h * 4, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_render_path_work(rt_scene* s, const rt_camera* cam, const float light[3], float sky, uint32_t max_depth,
                              uint32_t w, uint32_t h, uint32_t spp, uint64_t counters_out[3]) {
    if (!s || !cam || !light || !counters_out || !w || !h || !spp) return fail(RT_EINVAL, "bad arguments");
    if (max_depth > 64) return fail(RT_EINVAL, "max_depth exceeds 64");
    if (!s->built) return fail(RT_EINVAL, "scene not built (call rt_bvh_build)");
    rt_status st = ensure_stream(s);
    if (st) return st;
    if (!s->d_ctr) HIPR(hipMalloc((void**)&s->d_ctr, 32));
    HIPR(hipMemsetAsync(s->d_ctr, 0, 32, s->stream));
    if ((st = path_launch(s, cam, light, sky, max_depth, w, h, spp, nullptr, nullptr, s->d_ctr, s->stream))) return st;
    HIPR(hipStreamSynchronize(s->stream));
    HIPR(hipMemcpy(counters_out, s->d_ctr, 24, hipMemcpyDeviceToHost));
    return RT_OK;
}

static rt_status counters_impl(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp,
                               uint32_t rank, uint32_t nranks, bool packed, bool binary, uint64_t counters_out[2]) {
    if (!s || !cam || !counters_out || !w || !h || !spp || !nranks || rank >= nranks)
        return fail(RT_EINVAL, "bad arguments");
    if (!s->built) return fail(RT_EINVAL, "scene not built (call rt_bvh_build)");
    rt_status st = ensure_stream(s);
    if (st) return st;
    if (!s->d_ctr) HIPR(hipMalloc((void**)&s->d_ctr, 32));
    HIPR(hipMemsetAsync(s->d_ctr, 0, 16, s->stream));
    hipError_t e = rt::launch_trace(s->bufs.nodes, s->bufs.wnodes, s->bufs.tri_s, s->n, camf(cam), w, h, spp, rank,
                                    nranks, packed, nullptr, nullptr, s->d_ctr, binary, s->d_work, nullptr,
                                    s->stream);
    if (e != hipSuccess) return hip_fail(e, "launch_trace");
    HIPR(hipStreamSynchronize(s->stream));
    HIPR(hipMemcpy(counters_out, s->d_ctr, 16, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_render_counters(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp,
                             uint64_t counters_out[2]) {
    return counters_impl(s, cam, w, h, spp, 0, 1, false, true, counters_out);
}

rt_status rt_render_work(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp,
                         uint64_t counters_out[2]) {
    return counters_impl(s, cam, w, h, spp, 0, 1, false, false, counters_out);
}

rt_status rt_render_tiles_counters(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp,
                                   uint32_t rank, uint32_t nranks, uint64_t counters_out[2]) {
    return counters_impl(s, cam, w, h, spp, rank, nranks, true, true, counters_out);
}

rt_status rt_render_device(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp, void* d_hits,
                           void* d_rgba, void* stream, double* ms_out) {
    if (!s || !cam || !w || !h || !spp) return fail(RT_EINVAL, "bad render arguments");
    if (!s->built) return fail(RT_EINVAL, "scene not built (call rt_bvh_build)");
    if ((uint64_t)w * h * spp > 0xFFFFFFFFull) return fail(RT_EINVAL, "w*h*spp exceeds 2^32 samples");
    rt_status st = ensure_stream(s);
    if (st) return st;
    hipStream_t hs = stream ? (hipStream_t)stream : s->stream;
    if (ms_out) HIPR(hipEventRecord(s->r0, hs));
    hipError_t e = rt::launch_trace(s->bufs.nodes, s->bufs.wnodes, s->bufs.tri_s, s->n, camf(cam), w, h, spp, 0, 1,
                                    false, d_hits, d_rgba, nullptr, false, s->d_work,
                                    sched_for(s, w, h, spp, 0, 1), hs);
    if (e != hipSuccess) return hip_fail(e, "launch_trace");
    sched_done(s);
    if (ms_out) {
        HIPR(hipEventRecord(s->r1, hs));
        HIPR(hipEventSynchronize(s->r1));
        float ms = 0;
        HIPR(hipEventElapsedTime(&ms, s->r0, s->r1));
        *ms_out = ms;
    }
    return RT_OK;
}

uint32_t rt_tiles_for_rank(uint32_t w, uint32_t h, uint32_t rank, uint32_t nranks) {
    return rt::tiles_for_rank(w, h, rank, nranks);
}

rt_status rt_render_tiles_device(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp,
                                 uint32_t rank, uint32_t nranks, void* d_packed_rgba, void* d_packed_hits,
                                 void* stream, double* ms_out) {
    if (!s || !cam || !w || !h || !spp || !nranks || rank >= nranks) return fail(RT_EINVAL, "bad arguments");
    if (!s->built) return fail(RT_EINVAL, "scene not built (call rt_bvh_build)");
    rt_status st = ensure_stream(s);
    if (st) return st;
    hipStream_t hs = stream ? (hipStream_t)stream : s->stream;
    if (ms_out) HIPR(hipEventRecord(s->r0, hs));
    hipError_t e = rt::launch_trace(s->bufs.nodes, s->bufs.wnodes, s->bufs.tri_s, s->n, camf(cam), w, h, spp, rank,
                                    nranks, true, d_packed_hits, d_packed_rgba, nullptr, false, s->d_work,
                                    sched_for(s, w, h, spp, rank, nranks), hs);
    if (e != hipSuccess) return hip_fail(e, "launch_trace");
    sched_done(s);
    if (ms_out) {
        HIPR(hipEventRecord(s->r1, hs));
        HIPR(hipEventSynchronize(s->r1));
        float ms = 0;
        HIPR(hipEventElapsedTime(&ms, s->r0, s->r1));
        *ms_out = ms;
    }
    return RT_OK;
}

rt_status rt_unpack_tiles_device(const void* d_slabs, uint32_t tiles_per_slab, uint32_t w, uint32_t h,
                                 uint32_t nranks, void* d_rgba, int device, void* stream) {
    if (!d_slabs || !d_rgba || !w || !h || !nranks) return fail(RT_EINVAL, "bad arguments");
    rt_status st = ensure_device(device);
    if (st) return st;
    hipError_t e = rt::launch_unpack(d_slabs, tiles_per_slab, w, h, nranks, d_rgba, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "launch_unpack");
    return RT_OK;
}

// ------------------------------------------------------------------ stage entry points
rt_status rt_stage_bounds(int device, const float* tris, uint32_t n, float bounds9[9]) {
    if ((n && !tris) || !bounds9) return fail(RT_EINVAL, "null argument");
    rt_status st = ensure_device(device);
    if (st) return st;
    DevBuf dt, dp, dpar;
    HIPR(dt.alloc((size_t)n * 36));
    HIPR(dp.alloc((size_t)rt::bounds_grid(n) * 24));
    HIPR(dpar.alloc(sizeof(rt::BuildParams)));
    if (n) HIPR(hipMemcpy(dt.p, tris, (size_t)n * 36, hipMemcpyHostToDevice));
    HIPR(rt::launch_bounds_only(dt.as<float>(), n, dp.as<float>(), dpar.as<rt::BuildParams>(), 0));
    HIPR(hipDeviceSynchronize());
    HIPR(hipMemcpy(bounds9, dpar.p, 36, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_stage_morton(int device, const float* tris, uint32_t n, const float lo[3], const float inv[3],
                          uint32_t* keys, uint32_t* vals) {
    if ((n && (!tris || !keys || !vals)) || !lo || !inv) return fail(RT_EINVAL, "null argument");
    rt_status st = ensure_device(device);
    if (st) return st;
    if (!n) return RT_OK;
    DevBuf dt, dpar, dk, dv, dh, dc;
    HIPR(dt.alloc((size_t)n * 36));
    HIPR(dpar.alloc(sizeof(rt::BuildParams)));
    HIPR(dk.alloc((size_t)n * 4));
    HIPR(dv.alloc((size_t)n * 4));
    HIPR(dh.alloc(4096));
    HIPR(dc.alloc((size_t)rt::sort_tiles(n) * 1024));
    HIPR(hipMemset(dh.p, 0, 4096));
    rt::BuildParams p{};
    for (int c = 0; c < 3; ++c) { p.lo[c] = lo[c]; p.inv[c] = inv[c]; }
    HIPR(hipMemcpy(dpar.p, &p, sizeof(p), hipMemcpyHostToDevice));
    HIPR(hipMemcpy(dt.p, tris, (size_t)n * 36, hipMemcpyHostToDevice));
    HIPR(rt::launch_morton(dt.as<float>(), n, dpar.as<rt::BuildParams>(), dk.as<uint32_t>(), dv.as<uint32_t>(),
                           dh.as<uint32_t>(), dc.as<uint32_t>(), 0));
    HIPR(hipDeviceSynchronize());
    HIPR(hipMemcpy(keys, dk.p, (size_t)n * 4, hipMemcpyDeviceToHost));
    HIPR(hipMemcpy(vals, dv.p, (size_t)n * 4, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_stage_sort(int device, uint32_t* keys, uint32_t* vals, uint32_t n) {
    if (n && (!keys || !vals)) return fail(RT_EINVAL, "null argument");
    if (n > (1u << 30)) return fail(RT_EINVAL, "n exceeds 2^30");
    rt_status st = ensure_device(device);
    if (st) return st;
    if (n <= 1) return RT_OK;
    DevBuf k0, k1, v0, v1, gh, cnt;
    const size_t cs = (size_t)rt::sort_tiles(n) * 256;
    HIPR(k0.alloc((size_t)n * 4));
    HIPR(k1.alloc((size_t)n * 4));
    HIPR(v0.alloc((size_t)n * 4));
    HIPR(v1.alloc((size_t)n * 4));
    HIPR(gh.alloc(4096));
    HIPR(cnt.alloc(4 * cs * 4));
    HIPR(hipMemset(gh.p, 0, 4096));
    HIPR(hipMemcpy(k0.p, keys, (size_t)n * 4, hipMemcpyHostToDevice));
    HIPR(hipMemcpy(v0.p, vals, (size_t)n * 4, hipMemcpyHostToDevice));
    uint32_t* C[4] = {cnt.as<uint32_t>(), cnt.as<uint32_t>() + cs, cnt.as<uint32_t>() + 2 * cs,
                      cnt.as<uint32_t>() + 3 * cs};
    HIPR(rt::launch_digit_hist(k0.as<uint32_t>(), n, gh.as<uint32_t>(), 0));
    HIPR(rt::launch_tile_hist0(k0.as<uint32_t>(), n, C[0], 0));
    uint32_t* K[2] = {k0.as<uint32_t>(), k1.as<uint32_t>()};
    uint32_t* V[2] = {v0.as<uint32_t>(), v1.as<uint32_t>()};
    HIPR(rt::launch_sort(K, V, n, gh.as<uint32_t>(), C, 0));
    HIPR(hipDeviceSynchronize());
    HIPR(hipMemcpy(keys, k0.p, (size_t)n * 4, hipMemcpyDeviceToHost));
    HIPR(hipMemcpy(vals, v0.p, (size_t)n * 4, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_stage_topology(int device, const uint32_t* sorted_keys, uint32_t n, uint32_t* topo, uint32_t* parent,
                            uint32_t* leaf_esc) {
    if (n && !sorted_keys) return fail(RT_EINVAL, "null argument");
    rt_status st = ensure_device(device);
    if (st) return st;
    if (!n) return RT_OK;
    // K4 also emits the leaves; feed it identity indices and a zero soup
    DevBuf dk, dv, dtr, dt, dp, dn, dts;
    HIPR(dk.alloc((size_t)n * 4));
    HIPR(dv.alloc((size_t)n * 4));
    HIPR(dtr.alloc((size_t)n * 36));
    HIPR(dt.alloc((size_t)n * 16));
    HIPR(dp.alloc((size_t)(2 * n - 1) * 4));
    HIPR(dn.alloc((size_t)(2 * n - 1) * 32));
    HIPR(dts.alloc((size_t)n * 48));
    std::vector<uint32_t> iota(n);
    for (uint32_t i = 0; i < n; ++i) iota[i] = i;
    HIPR(hipMemcpy(dk.p, sorted_keys, (size_t)n * 4, hipMemcpyHostToDevice));
    HIPR(hipMemcpy(dv.p, iota.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    HIPR(hipMemset(dtr.p, 0, (size_t)n * 36));
    HIPR(rt::launch_karras(dk.as<uint32_t>(), dv.as<uint32_t>(), dtr.as<float>(), n, dt.as<uint4>(), dp.as<uint32_t>(),
                           dn.p, dts.as<float4>(), 0));
    HIPR(hipDeviceSynchronize());
    if (topo && n > 1) HIPR(hipMemcpy(topo, dt.p, (size_t)(n - 1) * 16, hipMemcpyDeviceToHost));
    if (parent) HIPR(hipMemcpy(parent, dp.p, (size_t)(2 * n - 1) * 4, hipMemcpyDeviceToHost));
    if (leaf_esc) {
        std::vector<uint32_t> nd((size_t)n * 8);
        HIPR(hipMemcpy(nd.data(), (char*)dn.p + (size_t)(n - 1) * 32, (size_t)n * 32, hipMemcpyDeviceToHost));
        for (uint32_t k = 0; k < n; ++k) leaf_esc[k] = nd[(size_t)k * 8 + 7];
    }
    return RT_OK;
}

rt_status rt_stage_trace(int device, const rt_node* nodes, uint32_t n, const float* tris, const rt_camera* cam,
                         uint32_t w, uint32_t h, uint32_t spp, rt_hit* hits, uint8_t* rgba, uint64_t counters[2]) {
    if ((n && (!nodes || !tris)) || !cam || !w || !h || !spp) return fail(RT_EINVAL, "bad arguments");
    rt_status st = ensure_device(device);
    if (st) return st;
    const size_t tot = n ? 2 * (size_t)n - 1 : 1, nh = (size_t)w * h * spp;
    DevBuf dn, dt, dh, dr, dc;
    HIPR(dn.alloc(tot * 32));
    HIPR(dt.alloc((size_t)(n ? n : 1) * 36));
    HIPR(dh.alloc(nh * 16));
    HIPR(dr.alloc((size_t)w * h * 4));
    HIPR(dc.alloc(16));
    HIPR(hipMemset(dc.p, 0, 16));
    if (n) {
        HIPR(hipMemcpy(dn.p, nodes, tot * 32, hipMemcpyHostToDevice));
        HIPR(hipMemcpy(dt.p, tris, (size_t)n * 36, hipMemcpyHostToDevice));
    }
    DevBuf dts, dw;
    HIPR(dts.alloc((size_t)(n ? n : 1) * 48));
    HIPR(dw.alloc(4096));
    HIPR(rt::launch_leaf_tris(dn.p, dt.as<float>(), n, dts.as<float4>(), 0));
    HIPR(rt::launch_trace(dn.p, nullptr, dts.as<float4>(), n, camf(cam), w, h, spp, 0, 1, false, dh.p, dr.p,
                          counters ? dc.as<unsigned long long>() : nullptr, true, dw.as<uint32_t>(), nullptr, 0));
    HIPR(hipDeviceSynchronize());
    if (hits) HIPR(hipMemcpy(hits, dh.p, nh * 16, hipMemcpyDeviceToHost));
    if (rgba) HIPR(hipMemcpy(rgba, dr.p, (size_t)w * h * 4, hipMemcpyDeviceToHost));
    if (counters) HIPR(hipMemcpy(counters, dc.p, 16, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_stage_intersect(int device, uint32_t count, const float* o, const float* d, const float* tri,
                             const float* t_best, uint32_t* hit, float* tuv) {
    if (count && (!o || !d || !tri || !t_best || !hit || !tuv)) return fail(RT_EINVAL, "null argument");
    rt_status st = ensure_device(device);
    if (st) return st;
    if (!count) return RT_OK;
    DevBuf a, b, c, e, f, g;
    HIPR(a.alloc(count * 12ull));
    HIPR(b.alloc(count * 12ull));
    HIPR(c.alloc(count * 36ull));
    HIPR(e.alloc(count * 4ull));
    HIPR(f.alloc(count * 4ull));
    HIPR(g.alloc(count * 12ull));
    HIPR(hipMemcpy(a.p, o, count * 12ull, hipMemcpyHostToDevice));
    HIPR(hipMemcpy(b.p, d, count * 12ull, hipMemcpyHostToDevice));
    HIPR(hipMemcpy(c.p, tri, count * 36ull, hipMemcpyHostToDevice));
    HIPR(hipMemcpy(e.p, t_best, count * 4ull, hipMemcpyHostToDevice));
    HIPR(rt::launch_intersect(count, a.as<float>(), b.as<float>(), c.as<float>(), e.as<float>(), f.as<uint32_t>(),
                              g.as<float>(), 0));
    HIPR(hipDeviceSynchronize());
    HIPR(hipMemcpy(hit, f.p, count * 4ull, hipMemcpyDeviceToHost));
    HIPR(hipMemcpy(tuv, g.p, count * 12ull, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_stage_minmax(int device, uint32_t count, const float* a, const float* b, float* out) {
    if (count && (!a || !b || !out)) return fail(RT_EINVAL, "null argument");
    rt_status st = ensure_device(device);
    if (st) return st;
    if (!count) return RT_OK;
    DevBuf da, db, dout;
    HIPR(da.alloc(count * 4ull));
    HIPR(db.alloc(count * 4ull));
    HIPR(dout.alloc(count * 8ull));
    HIPR(hipMemcpy(da.p, a, count * 4ull, hipMemcpyHostToDevice));
    HIPR(hipMemcpy(db.p, b, count * 4ull, hipMemcpyHostToDevice));
    HIPR(rt::launch_minmax(count, da.as<float>(), db.as<float>(), dout.as<float>(), 0));
    HIPR(hipDeviceSynchronize());
    HIPR(hipMemcpy(out, dout.p, count * 8ull, hipMemcpyDeviceToHost));
    return RT_OK;
}

// ------------------------------------------------------------------ I/O
rt_status rt_framebuffer_dump_ppm(const uint8_t* rgba, uint32_t w, uint32_t h, const char* path) {
    if (!rgba || !path || !w || !h) return fail(RT_EINVAL, "bad arguments");
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(RT_EIO, std::string("cannot open ") + path);
    std::fprintf(f, "P6\n%u %u\n255\n", w, h);
    std::vector<uint8_t> row((size_t)w * 3);
    bool ok = true;
    for (uint32_t y = 0; y < h && ok; ++y) {
        for (uint32_t x = 0; x < w; ++x)
            for (int c = 0; c < 3; ++c) row[(size_t)x * 3 + c] = rgba[((size_t)y * w + x) * 4 + c];
        ok = std::fwrite(row.data(), 1, row.size(), f) == row.size();
    }
    if (std::fclose(f) != 0) ok = false;
    return ok ? RT_OK : fail(RT_EIO, std::string("write failed: ") + path);
}

rt_status rt_hits_dump(const rt_hit* hits, size_t count, const char* path) {
    if ((count && !hits) || !path) return fail(RT_EINVAL, "bad arguments");
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(RT_EIO, std::string("cannot open ") + path);
    bool ok = std::fwrite(hits, sizeof(rt_hit), count, f) == count;
    if (std::fclose(f) != 0) ok = false;
    return ok ? RT_OK : fail(RT_EIO, std::string("write failed: ") + path);
}

#ifdef RT_STAMPS
// diagnostic build only: copy the per-block phase stamps (8 x u64 per block)
// of the build kernels (which = 0) or the sort kernels (which = 1)
rt_status rt_debug_tile_order(const uint32_t* d_order) {
    rt::g_trace_config.order_override = d_order;
    return RT_OK;
}

rt_status rt_debug_stamps(int which, void* out, size_t bytes) {
    HIPR(hipDeviceSynchronize());
    HIPR(which == 2 ? rt::read_stamps_trace(out, bytes) : which ? rt::read_stamps_sort(out, bytes) : rt::read_stamps_build(out, bytes));
    return RT_OK;
}
#endif

}  // extern "C"

// rt_abi.cpp -- extern "C" boundary of librtamd.so (include/gpu_raytracer_amd.h).
//
// Host C++ around the gfx950 kernels: scene objects holding one BVH replica
// per device (the BVH is replicated, every device builds its
// own bit-identical copy), one HIP stream per replica, hipEvent timing, the
// in-library multi-GPU render (tiles dealt round-robin to the replicas, packed
// slabs gathered to the root with RCCL over xGMI, unpacked there), error
// mapping (HIP -> RT_EDEVICE, RCCL -> RT_ECOMM) and a thread-local error
// message.  There is no CPU compute path here: without a gfx950 device every
// compute entry point returns RT_EDEVICE.
#include "../../include/gpu_raytracer_amd.h"
#include "rt_device.h"
#include "rt_launch.h"

#include <dlfcn.h>
#include <rccl/rccl.h>  // types and prototypes only: RCCL is dlopen'ed on first multi-GPU use

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstddef>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <limits>
#include <vector>

namespace rtio {
bool load_obj(const char* path, std::vector<float>& tris, std::string& err);
bool load_soup(const char* path, std::vector<float>& tris, std::string& err);
bool save_soup(const char* path, const float* tris, uint64_t n, std::string& err);
void soup_generate(uint32_t n, uint64_t seed, float* tris);
}  // namespace rtio

namespace {

constexpr uint32_t kMaxDbuildRanks = 64;             // rt_dbuild_*: ranks of one distributed build
constexpr uint32_t kRefitLeaves = (uint32_t)rt::kRefitT;  // leaves per refit block (a share is whole blocks)

// One device's copy of a scene's BVH plus that device's render scratch.
// Tile-order state of one frame shape: the device maps (TileSched) and the
// shape they belong to.
struct SchedState {
    void* d = nullptr;  // [order][order next][cost A][cost B][cost mean] u32, [px A][px B] u16 x 256 per
                        // tile slot, then the heavy-ray queue
    size_t cap = 0;
    rt::TileSched sched;
    uint32_t key[5] = {0, 0, 0, 0, 0};  // w, h, spp, rank, nranks of the maps
};

struct Replica {
    int device = 0;
    hipStream_t stream = nullptr;  // the replica's own stream (builds, synchronous renders)
    rt::BuildBufs bufs;
    bool uploaded = false, built = false;
    uint32_t msb_probe = 0;  // the sort (1 MSB, 2 gather) whose verdict this build wrote (BuildBufs::sort_mode)
    bool fused = false;      // this build ran K0 + K1 fused (its barrier's timeout flag is in h_flag)
    uint32_t* h_flag = nullptr;  // mapped pinned host copy of zero[kZDense .. kZDense + 8): the build's verdict words
    uint32_t* d_flag = nullptr;  // its device-side address
    rt::BuildEvents ev;
    rt_build_times times{};
    // render scratch (grown on demand)
    void* d_hits = nullptr;
    size_t hits_cap = 0;
    void* d_rgba = nullptr;
    size_t rgba_cap = 0;
    unsigned long long* d_ctr = nullptr;
    SchedState ord;       // the frames' tile-order state (sched_for)
    SchedState ord_diag;  // scratch state of the counting launches: a diagnostic call never
                          // perturbs the next frame's order
    rt::PathBufs path;                        // wavefront path-mode state (grown on demand)
    hipEvent_t r0 = nullptr, r1 = nullptr;
    // multi-GPU render: this rank's packed slabs; the root's gathered slabs
    void* d_slab = nullptr;
    size_t slab_cap = 0;
    void* d_slab_hits = nullptr;
    size_t slab_hits_cap = 0;
    void* d_recv = nullptr;
    size_t recv_cap = 0;
    void* d_recv_hits = nullptr;
    size_t recv_hits_cap = 0;
    // Ordering of device work issued on caller streams (the *_device entry
    // points): every launch of this replica waits for the previous one when
    // it runs on another stream, and build / load / free wait for the last
    // one -- so a rebuild never overwrites, and a free never releases, buffers
    // a trace on a caller stream is still reading, and the tile-order maps
    // are written and read in launch order.
    hipEvent_t last = nullptr;
    hipStream_t last_stream = nullptr;  // stream `last` was recorded on (when last_pending; 0 = the null stream)
    bool last_pending = false;          // device work on a caller stream not yet ordered before the replica's own
    // distributed build (rt_dbuild_*): pair scratch and the crossing lists
    uint32_t* dk[2] = {nullptr, nullptr};
    uint32_t* dv[2] = {nullptr, nullptr};
    uint32_t* dcross = nullptr;      // this rank's crossing nodes, compacted
    uint32_t* dcross_all = nullptr;  // every rank's (gathered by the caller)
    float* dboxes = nullptr;         // every rank's centroid box
    uint32_t d_n = 0;                // n the scratch was sized for (0: none)
};

// RCCL communicators of one device list (rt_render(ngpus > 1)).
struct Comms {
    std::vector<int> devs;
    std::vector<ncclComm_t> comms;
};

}  // namespace

struct rt_scene {
    std::vector<float> tris;  // host copy, n*9
    uint32_t n = 0;
    int device = 0;                                 // the primary replica's device
    std::vector<std::unique_ptr<Replica>> reps;     // reps[0] = primary; rank r of a multi-GPU render = reps[r]
    Comms comm;
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

rt_status hip_status(hipError_t e, const char* where) { return e == hipSuccess ? RT_OK : hip_fail(e, where); }

#define HIPR(expr)                                          \
    do {                                                    \
        hipError_t _e = (expr);                             \
        if (_e != hipSuccess) return hip_fail(_e, #expr);   \
    } while (0)
#define RTR(expr)                  \
    do {                           \
        rt_status _s = (expr);     \
        if (_s != RT_OK) return _s; \
    } while (0)

int visible_devices() {
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess) return 0;
    return cnt;
}

rt_status ensure_device(int dev) {
    const int cnt = visible_devices();
    if (cnt == 0) return fail(RT_EDEVICE, "no HIP device available (librtamd has no CPU path)");
    if (dev < 0 || dev >= cnt) return fail(RT_EINVAL, "device index out of range");
    HIPR(hipSetDevice(dev));
    return RT_OK;
}

// ---- roctx ranges (SURVEY.md §5 "tracing": the entry points show up as
// named ranges in rocprofv3 --marker-trace).  Opt-in with RT_ROCTX=1: the
// roctx library is then dlopen'ed on first use; otherwise (and when it is
// absent) a range costs one branch.
struct Roctx {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
};

const Roctx& roctx() {
    static Roctx r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* e = std::getenv("RT_ROCTX");
        if (!e || std::strcmp(e, "1") != 0) return;
        void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        auto push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
        auto pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
        if (push && pop) {
            r.push = push;
            r.pop = pop;
        }
    });
    return r;
}

struct RtRange {
    bool on;
    explicit RtRange(const char* name) : on(roctx().push != nullptr) {
        if (on) roctx().push(name);
    }
    ~RtRange() {
        if (on) roctx().pop();
    }
    RtRange(const RtRange&) = delete;
    RtRange& operator=(const RtRange&) = delete;
};

// ---- RCCL, loaded on first use (a host that never renders on several GPUs
// never maps it).  An RCCL already in the process (e.g. torch's) is reused.
struct Rccl {
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGather) gather = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclCommCount) count = nullptr;
    decltype(&ncclCommUserRank) user_rank = nullptr;
    std::string why;  // load failure
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = RTLD_DEFAULT;
        if (!dlsym(h, "ncclGather")) {
            h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
            if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        }
        if (!h) {
            const char* e = dlerror();
            r.why = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
            return;
        }
        r.init_all = reinterpret_cast<decltype(r.init_all)>(dlsym(h, "ncclCommInitAll"));
        r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(h, "ncclCommDestroy"));
        r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
        r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
        r.gather = reinterpret_cast<decltype(r.gather)>(dlsym(h, "ncclGather"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
        r.count = reinterpret_cast<decltype(r.count)>(dlsym(h, "ncclCommCount"));
        r.user_rank = reinterpret_cast<decltype(r.user_rank)>(dlsym(h, "ncclCommUserRank"));
        if (!r.init_all || !r.destroy || !r.group_start || !r.group_end || !r.gather || !r.error_string ||
            !r.count || !r.user_rank) {
            r.init_all = nullptr;
            r.why = "librccl.so.1 lacks ncclCommInitAll/ncclGather";
        }
    });
    return r;
}

rt_status nccl_fail(ncclResult_t e, const char* where) {
    const Rccl& R = rccl();
    return fail(RT_ECOMM, std::string(where) + ": " + (R.error_string ? R.error_string(e) : "RCCL error"));
}

#define NCCLR(expr)                                           \
    do {                                                      \
        ncclResult_t _r = (expr);                             \
        if (_r != ncclSuccess) return nccl_fail(_r, #expr);   \
    } while (0)

void free_comms(Comms& c) {
    const Rccl& R = rccl();
    for (ncclComm_t cm : c.comms)
        if (cm && R.destroy) (void)R.destroy(cm);
    c.comms.clear();
    c.devs.clear();
}

// ---- replicas
rt_status replica_init(Replica& r) {
    RTR(ensure_device(r.device));
    if (r.stream) return RT_OK;
    HIPR(hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking));
    // timing-only events: no system-scope fence (L2 writeback + invalidate)
    // at each record, which would add ~4.7 us per event to the GPU timeline
    // between the kernels being timed.  Every host read of results goes
    // through a stream synchronize or a blocking copy.
    const unsigned fl = hipEventDisableSystemFence;
    for (auto& e : r.ev.e) HIPR(hipEventCreateWithFlags(&e, fl));
    r.ev.valid = true;
    HIPR(hipEventCreateWithFlags(&r.r0, fl));
    HIPR(hipEventCreateWithFlags(&r.r1, fl));
    HIPR(hipEventCreateWithFlags(&r.last, hipEventDisableTiming | hipEventDisableSystemFence));
    return RT_OK;
}

void replica_free(Replica& r) {
    if (!r.stream) return;
    (void)hipSetDevice(r.device);
    if (r.last_pending) (void)hipEventSynchronize(r.last);  // device work on a caller stream
    (void)hipStreamSynchronize(r.stream);
    for (SchedState* o : {&r.ord, &r.ord_diag}) {  // the queue-skip words
        if (o->sched.q_host) (void)hipHostFree(o->sched.q_host);
        o->sched.q_host = o->sched.q_dev = nullptr;
    }
    rt::free_build(r.bufs);
    rt::free_path(r.path);
    for (void* p : {r.d_hits, r.d_rgba, (void*)r.d_ctr, r.ord.d, r.ord_diag.d, r.d_slab, r.d_slab_hits, r.d_recv,
                    r.d_recv_hits, (void*)r.dk[0], (void*)r.dk[1], (void*)r.dv[0], (void*)r.dv[1], (void*)r.dcross,
                    (void*)r.dcross_all, (void*)r.dboxes})
        if (p) (void)hipFree(p);
    for (auto& e : r.ev.e) (void)hipEventDestroy(e);
    (void)hipEventDestroy(r.r0);
    (void)hipEventDestroy(r.r1);
    (void)hipEventDestroy(r.last);
    if (r.h_flag) (void)hipHostFree(r.h_flag);
    r.h_flag = nullptr;
    (void)hipStreamDestroy(r.stream);
    r.stream = nullptr;
}

// the primary replica (created on the scene's device on first use)
rt_status primary(rt_scene* s, Replica** out) {
    if (s->reps.empty()) {
        std::unique_ptr<Replica> r(new (std::nothrow) Replica);
        if (!r) return fail(RT_ENOMEM, "host allocation failed");
        r->device = s->device;
        s->reps.push_back(std::move(r));
    }
    Replica* r = s->reps[0].get();
    RTR(replica_init(*r));
    *out = r;
    return RT_OK;
}

// record arity of the next build of an n-triangle scene (build.wide_arity;
// the 8-ary records' 32-bit buffer offsets need n <= kWide8MaxN) and record size
static_assert(rt::kWide8MaxN == RT_WIDE8_MAX_N, "header and library agree on the 8-ary size cap");
uint32_t build_arity(uint32_t n) { return (rt::config_snapshot().wide_arity == 8 && n <= rt::kWide8MaxN) ? 8u : 4u; }
uint64_t wide_bytes(uint32_t arity) { return arity == 8 ? 96u : 64u; }

// Write the binary leaf nodes from the triangle records (the build writes
// internal nodes only: store_leaf_tri) for readers of the whole node array
// (rt_bvh_read, rt_bvh_save); the trace never reads them.
rt_status materialize_leaves(Replica& r, uint32_t n) {
    HIPR(hipSetDevice(r.device));
    HIPR(rt::launch_leaf_nodes(r.bufs.tri_s, n, r.bufs.nodes, r.stream));
    HIPR(hipStreamSynchronize(r.stream));
    return RT_OK;
}

Replica* primary_built(const rt_scene* s) {
    return (!s->reps.empty() && s->reps[0]->built) ? s->reps[0].get() : nullptr;
}

// Before device work on stream hs: order it after this replica's previous
// device work when that ran on another stream.
rt_status order_before(Replica& r, hipStream_t hs) {
    if (r.last_pending && r.last_stream != hs) HIPR(hipStreamWaitEvent(hs, r.last, 0));
    return RT_OK;
}
// After device work on a caller stream hs: remember it (see Replica::last).
rt_status order_after(Replica& r, hipStream_t hs) {
    if (hs == r.stream) {
        r.last_pending = false;  // the replica's own stream orders itself
        return RT_OK;
    }
    HIPR(hipEventRecord(r.last, hs));
    r.last_stream = hs;
    r.last_pending = true;
    return RT_OK;
}
// Before the replica's own stream rewrites or frees its buffers.
rt_status join_caller_work(Replica& r) {
    if (r.last_pending) {
        HIPR(hipStreamWaitEvent(r.stream, r.last, 0));
        r.last_pending = false;
    }
    return RT_OK;
}

rt_status upload(const rt_scene* s, Replica& r) {
    RTR(replica_init(r));
    if (r.uploaded) return RT_OK;
    if (r.bufs.cap_n != s->n || !r.bufs.tris) {
        hipError_t e = rt::alloc_build(r.bufs, s->n);
        if (e == hipErrorOutOfMemory) return fail(RT_ENOMEM, "device allocation failed");
        if (e != hipSuccess) return hip_fail(e, "alloc_build");
    }
    if (s->n) HIPR(hipMemcpyAsync(r.bufs.tris, s->tris.data(), (size_t)s->n * 36, hipMemcpyHostToDevice, r.stream));
    HIPR(hipStreamSynchronize(r.stream));
    r.uploaded = true;
    return RT_OK;
}

// Build the BVH on every replica in `targets` concurrently (one stream each),
// then wait for all; ms_out = the longest build.
rt_status build_replicas(rt_scene* s, const std::vector<Replica*>& targets, double* ms_out) {
    // one config snapshot for every replica and both halves of the probe
    // logic (a concurrent rt_config_set between two snapshots
    // could make the host read a verdict no kernel wrote)
    const rt::TraceConfig cfg = rt::config_snapshot();
    const bool stages = cfg.stage_events != 0;
    // K0 + K1 fused (a grid barrier over co-resident blocks): only for a
    // replica alone on its device in this call that also wins its device's
    // fused gate, held until the build has finished -- two fused grids that
    // share a device could each wait for blocks the other holds
    std::vector<std::unique_lock<std::mutex>> gates;
    for (Replica* r : targets) {
        RTR(upload(s, *r));
        HIPR(hipSetDevice(r->device));
        RTR(join_caller_work(*r));
        r->bufs.warity = build_arity(s->n);
        // a rebuild that fails half-way must not leave the old flag over a
        // half-written BVH: built again only after the synchronize below
        r->built = false;
        bool alone = true;
        for (Replica* o : targets) alone = alone && (o == r || o->device != r->device);
        bool allow = false;
        if (alone && cfg.fuse_k01) {
            std::unique_lock<std::mutex> g(rt::fused_gate(r->device), std::try_to_lock);
            if (g.owns_lock()) {
                gates.push_back(std::move(g));
                allow = true;
            }
        }
        if (!r->h_flag) {
            HIPR(hipHostMalloc(reinterpret_cast<void**>(&r->h_flag), 32, hipHostMallocMapped));
            HIPR(hipHostGetDevicePointer(reinterpret_cast<void**>(&r->d_flag), r->h_flag, 0));
        }
        for (int i = 0; i < 8; ++i) r->h_flag[i] = 0;
        // the build's verdict words land in h_flag (written by its last
        // kernels, read after the synchronize below: no copy launch)
        hipError_t e = rt::launch_build(r->bufs, s->n, r->stream, &r->ev, stages, cfg, &r->msb_probe, allow,
                                        &r->fused, r->d_flag);
        if (e != hipSuccess) return hip_fail(e, "launch_build");
    }
    // Every replica is synchronized and checked before anything returns
    // (an early return left later replicas' flags unread while
    // their fused grids could still run after the gates were released).
    // (the synchronize loop itself must not return early either:
    // an error on one replica is recorded and the others are still waited for,
    // so no fused grid outlives the gates released on return)
    rt_status first_err = RT_OK;
    double worst = 0.0;
    std::vector<char> synced(targets.size(), 0);
    for (size_t i = 0; i < targets.size(); ++i) {
        Replica* r = targets[i];
        hipError_t e = hipSetDevice(r->device);
        if (e == hipSuccess) e = hipStreamSynchronize(r->stream);
        if (e != hipSuccess) {
            if (first_err == RT_OK) first_err = hip_fail(e, "synchronize build");
            continue;
        }
        synced[i] = 1;
    }
    // stage times of the build just synchronized; the total is what this
    // call spent on the replica: a discarded build's time is added to its redo
    auto read_times = [&](Replica* r, double spent_before) -> rt_status {
        float t[6] = {0, 0, 0, 0, 0, 0};
        if (stages)
            for (int i = 0; i < 6; ++i) HIPR(hipEventElapsedTime(&t[i], r->ev.e[i], r->ev.e[i + 1]));
        r->times.bounds = t[0];
        r->times.morton = t[1];
        r->times.sort = t[2];
        r->times.topology = t[3];
        r->times.refit = t[4];
        r->times.wide = t[5];
        float tot = 0;
        HIPR(hipEventElapsedTime(&tot, r->ev.e[0], r->ev.e[6]));
        r->times.total = spent_before + tot;
        return RT_OK;
    };
    for (size_t ri = 0; ri < targets.size(); ++ri) {
        Replica* r = targets[ri];
        if (!synced[ri]) continue;  // its error is already recorded
        if (rt_status st = hip_status(hipSetDevice(r->device), "hipSetDevice"); st != RT_OK) {
            if (first_err == RT_OK) first_err = st;
            continue;
        }
        if (rt_status st = read_times(r, 0.0); st != RT_OK) {
            if (first_err == RT_OK) first_err = st;
            continue;
        }
        const uint32_t* hf = r->h_flag;  // [0] dense, [1] clustered bins, [2] bucket overflow, [3] skewed, [5] barrier timeout
        r->times.fused_fallback = 0u;
        r->times.lsb_redo = 0u;
        if (r->fused && hf[rt::kZFuseErr - rt::kZDense]) {
            // A block of the fused grid gave up at the barrier: the grid was
            // not co-resident (another tenant held CUs).  Its later kernels
            // ran in bounds on a wrong box, so the build is discarded and
            // redone here with the two-launch K0 + K1 (VERDICT r04 item 3;
            // times.fused_fallback reports it).  The word lies past kZEnd
            // (no build zeroes it), so it is cleared first.
            if (rt_status st = hip_status(hipMemsetAsync(r->bufs.zero + rt::kZFuseErr, 0, 4, r->stream),
                                          "clear barrier flag");
                st != RT_OK) {
                if (first_err == RT_OK) first_err = st;
                continue;
            }
            const double spent = r->times.total;
            for (int i = 0; i < 8; ++i) r->h_flag[i] = 0;
            hipError_t e = rt::launch_build(r->bufs, s->n, r->stream, &r->ev, stages, cfg, &r->msb_probe, false,
                                            &r->fused, r->d_flag);
            if (e == hipSuccess) e = hipStreamSynchronize(r->stream);
            if (e != hipSuccess) {
                if (first_err == RT_OK) first_err = hip_fail(e, "launch_build (unfused redo)");
                continue;
            }
            if (rt_status st = read_times(r, spent); st != RT_OK) {
                if (first_err == RT_OK) first_err = st;
                continue;
            }
            r->times.fused_fallback = 1u;
        }
        const uint32_t kind = rt::build_sort_kind(r->bufs, s->n, cfg);
        if (kind == 2 && (hf[rt::kZGatherFlags + 1 - rt::kZDense] || cfg.force_lsb_redo)) {
            // a bucket outgrew its block's LDS (the verdict should have sent
            // this scene to the LSB sort): that bucket is unsorted -- keep
            // the LSB sort for this scene and build again with it
            // (debug.force_lsb_redo takes this branch for the tests)
            r->bufs.sort_mode = 2;
            r->bufs.sort_mode_of = kind;
            r->msb_probe = 0;
            const double spent = r->times.total;
            hipError_t e = rt::launch_build(r->bufs, s->n, r->stream, &r->ev, stages, cfg, nullptr, false, &r->fused);
            if (e == hipSuccess) e = hipStreamSynchronize(r->stream);
            if (e != hipSuccess) {
                if (first_err == RT_OK) first_err = hip_fail(e, "launch_build (LSB)");
                continue;
            }
            if (rt_status st = read_times(r, spent); st != RT_OK) {
                if (first_err == RT_OK) first_err = st;
                continue;
            }
            r->times.lsb_redo = 1u;
        } else if (r->msb_probe) {  // the scene's first build with this sort ran both sorts gated on its verdict
            const bool dense = hf[0] != 0;
            const bool clustered = r->msb_probe == 2 && hf[rt::kZGatherFlags - rt::kZDense] != 0;
            const bool skewed = r->msb_probe == 2 && hf[rt::kZGatherSkew - rt::kZDense] != 0;
            if ((clustered || skewed) && !dense) {
                r->bufs.gather_off = 1u;  // the next build probes the MSB sort (BuildBufs::gather_off)
            } else {
                r->bufs.sort_mode = dense || clustered ? 2u : 1u;
                r->bufs.sort_mode_of = r->msb_probe;
            }
            r->msb_probe = 0;
        }
        r->times.sort_kind = rt::build_sort_kind(r->bufs, s->n, cfg);
        r->times.fused_k01 = r->fused ? 1u : 0u;
        r->built = true;
        worst = std::max(worst, r->times.total);
    }
    if (first_err != RT_OK) return first_err;
    if (ms_out) *ms_out = worst;
    return RT_OK;
}

rt_status grow(void** p, size_t* cap, size_t need) {
    if (*cap >= need && *p) return RT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = rt::dev_alloc(p, need);
    if (e == hipErrorOutOfMemory) return fail(RT_ENOMEM, "device allocation failed");
    if (e != hipSuccess) return hip_fail(e, "hipMalloc");
    *cap = need;
    return RT_OK;
}

// Tile-order state for a frame of this shape (DESIGN.md "Tile order"): the
// cost map of the previous frame with the same w, h, spp, rank, nranks
// drives this frame's dispatch order.  A failed allocation is reported
// (RT_ENOMEM / RT_EDEVICE), never silently replaced by row-major order.
rt_status sched_for(SchedState& r, uint32_t w, uint32_t h, uint32_t spp, uint32_t rank, uint32_t nranks,
                    rt::TileSched** out) {
    const uint32_t nb = rt::tiles_for_rank(w, h, rank, nranks);
    const uint32_t key[5] = {w, h, spp, rank, nranks};
    const bool same = std::memcmp(key, r.key, sizeof(key)) == 0;
    // [order][order next][cost A][cost B][cost mean] u32, [px A][px B] u16 x 256 per tile slot,
    // then (trace.coop_cap) 2 queue counters and the heavy-ray queue
    const rt::TraceConfig cfg = rt::config_snapshot();
    // (64 shards of equal size, 2 x 64 counters)
    const uint32_t qcap = (cfg.coop_cap || cfg.coop_cap_tiles) ? (cfg.coop_max + 63u) & ~63u : 0u;
    const size_t maps = 5ull * nb * 4 + 2ull * nb * 512;
    const size_t qoff = (maps + 255) & ~size_t(255);
    const size_t need = qcap ? qoff + 512 + (size_t)rt::kCoopEntryBytes * qcap : maps;
    if (!r.sched.q_host) {  // the queue skip's queue-length word
        HIPR(hipHostMalloc(reinterpret_cast<void**>(&r.sched.q_host), 64, hipHostMallocMapped));
        HIPR(hipHostGetDevicePointer(reinterpret_cast<void**>(&r.sched.q_dev), r.sched.q_host, 0));
        __atomic_store_n(r.sched.q_host, ~0u, __ATOMIC_RELAXED);
    }
    if (!same || r.cap < need || r.sched.coop_qcap != qcap) {
        std::memset(r.key, 0, sizeof(r.key));  // invalid until the maps exist
        __atomic_store_n(r.sched.q_host, ~0u, __ATOMIC_RELAXED);  // a new shape: its queue length not yet known
        r.sched.q_frames = 0;
        RTR(grow(&r.d, &r.cap, need));
        uint32_t* b = static_cast<uint32_t*>(r.d);
        r.sched.order = b;
        r.sched.order_next = b + nb;
        r.sched.cost_prev = b + 2 * nb;
        r.sched.cost_cur = b + 3 * nb;
        r.sched.cost_ema = b + 4 * nb;
        r.sched.px_prev = reinterpret_cast<uint16_t*>(b + 5 * nb);
        r.sched.px_cur = r.sched.px_prev + (size_t)nb * 256;
        char* qb = static_cast<char*>(r.d) + qoff;
        r.sched.coop_ctr = qcap ? reinterpret_cast<uint32_t*>(qb) : nullptr;
        r.sched.coop_q = qcap ? reinterpret_cast<uint4*>(qb + 512) : nullptr;
        r.sched.coop_qcap = qcap;
        r.sched.coop_par = 0;
        r.sched.coop_fresh = true;
        r.sched.prev_cam_valid = false;
        r.sched.have_prev = false;
        r.sched.order_ready = false;
        r.sched.fresh = true;
        std::memcpy(r.key, key, sizeof(key));
    }
    *out = &r.sched;
    return RT_OK;
}

// after a launch that used sched_for: this frame's map becomes the previous one
void sched_done(SchedState& r, const rt::TraceConfig& cfg) {
    if (!cfg.tile_order) return;
    std::swap(r.sched.cost_prev, r.sched.cost_cur);
    std::swap(r.sched.px_prev, r.sched.px_cur);
    r.sched.have_prev = true;
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
    hipError_t alloc(size_t bytes) { return rt::dev_alloc(&p, bytes); }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

rt_status check_frame(uint32_t w, uint32_t h, uint32_t spp) {
    if (!w || !h || !spp) return fail(RT_EINVAL, "bad render arguments");
    if ((uint64_t)w * h * spp > 0xFFFFFFFFull) return fail(RT_EINVAL, "w*h*spp exceeds 2^32 samples");
    return RT_OK;
}

rt_status need_built(rt_scene* s, Replica** out) {
    if (!primary_built(s)) return fail(RT_EINVAL, "scene not built (call rt_bvh_build)");
    return primary(s, out);
}

bool apply_config(rt::TraceConfig& c, const char* key, int64_t value) {
    const std::string k(key);
    if (k == "trace.variant" && (value == 0 || value == 2)) c.variant = (uint32_t)value;
    else if (k == "trace.stack_cap" && value >= 0 && value <= rt::kWideStackMax) c.stack_cap = (uint32_t)value;
    else if (k == "trace.wg" && (value == 64 || value == 256)) c.wg = (uint32_t)value;
    else if (k == "trace.wg_tiles" && (value == 64 || value == 256)) c.wg_tiles = (uint32_t)value;
    else if (k == "trace.tile_order" && (value == 0 || value == 1)) c.tile_order = (uint32_t)value;
    else if (k == "trace.px_sort" && value >= 0 && value <= 2) c.px_sort = (uint32_t)value;
    else if (k == "trace.spp_lanes" && value >= 0 && value <= 2) c.spp_lanes = (uint32_t)value;
    else if (k == "build.sort" && value >= 0 && value <= 2) c.sort_msb = (uint32_t)value;
    else if (k == "build.fuse_k01" && value >= 0 && value <= 2) c.fuse_k01 = (uint32_t)value;
    else if (k == "build.wide_arity" && (value == 4 || value == 8)) c.wide_arity = (uint32_t)value;
    else if (k == "build.stage_events" && (value == 0 || value == 1)) c.stage_events = (uint32_t)value;
    else if (k == "path.wavefront" && (value == 0 || value == 1)) c.path_wave = (uint32_t)value;
    else if (k == "path.wg" && (value == 64 || value == 256)) c.path_wg = (uint32_t)value;
    else if (k == "path.sort" && value >= 0 && value <= 4) c.path_sort = (uint32_t)value;
    else if (k == "path.batch" && value >= 0 && value <= (1 << 28)) c.path_batch = (uint32_t)value;
    else if (k == "render.emulate" && (value == 0 || value == 1)) c.render_emulate = (uint32_t)value;
    else if (k == "render.rccl1" && (value == 0 || value == 1)) c.render_rccl1 = (uint32_t)value;
    else if (k == "trace.coop_cap" && value >= -1 && value <= (1 << 20))
        c.coop_cap = value < 0 ? rt::kCoopCapAuto : (uint32_t)value;
    else if (k == "trace.coop_cap_tiles" && value >= -1 && value <= (1 << 20))
        c.coop_cap_tiles = value < 0 ? rt::kCoopCapAuto : (uint32_t)value;
    else if (k == "trace.coop_lanes" && (value == 16 || value == 32 || value == 64)) c.coop_lanes = (uint32_t)value;
    else if (k == "trace.coop_max" && value >= 1 && value <= (1 << 24)) c.coop_max = (uint32_t)value;
    else if (k == "debug.poison" && (value == 0 || value == 1)) c.poison = (uint32_t)value;
    else if (k == "debug.lds_scribble" && (value == 0 || value == 1)) c.lds_scribble = (uint32_t)value;
    else if (k == "debug.force_lsb_redo" && (value == 0 || value == 1)) c.force_lsb_redo = (uint32_t)value;
    else return false;
    return true;
}

}  // namespace

extern "C" {

const char* rt_last_error(void) { return g_err.c_str(); }
const char* rt_version(void) { return "gpu_raytracer_amd 0.4 (gfx950)"; }

rt_status rt_config_set(const char* key, int64_t value) {
    if (!key) return fail(RT_EINVAL, "null key");
    if (!rt::config_apply(apply_config, key, value))
        return fail(RT_EINVAL, std::string("unknown config key or value out of range: ") + key);
    return RT_OK;
}

int rt_device_count(void) { return visible_devices(); }

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
    if (!s->reps.empty()) return fail(RT_EINVAL, "device must be set before the first build");
    if (device < 0) return fail(RT_EINVAL, "device index out of range");
    s->device = device;
    return RT_OK;
}

void rt_scene_free(rt_scene* s) {
    if (!s) return;
    for (auto& r : s->reps) replica_free(*r);
    free_comms(s->comm);
    delete s;
}

rt_status rt_scene_stream(rt_scene* s, void** stream_out) {
    if (!s || !stream_out) return fail(RT_EINVAL, "null argument");
    Replica* r = nullptr;
    RTR(primary(s, &r));
    *stream_out = (void*)r->stream;
    return RT_OK;
}

rt_status rt_scene_sync(rt_scene* s) {
    if (!s) return fail(RT_EINVAL, "null argument");
    for (auto& r : s->reps) {
        if (!r->stream) continue;
        HIPR(hipSetDevice(r->device));
        if (r->last_pending) HIPR(hipEventSynchronize(r->last));
        HIPR(hipStreamSynchronize(r->stream));
    }
    return RT_OK;
}

// ------------------------------------------------------------------ camera
// f = normalize(at-eye), r = normalize(f x up), u = r x f;
// w00 = f + u*tan - r*tan*aspect; du = r*(2 tan aspect/W); dv = -u*(2 tan/H).
rt_status rt_camera_look_at(const double eye[3], const double at[3], const double up[3], double vfov_deg,
                            uint32_t w, uint32_t h, rt_camera* out) {
    if (!eye || !at || !up || !out || !w || !h) return fail(RT_EINVAL, "bad camera arguments");
    double f[3] = {at[0] - eye[0], at[1] - eye[1], at[2] - eye[2]};
    // a degenerate frame (eye == at, up parallel to the view direction,
    // non-finite inputs) has no basis: refused rather than NaN rays
    auto norm = [](double* v) {
        const double l = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        if (!(l > 0.0) || !std::isfinite(l)) return false;
        v[0] /= l; v[1] /= l; v[2] /= l;
        return true;
    };
    auto cross = [](const double* a, const double* b, double* o) {
        o[0] = a[1] * b[2] - a[2] * b[1];
        o[1] = a[2] * b[0] - a[0] * b[2];
        o[2] = a[0] * b[1] - a[1] * b[0];
    };
    if (!(vfov_deg > 0.0 && vfov_deg < 180.0)) return fail(RT_EINVAL, "camera: vfov outside (0, 180)");
    if (!norm(f)) return fail(RT_EINVAL, "camera: eye == at or non-finite");
    double r[3], u[3];
    cross(f, up, r);
    if (!norm(r)) return fail(RT_EINVAL, "camera: up parallel to the view direction");
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
rt_status rt_bvh_build(rt_scene* s, int backend, uint32_t device_mask, double* ms_out) {
    RtRange range_("rt_bvh_build");
    if (!s) return fail(RT_EINVAL, "null scene");
    if (backend == RT_BACKEND_CPU)
        return fail(RT_EINVAL, "librtamd has no CPU backend (the CPU oracle under oracle/ is test infrastructure)");
    if (backend != RT_BACKEND_HIP) return fail(RT_EINVAL, "unknown backend");
    const int cnt = visible_devices();
    if (cnt == 0) return fail(RT_EDEVICE, "no HIP device available (librtamd has no CPU path)");
    if (cnt < 32 && (device_mask >> cnt)) return fail(RT_EDEVICE, "device_mask names a device that is not visible");
    std::vector<Replica*> targets;
    if (!device_mask) {
        Replica* r = nullptr;
        RTR(primary(s, &r));
        targets.push_back(r);
    } else {
        for (int d = 0; d < 32; ++d) {
            if (!((device_mask >> d) & 1u)) continue;
            if (s->reps.empty()) s->device = d;  // the lowest device of the first build is the primary
            Replica* found = nullptr;
            for (auto& r : s->reps)
                if (r->device == d) { found = r.get(); break; }
            if (!found) {
                std::unique_ptr<Replica> r(new (std::nothrow) Replica);
                if (!r) return fail(RT_ENOMEM, "host allocation failed");
                r->device = d;
                found = r.get();
                s->reps.push_back(std::move(r));
            }
            targets.push_back(found);
        }
    }
    return build_replicas(s, targets, ms_out);
}

rt_status rt_bvh_build_times(const rt_scene* s, rt_build_times* out) {
    if (!s || !out) return fail(RT_EINVAL, "null argument");
    const Replica* r = primary_built(s);
    if (!r) return fail(RT_EINVAL, "scene not built");
    *out = r->times;
    return RT_OK;
}

// the struct grew in 0.3 and carries no size of its own, so a
// caller states the size it was compiled with; the prefix that fits is
// written (never past out_size).  The 0.2 layout (64 B: seven doubles and
// sort_kind / fused_k01) is the smallest accepted.
rt_status rt_bvh_build_times_sized(const rt_scene* s, rt_build_times* out, size_t out_size) {
    if (!s || !out) return fail(RT_EINVAL, "null argument");
    if (out_size < offsetof(rt_build_times, fused_fallback))
        return fail(RT_EINVAL, "rt_build_times smaller than the 0.2 layout");
    const Replica* r = primary_built(s);
    if (!r) return fail(RT_EINVAL, "scene not built");
    std::memcpy(out, &r->times, std::min(out_size, sizeof(rt_build_times)));
    return RT_OK;
}

rt_status rt_bvh_read(const rt_scene* s, rt_node* nodes, uint32_t* keys, uint32_t* vals, uint32_t* parent,
                      float* bounds9) {
    if (!s) return fail(RT_EINVAL, "null scene");
    Replica* r = primary_built(s);
    if (!r) return fail(RT_EINVAL, "scene not built");
    HIPR(hipSetDevice(r->device));
    if (r->last_pending) HIPR(hipEventSynchronize(r->last));
    HIPR(hipStreamSynchronize(r->stream));
    const size_t n = s->n, tot = n ? 2 * n - 1 : 0;
    RTR(materialize_leaves(*r, s->n));
    if (nodes && tot) HIPR(hipMemcpy(nodes, r->bufs.nodes, tot * 32, hipMemcpyDeviceToHost));
    if (keys && n) HIPR(hipMemcpy(keys, r->bufs.keys[0], n * 4, hipMemcpyDeviceToHost));
    if (vals && n) HIPR(hipMemcpy(vals, r->bufs.vals[0], n * 4, hipMemcpyDeviceToHost));
    if (parent && tot) {
        // derived here from the nodes (the build does not write parents:
        // nothing on the trace path reads them): the children of internal
        // node i are a = left and the left child's escape link (a left
        // child's escape is its right sibling, §9.6)
        std::vector<rt_node> nd;
        const rt_node* np = nodes;
        if (!np) {
            nd.resize(tot);
            HIPR(hipMemcpy(nd.data(), r->bufs.nodes, tot * 32, hipMemcpyDeviceToHost));
            np = nd.data();
        }
        std::fill(parent, parent + tot, RT_SENTINEL);
        for (size_t i = 0; i + 1 < n; ++i) {
            const uint32_t a = np[i].a;
            if (a >= tot) continue;  // malformed: leave the sentinel
            const uint32_t b = np[a].esc;
            parent[a] = (uint32_t)i;
            if (b < tot) parent[b] = (uint32_t)i;
        }
    }
    if (bounds9) HIPR(hipMemcpy(bounds9, r->bufs.params, 9 * 4, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_bvh_read_wide(const rt_scene* s, void* records) {
    if (!s || !records) return fail(RT_EINVAL, "null argument");
    Replica* r = primary_built(s);
    if (!r) return fail(RT_EINVAL, "scene not built");
    HIPR(hipSetDevice(r->device));
    HIPR(hipStreamSynchronize(r->stream));
    if (s->n >= 2)
        HIPR(hipMemcpy(records, r->bufs.wnodes, (size_t)(s->n - 1) * wide_bytes(r->bufs.warity),
                       hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_bvh_wide_arity(const rt_scene* s, uint32_t* arity_out) {
    if (!s || !arity_out) return fail(RT_EINVAL, "null argument");
    const Replica* r = primary_built(s);
    if (!r) return fail(RT_EINVAL, "scene not built");
    *arity_out = r->bufs.warity;
    return RT_OK;
}

rt_status rt_bvh_replicas(const rt_scene* s, uint32_t max, int* devices, uint32_t* count_out) {
    if (!s || !count_out || (max && !devices)) return fail(RT_EINVAL, "null argument");
    uint32_t c = 0;
    for (auto& r : s->reps) {
        if (!r->built) continue;
        if (c < max) devices[c] = r->device;
        ++c;
    }
    *count_out = c;
    return RT_OK;
}

// ------------------------------------------------------------------ BVH cache
// RTBVH1: "RTBVH1\0\0", u32 version, u32 n, u64 FNV-1a hash of the n*36
// triangle bytes, u64 layout tag, then the device buffers the trace and
// rt_bvh_read use, in order: BuildParams (64 B), sorted keys and vals (n x 4),
// nodes ((2n-1) x 32), tri_s (n x 48), wide records ((n-1) x 64).  The tag
// changes whenever one of those layouts does (revision 2: no parent section;
// 3: triangle records carry the leaf escape link).
}  // extern "C"

namespace {
const char kBvhMagic[8] = {'R', 'T', 'B', 'V', 'H', '1', 0, 0};
constexpr uint32_t kBvhVersion = 1;
constexpr uint64_t kBvhLayout = 0x7274616d64000003ull;   // "rtamd" + layout revision 3 (4-ary records)
constexpr uint64_t kBvhLayout8 = 0x7274616d64000083ull;  // the same with 8-ary (K7w8) records

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

std::vector<BvhSection> bvh_sections(const rt_scene* s, const Replica& r) {
    const size_t n = s->n, tot = n ? 2 * n - 1 : 0;
    static_assert(sizeof(rt::BuildParams) == 64, "RTBVH1 stores a 64-B BuildParams");
    return {{r.bufs.params, sizeof(rt::BuildParams)},
            {r.bufs.keys[0], n * 4},
            {r.bufs.vals[0], n * 4},
            {r.bufs.nodes, tot * 32},
            {r.bufs.tri_s, n * 48},
            {r.bufs.wnodes, n >= 2 ? (n - 1) * wide_bytes(r.bufs.warity) : 0}};
}

struct File {
    FILE* f = nullptr;
    ~File() {
        if (f) std::fclose(f);
    }
};
}  // namespace

extern "C" {

rt_status rt_bvh_save(const rt_scene* s, const char* path) {
    if (!s || !path) return fail(RT_EINVAL, "null argument");
    Replica* r = primary_built(s);
    if (!r) return fail(RT_EINVAL, "scene not built");
    HIPR(hipSetDevice(r->device));
    HIPR(hipStreamSynchronize(r->stream));
    RTR(materialize_leaves(*r, s->n));
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(RT_EIO, std::string("cannot create ") + path);
    const uint32_t hv[2] = {kBvhVersion, s->n};
    const uint64_t hh[2] = {fnv1a(s->tris.data(), s->tris.size() * sizeof(float)),
                            r->bufs.warity == 8 ? kBvhLayout8 : kBvhLayout};
    bool ok = std::fwrite(kBvhMagic, 1, 8, f) == 8 && std::fwrite(hv, 4, 2, f) == 2 && std::fwrite(hh, 8, 2, f) == 2;
    std::vector<unsigned char> host;
    for (const BvhSection& sec : bvh_sections(s, *r)) {
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
    File f;
    f.f = std::fopen(path, "rb");
    if (!f.f) return fail(RT_EIO, std::string("cannot open ") + path);
    char magic[8];
    uint32_t hv[2] = {0, 0};
    uint64_t hh[2] = {0, 0};
    const bool hdr =
        std::fread(magic, 1, 8, f.f) == 8 && std::fread(hv, 4, 2, f.f) == 2 && std::fread(hh, 8, 2, f.f) == 2;
    if (!hdr || std::memcmp(magic, kBvhMagic, 8) != 0) return fail(RT_EIO, std::string(path) + ": not an RTBVH1 file");
    if (hv[0] != kBvhVersion || (hh[1] != kBvhLayout && hh[1] != kBvhLayout8))
        return fail(RT_EIO, std::string(path) + ": BVH cache from another library layout");
    if (hv[1] != s->n || hh[0] != fnv1a(s->tris.data(), s->tris.size() * sizeof(float)))
        return fail(RT_EINVAL, std::string(path) + ": BVH cache was built for different triangles");
    Replica* r = nullptr;
    RTR(primary(s, &r));
    RTR(upload(s, *r));
    HIPR(hipSetDevice(r->device));
    RTR(join_caller_work(*r));
    HIPR(hipStreamSynchronize(r->stream));
    // from here on the device buffers are being overwritten: any failure
    // leaves the scene unbuilt (and every other replica is now stale)
    r->built = false;
    for (size_t i = 1; i < s->reps.size(); ++i) s->reps[i]->built = false;
    r->bufs.warity = hh[1] == kBvhLayout8 ? 8u : 4u;
    if (r->bufs.warity == 8 && s->n > rt::kWide8MaxN) return fail(RT_EIO, std::string(path) + ": bad record arity");
    std::vector<unsigned char> host;
    for (const BvhSection& sec : bvh_sections(s, *r)) {
        if (!sec.bytes) continue;
        host.resize(sec.bytes);
        if (std::fread(host.data(), 1, sec.bytes, f.f) != sec.bytes)
            return fail(RT_EIO, std::string(path) + ": truncated BVH cache");
        HIPR(hipMemcpy(sec.dev, host.data(), sec.bytes, hipMemcpyHostToDevice));
    }
    if (std::fgetc(f.f) != EOF) return fail(RT_EIO, std::string(path) + ": trailing bytes in BVH cache");
    r->times = rt_build_times{};
    r->built = true;
    return RT_OK;
}

// Device-resident BVH exchange (SURVEY.md §8(e) "rank 0 builds and then
// broadcasts"): the same sections as the RTBVH1 file, as device pointers.
rt_status rt_bvh_prepare(rt_scene* s) {
    if (!s) return fail(RT_EINVAL, "null scene");
    Replica* r = nullptr;
    RTR(primary(s, &r));
    RTR(upload(s, *r));
    r->bufs.warity = build_arity(s->n);  // the sender's (same configuration on every rank)
    return RT_OK;
}

rt_status rt_bvh_device_sections(rt_scene* s, uint32_t max, void** ptrs, uint64_t* bytes, uint32_t* count_out) {
    if (!s || !count_out || (max && (!ptrs || !bytes))) return fail(RT_EINVAL, "null argument");
    if (s->reps.empty() || !s->reps[0]->uploaded)
        return fail(RT_EINVAL, "scene not prepared (rt_bvh_prepare or rt_bvh_build)");
    const std::vector<BvhSection> secs = bvh_sections(s, *s->reps[0]);
    *count_out = (uint32_t)secs.size();
    for (uint32_t i = 0; i < max && i < secs.size(); ++i) {
        ptrs[i] = secs[i].dev;
        bytes[i] = secs[i].bytes;
    }
    return RT_OK;
}

rt_status rt_bvh_mark_built(rt_scene* s) {
    if (!s) return fail(RT_EINVAL, "null scene");
    if (s->reps.empty() || !s->reps[0]->uploaded) return fail(RT_EINVAL, "scene not prepared (rt_bvh_prepare)");
    Replica* r = s->reps[0].get();
    HIPR(hipSetDevice(r->device));
    HIPR(hipDeviceSynchronize());  // the caller's writes (any stream) land before the first render
    r->times = rt_build_times{};
    r->built = true;
    return RT_OK;
}

// ------------------------------------------------------------------ render
}  // extern "C"

namespace {

// Replicas 0..P-1 for a P-rank render: one per device, or
// all on the scene's device under render.emulate; the missing ones are
// created and built (concurrently) -- the replicated build of the scheme.
rt_status ensure_replicas(rt_scene* s, uint32_t P, bool emulate) {
    Replica* r0 = nullptr;
    RTR(primary(s, &r0));
    const int cnt = visible_devices();
    std::vector<Replica*> todo;
    if (!r0->built) todo.push_back(r0);
    while (s->reps.size() < P) {
        int dev = r0->device;
        if (!emulate) {
            dev = -1;
            for (int d = 0; d < cnt && dev < 0; ++d) {
                bool used = false;
                for (auto& r : s->reps) used = used || r->device == d;
                if (!used) dev = d;
            }
            if (dev < 0) return fail(RT_EDEVICE, "not enough devices for the requested ngpus");
        }
        std::unique_ptr<Replica> r(new (std::nothrow) Replica);
        if (!r) return fail(RT_ENOMEM, "host allocation failed");
        r->device = dev;
        todo.push_back(r.get());
        s->reps.push_back(std::move(r));
    }
    for (uint32_t i = 1; i < P; ++i) {
        const int d = s->reps[i]->device;
        bool clash = emulate ? d != r0->device : false;
        for (uint32_t j = 0; j < i && !emulate; ++j) clash = clash || s->reps[j]->device == d;
        if (clash)
            return fail(RT_EINVAL, emulate ? "render.emulate needs every replica on the scene's device"
                                           : "two replicas share a device; multi-GPU render needs distinct devices");
        if (!s->reps[i]->built && std::find(todo.begin(), todo.end(), s->reps[i].get()) == todo.end())
            todo.push_back(s->reps[i].get());
    }
    return todo.empty() ? RT_OK : build_replicas(s, todo, nullptr);
}

rt_status comms_for(rt_scene* s, const std::vector<int>& devs, std::vector<ncclComm_t>** out) {
    const Rccl& R = rccl();
    if (!R.init_all) return fail(RT_ECOMM, R.why);
    if (s->comm.devs != devs) {
        free_comms(s->comm);
        s->comm.comms.assign(devs.size(), nullptr);
        NCCLR(R.init_all(s->comm.comms.data(), (int)devs.size(), devs.data()));
        // every communicator must span exactly the P devices, rank r on replica r:
        // a gather over a smaller or reordered communicator would hang or mix slabs
        for (size_t i = 0; i < devs.size(); ++i) {
            int cnt = -1, rk = -1;
            NCCLR(R.count(s->comm.comms[i], &cnt));
            NCCLR(R.user_rank(s->comm.comms[i], &rk));
            if (cnt != (int)devs.size() || rk != (int)i) {
                free_comms(s->comm);
                return fail(RT_ECOMM, "ncclCommInitAll gave a communicator of " + std::to_string(cnt) + " ranks (rank " +
                                          std::to_string(rk) + ") for " + std::to_string(devs.size()) + " devices");
            }
        }
        s->comm.devs = devs;
    }
    *out = &s->comm.comms;
    return RT_OK;
}

// rt_render with the tile scheme of SURVEY.md §8(e) inside the library: rank
// r traces tiles t = r mod P on replica r into a packed slab, RCCL gathers the
// slabs to rank 0 (one ncclGather per rank in one group, each on its
// replica's stream), and rank 0 unpacks them into the frame.  ms_out spans
// first trace launch .. unpack end on the root's stream (every rank's trace
// and the gather lie inside it).
rt_status render_tiled(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp, uint32_t P,
                       rt_hit* hits_out, uint8_t* rgba_out, double* ms_out, const rt::TraceConfig& cfg) {
    const bool emulate = cfg.render_emulate != 0;
    RTR(ensure_replicas(s, P, emulate));
    Replica& root = *s->reps[0];
    const uint32_t tmax = std::max(rt::tiles_for_rank(w, h, 0, P), 1u);  // rank 0 holds the most tiles
    const size_t slab = (size_t)tmax * 1024, slab_hits = (size_t)tmax * 256 * spp * 16;
    std::vector<int> devs;
    for (uint32_t r = 0; r < P; ++r) {
        Replica& R = *s->reps[r];
        devs.push_back(R.device);
        HIPR(hipSetDevice(R.device));
        RTR(grow(&R.d_slab, &R.slab_cap, slab));
        if (hits_out) RTR(grow(&R.d_slab_hits, &R.slab_hits_cap, slab_hits));
    }
    HIPR(hipSetDevice(root.device));
    RTR(grow(&root.d_recv, &root.recv_cap, slab * P));
    if (hits_out) RTR(grow(&root.d_recv_hits, &root.recv_hits_cap, slab_hits * P));
    RTR(grow(&root.d_rgba, &root.rgba_cap, (size_t)w * h * 4));
    if (hits_out) RTR(grow(&root.d_hits, &root.hits_cap, (size_t)w * h * spp * 16));
    std::vector<ncclComm_t>* comms = nullptr;
    if (!emulate) RTR(comms_for(s, devs, &comms));

    HIPR(hipEventRecord(root.r0, root.stream));
    for (uint32_t r = 0; r < P; ++r) {
        Replica& R = *s->reps[r];
        HIPR(hipSetDevice(R.device));
        RTR(join_caller_work(R));
        if (r) HIPR(hipStreamWaitEvent(R.stream, root.r0, 0));
        rt::TileSched* sched = nullptr;
        RTR(sched_for(R.ord, w, h, spp, r, P, &sched));
        hipError_t e = rt::launch_trace(R.bufs.nodes, R.bufs.wnodes, R.bufs.warity,
                                        R.bufs.tri_s, s->n, camf(cam), w, h, spp, r, P,
                                        true, hits_out ? R.d_slab_hits : nullptr, R.d_slab, nullptr, false,
                                        sched, R.stream);
        if (e != hipSuccess) return hip_fail(e, "launch_trace");
        sched_done(R.ord, cfg);
    }
    if (!emulate) {
        const Rccl& RC = rccl();
        NCCLR(RC.group_start());
        for (uint32_t r = 0; r < P; ++r) {
            Replica& R = *s->reps[r];
            HIPR(hipSetDevice(R.device));
            NCCLR(RC.gather(R.d_slab, r == 0 ? root.d_recv : nullptr, slab, ncclUint8, 0, (*comms)[r], R.stream));
            if (hits_out)
                NCCLR(RC.gather(R.d_slab_hits, r == 0 ? root.d_recv_hits : nullptr, slab_hits, ncclUint8, 0,
                                (*comms)[r], R.stream));
        }
        NCCLR(RC.group_end());
    } else {
        // one device plays every rank: the gather is a device copy per rank
        HIPR(hipSetDevice(root.device));
        for (uint32_t r = 0; r < P; ++r) {
            Replica& R = *s->reps[r];
            if (r) {
                HIPR(hipEventRecord(R.r1, R.stream));
                HIPR(hipStreamWaitEvent(root.stream, R.r1, 0));
            }
            HIPR(hipMemcpyAsync((char*)root.d_recv + r * slab, R.d_slab, slab, hipMemcpyDeviceToDevice, root.stream));
            if (hits_out)
                HIPR(hipMemcpyAsync((char*)root.d_recv_hits + r * slab_hits, R.d_slab_hits, slab_hits,
                                    hipMemcpyDeviceToDevice, root.stream));
        }
    }
    HIPR(hipSetDevice(root.device));
    hipError_t e = rt::launch_unpack(root.d_recv, tmax, w, h, P, root.d_rgba, root.stream);
    if (e != hipSuccess) return hip_fail(e, "launch_unpack");
    if (hits_out && (e = rt::launch_unpack_hits(root.d_recv_hits, tmax, w, h, spp, P, root.d_hits, root.stream)) !=
                        hipSuccess)
        return hip_fail(e, "launch_unpack_hits");
    HIPR(hipEventRecord(root.r1, root.stream));
    for (uint32_t r = 0; r < P; ++r) {
        HIPR(hipSetDevice(s->reps[r]->device));
        HIPR(hipStreamSynchronize(s->reps[r]->stream));
    }
    HIPR(hipSetDevice(root.device));
    float ms = 0;
    HIPR(hipEventElapsedTime(&ms, root.r0, root.r1));
    if (ms_out) *ms_out = ms;
    if (hits_out) HIPR(hipMemcpy(hits_out, root.d_hits, (size_t)w * h * spp * 16, hipMemcpyDeviceToHost));
    if (rgba_out) HIPR(hipMemcpy(rgba_out, root.d_rgba, (size_t)w * h * 4, hipMemcpyDeviceToHost));
    return RT_OK;
}

}  // namespace

extern "C" {

rt_status rt_render_timed(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp, uint32_t ngpus,
                          rt_hit* hits_out, uint8_t* rgba_out, double* ms_out) {
    RtRange range_("rt_render");
    if (!s || !cam) return fail(RT_EINVAL, "bad render arguments");
    RTR(check_frame(w, h, spp));
    if (ngpus == 0 || ngpus > 64) return fail(RT_EINVAL, "ngpus must be 1..64");
    const rt::TraceConfig cfg = rt::config_snapshot();
    const int cnt = visible_devices();
    if (cnt == 0) return fail(RT_EDEVICE, "no HIP device available (librtamd has no CPU path)");
    if ((int)ngpus > cnt && !cfg.render_emulate)
        return fail(RT_EDEVICE, "ngpus exceeds the " + std::to_string(cnt) + " visible device(s)");
    Replica* r = nullptr;
    RTR(need_built(s, &r));
    if (ngpus > 1 || cfg.render_rccl1) return render_tiled(s, cam, w, h, spp, ngpus, hits_out, rgba_out, ms_out, cfg);
    const size_t nh = (size_t)w * h * spp;
    if (hits_out) RTR(grow(&r->d_hits, &r->hits_cap, nh * 16));
    RTR(grow(&r->d_rgba, &r->rgba_cap, (size_t)w * h * 4));
    RTR(join_caller_work(*r));
    rt::TileSched* sched = nullptr;
    RTR(sched_for(r->ord, w, h, spp, 0, 1, &sched));
    HIPR(hipEventRecord(r->r0, r->stream));
    hipError_t e = rt::launch_trace(r->bufs.nodes, r->bufs.wnodes, r->bufs.warity,
                                    r->bufs.tri_s, s->n, camf(cam), w, h, spp, 0, 1,
                                    false, hits_out ? r->d_hits : nullptr, r->d_rgba, nullptr, false, sched,
                                    r->stream);
    if (e != hipSuccess) return hip_fail(e, "launch_trace");
    sched_done(r->ord, cfg);
    HIPR(hipEventRecord(r->r1, r->stream));
    HIPR(hipStreamSynchronize(r->stream));
    float ms = 0;
    HIPR(hipEventElapsedTime(&ms, r->r0, r->r1));
    if (ms_out) *ms_out = ms;
    if (hits_out) HIPR(hipMemcpy(hits_out, r->d_hits, nh * 16, hipMemcpyDeviceToHost));
    if (rgba_out) HIPR(hipMemcpy(rgba_out, r->d_rgba, (size_t)w * h * 4, hipMemcpyDeviceToHost));
    return RT_OK;
}

// SURVEY.md §8(b)'s prototype exactly (SURVEY.md:291-292): the timed form
// without its device-time output.
rt_status rt_render(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp, uint32_t ngpus,
                    rt_hit* hits_out, uint8_t* rgba_out) {
    return rt_render_timed(s, cam, w, h, spp, ngpus, hits_out, rgba_out, nullptr);
}

// Shared shape of the *_device entry points: launch `fn` on the caller's
// stream (or the replica's), ordered after this replica's previous device
// work, optionally bracketed by events and waited for.
}  // extern "C"

namespace {
template <class F>
rt_status device_launch(Replica& r, void* stream, double* ms_out, const char* what, F&& fn) {
    hipStream_t hs = stream ? rt::hip_stream((hipStream_t)stream) : r.stream;
    HIPR(hipSetDevice(r.device));
    RTR(order_before(r, hs));
    if (ms_out) HIPR(hipEventRecord(r.r0, hs));
    const hipError_t e = fn(hs);
    if (e != hipSuccess) return hip_fail(e, what);
    if (ms_out) HIPR(hipEventRecord(r.r1, hs));
    RTR(order_after(r, hs));
    if (ms_out) {
        HIPR(hipEventSynchronize(r.r1));
        float ms = 0;
        HIPR(hipEventElapsedTime(&ms, r.r0, r.r1));
        *ms_out = ms;
    }
    return RT_OK;
}
}  // namespace

extern "C" {

rt_status rt_render_shadow_device(rt_scene* s, const rt_camera* cam, const float light[3], float ambient,
                                  uint32_t w, uint32_t h, uint32_t spp, void* d_hits, void* d_rgba, void* stream,
                                  double* ms_out) {
    RtRange range_("rt_render_shadow_device");
    if (!s || !cam || !light) return fail(RT_EINVAL, "bad render arguments");
    RTR(check_frame(w, h, spp));
    Replica* r = nullptr;
    RTR(need_built(s, &r));
    return device_launch(*r, stream, ms_out, "launch_trace_shadow", [&](hipStream_t hs) {
        return rt::launch_trace_shadow(r->bufs.nodes, r->bufs.wnodes, r->bufs.warity,
                                       r->bufs.tri_s, r->bufs.tris, s->n, camf(cam), w,
                                       h, spp, light, ambient, d_hits, d_rgba, nullptr, hs);
    });
}

rt_status rt_render_shadow(rt_scene* s, const rt_camera* cam, const float light[3], float ambient, uint32_t w,
                           uint32_t h, uint32_t spp, rt_hit* hits_out, uint8_t* rgba_out, double* ms_out) {
    if (!s || !cam || !light) return fail(RT_EINVAL, "bad render arguments");
    RTR(check_frame(w, h, spp));
    Replica* r = nullptr;
    RTR(need_built(s, &r));
    const size_t nh = (size_t)w * h * spp;
    if (hits_out) RTR(grow(&r->d_hits, &r->hits_cap, nh * 16));
    RTR(grow(&r->d_rgba, &r->rgba_cap, (size_t)w * h * 4));
    RTR(rt_render_shadow_device(s, cam, light, ambient, w, h, spp, hits_out ? r->d_hits : nullptr, r->d_rgba, nullptr,
                                ms_out));
    HIPR(hipStreamSynchronize(r->stream));
    if (hits_out) HIPR(hipMemcpy(hits_out, r->d_hits, nh * 16, hipMemcpyDeviceToHost));
    if (rgba_out) HIPR(hipMemcpy(rgba_out, r->d_rgba, (size_t)w * h * 4, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_render_shadow_work(rt_scene* s, const rt_camera* cam, const float light[3], float ambient, uint32_t w,
                                uint32_t h, uint32_t spp, uint64_t counters_out[2]) {
    if (!s || !cam || !light || !counters_out) return fail(RT_EINVAL, "bad arguments");
    RTR(check_frame(w, h, spp));
    Replica* r = nullptr;
    RTR(need_built(s, &r));
    RTR(join_caller_work(*r));
    if (!r->d_ctr) HIPR(rt::dev_alloc(&r->d_ctr, 32));
    HIPR(hipMemsetAsync(r->d_ctr, 0, 16, r->stream));
    hipError_t e = rt::launch_trace_shadow(r->bufs.nodes, r->bufs.wnodes, r->bufs.warity,
                                           r->bufs.tri_s, r->bufs.tris, s->n, camf(cam),
                                           w, h, spp, light, ambient, nullptr, nullptr, r->d_ctr, r->stream);
    if (e != hipSuccess) return hip_fail(e, "launch_trace_shadow");
    HIPR(hipStreamSynchronize(r->stream));
    HIPR(hipMemcpy(counters_out, r->d_ctr, 16, hipMemcpyDeviceToHost));
    return RT_OK;
}

}  // extern "C"

// Path mode: the megakernel, or the wavefront schedule with ray reordering
// (config path.wavefront); with a sorted queue the wavefront reads each
// depth's queue length back to the host, so it synchronizes between depths.
static hipError_t path_launch(rt_scene* s, Replica& r, const rt_camera* cam, const float light[3], float sky,
                              uint32_t max_depth, uint32_t w, uint32_t h, uint32_t spp, void* d_hits, void* d_rgba,
                              unsigned long long* ctr, hipStream_t hs, std::string& err) {
    const rt::TraceConfig cfg = rt::config_snapshot();
    if (cfg.path_wave) {
        const uint64_t per_tile = 256ull * spp;
        const uint64_t tiles = rt::tiles_for_rank(w, h, 0, 1);
        const uint64_t want = cfg.path_batch ? cfg.path_batch : (1u << 22);
        uint64_t cap = std::min<uint64_t>(tiles * per_tile, std::max<uint64_t>(per_tile, want / per_tile * per_tile));
        if (cap > (1u << 30)) {
            err = "path batch exceeds 2^30 paths (lower spp or path.batch)";
            return hipErrorInvalidValue;
        }
        if (r.path.cap < cap) {
            hipError_t e = rt::alloc_path(r.path, (uint32_t)cap);
            if (e != hipSuccess) {
                rt::free_path(r.path);
                err = "alloc_path";
                return e;
            }
        }
        return rt::launch_path_wavefront(r.bufs.nodes, r.bufs.wnodes, r.bufs.warity,
                                         r.bufs.tri_s, r.bufs.tris, r.bufs.params, s->n,
                                         camf(cam), w, h, spp, light, sky, max_depth, d_hits, d_rgba, ctr, r.path,
                                         cfg.path_sort, hs);
    }
    return rt::launch_trace_path(r.bufs.nodes, r.bufs.wnodes, r.bufs.warity,
                                 r.bufs.tri_s, r.bufs.tris, s->n, camf(cam), w, h, spp,
                                 light, sky, max_depth, d_hits, d_rgba, ctr, hs);
}

extern "C" {

rt_status rt_render_path_device(rt_scene* s, const rt_camera* cam, const float light[3], float sky,
                                uint32_t max_depth, uint32_t w, uint32_t h, uint32_t spp, void* d_hits, void* d_rgba,
                                void* stream, double* ms_out) {
    RtRange range_("rt_render_path_device");
    if (!s || !cam || !light) return fail(RT_EINVAL, "bad render arguments");
    RTR(check_frame(w, h, spp));
    if (max_depth > 64) return fail(RT_EINVAL, "max_depth exceeds 64");
    Replica* r = nullptr;
    RTR(need_built(s, &r));
    std::string err;
    rt_status st = device_launch(*r, stream, ms_out, "launch_path", [&](hipStream_t hs) {
        return path_launch(s, *r, cam, light, sky, max_depth, w, h, spp, d_hits, d_rgba, nullptr, hs, err);
    });
    if (st && !err.empty()) g_err = err + ": " + g_err;
    return st;
}

rt_status rt_render_path(rt_scene* s, const rt_camera* cam, const float light[3], float sky, uint32_t max_depth,
                         uint32_t w, uint32_t h, uint32_t spp, rt_hit* hits_out, uint8_t* rgba_out, double* ms_out) {
    if (!s || !cam || !light) return fail(RT_EINVAL, "bad render arguments");
    RTR(check_frame(w, h, spp));
    Replica* r = nullptr;
    RTR(need_built(s, &r));
    const size_t nh = (size_t)w * h * spp;
    if (hits_out) RTR(grow(&r->d_hits, &r->hits_cap, nh * 16));
    RTR(grow(&r->d_rgba, &r->rgba_cap, (size_t)w * h * 4));
    RTR(rt_render_path_device(s, cam, light, sky, max_depth, w, h, spp, hits_out ? r->d_hits : nullptr, r->d_rgba,
                              nullptr, ms_out));
    HIPR(hipStreamSynchronize(r->stream));
    if (hits_out) HIPR(hipMemcpy(hits_out, r->d_hits, nh * 16, hipMemcpyDeviceToHost));
    if (rgba_out) HIPR(hipMemcpy(rgba_out, r->d_rgba, (size_t)w * h * 4, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_render_path_work(rt_scene* s, const rt_camera* cam, const float light[3], float sky, uint32_t max_depth,
                              uint32_t w, uint32_t h, uint32_t spp, uint64_t counters_out[3]) {
    if (!s || !cam || !light || !counters_out) return fail(RT_EINVAL, "bad arguments");
    RTR(check_frame(w, h, spp));
    if (max_depth > 64) return fail(RT_EINVAL, "max_depth exceeds 64");
    Replica* r = nullptr;
    RTR(need_built(s, &r));
    RTR(join_caller_work(*r));
    if (!r->d_ctr) HIPR(rt::dev_alloc(&r->d_ctr, 32));
    HIPR(hipMemsetAsync(r->d_ctr, 0, 32, r->stream));
    std::string err;
    hipError_t e = path_launch(s, *r, cam, light, sky, max_depth, w, h, spp, nullptr, nullptr, r->d_ctr, r->stream, err);
    if (e != hipSuccess) return hip_fail(e, err.empty() ? "launch_path" : err.c_str());
    HIPR(hipStreamSynchronize(r->stream));
    HIPR(hipMemcpy(counters_out, r->d_ctr, 24, hipMemcpyDeviceToHost));
    return RT_OK;
}

}  // extern "C"

static rt_status counters_impl(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp,
                               uint32_t rank, uint32_t nranks, bool packed, bool binary, uint64_t counters_out[2]) {
    if (!s || !cam || !counters_out || !nranks || rank >= nranks) return fail(RT_EINVAL, "bad arguments");
    RTR(check_frame(w, h, spp));
    Replica* r = nullptr;
    RTR(need_built(s, &r));
    RTR(join_caller_work(*r));
    if (!r->d_ctr) HIPR(rt::dev_alloc(&r->d_ctr, 32));
    HIPR(hipMemsetAsync(r->d_ctr, 0, 16, r->stream));
    // the kernels' own work counters include the heavy-ray queue's pass when
    // it is on (trace.coop_cap*), which needs the frame shape's queue
    rt::TileSched* sched = nullptr;
    // (the replica's scratch state, reset every call: the counts do not
    // depend on the dispatch order, and the frames' own maps stay untouched)
    if (!binary) {
        std::memset(r->ord_diag.key, 0, sizeof(r->ord_diag.key));
        RTR(sched_for(r->ord_diag, w, h, spp, rank, nranks, &sched));
    }
    hipError_t e = rt::launch_trace(r->bufs.nodes, r->bufs.wnodes, r->bufs.warity,
                                    r->bufs.tri_s, s->n, camf(cam), w, h, spp, rank,
                                    nranks, packed, nullptr, nullptr, r->d_ctr, binary, sched, r->stream);
    if (e != hipSuccess) return hip_fail(e, "launch_trace");
    HIPR(hipStreamSynchronize(r->stream));
    HIPR(hipMemcpy(counters_out, r->d_ctr, 16, hipMemcpyDeviceToHost));
    return RT_OK;
}

extern "C" {

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

rt_status rt_render_tiles_work(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp,
                               uint32_t rank, uint32_t nranks, uint64_t counters_out[2]) {
    return counters_impl(s, cam, w, h, spp, rank, nranks, true, false, counters_out);
}

rt_status rt_render_step_map(rt_scene* s, uint32_t w, uint32_t h, uint32_t spp, uint32_t rank, uint32_t nranks,
                             uint16_t* out, size_t count) {
    if (!s || !out || !nranks || rank >= nranks) return fail(RT_EINVAL, "bad step-map arguments");
    Replica* r = nullptr;
    RTR(need_built(s, &r));
    const uint32_t key[5] = {w, h, spp, rank, nranks};
    if (!r->ord.sched.have_prev || std::memcmp(key, r->ord.key, sizeof(key)) != 0)
        return fail(RT_EINVAL, "no previous frame of this shape");
    const size_t nb = rt::tiles_for_rank(w, h, rank, nranks);
    if (count < nb * 256) return fail(RT_EINVAL, "step map buffer too small");
    HIPR(hipSetDevice(r->device));
    if (r->last_pending) HIPR(hipEventSynchronize(r->last));
    HIPR(hipStreamSynchronize(r->stream));
    HIPR(hipMemcpy(out, r->ord.sched.px_prev, nb * 256 * sizeof(uint16_t), hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_render_device(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp, void* d_hits,
                           void* d_rgba, void* stream, double* ms_out) {
    RtRange range_("rt_render_device");
    if (!s || !cam) return fail(RT_EINVAL, "bad render arguments");
    RTR(check_frame(w, h, spp));
    Replica* r = nullptr;
    RTR(need_built(s, &r));
    const rt::TraceConfig cfg = rt::config_snapshot();
    rt::TileSched* sched = nullptr;
    RTR(sched_for(r->ord, w, h, spp, 0, 1, &sched));
    RTR(device_launch(*r, stream, ms_out, "launch_trace", [&](hipStream_t hs) {
        return rt::launch_trace(r->bufs.nodes, r->bufs.wnodes, r->bufs.warity,
                                r->bufs.tri_s, s->n, camf(cam), w, h, spp, 0, 1, false,
                                d_hits, d_rgba, nullptr, false, sched, hs);
    }));
    sched_done(r->ord, cfg);
    return RT_OK;
}

uint32_t rt_tiles_for_rank(uint32_t w, uint32_t h, uint32_t rank, uint32_t nranks) {
    return rt::tiles_for_rank(w, h, rank, nranks);
}

rt_status rt_render_tiles_device(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp,
                                 uint32_t rank, uint32_t nranks, void* d_packed_rgba, void* d_packed_hits,
                                 void* stream, double* ms_out) {
    RtRange range_("rt_render_tiles_device");
    if (!s || !cam || !nranks || rank >= nranks) return fail(RT_EINVAL, "bad arguments");
    RTR(check_frame(w, h, spp));
    Replica* r = nullptr;
    RTR(need_built(s, &r));
    const rt::TraceConfig cfg = rt::config_snapshot();
    rt::TileSched* sched = nullptr;
    RTR(sched_for(r->ord, w, h, spp, rank, nranks, &sched));
    RTR(device_launch(*r, stream, ms_out, "launch_trace", [&](hipStream_t hs) {
        return rt::launch_trace(r->bufs.nodes, r->bufs.wnodes, r->bufs.warity,
                                r->bufs.tri_s, s->n, camf(cam), w, h, spp, rank, nranks,
                                true, d_packed_hits, d_packed_rgba, nullptr, false, sched, hs);
    }));
    sched_done(r->ord, cfg);
    return RT_OK;
}

rt_status rt_unpack_tiles_device(const void* d_slabs, uint32_t tiles_per_slab, uint32_t w, uint32_t h,
                                 uint32_t nranks, void* d_rgba, int device, void* stream) {
    if (!d_slabs || !d_rgba || !w || !h || !nranks) return fail(RT_EINVAL, "bad arguments");
    RTR(ensure_device(device));
    hipError_t e = rt::launch_unpack(d_slabs, tiles_per_slab, w, h, nranks, d_rgba, rt::hip_stream((hipStream_t)stream));
    if (e != hipSuccess) return hip_fail(e, "launch_unpack");
    return RT_OK;
}

// ------------------------------------------------------------------ stage entry points
rt_status rt_stage_bounds(int device, const float* tris, uint32_t n, float bounds9[9]) {
    if ((n && !tris) || !bounds9) return fail(RT_EINVAL, "null argument");
    RTR(ensure_device(device));
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
    RTR(ensure_device(device));
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
    RTR(ensure_device(device));
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
    RTR(ensure_device(device));
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

// K4 + K5 + K6 (+ K7w) over already sorted keys/vals: the refit stage as the
// build runs it (fused with the topology in k_topo_refit, crossing nodes in
// k_refit_cross).  nodes_out: (2n-1) x 32-B records.
rt_status rt_stage_refit(int device, const uint32_t* sorted_keys, const uint32_t* sorted_vals, const float* tris,
                         uint32_t n, rt_node* nodes_out) {
    if (n && (!sorted_keys || !sorted_vals || !tris || !nodes_out)) return fail(RT_EINVAL, "null argument");
    if (n > (1u << 30)) return fail(RT_EINVAL, "n exceeds 2^30");
    RTR(ensure_device(device));
    if (!n) return RT_OK;
    for (uint32_t i = 0; i < n; ++i)
        if (sorted_vals[i] >= n) return fail(RT_EINVAL, "sorted_vals holds an index >= n");
    rt::BuildBufs b;
    hipError_t e = rt::alloc_build(b, n);
    if (e != hipSuccess) {
        rt::free_build(b);
        return e == hipErrorOutOfMemory ? fail(RT_ENOMEM, "device allocation failed") : hip_fail(e, "alloc_build");
    }
    struct Guard {
        rt::BuildBufs& b;
        ~Guard() { rt::free_build(b); }
    } guard{b};
    b.warity = build_arity(n);
    HIPR(hipMemcpy(b.tris, tris, (size_t)n * 36, hipMemcpyHostToDevice));
    HIPR(hipMemcpy(b.keys[0], sorted_keys, (size_t)n * 4, hipMemcpyHostToDevice));
    HIPR(hipMemcpy(b.vals[0], sorted_vals, (size_t)n * 4, hipMemcpyHostToDevice));
    HIPR(rt::launch_refit_stage(b, n, 0));
    HIPR(rt::launch_leaf_nodes(b.tri_s, n, b.nodes, 0));
    HIPR(hipDeviceSynchronize());
    HIPR(hipMemcpy(nodes_out, b.nodes, (size_t)(2 * n - 1) * 32, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_stage_trace(int device, const rt_node* nodes, uint32_t n, const float* tris, const rt_camera* cam,
                         uint32_t w, uint32_t h, uint32_t spp, rt_hit* hits, uint8_t* rgba, uint64_t counters[2]) {
    if ((n && (!nodes || !tris)) || !cam) return fail(RT_EINVAL, "bad arguments");
    RTR(check_frame(w, h, spp));
    RTR(ensure_device(device));
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
    DevBuf dts;
    HIPR(dts.alloc((size_t)(n ? n : 1) * 48));
    HIPR(rt::launch_leaf_tris(dn.p, dt.as<float>(), n, dts.as<float4>(), 0));
    HIPR(rt::launch_trace(dn.p, nullptr, 4u, dts.as<float4>(), n, camf(cam), w, h, spp, 0, 1, false, dh.p, dr.p,
                          counters ? dc.as<unsigned long long>() : nullptr, true, nullptr, 0));
    HIPR(hipDeviceSynchronize());
    if (hits) HIPR(hipMemcpy(hits, dh.p, nh * 16, hipMemcpyDeviceToHost));
    if (rgba) HIPR(hipMemcpy(rgba, dr.p, (size_t)w * h * 4, hipMemcpyDeviceToHost));
    if (counters) HIPR(hipMemcpy(counters, dc.p, 16, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_stage_intersect(int device, uint32_t count, const float* o, const float* d, const float* tri,
                             const float* t_best, uint32_t* hit, float* tuv) {
    if (count && (!o || !d || !tri || !t_best || !hit || !tuv)) return fail(RT_EINVAL, "null argument");
    RTR(ensure_device(device));
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
    RTR(ensure_device(device));
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

// ------------------------------------------------------- distributed build
// SURVEY.md §8(f) row 4; DESIGN.md "Distributed build".  SPMD over P ranks:
// every rank holds the whole soup (a scene), runs these phases on its own
// share and moves the bytes between them itself (gpu_raytracer_amd/dist.py:
// torch.distributed over RCCL, or gloo).  Each phase runs the single-GPU
// build's own kernels on a slice of triangles or a range of refit blocks, so
// every rank ends with the BVH rt_bvh_build makes, bit for bit.

rt_status rt_dbuild_shares(uint32_t n, uint32_t rank, uint32_t nranks, uint32_t out[6]) {
    if (!out || !nranks || rank >= nranks) return fail(RT_EINVAL, "bad arguments");
    const uint32_t m = rt::refit_blocks(n);
    out[0] = (uint32_t)((uint64_t)n * rank / nranks);
    out[1] = (uint32_t)((uint64_t)n * (rank + 1) / nranks);
    out[2] = (uint32_t)((uint64_t)m * rank / nranks);
    out[3] = (uint32_t)((uint64_t)m * (rank + 1) / nranks);
    out[4] = std::min<uint64_t>((uint64_t)out[2] * kRefitLeaves, n);
    out[5] = std::min<uint64_t>((uint64_t)out[3] * kRefitLeaves, n);
    return RT_OK;
}

namespace {
rt_status dbuild_replica(rt_scene* s, uint32_t rank, uint32_t nranks, Replica** out) {
    if (!s || !nranks || rank >= nranks || nranks > kMaxDbuildRanks) return fail(RT_EINVAL, "bad rank / nranks");
    Replica* r = nullptr;
    RTR(primary(s, &r));
    RTR(upload(s, *r));
    HIPR(hipSetDevice(r->device));
    RTR(join_caller_work(*r));
    if (r->d_n != s->n || !r->dboxes) {
        const size_t n4 = (size_t)(s->n ? s->n : 1) * 4;
        const size_t cc = (size_t)rt::dbuild_cross_cap(s->n) * rt::kCrossShards * 4;
        for (uint32_t** p : {&r->dk[0], &r->dk[1], &r->dv[0], &r->dv[1], &r->dcross, &r->dcross_all})
            if (*p) { (void)hipFree(*p); *p = nullptr; }
        if (r->dboxes) { (void)hipFree(r->dboxes); r->dboxes = nullptr; }
        r->d_n = 0;
        for (uint32_t** p : {&r->dk[0], &r->dk[1], &r->dv[0], &r->dv[1]}) {
            hipError_t e = rt::dev_alloc(p, n4);
            if (e != hipSuccess) return e == hipErrorOutOfMemory ? fail(RT_ENOMEM, "device allocation failed") : hip_fail(e, "hipMalloc");
        }
        for (uint32_t** p : {&r->dcross, &r->dcross_all}) {
            hipError_t e = rt::dev_alloc(p, cc);
            if (e != hipSuccess) return e == hipErrorOutOfMemory ? fail(RT_ENOMEM, "device allocation failed") : hip_fail(e, "hipMalloc");
        }
        hipError_t e = rt::dev_alloc(&r->dboxes, kMaxDbuildRanks * 6 * sizeof(float));
        if (e != hipSuccess) return e == hipErrorOutOfMemory ? fail(RT_ENOMEM, "device allocation failed") : hip_fail(e, "hipMalloc");
        r->d_n = s->n;
    }
    *out = r;
    return RT_OK;
}
}  // namespace

rt_status rt_dbuild_bounds(rt_scene* s, uint32_t rank, uint32_t nranks, float box_out[6]) {
    RtRange range_("rt_dbuild_bounds");
    if (!box_out) return fail(RT_EINVAL, "null argument");
    Replica* r = nullptr;
    RTR(dbuild_replica(s, rank, nranks, &r));
    r->built = false;  // the BVH is rewritten from here on; other replicas are stale
    for (size_t i = 1; i < s->reps.size(); ++i) s->reps[i]->built = false;
    uint32_t sh[6];
    RTR(rt_dbuild_shares(s->n, rank, nranks, sh));
    if (sh[1] > sh[0]) {
        HIPR(rt::launch_dbuild_bounds(r->bufs, sh[0], sh[1] - sh[0], r->stream));
        HIPR(hipMemcpyAsync(box_out, r->bufs.params, 6 * sizeof(float), hipMemcpyDeviceToHost, r->stream));
        HIPR(hipStreamSynchronize(r->stream));
    } else {  // an empty slice: the identity of min/max
        for (int c = 0; c < 3; ++c) {
            box_out[c] = std::numeric_limits<float>::infinity();
            box_out[3 + c] = -std::numeric_limits<float>::infinity();
        }
    }
    return RT_OK;
}

rt_status rt_dbuild_keys(rt_scene* s, uint32_t rank, uint32_t nranks, const float* boxes, uint32_t hist_out[1024]) {
    RtRange range_("rt_dbuild_keys");
    if (!boxes || !hist_out) return fail(RT_EINVAL, "null argument");
    Replica* r = nullptr;
    RTR(dbuild_replica(s, rank, nranks, &r));
    uint32_t sh[6];
    RTR(rt_dbuild_shares(s->n, rank, nranks, sh));
    const uint32_t cnt = sh[1] - sh[0];
    HIPR(hipMemcpyAsync(r->dboxes, boxes, (size_t)nranks * 6 * sizeof(float), hipMemcpyHostToDevice, r->stream));
    HIPR(rt::launch_dbuild_keys(r->bufs, sh[0], cnt, r->dboxes, nranks, r->stream));
    HIPR(hipMemcpyAsync(hist_out, r->bufs.zero + rt::kZHist, 1024 * 4, hipMemcpyDeviceToHost, r->stream));
    HIPR(hipStreamSynchronize(r->stream));
    // the slice sorted by (key, index): grouped by bucket, hence by destination
    uint32_t* K[2] = {r->bufs.keys[1], r->dk[0]};
    uint32_t* V[2] = {r->bufs.vals[1], r->dv[0]};
    HIPR(rt::launch_dbuild_sort(K, V, cnt, r->bufs, r->stream));
    HIPR(hipStreamSynchronize(r->stream));
    return RT_OK;
}

rt_status rt_dbuild_sort(rt_scene* s, uint32_t count) {
    RtRange range_("rt_dbuild_sort");
    if (!s || count > s->n) return fail(RT_EINVAL, "bad arguments");
    if (s->reps.empty() || !s->reps[0]->d_n) return fail(RT_EINVAL, "rt_dbuild_keys first");
    Replica* r = s->reps[0].get();
    HIPR(hipSetDevice(r->device));
    uint32_t* K[2] = {r->dk[1], r->dk[0]};
    uint32_t* V[2] = {r->dv[1], r->dv[0]};
    HIPR(rt::launch_dbuild_sort(K, V, count, r->bufs, r->stream));
    HIPR(hipStreamSynchronize(r->stream));
    return RT_OK;
}

rt_status rt_dbuild_subtrees(rt_scene* s, uint32_t rank, uint32_t nranks, uint32_t* ncross_out) {
    RtRange range_("rt_dbuild_subtrees");
    if (!ncross_out) return fail(RT_EINVAL, "null argument");
    Replica* r = nullptr;
    RTR(dbuild_replica(s, rank, nranks, &r));
    uint32_t sh[6];
    RTR(rt_dbuild_shares(s->n, rank, nranks, sh));
    r->bufs.warity = build_arity(s->n);
    HIPR(rt::launch_dbuild_subtrees(r->bufs, s->n, sh[2], sh[3] - sh[2], r->stream));
    uint32_t ctr[rt::kCrossShards];
    HIPR(hipMemcpyAsync(ctr, r->bufs.zero + rt::kZCrossCtr, sizeof(ctr), hipMemcpyDeviceToHost, r->stream));
    HIPR(hipStreamSynchronize(r->stream));
    // compact the sharded list into dcross
    const uint32_t cap = rt::dbuild_cross_cap(s->n);
    uint32_t tot = 0;
    for (uint32_t j = 0; j < rt::kCrossShards; ++j) {
        if (ctr[j] > cap) return fail(RT_EDEVICE, "crossing list overflow");
        if (ctr[j])
            HIPR(hipMemcpyAsync(r->dcross + tot, r->bufs.cross + (size_t)j * cap, ctr[j] * 4, hipMemcpyDeviceToDevice,
                                r->stream));
        tot += ctr[j];
    }
    HIPR(hipStreamSynchronize(r->stream));
    *ncross_out = tot;
    return RT_OK;
}

rt_status rt_dbuild_merge(rt_scene* s, uint32_t ncross_total) {
    RtRange range_("rt_dbuild_merge");
    if (!s) return fail(RT_EINVAL, "null scene");
    if (s->reps.empty() || !s->reps[0]->d_n) return fail(RT_EINVAL, "rt_dbuild_subtrees first");
    Replica* r = s->reps[0].get();
    HIPR(hipSetDevice(r->device));
    const uint32_t cap = rt::dbuild_cross_cap(s->n);
    if (ncross_total > cap * rt::kCrossShards) return fail(RT_EINVAL, "ncross_total exceeds the crossing-list capacity");
    // the gathered list (dcross_all) dealt into the build's shards
    uint32_t ctr[rt::kCrossShards] = {};
    uint32_t done = 0;
    for (uint32_t j = 0; j < rt::kCrossShards && done < ncross_total; ++j) {
        ctr[j] = std::min(cap, ncross_total - done);
        HIPR(hipMemcpyAsync(r->bufs.cross + (size_t)j * cap, r->dcross_all + done, ctr[j] * 4, hipMemcpyDeviceToDevice,
                            r->stream));
        done += ctr[j];
    }
    HIPR(hipMemcpyAsync(r->bufs.zero + rt::kZCrossCtr, ctr, sizeof(ctr), hipMemcpyHostToDevice, r->stream));
    HIPR(rt::launch_dbuild_merge(r->bufs, s->n, r->stream));
    HIPR(hipStreamSynchronize(r->stream));
    r->times = rt_build_times{};
    r->built = true;
    return RT_OK;
}

rt_status rt_dbuild_buffer(rt_scene* s, int which, void** ptr, uint64_t* bytes) {
    if (!s || !ptr || !bytes) return fail(RT_EINVAL, "null argument");
    if (s->reps.empty() || !s->reps[0]->d_n) return fail(RT_EINVAL, "rt_dbuild_bounds first");
    const Replica& r = *s->reps[0];
    const uint64_t n = s->n, tot = n ? 2 * n - 1 : 0, ni = n ? n - 1 : 0;
    const uint64_t cc = (uint64_t)rt::dbuild_cross_cap(s->n) * rt::kCrossShards * 4;
    switch (which) {
        case RT_DB_SEND_KEYS: *ptr = r.bufs.keys[1]; *bytes = n * 4; break;
        case RT_DB_SEND_VALS: *ptr = r.bufs.vals[1]; *bytes = n * 4; break;
        case RT_DB_RECV_KEYS: *ptr = r.dk[1]; *bytes = n * 4; break;
        case RT_DB_RECV_VALS: *ptr = r.dv[1]; *bytes = n * 4; break;
        case RT_DB_KEYS: *ptr = r.bufs.keys[0]; *bytes = n * 4; break;
        case RT_DB_VALS: *ptr = r.bufs.vals[0]; *bytes = n * 4; break;
        case RT_DB_NODES: *ptr = r.bufs.nodes; *bytes = tot * 32; break;
        case RT_DB_TRI_S: *ptr = r.bufs.tri_s; *bytes = n * 48; break;
        case RT_DB_WIDE: *ptr = r.bufs.wnodes; *bytes = ni * wide_bytes(r.bufs.warity); break;
        case RT_DB_TOPO: *ptr = r.bufs.topo; *bytes = ni * 16; break;
        case RT_DB_PRE: *ptr = r.bufs.prebuf; *bytes = n * 24; break;
        case RT_DB_SUF: *ptr = r.bufs.sufbuf; *bytes = n * 24; break;
        case RT_DB_TOTALS: *ptr = r.bufs.table; *bytes = (uint64_t)rt::refit_blocks(s->n) * 24; break;
        case RT_DB_CROSS: *ptr = r.dcross; *bytes = cc; break;
        case RT_DB_CROSS_ALL: *ptr = r.dcross_all; *bytes = cc; break;
        default: return fail(RT_EINVAL, "unknown rt_dbuild_buffer selector");
    }
    return RT_OK;
}

#ifdef RT_STAMPS
// diagnostic build only: copy the per-block phase stamps (8 x u64 per block)
// of the build kernels (which = 0) or the sort kernels (which = 1)
rt_status rt_debug_tile_order(const uint32_t* d_order) {
    rt::config_apply(
        [](rt::TraceConfig& c, const char*, int64_t v) {
            c.order_override = reinterpret_cast<const uint32_t*>(v);
            return true;
        },
        "", (int64_t)(intptr_t)d_order);
    return RT_OK;
}

rt_status rt_debug_stamps(int which, void* out, size_t bytes) {
    HIPR(hipDeviceSynchronize());
    HIPR(which == 2 ? rt::read_stamps_trace(out, bytes) : which ? rt::read_stamps_sort(out, bytes) : rt::read_stamps_build(out, bytes));
    return RT_OK;
}
#endif

}  // extern "C"

// rt_launch.h -- host-side launchers of the gfx950 kernels (defined next to
// the kernels in build_kernels.hip / trace_kernels.hip) and the device
// buffer layout of one BVH build.  Used by rt_abi.cpp only.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

namespace rt {

struct BuildParams;

// Device buffers of one scene (SURVEY.md §8(a) layouts; sized for cap_n prims).
struct BuildBufs {
    uint32_t cap_n = 0;
    float* tris = nullptr;          // n*9 fp32, AoS (36 B/tri), 256-B aligned
    uint32_t* keys[2] = {nullptr, nullptr};
    uint32_t* vals[2] = {nullptr, nullptr};
    void* nodes = nullptr;          // (2n-1) x 32 B {lo[3], hi[3], a, esc}; the build writes the internal
                                    // n-1 (leaves: tri_s, launch_leaf_nodes)
    float4* tri_s = nullptr;        // n x 48 B leaf-ordered {v0, v1, v2, prim, leaf escape, 0} for the trace
    uint32_t* parent = nullptr;     // 2n-1, unified index space
    uint4* topo = nullptr;          // n-1 x {left, esc, range_lo, range_hi}
    uint4* wnodes = nullptr;        // n-1 x 64 B (K7w, 4-ary) or 96 B (K7w8, 8-ary) wide trace records
    uint32_t warity = 4;            // the arity wnodes was (or is being) built with: 4 or 8
    uint32_t* counts = nullptr;     // 4 x [tile][256] radix-sort tile digit counts (MSB: [tile][1024])
    uint32_t* bstart = nullptr;     // [1025] MSB bucket starts
    float* prebuf = nullptr;        // n x 6: block-prefix AABB at crossing ends
    float* sufbuf = nullptr;        // n x 6: block-suffix AABB at crossing ends
    float* table = nullptr;         // sparse table over refit-block totals, levels x M x 6
    uint32_t* cross = nullptr;      // crossing internal nodes (list)
    float* partials = nullptr;      // K0 per-block partial bounds
    BuildParams* params = nullptr;  // lo/hi/inv
    uint32_t* zero = nullptr;       // per-build zeroed control words, see zero_layout()
    uint32_t nzero = 0;
    uint32_t ntiles = 0;            // sort tiles at cap_n
    uint32_t m_blocks = 0;          // refit blocks at cap_n
    uint32_t levels = 0;            // sparse-table levels at cap_n
    // the scene's sort: 0 = not yet known (the MSB bucket sort), 1 = MSB, 2 = the
    // 4-pass LSB sort -- a bucket of the first MSB build outgrew one block's LDS
    // sort (clustered geometry: that bucket is sorted by one block through
    // global memory, ~10x the build); a scene's triangles never change
    uint32_t sort_mode = 0;
    uint32_t sort_mode_of = 0;  // the sort (build.sort 1 or 2) whose probe build set sort_mode
    // the gather sort's probe found a run of more than kGatherBinFast
    // identical keys (duplicated geometry; r06: clustered bins alone take the
    // gather's radix path and stay) or, with -DRT_GATHER_SKEW=k, a bucket over
    // k x the mean, but no bucket beyond its LDS: later builds use the MSB
    // bucket sort instead, with its own verdict (r05: the bunny substitute's
    // 70K-tri build 105 -> 82 us, profiles/sort_verdict_r05.log)
    uint32_t gather_off = 0;
};
// keys one MSB bucket may hold for the LDS bucket sort at this n
uint32_t msb_bucket_cap(uint32_t n);
// the same for the gather sort, and whether it handles n at all
uint32_t gather_bucket_cap(uint32_t n);
bool gather_sort_fits(uint32_t n);
struct TraceConfig;

// zero region layout (uint32 words)
constexpr uint32_t kZHist = 0;          // [4][256] digit histograms
constexpr uint32_t kZTileCtr = 1024;    // [4] onesweep tile tickets
constexpr uint32_t kZErr = 1028;        // sticky error bits (reserved)
constexpr uint32_t kZCrossCtr = 1040;   // [kCrossShards] crossing-list shard lengths
constexpr uint32_t kCrossShards = 16;
constexpr uint32_t kZHist4 = 1056;      // [4][256] digit histograms of a probe build's LSB leg
constexpr uint32_t kZDense = 2080;      // a probe build's verdict (k_msb_scan / k_bucket_dense write it)
constexpr uint32_t kZGatherFlags = 2081;  // [2] k_bucket_gather: clustered bins, bucket overflow
constexpr uint32_t kZGatherSkew = 2083;   // k_bucket_dense: the largest bucket > 4x the mean (a probe build)
constexpr uint32_t kZEnd = 2084;        // words zeroed by K0 every build
// past kZEnd, never zeroed by a build: the fused K0+K1's grid barrier
// (self-resetting) and its timeout flag (cleared by the host when it sees it)
constexpr uint32_t kZBar = 2084;
constexpr uint32_t kZFuseErr = 2085;
constexpr uint32_t kZBox = 2088;        // [6] the fused K0+K1's global centroid box (its last block writes it)
constexpr uint32_t kZAlloc = 2096;      // words of the zero region


hipError_t alloc_build(BuildBufs& b, uint32_t n);
void free_build(BuildBufs& b);

struct BuildEvents { hipEvent_t e[7]; bool valid = false; };

// K0..K7w on `stream` for the n tris already in b.tris.  Sorted keys/vals end
// in keys[0]/vals[0].  With ev: e[0] and e[6] around the build, and e[1..5]
// between the stages when `stages`.  cfg: the caller's one config snapshot.
// probed (nullable): the sort (1 MSB, 2 gather) whose verdict this build
// wrote to zero[kZDense] -- the caller reads it after the build to set
// sort_mode/sort_mode_of -- else 0.
// allow_fused: the caller holds fused_gate(device) for this build (no other
// fused build can be in flight on the device); launch_build then runs K0 + K1
// as one launch with a grid barrier when the gather sort is used and the
// grid fits the device at once (fused_k01_fits).  *fused_out: whether it did
// (the caller then checks zero[kZFuseErr] after the build).
// host_flags (nullable): device pointer of 8 mapped pinned host words that
// receive zero[kZDense .. kZDense + 8) at the end of the build (k_topo_refit
// block 0 writes them; n >= 1), the verdict words the caller reads after its
// synchronize.
hipError_t launch_build(const BuildBufs& b, uint32_t n, hipStream_t stream, BuildEvents* ev, bool stages,
                        const TraceConfig& cfg, uint32_t* probed, bool allow_fused = false,
                        bool* fused_out = nullptr, uint32_t* host_flags = nullptr);
bool fused_k01_fits(uint32_t n);  // every sort tile's block co-resident on the current device
std::mutex& fused_gate(int device);
// the sort launch_build would use: 0 LSB, 1 MSB scatter, 2 gather
uint32_t build_sort_kind(const BuildBufs& b, uint32_t n, const TraceConfig& cfg);

// K4..K7w alone (rt_stage_refit): sorted keys/vals already in keys[0]/vals[0]
// and the soup in tris.
hipError_t launch_refit_stage(const BuildBufs& b, uint32_t n, hipStream_t stream);

// Distributed build phases (rt_dbuild_*; DESIGN.md "Distributed build").
hipError_t launch_dbuild_bounds(const BuildBufs& b, uint32_t lo, uint32_t cnt, hipStream_t s);
hipError_t launch_dbuild_keys(const BuildBufs& b, uint32_t lo, uint32_t cnt, const float* boxes, uint32_t nboxes,
                              hipStream_t s);
hipError_t launch_dbuild_sort(uint32_t* keys[2], uint32_t* vals[2], uint32_t cnt, const BuildBufs& b, hipStream_t s);
hipError_t launch_dbuild_subtrees(const BuildBufs& b, uint32_t n, uint32_t block0, uint32_t nblocks, hipStream_t s);
hipError_t launch_dbuild_merge(const BuildBufs& b, uint32_t n, hipStream_t s);
uint32_t dbuild_cross_cap(uint32_t n);  // crossing-list entries per shard (kCrossShards shards)
uint32_t refit_blocks(uint32_t n);      // kRefitT-leaf blocks of k_topo_refit

// Stage launchers for parity entry points (buffers sized by the caller).
hipError_t launch_bounds_only(const float* tris, uint32_t n, float* partials, BuildParams* params, hipStream_t s);
hipError_t launch_morton(const float* tris, uint32_t n, const BuildParams* params, uint32_t* keys,
                         uint32_t* vals, uint32_t* ghist, uint32_t* counts0, hipStream_t s);
hipError_t launch_digit_hist(const uint32_t* keys, uint32_t n, uint32_t* ghist, hipStream_t s);
hipError_t launch_tile_hist0(const uint32_t* keys, uint32_t n, uint32_t* counts0, hipStream_t s);
// 4 passes 0->1->0->1->0; ghist = [4][256] digit totals; counts[p] = [tile][256]
// (counts[0] filled by K1 or launch_tile_hist0, counts[1..3] scratch).
hipError_t launch_sort(uint32_t* keys[2], uint32_t* vals[2], uint32_t n, const uint32_t* ghist, uint32_t* counts[4],
                       hipStream_t s);
hipError_t launch_karras(const uint32_t* keys, const uint32_t* svals, const float* tris, uint32_t n, uint4* topo,
                         uint32_t* parent, void* nodes, float4* tri_s, hipStream_t s);
uint32_t sort_tiles(uint32_t n);
uint32_t bounds_grid(uint32_t n);  // K0/K1 workgroups (8 tris per thread)
hipError_t launch_leaf_tris(const void* nodes, const float* tris, uint32_t n, float4* tri_s, hipStream_t s);
// binary leaf nodes (2n-1 node array, leaves L0 + k) from the triangle
// records: the build writes internal nodes only (store_leaf_tri)
hipError_t launch_leaf_nodes(const float4* tri_s, uint32_t n, void* nodes, hipStream_t s);

struct CamF { float eye[3], w00[3], du[3], dv[3]; };

// trace.coop_cap_tiles = -1 (the default): the step cap one rank's tiles use,
// by rank count.  A rank of a two-way split holds twice the tiles of P = 4
// and is partly throughput-bound, so it gains from queueing fewer rays:
// P=2 0.213 -> 0.206 ms at 88 against 80, while P=4 is best at 80.  With the
// rank kernels' 20-entry stacks (r04) P=8 is best lower: 72 steps, orbit max
// over ranks 0.1172 / 0.1182 ms against 0.1229 / 0.1218 at 80 (64: 0.1187 /
// 0.1180; profiles/coop_cap_tiles_orbit_r04.log).
constexpr uint32_t kCoopCapAuto = 0xFFFFFFFFu;
inline uint32_t coop_cap_for_tiles(uint32_t knob, uint32_t nranks) {
    if (knob != kCoopCapAuto) return knob;
    return nranks <= 2 ? 88u : nranks <= 4 ? 80u : 72u;
}
// full frames: auto = 96 steps for 1-spp frames on 256-thread tiles, whose
// k_trace instance (SPPC = 1) has the queue at no register cost (72 VGPRs
// either way); off otherwise (the generic queue kernel drops a wave per SIMD).
// tools/ab_moving.py, profiles/ab_coop_full_r03.log
inline uint32_t coop_cap_for_frame(uint32_t knob, uint32_t spp, bool small) {
    if (knob != kCoopCapAuto) return knob;
    return spp == 1 && !small ? 96u : 0u;
}
// samples in lanes (k_trace_sl, one ray per lane): auto = no queue.  r05,
// bench orbit (tools/rank_emul.py, profiles/ab_sl_coop_cap_r05.log): the
// queue's group pass costs more than the single-ray tail it removes -- soup-10M
// 4Kx4 full frame 3.98 ms off / 4.09 at 160 / 4.16 at 96, P=8 max rank 0.607 /
// 0.632 at 128 / 0.77 at 72 / 0.81 at 48; Sponza substitute 16 spp full 1.97 /
// 1.97 / 1.94, P=8 0.256 / 0.262 / 0.277 ms.
inline uint32_t coop_cap_for_sl(uint32_t knob) { return knob == kCoopCapAuto ? 0u : knob; }

// Trace kernel selection / tuning (rt_config_set); every setting gives
// bit-identical hits and images.
struct TraceConfig {
    uint32_t variant = 0;       // 0 wide per-pixel (default), 2 binary per-pixel (1, the r01 wide pool with
                                // refill, was removed in r06: measured slower, profiles/rejected_knobs_r06.patch)
    uint32_t wg = 256;          // per-pixel kernels: threads per workgroup (256 = 16x16 tile, 64 = 8x8)
    uint32_t wg_tiles = 64;     // same, for one rank's tiles of a multi-GPU frame (nranks > 1)
    uint32_t spp_lanes = 2;     // samples in lanes (k_trace_sl) for 2..16 (power of two) spp: 2 = full frames and
                                // one rank's tiles (default), 1 = tiles only, 0 = off (a lane loops over its samples)
    uint32_t stack_cap = 0;     // wide stack entries used (tests force the overflow path); 0 = the arity's
                                // whole stack (14 entries for 4-ary records, 18 for 8-ary)
    uint32_t path_wave = 1;     // path mode: 0 megakernel, 1 wavefront (default: faster on soup-1M and Sponza)
    uint32_t path_wg = 64;      // path megakernel: threads per block (64 = 8x8 quadrant, 256 = 16x16 tile)
    uint32_t path_sort = 0;     // wavefront: top key bytes the ray queue is sorted by (0 = unsorted, default)
    uint32_t path_batch = 0;    // wavefront: paths per batch (0 = 4M)
    uint32_t stage_events = 0;  // build: record the per-stage events (rt_bvh_build_times); else total only
    uint32_t tile_order = 1;    // 1: longest-first from the previous same-size frame's wave times; 0: row-major
    uint32_t px_sort = 1;       // with tile_order: each tile's pixels to lanes costliest first (previous
                                // frame); 1 = full frames only, 2 = also one rank's tiles, 0 = off
    uint32_t wide_arity = 4;    // build.wide_arity: 4 = K7w 64-B records, 8 = K7w8 96-B records (greedy cut)
    uint32_t fuse_k01 = 1;      // build.fuse_k01: 1 = K0 + K1 as one launch with a grid barrier when the grid
                                // is co-resident and no other fused build runs on the device (gather sort);
                                // 2 = even when it cannot be co-resident (tests of the barrier's timeout)
    uint32_t sort_msb = 2;      // build.sort, for 2 <= n <= kMsbBigMaxN: 2 = tile-bucketed gather sort (default),
                                // 1 = MSB scatter + bucket sort, 0 = 4-pass LSB always
    uint32_t render_emulate = 0;  // rt_render(ngpus > 1): 1 = every rank's replica on the scene's device, gather
                                  // by device copies (tests on a one-GPU box); 0 = one device per rank + RCCL
    uint32_t render_rccl1 = 0;    // rt_render(ngpus = 1) through the tiled + RCCL path (1-rank communicator)
    uint32_t coop_cap = kCoopCapAuto;  // primary full frames: rays past this many wide steps finish in
                                  // k_trace_coop (lane groups per ray); 0 = off; auto (default):
                                  // coop_cap_for_frame
    uint32_t coop_cap_tiles = kCoopCapAuto;  // the same for one rank's tiles of a multi-GPU frame;
                                  // auto (default): coop_cap_for_tiles (tools/coop_sweep.py,
                                  // profiles/coop_sweep_r02b.log, profiles/coop_sweep_hi_r02.log)
    uint32_t coop_lanes = 32;     // lanes per queued ray in k_trace_coop: 16, 32 or 64
    uint32_t coop_max = 65536;    // heavy-ray queue entries per frame shape (rays beyond it trace on alone)
    const uint32_t* order_override = nullptr;  // diagnostic builds: a caller-given dispatch order
    uint32_t poison = 0;          // debug.poison: fill every new device allocation with 0xFF bytes, so a
                                  // read of a byte nothing wrote is deterministic (and visible)
    uint32_t lds_scribble = 0;    // debug.lds_scribble: before every kernel launch, fill the LDS of the
                                  // CUs with a fresh pseudo-random pattern, so a kernel that reads LDS
                                  // it did not write gives a different (wrong) result every launch
    uint32_t force_lsb_redo = 0;  // debug.force_lsb_redo: treat every gather-sort build as if a bucket
                                  // had overflowed (tests the host's discard-and-redo branch)
};
// Both debug knobs also start on from the environment (RT_DEBUG_POISON=1,
// RT_DEBUG_LDS_SCRIBBLE=1), so a whole test suite can run under them.

// Every kernel launch of the library goes through RT_KLAUNCH: with
// debug.lds_scribble on, the scribble kernel runs first on the same stream.
void lds_scribble_if(hipStream_t s);
#define RT_KLAUNCH(kernel, grid, block, lds, stream, ...)                  \
    do {                                                                   \
        ::rt::lds_scribble_if(stream);                                     \
        hipLaunchKernelGGL(kernel, grid, block, lds, stream, __VA_ARGS__); \
    } while (0)

// Every device buffer of the library is allocated here: hipMalloc, then
// with debug.poison a 0xFF fill completed before the buffer is handed out.
hipError_t dev_alloc(void** p, size_t bytes);
template <class T>
inline hipError_t dev_alloc(T** p, size_t bytes) { return dev_alloc(reinterpret_cast<void**>(p), bytes); }

constexpr uint32_t kCoopEntryBytes = 208;  // heavy-ray queue entry (trace_kernels.hip kCoopEntry x 16 B: 19 pending subtrees)
// 8-ary records are read through 32-bit buffer offsets: the last record ends
// at (n-1) x 96 B, which must not pass 2^32 - 1 (n <= 44,739,243; above that
// the build writes 4-ary records, whose (n-1) x 64 B fit up to n = 2^26)
constexpr uint32_t kWide8MaxN = 0xFFFFFFFFu / 96u + 1u;
static_assert((uint64_t)(kWide8MaxN - 1) * 96u <= 0xFFFFFFFFull && (uint64_t)kWide8MaxN * 96u > 0xFFFFFFFFull,
              "largest n whose 8-ary records fit 32-bit offsets");

// Per-launch tile scheduling state (owned by the scene, one per frame shape).
struct TileSched {
    uint32_t* order = nullptr;      // [nb] dispatch index -> tile slot
    uint32_t* order_next = nullptr; // [nb] the next frame's, sorted by this frame's k_trace (full frames)
    uint32_t* cost_prev = nullptr;  // [nb] previous frame's per-tile wave time
    uint32_t* cost_cur = nullptr;   // [nb] this frame's, written by k_trace
    uint32_t* cost_ema = nullptr;   // [nb] running mean of the frames' tile costs: the order's key
    uint16_t* px_prev = nullptr;    // [nb][256] previous frame's per-pixel steps (trace.px_sort)
    uint16_t* px_cur = nullptr;     // [nb][256] this frame's
    uint4* coop_q = nullptr;        // [coop_qcap] x kCoopEntryBytes heavy-ray queue (trace.coop_cap)
    uint32_t* coop_ctr = nullptr;   // [2] queue counters, alternating frames
    uint32_t coop_qcap = 0;
    uint32_t coop_par = 0;          // which counter this frame uses
    CamF prev_cam{};                // camera of the previous frame of this shape (pixel order only if equal)
    bool prev_cam_valid = false;
    bool coop_fresh = true;         // queue (re)allocated: zero both counters before the first launch
    bool have_prev = false;
    bool order_ready = false;       // `order` for this frame already sorted by the previous frame's k_trace_coop
    bool fresh = true;              // maps (re)allocated: clear both before the first launch
    // Queue skip (automatic caps): the queue length k_trace_coop reported for
    // the latest queue-on frame of this shape (mapped pinned host word; ~0u =
    // not yet known), and the queue-off frames since.  Best effort (ADVICE
    // r05): the host reads the word without waiting for the frame that writes
    // it, so with frames queued ahead of the host the value may be a few
    // frames old; it only decides whether a frame runs the queue, never a
    // pixel's result.
    uint32_t* q_host = nullptr;
    uint32_t* q_dev = nullptr;
    uint32_t q_frames = 0;
};
// The HIP handle for a stream argument: the ABI's hipStreamLegacy (the null
// stream, torch's default) is passed to HIP as 0, which every HIP call takes
// (hipStreamWaitEvent on the legacy handle itself does not).
inline hipStream_t hip_stream(hipStream_t s) { return s == hipStreamLegacy ? nullptr : s; }

// The process-wide knobs (rt_config_set).  Every launcher works on one
// consistent copy taken under the config lock, so a concurrent rt_config_set
// on another thread never tears a launch's settings.
TraceConfig config_snapshot();
// apply f to the config under the lock; f returns false to reject (no change)
bool config_apply(bool (*f)(TraceConfig&, const char*, int64_t), const char* key, int64_t value);
// highest device index the per-device caches cover
constexpr int kMaxDevices = 64;

// sched: the scene's tile-order state for this frame shape (nullptr:
// row-major order, no cost map).
// wnodes: the K7w wide records (nullptr: binary traversal only).  With
// binary_counts the kernel is the binary one, so `counters` are the §9.7
// node/triangle counts the oracle reports; otherwise they count the running
// kernel's own fetches (wide: records and triangle loads).
// warity: the arity wnodes holds (BuildBufs::warity).
hipError_t launch_trace(const void* nodes, const uint4* wnodes, uint32_t warity, const float4* tri_s, uint32_t n,
                        const CamF& cam,
                        uint32_t w, uint32_t h, uint32_t spp, uint32_t rank, uint32_t nranks, bool packed,
                        void* hits, void* rgba, unsigned long long* counters, bool binary_counts,
                        TileSched* sched, hipStream_t s);
// Shadow mode: primary hits into `hits`, Lambert + shadow-ray
// shaded image into `rgba`; tris = the scene's AoS triangles (normals).
hipError_t launch_trace_shadow(const void* nodes, const uint4* wnodes, uint32_t warity, const float4* tri_s,
                               const float* tris,
                               uint32_t n, const CamF& cam, uint32_t w, uint32_t h, uint32_t spp,
                               const float light[3], float ambient, void* hits, void* rgba,
                               unsigned long long* counters, hipStream_t s);
// Path mode: primary hits into `hits`, diffuse-path image into
// `rgba`; counters (nullable): [0] node records, [1] tri records, [2] rays.
hipError_t launch_trace_path(const void* nodes, const uint4* wnodes, uint32_t warity, const float4* tri_s,
                             const float* tris,
                             uint32_t n, const CamF& cam, uint32_t w, uint32_t h, uint32_t spp, const float light[3],
                             float sky, uint32_t max_depth, void* hits, void* rgba, unsigned long long* counters,
                             hipStream_t s);
// Wavefront path mode (same images as launch_trace_path): per-path state in
// SoA arrays, a ray queue per depth, optionally sorted by a coherence key.
struct PathBufs {
    uint32_t cap = 0;               // paths per batch (a multiple of 256*spp is used)
    float* f = nullptr;             // [16][cap] o(3) d(3) L(3) beta(3) w(3) seg_t
    uint32_t* u = nullptr;          // [4][cap] rng state, flags, seg_prim, shadow visibility
    float4* rays = nullptr;         // [2*cap][2] {o, tmax}, {d, pid | shadow << 31}
    uint32_t* keys[2] = {nullptr, nullptr};  // [2*cap] ray coherence keys (ping-pong)
    uint32_t* vals[2] = {nullptr, nullptr};  // [2*cap] queue slots (ping-pong)
    uint32_t* counts = nullptr;     // [tiles(2*cap)][256] sort tile counts
    uint32_t* ghist = nullptr;      // [4][256] digit histograms of the keys
    uint32_t* qcount = nullptr;     // queue length (device word)
    uint32_t* hq = nullptr;         // pinned host copy of qcount
};
hipError_t alloc_path(PathBufs& b, uint32_t cap);
void free_path(PathBufs& b);
// sort_digits: 0 = trace the queue in emission order; 1..4 = stable LSB radix
// sort of the queue by the top `sort_digits` bytes of the ray key first.
hipError_t launch_path_wavefront(const void* nodes, const uint4* wnodes, uint32_t warity, const float4* tri_s,
                                 const float* tris,
                                 const BuildParams* params, uint32_t n, const CamF& cam, uint32_t w, uint32_t h,
                                 uint32_t spp, const float light[3], float sky, uint32_t max_depth, void* hits,
                                 void* rgba, unsigned long long* counters, PathBufs& pb, uint32_t sort_digits,
                                 hipStream_t s);
// top `digits` (1..4) bytes of 32-bit keys, stable; returns the buffer index
// (0 or 1) holding the result.  counts: tiles(n)*256 words; ghist: [4][256]
// totals of all four digits (launch_digit_hist).
// MSB bucket sort of 30-bit keys (2 <= n <= kMsbBigMaxN): keys[0]/vals[0] ->
// keys[0]/vals[0] via keys[1]/vals[1]; ghist = [1024] bucket totals and
// counts = [tile][1024] bucket counts (both from k_morton<true>); scratch:
// ceil(tiles/32) x 1024 words, needed above kMsbMaxN.
// dense: when set, k_msb_scan writes 1 there if a bucket holds more than
// msb_bucket_cap(n) keys (else 0) and the scatter/bucket kernels run only on 0.
hipError_t launch_sort_msb(uint32_t* keys[2], uint32_t* vals[2], uint32_t n, const uint32_t* ghist, uint32_t* counts,
                           uint32_t* bstart, uint32_t* scratch, hipStream_t s, uint32_t* dense = nullptr);
// A scene's first sort: the MSB sort gated on its own verdict (*dense == 0),
// then the 4-pass LSB sort gated on *dense == 1 (ghist4: [4][256] zeroed
// words; counts as for launch_sort_msb).  The caller reads *dense afterwards.
hipError_t launch_sort_probe(uint32_t* keys[2], uint32_t* vals[2], uint32_t n, const uint32_t* ghist,
                             uint32_t* counts, uint32_t* bstart, uint32_t* scratch, uint32_t* ghist4,
                             uint32_t* dense, hipStream_t s);
// The tile-bucketed gather sort (sort_kernels.hip): words = K1's
// (k_morton_tb) tile-bucketed words, tb = its [tile][1024] run table, ghist =
// its [1024] bucket totals -> kout/vout sorted by (key, index).  flags: [0]
// set when a bin of 2^10 keys' low bits held more than 64 keys (clustered:
// exact, but the scene's later builds should use the LSB sort), [1] set when
// a bucket did not fit one block's LDS (that bucket is NOT sorted: rebuild
// with the LSB sort).  dense (a probe build): k_bucket_dense writes 1 there
// when a bucket exceeds the LDS capacity, and the bucket kernel runs on 0.
// bstart: [1025] bucket starts written by the bucket blocks.
hipError_t launch_sort_gather(const uint32_t* words, const uint32_t* tb, uint32_t n, const uint32_t* ghist,
                              uint32_t* kout, uint32_t* vout, uint32_t* flags, uint32_t* bstart, uint32_t* dense,
                              hipStream_t s);
// the 4-pass LSB sort of keys[0]/vals[0] (index order), every launch gated on
// *dense == 1; ghist4 and counts[0] from k_morton<false>
hipError_t launch_sort_lsb_gated(uint32_t* keys[2], uint32_t* vals[2], uint32_t n, const uint32_t* ghist4,
                                 uint32_t* counts, const uint32_t* dense, hipStream_t s);
hipError_t launch_sort_top(uint32_t* keys[2], uint32_t* vals[2], uint32_t n, const uint32_t* ghist, uint32_t* counts,
                           uint32_t digits, uint32_t* out_buf, hipStream_t s);
hipError_t launch_unpack(const void* slabs, uint32_t tiles_per_slab, uint32_t w, uint32_t h, uint32_t nranks,
                         void* img, hipStream_t s);
// the same for packed hit slabs [rank][tile][256 px][spp] -> hits[(y*w+x)*spp+s]
hipError_t launch_unpack_hits(const void* slabs, uint32_t tiles_per_slab, uint32_t w, uint32_t h, uint32_t spp,
                              uint32_t nranks, void* hits, hipStream_t s);
uint32_t tiles_for_rank(uint32_t w, uint32_t h, uint32_t rank, uint32_t nranks);
hipError_t launch_intersect(uint32_t count, const float* o, const float* d, const float* tri, const float* tb,
                            uint32_t* hit, float* tuv, hipStream_t s);
#ifdef RT_STAMPS
hipError_t read_stamps_build(void* out, size_t bytes);
hipError_t read_stamps_sort(void* out, size_t bytes);
hipError_t read_stamps_trace(void* out, size_t bytes);
#endif
hipError_t launch_minmax(uint32_t count, const float* a, const float* b, float* out, hipStream_t s);

}  // namespace rt

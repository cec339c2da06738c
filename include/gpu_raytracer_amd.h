/*
 * gpu_raytracer_amd.h -- the drop-in C-ABI of the MI355X-native BVH-build +
 * ray-trace hot path (librtamd.so).
 *
 * Reference interface: NONE EXISTS.  SoslanGM/gpu_raytracer @ v0 (mounted at
 * /root/reference) contains only README.md:1-2 and test.txt:1; the
 * "scene-load / framebuffer-dump entry points" that BASELINE.json:5 asks to
 * keep drop-in are not present at that revision.  Each
 * entry point below therefore cites the SURVEY.md §8(b) line it implements;
 * a future GLSL/Vulkan-era reference host would bind these (see
 * INTEGRATION.md for the ctypes/C binding a maintainer adds).
 *
 * Conventions:
 *   - every function returns rt_status: 0 = RT_OK, negative = error; the
 *     thread-local message is rt_last_error();
 *   - the caller owns every pointer argument; the library copies inputs and
 *     writes into caller buffers; scenes are opaque, freed by rt_scene_free;
 *   - distinct scenes may be used from distinct threads; calls on one scene
 *     are not reentrant; rt_config_set may be called from any thread (every
 *     launch works on one consistent snapshot of the knobs);
 *   - a scene holds one BVH replica per device it was built on (SURVEY.md
 *     §8(e): the BVH is replicated); multi-GPU rendering is internal to
 *     rt_render(ngpus > 1) -- replicas, tile deal, RCCL gather, unpack;
 *   - device work the *_device entry points queue on a caller stream is
 *     ordered by the library: a later launch of the same scene on another
 *     stream waits for it, and rt_bvh_build / rt_bvh_load / rt_scene_free
 *     wait for it before touching the scene's buffers;
 *   - HIP failures map to RT_EDEVICE, RCCL-side failures to RT_ECOMM;
 *   - there is NO CPU fallback: without a usable gfx950 device every compute
 *     entry point fails with RT_EDEVICE.
 *   - environment RT_ROCTX=1: the device entry points are wrapped in roctx
 *     ranges named after them (rocprofv3 --marker-trace).
 *
 * Numeric contract: SURVEY.md §9 (Appendix A).  Morton codes, sorted indices,
 * topology, AABBs and images are bit-exact vs the CPU oracle; hits match the
 * oracle's prim and are within 1 ulp per component (0 ulp expected).
 */
#ifndef GPU_RAYTRACER_AMD_H
#define GPU_RAYTRACER_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_SENTINEL 0xFFFFFFFFu
/* rt_bvh_build backends: the library has no CPU backend --
 * RT_BACKEND_CPU is rejected with RT_EINVAL (the CPU oracle under oracle/ is
 * test infrastructure, never a fallback). */
#define RT_BACKEND_CPU 0
#define RT_BACKEND_HIP 1

typedef struct rt_scene rt_scene; /* opaque, owned by the library */

/* host-precomputed ray frame (floats). */
typedef struct { float eye[3], w00[3], du[3], dv[3]; } rt_camera;
/* 16-B hit record; miss = {+inf, 0, 0, RT_SENTINEL}. */
typedef struct { float t, u, v; uint32_t prim; } rt_hit;
/* 32-B node; internal 0..n-2, leaf k at n-1+k; a = left
 * child (internal) or prim index (leaf); esc = escape link or RT_SENTINEL. */
typedef struct { float lo[3], hi[3]; uint32_t a, esc; } rt_node;

typedef enum {
    RT_OK = 0,
    RT_EINVAL = -1,
    RT_ENOMEM = -2,
    RT_EIO = -3,
    RT_EDEVICE = -4,
    RT_ECOMM = -5
} rt_status;

/* per-stage device times of the last build, milliseconds (hipEvents);
 * wide = K7w, the 4-ary trace records derived from the binary tree.
 * sort_kind: the sort this scene's builds use after the last one (its
 * verdict applied): 0 the 4-pass LSB radix sort, 1 MSB scatter + bucket
 * sort, 2 the tile-bucketed gather sort; fused_k01: the last build ran
 * K0 + K1 as one launch (build.fuse_k01).  fused_fallback: the fused
 * launch's grid barrier gave up (its grid was not co-resident) and the build
 * was redone with two launches; lsb_redo: a gather-sort bucket overflowed and
 * the build was redone with the LSB sort.  After a redo the stage fields are
 * the redo's and `total` is both builds together.  (Layout of rt_version 0.3:
 * 0.2 had neither redo field.) */
typedef struct {
    double bounds, morton, sort, topology, refit, wide, total;
    uint32_t sort_kind, fused_k01, fused_fallback, lsb_redo;
} rt_build_times;

/* ---- scene ingest (SURVEY.md §8(b) rt_scene_load_obj / rt_scene_from_soup) ---- */
rt_status rt_scene_from_soup(const float* tris, uint32_t n, rt_scene** out); /* copies n*9 floats */
rt_status rt_scene_load_obj(const char* path, rt_scene** out);
rt_status rt_scene_generate_soup(uint32_t n, uint64_t seed, rt_scene** out); /* SURVEY.md §9.9 */
/* RTSOUP1 binary soup: "RTSOUP1\0", u32 version 1,
 * u32 0, u64 n, then n x 9 little-endian float32 -- the rt_scene_from_soup layout. */
rt_status rt_scene_load_soup(const char* path, rt_scene** out);
rt_status rt_scene_save_soup(const rt_scene* s, const char* path);
rt_status rt_scene_num_tris(const rt_scene* s, uint32_t* n_out);
rt_status rt_scene_get_tris(const rt_scene* s, float* tris_out); /* n*9 floats */
rt_status rt_scene_set_device(rt_scene* s, int device);          /* default 0; before first build */
void rt_scene_free(rt_scene* s);

/* SURVEY.md §9.7 camera: double math on the host, rounded to float. */
rt_status rt_camera_look_at(const double eye[3], const double at[3], const double up[3],
                            double vfov_deg, uint32_t w, uint32_t h, rt_camera* out);

/* ---- BVH build (SURVEY.md §8(b) rt_bvh_build(scene, backend, device_mask,
 * ms)).  backend: RT_BACKEND_HIP (RT_BACKEND_CPU -> RT_EINVAL).  device_mask:
 * bit d = build a replica on device d, concurrently, one stream each (the
 * lowest device of a scene's first build becomes its primary device); 0 = the
 * scene's device (rt_scene_set_device, default 0).  A bit naming a device
 * that is not visible -> RT_EDEVICE.  Uploads the soup once per device (H2D
 * is not part of ms_out), then runs K0..K7w.  ms_out: device time of the
 * build (hipEvents around it; the longest replica). */
rt_status rt_bvh_build(rt_scene* s, int backend, uint32_t device_mask, double* ms_out);
/* devices holding a built replica, primary first (call with max = 0 to size) */
rt_status rt_bvh_replicas(const rt_scene* s, uint32_t max, int* devices, uint32_t* count_out);
/* times of the last build: `total` always; the per-stage fields only when
 * the build ran with rt_config_set("build.stage_events", 1) (0 otherwise --
 * the extra events cost GPU time, so timed builds run without them) */
rt_status rt_bvh_build_times(const rt_scene* s, rt_build_times* out);
/* the same, size-checked: out_size = sizeof(rt_build_times) as
 * the caller was compiled; only that many bytes are written, so a caller
 * built against the 0.2 header (64 B, no redo fields) is safe.  Smaller than
 * 64 -> RT_EINVAL.  Prefer this entry point. */
rt_status rt_bvh_build_times_sized(const rt_scene* s, rt_build_times* out, size_t out_size);
/* Device-resident BVH exchange ("rank 0 builds and then
 * broadcasts", the alternative to every rank building its replica):
 * rt_bvh_prepare uploads the soup and allocates the BVH buffers without
 * building; rt_bvh_device_sections lists the device buffers that make up a
 * built BVH (the RTBVH1 sections: params, sorted keys, sorted vals, nodes,
 * parent, tri_s, wide records) -- a receiver fills them (e.g. an RCCL
 * broadcast from a rank that built) and calls rt_bvh_mark_built.  count_out
 * = number of sections (call with max = 0 to size the arrays). */
rt_status rt_bvh_prepare(rt_scene* s);
rt_status rt_bvh_device_sections(rt_scene* s, uint32_t max, void** ptrs, uint64_t* bytes, uint32_t* count_out);
rt_status rt_bvh_mark_built(rt_scene* s);
/* Read back the device BVH (any pointer may be NULL): nodes[2n-1],
 * sorted keys/vals[n], parent[2n-1], bounds[9] = lo[3], hi[3], inv[3]. */
rt_status rt_bvh_read(const rt_scene* s, rt_node* nodes, uint32_t* sorted_keys,
                      uint32_t* sorted_vals, uint32_t* parent, float* bounds9);
/* BVH cache: rt_bvh_save writes a built scene's
 * device BVH (RTBVH1: header with a hash of the triangles, then the buffers
 * the trace reads); rt_bvh_load restores it into a scene with the SAME
 * triangles instead of rt_bvh_build (RT_EINVAL for other triangles, RT_EIO
 * for a bad file). */
rt_status rt_bvh_save(const rt_scene* s, const char* path);
rt_status rt_bvh_load(rt_scene* s, const char* path);
/* Read back the wide trace records, one per binary internal node: (n-1) x 64 B
 * for 4-ary K7w records, (n-1) x 96 B for 8-ary K7w8 records (layouts:
 * gpu_raytracer_amd/csrc/rt_device.h); nothing for n < 2.  The arity is the
 * build's rt_config_set("build.wide_arity", 4 | 8) (8 only for n <= RT_WIDE8_MAX_N), as
 * reported by rt_bvh_wide_arity.  SURVEY.md §8(f) row 1 ("4/8-wide"). */
rt_status rt_bvh_read_wide(const rt_scene* s, void* records);
/* largest n built with 8-ary records: the trace reads them through 32-bit
 * byte offsets, and the last record ends at (n-1) x 96 B <= 2^32 - 1; larger
 * scenes get 4-ary records whatever build.wide_arity says */
#define RT_WIDE8_MAX_N 44739243u
rt_status rt_bvh_wide_arity(const rt_scene* s, uint32_t* arity_out);

/* ---- render (SURVEY.md §8(b) rt_render(scene, cam, w, h, spp, ngpus, hits,
 * rgba)).  hits_out: w*h*spp records, rgba_out: w*h*4 bytes; either may be
 * NULL.  ngpus = 1: the primary replica renders the frame.  ngpus > 1
 * (SURVEY.md §3(iii), §8(e)): replicas on ngpus devices (the scene's build
 * replicas first, the missing ones built on the lowest free devices), tile t
 * traced by replica t mod ngpus into a packed slab, the slabs gathered to
 * the primary with RCCL (ncclGather over xGMI, one communicator per device
 * list, cached on the scene) and unpacked there.  ngpus > visible devices ->
 * RT_EDEVICE; RCCL failures -> RT_ECOMM.  The image and hits are identical
 * for every ngpus.  Exactly SURVEY.md §8(b)'s prototype (SURVEY.md:291-292). */
rt_status rt_render(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp, uint32_t ngpus,
                    rt_hit* hits_out, uint8_t* rgba_out);
/* rt_render plus ms_out (nullable): device time of the frame (trace ..
 * unpack), from events on the stream the kernels run on. */
rt_status rt_render_timed(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp, uint32_t ngpus,
                          rt_hit* hits_out, uint8_t* rgba_out, double* ms_out);
/* deterministic work counters of a render with the §9.7 binary traversal
 * (the oracle's counters): [0] nodes fetched, [1] tris tested */
rt_status rt_render_counters(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h,
                             uint32_t spp, uint64_t counters_out[2]);
/* Shadow mode (contract in DESIGN.md "Shadow mode"):
 * the §9.7 primary render, then one any-hit shadow ray per primary hit
 * toward the point light light[3]; the image is (u, v, 1-u-v) scaled by
 * ambient + (1 - ambient) * Lambert * visibility.  hits_out = primary hits. */
rt_status rt_render_shadow(rt_scene* s, const rt_camera* cam, const float light[3], float ambient,
                           uint32_t w, uint32_t h, uint32_t spp, rt_hit* hits_out, uint8_t* rgba_out,
                           double* ms_out);
rt_status rt_render_shadow_device(rt_scene* s, const rt_camera* cam, const float light[3], float ambient,
                                  uint32_t w, uint32_t h, uint32_t spp, void* d_hits, void* d_rgba,
                                  void* stream, double* ms_out);
/* work of the shadow-mode kernel (primary + shadow rays): [0] node records
 * fetched, [1] triangle records loaded */
rt_status rt_render_shadow_work(rt_scene* s, const rt_camera* cam, const float light[3], float ambient,
                                uint32_t w, uint32_t h, uint32_t spp, uint64_t counters_out[2]);
/* Path mode (SURVEY.md §8(f) row 3 "simple path tracing"; contract in
 * DESIGN.md "Path mode"): per sample a diffuse path of up to 1 + max_depth
 * segments (max_depth <= 64) with next-event estimation toward the point
 * light light[3] and sky radiance `sky` for escaped bounce rays; per-triangle
 * albedo from pcg_hash(prim).  hits_out = primary hits.  Bit-identical to the
 * oracle's orc_render_path. */
rt_status rt_render_path(rt_scene* s, const rt_camera* cam, const float light[3], float sky,
                         uint32_t max_depth, uint32_t w, uint32_t h, uint32_t spp, rt_hit* hits_out,
                         uint8_t* rgba_out, double* ms_out);
rt_status rt_render_path_device(rt_scene* s, const rt_camera* cam, const float light[3], float sky,
                                uint32_t max_depth, uint32_t w, uint32_t h, uint32_t spp, void* d_hits,
                                void* d_rgba, void* stream, double* ms_out);
/* work of the path-mode kernel: [0] node records fetched, [1] triangle
 * records loaded, [2] rays traced (primary + bounce + shadow) */
rt_status rt_render_path_work(rt_scene* s, const rt_camera* cam, const float light[3], float sky,
                              uint32_t max_depth, uint32_t w, uint32_t h, uint32_t spp,
                              uint64_t counters_out[3]);
/* work of the configured (default: wide) trace kernel itself: [0] node
 * records fetched (64 B wide / 32 B binary), [1] triangle records loaded */
rt_status rt_render_work(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h,
                         uint32_t spp, uint64_t counters_out[2]);
/* Device-resident render of the full image into caller device buffers
 * (d_hits: w*h*spp records or NULL; d_rgba: w*h*4 bytes or NULL) on `stream`
 * (NULL = the scene's own non-blocking stream, unordered with the caller's
 * other work; the HIP null stream, e.g. torch's default stream, is selected
 * with hipStreamLegacy, (void*)1).  Asynchronous unless ms_out != NULL, in
 * which case the trace kernel is bracketed by hipEvents and waited for. */
rt_status rt_render_device(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp,
                           void* d_hits, void* d_rgba, void* stream, double* ms_out);

/* ---- image-tile sharding: 16x16-pixel tiles, tile t goes
 * to rank t mod nranks.  Device pointers; stream = hipStream_t (hipStreamLegacy
 * for the null stream) or NULL for the scene's stream.  packed_rgba: rt_tiles_for_rank() * 1024 bytes;
 * packed_hits (nullable): tiles * 256 * spp records. */
uint32_t rt_tiles_for_rank(uint32_t w, uint32_t h, uint32_t rank, uint32_t nranks);
rt_status rt_render_tiles_device(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h,
                                 uint32_t spp, uint32_t rank, uint32_t nranks,
                                 void* d_packed_rgba, void* d_packed_hits, void* stream,
                                 double* ms_out);
/* counters of the rays of `rank`'s tiles only (synchronous) */
rt_status rt_render_tiles_counters(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h,
                                   uint32_t spp, uint32_t rank, uint32_t nranks,
                                   uint64_t counters_out[2]);
/* the trace kernel's own fetches for `rank`'s tiles (rt_render_work's counters) */
rt_status rt_render_tiles_work(rt_scene* s, const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp,
                               uint32_t rank, uint32_t nranks, uint64_t counters_out[2]);
/* diagnostics: per-pixel wide-traversal step counts of the previous frame of
 * this shape (w, h, spp, rank, nranks), tile-slot-major (256 per 16x16 tile
 * slot, local pixel ly*16+lx; a ray finished by the binary hand-off is
 * charged 64 extra).  Written by the full-frame primary kernel only (the
 * trace.px_sort path); RT_EINVAL without such a frame. */
rt_status rt_render_step_map(rt_scene* s, uint32_t w, uint32_t h, uint32_t spp, uint32_t rank, uint32_t nranks,
                             uint16_t* out, size_t count);
/* Unpack nranks gathered slabs (each tiles_per_slab*1024 B, slab r = rank r)
 * into a w*h*4 device image. */
rt_status rt_unpack_tiles_device(const void* d_slabs, uint32_t tiles_per_slab, uint32_t w,
                                 uint32_t h, uint32_t nranks, void* d_rgba, int device,
                                 void* stream);
/* Stream of the scene (hipStream_t) for callers that order their own work. */
rt_status rt_scene_stream(rt_scene* s, void** stream_out);
rt_status rt_scene_sync(rt_scene* s);

/* ---- distributed BVH build (SURVEY.md §8(f) row 4 "distributed BVH build
 * (multi-GPU sort by Morton prefix with all-to-all)"; DESIGN.md "Distributed
 * build").  SPMD over nranks ranks, one scene each (the whole soup on every
 * rank); the caller moves the bytes between the phases (gpu_raytracer_amd/
 * dist.py drives them over torch.distributed: RCCL on GPUs, gloo on CPU).
 * Every rank ends with the BVH rt_bvh_build makes, bit for bit:
 *   1. rt_dbuild_bounds: centroid box of the rank's triangle slice
 *      -> all-gather the nranks boxes;
 *   2. rt_dbuild_keys: Morton codes of the slice against the global bounds,
 *      the slice sorted by (key, index) in RT_DB_SEND_*, and its 1024-bucket
 *      histogram of the top 10 key bits -> all-gather the histograms; rank d
 *      owns the bucket range dist.split_buckets gives it; all-to-all the
 *      (key, index) runs into RT_DB_RECV_* (ordered by source rank);
 *   3. rt_dbuild_sort: the received pairs sorted -> the rank's run of the
 *      global order; all-gather the runs into RT_DB_KEYS / RT_DB_VALS;
 *   4. rt_dbuild_subtrees: topology, leaves, local boxes and wide records of
 *      the rank's refit blocks (rt_dbuild_shares) and its crossing-node list
 *      (RT_DB_CROSS) -> all-gather every section's share (nodes, tri_s, wide
 *      records, topology, block prefix/suffix boxes, block totals) and the
 *      crossing lists into RT_DB_CROSS_ALL.  RT_DB_TOPO holds {left, esc,
 *      range lo, range hi} for the crossing nodes only (the merge reads no
 *      other entry; their contents are unspecified);
 *   5. rt_dbuild_merge: boxes and wide records of every crossing node; the
 *      scene is then built (rt_render, rt_bvh_read ...). */
enum {
    RT_DB_SEND_KEYS = 0, RT_DB_SEND_VALS, RT_DB_RECV_KEYS, RT_DB_RECV_VALS, RT_DB_KEYS, RT_DB_VALS,
    RT_DB_NODES, RT_DB_TRI_S, RT_DB_WIDE, RT_DB_TOPO, RT_DB_PRE, RT_DB_SUF, RT_DB_TOTALS, RT_DB_CROSS,
    RT_DB_CROSS_ALL
};
/* shares of rank `rank`: out = {tri_lo, tri_hi, block_lo, block_hi,
 * leaf_lo, leaf_hi} (triangles [tri_lo, tri_hi) for phases 1-2; refit blocks
 * of 512 leaves [block_lo, block_hi) = sorted leaves [leaf_lo, leaf_hi) and
 * internal nodes [leaf_lo, min(leaf_hi, n - 1)) for phase 4). */
rt_status rt_dbuild_shares(uint32_t n, uint32_t rank, uint32_t nranks, uint32_t out[6]);
rt_status rt_dbuild_bounds(rt_scene* s, uint32_t rank, uint32_t nranks, float box_out[6]);
rt_status rt_dbuild_keys(rt_scene* s, uint32_t rank, uint32_t nranks, const float* boxes /* nranks x 6 */,
                         uint32_t hist_out[1024]);
rt_status rt_dbuild_sort(rt_scene* s, uint32_t count);
rt_status rt_dbuild_subtrees(rt_scene* s, uint32_t rank, uint32_t nranks, uint32_t* ncross_out);
rt_status rt_dbuild_merge(rt_scene* s, uint32_t ncross_total);
/* device pointer and size in bytes of an exchange buffer (RT_DB_*) */
rt_status rt_dbuild_buffer(rt_scene* s, int which, void** ptr, uint64_t* bytes);

/* ---- per-stage entry points for parity tests; host
 * buffers in/out, device compute on `device`. ---- */
rt_status rt_stage_bounds(int device, const float* tris, uint32_t n, float bounds9[9]);
rt_status rt_stage_morton(int device, const float* tris, uint32_t n, const float lo[3],
                          const float inv[3], uint32_t* keys, uint32_t* vals);
rt_status rt_stage_sort(int device, uint32_t* keys, uint32_t* vals, uint32_t n); /* in place */
/* Karras topology of sorted keys: topo[4*(n-1)] = {left, esc, range_lo,
 * range_hi} per internal node; parent[2n-1]; leaf_esc[n]. */
rt_status rt_stage_topology(int device, const uint32_t* sorted_keys, uint32_t n, uint32_t* topo,
                            uint32_t* parent, uint32_t* leaf_esc);
/* K5 + K6 (+ K7w) over sorted keys/vals (the build fuses them with K4 in
 * k_topo_refit): nodes_out[2n-1] with every AABB, child and escape link. */
rt_status rt_stage_refit(int device, const uint32_t* sorted_keys, const uint32_t* sorted_vals, const float* tris,
                         uint32_t n, rt_node* nodes_out);
rt_status rt_stage_trace(int device, const rt_node* nodes, uint32_t n, const float* tris,
                         const rt_camera* cam, uint32_t w, uint32_t h, uint32_t spp,
                         rt_hit* hits, uint8_t* rgba, uint64_t counters[2]);
/* Moller-Trumbore on the device: count rays, each o[3], d[3], tri[9],
 * t_best -> hit flag + t/u/v (KAT entry point). */
rt_status rt_stage_intersect(int device, uint32_t count, const float* o, const float* d,
                             const float* tri, const float* t_best, uint32_t* hit, float* tuv);
/* Device fminf/fmaxf semantics probe: out[2*i] = fmin(a[i],b[i]), out[2*i+1] = fmax. */
rt_status rt_stage_minmax(int device, uint32_t count, const float* a, const float* b, float* out);

/* ---- I/O (SURVEY.md §8(b) rt_framebuffer_dump_ppm / rt_hits_dump) ---- */
rt_status rt_framebuffer_dump_ppm(const uint8_t* rgba, uint32_t w, uint32_t h, const char* path);
rt_status rt_hits_dump(const rt_hit* hits, size_t count, const char* path);

/* Tuning knobs (process-wide; 24 keys since r06, which removed the
 * measured-slower alternatives -- DESIGN.md, "Round 6", item 5).  Trace:
 * "trace.variant" 0 = one thread per pixel, wide (4-ary) traversal over the
 * K7w records (default), 2 = one thread per pixel, binary traversal;
 * "trace.stack_cap" (1..18; 0 = all, the default: 14 for 4-ary records on
 * 256-thread blocks, 16 on 64-thread blocks -- one rank's tiles --, 18 for
 * 8-ary) wide-traversal stack entries -- rays that need more are re-traced by
 * the binary traversal; "trace.wg" 64/256 threads per block (8x8 quadrant /
 * 16x16 tile), default 256; "trace.wg_tiles" the same for one rank's tiles
 * of a multi-GPU frame (rt_render_tiles_device), default 64;
 * "trace.tile_order" 1 = dispatch a frame's tiles longest-first from the
 * previous frame of the same shape's per-tile wave times (the first frame of
 * a shape runs row-major), 0 = row-major always; "trace.px_sort" 1 (default)
 * / 2 / 0: each tile's pixels dealt to lanes costliest first from the
 * previous frame, full frames / also one rank's tiles / never;
 * "trace.spp_lanes" 2 (default) / 1 / 0: 2..16 spp (a power of two) traced
 * one ray per lane, a pixel's samples in adjacent lanes, for full frames and
 * one rank's tiles / tiles only / never.  Heavy-ray queue:
 * "trace.coop_cap" / "trace.coop_cap_tiles" 0..2^20: a primary ray still
 * traversing after that many wide steps is queued and finished by a lane
 * group (k_trace_coop, DESIGN.md "Cooperative heavy rays"); 0 = off; -1 =
 * auto, the defaults: for full frames 96 steps at 1 spp on 256-thread tiles
 * (off otherwise) and, for one rank's tiles of a multi-GPU frame, by rank
 * count (88 steps for P = 2, 80 for P = 3..4, 72 above); samples-in-lanes
 * frames run without it unless a cap is given; with an automatic cap a
 * frame shape whose last queue-on frame queued fewer than 64 rays runs
 * without the queue, re-probing every 16th frame; "trace.coop_lanes"
 * 16/32/64 lanes per queued ray (default 32); "trace.coop_max" queue
 * entries per frame shape (default 65536; rays beyond it keep tracing
 * alone).  Build: "build.wide_arity" 4 (default) / 8: K7w 4-ary or K7w8
 * 8-ary trace records (8-ary: about a quarter fewer dependent record
 * fetches for the costliest rays, more instructions per step; n <= 2^26);
 * "build.stage_events" 0/1: per-stage build events (rt_bvh_build_times);
 * "build.sort" (n in 2..12M): 2 = the tile-bucketed gather sort (default:
 * K1 sorts each 4096-key tile by the top 10 key bits, then one block per
 * bucket gathers its runs and sorts them in LDS), 1 = the r01-r03 MSB
 * scatter + bucket sort, 0 = the 4-pass LSB radix sort; a scene whose first
 * build finds a bucket beyond one block's LDS sort keeps the LSB sort, and
 * one whose gather probe finds a run of more than 64 identical keys
 * (duplicated triangles) moves on to the MSB sort; clustered bins stay on
 * the gather sort, whose blocks sort such buckets by LDS radix passes.  "build.fuse_k01" 1 (default) / 0: with the gather sort,
 * K0 (bounds) and K1 (Morton) as one launch whose blocks meet at a grid
 * barrier, when every sort tile's block fits the device at once (n up to
 * ~1M) and no other such build runs on the device; else two launches.  2
 * (test only): fused even when the grid cannot be co-resident -- the
 * barrier's bounded waits give up and the build is redone with two launches
 * (rt_build_times.fused_fallback) instead of hanging.  Path mode:
 * "path.wavefront" 0 = megakernel ("path.wg" 64/256 threads per block), 1 =
 * wavefront schedule with per-depth ray queues (default); "path.sort" 0..4
 * = top key bytes each queue is radix-sorted by for coherence (ray kind,
 * direction octant, Morton code of the origin; 0 = unsorted, the default;
 * sorting reads each queue length back to the host); "path.batch" paths per
 * wavefront batch (0 = 4M).  Multi-GPU: "render.emulate" 0/1: rt_render(ngpus
 * > 1) puts every rank's replica on the scene's device and gathers with
 * device copies instead of RCCL (multi-rank tests on one GPU);
 * "render.rccl1" 0/1: rt_render(ngpus = 1) through the tiled + RCCL path (a
 * 1-rank communicator).  Debug: "debug.force_lsb_redo" 0/1 (tests): take
 * the gather-overflow branch, i.e. redo the build with the LSB sort;
 * "debug.poison" 0/1: every device buffer the library allocates from then on
 * is filled with 0xFF bytes before first use, so reading a byte no kernel
 * wrote gives the same (wrong) value every run instead of allocator luck;
 * "debug.lds_scribble" 0/1: before every kernel launch a scribble kernel
 * fills the CUs' LDS with a pattern that changes every launch, so a kernel
 * reading LDS it did not write differs run to run.  Both debug knobs can
 * start on from the environment: RT_DEBUG_POISON=1, RT_DEBUG_LDS_SCRIBBLE=1.
 * Results are bit-identical for every setting. */
rt_status rt_config_set(const char* key, int64_t value);

const char* rt_last_error(void);
int rt_device_count(void);
const char* rt_version(void);

#ifdef __cplusplus
}
#endif
#endif

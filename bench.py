#!/usr/bin/env python3
"""Headline benchmark: Mrays/s @1920x1080x1spp + BVH-build Mprims/s on the
1M-triangle synthetic soup (BASELINE.json configs[2]), 1..N GPUs.

One STEP = one frame of the hot path on inputs already resident in HBM:
  rt_bvh_build (K0..K6, replicated on every rank) -> trace this rank's image
  tiles (K8/K9; full image on one GPU) -> [N>1] RCCL gather of the packed
  tiles to rank 0 (torch.distributed 'nccl' == RCCL) + unpack kernel.
W untimed warm-up steps, then K timed steps between barrier+synchronize on
both sides; the max over ranks is reported by rank 0 as ONE JSON line.

  value      = W*H*spp / (mean over steps of max-rank trace time + gather time)
               [Mrays/s, whole image, all ranks; SURVEY.md §8(e)].  At N>1 the
               trace, the RCCL gather and the unpack are queued back to back
               on torch's stream and timed together with events on it
               (gather time = that span minus the trace)
  build_mprims_per_s = N_tris / mean build time (per GPU; replicated)
  ms_per_step = wall time per frame incl. build, trace, gather and host syncs
Device times come from hipEvents recorded on the stream each kernel runs on
(the scene's stream inside librtamd).

roofline: the dominant kernel (trace) -- algorithmic bytes per launch =
  32 B x nodes fetched + 36 B x tris tested + 16 B x rays (SURVEY.md §8(d):
  the §9.7 binary traversal's deterministic counters, which the oracle
  reproduces), over its mean event-timed duration, against 8.0 TB/s HBM.
  The default kernel traverses the K7w wide (4-ary) records instead; the
  bytes IT requests (64 B x records + 48 B x triangle records + 20 B x rays,
  its own deterministic counters) are reported beside as kernel_bytes.
cpu_baseline (rank 0, N=1 only): the CPU oracle (oracle/, a port of the same
  contract -- the reference has no runnable code) builds the same 1M soup
  single-threaded and traces the same full frame on up to 16 host threads.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # /opt/skills/guides/MI355X_MICROARCH.md: 8.0 TB/s spec
BUILD_BYTES_PER_PRIM = 404  # SURVEY.md §8(d) canonical build byte model
METRIC = "Mrays/s @1920×1080×1spp + BVH build Mprims/s, 1M-tri scene, 1/2/4/8 GPUs"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3, help="scenes.CONFIGS key (3 = soup-1M headline)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_trace.json"))
    ap.add_argument("--dump", default="", help="write the rank-0 image as PPM")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI) for the benchmark; gloo only to rehearse N>1 on one GPU")
    return ap.parse_args()


def cpu_baseline(tris, view, w, h, spp, threads, gpu_counters):
    """Oracle build (1 thread) + full-frame trace (threads); returns dict."""
    from oracle import oracle as O  # cpu_baseline leg only
    if not os.path.exists(O._LIB_PATH):
        O.build_oracle()
    t0 = time.perf_counter()
    b = O.build(tris)
    t_build = time.perf_counter() - t0
    cam = O.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
    t0 = time.perf_counter()
    _, cnt = O.trace(b["nodes"], tris, cam, w, h, spp, nthreads=threads)
    t_trace = time.perf_counter() - t0
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    rays = w * h * spp
    return {
        "value": rays / t_trace / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
        "sample": f"full frame {w}x{h}x{spp} traced on {threads} threads ({t_trace:.2f} s); "
                  f"full {len(tris)}-tri BVH built on 1 thread ({t_build:.2f} s)",
        "build_mprims_per_s": len(tris) / t_build / 1e6, "build_threads": 1,
        "cpu_model": model,
        "counters_match_gpu": bool(int(cnt[0]) == int(gpu_counters[0]) and int(cnt[1]) == int(gpu_counters[1])),
    }


def secondary_rays(R, S, scene, cfg, cam, w, h, spp, img, hits, args, torch, dev, primary_ms):
    """SURVEY.md §8(f) row 3, shadow mode: the same frame with one
    any-hit shadow ray per primary hit.  Untimed by the step contract; its own
    warm-up and timed launches (hipEvents), median reported."""
    light = S.LIGHTS[cfg.scene]
    ms = []
    for i in range(args.warmup + max(args.steps, 3)):
        t = scene.render_shadow_device(cam, w, h, spp, light, S.AMBIENT, d_rgba=img.data_ptr(),
                                       d_hits=hits.data_ptr(), timed=True)
        if i >= args.warmup:
            ms.append(t)
    torch.cuda.synchronize(dev)
    prim = hits.view(-1, 4)[:, 3].view(torch.int32)
    shadow_rays = int((prim != -1).sum().item())
    rays = w * h * spp
    med = float(np.median(ms))
    return {"mode": "shadow rays: 1 any-hit ray per primary hit toward a point light (DESIGN.md)",
            "light": list(light), "ambient": S.AMBIENT, "ms": round(med, 4),
            "primary_rays": rays, "shadow_rays": shadow_rays,
            "mrays_per_s": round((rays + shadow_rays) / (med * 1e-3) / 1e6, 2),
            "shadow_mrays_per_s": round(shadow_rays / (max(med - primary_ms, 1e-6) * 1e-3) / 1e6, 2)}


PATH_DEPTH = 2   # bounces after the primary segment
PATH_SKY = 0.3


def path_tracing(R, S, scene, cfg, cam, w, h, spp, img, args, torch, dev):
    """SURVEY.md §8(f) row 3, path mode: diffuse paths of up to
    1 + PATH_DEPTH segments with a shadow ray at every hit, same frame.
    Untimed by the step contract; its own warm-up and timed launches
    (hipEvents), median reported; the ray count comes from the kernel's own
    counters (deterministic: the same paths every launch)."""
    light = S.LIGHTS[cfg.scene]
    ms = []
    for i in range(args.warmup + max(args.steps, 3)):
        t = scene.render_path_device(cam, w, h, spp, light, PATH_SKY, PATH_DEPTH, d_rgba=img.data_ptr(), timed=True)
        if i >= args.warmup:
            ms.append(t)
    torch.cuda.synchronize(dev)
    work = scene.render_path_work(cam, w, h, spp, light, PATH_SKY, PATH_DEPTH)
    med = float(np.median(ms))
    return {"mode": f"diffuse path tracing, max_depth {PATH_DEPTH}, next-event shadow rays (DESIGN.md); "
                    "wavefront schedule, unsorted ray queues (the default)",
            "light": list(light), "sky": PATH_SKY, "ms": round(med, 4), "rays": int(work[2]),
            "rays_per_pixel": round(int(work[2]) / (w * h * spp), 3),
            "mrays_per_s": round(int(work[2]) / (med * 1e-3) / 1e6, 2),
            "node_records": int(work[0]), "tri_records": int(work[1])}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if args.gpus > 1 and world == 1:
            raise SystemExit("for --gpus N>1 launch with torch.distributed.run --nproc-per-node N")
        world = max(world, 1)

    import torch
    import torch.distributed as dist
    import gpu_raytracer_amd as R
    from gpu_raytracer_amd import dist as D
    from gpu_raytracer_amd import scenes as S

    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)  # rehearsal: several ranks may share one GPU (gloo only)
    torch.cuda.set_device(local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    cfg = S.CONFIGS[args.config]
    view = S.VIEWS[cfg.scene]
    w, h, spp = cfg.w, cfg.h, cfg.spp
    rays = w * h * spp
    if cfg.scene == "soup":
        scene = R.Scene.generate_soup(cfg.n, 1)
    else:
        scene = R.Scene.from_soup(S.tris_for(cfg.scene))
    n_tris = scene.num_tris
    scene.set_device(local)
    cam = R.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)

    tmax = D.slab_tiles(w, h, world)
    dev = torch.device("cuda", local)
    img = torch.zeros(w * h, dtype=torch.int32, device=dev)
    hits = torch.empty(rays * 4, dtype=torch.float32, device=dev)
    slab = torch.zeros(max(tmax, 1) * 256, dtype=torch.int32, device=dev) if world > 1 else None
    # every rank writes its hit records too (16 B/ray, part of the byte model); only RGBA is gathered
    slab_hits = torch.empty(max(tmax, 1) * 256 * spp * 4, dtype=torch.float32, device=dev) if world > 1 else None
    slabs_all = torch.zeros(world * max(tmax, 1) * 256, dtype=torch.int32, device=dev) if (world > 1 and rank == 0) else None
    gather_list = None  # gather_slabs receives straight into slabs_all's per-rank rows

    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

    def step():
        build_ms = scene.build()
        if world == 1:
            trace_ms = scene.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), d_hits=hits.data_ptr(), timed=True)
            return build_ms, trace_ms, 0.0
        cur = torch.cuda.current_stream(dev)
        if args.dist_backend == "nccl":
            # trace -> RCCL gather -> unpack queued back to back on torch's
            # stream (the collective waits on it; no host round trip between
            # them), timed with events on that stream
            ev[0].record(cur)
            scene.render_tiles_device(cam, w, h, spp, rank, world, slab.data_ptr(), slab_hits.data_ptr(),
                                      stream=cur.cuda_stream)
            ev[1].record(cur)
            D.gather_slabs(slab, rank, world, gather_list, slabs_all)
            if rank == 0:
                R.unpack_tiles_device(slabs_all.data_ptr(), max(tmax, 1), w, h, world, img.data_ptr(), local,
                                      cur.cuda_stream)
            ev[2].record(cur)
            ev[2].synchronize()
            trace_ms = ev[0].elapsed_time(ev[1])
            return build_ms, trace_ms, ev[0].elapsed_time(ev[2]) - trace_ms
        # gloo rehearsal: stage through host memory, host-timed
        trace_ms = scene.render_tiles_device(cam, w, h, spp, rank, world, slab.data_ptr(), slab_hits.data_ptr(),
                                             timed=True)
        t0 = time.perf_counter()
        g = D.gather_slabs(slab.cpu(), rank, world)
        if rank == 0:
            slabs_all.copy_(g)
            R.unpack_tiles_device(slabs_all.data_ptr(), max(tmax, 1), w, h, world, img.data_ptr(), local,
                                  cur.cuda_stream)
        torch.cuda.synchronize(dev)
        return build_ms, trace_ms, (time.perf_counter() - t0) * 1e3

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    rec = [step() for _ in range(args.steps)]
    barrier()
    wall = time.perf_counter() - t0
    per = np.array(rec, dtype=np.float64)  # [steps, 3] build, trace, gather (ms)
    # the same frame with row-major tile dispatch (untimed by the step contract):
    # the timed steps dispatch tiles longest-first from the previous frame's
    # per-tile wave times (trace.tile_order 1, DESIGN.md "Tile order")
    R.config_set("trace.tile_order", 0)
    rm = []
    for _ in range(6):
        if world == 1:
            rm.append(scene.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), d_hits=hits.data_ptr(), timed=True))
        else:
            rm.append(scene.render_tiles_device(cam, w, h, spp, rank, world, slab.data_ptr(), slab_hits.data_ptr(),
                                                timed=True))
    R.config_set("trace.tile_order", 1)
    trace_ms_row_major = float(np.median(rm[1:]))
    # per-stage breakdown from one extra, untimed build with the stage events
    # on (each adds a little to the GPU timeline, so the timed steps run without)
    R.config_set("build.stage_events", 1)
    stage_total_ms = scene.build()
    stimes = scene.build_times()
    R.config_set("build.stage_events", 0)

    # max over ranks (per step), then mean over steps
    if world > 1:
        rdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
        t = torch.tensor(per, dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        per = t.cpu().numpy()
        wt = torch.tensor([wall], dtype=torch.float64, device=rdev)
        dist.all_reduce(wt, op=dist.ReduceOp.MAX)
        wall = float(wt.item())
    build_ms, trace_ms, gather_ms = (float(x) for x in per.mean(axis=0))
    trace_ms_min = float(per[:, 1].min())

    # "rank 0 builds and then broadcasts" measured next to the
    # replicated build (untimed by the step contract; 1 warm-up + 3 timed)
    bvh_exchange = None
    if world > 1 and args.dist_backend == "nccl":
        try:
            bms = []
            for i in range(4):
                barrier()
                tb0 = time.perf_counter()
                nbytes = D.broadcast_bvh(scene, dev)
                torch.cuda.synchronize(dev)
                barrier()
                if i:
                    bms.append((time.perf_counter() - tb0) * 1e3)
            bt = torch.tensor([float(np.median(bms))], dtype=torch.float64, device=dev)
            dist.all_reduce(bt, op=dist.ReduceOp.MAX)
            bvh_exchange = {"replicated_build_ms": round(build_ms, 4), "broadcast_ms": round(float(bt.item()), 4),
                            "broadcast_bytes": int(nbytes),
                            "used": "replicated build (every rank builds; no BVH traffic)"}
        except Exception as exc:  # a measurement only: never fail the bench line over it
            bvh_exchange = {"error": f"{type(exc).__name__}: {exc}"[:200]}

    # work counters of this rank's trace launch (deterministic; untimed)
    cnt = scene.render_tiles_counters(cam, w, h, spp, rank, world) if world > 1 else scene.render_counters(cam, w, h, spp)
    rank_rays = D.rays_of_rank(w, h, spp, rank, world)
    algo_bytes = 32.0 * float(cnt[0]) + 36.0 * float(cnt[1]) + 16.0 * rank_rays
    rank_trace_ms = float(np.array(rec)[:, 1].mean())
    achieved = algo_bytes / (rank_trace_ms * 1e-3) / 1e9
    kernel_bytes = None
    if world == 1:
        wk = scene.render_work(cam, w, h, spp)
        kernel_bytes = 64.0 * float(wk[0]) + 48.0 * float(wk[1]) + 20.0 * rank_rays
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("config") == cfg.name and tj.get("n_gpus", 1) == world:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    out = None
    if rank == 0:
        value = rays / ((trace_ms + gather_ms) * 1e-3) / 1e6
        build_gbs = BUILD_BYTES_PER_PRIM * n_tris / (build_ms * 1e-3) / 1e9
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: random-triangle soup, splitmix64 seed 1, r=1/cbrt(N) (SURVEY.md §9.9)"
                    if cfg.scene == "soup" else f"synthetic: procedural {cfg.name} (SURVEY.md §9.9)",
            "config": {"workload": f"{cfg.name} {w}x{h}x{spp} (BASELINE.json configs[{args.config - 1}])",
                       "n_tris": n_tris, "width": w, "height": h, "spp": spp,
                       "parallelism": f"image tiles 16x16 round-robin over {world} GPU(s), BVH replicated"
                                      + ((", RCCL gather to rank 0" if args.dist_backend == "nccl" else ", gloo gather (rehearsal)") if world > 1 else "")},
            "build_mprims_per_s": round(n_tris / (build_ms * 1e-3) / 1e6, 2),
            "build_ms": round(build_ms, 4),
            "trace_ms": round(trace_ms, 4),
            "trace_ms_min": round(trace_ms_min, 4),
            "tile_order": "longest-first from the previous frame's per-tile wave times (32 KB cost map per frame "
                          "shape; the first frame runs row-major)",
            "trace_ms_row_major_rank0": round(trace_ms_row_major, 4),
            "gather_ms": round(gather_ms, 4),
            "bvh_exchange": bvh_exchange,
            "frame_mrays_per_s": round(rays / (wall / args.steps) / 1e6, 2),
            "build_stages_ms_last": {"bounds": round(stimes.bounds, 4), "morton": round(stimes.morton, 4),
                                     "sort": round(stimes.sort, 4), "topology": round(stimes.topology, 4),
                                     "refit": round(stimes.refit, 4), "wide": round(stimes.wide, 4),
                                     "total_with_stage_events": round(stage_total_ms, 4)},
            "trace_counters_rank0": {"nodes_fetched": int(cnt[0]), "tris_tested": int(cnt[1]), "rays": rank_rays},
            "roofline": {"bound": "hbm", "kernel": "k_trace<wide>", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "algo_bytes_per_launch": algo_bytes,
                         "kernel_bytes_per_launch": kernel_bytes,
                         "kernel_frac": (round(kernel_bytes / (rank_trace_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                         if kernel_bytes else None),
                         "note": "algorithmic bytes (SURVEY.md §8(d): 32/node + 36/tri + 16/ray over the §9.7 "
                                 "binary traversal's counters); kernel_bytes = what the wide kernel requests "
                                 "(64/record + 48/tri record + 20/ray). frac can exceed 1: the §8(d) model "
                                 "charges every binary node visit 32 B as if from HBM, while the kernel fetches "
                                 "~4x fewer (wide) records from the Infinity-Cache-resident structures; 'traffic' "
                                 "is the PMC-measured HBM bytes per launch. The kernel is bound by dependent-fetch "
                                 "latency and VALU issue (DESIGN.md), not HBM bandwidth"},
            "roofline_build": {"bound": "hbm", "achieved": round(build_gbs, 1), "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": round(build_gbs / HBM_PEAK_GBS, 4),
                               "bytes_per_prim": BUILD_BYTES_PER_PRIM},
            "cpu_baseline": None,
        }
        host_img = img.cpu().numpy().view(np.uint8)   # the primary frame, before the secondary modes reuse img
        if world == 1:
            out["secondary"] = secondary_rays(R, S, scene, cfg, cam, w, h, spp, img, hits, args, torch, dev,
                                              float(np.median(per[:, 1])))
            out["path"] = path_tracing(R, S, scene, cfg, cam, w, h, spp, img, args, torch, dev)
        if world == 1 and not args.no_cpu_baseline:
            threads = max(1, min(args.cpu_threads, len(os.sched_getaffinity(0))))
            out["cpu_baseline"] = cpu_baseline(scene.tris(), view, w, h, spp, threads, cnt)
        import zlib
        out["image_crc32"] = zlib.crc32(host_img.tobytes()) & 0xFFFFFFFF  # same for every N (bit-exact tiles)
        if args.dump:
            R.dump_ppm(host_img, w, h, args.dump)
        print(json.dumps(out), flush=True)
    scene.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Headline benchmark: Mrays/s @1920x1080x1spp + BVH-build Mprims/s on the
1M-triangle synthetic soup (BASELINE.json configs[2]), 1..N GPUs.

One STEP = one frame of the hot path on inputs already resident in HBM, with
the camera orbiting the scene 0.25 degrees per step (so no frame repeats the
previous one):
  rt_bvh_build (K0..K7w, replicated on every rank) -> trace this rank's image
  tiles (K8/K9; full image on one GPU) -> [N>1] RCCL gather of the packed
  tiles to rank 0 (torch.distributed 'nccl' == RCCL) + unpack kernel.
W untimed warm-up steps, then K timed steps between barrier+synchronize on
both sides; the max over ranks is reported by rank 0 as ONE JSON line.

  value      = W*H*spp / (mean over steps of the max-rank frame span)
               [Mrays/s, whole image, all ranks; SURVEY.md §8(e)].  At N>1 the
               trace, the RCCL gather and the unpack are queued back to back
               on torch's stream and timed together with events on it: the
               frame span is trace start -> the gathered image unpacked (rank
               0) or the slab sent (others); gather_ms = span - trace.  (Until
               r02 value used max trace + max gather, which counted a slow
               rank's lead twice: in its trace and in rank 0's wait.)
  value_cold = the same frame with row-major tile dispatch (a first frame: no
               previous frame's cost map); static_camera = the same camera
               every frame (the map replays an identical frame: best case)
  build_mprims_per_s = N_tris / mean build time (per GPU; replicated)
  ms_per_step = wall time per frame incl. build, trace, gather and host syncs
Device times come from hipEvents recorded on the stream each kernel runs on
(the scene's stream inside librtamd, or torch's stream at N>1).

Launch: `python bench.py --gpus N` spawns N rank processes itself (one per
GPU, before any of them touches the GPU); under torch.distributed.run the
ranks come from the environment.

roofline: the trace launch (k_trace, then k_trace_coop for the rays past the heavy-ray cap, whose block 0
  sorts the next frame's tile order), priced against the resource that
  measurably bounds it (`bound`, roofline_of): HBM (PMC bytes), L2 (the bytes
  the kernels request: 64 B per K7w record + 48 B per triangle record fetched,
  their own deterministic counters, + 16 B hit + 4 B RGBA per ray -- served
  by L2/MALL, so never priced against HBM) or VALU issue (SQ_INSTS_VALU over
  the issue capacity), the PMC figures from the committed profile of the same
  command (profiles/pmc_summary.json, tools/gpu_run.sh profile).  Every frac
  is <= 1.  other_configs.config5 (soup-10M, the config whose trace structures exceed
  the MALL) carries the same block from its own profile entry.  The SURVEY.md §8(d) binary-traversal byte model
  is kept as algo_bytes_binary_model (it charges node visits the wide kernel
  does not make, so its fraction is not a roofline of this kernel).
cpu_baseline (rank 0, N=1 only): the CPU oracle (oracle/, a port of the same
  contract -- the reference has no runnable code), built on this host with
  -O3 -march=native, builds the same 1M soup single-threaded and traces the
  same full frame on every CPU this process may use.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # /opt/skills/guides/MI355X_MICROARCH.md: 8.0 TB/s spec
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md §L2: ~34.5 TB/s aggregate over the 8 XCD L2s
BUILD_BYTES_PER_PRIM = 404  # SURVEY.md §8(d) canonical build byte model
METRIC = "Mrays/s @1920×1080×1spp + BVH build Mprims/s, 1M-tri scene, 1/2/4/8 GPUs"
ORBIT_DEG = 0.25  # camera motion per step
# VALU issue peak: 256 CUs x 4 SIMDs, a wave64 VALU op issues over 2 cycles
# (MI355X_MICROARCH.md "v_fma_f32 (wave64) 2 cyc (SIMD-32)")
VALU_ISSUE_PER_CYCLE = 1024 * 0.5


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3, help="scenes.CONFIGS key (3 = soup-1M headline)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the other configs / secondary modes")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this process may use")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_summary.json"))
    ap.add_argument("--dump", default="", help="write the rank-0 image as PPM")
    ap.add_argument("--only-timed", action="store_true",
                    help="warm-up + timed steps only (the PMC passes of tools/gpu_run.sh profile)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI) for the benchmark; gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--extras", action="store_true",
                    help="N>1: also time the BVH broadcast and the distributed build after the headline "
                         "(off by default: the headline line must not depend on them)")
    ap.add_argument("--pg-timeout", type=float, default=120.0,
                    help="seconds before a stuck collective fails the process group")
    ap.add_argument("--deadline", type=float, default=900.0,
                    help="`--gpus N` without a launcher: seconds before the parent kills its rank processes")
    ap.add_argument("--inject-hang", type=int, default=-1,
                    help="testing only: this rank sleeps forever in the --extras leg")
    return ap.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def supervise(procs, deadline_s, grace_s=10.0, poll_s=0.2) -> int:
    """Wait for the rank processes; never forever.  A rank that exits non-zero
    (or by a signal) fails the run: the others get `grace_s` to finish, then
    are killed (they would otherwise sit in a collective with a dead peer).
    Past `deadline_s` every rank still running is killed and the result is
    124.  The parent never touched a GPU, so killing its children is safe.
    Returns 0 only when every rank exited 0."""
    t0 = time.monotonic()
    fail_at, rc = None, 0
    while True:
        alive = [p for p in procs if p.poll() is None]
        for p in procs:
            if p.returncode not in (None, 0):
                rc = max(rc, abs(p.returncode))
                fail_at = fail_at if fail_at is not None else time.monotonic()
        if not alive:
            return rc
        now = time.monotonic()
        late = now - t0 > deadline_s
        if late or (fail_at is not None and now - fail_at > grace_s):
            for p in alive:
                p.kill()
            for p in alive:
                p.wait()
            print(f"bench: {'deadline of %.0f s passed' % deadline_s if late else 'a rank failed'}; killed "
                  f"{len(alive)} rank process(es)", file=sys.stderr)
            return 124 if late else max(rc, 1)
        time.sleep(poll_s)


def spawn_ranks(args) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes (one per
    GPU) with the torch.distributed env, before anything here touches a GPU;
    rank 0 prints the JSON line.  Returns the worst exit status (124 when the
    --deadline passed and the ranks were killed)."""
    port = str(_free_port())
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    return supervise(procs, args.deadline)


def orbit_view(view, step):
    """The view's eye rotated about the vertical axis through `at` by
    ORBIT_DEG per step (host double math, like rt_camera_look_at)."""
    a = math.radians(ORBIT_DEG * step)
    ex, ey, ez = (e - c for e, c in zip(view.eye, view.at))
    rx, rz = ex * math.cos(a) + ez * math.sin(a), -ex * math.sin(a) + ez * math.cos(a)
    return (view.at[0] + rx, view.at[1] + ey, view.at[2] + rz)


def cpu_quota():
    """CPUs this process's cgroup may run on at once (cpu.max quota/period),
    or None when unlimited / unknown."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except Exception:
        return None


def cpu_baseline(tris, view, w, h, spp, threads, gpu_counters, min_seconds=10.0):
    """Oracle (-march=native build): the same 1M-soup BVH built on 1 thread,
    then full frames of the bench's orbiting camera traced on `threads`
    threads until at least `min_seconds` of wall time (a bounded sample of the
    same workload); returns dict.  The first frame's counters are checked
    against the GPU's (static camera)."""
    from oracle import oracle as O  # cpu_baseline leg only
    O.use_native_build()
    t0 = time.perf_counter()
    b = O.build(tris)
    t_build = time.perf_counter() - t0
    cam = O.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
    _, cnt = O.trace(b["nodes"], tris, cam, w, h, spp, nthreads=threads)
    frames, t_trace, i = 0, 0.0, 0
    while t_trace < min_seconds:
        c = O.camera_look_at(orbit_view(view, i), view.at, view.up, view.vfov, w, h)
        t0 = time.perf_counter()
        O.trace(b["nodes"], tris, c, w, h, spp, nthreads=threads)
        t_trace += time.perf_counter() - t0
        frames += 1
        i += 1
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    rays = w * h * spp * frames
    return {
        "value": rays / t_trace / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
        "threads_used": threads, "cores_available": len(os.sched_getaffinity(0)),
        "cpus_in_machine": os.cpu_count(), "cgroup_cpu_quota": cpu_quota(),
        "sample": f"{frames} full frames {w}x{h}x{spp} of the bench's orbiting camera traced on {threads} threads "
                  f"({t_trace:.1f} s); full {len(tris)}-tri BVH built on 1 thread ({t_build:.2f} s); oracle built "
                  f"-O3 -march=native -ffp-contract=off on this host",
        "build_mprims_per_s": len(tris) / t_build / 1e6, "build_threads": 1,
        "cpu_model": model,
        "counters_match_gpu": bool(int(cnt[0]) == int(gpu_counters[0]) and int(cnt[1]) == int(gpu_counters[1])),
    }


def config0_leg(R, S, torch, dev, threads, min_seconds=1.0):
    """BASELINE.json configs[0] (Cornell box, 32 triangles, 256x256x1): the
    scalar CPU path it names -- the oracle's build + trace + shade of one
    frame -- timed on 1 thread and on `threads` threads (repeated until
    `min_seconds` each), with the same frame on the GPU beside it.  Both
    images must equal the committed fixture tests/golden/cornell.npz
    (`r256x256x1_rgba`); a mismatch fails the bench."""
    from oracle import oracle as O  # cpu_baseline leg only
    g = np.load(os.path.join(ROOT, "tests", "golden", "cornell.npz"))
    cfg = S.CONFIGS[1]
    view = S.VIEWS[cfg.scene]
    w, h, spp = cfg.w, cfg.h, cfg.spp
    tris = S.tris_for(cfg.scene)
    assert np.array_equal(tris, g["tris"]), "Cornell generator differs from the fixture"
    cam = O.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
    assert np.array_equal(cam.as_array(), g["r256x256x1_cam"]), "Cornell camera differs from the fixture"

    def cpu_frame(nt):
        b = O.build(tris)
        hits, _ = O.trace(b["nodes"], tris, cam, w, h, spp, nthreads=nt)
        return O.shade(hits, w, h, spp)

    out = {"workload": f"{cfg.name} {cfg.n} tris {w}x{h}x{spp} (BASELINE.json configs[0])",
           "path": "oracle build (1 thread) + trace + shade of one full frame, -O3 -march=native",
           "rays": w * h * spp}
    for label, nt in (("cpu_1thread", 1), ("cpu_nthreads", threads)):
        rgba = cpu_frame(nt)
        assert np.array_equal(rgba, g["r256x256x1_rgba"]), f"configs[0] CPU image ({nt} threads) != fixture"
        reps, t = 0, 0.0
        while t < min_seconds:
            t0 = time.perf_counter()
            cpu_frame(nt)
            t += time.perf_counter() - t0
            reps += 1
        ms = t / reps * 1e3
        out[label] = {"threads": nt, "ms": round(ms, 4), "frames": reps,
                      "mrays_per_s": round(w * h * spp / (ms * 1e-3) / 1e6, 2)}
    # the GPU beside it: build + frame through the C-ABI (event-timed, median)
    with R.Scene.from_soup(tris) as s:
        s.set_device(dev.index or 0)
        rcam = R.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
        img = torch.zeros(w * h, dtype=torch.int32, device=dev)
        hits = torch.empty(w * h * spp * 4, dtype=torch.float32, device=dev)
        bms, tms = [], []
        for i in range(23):
            b = s.build()
            t = s.render_device(rcam, w, h, spp, d_rgba=img.data_ptr(), d_hits=hits.data_ptr(), timed=True)
            if i >= 3:
                bms.append(b)
                tms.append(t)
        torch.cuda.synchronize(dev)
        assert np.array_equal(img.cpu().numpy().view(np.uint8), g["r256x256x1_rgba"]), "configs[0] GPU image != fixture"
        del img, hits
    bm, tm = float(np.median(bms)), float(np.median(tms))
    out["gpu"] = {"build_ms": round(bm, 4), "trace_ms": round(tm, 4), "frame_ms": round(bm + tm, 4),
                  "mrays_per_s": round(w * h * spp / (tm * 1e-3) / 1e6, 2),
                  "note": "event-timed medians of 20 build + frame steps (static camera); the GPU image equals "
                          "the fixture too. A 65K-ray, 32-triangle frame is launch/latency-bound on the GPU"}
    out["image_equals_fixture"] = True
    return out


def load_pmc(path, cfg_name, world):
    """PMC summary of the trace kernel (tools/pmc_summary.py output) for this
    config and GPU count, or None."""
    try:
        pj = json.load(open(path))
    except Exception:
        return None
    for e in pj.get("entries", []):
        if e.get("config") == cfg_name and e.get("n_gpus", 1) == world:
            return e
    return None


def secondary_rays(S, scene, cfg, cam, w, h, spp, img, hits, args, torch, dev, primary_ms):
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


def path_tracing(S, scene, cfg, cam, w, h, spp, img, args, torch, dev):
    """SURVEY.md §8(f) row 3, path mode: diffuse paths of up to
    1 + PATH_DEPTH segments with a shadow ray at every hit, same frame."""
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


def make_scene(R, S, cfg):
    if cfg.scene == "soup":
        return R.Scene.generate_soup(cfg.n, 1)
    return R.Scene.from_soup(S.tris_for(cfg.scene))


VALU_CLOCK_GHZ = 2.4  # MI355X_MICROARCH.md: nominal shader clock


def roofline_of(kernel_bytes, trace_ms, pmc):
    """The trace kernel's roofline block, priced against the resource that
    MEASURABLY bounds it:
      hbm_frac   = PMC HBM bytes per launch (2*FETCH_SIZE + WRITE_SIZE) over
                   the event-timed launch, against the 8 TB/s HBM peak;
      l2_frac    = the bytes the kernel requests (its own record/triangle
                   counters + outputs) against the aggregate L2 bandwidth --
                   every request passes L2, and most are served there or from
                   the MALL, so they are never priced against HBM;
      issue_frac = SQ_INSTS_VALU / (1024 SIMDs x 0.5 x GRBM_GUI_ACTIVE/8), the
                   VALU issue share, from the committed profile of the same
                   command.
    `bound` is the largest of these; achieved/peak/unit/frac are that
    resource's.  Without a PMC entry only l2_frac is known and bound = l2."""
    t = trace_ms * 1e-3
    req_gbs = kernel_bytes / t / 1e9
    hbm_frac = issue_frac = traffic = None
    if pmc:
        traffic = pmc.get("hbm_bytes_per_launch")
        if traffic:
            hbm_frac = traffic / t / 1e9 / HBM_PEAK_GBS
        if pmc.get("valu_insts_per_launch") and pmc.get("cycles_per_launch"):
            issue_frac = pmc["valu_insts_per_launch"] / (VALU_ISSUE_PER_CYCLE * pmc["cycles_per_launch"])
    l2_frac = req_gbs / L2_PEAK_GBS
    fr = {"hbm": hbm_frac, "l2": l2_frac, "valu_issue": issue_frac}
    bound = max((k for k in fr if fr[k] is not None), key=lambda k: fr[k])
    if bound == "hbm":
        achieved, peak, unit = traffic / t / 1e9, HBM_PEAK_GBS, "GB/s"
    elif bound == "l2":
        achieved, peak, unit = req_gbs, L2_PEAK_GBS, "GB/s"
    else:
        peak = VALU_ISSUE_PER_CYCLE * VALU_CLOCK_GHZ
        achieved, unit = issue_frac * peak, "G VALU wave-instructions/s"
    return {"bound": bound, "achieved": round(achieved, 1), "peak": peak, "unit": unit,
            "frac": round(fr[bound], 4), "traffic": traffic,
            "hbm_frac": round(hbm_frac, 4) if hbm_frac is not None else None,
            "l2_frac": round(l2_frac, 4), "l2_peak": L2_PEAK_GBS,
            "issue_frac": round(issue_frac, 4) if issue_frac is not None else None,
            "requested_bytes_per_launch": kernel_bytes, "requested_gbs": round(req_gbs, 1),
            "pmc_trace_kernel_us": pmc.get("trace_kernel_avg_us") if pmc else None}


EMU_RANKS = (2, 4, 8)


def rank_emulation(R, S, scene, key, torch, dev, frames=6, drop=2, ranks=EMU_RANKS, full_ms=None):
    """EMULATED multi-GPU scaling on ONE GPU (SURVEY.md
    §8(e)): the GPU plays each rank r < P in turn and traces only that rank's
    image tiles (t = r mod P, rt_render_tiles_device -- the exact launch a
    rank of `bench.py --gpus P` makes), `frames` successive frames of the
    bench's orbiting camera per rank (the tile / pixel order maps are per
    frame shape, so each rank warms its own; the first `drop` frames are
    dropped), median per rank.  No RCCL gather and no concurrency between
    ranks: this projects the trace's strong scaling only.  Reported: every
    rank's median, max and mean over ranks, and speedup / efficiency of the
    max-rank time against the full frame on the same cameras (`full_ms`,
    measured here the same way unless given)."""
    cfg = S.CONFIGS[key]
    view = S.VIEWS[cfg.scene]
    w, h, spp = cfg.w, cfg.h, cfg.spp
    cams = [R.camera_look_at(orbit_view(view, i), view.at, view.up, view.vfov, w, h) for i in range(frames)]
    if full_ms is None:
        img = torch.zeros(w * h, dtype=torch.int32, device=dev)
        hits = torch.empty(w * h * spp * 4, dtype=torch.float32, device=dev)
        full = [scene.render_device(c, w, h, spp, d_rgba=img.data_ptr(), d_hits=hits.data_ptr(), timed=True)
                for c in cams]
        del img, hits
        full_ms = float(np.median(full[drop:]))
    out = {"emulated": True,
           "method": f"one GPU plays each rank in turn (rt_render_tiles_device of rank r's tiles, t = r mod P), "
                     f"{frames} orbit frames per rank, median of the last {frames - drop}; no gather, no overlap",
           "workload": f"{cfg.name} {w}x{h}x{spp} (BASELINE.json configs[{key - 1}])",
           "full_frame_ms": round(full_ms, 4), "P": {}}
    for P in ranks:
        tmax = max(R.tiles_for_rank(w, h, r, P) for r in range(P))
        slab = torch.zeros(max(tmax, 1) * 256, dtype=torch.int32, device=dev)
        slab_hits = torch.empty(max(tmax, 1) * 256 * spp * 4, dtype=torch.float32, device=dev)
        per = []
        for r in range(P):
            ms = [scene.render_tiles_device(c, w, h, spp, r, P, slab.data_ptr(), slab_hits.data_ptr(), timed=True)
                  for c in cams]
            per.append(float(np.median(ms[drop:])))
        del slab, slab_hits
        mx = max(per)
        out["P"][str(P)] = {"max_ms": round(mx, 4), "mean_ms": round(float(np.mean(per)), 4),
                            "per_rank_ms": [round(x, 4) for x in per],
                            "speedup": round(full_ms / mx, 3), "efficiency": round(full_ms / (P * mx), 3),
                            "mrays_per_s_projected": round(w * h * spp / (mx * 1e-3) / 1e6, 1)}
    return out


def build_stage_rooflines(pmc, n):
    """Per build stage, from the committed profile of the
    same command (profiles/pmc_summary.json build_stages, tools/pmc_summary.py):
    its rocprof time per build, the SURVEY.md §8(d) bytes it stands for
    (K0 + K1 + K2 84 B/prim, K3 64, K4-K7 256 for k_topo_refit; the crossing
    stage's K6/K7 share of the crossing nodes is inside the 256), the measured
    HBM bytes (2 x FETCH_SIZE + WRITE_SIZE), and both as fractions of 8 TB/s.
    `limiter` = the stage with the most time."""
    st = (pmc or {}).get("build_stages") or {}
    out = {}
    for k, v in st.items():
        us, hb, bpp = v.get("us"), v.get("hbm_bytes"), v.get("algo_bytes_per_prim")
        if not us:
            continue
        algo = bpp * n if bpp else None
        out[k] = {"us": round(us, 2),
                  "algo_bytes": algo, "algo_bytes_per_prim": bpp,
                  "frac": round(algo / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4) if algo else None,
                  "traffic": hb,
                  "hbm_frac_measured": round(hb / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4) if hb else None,
                  "traffic_vs_algo": round(hb / algo, 3) if hb and algo else None}
    if out:
        out["limiter"] = max((k for k in out), key=lambda k: out[k]["us"])
    return out or None


def other_config(R, S, key, torch, dev, steps=20, warmup=3, pmc_json=None, emulate=False):
    """One N=1 line for another BASELINE config (untimed by the step
    contract): build + full-frame trace per step on the same orbiting camera
    as the headline (so it is the frame `bench.py --only-timed --config k`
    profiles: profiles/pmc_summary.json), with its row-major (cold) time and
    the kernel's own byte rate (its record/triangle counters averaged over
    the timed cameras)."""
    cfg = S.CONFIGS[key]
    view = S.VIEWS[cfg.scene]
    w, h, spp = cfg.w, cfg.h, cfg.spp
    scene = make_scene(R, S, cfg)
    scene.set_device(dev.index or 0)
    cams = [R.camera_look_at(orbit_view(view, i), view.at, view.up, view.vfov, w, h) for i in range(warmup + steps)]
    img = torch.zeros(w * h, dtype=torch.int32, device=dev)
    hits = torch.empty(w * h * spp * 4, dtype=torch.float32, device=dev)
    b, t = [], []
    for i in range(warmup + steps):
        bm = scene.build()
        tm = scene.render_device(cams[i], w, h, spp, d_rgba=img.data_ptr(), d_hits=hits.data_ptr(), timed=True)
        if i >= warmup:
            b.append(bm)
            t.append(tm)
    R.config_set("trace.tile_order", 0)
    cold = float(np.median([scene.render_device(c, w, h, spp, d_rgba=img.data_ptr(), d_hits=hits.data_ptr(),
                                                timed=True) for c in cams[warmup:warmup + 4]]))
    R.config_set("trace.tile_order", 1)
    wks = [scene.render_work(c, w, h, spp) for c in cams[warmup::max(1, steps // 4)]]
    rays = w * h * spp
    kb = float(np.mean([64.0 * float(wk[0]) + 48.0 * float(wk[1]) for wk in wks])) + 16.0 * rays + 4.0 * w * h
    tr, bd = float(np.mean(t)), float(np.mean(b))
    del img, hits
    emu = rank_emulation(R, S, scene, key, torch, dev) if emulate else None
    scene.close()
    pmc = load_pmc(pmc_json, cfg.name, 1) if pmc_json else None
    return {"workload": f"{cfg.name} {w}x{h}x{spp} (BASELINE.json configs[{key - 1}])", "n_tris": cfg.n,
            "camera": f"orbiting {ORBIT_DEG} deg/step, {steps} timed steps after {warmup} (the profiled frames)",
            "roofline": roofline_of(kb, tr, pmc),
            "pmc_source": (os.path.relpath(pmc_json, ROOT) + f" [{pmc.get('tree', '?')}]") if pmc else None,
            "n_gpus": 1, "value": round(rays / (tr * 1e-3) / 1e6, 2), "unit": "Mrays/s",
            "value_cold": round(rays / (cold * 1e-3) / 1e6, 2), "trace_ms": round(tr, 4),
            "trace_ms_row_major": round(cold, 4), "build_ms": round(bd, 4),
            "build_mprims_per_s": round(cfg.n / (bd * 1e-3) / 1e6, 2),
            "build_roofline_frac": round(BUILD_BYTES_PER_PRIM * cfg.n / (bd * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "build_stage_rooflines": build_stage_rooflines(pmc, cfg.n),
            "kernel_bytes_per_launch": kb,
            # requested bytes mostly hit L2/MALL (they can exceed the HBM peak),
            # so they are priced against the aggregate L2 bandwidth
            "kernel_l2_frac": round(kb / (tr * 1e-3) / 1e9 / L2_PEAK_GBS, 4),
            "rank_emulation": emu,
            "scene_variant": "splitmix64 soup (SURVEY.md §9.9)" if cfg.scene == "soup"
            else "procedural substitute (SURVEY.md §9.9; no asset files offline)"}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    # stdout carries exactly one line, the JSON result: anything else a
    # library prints there (gloo's connection notes, RCCL banners) goes to stderr
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist
    import gpu_raytracer_amd as R
    from gpu_raytracer_amd import _lib as L
    from gpu_raytracer_amd import dist as D
    from gpu_raytracer_amd import scenes as S

    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)  # rehearsal: several ranks may share one GPU (gloo only)
    torch.cuda.set_device(local)
    if world > 1:
        # a collective stuck longer than --pg-timeout fails the process group
        # (the rank exits) instead of holding the run until an outside limit
        from datetime import timedelta
        tmo = timedelta(seconds=args.pg_timeout)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
        else:
            dist.init_process_group("gloo", timeout=tmo)

    cfg = S.CONFIGS[args.config]
    view = S.VIEWS[cfg.scene]
    w, h, spp = cfg.w, cfg.h, cfg.spp
    rays = w * h * spp
    scene = make_scene(R, S, cfg)
    n_tris = scene.num_tris
    scene.set_device(local)
    cam_static = R.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
    cams = [R.camera_look_at(orbit_view(view, i), view.at, view.up, view.vfov, w, h)
            for i in range(args.warmup + args.steps)]

    tmax = D.slab_tiles(w, h, world)
    dev = torch.device("cuda", local)
    img = torch.zeros(w * h, dtype=torch.int32, device=dev)
    hits = torch.empty(rays * 4, dtype=torch.float32, device=dev)
    slab = torch.zeros(max(tmax, 1) * 256, dtype=torch.int32, device=dev) if world > 1 else None
    # every rank writes its hit records too (16 B/ray, part of the byte model); only RGBA is gathered
    slab_hits = torch.empty(max(tmax, 1) * 256 * spp * 4, dtype=torch.float32, device=dev) if world > 1 else None
    slabs_all = torch.zeros(world * max(tmax, 1) * 256, dtype=torch.int32, device=dev) if (world > 1 and rank == 0) else None
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

    def frame(cam):
        """trace (+ gather + unpack) of one frame; returns (trace_ms, frame_ms)."""
        if world == 1:
            t = scene.render_device(cam, w, h, spp, d_rgba=img.data_ptr(), d_hits=hits.data_ptr(), timed=True)
            return t, t
        cur = torch.cuda.current_stream(dev)
        if args.dist_backend == "nccl":
            # trace -> RCCL gather -> unpack queued back to back on torch's
            # stream (the collective waits on it; no host round trip between
            # them), timed with events on that stream
            ev[0].record(cur)
            scene.render_tiles_device(cam, w, h, spp, rank, world, slab.data_ptr(), slab_hits.data_ptr(),
                                      stream=cur.cuda_stream)
            ev[1].record(cur)
            D.gather_slabs(slab, rank, world, None, slabs_all)
            if rank == 0:
                R.unpack_tiles_device(slabs_all.data_ptr(), max(tmax, 1), w, h, world, img.data_ptr(), local,
                                      cur.cuda_stream)
            ev[2].record(cur)
            ev[2].synchronize()
            return ev[0].elapsed_time(ev[1]), ev[0].elapsed_time(ev[2])
        # gloo rehearsal: stage through host memory, host-timed
        trace_ms = scene.render_tiles_device(cam, w, h, spp, rank, world, slab.data_ptr(), slab_hits.data_ptr(),
                                             timed=True)
        t0 = time.perf_counter()
        g = D.gather_slabs(slab.cpu(), rank, world)
        if rank == 0:
            slabs_all.copy_(g)
            R.unpack_tiles_device(slabs_all.data_ptr(), max(tmax, 1), w, h, world, img.data_ptr(), local,
                                  torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        return trace_ms, trace_ms + (time.perf_counter() - t0) * 1e3

    def step(i):
        build_ms = scene.build()
        return (build_ms,) + frame(cams[i])

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()

    for i in range(args.warmup):
        step(i)
    barrier()
    t0 = time.perf_counter()
    rec = [step(args.warmup + i) for i in range(args.steps)]
    barrier()
    wall = time.perf_counter() - t0
    per = np.array(rec, dtype=np.float64)  # [steps, 3] build, trace, frame span (ms)
    rank_trace_ms = float(per[:, 1].mean())
    if args.only_timed:  # profiler passes: the dispatches after the warm-up are the timed ones
        if rank == 0:
            json_out.write(json.dumps({"only_timed": True, "trace_ms_rank0": rank_trace_ms,
                                       "build_ms_rank0": float(per[:, 0].mean())}) + "\n")
            json_out.flush()
        scene.close()
        if world > 1:
            dist.destroy_process_group()
        return

    # ---- beside the timed steps (untimed by the step contract)
    # the same moving sequence with row-major dispatch = every frame cold
    R.config_set("trace.tile_order", 0)
    cold = [frame(cams[args.warmup + i])[0] for i in range(args.steps)]
    R.config_set("trace.tile_order", 1)
    # static camera: the map replays an identical frame (best case)
    static = [frame(cam_static)[0] for _ in range(args.steps + 1)][1:]
    # per-stage breakdown from one extra build with the stage events on
    R.config_set("build.stage_events", 1)
    stage_total_ms = scene.build()
    stimes = scene.build_times()
    R.config_set("build.stage_events", 0)

    # work counters of this rank's timed frames (deterministic; untimed)
    kernel_bytes = 0.0
    algo_bytes = 0.0
    rank_rays = D.rays_of_rank(w, h, spp, rank, world)
    rank_px = rank_rays // spp
    cnt0 = None
    for i in range(args.steps):
        c = cams[args.warmup + i]
        if world > 1:
            wk, bc = scene.render_tiles_work(c, w, h, spp, rank, world), scene.render_tiles_counters(c, w, h, spp, rank, world)
        else:
            wk, bc = scene.render_work(c, w, h, spp), scene.render_counters(c, w, h, spp)
        kernel_bytes += 64.0 * float(wk[0]) + 48.0 * float(wk[1]) + 16.0 * rank_rays + 4.0 * rank_px
        algo_bytes += 32.0 * float(bc[0]) + 36.0 * float(bc[1]) + 16.0 * rank_rays
    cnt_static = (scene.render_tiles_counters(cam_static, w, h, spp, rank, world) if world > 1
                  else scene.render_counters(cam_static, w, h, spp))
    kernel_bytes /= args.steps
    algo_bytes /= args.steps

    # max over ranks (per step), then mean over steps
    extra = np.array([float(np.mean(cold)), float(np.median(static))], dtype=np.float64)
    if world > 1:
        rdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
        t = torch.tensor(per, dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        per = t.cpu().numpy()
        t = torch.tensor(np.append(extra, wall), dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        extra, wall = t.cpu().numpy()[:2], float(t[2].item())
    build_ms, trace_ms, frame_ms = (float(x) for x in per.mean(axis=0))
    gather_ms = max(frame_ms - trace_ms, 0.0)
    cold_ms, static_ms = (float(x) for x in extra)

    # "rank 0 builds and then broadcasts" measured next to the
    # replicated build (untimed by the step contract; 1 warm-up + 3 timed)
    # Both are opt-in (--extras): the headline line must not wait on legs
    # that are not part of it.
    if world > 1 and args.extras and rank == args.inject_hang:
        time.sleep(1e9)  # testing: a rank that never reaches the next collective
    bvh_exchange = None
    if world > 1 and args.extras and args.dist_backend == "nccl":
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

    # the distributed build (rt_dbuild_* phases, Morton-
    # prefix all-to-all, share gathers) timed next to the replicated build;
    # its BVH must equal the replicated one bit for bit (checked on device).
    dbuild = None
    if world > 1 and args.extras:
        try:
            dms, info = [], None
            for i in range(4):
                barrier()
                tb0 = time.perf_counter()
                info = D.distributed_build(D.LibStages(scene, dev),
                                           D.Exchange(stage=args.dist_backend == "gloo", device=dev))
                barrier()
                if i:
                    dms.append((time.perf_counter() - tb0) * 1e3)
                if i == 0:  # the distributed build's sections (sorted keys/indices, nodes, wide records)
                    st = D.LibStages(scene, dev)
                    got = {k: st.buf(k).clone() for k in (L.RT_DB_KEYS, L.RT_DB_VALS, L.RT_DB_NODES, L.RT_DB_WIDE)}
            scene.build()  # the replicated build again: must give the same bytes
            st = D.LibStages(scene, dev)
            same = all(torch.equal(st.buf(k), got[k]) for k in got)
            rdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
            t = torch.tensor([float(np.median(dms)), 0.0 if same else 1.0, float(info["bytes_in"])],
                             dtype=torch.float64, device=rdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dbuild = {"distributed_build_ms": round(float(t[0].item()), 4), "replicated_build_ms": round(build_ms, 4),
                      "bit_identical": bool(t[1].item() == 0.0), "bytes_in_max_rank": int(t[2].item()),
                      "crossing_nodes": info["crossing"],
                      "exchange": "RCCL (all_to_all_single, broadcasts)" if args.dist_backend == "nccl"
                      else "gloo staged through host (rehearsal)",
                      "used": "replicated build (every rank builds; DESIGN.md 'Distributed build')"}
        except Exception as exc:  # a measurement only: never fail the bench line over it
            dbuild = {"error": f"{type(exc).__name__}: {exc}"[:200]}

    out = None
    if rank == 0:
        value = rays / (frame_ms * 1e-3) / 1e6
        pmc = load_pmc(args.pmc_json, cfg.name, world)
        roof = roofline_of(kernel_bytes, rank_trace_ms, pmc)
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
            "data": ("synthetic: random-triangle soup, splitmix64 seed 1, r=1/cbrt(N) (SURVEY.md §9.9)"
                     if cfg.scene == "soup" else f"synthetic: procedural {cfg.name} (SURVEY.md §9.9)")
                    + f"; camera orbiting {ORBIT_DEG} deg per step (every frame differs)",
            "config": {"workload": f"{cfg.name} {w}x{h}x{spp} (BASELINE.json configs[{args.config - 1}])",
                       "n_tris": n_tris, "width": w, "height": h, "spp": spp,
                       "camera": f"soup view orbiting {ORBIT_DEG} deg/step about the vertical axis through look-at",
                       "parallelism": f"image tiles 16x16 round-robin over {world} GPU(s), BVH replicated"
                                      + ((", RCCL gather to rank 0" if args.dist_backend == "nccl" else ", gloo gather (rehearsal)") if world > 1 else "")},
            "build_mprims_per_s": round(n_tris / (build_ms * 1e-3) / 1e6, 2),
            "build_ms": round(build_ms, 4),
            "build_ms_steps": {"median": round(float(np.median(per[:, 0])), 4), "min": round(float(per[:, 0].min()), 4),
                               "max": round(float(per[:, 0].max()), 4)},
            "trace_ms": round(trace_ms, 4),
            "gather_ms": round(gather_ms, 4),
            "value_cold": round(rays / ((cold_ms + gather_ms) * 1e-3) / 1e6, 2),
            "value_static_camera_best_case": round(rays / ((static_ms + gather_ms) * 1e-3) / 1e6, 2),
            "tile_order": {"timed": "longest-first from the previous frame's per-tile wave times (the camera moved "
                                    f"{ORBIT_DEG} deg since)",
                           "trace_ms_moving_ordered": round(trace_ms, 4),
                           "trace_ms_moving_row_major": round(cold_ms, 4),
                           "trace_ms_static_ordered": round(static_ms, 4),
                           "gain_moving": round(cold_ms / trace_ms, 4)},
            "bvh_exchange": bvh_exchange,
            "distributed_build": dbuild,
            "frame_mrays_per_s": round(rays / (wall / args.steps) / 1e6, 2),
            "build_stages_ms_last": {"bounds": round(stimes.bounds, 4), "morton": round(stimes.morton, 4),
                                     "sort": round(stimes.sort, 4), "topology": round(stimes.topology, 4),
                                     "refit": round(stimes.refit, 4), "wide": round(stimes.wide, 4),
                                     "total_with_stage_events": round(stage_total_ms, 4)},
            "trace_counters_rank0_static": {"nodes_fetched": int(cnt_static[0]), "tris_tested": int(cnt_static[1]),
                                            "rays": rank_rays},
            "roofline": dict(roof, kernel="trace launch: k_trace<wide> + k_trace_coop (the heavy-ray pass) (+ k_tile_order when not folded)",
                             pmc_source=(os.path.relpath(args.pmc_json, ROOT) + f" [{pmc.get('tree', '?')}]")
                             if pmc else None,
                             algo_bytes_binary_model=algo_bytes,
                             # the metric's co-headline, where the driver's parsed record keeps it
                             build={"ms": round(build_ms, 4),
                                    "mprims_per_s": round(n_tris / (build_ms * 1e-3) / 1e6, 2),
                                    "bound": "hbm", "achieved_gbs": round(build_gbs, 1),
                                    "frac": round(build_gbs / HBM_PEAK_GBS, 4),
                                    "bytes_per_prim": BUILD_BYTES_PER_PRIM,
                                    "detail": "roofline_build (per-stage kernels, PMC traffic)"},
                             note="bound = the resource with the largest measured fraction: hbm (PMC HBM bytes "
                                  "2*FETCH_SIZE + WRITE_SIZE per launch, gfx950 correction, over the event-timed "
                                  "launch vs 8 TB/s), l2 (the bytes the wide kernel requests -- 64 B per K7w record "
                                  "+ 48 B per triangle record, its own counters, + 16 B hit + 4 B RGBA per ray -- vs "
                                  "the aggregate L2; they are served by L2/MALL, so never priced against HBM) or "
                                  "valu_issue (SQ_INSTS_VALU / (1024 SIMDs x 0.5 x GRBM_GUI_ACTIVE/8), committed "
                                  "profile); achieved/peak/frac are that resource's. algo_bytes_binary_model = "
                                  "SURVEY.md §8(d) 32/node + 36/tri + 16/ray over the §9.7 binary traversal (node "
                                  "visits the wide kernel does not make: not a roofline of this kernel)"),
            "roofline_build": {"kernels": build_stage_rooflines(pmc, n_tris),
                               "bound": "hbm", "achieved": round(build_gbs, 1), "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": round(build_gbs / HBM_PEAK_GBS, 4),
                               "bytes_per_prim": BUILD_BYTES_PER_PRIM,
                               "traffic": pmc.get("build_hbm_bytes") if pmc else None,
                               "hbm_frac_measured": (round(pmc["build_hbm_bytes"] / (build_ms * 1e-3) / 1e9
                                                           / HBM_PEAK_GBS, 4)
                                                     if pmc and pmc.get("build_hbm_bytes") else None),
                               "kernel_sum_ms": pmc.get("build_kernel_sum_ms") if pmc else None,
                               "note": "SURVEY.md §8(d) 404 B/prim over the event-timed build (launch gaps "
                                       "included); traffic = PMC HBM bytes of one build's kernels, kernel_sum_ms = "
                                       "their rocprof durations (profiles/pmc_summary.json); hbm_frac_measured = "
                                       "traffic over the event-timed build vs 8 TB/s.  bound: HBM is the build's "
                                       "largest measured fraction (its kernels' VALU issue is ~0.2), though "
                                       "k_topo_refit itself is bound by its two block rounds and the random "
                                       "triangle gather's latency (DESIGN.md)"},
            "cpu_baseline": None,
        }
        # the static frame: same CRC for every N (bit-exact tiles)
        frame(cam_static)
        torch.cuda.synchronize(dev)
        host_img = img.cpu().numpy().view(np.uint8)
        import zlib
        out["image_crc32"] = zlib.crc32(host_img.tobytes()) & 0xFFFFFFFF
        if args.dump:
            R.dump_ppm(host_img, w, h, args.dump)
        if world == 1 and not args.no_extra:
            out["secondary"] = secondary_rays(S, scene, cfg, cam_static, w, h, spp, img, hits, args, torch, dev,
                                              static_ms)
            out["path"] = path_tracing(S, scene, cfg, cam_static, w, h, spp, img, args, torch, dev)
        if world == 1 and not args.no_extra:
            out["rank_emulation"] = {f"configs[{args.config - 1}]": rank_emulation(R, S, scene, args.config, torch,
                                                                                   dev)}
        if world == 1 and not args.no_cpu_baseline:
            # every CPU this process may run on at once: the affinity set,
            # capped by the cgroup quota (oversubscribing a quota only adds switches)
            q = cpu_quota()
            threads = args.cpu_threads or max(1, min(len(os.sched_getaffinity(0)), int(q) if q else 1 << 30))
            out["cpu_baseline"] = cpu_baseline(scene.tris(), view, w, h, spp, threads, cnt_static)
            out["cpu_baseline"]["config0"] = config0_leg(R, S, torch, dev, threads)
    elif world > 1 and rank != 0:
        frame(cam_static)  # rank 0's CRC frame needs every rank's tiles
    scene.close()
    if rank == 0 and world == 1 and not args.no_extra:
        out["other_configs"] = {}
        for key in (2, 4, 5):
            if key == args.config:
                continue
            try:
                oc = other_config(R, S, key, torch, dev, pmc_json=args.pmc_json, emulate=key in (4, 5))
                emu = oc.pop("rank_emulation")
                if emu:
                    out.setdefault("rank_emulation", {})[f"configs[{key - 1}]"] = emu
                out["other_configs"][f"config{key}"] = oc
            except Exception as exc:  # a side measurement: never lose the headline line over it
                out["other_configs"][f"config{key}"] = {"error": f"{type(exc).__name__}: {exc}"[:200]}
    if rank == 0:
        json_out.write(json.dumps(out) + "\n")
        json_out.flush()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

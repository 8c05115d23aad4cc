#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: Mrays/s + reconstructed fps at 4K, 10% foveal density.

Workload (BASELINE.json configs[2], the one the metric is quoted on): bunny scene, 3840x2160,
4 spp, GI with diffuse_max_depth 3, 10% foveated log-polar mask, full reconstruction chain. One
"step" is one frame of the reference's main loop (FR/main.cpp:253-358): G-buffer trace ->
sampling mask -> compaction -> foveated path trace -> JumpFlooding -> Sibson -> pull-push ->
A-Trous, every stage a gfx950 HIP kernel behind the C ABI (include/fovrt.h).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process per
GPU; by default the one 4K view is tile-sharded over the N ranks (strong scaling) through libfovrt's
multi-GPU group (fr_group_*: RCCL ncclSend/ncclRecv of the traced pixels to the two reconstruction
ranks); --views N renders one view per rank instead (weak scaling). value = ray segments of all ranks
(the G-buffer counted once per view) / max elapsed over ranks.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "foveated-rendering-using-ray-tracing_amd"))

import numpy as np  # noqa: E402

import fovrt  # noqa: E402

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, spec)


def stage_bytes(W, H, rho, spp, jfa_passes):
    """Algorithmic HBM bytes per frame of each stage (per pixel x N)."""
    N = W * H
    return {
        "geometry": 52 * N,
        "sampling": 57 * N,
        "optimize": (1 + 4 * rho) * N,
        "shading": (56 + 4 * rho) * N,
        "jfa": (56 + 8 * jfa_passes) * N,
        "sibson": 36 * N,
        "pullpush": 74.7 * N,
        "atrous": 60 * N,
    }


def jfa_passes(W, H):
    m = 1
    while m * 2 < W or m * 2 < H:
        m *= 2
    return int(np.log2(m)) + 1


def cpu_baseline(args, cfg_scene_arrays, cam_uni_fn, gpu_segments_per_frame=None):
    """The CPU oracle (oracle/, a literal restatement of the reference path, OpenMP over rows) timed on
    this host on a bounded sample of the same workload (scene, resolution, spp, GI, mask), SURVEY §8(d)'s
    method shortened to fit the bench: frame 0 is the warm-up (it also establishes the temporal history),
    frames 1..3 are timed and the median is reported."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    W, H = args.width // args.cpu_scale, args.height // args.cpu_scale
    sc = po.OracleScene(cfg_scene_arrays, refraction_max_depth=args.refraction_max_depth,
                        diffuse_max_depth=args.dmd)
    uni = cam_uni_fn(W, H)
    hist = np.zeros((H, W, 4), np.float32)
    depth_cache = np.zeros((H, W, 4), np.float32)
    pp = po.PullPushState(W, H)
    times, segs, t_all = [], [], time.perf_counter()
    for frame in range(1 + args.cpu_frames):
        sc.segments(reset=True)
        t0 = time.perf_counter()
        g = po.gbuffer(sc, uni, W, H, frame)
        s = po.sampling(sc, uni, W, H, args.mask, g["position"], g["depth"], depth_cache, g["weight"],
                        g["normal"], g["diffuse"])
        n, _ = po.warp_sort(s["mask"])
        sh = po.shading(sc, uni, W, H, frame, args.spp, s["mask"], s["weight"], hist)
        coord, color = po.jfa(sh["shading"])
        po.sibson(coord, color)
        out = pp.render(sh["shading"])
        po.atrous(1, g["position"], g["normal"], out)
        dt = time.perf_counter() - t0
        hist, depth_cache = sh["history"], g["depth"]
        if frame >= 1:
            times.append(dt)
            segs.append(sc.segments(reset=True))
    t_med = float(np.median(times))
    seg_med = float(np.median(segs))
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    scale = "" if args.cpu_scale == 1 else f" at 1/{args.cpu_scale} x 1/{args.cpu_scale} resolution"
    res = {"value": round(seg_med / t_med / 1e6, 4), "unit": "Mrays/s", "cores": cores, "kind": "port",
           "sample": f"oracle (OpenMP) full frames {W}x{H}{scale}, same scene/spp/GI/mask as the GPU workload; "
                     f"frame 0 the warm-up (it builds the history), median of frames 1-{args.cpu_frames} timed "
                     f"({', '.join(f'{t:.2f}' for t in times)} s); {time.perf_counter() - t_all:.1f} s of CPU work "
                     f"in total",
           "frame_s": round(t_med, 3), "frames_s": [round(t, 3) for t in times], "fps": round(1.0 / t_med, 4),
           "segments_per_frame": int(seg_med),
           "segments_definition": "every segment the reference traces, including the G-buffer shadow rays whose "
                                  "result g_diffuse.cu:110-143 never reads and the grandchildren diffuse.cu:142 / "
                                  "reflection.cu:144 discard (the GPU engine does not trace those: its "
                                  "segments_per_frame counts only segments traced), so Mrays/s ratios mix two "
                                  "definitions; compare fps"}
    if gpu_segments_per_frame:
        res["gpu_segments_per_frame"] = int(gpu_segments_per_frame)
    return res


def pct(a):
    """p50 / p99 / max / mean of a sample of milliseconds."""
    a = np.asarray(a, np.float64)
    return {"p50": round(float(np.median(a)), 4), "p99": round(float(np.percentile(a, 99)), 4),
            "max": round(float(a.max()), 4), "mean": round(float(a.mean()), 4), "n": int(a.size)}


def view_offset(rank, world):
    """Views of a multi-view job: view v is an eye offset along x by 6.4 cm per view around the preset
    camera (the stereo pair of BASELINE configs[4] at 2 views)."""
    return np.array([0.064 * (rank - (world - 1) / 2.0), 0.0, 0.0], np.float32)


def reduce_over_ranks(dist, device, elapsed, segs):
    """Max of the elapsed times and sum of the ray segments over all ranks (value = all ranks' rays /
    slowest rank's time)."""
    import torch
    if dist is None:
        return elapsed, float(segs)
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    s = torch.tensor([float(segs)], dtype=torch.float64, device=device)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    return float(t.item()), float(s.item())


def view_segments(st, G, vrank):
    """Ray segments a rank contributes to `value`, and its redundant ones. A tile-sharded view (G > 1)
    traces its full G-buffer on every one of its G ranks (the saliency stencils and the reconstruction
    ranks read all of it): those W*H primaries count once per view, on the view's first rank; the other
    ranks' copies are reported apart as redundant work, never as throughput."""
    segs = int(st["segments"])
    if G > 1 and vrank != 0:
        return segs - int(st["gbuffer_primary"]), int(st["gbuffer_primary"])
    return segs, 0


def view_layout(rank, world, views):
    """Ranks -> views: `views` views of world / views ranks each (fr_group: rank r renders view r / G as
    view rank r % G). Returns (view, rank in view, ranks per view)."""
    if views <= 0:
        views = 1
    if world % views:
        raise SystemExit(f"--views {views} must divide the number of ranks {world}")
    g = world // views
    return rank // g, rank % g, g


def broadcast_id(dist, rank, make_id):
    """The 128-byte RCCL unique id of rank 0 (fr_rccl_unique_id) to every rank over the bootstrap
    process group (gloo): the only use of torch.distributed besides the barrier and the reductions."""
    import torch
    t = torch.zeros(128, dtype=torch.uint8)
    if rank == 0:
        t.copy_(torch.frombuffer(bytearray(make_id()), dtype=torch.uint8))
    dist.broadcast(t, 0)
    return bytes(t.numpy().tobytes())


def profile_paths(suffix):
    """profiles/*_<suffix> newest first: the tag named in profiles/CURRENT (the last evidence run of the shipped
    build, scripts/r06_evidence.sh) leads, then the rest by name."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_" + suffix)), reverse=True)
    try:
        with open(os.path.join(ROOT, "profiles", "CURRENT")) as f:
            cur = os.path.join(ROOT, "profiles", f.read().strip() + "_" + suffix)
    except OSError:
        cur = None
    if cur in paths:
        paths.remove(cur)
        paths.insert(0, cur)
    return paths


def load_traffic(kernels, config):
    """HBM bytes per launch of `kernels` from the newest profiles/*_pmc_traffic.json recorded on the
    same workload (scripts/profile.sh), else None."""
    for path in profile_paths("pmc_traffic.json"):
        try:
            with open(path) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            continue
        cfg = doc.get("config") or {}
        if any(cfg.get(k) != config.get(k) for k in ("scene", "width", "height", "spp", "diffuse_max_depth",
                                                     "mask_mode")):
            continue
        # by base name: "void k_carry_history<false>" is k_carry_history (every template instance counts)
        base = {}
        for name, v in doc.get("kernels", {}).items():
            b = name.split("<")[0].split("(")[0].split()[-1] if name.strip() else ""
            base[b] = base.get(b, 0.0) + v["hbm_bytes"]
        if all(k in base for k in kernels):
            return sum(base[k] for k in kernels), os.path.relpath(path, ROOT)
    return None, None


def load_issue(kernel, config):
    """The SIMD issue picture of `kernel` from the newest profiles/*_pmc_issue.json recorded on the same
    workload (scripts/pmc_sq.sh + scripts/pmc_issue.py), else None."""
    for path in profile_paths("pmc_issue.json"):
        try:
            with open(path) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            continue
        cfg = doc.get("config") or {}
        if any(cfg.get(k) != config.get(k) for k in ("scene", "width", "height", "spp", "diffuse_max_depth",
                                                     "mask_mode")):
            continue
        ent = doc.get("kernels", {}).get(kernel)
        if ent:
            return dict(ent, source=os.path.relpath(path, ROOT))
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--scene", default="bunny", choices=list(fovrt.SCENES))
    ap.add_argument("--mask", default="logpolar10", choices=list(fovrt.MASKS))
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--dmd", type=int, default=3, help="diffuse_max_depth (GI bounces)")
    ap.add_argument("--refraction-max-depth", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-scale", type=int, default=1, help="CPU baseline at 1/scale resolution per axis")
    ap.add_argument("--cpu-frames", type=int, default=3, help="CPU baseline: timed frames after the warm-up")
    ap.add_argument("--serial-frames", type=int, default=50,
                    help="frames of the serial frame-time measurement (after 5 warm-ups; SURVEY §8(d))")
    ap.add_argument("--views", type=int, default=1,
                    help="views rendered by the job (default 1: one 4K view tile-sharded over all ranks, strong "
                         "scaling; --views N with N ranks: one view per rank, weak scaling)")
    ap.add_argument("--tile", type=int, default=128, help="screen tile size of the tile sharding (multiple of 16)")
    ap.add_argument("--no-split", action="store_true",
                    help="both reconstruction chains on the view's rank 0 (default: JFA -> Sibson on view rank 0, "
                         "pull-push -> A-Trous on view rank 1)")
    ap.add_argument("--jfa-ranks", type=int, default=0,
                    help="view ranks taking JFA -> Sibson in turns, one frame each (fr_group_config.jfa_ranks; "
                         "0 = auto: 2 at 6+ ranks per view, else 1)")
    ap.add_argument("--no-front-local", action="store_true",
                    help="every rank runs the full-screen front stages (default: a still camera's tracing ranks "
                         "run them on their own tiles plus halo)")
    ap.add_argument("--recon-cost", type=float, nargs=2, default=None,
                    help="reconstruction work of view ranks 0 and 1 as fractions of a frame's trace work, for "
                         "the tile dealing (default: fr_group_config_default's)")
    ap.add_argument("--composite", action="store_true",
                    help="every frame, gather the views' A-Trous images to rank 0 over RCCL and lay them side by "
                         "side (the final composite of the stereo configuration)")
    ap.add_argument("--local-ranks", type=int, default=1,
                    help="rehearsal on one device: this many ranks as contexts of one process (fr_group with "
                         "device-to-device copies instead of RCCL); not a measurement of multi-GPU scaling")
    ap.add_argument("--bvh", default="host", choices=["host", "gpu"],
                    help="BVH builder: host binned SAH (default) or the GPU LBVH (k_bvh.hip)")
    ap.add_argument("--pan", type=float, default=0.0,
                    help="per-frame step of the camera's look-at target in scene units (0: static camera). A "
                         "moving camera makes the history reprojection read across tiles; every rank of a "
                         "tile-sharded view then receives every other rank's traced pixels")
    ap.add_argument("--gaze-path", nargs="?", const="circle", default=None, choices=["circle", "saccade"],
                    help="the gaze follows a scripted cursor path every frame (cursorPosCallback, FR/gui.cpp:48-66), "
                         "so the mask is recomputed every frame (an eye-tracked frame): 'circle' (the bare flag) "
                         "circles the screen centre at a quarter of the height, one degree per frame; 'saccade' "
                         "jumps 90 degrees along the same circle every 30 frames")
    args = ap.parse_args()
    args.mask = fovrt.MASKS[args.mask]
    scene = fovrt.SCENES[args.scene]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        # torch.distributed (gloo, CPU) is the bootstrap only: the RCCL id, barriers, max/sum reductions.
        # Every frame's data path is libfovrt's own RCCL group (fr_group_*).
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend="gloo")
    has_gpu = torch.cuda.is_available()
    if world > 1 and args.local_ranks > 1:
        raise SystemExit("--local-ranks is a one-process rehearsal; do not combine it with torch.distributed")

    def sync():
        if has_gpu:
            torch.cuda.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()

    W, H = args.width, args.height
    ndev = max(1, torch.cuda.device_count())
    R = world if world > 1 else args.local_ranks   # ranks of the group
    views = args.views
    my_ranks = [rank] if world > 1 else list(range(R))
    layouts = [view_layout(r, R, views) for r in my_ranks]
    G = layouts[0][2]
    cfg_kw = dict(width=W, height=H, scene=scene, mask_mode=args.mask, spp=args.spp, diffuse_max_depth=args.dmd,
                  refraction_max_depth=args.refraction_max_depth, bvh_builder=1 if args.bvh == "gpu" else 0)
    tracers = []
    for r in my_ranks:
        t = fovrt.PathTracer(fovrt.Config(device=(local_rank if world > 1 else 0) % ndev, **cfg_kw))
        t.initialize()
        tracers.append(t)
    tracer = tracers[0]
    cams = {}
    for (view, _, _), t in zip(layouts, tracers):
        if view not in cams:
            cam = fovrt.Camera.preset(scene, W, H)
            if views > 1:  # each view is its own eye (offset along x, 6.4 cm per view)
                cam.setPosition(np.asarray(cam.pos) + view_offset(view, views))
                cam.lookAt(cam.target)
            cams[view] = cam
        t.update_optix_variables(cams[view])

    group = None
    if R > 1:
        gkw = dict(views=views, tile=args.tile, split_recon=not args.no_split, moving_camera=args.pan != 0.0,
                   composite=args.composite and views > 1, recon_cost=args.recon_cost, jfa_ranks=args.jfa_ranks,
                   front_local=not args.no_front_local)
        if world > 1:
            uid = broadcast_id(dist, rank, fovrt.rccl_unique_id)
            group = fovrt.Group.rccl(tracer, uid, world, rank, **gkw)
        else:
            group = fovrt.Group(tracers, **gkw)
    roles = [group.rank_info(i) for i in range(len(tracers))] if group else [{"view": 0, "view_rank": 0, "chains": 3,
                                                                             "tiles": -1}]

    step_dir = np.array([1.0, 0.5, 0.0], np.float32)
    step_dir *= np.float32(args.pan) / np.linalg.norm(step_dir)
    frame_no = [0]

    def move_camera():
        """Camera path of the moving-camera runs: the eye stays, the look-at target moves a fixed step per
        frame (setPrevState first, so frame N reprojects into frame N-1 as FR/main.cpp:443 does)."""
        for cam in cams.values():
            cam.setPrevState()
            cam.lookAt(np.asarray(cam.target) + step_dir)
        for (view, _, _), t in zip(layouts, tracers):
            t.update_optix_variables(cams[view])

    def move_gaze():
        """A scripted cursor (window coordinates, y down) circling the screen centre at a quarter of the
        height, one degree per frame, fed through cursorPosCallback's mapping (fr_set_gaze, windowed)."""
        deg = frame_no[0] if args.gaze_path == "circle" else 90 * (frame_no[0] // 30)
        a = np.deg2rad(deg)
        x = W / 2 + 0.25 * H * np.cos(a)
        y = (H / 2 + 0.25 * H * np.sin(a)) / 1.25  # the callback scales y by 1.25 in a window
        for t in tracers:
            t.set_gaze(x, y)

    def step(timing):
        if args.pan:
            move_camera()
        if args.gaze_path:
            move_gaze()
        frame_no[0] += 1
        if group is None:
            return tracer.frame(timing=timing)
        tm = group.frame(timing=timing)
        return tm[0] if timing else None

    for _ in range(args.warmup):
        step(False)
    if group:
        group.synchronize()
    for t in tracers:
        t.synchronize()
    sync()
    for t in tracers:
        t.reset_stats()

    # The timed region: K frames enqueued back to back; consecutive frames pipeline (frame N's
    # reconstruction runs while frame N+1 traces). Entry 3 (the roofline stage) is timed live inside it:
    # HIP events on the context stream around the stage and its megakernel, no synchronisation added.
    tracer.kernel_timing(True)
    if group is None:
        tracer.frame_clock(True)  # per-frame latency (gaze -> image) and display interval, HIP events
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(False)
    if group:
        group.synchronize()
    for t in tracers:
        t.synchronize()
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    live = tracer.kernel_times()
    tracer.kernel_timing(False)
    clock = None
    if group is None:
        lat, itv = tracer.frame_clock_read()
        tracer.frame_clock(False)
        if len(lat) and len(itv):
            clock = {"latency_ms": pct(lat), "interval_ms": pct(itv)}

    segs = redundant = 0
    for (view, vrank, g), t in zip(layouts, tracers):
        a, b = view_segments(t.stats(), g, vrank)
        segs += a
        redundant += b
    st = tracer.stats()
    dev = torch.device("cpu") if dist is not None else None
    elapsed, total_segs = reduce_over_ranks(dist, dev, elapsed, segs)
    _, total_redundant = reduce_over_ranks(dist, dev, 0.0, redundant)

    # The latency-bounded mode (fr_set_pipeline_mode LATENCY: one trace half in flight, the previous frame's
    # reconstruction beside the next trace half) on the same workload: K more frames after a few warm-ups,
    # wall-clock fps and the frame clock. Measured after `value`'s timed region, never inside it.
    latency_mode = None
    if group is None:
        tracer.set_pipeline_mode(fovrt.PIPELINE_LATENCY)
        for _ in range(3):
            step(False)
        tracer.synchronize()
        tracer.frame_clock(True)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step(False)
        tracer.synchronize()
        el = time.perf_counter() - t1
        lat, itv = tracer.frame_clock_read()
        tracer.frame_clock(False)
        tracer.set_pipeline_mode(fovrt.PIPELINE_THROUGHPUT)
        latency_mode = {"fps": round(args.steps / el, 2), "ms_per_step": round(el / args.steps * 1e3, 4),
                        "frame_clock": {"latency_ms": pct(lat), "interval_ms": pct(itv)} if len(lat) and len(itv) else None,
                        "note": "fr_set_pipeline_mode(FR_PIPELINE_LATENCY): fr_frame waits on the host for the previous "
                                "frame's JumpFlooding (and, just in time, for the part of its Sibson the front stages "
                                "would not cover), then samples the gaze and enqueues the frame; its front stages "
                                "overlap the previous frame's Sibson and pull-push -> A-Trous, its path trace starts "
                                "after them. Same frames (bit-identical results), measured after the throughput run; "
                                "fps = frames / wall time, to compare with fps_serial_mean on a varying workload"}


    # Per-stage HIP-event breakdown of the same frames, serialised (each frame synchronised, so the
    # stage times do not overlap the next frame): the stage table and the roofline kernel time.
    # The same frames are SURVEY §8(d)'s reconstructed-frame time: HIP events around one whole
    # synchronised frame (update -> entries 0-3 -> JFA -> Sibson -> pull-push -> A-Trous, nothing of the
    # next frame overlapping), the median of --serial-frames after 5 warm-ups.
    stage_ms, stage_n = {}, {}
    for _ in range(5):
        step(True)
    n_timed = max(3, args.serial_frames)
    totals = []
    for _ in range(n_timed):
        tm = step(True)
        totals.append(tm["total_ms"])
        for k, v in tm.items():
            if k.endswith("_ms"):
                stage_ms[k] = stage_ms.get(k, 0.0) + v
                stage_n[k] = stage_n.get(k, 0) + (v > 0)
    serial = pct(np.asarray(totals, np.float64))
    for t in tracers:
        t.synchronize()
    # foveal density: every rank's active pixels of the last frame (a rank traces only its tiles)
    count_sum = float(sum(t.ray_count() for t in tracers))
    _, count_sum = reduce_over_ranks(dist, dev, 0.0, count_sum)

    K = args.steps
    # (per stage over the frames that ran it: with jfa_ranks > 1 rank 0 runs JFA -> Sibson every m-th frame)
    avg = {k[:-3]: v / max(1, stage_n[k]) for k, v in stage_ms.items()}
    rho = count_sum / views / (W * H)
    L = jfa_passes(W, H)
    sb = stage_bytes(W, H, rho, args.spp, L)
    # (a rank that runs no reconstruction chain reports 0 ms for those stages)
    stage_table = {k: {"ms": round(avg[k], 4),
                       "GB/s": round(sb[k] / (avg[k] * 1e-3) / 1e9, 1) if avg[k] > 0 else None} for k in sb}
    # the dominant stage is entry 3 (shading_launch): k_shade_paths (path-trace megakernel) +
    # k_shade_resolve + k_carry_history; its algorithmic bytes are SURVEY §8(d)'s (56 + 4 rho) B/px.
    dominant = max(sb, key=lambda k: avg[k])
    launch_ms = avg[dominant]
    kernel_ms = avg.get("shade_paths", 0.0)
    timing_src = "HIP events on the context stream, serialised frames after the timed region"
    if dominant == "shading" and live["frames"] > 0:
        launch_ms = live["shading_ms"] / live["frames"]
        kernel_ms = live["shade_paths_ms"] / live["frames"]
        timing_src = (f"HIP events on the context stream around every entry-3 launch of the timed region "
                      f"({live['frames']} pipelined frames)")
    achieved = sb[dominant] / (launch_ms * 1e-3) / 1e9
    stage_kernels = {"shading": ["k_shade_paths", "k_shade_resolve", "k_carry_history"],
                     "geometry": ["k_gbuffer"], "sibson": ["k_sibson_runs"]}
    image_stages = ["sampling", "optimize", "jfa", "sibson", "pullpush", "atrous"]
    img_bytes = sum(sb[k] for k in image_stages)
    img_ms = sum(avg[k] for k in image_stages)
    n_ranks = R
    n_jfa = args.jfa_ranks or (2 if not args.no_split and G >= 6 else 1)  # group.cpp's auto rule
    jfa_vranks = [0] + list(range(2, n_jfa + 1))
    if R == 1:
        parallelism = "one view on one GPU"
    elif G == 1:
        parallelism = f"{views} views, one per rank (weak scaling), no data-path collective"
    else:
        parallelism = (f"{views} view(s) x {G}-way {args.tile}px tile sharding (fr_group, tiles dealt by reconstruction "
                       f"load); traced pixels (20 B each) to the view's reconstruction ranks over RCCL "
                       f"ncclSend/ncclRecv; " + ("both chains on view rank 0" if args.no_split else
                                                 f"JFA -> Sibson on view rank(s) {jfa_vranks} in turns, pull-push -> "
                                                 "A-Trous on view rank 1") +
                       (" (every rank receives every rank's pixels: moving camera)" if args.pan else
                        "" if args.no_front_local else "; tracing ranks run tile-local front stages"))
    if args.local_ranks > 1:
        parallelism += f"; REHEARSAL: {R} ranks as contexts of one process on one device (not a scaling measurement)"
    result = {
        "metric": "Mrays/s + reconstructed fps @4K, 10% foveal density, 1/2/4/8 GPU",
        "value": round(total_segs / elapsed / 1e6, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / K * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak" if G == 1 else "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": f"{args.scene} {W}x{H}, {args.spp} spp, diffuse_max_depth {args.dmd}, "
                               f"log-polar mask ({'signed, ~10%' if args.mask == 4 else 'mode %d' % args.mask}), "
                               "JFA + Sibson + pull-push + A-Trous",
                   "scene": args.scene, "width": W, "height": H, "spp": args.spp, "diffuse_max_depth": args.dmd,
                   "mask_mode": args.mask, "foveal_density": round(rho, 5), "views": views, "ranks": n_ranks,
                   "composite": bool(args.composite and views > 1), "camera_step": args.pan,
                   "gaze": {None: "screen centre",
                            "circle": "scripted cursor circle, one degree per frame, mask recomputed every frame",
                            "saccade": "scripted saccades: 90 degrees along the cursor circle every 30 frames, mask "
                                       "recomputed every frame"}[args.gaze_path],
                   "parallelism": parallelism,
                   "procedural_meshes": "box/bunny/earth stand-ins (the reference's .obj files are absent)"},
        "fps": round(K / elapsed, 2),
        "fps_definition": "pipelined throughput: K frames enqueued back to back, frame N's reconstruction "
                          "overlapping frame N+1's trace half (frames per second of the timed region); "
                          "fps_serial is SURVEY §8(d)'s 1 / (wall time of one whole frame)",
        "frames_per_s_total": round(views * K / elapsed, 2),
        "frame_ms_serial": serial,
        "fps_serial": round(1e3 / serial["p50"], 2),
        "fps_serial_mean": round(1e3 / float(np.mean(totals)), 2),
        "frame_ms_serial_note": f"HIP events around one synchronised frame (update -> A-Trous, the two reconstruction "
                                f"chains on their own streams), {n_timed} frames after 5 warm-ups, rank 0"
                                + ("" if group is None else "; a group frame includes the exchange"),
        "frame_clock_pipelined": clock,
        "pipeline_latency_mode": latency_mode,
        "frame_clock_note": "every frame of the timed region: latency = from where its G-buffer may start (the "
                            "gaze sample) to the end of its Sibson and A-Trous; interval = between consecutive "
                            "frames' ends (what a display sees). HIP events, one context",
        "rays": {k: st[k] for k in ("gbuffer_primary", "primary", "shadow", "diffuse_bounce", "mirror",
                                    "refraction", "reflection", "truncated", "overflow")},
        "rays_note": "rank 0's counters over the timed frames",
        "gbuffer_redundant_segments": int(total_redundant),
        "rank0_role": roles[0],
        "stages": stage_table,
        "stages_note": f"rank 0's HIP events, {n_timed} serialised frames; the timed region pipelines frame N's "
                       "reconstruction with frame N+1's trace half, so ms_per_step < the sum of the stages",
        "roofline": {"bound": "hbm", "kernel": f"{dominant} stage ({' + '.join(stage_kernels.get(dominant, []))})",
                     "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 5), "traffic": None,
                     "ms_per_launch": round(launch_ms, 4),
                     "algorithmic_bytes_per_launch": int(sb[dominant]),
                     "megakernel_ms": round(kernel_ms, 4),
                     "ms_per_launch_serialised": round(avg[dominant], 4),
                     "megakernel_ms_serialised": round(avg.get("shade_paths", 0.0), 4),
                     "timing": timing_src,
                     "note": "achieved = SURVEY §8(d) algorithmic bytes of the stage / its average duration; the "
                             "path-trace megakernel is latency/divergence bound (BVH pointer chasing), so Mrays/s "
                             "is its figure of merit, image passes are HBM bound"},
        "roofline_image_passes": {"bound": "hbm", "achieved": round(img_bytes / (img_ms * 1e-3) / 1e9, 1),
                                  "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                  "frac": round(img_bytes / (img_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)},
    }
    traffic, src = load_traffic(stage_kernels.get(dominant, []), result["config"]) if R == 1 else (None, None)
    if traffic is not None:
        result["roofline"]["traffic"] = int(traffic)
        result["roofline"]["traffic_source"] = src
        result["roofline"]["measured_hbm_GBs"] = round(traffic / (launch_ms * 1e-3) / 1e9, 1)
    issue = load_issue("k_shade_paths", result["config"]) if R == 1 else None
    if issue is not None:
        # what bounds the megakernel instead of HBM: the SIMD's VALU issue (profiles/*_pmc_issue.json). It comes
        # from a separate counter pass (an earlier run, possibly of an earlier build), never from this run
        issue["measured_in_this_run"] = False
        result["roofline"]["issue"] = issue
    if traffic is not None:
        result["roofline"]["traffic_measured_in_this_run"] = False
    if group:
        group.destroy()
    # the GPU BVH builder on this scene (after every measurement: it replaces the BVH)
    builds = [tracer.rebuild_bvh() for _ in range(6)]
    result["bvh"] = {"builder": args.bvh, "gpu_rebuild_ms": round(float(np.median(builds)), 3),
                     "max_rebuild_ms": round(float(max(builds)), 3),
                     "rebuild_ms": [round(b, 3) for b in builds],
                     "note": "fr_rebuild_bvh wall time of six rebuilds in a row (median, max and all); the context "
                             "allocates the builder and both trees at fr_create and releases the host-built tree there "
                             "(no allocation or release in a rebuild; DESIGN.md section 8, row 2)",
                     "triangles": int(tracer.scene_arrays()["pos"].shape[0])}
    if rank == 0 and R == 1 and not args.no_cpu_baseline:
        try:
            arrays = tracer.scene_arrays()

            def uni_fn(w, h):
                return fovrt.Camera.preset(scene, w, h).uniforms(w, h)
            result["cpu_baseline"] = cpu_baseline(args, arrays, uni_fn, total_segs / K)
            result["cpu_baseline"]["gpu_cpu_fps_ratio"] = {
                "serial": round(result["fps_serial"] / result["cpu_baseline"]["fps"], 1),
                "pipelined": round(result["fps"] / result["cpu_baseline"]["fps"], 1)}
        except Exception as e:  # report, never fake
            result["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    for t in tracers:
        t.destroy()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

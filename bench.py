#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: Mrays/s + reconstructed fps at 4K, 10% foveal density.

Workload (BASELINE.json configs[2], the one the metric is quoted on): bunny scene, 3840x2160,
4 spp, GI with diffuse_max_depth 3, 10% foveated log-polar mask, full reconstruction chain. One
"step" is one frame of the reference's main loop (FR/main.cpp:253-358): G-buffer trace ->
sampling mask -> compaction -> foveated path trace -> JumpFlooding -> Sibson -> pull-push ->
A-Trous, every stage a gfx950 HIP kernel behind the C ABI (include/fovrt.h).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process per
GPU, each rendering its own view (the eyes / views of a multi-view frame) with no data-path
collective -> weak scaling; value = ray segments of all ranks / max elapsed over ranks.

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


def cpu_baseline(args, cfg_scene_arrays, cam_uni_fn):
    """The CPU oracle (oracle/, a literal restatement of the reference path, OpenMP over rows) timed on
    this host on a bounded sample: the full bench workload (same scene/resolution/spp/GI/mask), two
    frames, the second one timed (frame 0 only establishes the temporal history)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    W, H = args.width // args.cpu_scale, args.height // args.cpu_scale
    sc = po.OracleScene(cfg_scene_arrays, refraction_max_depth=args.refraction_max_depth,
                        diffuse_max_depth=args.dmd)
    uni = cam_uni_fn(W, H)
    hist = np.zeros((H, W, 4), np.float32)
    depth_cache = np.zeros((H, W, 4), np.float32)
    pp = po.PullPushState(W, H)
    t_total, segs, t_all = 0.0, 0, time.perf_counter()
    for frame in range(2):
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
        if frame == 1:
            t_total, segs = dt, sc.segments(reset=True)
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    scale = "" if args.cpu_scale == 1 else f" at 1/{args.cpu_scale} x 1/{args.cpu_scale} resolution"
    return {"value": round(segs / t_total / 1e6, 4), "unit": "Mrays/s", "cores": cores, "kind": "port",
            "sample": f"oracle (OpenMP) full frame {W}x{H}{scale}, same scene/spp/GI/mask as the GPU workload; "
                      f"frame 0 untimed (history), frame 1 timed: {segs} ray segments counted as the reference "
                      f"traces them (incl. rays whose results it never reads) in {t_total:.2f} s "
                      f"({time.perf_counter() - t_all:.1f} s of CPU work in total)",
            "frame_s": round(t_total, 3), "fps": round(1.0 / t_total, 4)}


def view_offset(rank, world):
    """Weak scaling over views: rank r renders its own eye/view, offset along x by 6.4 cm per view
    around the preset camera (the stereo pair of BASELINE configs[4] at world 2)."""
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
    traces its full G-buffer on every one of its G ranks (the saliency stencils and the root's A-Trous
    read all of it): those W*H primaries count once per view, on the view's first rank; the other
    ranks' copies are reported apart as redundant work, never as throughput."""
    segs = int(st["segments"])
    if G > 1 and vrank != 0:
        return segs - int(st["gbuffer_primary"]), int(st["gbuffer_primary"])
    return segs, 0


def view_layout(rank, world, views):
    """Ranks -> views: `views` views of world / views ranks each; the ranks of a view tile-shard it
    and composite on the view's first rank. Returns (view, rank in view, ranks per view)."""
    if views <= 0:
        views = world
    if world % views:
        raise SystemExit(f"--views {views} must divide the number of ranks {world}")
    g = world // views
    return rank // g, rank % g, g


def make_view_groups(dist, world, views):
    """One process group per view (every rank creates every group, in the same order)."""
    g = world // views
    return [dist.new_group(list(range(v * g, (v + 1) * g))) for v in range(views)]


def gather_slabs(dist, group, slab, gather_list, dst):
    """RCCL gather of every rank's packed tiles to the view's compositing rank `dst` (over gloo, as
    in the one-GPU rehearsal, device slabs are staged through host memory)."""
    if dist.get_backend() == "gloo" and slab.is_cuda:
        host = slab.cpu()
        hl = [t.cpu() for t in gather_list] if gather_list is not None else None
        dist.gather(host, gather_list=hl, dst=dst, group=group)
        if gather_list is not None:
            for t, h in zip(gather_list, hl):
                t.copy_(h)
        return
    dist.gather(slab, gather_list=gather_list, dst=dst, group=group)


def allgather_slabs(dist, group, slab, out_list):
    """All-gather of every rank's packed tiles (the moving-camera history exchange), staged through
    host memory over gloo like gather_slabs."""
    if dist.get_backend() == "gloo" and slab.is_cuda:
        hl = [t.cpu() for t in out_list]
        dist.all_gather(hl, slab.cpu(), group=group)
        for t, h in zip(out_list, hl):
            t.copy_(h)
        return
    dist.all_gather(out_list, slab, group=group)


def load_traffic(kernels, config):
    """HBM bytes per launch of `kernels` from the newest profiles/*_pmc_traffic.json recorded on the
    same workload (scripts/profile.sh), else None."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")), reverse=True):
        try:
            with open(path) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            continue
        cfg = doc.get("config") or {}
        if any(cfg.get(k) != config.get(k) for k in ("scene", "width", "height", "spp", "diffuse_max_depth",
                                                     "mask_mode")):
            continue
        ks = doc.get("kernels", {})
        if all(k in ks for k in kernels):
            return sum(ks[k]["hbm_bytes"] for k in kernels), os.path.relpath(path, ROOT)
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--scene", default="bunny", choices=list(fovrt.SCENES))
    ap.add_argument("--mask", default="logpolar10", choices=list(fovrt.MASKS))
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--dmd", type=int, default=3, help="diffuse_max_depth (GI bounces)")
    ap.add_argument("--refraction-max-depth", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-scale", type=int, default=1, help="CPU baseline at 1/scale resolution per axis")
    ap.add_argument("--views", type=int, default=0,
                    help="views rendered by the job (0: one per rank = weak scaling); the ranks of a view "
                         "tile-shard it and gather the tiles to the view's first rank for reconstruction")
    ap.add_argument("--tile", type=int, default=128, help="screen tile size of the tile sharding")
    ap.add_argument("--dense-gather", action="store_true",
                    help="tile sharding with a static camera: gather the ranks' whole tile slabs of SHADING instead "
                         "of only the pixels they traced (the moving camera always uses the tile slabs)")
    ap.add_argument("--root-traces", action="store_true",
                    help="tile sharding: the view's compositing rank also traces tiles (default: its tiles go to "
                         "the other ranks, and it runs the G-buffer and the reconstruction half only)")
    ap.add_argument("--composite", action="store_true",
                    help="every frame, gather the views' reconstructed images to rank 0 over RCCL and compose them "
                         "side by side (the final composite of the stereo configuration)")
    ap.add_argument("--bvh", default="host", choices=["host", "gpu"],
                    help="BVH builder: host binned SAH (default) or the GPU LBVH (k_bvh.hip)")
    ap.add_argument("--pan", type=float, default=0.0,
                    help="per-frame step of the camera's look-at target in scene units (0: static camera). A "
                         "moving camera makes the history reprojection read across tiles; tile-sharded views "
                         "then all-gather HISTORY_CACHE every frame")
    args = ap.parse_args()
    args.mask = fovrt.MASKS[args.mask]
    scene = fovrt.SCENES[args.scene]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("FOVRT_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        dist.init_process_group(backend=backend)
    has_gpu = torch.cuda.is_available()

    def sync():
        if has_gpu:
            torch.cuda.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()

    W, H = args.width, args.height
    # one GPU per rank; more ranks than GPUs (the gloo rehearsal on a one-GPU box) share them
    ndev = max(1, torch.cuda.device_count())
    device = local_rank % ndev
    views = args.views or world
    view, vrank, G = view_layout(rank, world, views)
    groups = make_view_groups(dist, world, views) if dist is not None and G > 1 else None
    # the first rank of every view, for the final composite on rank 0
    roots_group = (dist.new_group([v * (world // views) for v in range(views)])
                   if dist is not None and args.composite and views > 1 else None)
    cfg = fovrt.Config(width=W, height=H, scene=scene, mask_mode=args.mask, spp=args.spp, diffuse_max_depth=args.dmd,
                       refraction_max_depth=args.refraction_max_depth, device=device,
                       bvh_builder=1 if args.bvh == "gpu" else 0)
    tracer = fovrt.PathTracer(cfg)
    tracer.initialize()
    cam = fovrt.Camera.preset(scene, W, H)
    # each view is its own eye/camera (offset along x, 6.4 cm per view)
    if views > 1:
        cam.setPosition(np.asarray(cam.pos) + view_offset(view, views))
        cam.lookAt(cam.target)
    tracer.update_optix_variables(cam)

    slab = gather_list = None
    if G > 1:
        # the compositing rank runs the reconstruction half, which no other rank can share (JFA's
        # reach, the global pull-push pyramid): by default it traces no tiles (fr_set_shard_ex)
        first_tracer = 0 if args.root_traces else 1
        tracer.set_shard(vrank, G, args.tile, first_tracer)
        n_tex = tracer.shard_texels()
        slab = torch.empty(n_tex * 4, dtype=torch.float32, device=f"cuda:{device}")
        if vrank == 0:
            gather_list = [torch.empty_like(slab) for _ in range(G)]
        nbytes = n_tex * 16
        root = view * G
        if args.pan:
            hist_slab = torch.empty_like(slab)
            hist_list = [torch.empty_like(slab) for _ in range(G)]
        # sparse gather (static camera): the traced pixels only, 20 B each (fr_shard_pack_active); a rank
        # traces at most its tiles' pixels, so n_tex entries always fit
        sparse = not args.pan and not args.dense_gather
        if sparse:
            act = torch.empty(n_tex * 5, dtype=torch.float32, device=f"cuda:{device}")
            act_list = [torch.empty_like(act) for _ in range(G)] if vrank == 0 else None
            cnt_t = torch.zeros(1, dtype=torch.int64, device=f"cuda:{device}")
            cnt_list = [torch.zeros_like(cnt_t) for _ in range(G)]

    comp_img = comp_list = comp_out = None
    if roots_group is not None and vrank == 0:
        comp_img = torch.empty(W * H * 4, dtype=torch.float32, device=f"cuda:{device}")
        if rank == 0:
            comp_stack = torch.empty(views * W * H * 4, dtype=torch.float32, device=f"cuda:{device}")
            comp_list = list(comp_stack.chunk(views))  # the gather lands the views consecutively
            comp_out = torch.empty_like(comp_stack)

    def composite():
        """Final composite: view roots send their A-Trous image to rank 0, which lays them side by side."""
        if comp_img is None:
            return
        tracer.copy_buffer(fovrt.TextureName.ATROUS, comp_img.data_ptr(), W * H * 16)
        gather_slabs(dist, roots_group, comp_img, comp_list, 0)
        if rank == 0:
            sync()
            tracer.composite_views(comp_list[0].data_ptr(), views, comp_out.data_ptr(), comp_out.numel() * 4)

    def step(timing):
        """One frame of the view: the whole chain on one rank, or trace -> pack -> gather -> (root)
        unpack + reconstruct when the view is tile-sharded; then the optional final composite."""
        if args.pan:
            move_camera()
        tm = view_frame(timing)
        composite()
        return tm

    step_dir = np.array([1.0, 0.5, 0.0], np.float32)
    step_dir *= np.float32(args.pan) / np.linalg.norm(step_dir)

    def move_camera():
        """Camera path of the moving-camera runs: the eye stays, the look-at target moves a fixed step per
        frame (setPrevState first, so frame N reprojects into frame N-1 as FR/main.cpp:357 does)."""
        cam.setPrevState()
        cam.lookAt(np.asarray(cam.target) + step_dir)
        tracer.update_optix_variables(cam)

    def exchange_history():
        """Reprojection reads the previous frame's history anywhere on the screen, so with a moving camera
        every rank of a view needs the others' tiles of HISTORY_CACHE before its next trace."""
        tracer.shard_pack(fovrt.TextureName.HISTORY_CACHE, hist_slab.data_ptr(), nbytes)
        allgather_slabs(dist, groups[view], hist_slab, hist_list)
        sync()
        for r in range(G):
            if r != vrank:
                tracer.shard_unpack(fovrt.TextureName.HISTORY_CACHE, r, hist_list[r].data_ptr(), nbytes)

    def view_frame(timing):
        if G == 1:
            return tracer.frame(timing=timing)
        tm = tracer.trace_frame(timing=timing)
        if args.pan:
            exchange_history()
        sync()  # the previous frame's gather of `slab` has finished on torch's stream
        if sparse:
            cnt_t.fill_(tracer.ray_count())
            allgather_slabs(dist, groups[view], cnt_t, cnt_list)
            counts = [int(c.item()) for c in cnt_list]
            cap = max(max(counts), 1)
            n_packed = tracer.shard_pack_active(act.data_ptr(), cap)
            assert n_packed == counts[vrank]
            gather_slabs(dist, groups[view], act[:cap * 5],
                         [a[:cap * 5] for a in act_list] if act_list is not None else None, root)
            if vrank == 0:
                sync()
                for r in range(1, G):
                    tracer.shard_unpack_active(act_list[r].data_ptr(), cap, counts[r])
        else:
            tracer.shard_pack(fovrt.TextureName.SHADING, slab.data_ptr(), nbytes)
            gather_slabs(dist, groups[view], slab, gather_list, root)
        if vrank == 0:
            sync()
            if not sparse:
                for r in range(1, G):
                    tracer.shard_unpack(fovrt.TextureName.SHADING, r, gather_list[r].data_ptr(), nbytes)
            rec = tracer.reconstruct_frame(timing=timing)
            if timing:
                for k in ("jfa_ms", "sibson_ms", "pullpush_ms", "atrous_ms"):
                    tm[k] = rec[k]
        return tm

    for _ in range(args.warmup):
        step(False)
    tracer.synchronize()
    sync()
    tracer.reset_stats()

    # The timed region: K frames enqueued back to back. fr_frame pipelines them: frame N's
    # reconstruction (JFA/Sibson and pull-push/A-Trous streams) runs while frame N+1 traces.
    # entry 3 (the roofline stage) is timed live inside the timed region: HIP events on the context
    # stream around the stage and its megakernel, recorded by the library, no synchronisation added
    tracer.kernel_timing(True)
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(False)
    tracer.synchronize()
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    live = tracer.kernel_times()
    tracer.kernel_timing(False)

    st = tracer.stats()
    segs, redundant = view_segments(st, G, vrank)
    dev = None
    if dist is not None:
        dev = torch.device("cuda", device) if has_gpu and dist.get_backend() == "nccl" else torch.device("cpu")
    elapsed, total_segs = reduce_over_ranks(dist, dev, elapsed, segs)
    _, total_redundant = reduce_over_ranks(dist, dev, 0.0, redundant)

    # Per-stage HIP-event breakdown of the same frames, serialised (each frame synchronised, so the
    # stage times do not overlap the next frame): the stage table and the roofline kernel time.
    stage_ms = {}
    ray_counts = []
    n_timed = max(3, min(args.steps, 10))
    for _ in range(n_timed):
        tm = step(True)
        for k, v in tm.items():
            if k.endswith("_ms"):
                stage_ms[k] = stage_ms.get(k, 0.0) + v
        ray_counts.append(tm["ray_count"])
    tracer.synchronize()

    K = args.steps
    avg = {k[:-3]: v / n_timed for k, v in stage_ms.items()}
    # foveal density: the active pixels of all ranks of all views (a tile-sharded view's ranks each trace
    # a part; with first_tracer 1 the compositing rank traces none)
    _, count_sum = reduce_over_ranks(dist, dev, 0.0, float(np.mean(ray_counts)))
    rho = count_sum / views / (W * H)
    L = jfa_passes(W, H)
    sb = stage_bytes(W, H, rho, args.spp, L)
    # (a non-compositing rank of a tile-sharded view runs no reconstruction: its image stages are 0 ms)
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
                     "geometry": ["k_gbuffer"], "sibson": ["k_sibson"]}
    image_stages = ["sampling", "optimize", "jfa", "sibson", "pullpush", "atrous"]
    img_bytes = sum(sb[k] for k in image_stages)
    img_ms = sum(avg[k] for k in image_stages)
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
                   "mask_mode": args.mask, "foveal_density": round(rho, 5), "views": views,
                   "composite": bool(args.composite and views > 1), "camera_step": args.pan,
                   "parallelism": (f"views x{world} (one view per GPU)" if G == 1 else
                                   f"{views} view(s) x {G}-way {args.tile}px tile sharding, RCCL gather to the "
                                   f"view's first rank" + ("" if args.root_traces else
                                                          ", which traces no tiles and reconstructs") +
                                   (" (tile slabs of SHADING)" if args.pan or args.dense_gather else
                                    " (only the traced pixels, 20 B each)")),
                   "procedural_meshes": "box/bunny/earth stand-ins (the reference's .obj files are absent)"},
        "fps": round(K / elapsed, 2),
        "frames_per_s_total": round(views * K / elapsed, 2),
        "rays": {k: st[k] for k in ("gbuffer_primary", "primary", "shadow", "diffuse_bounce", "mirror",
                                    "refraction", "reflection", "truncated", "overflow")},
        "rays_note": "rank 0's counters over the timed frames",
        "gbuffer_redundant_segments": int(total_redundant),
        "stages": stage_table,
        "stages_note": f"HIP events, {n_timed} serialised frames; the timed region pipelines frame N's reconstruction "
                       "with frame N+1's trace half, so ms_per_step < the sum of the stages",
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
    traffic, src = load_traffic(stage_kernels.get(dominant, []), result["config"])
    if traffic is not None:
        result["roofline"]["traffic"] = int(traffic)
        result["roofline"]["traffic_source"] = src
        result["roofline"]["measured_hbm_GBs"] = round(traffic / (launch_ms * 1e-3) / 1e9, 1)
    # the GPU BVH builder on this scene (after every measurement: it replaces the BVH)
    builds = sorted(tracer.rebuild_bvh() for _ in range(3))
    result["bvh"] = {"builder": args.bvh, "gpu_rebuild_ms": round(builds[1], 3),
                     "triangles": int(tracer.scene_arrays()["pos"].shape[0])}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            arrays = tracer.scene_arrays()

            def uni_fn(w, h):
                return fovrt.Camera.preset(scene, w, h).uniforms(w, h)
            result["cpu_baseline"] = cpu_baseline(args, arrays, uni_fn)
        except Exception as e:  # report, never fake
            result["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    tracer.destroy()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

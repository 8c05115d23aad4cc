#!/usr/bin/env python3
"""Strong-scaling model of one 4K view tile-sharded over G ranks by fr_group (BASELINE configs[2]-[4]),
from one-GPU measurements of every rank's role.

fr_group's roles in a view of G ranks (include/fovrt.h): view rank 0 runs JumpFlooding -> Sibson, view
rank 1 pull-push -> A-Trous, and the screen tiles are dealt over all ranks by water filling on those
reconstruction loads (fr_group_config.recon_cost, the same rule as group.cpp). Every rank runs the front
stages (a tracer on its own tiles plus halo only, fr_set_front_local) and traces its tiles. On one GPU this script runs each distinct role's work as that rank would:
a context warmed up on whole frames (so its carried history holds the view's seeds, as the gathered pixels
keep it in the group), then switched to the role's tiles and chains, and K pipelined frames timed back to
back (trace half + its reconstruction chain). The frame rate of the view is the slowest role's (the ranks
pipeline against each other; the traced pixels, 20 B each, travel on the comm streams beside compute:
their xGMI time is printed, priced at an assumed link rate, and not on the throughput path unless it
exceeds a rank's frame). Prints one JSON line per G.
  python scripts/shard_model.py [scene=bunny|vokselia] [xgmi_GBs=64]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "foveated-rendering-using-ray-tracing_amd"))
import torch  # noqa: E402,F401
import fovrt  # noqa: E402

def main():
    import torch
    scene_name = sys.argv[1] if len(sys.argv) > 1 else "bunny"
    link = float(sys.argv[2]) if len(sys.argv) > 2 else 64.0
    W, H, T, K = 3840, 2160, 128, 12
    vok = scene_name == "vokselia"
    scene = fovrt.SCENES[scene_name]
    cfg = dict(width=W, height=H, scene=scene, mask_mode=fovrt.MASK_SALIENCY if vok else fovrt.MASK_LOGPOLAR_SIGNED,
               spp=8 if vok else 4, diffuse_max_depth=3)
    cam = fovrt.Camera.preset(scene, W, H)
    t = fovrt.PathTracer(fovrt.Config(**cfg))
    t.initialize()
    t.update_optix_variables(cam)
    # the pixels a reconstruction rank receives from the others: every traced pixel of the frame, packed by a
    # context that owns all tiles (rank 1 of 2, rank 0 empty), 20 B each
    src = fovrt.PathTracer(fovrt.Config(**cfg))
    src.initialize()
    src.update_optix_variables(cam)
    nt = ((W + T - 1) // T) * ((H + T - 1) // T)
    src.set_shard_plan(1, 2, T, np.ones(nt, np.uint8))
    for _ in range(3):
        src.trace_frame(timing=False)
    src.synchronize()
    n_all = src.ray_count()
    slab = torch.empty(n_all * 5, dtype=torch.float32, device="cuda")
    assert src.shard_pack_active(slab.data_ptr(), n_all) == n_all
    src.destroy()

    def pipelined(role_recon, n=K, every=1):
        """ms per frame of K pipelined frames: role_recon None = whole one-GPU frames; else the trace half,
        and (role_recon True) the other ranks' pixels scattered in and the reconstruction chains run on
        every `every`-th frame (a rank taking JFA -> Sibson in turns with others, fr_group jfa_ranks)."""
        state = {"f": 0}

        def one():
            if role_recon is None:
                t.frame(timing=False)
                return
            t.trace_frame(timing=False)
            if role_recon:
                t.shard_unpack_active_enqueue(slab.data_ptr(), n_all, n_all)
                if state["f"] % every == 0:
                    t.reconstruct_frame(timing=False)
            state["f"] += 1
        for _ in range(3 * every):
            one()
        t.synchronize()
        t0 = time.perf_counter()
        for _ in range(n * every):
            one()
        t.synchronize()
        return (time.perf_counter() - t0) / (n * every) * 1e3

    t.set_shard_plan(0, 1, T, np.zeros(1, np.uint8))
    t.set_recon_chains(3)
    one = pipelined(None)
    print(json.dumps({"G": 1, "scene": scene_name, "pipelined_frame_ms": round(one, 4), "fps": round(1e3 / one, 1),
                      "pixels_received_by_recon_ranks": n_all}), flush=True)
    layouts = ((2, 1), (4, 1), (6, 1), (6, 2), (8, 1), (8, 2), (8, 3))
    if os.environ.get("FOVRT_MODEL_LAYOUTS"):  # e.g. "4:1,8:2": only these (G, jfa_ranks)
        layouts = tuple(tuple(int(v) for v in x.split(":")) for x in os.environ["FOVRT_MODEL_LAYOUTS"].split(","))
    # FOVRT_RECON_COST="a,b": the plan's reconstruction costs (fr_group_config.recon_cost; default 0.5, 0.17)
    rc = tuple(float(v) for v in os.environ["FOVRT_RECON_COST"].split(",")) if os.environ.get("FOVRT_RECON_COST") else None
    for G, m in layouts:
        # group.cpp's layout: view rank 0 and ranks 2..m take JFA -> Sibson in turns (cost / m each),
        # view rank 1 pull-push -> A-Trous, the rest trace; tiles by water filling
        jfa = [0] + list(range(2, m + 1))
        owner = fovrt.group_plan(W, H, G, tile=T, jfa_ranks=m, recon_cost=rc)  # the plan fr_group_create deals
        tiles = np.bincount(owner, minlength=G)
        w = (tiles / tiles.sum()).tolist()
        roles = {r: 1 for r in jfa}
        roles[1] = 2
        tracers = [r for r in range(G) if r not in roles]
        if tracers:
            roles[max(tracers, key=lambda r: tiles[r])] = 0
        res = {}
        for r, chains in roles.items():
            t.set_shard_plan(r, G, T, owner)
            t.set_front_local(chains == 0)  # group.cpp: a still camera's tracers run a tile-local front
            t.set_recon_chains(max(chains, 1))
            for form in (1, 2):
                t.set_sample_sum(form)
                ms = pipelined(chains != 0, every=m if chains == 1 else 1)
                res.setdefault(r, {"chains": chains, "tiles": int(tiles[r])})["pipelined_frame_ms_form%d" % form] = round(ms, 4)
            t.set_sample_sum(1)
            st = t.trace_frame(timing=True)
            res[r].update({"active_px": int(st["ray_count"]),
                           "trace_ms": round(st["geometry_ms"] + st["sampling_ms"] + st["optimize_ms"] + st["shading_ms"], 4),
                           "megakernel_ms": round(st["shade_paths_ms"], 4)})
            if chains:
                t.shard_unpack_active_enqueue(slab.data_ptr(), n_all, n_all)
                rt = t.reconstruct_frame(timing=True)
                res[r]["recon_ms"] = round(rt["jfa_ms"] + rt["sibson_ms"] + rt["pullpush_ms"] + rt["atrous_ms"], 4)
        out = {"G": G, "jfa_ranks": m, "scene": scene_name, "weights": [round(x, 3) for x in w], "tiles": tiles.tolist(),
               "roles": res}
        for form in (1, 2):
            frame = max(v["pipelined_frame_ms_form%d" % form] for v in res.values())
            out["model_frame_ms_form%d" % form] = round(frame, 4)
            out["model_fps_form%d" % form] = round(1e3 / frame, 1)
            out["speedup_form%d" % form] = round(one / frame, 3)
        send = max(v["active_px"] for v in res.values()) * 20
        out["max_send_MB"] = round(send / 1e6, 2)
        out["xgmi_ms_at_%gGBs" % link] = round(send / (link * 1e9) * 1e3, 4)
        print(json.dumps(out), flush=True)
    t.destroy()


if __name__ == "__main__":
    main()

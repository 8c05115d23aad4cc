#!/usr/bin/env python3
"""Strong-scaling model of a tile-sharded view (BASELINE configs[3]/[4]) from one-GPU measurements.

A G-rank view with fr_set_shard_ex(first_tracer = 1): ranks 1..G-1 trace the screen tiles round robin, rank 0
computes the G-buffer and sampling (both needed by the reconstruction) and runs the reconstruction half on
the gathered SHADING. On one GPU this measures, per G, the work of one tracing rank (its whole trace half,
timed frames, median) and of the compositing rank (its front stages + the reconstruction half), plus the
slab each tracer sends: its traced pixels, 20 B each (the sparse gather, bench.py's default for a static
camera; the tile slabs of SHADING are reported beside it). The gather over xGMI is not measured here (one GPU): it is priced at an assumed
link rate (each tracer has its own link to the root). Prints one JSON line per G.
  python scripts/shard_model.py [scene=bunny|vokselia] [xgmi_GBs=64]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "foveated-rendering-using-ray-tracing_amd"))
import torch  # noqa: E402,F401
import fovrt  # noqa: E402


def main():
    scene_name = sys.argv[1] if len(sys.argv) > 1 else "bunny"
    link = float(sys.argv[2]) if len(sys.argv) > 2 else 64.0
    W, H = 3840, 2160
    vok = scene_name == "vokselia"
    scene = fovrt.SCENES[scene_name]
    cfg = dict(width=W, height=H, scene=scene, mask_mode=fovrt.MASK_SALIENCY if vok else fovrt.MASK_LOGPOLAR_SIGNED,
               spp=8 if vok else 4, diffuse_max_depth=3)
    K = 7
    t = fovrt.PathTracer(fovrt.Config(**cfg))
    t.initialize()
    t.update_optix_variables(fovrt.Camera.preset(scene, W, H))

    def med(f, key="total_ms"):
        v = []
        for _ in range(K):
            v.append(f()[key])
        return float(np.median(v[2:]))

    # the compositing rank reconstructs the gathered SHADING of the whole view: its cost does not depend
    # on G, so it is measured on a complete frame (its own SHADING after a no-tile trace half would hold
    # only carried history, without the sky's fresh samples: a different, much sparser seed set)
    t.set_shard(0, 1, 128, 0)
    full = med(lambda: t.frame(timing=True))
    recon = med(lambda: t.reconstruct_frame(timing=True))
    print(json.dumps({"G": 1, "scene": scene_name, "frame_ms": round(full, 4), "fps": round(1e3 / full, 1),
                      "recon_ms": round(recon, 4)}))
    for G in (2, 4, 8):
        t.set_shard(1, G, 128, 1)  # one tracing rank
        tr = med(lambda: t.trace_frame(timing=True))
        dense = t.shard_texels() * 16
        slab = t.ray_count() * 20  # the sparse gather (fr_shard_pack_active): the traced pixels only
        t.set_shard(0, G, 128, 1)  # the compositing rank: front stages (G-buffer, sampling), no tiles
        front = med(lambda: t.trace_frame(timing=True))
        gather = slab / (link * 1e9) * 1e3
        # ranks overlap across frames: tracers trace frame N+1 while the root reconstructs frame N
        frame = max(tr + gather, front + gather + recon)
        print(json.dumps({"G": G, "scene": scene_name, "tracer_trace_ms": round(tr, 4), "root_front_ms": round(front, 4),
                          "root_recon_ms": round(recon, 4), "slab_MB_per_tracer": round(slab / 1e6, 2),
                          "dense_slab_MB_per_tracer": round(dense / 1e6, 1),
                          "gather_ms_at_%gGBs" % link: round(gather, 4), "model_frame_ms": round(frame, 4),
                          "model_fps": round(1e3 / frame, 1)}))
    t.destroy()


if __name__ == "__main__":
    main()

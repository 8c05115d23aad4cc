#!/usr/bin/env python3
"""Sibson alone and the JFA disc radii per gaze position of bench.py --gaze-path's cursor circle (4K
bunny, signed log-polar mask): what sets the eye-tracked frame's Sibson time. Usage:
python scripts/gaze_probe.py [angle ...] (default: centred, 0, 1, 2, 45, 90, 180)"""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "foveated-rendering-using-ray-tracing_amd"))
import fovrt

W, H = 3840, 2160
t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=fovrt.SCENE_BUNNY, mask_mode=fovrt.MASK_LOGPOLAR_SIGNED,
                                  spp=4, diffuse_max_depth=3))
t.initialize()
t.update_optix_variables(fovrt.Camera.preset(fovrt.SCENE_BUNNY, W, H))
TN = fovrt.TextureName
si = fovrt.SibsonInterpolation(t)
yy, xx = np.mgrid[0:H, 0:W]
fx, fy = (xx + 0.5) / W, (yy + 0.5) / H
angles = [None if a == "c" else float(a) for a in sys.argv[1:]] or [None, 0, 1, 2, 45, 90, 180]
for ang in angles:
    if ang is None:
        t.reset_gaze()
    else:
        a = np.deg2rad(ang)
        t.set_gaze(W / 2 + 0.25 * H * np.cos(a), (H / 2 + 0.25 * H * np.sin(a)) / 1.25)
    for _ in range(2):
        tm = t.frame(True)
    t.synchronize()
    # (timed before JFA_COORD is read: handing out a JFA output makes Sibson re-derive its seeds and prefix sums)
    ms = np.median([si.render() / 1e6 for _ in range(5)])
    c = t.read(TN.JFA_COORD)
    d = np.sqrt((c[..., 0] - fx) ** 2 + (c[..., 1] - fy) ** 2)
    rows = 2 * d * H
    print(f"gaze {ang}: rays {t.ray_count()} sibson_frame {tm['sibson_ms']:.3f} ms alone {ms:.3f} ms; rows/px mean "
          f"{rows.mean():.2f} p99 {np.percentile(rows, 99):.1f} max {rows.max():.1f}; nonfinite {int((~np.isfinite(d)).sum())}",
          flush=True)
t.destroy()

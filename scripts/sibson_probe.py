#!/usr/bin/env python3
"""Sibson alone at 4K on the bench frame's JFA output, K times (for rocprofv3 counter passes and A/B
timing of the run form): python scripts/sibson_probe.py [K]"""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "foveated-rendering-using-ray-tracing_amd"))
import fovrt

K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
W, H = 3840, 2160
t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=fovrt.SCENE_BUNNY, mask_mode=fovrt.MASK_LOGPOLAR_SIGNED,
                                  spp=4, diffuse_max_depth=3))
t.initialize()
t.update_optix_variables(fovrt.Camera.preset(fovrt.SCENE_BUNNY, W, H))
for _ in range(3):
    t.frame(False)
t.synchronize()
si = fovrt.SibsonInterpolation(t)
ms = [si.render() / 1e6 for _ in range(K)]
print(f"sibson median {np.median(ms):.4f} ms min {np.min(ms):.4f} (K={K})")
t.destroy()

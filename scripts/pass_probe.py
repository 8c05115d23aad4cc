#!/usr/bin/env python3
"""One reconstruction pass alone at 4K on the bench frame's shading, K times (A/B timing of library
variants, FOVRT_LIB=... or an env knob; FR_PASS_DUMP=<file.npy> saves the pass's output): python scripts/pass_probe.py <jfa|sibson|pullpush|atrous> [K]"""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "foveated-rendering-using-ray-tracing_amd"))
import fovrt

name = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
W, H = 3840, 2160
t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=fovrt.SCENE_BUNNY, mask_mode=fovrt.MASK_LOGPOLAR_SIGNED,
                                  spp=4, diffuse_max_depth=3))
t.initialize()
t.update_optix_variables(fovrt.Camera.preset(fovrt.SCENE_BUNNY, W, H))
for _ in range(3):
    t.frame(False)
t.synchronize()
p = {"jfa": fovrt.JumpFlooding, "sibson": fovrt.SibsonInterpolation, "pullpush": fovrt.PullPushInterpolation,
     "atrous": fovrt.ATrous}[name](t)
ms = [p.render() / 1e6 for _ in range(K)]
print(f"{name} median {np.median(ms):.4f} ms min {np.min(ms):.4f} (K={K})")
if os.environ.get("FR_PASS_DUMP"):  # the pass's output, for bit-exact comparisons between variants
    out = {"jfa": fovrt.TextureName.JFA_COLOR, "sibson": fovrt.TextureName.SIBSON,
           "pullpush": fovrt.TextureName.PULLPUSH, "atrous": fovrt.TextureName.ATROUS}[name]
    np.save(os.environ["FR_PASS_DUMP"], t.read(out))
t.destroy()

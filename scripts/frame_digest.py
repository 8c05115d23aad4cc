#!/usr/bin/env python3
"""Digest of a few frames' outputs (SHADING, HISTORY_CACHE, SIBSON, ATROUS) and ray counters: compares library builds
(FOVRT_LIB) that must render identical frames. Usage: python scripts/frame_digest.py [W H spp frames]"""
import hashlib
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "foveated-rendering-using-ray-tracing_amd"))
import fovrt

W, H, spp, frames = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (3840, 2160, 4, 3)))
t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=fovrt.SCENE_BUNNY, mask_mode=fovrt.MASK_LOGPOLAR_SIGNED, spp=spp,
                                  diffuse_max_depth=3))
t.initialize()
cam = fovrt.Camera.preset(fovrt.SCENE_BUNNY, W, H)
TN = fovrt.TextureName
for f in range(frames):
    cam.setPrevState()
    cam.lookAt(np.asarray(cam.target) + np.array([0.01, 0.005, 0.0], np.float32))
    t.update_optix_variables(cam)
    t.frame(timing=False)
out = []
for tid in (TN.SHADING, TN.HISTORY_CACHE, TN.SIBSON, TN.ATROUS):
    out.append(hashlib.sha1(t.read(tid).tobytes()).hexdigest()[:16])
st = t.stats()
print(W, H, spp, frames, " ".join(out), {k: st[k] for k in ("primary", "shadow", "diffuse_bounce", "mirror", "refraction", "reflection")})
t.destroy()

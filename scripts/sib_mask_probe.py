#!/usr/bin/env python3
"""Sibson run form alone at 4K on a log-polar mask whose holes are hundreds of texels wide (the gaze of
tests/test_gpu_parity.py::test_sibson_run_form_offcentre_gaze_4k, or the one given): JFA once, then K timed
Sibson passes. For kernel traces and the FOVRT_SIB_STRIP A/B. Usage: sib_mask_probe.py [K] [gx gy]"""
import os
import sys
import numpy as np
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "foveated-rendering-using-ray-tracing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import fovrt
from helpers import logpolar_mask_np, sparse_image

K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
gx, gy = (float(sys.argv[2]), float(sys.argv[3])) if len(sys.argv) > 3 else (1380, 1080)
W, H = 3840, 2160
TN = fovrt.TextureName
mask = logpolar_mask_np(W, H, gx, gy, signed=True)
img = sparse_image(W, H, mask, seed=11)
t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=fovrt.SCENE_BOX, mask_mode=fovrt.MASK_ALL, spp=1,
                                  diffuse_max_depth=1, texture_mode=1))
t.initialize()
t.write(TN.SHADING, img)
fovrt.JumpFlooding(t).render(TN.SHADING)
coord = t.read(TN.JFA_COORD)
yy, xx = np.mgrid[0:H, 0:W]
d = np.hypot(coord[..., 0] - (xx + 0.5) / W, coord[..., 1] - (yy + 0.5) / H) * H
si = fovrt.SibsonInterpolation(t)
ms = [si.render() / 1e6 for _ in range(K)]
import ctypes as C
cnt = (C.c_uint32 * 3)()
fovrt.load_library().fr__sibson_counts(t._ctx, cnt)
print(f"lists: strips {cnt[0]}, wide[0] {cnt[1]}, wide[1] {cnt[2]}")
big = d > 64
strips = int(np.any(big.reshape(H, -1, 64) if W % 64 == 0 else big, axis=-1).sum())
print(f"mask density {mask.mean():.4f}; disc half-rows mean {d.mean():.1f} max {d.max():.1f}; big pixels "
      f"{big.mean():.3f} (rows {2 * d[big].sum():.3e}), strips with a big pixel {strips}; sibson ms median "
      f"{np.median(ms):.2f} min {np.min(ms):.2f} (strip={os.environ.get('FOVRT_SIB_STRIP', '1')})", flush=True)
t.destroy()

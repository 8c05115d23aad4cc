#!/usr/bin/env python3
"""Each stage of the bench workload alone (synchronous ABI calls, nothing overlapping), median of
K runs: the per-kernel view behind the pipelined bench line. Usage: python scripts/stage_probe.py [K]
(under rocprofv3 --kernel-trace --stats for per-kernel durations)."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "foveated-rendering-using-ray-tracing_amd"))
import fovrt

K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
W, H = 3840, 2160
# FOVRT_PROBE_SCENE=vokselia: configs[4]'s view (8 spp, saliency mask); default: the bench workload
VOK = os.environ.get("FOVRT_PROBE_SCENE") == "vokselia"
scene = fovrt.SCENE_VOKSELIA if VOK else fovrt.SCENE_BUNNY
t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=scene,
                                  mask_mode=fovrt.MASK_SALIENCY if VOK else fovrt.MASK_LOGPOLAR_SIGNED,
                                  spp=8 if VOK else 4, diffuse_max_depth=3))
t.initialize()
t.update_optix_variables(fovrt.Camera.preset(scene, W, H))
for _ in range(3):
    t.frame(False)
t.synchronize()
TN = fovrt.TextureName
jfa, si, pp, at = fovrt.JumpFlooding(t), fovrt.SibsonInterpolation(t), fovrt.PullPushInterpolation(t), fovrt.ATrous(t)
runs = {"geometry": t.geometry_launch, "sampling": t.sampling_launch,  # ms
        "optimize": t.optimize_launch, "shading": t.shading_launch,
        "jfa": lambda: jfa.render(TN.SHADING) / 1e6, "sibson": lambda: si.render() / 1e6,  # ns -> ms
        "pullpush": lambda: pp.render(TN.SHADING) / 1e6,
        "atrous": lambda: at.render(1, TN.POSITION, TN.NORMAL, TN.PULLPUSH) / 1e6}
res = {k: [] for k in runs}
for _ in range(K):
    for k, f in runs.items():
        res[k].append(f())
print(" ".join(f"{k}={np.median(v):.3f}" for k, v in res.items()), "ms (median of", K, ")")
t.destroy()

"""fr_rebuild_bvh wall times: seven rebuilds in a row after a frame, per scene (bunny, vokselia), at 4K.
Usage: rebuild_probe.py [scene ...] (default 1 2)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'foveated-rendering-using-ray-tracing_amd'))
import fovrt
scenes = [int(a) for a in sys.argv[1:]] or [1, 2]
for scene in scenes:
    t = fovrt.PathTracer(fovrt.Config(width=3840, height=2160, scene=scene, mask_mode=4, spp=4, diffuse_max_depth=3))
    t.initialize()
    t.frame(False); t.synchronize()
    ms = [t.rebuild_bvh() for _ in range(7)]
    print("scene", scene, "rebuild ms", [round(m, 3) for m in ms], flush=True)
    t.frame(False); t.synchronize()
    ms = [t.rebuild_bvh() for _ in range(3)]
    print("scene", scene, "after a frame", [round(m, 3) for m in ms], flush=True)
    t.destroy()

import sys, os, time
sys.path.insert(0, 'foveated-rendering-using-ray-tracing_amd')
import fovrt
for scene in (1, 2):
    t = fovrt.PathTracer(fovrt.Config(width=3840, height=2160, scene=scene, mask_mode=4, spp=4, diffuse_max_depth=3))
    t.initialize()
    t.frame(False); t.synchronize()
    ms = [t.rebuild_bvh() for _ in range(7)]
    print("scene", scene, "rebuild ms", [round(m, 3) for m in ms], flush=True)
    t.frame(False); t.synchronize()
    t.destroy()

#!/usr/bin/env python3
"""Probe of the query-stream traversal kernel (k_trace_queries) on the bench workload: records every
query one megakernel launch issues (diagnostic library, FOVRT_LIB=.../libfovrt_diag*.so) and times
k_trace_queries over the recorded stream. Prints one JSON line."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "foveated-rendering-using-ray-tracing_amd"))
import torch  # noqa: E402,F401  (torch's HIP runtime first)
import fovrt  # noqa: E402


def main():
    W, H = 3840, 2160
    t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=1, mask_mode=4, spp=4, diffuse_max_depth=3))
    t.initialize()
    t.update_optix_variables(fovrt.Camera.preset(1, W, H))
    for _ in range(3):
        t.frame(timing=False)
    t.synchronize()
    t.geometry_launch()
    t.sampling_launch()
    t.optimize_launch()
    lib = fovrt.load_library()
    fn = lib.fr_diag_trace_queries
    fn.argtypes = [C.c_void_p, C.POINTER(C.c_float)]
    out = (C.c_float * 8)()
    rc = fn(t._ctx, out)
    assert rc == 0, rc
    n, ms, shadow = out[0], out[1], out[2]
    print(json.dumps({"lib": os.path.basename(os.environ.get("FOVRT_LIB", "default")), "queries": int(n),
                      "shadow": int(shadow), "trace_ms": round(ms, 4), "Mq_per_s": round(n / ms / 1e3, 1),
                      "max_stack": t.scene_arrays()["bvh_max_stack"], "sorted_ms": round(out[3], 4),
                      "closest_only_ms": round(out[4], 4), "shadow_only_ms": round(out[5], 4),
                      "split_ms": round(out[4] + out[5], 4)}))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Host-side cost of enqueuing pipelined frames (bench workload): per fr_frame call, how long the host
spends inside the call. A call that takes about a frame's GPU time means the host is throttled by the
runtime's queues and the frames no longer run ahead. Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "foveated-rendering-using-ray-tracing_amd"))
import torch  # noqa: E402,F401  (torch's HIP runtime first)
import fovrt  # noqa: E402


def main():
    W, H = 3840, 2160
    t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=1, mask_mode=4, spp=4, diffuse_max_depth=3))
    t.initialize()
    t.update_optix_variables(fovrt.Camera.preset(1, W, H))
    for _ in range(5):
        t.frame(timing=False)
    t.synchronize()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    calls = []
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        t.frame(timing=False)
        calls.append((time.perf_counter() - a) * 1e3)
    t_enq = time.perf_counter() - t0
    t.synchronize()
    total = time.perf_counter() - t0
    print(json.dumps({"frames": n, "ms_per_frame": round(total / n * 1e3, 3), "enqueue_ms_total": round(t_enq * 1e3, 2),
                      "call_ms": [round(c, 3) for c in calls],
                      "env": {k: os.environ[k] for k in ("GPU_MAX_HW_QUEUES", "FOVRT_SLOTS") if k in os.environ}}))


if __name__ == "__main__":
    main()

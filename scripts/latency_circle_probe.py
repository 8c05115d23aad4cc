"""The eye-tracked circle (bench.py --gaze-path circle: one degree per frame, 360 frames after 5 warm-up frames)
in one pipeline mode, with the frame clock: latency p50 / p99 / max, wall-clock fps, and the slowest frames with
their gaze angle. Usage: python scripts/latency_circle_probe.py [latency|throughput] [frames]"""
import os
import sys
import time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "foveated-rendering-using-ray-tracing_amd"))
import fovrt

mode = sys.argv[1] if len(sys.argv) > 1 else "latency"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 360
W, H = 3840, 2160
t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=1, mask_mode=4, spp=4, diffuse_max_depth=3))
t.initialize()
t.update_optix_variables(fovrt.Camera.preset(1, W, H))
t.set_pipeline_mode(fovrt.PIPELINE_LATENCY if mode == "latency" else fovrt.PIPELINE_THROUGHPUT)


def gaze(deg):
    a = np.deg2rad(deg)
    t.set_gaze(W / 2 + 0.25 * H * np.cos(a), (H / 2 + 0.25 * H * np.sin(a)) / 1.25)


for f in range(5):
    gaze(f - 5)
    t.frame(timing=False)
t.synchronize()
t.frame_clock(True)
t0 = time.perf_counter()
for f in range(n):
    gaze(f)
    t.frame(timing=False)
t.synchronize()
wall = time.perf_counter() - t0
lat, itv = t.frame_clock_read()
t.frame_clock(False)
order = np.argsort(lat)[::-1][:8]
print(f"{mode} FOVRT_LAT_SIB_MAX={os.environ.get('FOVRT_LAT_SIB_MAX', '1')}: fps {n / wall:.1f} latency p50 "
      f"{np.percentile(lat, 50):.2f} p99 {np.percentile(lat, 99):.2f} max {lat.max():.2f} ms; slowest (deg, ms): "
      + " ".join(f"{int(i)}:{lat[i]:.1f}" for i in order), flush=True)
t.destroy()

"""k_sibson_strip's work at the eye-tracked probe gazes: the strips (64 pixels of a row holding a disc of more than
128 tap rows), their trip counts (the widest disc's tap rows / 4 waves) and a greedy claim over 1024 blocks.
Usage: python scripts/strip_stats.py [angle ...]"""
import heapq
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "foveated-rendering-using-ray-tracing_amd"))
import fovrt

W, H = 3840, 2160
t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=fovrt.SCENE_BUNNY, mask_mode=fovrt.MASK_LOGPOLAR_SIGNED,
                                  spp=4, diffuse_max_depth=3))
t.initialize()
t.update_optix_variables(fovrt.Camera.preset(fovrt.SCENE_BUNNY, W, H))
TN = fovrt.TextureName
yy, xx = np.mgrid[0:H, 0:W]
fx, fy = (xx + 0.5) / W, (yy + 0.5) / H
for ang in [float(a) for a in sys.argv[1:]] or [90.0, 180.0]:
    a = np.deg2rad(ang)
    t.set_gaze(W / 2 + 0.25 * H * np.cos(a), (H / 2 + 0.25 * H * np.sin(a)) / 1.25)
    for _ in range(2):
        t.frame(True)
    t.synchronize()
    c = t.read(TN.JFA_COORD)
    d = np.sqrt((c[..., 0] - fx) ** 2 + (c[..., 1] - fy) ** 2)
    rows = 2 * d * H
    big = d * H > 64
    sid = (yy // 1) * ((W + 63) // 64) + xx // 64
    strip_rows = {}
    for s, r in zip(sid[big], rows[big]):
        strip_rows[s] = max(strip_rows.get(s, 0.0), r)
    its = np.array(sorted(strip_rows.values(), reverse=True)) / 4.0
    lane_eff = rows[big].sum() / max(64.0 * sum(strip_rows.values()), 1.0)  # lane-rows used / lane-rows issued
    # greedy: blocks claim strips in list order (the list is in k_sibson_runs' completion order; take the
    # descending order as the best case and a random order as the typical one)
    def makespan(order, nb=1024):
        h = [0.0] * nb
        for v in order:
            x = heapq.heappop(h); heapq.heappush(h, x + v)
        return max(h)
    rng = np.random.default_rng(0)
    print(f"gaze {ang}: big pixels {int(big.sum())}, strips {len(its)}, iterations per strip max {its.max():.0f} "
          f"mean {its.mean():.1f}, total {its.sum():.0f}; makespan (1024 blocks) desc {makespan(its):.0f} "
          f"random {makespan(rng.permutation(its)):.0f}; mean big-lanes per strip {big.sum() / max(len(its), 1):.1f}; "
          f"lane efficiency {lane_eff:.2f}",
          flush=True)
t.destroy()

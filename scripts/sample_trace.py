#!/usr/bin/env python3
"""Critical path of the path-trace megakernel (diagnostic build, make -C ... diag): one shading launch
with per-sample (queries, traversal steps, start, end) and per-wave (start, refill dry, end) records.
  python scripts/sample_trace.py [W H spp dmd rmd]   -> summary on stdout, gpurun_out/sample_trace_WxH.npz"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FOVRT_LIB", os.path.join(ROOT, "foveated-rendering-using-ray-tracing_amd", "build", "diag",
                                                "libfovrt_diag.so"))
sys.path.insert(0, os.path.join(ROOT, "foveated-rendering-using-ray-tracing_amd"))
import torch  # noqa: E402,F401
import fovrt  # noqa: E402


def main():
    a = [int(x) for x in sys.argv[1:]]
    W, H, spp, dmd, rmd = (a + [3840, 2160, 4, 3, 16][len(a):])[:5]
    t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=fovrt.SCENE_BUNNY, mask_mode=fovrt.MASK_LOGPOLAR_SIGNED,
                                      spp=spp, diffuse_max_depth=dmd, refraction_max_depth=rmd, device=0))
    t.initialize()
    t.update_optix_variables(fovrt.Camera.preset(fovrt.SCENE_BUNNY, W, H))
    for _ in range(3):
        t.frame(timing=False)
    # a tile-sharded tracer's launch (FR_TRACE_G ranks, view rank FR_TRACE_RANK, the group's plan with one JFA
    # rank) in the sample-sum form FR_TRACE_FORM (the group default 2)
    G = int(os.environ.get("FR_TRACE_G", "1"))
    if G > 1:
        owner = fovrt.group_plan(W, H, G)
        t.set_shard_plan(int(os.environ.get("FR_TRACE_RANK", "2")), G, 128, owner)
        t.set_sample_sum(int(os.environ.get("FR_TRACE_FORM", "2")))
        t.set_recon_chains(1)
        for _ in range(3):
            t.trace_frame(timing=False)
        t.synchronize()
    t.synchronize()
    t.geometry_launch()
    t.sampling_launch()
    t.optimize_launch()
    n = t.ray_count() * spp
    wcap = 256 * 12
    srec = np.zeros((n, 4), np.uint32)
    wrec = np.zeros((wcap, 4), np.uint32)
    lib = fovrt.load_library()
    fn = lib.fr_diag_sample_trace
    fn.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]
    rc = fn(t._ctx, srec.ctypes.data, n, wrec.ctypes.data, wcap)
    assert rc == 0, rc
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"sample_trace_{W}x{H}_spp{spp}_dmd{dmd}_rmd{rmd}.npz"),
                        srec=srec, wrec=wrec)
    w = wrec[wrec[:, 2] != 0].astype(np.int64)
    t0 = w[:, 0].min()
    us = 0.01  # s_memrealtime: 100 MHz
    print(f"{W}x{H} spp {spp} dmd {dmd} rmd {rmd}: {n} samples, {len(w)} waves")
    print(f"  kernel span {(w[:, 2].max() - t0) * us:.0f} us; refill dry: first {(w[:, 1].min() - t0) * us:.0f}, "
          f"median {(np.median(w[:, 1]) - t0) * us:.0f}, last {(w[:, 1].max() - t0) * us:.0f} us; wave end: median "
          f"{(np.median(w[:, 2]) - t0) * us:.0f}, p90 {(np.percentile(w[:, 2], 90) - t0) * us:.0f}, p99 "
          f"{(np.percentile(w[:, 2], 99) - t0) * us:.0f}")
    s = srec.astype(np.int64)
    dur = (s[:, 3] - s[:, 2]) * us
    st = (s[:, 2] - t0) * us
    en = (s[:, 3] - t0) * us
    for name, v in (("queries", s[:, 0]), ("steps", s[:, 1]), ("duration us", dur)):
        print(f"  {name:12s} mean {v.mean():8.1f}  p50 {np.percentile(v, 50):8.1f}  p90 {np.percentile(v, 90):8.1f}  "
              f"p99 {np.percentile(v, 99):8.1f}  p99.9 {np.percentile(v, 99.9):8.1f}  max {v.max():8.1f}")
    order = np.argsort(-en)[:12]
    print("  last-finishing samples: slot, queries, steps, start us, end us")
    for i in order:
        print(f"    {i:8d} {s[i, 0]:5d} {s[i, 1]:6d} {st[i]:8.0f} {en[i]:8.0f}")
    for q in (10, 20, 40, 80):
        sel = s[:, 0] >= q
        print(f"  samples with >= {q} queries: {sel.sum()}, mean steps {s[sel, 1].mean() if sel.any() else 0:.0f}, "
              f"mean duration {dur[sel].mean() if sel.any() else 0:.0f} us")
    print(f"  steps per query overall {s[:, 1].sum() / s[:, 0].sum():.1f}")
    t.destroy()


if __name__ == "__main__":
    main()

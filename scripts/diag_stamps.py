#!/usr/bin/env python3
"""Phase shares of the path-trace megakernel from the -DFR_STAMPS diagnostic build
(make -C foveated-rendering-using-ray-tracing_amd diag). Wave-level s_memtime sums:
diag = [total, refill, shade, traversal, node visits, wave traversal steps]. Shares only; the stamped build's run time is not a
measurement."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FOVRT_LIB", os.path.join(ROOT, "foveated-rendering-using-ray-tracing_amd", "build", "diag",
                                                "libfovrt_diag.so"))
sys.path.insert(0, os.path.join(ROOT, "foveated-rendering-using-ray-tracing_amd"))
import fovrt  # noqa: E402


def main():
    W, H = int(sys.argv[1]) if len(sys.argv) > 1 else 3840, int(sys.argv[2]) if len(sys.argv) > 2 else 2160
    dmd = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=fovrt.SCENE_BUNNY, mask_mode=fovrt.MASK_LOGPOLAR_SIGNED,
                                      spp=4, diffuse_max_depth=dmd, device=0))
    t.initialize()
    t.update_optix_variables(fovrt.Camera.preset(fovrt.SCENE_BUNNY, W, H))
    for _ in range(3):
        t.frame(timing=False)
    t.synchronize()
    t.reset_stats()
    for _ in range(5):
        tm = t.frame(timing=True)
    st = t.stats()
    total, refill, step, trav, visits, wsteps = st["diag"]
    print(f"{W}x{H} dmd {dmd}: megakernel {tm['shade_paths_ms']:.3f} ms (stamped build)")
    print(f"  refill {refill / total:.3f}  traversal {trav / total:.3f}  shading {step / total:.3f}  "
          f"other {(total - refill - step - trav) / total:.3f}")
    segs = st["primary"] + st["shadow"] + st["diffuse_bounce"] + st["mirror"] + st["refraction"] + st["reflection"]
    print(f"  node visits {visits / 5 / 1e6:.1f} M/frame, {visits / segs:.1f} per segment; wave traversal steps "
          f"{wsteps / 5 / 1e6:.2f} M/frame -> lane utilisation of the traversal loop {visits / (64 * wsteps):.2f}")
    t.destroy()


if __name__ == "__main__":
    main()

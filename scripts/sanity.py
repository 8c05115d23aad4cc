"""Quick GPU sanity run: renders a few frames of a preset and dumps stats + PPM previews."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "foveated-rendering-using-ray-tracing_amd"))
import numpy as np
import fovrt

def save_ppm(path, img):
    a = np.clip(np.nan_to_num(img[::-1, :, :3]) * 255.0, 0, 255).astype(np.uint8)
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (a.shape[1], a.shape[0]))
        f.write(a.tobytes())

def main():
    W, H = int(sys.argv[1]), int(sys.argv[2])
    scene = fovrt.SCENES[sys.argv[3]] if len(sys.argv) > 3 else fovrt.SCENE_BUNNY
    mask = fovrt.MASKS[sys.argv[4]] if len(sys.argv) > 4 else fovrt.MASK_LOGPOLAR
    spp = int(sys.argv[5]) if len(sys.argv) > 5 else 4
    out = os.environ.get("OUT", "gpurun_out")
    os.makedirs(out, exist_ok=True)
    t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=scene, mask_mode=mask, spp=spp, diffuse_max_depth=3))
    t0 = time.time(); t.initialize(); print("init s", time.time() - t0, flush=True)
    cam = fovrt.Camera.preset(scene, W, H)
    t.update_optix_variables(cam)
    for i in range(6):
        tm = t.frame(timing=True)
        print("frame", i, {k: round(v, 3) for k, v in tm.items()}, flush=True)
    print("stats", t.stats())
    for name, b in [("shading", fovrt.TextureName.SHADING), ("diffuse", fovrt.TextureName.DIFFUSE),
                    ("pullpush", fovrt.TextureName.PULLPUSH), ("atrous", fovrt.TextureName.ATROUS),
                    ("sibson", fovrt.TextureName.SIBSON)]:
        img = t.read(b)
        print(name, "mean", np.nanmean(img[..., :3], axis=(0, 1)), "nan", int(np.isnan(img).sum()))
        save_ppm(os.path.join(out, f"{name}.ppm"), img)

if __name__ == "__main__":
    main()

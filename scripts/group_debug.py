#!/usr/bin/env python3
"""A group frame's tracer tiles against the single-context frame, per rank: how many own pixels of SHADING /
HISTORY_CACHE / MASK / WEIGHT differ and by how much (the C4 / C5 group shapes of tests/test_gpu_parity.py and
variations). Usage: group_debug.py R V scene spp dmd [frames] [sample_sum]"""
import os
import sys
import numpy as np
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "foveated-rendering-using-ray-tracing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import fovrt
from helpers import ASSET_DIR, TEXTURE_MODE

R, V, scene, spp, dmd = (int(a) for a in sys.argv[1:6])
frames = int(sys.argv[6]) if len(sys.argv) > 6 else 4
ssum = int(sys.argv[7]) if len(sys.argv) > 7 else 2
W, H, tile, mask = 3840, 2160, 128, 0
G = R // V
TN = fovrt.TextureName


def mk():
    t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=scene, mask_mode=mask, spp=spp, diffuse_max_depth=dmd,
                                      refraction_max_depth=16, texture_mode=TEXTURE_MODE, asset_dir=ASSET_DIR))
    assert t.initialize()
    return t


ranks = [mk() for _ in range(R)]
fulls = [mk() for _ in range(V)]
if G > 1:
    for f in fulls:
        f.set_sample_sum(ssum)
cams = []
for v in range(V):
    cam = fovrt.Camera.preset(scene, W, H)
    cam.setPosition(np.asarray(cam.pos) + np.array([0.064 * (v - (V - 1) / 2), 0, 0], np.float32))
    cam.lookAt(cam.target)
    cams.append(cam)
g = fovrt.Group(ranks, views=V, tile=tile, split_recon=True, moving_camera=False, composite=True, jfa_ranks=0)
info = [g.rank_info(i) for i in range(R)]
for f in range(frames):
    for v in range(V):
        fulls[v].update_optix_variables(cams[v])
        for r in range(v * G, (v + 1) * G):
            ranks[r].update_optix_variables(cams[v])
        fulls[v].frame(timing=False)
    g.frame(timing=False)
    g.synchronize()
    owners = g.tile_owners(W, H)
    own_px = np.repeat(np.repeat(owners, tile, 0), tile, 1)[:H, :W]
    for v in range(V):
        for r in range(v * G, (v + 1) * G):
            if info[r]["chains"]:
                sel = np.ones((H, W), bool)
            else:
                sel = own_px == r - v * G
            out = []
            for name in ("SHADING", "HISTORY_CACHE", "MASK", "WEIGHT", "POSITION", "EXTRA"):
                tid = getattr(TN, name)
                a, b = ranks[r].read(tid)[sel], fulls[v].read(tid)[sel]
                a = a.reshape(a.shape[0], -1).astype(np.float64)
                b = b.reshape(b.shape[0], -1).astype(np.float64)
                bad = ~((a == b) | (np.isnan(a) & np.isnan(b))).all(axis=1)
                err = np.nanmax(np.abs(a - b)) if bad.any() else 0.0
                out.append(f"{name} {int(bad.sum())}/{sel.sum()} {err:.3g}")
                if name in ("SHADING", "HISTORY_CACHE") and 0 < bad.sum() <= 4:
                    ys, xs = np.nonzero(sel)
                    for i in np.flatnonzero(bad):
                        print(f"   {name} pixel ({xs[i]}, {ys[i]}) group {a[i].tolist()} single {b[i].tolist()}", flush=True)
            print(f"frame {f} view {v} rank {r} chains {info[r]['chains']}: " + "; ".join(out), flush=True)

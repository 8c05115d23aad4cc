"""Regenerates the committed golden vectors in tests/golden/ from the CPU oracle.

The reference has no fixtures of its own, so these vectors are the oracle's output
on fixed synthetic inputs; tests/test_cpu_oracle.py re-derives several of them from independent
numpy / pure-Python restatements, and the GPU tests hold the HIP kernels to them.
Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import pyoracle as po  # noqa: E402
from helpers import logpolar_mask_np, sparse_image  # noqa: E402


def main():
    rng = np.random.default_rng(20180920)
    # known answers
    tea_in = np.array([[0, 0], [1, 0], [12345, 7], [0xFFFFFFFF, 0xFFFFFFFF], [3840 * 1080 + 1920, 41]], np.uint64)
    tea_out = np.array([po.tea16(int(a), int(b)) for a, b in tea_in], np.uint64)
    tm_in = np.array([[0, 0.1, 1], [10, 0.5, 2], [100, 1e-3, 3.3]], np.float32)
    np.savez_compressed(os.path.join(HERE, "kat.npz"), tea_in=tea_in, tea_out=tea_out, rnd_seed=np.uint64(0xDEADBEEF),
                        rnd_out=po.rnd_seq(0xDEADBEEF, 32), tm_in=tm_in, tm_out=po.tonemap(tm_in))
    # JFA + Sibson on a log-polar-masked 64x48 image (gaze = screen centre)
    W, H = 64, 48
    mask = logpolar_mask_np(W, H, W // 2, H - H // 2)
    img = sparse_image(W, H, mask, seed=1)
    coord, color = po.jfa(img)
    np.savez_compressed(os.path.join(HERE, "jfa_64x48.npz"), input=img, coord=coord, color=color)
    np.savez_compressed(os.path.join(HERE, "sibson_64x48.npz"), coord=coord, color=color, output=po.sibson(coord, color))
    # pull-push: three frames through the same atlases (cross-frame state)
    inputs = np.stack([sparse_image(64, 64, (rng.random((64, 64)) < p).astype(np.uint8), seed=k)
                       for k, p in enumerate((0.1, 0.02, 0.25))])
    st = po.PullPushState(64, 64)
    outputs = np.stack([st.render(x) for x in inputs])
    np.savez_compressed(os.path.join(HERE, "pullpush_64.npz"), inputs=inputs, outputs=outputs)
    # A-Trous, two iterations
    pos = rng.random((32, 32, 4), dtype=np.float32)
    nrm = rng.random((32, 32, 4), dtype=np.float32)
    col = rng.random((32, 32, 4), dtype=np.float32)
    np.savez_compressed(os.path.join(HERE, "atrous_32.npz"), pos=pos, nrm=nrm, col=col, count=np.int32(2),
                        output=po.atrous(2, pos, nrm, col))
    # log-polar mask at 512x512
    np.savez_compressed(os.path.join(HERE, "logpolar_512.npz"), gaze=np.array([256.0, 256.0], np.float32),
                        mask=logpolar_mask_np(512, 512, 256, 256))
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main()

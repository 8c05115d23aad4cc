"""World-size-2 gloo rehearsal of bench.py's multi-GPU path (one process per GPU, weak scaling over
views): per-rank view offsets and the max-time / sum-of-rays reduction over ranks."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    elapsed = 1.0 + rank  # rank 1 is the slow one
    segs = 1000 * (rank + 1)
    t, s = bench.reduce_over_ranks(dist, torch.device("cpu"), elapsed, segs)
    q.put((rank, t, s, bench.view_offset(rank, world).tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_reduce_over_ranks_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, t, s, off in out:
        assert t == pytest.approx(2.0)     # max over ranks
        assert s == pytest.approx(3000.0)  # all ranks' ray segments
    offs = np.array([o for _, _, _, o in out])
    assert np.allclose(offs[0], -offs[1]) and offs[1][0] > 0  # symmetric stereo pair


def test_single_process_passthrough():
    import bench
    assert bench.reduce_over_ranks(None, None, 1.5, 7) == (1.5, 7.0)
    assert np.allclose(bench.view_offset(0, 1), 0)

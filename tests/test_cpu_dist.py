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


def _tile_worker(rank, world, views, port, q):
    import torch
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    view, vrank, g = bench.view_layout(rank, world, views)
    groups = bench.make_view_groups(dist, world, views)
    slab = torch.full((8,), float(rank))
    gl = [torch.empty_like(slab) for _ in range(g)] if vrank == 0 else None
    bench.gather_slabs(dist, groups[view], slab, gl, view * g)
    al = [torch.empty_like(slab) for _ in range(g)]  # the moving-camera history exchange
    bench.allgather_slabs(dist, groups[view], slab, al)
    q.put((rank, view, vrank, g, None if gl is None else [float(t[0]) for t in gl], [float(t[0]) for t in al]))
    dist.barrier()
    dist.destroy_process_group()


def test_tile_gather_groups_gloo_world4():
    """4 ranks, 2 views (the stereo layout of BASELINE configs[4] at half size): each view's 2 ranks
    gather their slabs to the view's first rank, and all-gather them within the view."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tile_worker, args=(r, 4, 2, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    out = {r: rest for r, *rest in (q.get(timeout=120) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0][:4] == [0, 0, 2, [0.0, 1.0]] and out[2][:4] == [1, 0, 2, [2.0, 3.0]]
    assert out[1][3] is None and out[3][3] is None
    assert out[0][4] == out[1][4] == [0.0, 1.0] and out[2][4] == out[3][4] == [2.0, 3.0]


def test_view_layout():
    import bench
    assert bench.view_layout(5, 8, 0) == (5, 0, 1)   # default: one view per rank
    assert bench.view_layout(5, 8, 2) == (1, 1, 4)   # stereo, 4-way tiles per eye
    assert bench.view_layout(3, 4, 1) == (0, 3, 4)   # one view tiled over 4 ranks
    with pytest.raises(SystemExit):
        bench.view_layout(0, 6, 4)


def test_view_segments_count_the_gbuffer_once_per_view():
    """Tile sharding: every rank of a view traces the full G-buffer; value counts it once (vrank 0)."""
    import bench
    st = {"segments": 1000, "gbuffer_primary": 600}
    assert bench.view_segments(st, 1, 0) == (1000, 0)     # one view per rank: everything counts
    assert bench.view_segments(st, 4, 0) == (1000, 0)     # the view's first rank keeps its G-buffer
    assert bench.view_segments(st, 4, 3) == (400, 600)    # the others' copies are redundant work
    W, H, G = 64, 32, 4                                   # summed over a view: W*H primaries once
    ranks = [{"segments": W * H + 10 * r, "gbuffer_primary": W * H} for r in range(G)]
    total = sum(bench.view_segments(s, G, r)[0] for r, s in enumerate(ranks))
    assert total == W * H + sum(10 * r for r in range(G))

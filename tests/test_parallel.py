"""View sharding and the cloud gather (the only exchange step), world_size 2 on gloo.

Each rank runs the oracle on the views shard_views gives it (stand-in for the
GPU path, whose per-view parity the GPU tests prove) and gather_cloud must
rebuild exactly the serial merged cloud, in view order.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from structured_light_for_3d_model_replication_amd import parallel, synth


@pytest.mark.parametrize("V,G", [(1, 1), (5, 2), (36, 8), (3, 8), (8, 8), (0, 3)])
def test_shard_views_partition(V, G):
    shards = [parallel.shard_views(V, G, r) for r in range(G)]
    assert [v for s in shards for v in s] == list(range(V))
    sizes = [len(s) for s in shards]
    assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        parallel.shard_views(V, G, G)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _views(V):
    rig = synth.Rig(H=24, W=32, Wp=16, Hp=8)
    calib = synth.make_calibration(rig, with_Nc=False)
    out = []
    for v in range(V):
        s, t = synth.render_stack(rig, seed=v, include_rows=False, view_deg=40.0 * v, device="cpu")
        out.append((s.numpy(), t.numpy(), synth.turntable_pose(40.0 * v)))
    return calib, out


def _worker(rank, world, port, V, q):
    from oracle import sl_oracle as o
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calib, views = _views(V)
        xs, cs = [], []
        for v in parallel.shard_views(V, world, rank):
            s, t, pose = views[v]
            P, C = o.decode_triangulate(list(s), t, calib, 16, 8, pose=pose)[3:]
            xs.append(P)
            cs.append(C)
        xyz = torch.from_numpy(np.concatenate(xs) if xs else np.zeros((0, 3)))
        bgr = torch.from_numpy(np.concatenate(cs) if cs else np.zeros((0, 3), np.uint8))
        xa, ca, counts = parallel.gather_cloud(xyz, bgr, dst=0)
        if rank == 0:
            q.put((xa.numpy(), ca.numpy(), counts))
        else:
            assert xa is None and ca is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("V", [3, 1])
def test_gather_cloud_gloo_world2(V):
    from oracle import sl_oracle as o
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, V, q)) for r in range(2)]
    for p in procs:
        p.start()
    xa, ca, counts = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    calib, views = _views(V)
    ref = [o.decode_triangulate(list(s), t, calib, 16, 8, pose=pose)[3:] for s, t, pose in views]
    np.testing.assert_array_equal(xa, np.concatenate([r[0] for r in ref]))
    np.testing.assert_array_equal(ca, np.concatenate([r[1] for r in ref]))
    assert sum(counts) == xa.shape[0] and xa.shape[0] > 0


def _sub_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # ranks 1 and 2 of a 3-rank world form the group; group ranks 0, 1
        sub = dist.new_group([1, 2])
        if rank in (1, 2):
            n = 3 + rank
            xyz = torch.full((n, 3), float(rank), dtype=torch.float64)
            bgr = torch.full((n, 3), rank, dtype=torch.uint8)
            xa, ca, counts = parallel.gather_cloud(xyz, bgr, dst=0, group=sub)
            if rank == 1:  # group rank 0 = global rank 1
                q.put((xa.numpy(), ca.numpy(), counts))
            else:
                assert xa is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gather_cloud_on_a_subgroup():
    """gather_cloud over a 2-rank subgroup of a 3-rank world: group ranks are
    mapped to global peers (dst = group rank 0 = global rank 1)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sub_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    xa, ca, counts = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert counts == [4, 5]
    np.testing.assert_array_equal(xa[:, 0], [1.0] * 4 + [2.0] * 5)
    np.testing.assert_array_equal(ca[:, 0], [1] * 4 + [2] * 5)

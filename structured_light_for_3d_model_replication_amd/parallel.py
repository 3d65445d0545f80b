"""Multi-GPU turntable scans: views sharded over ranks, one gather at the end.

Views are independent, so each rank decodes + triangulates its contiguous block
of views with no communication (view v -> rank floor(v*G/V), rank-order
concatenation == view order).  The only exchange is the final cloud gather
for the merge (the reference merges per-view PLY files sequentially,
server/processing.py:116-182):

1. all_gather of the per-rank point counts (int64),
2. point-to-point send/recv of each rank's xyz and colour payload straight
   into the destination's merged buffer at exclusive-scan offsets.  RCCL has no
   gatherv and a ring all-gather would push every payload over every link;
   on xGMI each sender uses its own direct link to the destination.

Backend-agnostic torch.distributed: "nccl" (= RCCL over xGMI) on the GPU box,
"gloo" for the CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_views(n_views: int, world: int, rank: int) -> range:
    """Contiguous block of views owned by ``rank`` (view v -> rank floor(v*G/V))."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    lo = -(-rank * n_views // world)            # ceil(rank*V/G)
    hi = -(-(rank + 1) * n_views // world)
    return range(lo, hi)


def gather_counts(n_local: int, device, group=None) -> list[int]:
    world = dist.get_world_size(group)
    mine = torch.tensor([int(n_local)], dtype=torch.int64, device=device)
    outs = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(outs, mine, group=group)
    return [int(t.item()) for t in outs]


def gather_cloud(xyz: torch.Tensor, bgr: torch.Tensor, dst: int = 0, group=None):
    """Gather every rank's (xyz [n,3], bgr [n,3]) to ``dst`` in rank order.

    Returns ``(xyz_all, bgr_all, counts)`` on ``dst`` and ``(None, None, counts)``
    elsewhere.  Payloads move rank -> dst directly (batched isend/irecv).
    ``dst`` and the ranks are those of ``group`` (default: the world).
    """
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    xyz = xyz.contiguous()
    bgr = bgr.contiguous()
    counts = gather_counts(xyz.shape[0], xyz.device, group)

    def peer(r):  # P2POp peers are global ranks; r and dst are ranks of `group`
        return r if group is None else dist.get_global_rank(group, r)
    if world == 1:
        return xyz, bgr, counts
    ops = []
    if rank == dst:
        total = sum(counts)
        xyz_all = torch.empty((total, 3), dtype=xyz.dtype, device=xyz.device)
        bgr_all = torch.empty((total, 3), dtype=bgr.dtype, device=bgr.device)
        off = 0
        for r in range(world):
            n = counts[r]
            if r == rank:
                xyz_all[off:off + n].copy_(xyz)
                bgr_all[off:off + n].copy_(bgr)
            elif n:
                ops.append(dist.P2POp(dist.irecv, xyz_all[off:off + n], peer(r), group))
                ops.append(dist.P2POp(dist.irecv, bgr_all[off:off + n], peer(r), group))
            off += n
    elif counts[rank]:
        ops.append(dist.P2POp(dist.isend, xyz, peer(dst), group))
        ops.append(dist.P2POp(dist.isend, bgr, peer(dst), group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if rank == dst:
        return xyz_all, bgr_all, counts
    return None, None, counts


def gather_cloud_native(engine, xyz: torch.Tensor, bgr: torch.Tensor, dst: int = 0, group=None):
    """gather_cloud through the library's own RCCL communicator (sl_gather,
    include/slgpu.h) instead of torch.distributed's: rank 0 of ``group`` makes
    the RCCL unique id, torch.distributed shares it once per engine, then
    counts and payloads move as in gather_cloud.  Same result and order."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    key = (world, rank, id(group))
    if getattr(engine, "_gather_key", None) != key:
        uid = [engine.gather_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                   group=group)
        engine.gather_init(world, rank, uid[0])
        engine._gather_key = key
    return engine.gather(xyz, bgr, root=dst)

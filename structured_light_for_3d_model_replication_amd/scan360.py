"""Multi-GPU turntable scan: view folders sharded over the ranks of one node,
one RCCL gather for the merge.

The reference processes the views of a scan one after another
(multi_point_cloud_process.py:241-257) and merges their PLY files on one host
(server/processing.py:116-182).  Here every rank (one process per GPU, launched
by ``torch.distributed.run``) takes its contiguous block of view folders
(``parallel.shard_views``: view v -> rank floor(v*G/V)), decodes and
triangulates them on its GPU with the batch module's streamed pipeline
(per-view PLY files written by the owning rank, as the reference writes them,
unless ``write_views=False``: the points then never leave HBM and the turntable
pose is applied inside k_cloud), and the merged cloud -- float32 xyz by
default, f64 on request -- is gathered to rank 0 in view order over RCCL
(``parallel.gather_cloud``: counts all-gathered, payloads point to point; or
the C-ABI ``sl_gather`` with ``native_gather``).  Rank 0 optionally runs the
merge post-processing of processing.py:171-175 (voxel downsample + statistical
outlier removal, merge.py), estimates the normals (:178) and writes the
merged PLY in Open3D's layout.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m structured_light_for_3d_model_replication_amd.scan360 SCAN_DIR calib.mat \\
        [--poses poses.npy] [--merge merged.ply --voxel 1.0]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

from . import parallel


def _gpu_views(views, calib_data, poses, *, n_cols, n_rows, device, write, log, xyz_dtype=torch.float32):
    """Default per-rank work: the batch module's streamed GPU pipeline on this
    rank's folders -> [(P, C)] device tensors (``xyz_dtype`` xyz, u8 BGR) in
    folder order.  The clouds stay in HBM: each view's points are copied from
    its pipeline slot into a device tensor of its own.

    ``write=False``: the pose is applied inside k_cloud (decode_triangulate's
    f64 epilogue, rounded once to ``xyz_dtype``) and no point crosses PCIe.
    ``write=True``: the per-view PLY files hold the camera-frame cloud, as the
    reference writes them (multi_point_cloud_process.py:205-213), so the views
    are triangulated in f64 without pose, written from the host copy, and
    moved by their pose on the device (sl_transform_points, the same
    ((m0 x + m1 y) + m2 z) + m3 arithmetic as the k_cloud epilogue) before the
    cast to ``xyz_dtype``: both modes give the same bits."""
    from . import merge, multi_point_cloud_process as mpp
    pose_of = dict(zip(views, poses))
    have_poses = any(M is not None for M in poses)
    if have_poses and not all(M is not None for M in poses):
        raise ValueError("poses must be given for every view or for none")
    parts = {}

    def sink(f, xyz, bgr):
        M = pose_of[f]
        if write and M is not None:
            xyz = merge.transform(xyz, M, device=xyz.device)
        parts[f] = (xyz.to(xyz_dtype, copy=True), bgr.clone())

    mpp._process_streamed(views, calib_data, n_cols, n_rows, device, write, log, 3, False,
                          xyz_dtype=torch.float64 if write else xyz_dtype,
                          poses=pose_of if have_poses and not write else None, device_sink=sink, host=write)
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    torch.cuda.synchronize(dev)
    empty = (torch.zeros((0, 3), dtype=xyz_dtype, device=dev), torch.zeros((0, 3), dtype=torch.uint8, device=dev))
    return [parts.get(f, empty) for f in views]


def scan_distributed(parent_dir, calib_data, *, poses=None, n_cols=1920, n_rows=1080, voxel_size=None,
                     nb_neighbors=20, std_ratio=2.0, merge_output=None, write_views=True, device=None,
                     group=None, log=print, process=None, xyz_dtype=torch.float32, native_gather=False):
    """One multi-GPU scan; every rank of ``group`` calls it with the same
    arguments.  ``poses``: optional per-view 4x4 (sorted folder order).
    Returns ``(P, C, counts)`` on rank 0 -- the merged (and, with
    ``voxel_size``, post-processed) cloud and the points per rank -- and
    ``(None, None, counts)`` elsewhere.  ``process(views, calib, poses)``
    replaces the per-rank GPU work (tests).

    ``xyz_dtype``: the gathered coordinates, float32 by default (12 B/point
    over xGMI: the correctly rounded float32 of the reference's f64 point) or
    torch.float64 on request (bit-identical to the reference's f64).  The merge
    post-processing runs in f64 on whichever was gathered.  ``native_gather``:
    gather through the library's own RCCL communicator (sl_gather) instead of
    torch.distributed's."""
    from .multi_point_cloud_process import view_folders
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    views = view_folders(parent_dir, log if rank == 0 else (lambda *a, **k: None))
    if poses is not None:
        poses = np.asarray(poses, dtype=np.float64).reshape(-1, 4, 4)
        if len(poses) != len(views):
            raise ValueError(f"{len(views)} views but {len(poses)} poses")
    mine = list(parallel.shard_views(len(views), world, rank))
    my_views = [views[v] for v in mine]
    my_poses = [poses[v] if poses is not None else None for v in mine]
    if process is None:
        parts = _gpu_views(my_views, calib_data, my_poses, n_cols=n_cols, n_rows=n_rows, device=device,
                           write=write_views, log=log, xyz_dtype=xyz_dtype)
    else:
        parts = process(my_views, calib_data, my_poses)
    if parts:
        xyz = torch.cat([p for p, _ in parts])
        bgr = torch.cat([c for _, c in parts])
    else:
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
        xyz = torch.zeros((0, 3), dtype=xyz_dtype, device=dev)
        bgr = torch.zeros((0, 3), dtype=torch.uint8, device=dev)
    if native_gather:
        from . import core
        P, C, counts = parallel.gather_cloud_native(core.engine(xyz.device), xyz, bgr, dst=0, group=group)
    else:
        P, C, counts = parallel.gather_cloud(xyz, bgr, dst=0, group=group)
    if rank != 0:
        return None, None, counts
    N = None
    if voxel_size:
        from . import merge
        P, C = merge.postprocess(P, C, voxel_size, nb_neighbors, std_ratio, device=P.device)
        if merge_output:  # processing.py:178
            N = merge.estimate_normals(P, voxel_size * 2, 30, device=P.device)
    if merge_output:
        from . import ply
        ply.save_ply_open3d(P.cpu().numpy(), C.cpu().numpy(), merge_output,
                            normals=None if N is None else N.cpu().numpy())
        log(f"[scan360] merged {sum(counts)} points from {len(views)} views on {world} GPU(s) -> "
            f"{len(P)} points, {merge_output}")
    return P, C, counts


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("scan_dir")
    ap.add_argument("calib_file")
    ap.add_argument("--poses", help=".npy of per-view 4x4 poses (sorted folder order)")
    ap.add_argument("--merge", dest="merge_output", help="merged PLY (binary) written by rank 0")
    ap.add_argument("--voxel", type=float, default=None, help="voxel size of the merge post-processing")
    ap.add_argument("--n-cols", type=int, default=1920)
    ap.add_argument("--n-rows", type=int, default=1080)
    ap.add_argument("--no-view-ply", action="store_true",
                    help="do not write per-view PLY files (the clouds then never leave HBM before the gather)")
    ap.add_argument("--f64", action="store_true", help="gather f64 coordinates (default: float32)")
    ap.add_argument("--native-gather", action="store_true", help="gather through sl_gather (the C-ABI RCCL path)")
    a = ap.parse_args(argv)
    from .multi_point_cloud_process import load_calibration
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    try:
        calib = load_calibration(a.calib_file)
        poses = np.load(a.poses) if a.poses else None  # a plain array: np.load without pickles
        scan_distributed(a.scan_dir, calib, poses=poses, n_cols=a.n_cols, n_rows=a.n_rows, voxel_size=a.voxel,
                         merge_output=a.merge_output, write_views=not a.no_view_ply,
                         xyz_dtype=torch.float64 if a.f64 else torch.float32, native_gather=a.native_gather)
        dist.barrier()
    finally:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""scan360.scan_distributed: view folders sharded over ranks, clouds gathered
to rank 0 in view order.  CPU: world_size 2 on gloo with the oracle as the
per-rank work (the GPU path's per-view parity is proven by the GPU tests).
GPU: world_size 1 on nccl through the real per-rank pipeline."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from PIL import Image

from structured_light_for_3d_model_replication_amd import synth

RIG = dict(H=24, W=32, Wp=16, Hp=8)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _write_scan(parent, V):
    rig = synth.Rig(**RIG)
    for v in range(V):
        s, _ = synth.render_stack(rig, seed=40 + v, include_rows=False, view_deg=30.0 * v, device="cpu")
        d = os.path.join(parent, f"view_{v:02d}")
        os.makedirs(d)
        for i, im in enumerate(s.numpy()):
            Image.fromarray(im).save(os.path.join(d, f"{i + 1:02d}.png"))
    os.makedirs(os.path.join(parent, "zz_empty"))
    return synth.make_calibration(rig, with_Nc=False)


def _oracle_views(views, calib, poses):
    from oracle import sl_oracle as o
    from structured_light_for_3d_model_replication_amd import io
    out = []
    for f, M in zip(views, poses):
        st, tex, _ = io.read_stack(f)
        P, C = o.decode_triangulate(list(st), tex, calib, RIG["Wp"], RIG["Hp"], mask_mode="fixed", pose=M)[3:]
        out.append((torch.from_numpy(P), torch.from_numpy(C)))
    return out


def _worker(rank, world, port, parent, V, q):
    from structured_light_for_3d_model_replication_amd import scan360
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calib = synth.make_calibration(synth.Rig(**RIG), with_Nc=False)
        poses = [synth.turntable_pose(30.0 * v) for v in range(V)]
        P, C, counts = scan360.scan_distributed(parent, calib, poses=poses, process=_oracle_views,
                                                log=lambda *a: None)
        if rank == 0:
            q.put((P.numpy(), C.numpy(), counts))
        else:
            assert P is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("V", [5, 1])
def test_scan_distributed_gloo_world2(tmp_path, V):
    parent = str(tmp_path / "scan")
    calib = _write_scan(parent, V)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, parent, V, q)) for r in range(2)]
    for p in procs:
        p.start()
    P, C, counts = q.get(timeout=180)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    views = sorted(os.path.join(parent, f"view_{v:02d}") for v in range(V))
    ref = _oracle_views(views, calib, [synth.turntable_pose(30.0 * v) for v in range(V)])
    np.testing.assert_array_equal(P, np.concatenate([p.numpy() for p, _ in ref]))
    np.testing.assert_array_equal(C, np.concatenate([c.numpy() for _, c in ref]))
    assert sum(counts) == len(P) and len(counts) == 2


@pytest.mark.gpu
def test_scan_distributed_gpu_world1(tmp_path):
    """The real per-rank path (streamed GPU pipeline, device pose transform,
    RCCL process group of one, merge post-processing) vs the oracle."""
    from structured_light_for_3d_model_replication_amd import merge, ply, scan360
    V = 4
    parent = str(tmp_path / "scan")
    calib = _write_scan(parent, V)
    poses = [synth.turntable_pose(30.0 * v) for v in range(V)]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        out = str(tmp_path / "merged.ply")
        P, C, counts = scan360.scan_distributed(parent, calib, poses=poses, n_cols=RIG["Wp"], n_rows=RIG["Hp"],
                                                log=lambda *a: None)
        views = sorted(os.path.join(parent, f"view_{v:02d}") for v in range(V))
        ref = _oracle_views(views, calib, poses)
        np.testing.assert_array_equal(P.cpu().numpy(), np.concatenate([p.numpy() for p, _ in ref]))
        np.testing.assert_array_equal(C.cpu().numpy(), np.concatenate([c.numpy() for _, c in ref]))
        assert counts == [len(P)]
        for f in views:
            assert os.path.exists(os.path.join(f, os.path.basename(f) + ".ply"))
        Pm, Cm, _ = scan360.scan_distributed(parent, calib, poses=poses, n_cols=RIG["Wp"], n_rows=RIG["Hp"],
                                             voxel_size=5.0, merge_output=out, write_views=False,
                                             log=lambda *a: None)
        Pe, Ce = merge.postprocess(P, C, 5.0)
        np.testing.assert_array_equal(Pm.cpu().numpy(), Pe.cpu().numpy())
        Pr, Cr = ply.read_ply(out)  # binary PLY: float32 xyz
        np.testing.assert_array_equal(np.asarray(Pr, np.float32), Pm.cpu().numpy().astype(np.float32))
        np.testing.assert_array_equal(np.asarray(Cr), Cm.cpu().numpy())
    finally:
        dist.destroy_process_group()

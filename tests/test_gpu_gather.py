"""sl_gather (the library's RCCL gather, include/slgpu.h) on one GPU: a
communicator of one rank, alone and under a torch.distributed RCCL group
(PyTorch's RCCL already loaded in the process)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _cloud(n, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn((n, 3), generator=g, dtype=torch.float64).to(dtype).cuda(),
            torch.randint(0, 256, (n, 3), generator=g, dtype=torch.uint8).cuda())


@pytest.mark.parametrize("dtype,n", [(torch.float64, 100_003), (torch.float32, 7), (torch.float32, 0)])
def test_gather_world1(dtype, n):
    from structured_light_for_3d_model_replication_amd import core
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.gather_init(1, 0, core.Reconstructor.gather_unique_id())
    xyz, bgr = _cloud(n, dtype, n)
    xa, ca, counts = eng.gather(xyz, bgr, root=0)
    eng.sync()
    assert counts == [n]
    assert torch.equal(xa, xyz) and torch.equal(ca, bgr)
    with pytest.raises(ValueError):
        eng.gather(xyz.to(torch.float16), bgr)


def test_gather_native_under_torch_rccl():
    from structured_light_for_3d_model_replication_amd import core, parallel
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        eng = core.Reconstructor(torch.device("cuda", 0))
        xyz, bgr = _cloud(50_000, torch.float32, 5)
        xa, ca, counts = parallel.gather_cloud_native(eng, xyz, bgr)
        xb, cb, counts_b = parallel.gather_cloud(xyz, bgr)
        torch.cuda.synchronize()
        assert counts == counts_b == [50_000]
        assert torch.equal(xa, xb) and torch.equal(ca, cb)
        t = torch.ones(4, device="cuda")
        dist.all_reduce(t)  # torch's own RCCL still works beside the library's communicator
        assert float(t.sum()) == 4.0
    finally:
        dist.destroy_process_group()

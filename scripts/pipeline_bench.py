"""Host-resident scans through pipeline.ViewPipeline: PCIe-inclusive px/s.

    python scripts/pipeline_bench.py [--views 16] [--H 2160 --W 3840] [--files 4]

Lines printed (JSON):
  h2d          raw pinned H2D bandwidth of one cloud-plane stack
  serial       per view: H2D of all 46 planes + texture, kernels, D2H, sync
               (the one-shot path on a host stack, nothing overlapped)
  pipeline     ViewPipeline over caller-pinned views (HostView): 24 cloud
               planes + texture up, f32-fast xyz + BGR down, overlapped
  files        process_batch(streamed) over BMP scan folders on local disk
               (PIL decode into pinned slots, 16 threads), clouds kept on host
Views cycle over 4 distinct synthetic 4K stacks (config-2 rig).
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from structured_light_for_3d_model_replication_amd import core, pipeline, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--views", type=int, default=16)
ap.add_argument("--H", type=int, default=2160)
ap.add_argument("--W", type=int, default=3840)
ap.add_argument("--files", type=int, default=4, help="scan folders for the file-ingest leg (0: skip)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
rig = synth.Rig(H=a.H, W=a.W)
cal = synth.make_calibration(rig, with_Nc=False)
eng = core.Reconstructor(dev)
eng.set_calibration(cal, a.H, a.W)
D = 4
host = []
for v in range(D):
    s, t = synth.render_stack(rig, seed=2000 + v, view_deg=10.0 * v, device=dev)
    host.append(pipeline.HostView(s.cpu().pin_memory(), t.cpu().pin_memory()))
    del s, t
n_img = host[0].stack.shape[0]
px = a.H * a.W

# raw H2D of the 24 cloud planes
n_up = pipeline.planes_for_cloud(n_img)
dst = torch.empty((n_up, a.H, a.W), dtype=torch.uint8, device=dev)
for _ in range(2):
    dst.copy_(host[0].stack[:n_up], non_blocking=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    dst.copy_(host[0].stack[:n_up], non_blocking=True)
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / 5
print(json.dumps({"leg": "h2d", "bytes": dst.numel(), "ms": 1e3 * el, "GBps": dst.numel() / el / 1e9}))
del dst

# serial one-shot path: full stack up, kernels, points down, per view
ds = torch.empty((n_img, a.H, a.W), dtype=torch.uint8, device=dev)
dt = torch.empty((a.H, a.W, 3), dtype=torch.uint8, device=dev)
out = {}
hx = torch.empty((px, 3), dtype=torch.float32, pin_memory=True)
hb = torch.empty((px, 3), dtype=torch.uint8, pin_memory=True)


def serial_view(i):
    hv = host[i % D]
    ds.copy_(hv.stack, non_blocking=True)
    dt.copy_(hv.texture, non_blocking=True)
    r = eng.decode_triangulate(ds, texture=dt, cloud=True, xyz_dtype=torch.float32, fast_f32=True, out=out)
    n = r["cloud"].total()
    hx[:n].copy_(r["cloud"].xyz[:n], non_blocking=True)
    hb[:n].copy_(r["cloud"].bgr[:n], non_blocking=True)
    torch.cuda.synchronize()
    return n


serial_view(0)
t0 = time.perf_counter()
pts = sum(serial_view(i) for i in range(a.views))
el = time.perf_counter() - t0
print(json.dumps({"leg": "serial", "views": a.views, "px_per_s": a.views * px / el, "ms_per_view": 1e3 * el / a.views,
                  "points": pts}))
del ds, dt, out

# overlapped pipeline over caller-pinned views
pipe = pipeline.ViewPipeline(eng, H=a.H, W=a.W, n_img=n_img, xyz_dtype=torch.float32, fast_f32=True, slots=3)
pipe.run(3, lambda i, s, t: host[i % D])
st = pipe.run(a.views, lambda i, s, t: host[i % D])
d = st.as_dict()
d.update({"leg": "pipeline", "ms_per_view": 1e3 * st.wall_s / a.views, "planes_up": n_up, "slots": 3})
print(json.dumps(d))
del pipe

if a.files > 0:
    from PIL import Image

    from structured_light_for_3d_model_replication_amd import io, multi_point_cloud_process as mp
    root = tempfile.mkdtemp(prefix="sl_scan_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        for v in range(a.files):
            f = os.path.join(root, f"view_{v:03d}")
            os.makedirs(f)
            stk = host[v % D].stack.numpy()
            for j in range(n_img):
                Image.fromarray(stk[j]).save(os.path.join(f, f"{j + 1:02d}.bmp"))
        mp.process_batch(root, cal, write=False, keep=False, log=lambda s: None)  # warm page cache + pools
        t0 = time.perf_counter()
        mp.process_batch(root, cal, write=False, keep=False, log=lambda s: None)
        el = time.perf_counter() - t0
        t1 = time.perf_counter()
        files = io.list_stack_files(os.path.join(root, "view_000"))
        buf = np.empty((n_up, a.H, a.W), dtype=np.uint8)
        tex = np.empty((a.H, a.W, 3), dtype=np.uint8)
        io.fill_stack(files, buf, tex)
        el_fill = time.perf_counter() - t1
        print(json.dumps({"leg": "files", "views": a.files, "px_per_s": a.files * px / el,
                          "ms_per_view": 1e3 * el / a.files, "ingest_ms_per_view": 1e3 * el_fill,
                          "format": "8-bit BMP, single channel (texture = white plane)", "threads": 8}))
    finally:
        shutil.rmtree(root, ignore_errors=True)

"""Is config 1 host-bound?  bench.py's c1 call (one resident 1280x720 view
per lane, prepared, next-stats chained) over S lanes at priority P: K calls
enqueued back to back -- the host's enqueue time (loop end) against the
total (after the final sync), and the same K calls with the GPU work already
queued far ahead (the host's own cost per call when it never waits)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from structured_light_for_3d_model_replication_amd import core, synth  # noqa: E402

dev = torch.device("cuda", 0)
rig = synth.Rig(H=720, W=1280, Wp=1024, Hp=768)
cal = synth.make_calibration(rig, with_Nc=False)
st, tx = synth.render_stack(rig, seed=1000, include_rows=False, device=dev)
for S, P in ((4, -1), (3, 0), (1, 0)):
    pool = core.ReconstructorPool(dev, lanes=S, reuse_outputs=True, stream_priority=P)
    pool.set_calibration(cal, rig.H, rig.W)
    outs = [{} for _ in range(S)]

    def call(i):
        pool.decode_triangulate(st, 1024, 768, texture=tx, maps=True, cloud=True, xyz_dtype=torch.float32,
                                out=outs[i % S], next_stack=st, wait_inputs=False, lane=i % S, prepared=True)
    for i in range(200):
        call(i)
    torch.cuda.synchronize(dev)
    for K in (2000, 4000):
        t0 = time.perf_counter()
        for i in range(K):
            call(i)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        print(f"lanes {S} prio {P} K {K}: enqueue {1e6 * (t1 - t0) / K:.2f} us/call, total {1e6 * (t2 - t0) / K:.2f} us/call",
              flush=True)
    pool.close()

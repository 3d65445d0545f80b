"""Where a prepared c1 call's host time goes (4 high-priority lanes, one
resident 1280x720 view, maps + cloud): K calls enqueued per variant --
  pool     ReconstructorPool.decode_triangulate (bench.py's path)
  run      PreparedCall.run(stream, next_stack)
  raw2     sl_stack_next + sl_call_run through the bound ctypes functions
  raw1     sl_call_run alone (no next-stats: the call then runs k_stats)
-> host enqueue us/call and total us/call (after the final sync)."""
import ctypes
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
S = 4
pool = core.ReconstructorPool(dev, lanes=S, reuse_outputs=True, stream_priority=-1)
pool.set_calibration(cal, rig.H, rig.W)
outs = [{} for _ in range(S)]


def pcall(i):
    pool.decode_triangulate(st, 1024, 768, texture=tx, maps=True, cloud=True, xyz_dtype=torch.float32,
                            out=outs[i % S], next_stack=st, wait_inputs=False, lane=i % S, prepared=True)


for i in range(100):
    pcall(i)
torch.cuda.synchronize(dev)
plans = [next(iter(pool._plans[k].values()))[1] for k in range(S)]
streams = pool.streams
nargs = plans[0].eng._next_args(st, rig.H, rig.W)
raw = [(p.eng._L.sl_stack_next, p.eng._ctx, p._run, p._h, s.cuda_stream) for p, s in zip(plans, streams)]


def run(i):
    plans[i % S].run(streams[i % S], next_stack=st)


def raw2(i):
    nx, ctx, rn, h, s = raw[i % S]
    nx(ctx, *nargs)
    rn(h, s)


def raw1(i):
    _, _, rn, h, s = raw[i % S]
    rn(h, s)


for name, f in (("pool", pcall), ("run", run), ("raw2", raw2), ("raw1", raw1), ("pool", pcall)):
    for i in range(200):
        f(i)
    torch.cuda.synchronize(dev)
    K = 4000
    t0 = time.perf_counter()
    for i in range(K):
        f(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    print(f"{name}: enqueue {1e6 * (t1 - t0) / K:.2f} us/call, total {1e6 * (t2 - t0) / K:.2f} us/call", flush=True)

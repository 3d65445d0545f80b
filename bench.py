#!/usr/bin/env python3
"""Benchmark: decoded+triangulated camera px/s (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

A step is one pass of the hot path over one batch of synthetic views resident
in HBM -- k_stats (black-plane histogram, max(white - black)), k_decode (Gray
decode, Gray->binary, adaptive-mask thresholds, mask, point/no-point decision,
chunk counts), k_cloud (chunk offsets, ray/plane intersection, ordered
stores) -- producing what the reference's gray_decode + reconstruct_point_cloud
return: col_map, row_map, mask and the (xyz, BGR) cloud.

Arithmetic: by default the triangulation is the reference's float64
arithmetic (server/sl_system.py:614-648, same operation order, no contraction;
xyz stored as the correctly rounded float32 of that f64: SL_XYZ_F32).
``--xyz fast`` (SL_XYZ_F32_FAST: f32 arithmetic, per-coordinate relative
error <= 1.02e-5) is reported beside it in "alt_xyz_mode", never as `value`.

Timing: W warm-up steps, then a declared untimed pre-roll (``--preroll-ms``,
default 300 ms of back-to-back steps, so the GPU's clocks and power state are
at their steady state when the timed window opens -- a bench that follows an
idle GPU would otherwise time the clock ramp), then, with no idle gap,
exactly K steps between barrier + synchronize pairs (garbage collection off);
then an identical window with one HIP event per step boundary on the stream
(per-step min / median / max in "timing.step_us"; the events add idle time,
so they stay out of the headline window).  Max over ranks.

Default workload = BASELINE config 2: one 3840x2160 view, 11+11-bit
column+row Gray code with inverses (46 planes), per GPU per step; the steps
cycle through three distinct resident views (--ring), so that nothing of a
view stays in the 256 MB Infinity Cache until its next step.
Multi-GPU: weak scaling by default (views sharded over ranks with no
data-path collective); the gather of the clouds to rank 0 (RCCL: torch's
communicator, or ``--gather native`` = the library's own sl_gather) is timed
separately and described in "multi_gpu".
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import statistics
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from structured_light_for_3d_model_replication_amd import core, parallel, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# the committed calibrated-PMC traffic profiles the lines cite (scripts/gpu_r4_traffic.sh)
TRAFFIC_DIR = os.path.join("profiles", "r06_traffic")

CONFIGS = {
    # BASELINE.json configs.  views = views per GPU per step (weak scaling;
    # strong: views in total); maps: also write the col/row/mask maps (what
    # gray_decode returns); pose: turntable pose epilogue (config 5's merge
    # into one frame).  c4 / c5: 45 views per GPU = the per-GPU share of the
    # 360-view scan over 8 GPUs (24.8 / 17.2 GB of stacks resident in HBM);
    # c3: the 36-view turntable scan (strong scaling shards it).
    "c1": dict(H=720, W=1280, Wp=1024, Hp=768, rows=False, views=1, maps=True, pose=False, deg=10.0,
               streams=4, lane_priority=-1,  # 4 lanes on high-priority streams, each with a hardware queue of
                                             # its own (normal-priority lanes share 2 of the 4 queues)
               steps=200,  # 20 steps of ~11 us: 14 us per step measured, the lanes' fill and drain
               ring_control=12),  # the control window's distinct views: 12 x 23 MB > the 256 MiB Infinity Cache
    "c2": dict(H=2160, W=3840, Wp=1920, Hp=1080, rows=True, views=1, maps=True, pose=False, deg=10.0,
               ring=3, streams=2),  # distinct resident views cycled (no Infinity-Cache
                                    # carry-over; 3 rounded up to 4, a multiple of the lanes), 2 lanes (5.2)
    "c3": dict(H=1080, W=1920, Wp=1920, Hp=1080, rows=True, views=36, maps=False, pose=False, deg=10.0,
               streams=2),
    "c4": dict(H=3000, W=4000, Wp=1920, Hp=1080, rows=True, views=45, maps=False, pose=False, deg=1.0,
               streams=3, lane_priority=-1),  # 3 lanes, a hardware queue each
    "c5": dict(H=2160, W=3840, Wp=1920, Hp=1080, rows=True, views=45, maps=False, pose=True, deg=1.0,
               streams=3, lane_priority=-1),
}


XYZ_MODES = {True: "SL_XYZ_F32_FAST: f32 arithmetic, per-coordinate rel err <= 1.02e-5 of the reference's "
                    "f64 (tolerance 1e-4); kappa > 16 points exact",
             False: "SL_XYZ_F32: the reference's f64 arithmetic (sl_system.py:614-648, same order, no "
                    "contraction), xyz = correctly rounded float32 of that f64"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (ranks) of one node; without torch.distributed.run, N > 1 starts N ranks itself")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: the config's views per GPU; strong: the config's views in total, sharded")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend (gloo only with --selftest)")
    ap.add_argument("--selftest", action="store_true",
                    help="CPU plumbing test of the launcher / timing / gather (no GPU, no kernels)")
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default per config: 20; c1 200 -- its 11-us steps on 4 lanes would otherwise "
                         "leave a quarter of a 20-step window to the lanes' fill and drain)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--preroll-ms", dest="preroll_ms", type=float, default=300.0,
                    help="untimed back-to-back steps after the warm-up, before the timed window (ms)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--views", type=int, default=None, help="views per GPU per step (default per config)")
    ap.add_argument("--cpu-baseline", dest="cpu_baseline", action="store_true", default=True)
    ap.add_argument("--no-cpu-baseline", dest="cpu_baseline", action="store_false")
    ap.add_argument("--xyz", default="exact", choices=["exact", "fast"],
                    help="exact: SL_XYZ_F32 (the reference's f64 arithmetic, correctly rounded float32 out); "
                         "fast: SL_XYZ_F32_FAST (f32 arithmetic, rel err <= 1.02e-5 of the reference's f64)")
    ap.add_argument("--streams", type=int, default=None,
                    help="default per config (CONFIGS: measured best, DESIGN.md 6.2); views in flight per GPU: "
                         "successive steps round-robin over this many contexts, each on its own HIP stream "
                         "with its own outputs (one step's kernels overlap the next one's on the other stream)")
    ap.add_argument("--lane-priority", dest="lane_priority", type=int, default=None,
                    help="HIP stream priority of the lanes (default per config)")
    ap.add_argument("--gather", default="torch", choices=["torch", "native"],
                    help="N > 1: the cloud gather through torch.distributed's RCCL communicator, or the "
                         "library's own (sl_gather_init / sl_gather_counts / sl_gather)")
    ap.add_argument("--secondary", dest="secondary", action="store_true", default=True,
                    help="also time the cloud-only and the other xyz mode (default on)")
    ap.add_argument("--no-secondary", dest="secondary", action="store_false")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget for the CPU baseline sample")
    ap.add_argument("--cpu-procs", type=int, default=None,
                    help="processes of the multi-process CPU leg (default: the core share, multi-view "
                         "configs only; 0: off)")
    ap.add_argument("--next-stats", dest="next_stats", action="store_true", default=True,
                    help="every call names the next call's (resident) stack (sl_stack_next): its triangulation "
                         "kernel also computes the next call's adaptive-mask histograms (default)")
    ap.add_argument("--no-next-stats", dest="next_stats", action="store_false")
    ap.add_argument("--graph", dest="graph", action="store_true", default=True,
                    help="one lane: the headline window replays a hipGraph of its K steps, captured (untimed) "
                         "right after the pre-roll -- every kernel of every step runs, the host enqueues nothing "
                         "inside the window (default; falls back to eager calls if capture fails; with lanes the "
                         "window is eager: captured lanes measured slower)")
    ap.add_argument("--no-graph", dest="graph", action="store_false")
    ap.add_argument("--verify", dest="verify", action="store_true", default=True,
                    help="after the windows, check the last timed step's outputs of a sample of views (the first "
                         "and the last of this rank) against the oracle run on the same resident inputs (default)")
    ap.add_argument("--no-verify", dest="verify", action="store_false")
    ap.add_argument("--single-shot", dest="single_shot", type=int, default=24,
                    help="isolated unchained calls timed for the one-shot latency block (0: off)")
    ap.add_argument("--strong-leg", dest="strong_leg", action="store_true", default=True,
                    help="N > 1: also time BASELINE config 3 strong-scaled (36 views sharded over the N ranks) "
                         "and report it in multi_gpu.strong_c3 (default)")
    ap.add_argument("--no-strong-leg", dest="strong_leg", action="store_false")
    ap.add_argument("--ring", type=int, default=None,
                    help="one view in flight: the headline window cycles through this many distinct resident "
                         "views (stack, texture and outputs each), chained; 1 = the same view every step.  Default "
                         "(CONFIGS): c2 3 -- one view's texture, records and outputs stayed in the 256 MB Infinity "
                         "Cache from step to step and made the one-view window 3.5 %% faster (DESIGN.md 6.1)"),
    ap.add_argument("--ring-control", dest="ring_control", type=int, default=None,
                    help="one view in flight: a second window with this many distinct views when the headline "
                         "uses one (or one view when the headline cycles several), reported in "
                         "timing.distinct_views -- does the 256 MB Infinity Cache help the one-view window? "
                         "(default per config: c1 12 -- 12 x 23 MB of inputs exceed the cache --, else 3; 0: off)")
    ap.add_argument("--traffic", default=None,
                    help="PMC-derived HBM bytes per step (committed profile of the same workload, "
                         "scripts/traffic_from_pmc.py); default " + TRAFFIC_DIR + "/traffic_<config>.json")
    a = ap.parse_args(argv)
    if a.steps is None:
        a.steps = CONFIGS[a.config].get("steps", 20)
    return a


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a) -> int:
    """``--gpus N`` run without torch.distributed.run: start the N ranks (one
    process per GPU) as a child ``torch.distributed.run`` on 127.0.0.1 and
    return its exit status.  This process touches no GPU (the ranks do), and it
    starts the launcher as a child, not by exec."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__),
           *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def rank_env():
    """(world, rank, local_rank, distributed) from torch.distributed.run's env."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1 or ("RANK" in os.environ and "MASTER_ADDR" in os.environ)
    return world, rank, local, distributed


def my_views(scaling: str, V_cfg: int, world: int, rank: int) -> list[int]:
    """Global view indices of this rank: weak = V_cfg per GPU (contiguous
    blocks), strong = V_cfg in total sharded in contiguous blocks (view v ->
    rank floor(v*G/V), parallel.shard_views)."""
    if scaling == "strong":
        return list(parallel.shard_views(V_cfg, world, rank))
    return [rank * V_cfg + v for v in range(V_cfg)]


def gather_report(el_s: float, n_local: int, bytes_per_point: int, device, gather_fn, distributed: bool):
    """Multi-rank facts of the timed run, identical on every rank, for rank 0's
    line: the communicator size torch.distributed sees, every rank's seconds
    for the K steps and its point count; then one timed gather of the clouds
    to rank 0 (gather_fn() -> counts as the gather's own communicator saw
    them) with its bytes (the payload that crossed to rank 0) and GB/s."""
    world = dist.get_world_size() if distributed else 1
    t = torch.tensor([el_s, float(n_local)], dtype=torch.float64, device=device)
    if distributed:
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
    else:
        outs = [t]
    per_rank_s = [float(o[0].item()) for o in outs]
    per_rank_pts = [int(o[1].item()) for o in outs]
    rep = {"comm_size": world, "per_rank_s": per_rank_s, "per_rank_points": per_rank_pts}
    if not distributed:
        return rep
    dist.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    tg = time.perf_counter()
    counts = gather_fn()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    gt = torch.tensor([time.perf_counter() - tg], dtype=torch.float64, device=device)
    dist.all_reduce(gt, op=dist.ReduceOp.MAX)
    g_s = float(gt.item())
    moved = sum(c for r, c in enumerate(counts) if r != 0) * bytes_per_point
    rep.update({"gather_counts": [int(c) for c in counts], "gather_counts_len": len(counts),
                "gather_bytes_to_root": int(moved), "gather_ms": 1e3 * g_s,
                "gather_GBps": moved / g_s / 1e9 if g_s > 0 else None,
                # what the gather must move, from every rank's point count before it ran
                "expected_gather_bytes_to_root": int(sum(per_rank_pts[1:]) * bytes_per_point),
                "bytes_per_point": bytes_per_point})
    return rep


def selftest(a) -> None:
    """CPU plumbing test of the multi-rank bench (``--selftest --backend gloo``):
    the same launch, barrier + max-over-ranks timing, multi-rank report and
    rank-order gather as the GPU bench, with a stand-in per-rank cloud of
    known size instead of the kernels (the kernels' parity is the GPU tests'
    job).  Rank 0 prints one JSON line with n_gpus, the gathered point count
    and the "multi_gpu" block of the GPU line."""
    world, rank, _, distributed = rank_env()
    if distributed:
        dist.init_process_group("gloo")
    V = a.views or 3
    views = my_views(a.scaling, V, world, rank)
    n_per_view = 1000
    if distributed:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        xyz = torch.cat([torch.full((n_per_view, 3), float(v), dtype=torch.float32) for v in views]) \
            if views else torch.zeros((0, 3), dtype=torch.float32)
        bgr = torch.zeros((xyz.shape[0], 3), dtype=torch.uint8)
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64)
    if distributed:
        dist.barrier()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    got = {}

    def gfn():
        xa, _, counts = parallel.gather_cloud(xyz, bgr, dst=0)
        got["xa"] = xa
        return counts
    rep = gather_report(el, xyz.shape[0], 15, torch.device("cpu"), gfn, distributed)
    xa = got.get("xa", xyz)
    if distributed and a.strong_leg:
        # the strong-scaled config-3 leg's plumbing: 36 views sharded, stand-in clouds
        def leg_step(views3):
            return torch.cat([torch.full((n_per_view, 3), float(v), dtype=torch.float32) for v in views3]) \
                if views3 else torch.zeros((0, 3), dtype=torch.float32)
        rep["strong_c3"] = strong_leg_report(
            a, world, rank, distributed, torch.device("cpu"), px_per_view=1920 * 1080,
            run=lambda views3: _stand_in_leg(a, views3, leg_step))
    if rank == 0:
        order_ok = bool(torch.equal(xa[::n_per_view, 0], torch.arange(xa.shape[0] // n_per_view,
                                                                      dtype=torch.float32)))
        print(json.dumps({"metric": "selftest", "n_gpus": world, "steps": a.steps, "scaling": a.scaling,
                          "views_total": V * world if a.scaling == "weak" else V,
                          "gathered_points": int(xa.shape[0]), "counts": rep.get("gather_counts", [xyz.shape[0]]),
                          "view_order_ok": order_ok, "max_rank_s": float(t.item()), "multi_gpu": rep}))
    if distributed:
        dist.destroy_process_group()


def _stand_in_leg(a, views3, leg_step):
    """selftest: the strong leg's K steps on stand-in clouds -> (seconds, xyz, bgr)."""
    t0 = time.perf_counter()
    for _ in range(a.steps):
        xyz = leg_step(views3)
    el = time.perf_counter() - t0
    return el, xyz, torch.zeros((xyz.shape[0], 3), dtype=torch.uint8)


def ideal_strong_efficiency(V: int, world: int) -> float:
    """The bound contiguous view shards put on strong-scaling efficiency:
    V / (N x the largest shard) (36 views: 1.0 at N = 2, 3, 4; 0.9 at N = 8)."""
    return V / (world * max(len(parallel.shard_views(V, world, r)) for r in range(world)))


def strong_leg_report(a, world, rank, distributed, device, px_per_view, run, V=36):
    """BASELINE config 3 as the N-GPU run's second line: V views in total,
    sharded over the ranks (parallel.shard_views, view v -> rank
    floor(v*G/V)); run(views) -> (this rank's seconds for the K steps after a
    barrier, xyz, bgr of its last step); then the same multi-rank report and
    timed gather to rank 0 as the headline's."""
    views3 = list(parallel.shard_views(V, world, rank))
    if distributed:
        dist.barrier()
    el, xyz, bgr = run(views3)

    def gfn():
        _, _, counts = parallel.gather_cloud(xyz, bgr, dst=0)
        return counts
    rep = gather_report(el, xyz.shape[0], 15 if xyz.dtype == torch.float32 else 27, device, gfn, distributed)
    per_views = [len(parallel.shard_views(V, world, r)) for r in range(world)]
    t_max = max(rep["per_rank_s"])
    rep.update({"config": f"BASELINE config 3: {V} x 1920x1080 views in total, sharded over {world} rank(s) "
                          "(strong scaling), cloud only, exact xyz",
                "views_total": V, "per_rank_views": per_views, "steps": a.steps,
                # the slowest rank sets the step: V / (N x its views) is the best
                # efficiency against one GPU that contiguous view shards allow
                # (36 / (8 x 5) = 0.9 at N = 8), before any cost of the path
                "ideal_strong_efficiency": ideal_strong_efficiency(V, world),
                "ideal_strong_efficiency_note": "V / (N x max views per rank): the bound the shard imbalance "
                                                "puts on px/s(N) / (N x px/s(1)) with per-view work constant",
                "per_rank_ms_per_step": [1e3 * t / a.steps for t in rep["per_rank_s"]],
                "ms_per_step": 1e3 * t_max / a.steps,
                "px_per_s": V * px_per_view * a.steps / t_max if t_max > 0 else None})
    return rep


def single_shot(eng, call, n, stream):
    """One-shot latency (the GUI's generate_cloud: one call at a time,
    sl_system.py:655-661): ``n`` isolated calls -- synchronize, enqueue one
    unchained call (its own k_stats included), synchronize -- after two
    untimed ones; host wall µs and HIP-event µs on the call's stream."""
    eng.drop_next()  # no pass queued by an earlier chained call is taken
    wall, gpu = [], []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(n + 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        call()
        e1.record(stream)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if i >= 2:
            wall.append(1e6 * (t1 - t0))
            gpu.append(1e3 * e0.elapsed_time(e1))
    return {"calls": n, "wall_us": spread(wall), "gpu_us": spread(gpu)}


def run_c3_leg(a, dev, views3):
    """The strong leg on the GPU: this rank's shard of config 3's views,
    resident, through config 3's lanes (CONFIGS["c3"]), chained as the
    headline; warm-up, a 100-ms pre-roll, then K steps between synchronizes
    -> (seconds, xyz, bgr of lane 0's last step)."""
    cfg = CONFIGS["c3"]
    H, W = cfg["H"], cfg["W"]
    rig = synth.Rig(H=H, W=W, Wp=cfg["Wp"], Hp=cfg["Hp"])
    calib = synth.make_calibration(rig, with_Nc=False)
    stack = tex = None
    for k, gv in enumerate(views3):
        s_, t_ = synth.render_stack(rig, seed=1000 * 3 + gv, include_rows=True, view_deg=cfg["deg"] * gv, device=dev)
        if stack is None:
            stack = torch.empty((len(views3),) + tuple(s_.shape), dtype=torch.uint8, device=dev)
            tex = torch.empty((len(views3), H, W, 3), dtype=torch.uint8, device=dev)
        stack[k].copy_(s_)
        tex[k].copy_(t_)
        del s_, t_
    pool = core.ReconstructorPool(dev, lanes=cfg["streams"], reuse_outputs=True)
    pool.set_calibration(calib, H, W)

    def one():
        pool.decode_triangulate(stack, cfg["Wp"], cfg["Hp"], texture=tex, maps=False, cloud=True,
                                xyz_dtype=torch.float32, wait_inputs=False, next_stack=stack)
    if stack is not None:
        for _ in range(max(a.warmup, pool.lanes)):
            one()
        torch.cuda.synchronize(dev)
        t_pr = time.perf_counter()
        while (time.perf_counter() - t_pr) * 1e3 < min(a.preroll_ms, 100.0):
            for _ in range(4):
                one()
            torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if stack is not None:
        for _ in range(a.steps):
            one()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    if stack is None:
        xyz, bgr = torch.zeros((0, 3), dtype=torch.float32, device=dev), torch.zeros((0, 3), dtype=torch.uint8, device=dev)
    else:
        o = pool._outs[0]
        n = int(o["view_offsets"][-1].item())
        xyz, bgr = o["xyz"][:n], o["bgr"][:n]
    return el, xyz, bgr


def single_shot_c1(dev, n, stream):
    """single_shot of BASELINE config 1's view (1280x720, 10 column bits,
    maps + cloud) on a context of its own."""
    cfg = CONFIGS["c1"]
    rig = synth.Rig(H=cfg["H"], W=cfg["W"], Wp=cfg["Wp"], Hp=cfg["Hp"])
    st, tx = synth.render_stack(rig, seed=1000, include_rows=False, device=dev)
    e = core.Reconstructor(dev)
    e.set_calibration(synth.make_calibration(rig, with_Nc=False), cfg["H"], cfg["W"])
    o = {}

    def call():
        e.decode_triangulate(st, cfg["Wp"], cfg["Hp"], texture=tx, maps=True, cloud=True, xyz_dtype=torch.float32,
                             out=o, stream=stream)
    r = single_shot(e, call, n, stream)
    e.close()
    return r


def snap_alloc(out, V, maps):
    """Pinned host buffers for the outputs of views 0 and V-1 (the verified
    sample), sized from the warm-up's offsets (the same inputs every step)."""
    vo = out["view_offsets"].cpu().numpy()
    pin = dict(pin_memory=True)
    snap = {"vo": vo, "vo_dev": torch.empty(V + 1, dtype=torch.int64, **pin), "views": {}}
    for v in sorted({0, V - 1}):
        n = int(vo[v + 1] - vo[v])
        d = {"xyz": torch.empty((n, 3), dtype=out["xyz"].dtype, **pin), "bgr": torch.empty((n, 3), dtype=torch.uint8, **pin)}
        if maps:
            d.update(col=torch.empty(out["col_map"].shape[1:], dtype=torch.int32, **pin),
                     row=torch.empty(out["row_map"].shape[1:], dtype=torch.int32, **pin),
                     mask=torch.empty(out["mask_u8"].shape[1:], dtype=torch.uint8, **pin))
        snap["views"][v] = d
    return snap


def snap_copy(snap, out, stream):
    """Enqueue the copies of the current outputs into the pinned buffers on
    ``stream`` (right after the headline window: they hold its last step's)."""
    vo = snap["vo"]
    with torch.cuda.stream(stream):
        snap["vo_dev"].copy_(out["view_offsets"], non_blocking=True)
        for v, d in snap["views"].items():
            d["xyz"].copy_(out["xyz"][vo[v]:vo[v + 1]], non_blocking=True)
            d["bgr"].copy_(out["bgr"][vo[v]:vo[v + 1]], non_blocking=True)
            if "col" in d:
                d["col"].copy_(out["col_map"][v], non_blocking=True)
                d["row"].copy_(out["row_map"][v], non_blocking=True)
                d["mask"].copy_(out["mask_u8"][v], non_blocking=True)


def verify(snap, stack, tex, poses, calib, n_cols, n_rows, fast):
    """The snapshot (the last timed step's outputs) against the oracle
    (oracle/sl_oracle.py: the reference's gray_decode + reconstruct_point_cloud,
    sl_system.py:508-653) run on the same resident inputs: maps, mask, point
    count and colours bit-exact; xyz = float32 of the oracle's f64 (exact
    mode) or within 1.02e-5 relative per coordinate (fast mode)."""
    from oracle import sl_oracle
    t0 = time.perf_counter()
    ok = bool(np.array_equal(snap["vo_dev"].numpy(), snap["vo"]))  # the window's offsets = the warm-up's
    notes = []
    for v, dt in snap["views"].items():
        d = {k: t.numpy() for k, t in dt.items()}
        if "mask" in d:
            d["mask"] = d["mask"].astype(bool)
        st = stack[v].cpu().numpy()
        tx = tex[v].cpu().numpy()
        pose = None if poses is None else poses[v].cpu().numpy().reshape(4, 4)
        col, row, mask, P, C = sl_oracle.decode_triangulate(list(st), tx, calib, n_cols, n_rows, pose=pose)
        good = len(P) == len(d["xyz"]) and np.array_equal(d["bgr"], C)
        if good and fast:
            P32 = P.astype(np.float32)
            good = bool(np.all(np.abs(d["xyz"].astype(np.float64) - P) <= 1.02e-5 * np.abs(P) + 1e-30)) and \
                bool(np.isfinite(P32).all())
        elif good:
            good = np.array_equal(d["xyz"].view(np.uint32), P.astype(np.float32).view(np.uint32))
        if "col" in d:
            good = good and np.array_equal(d["col"], col) and np.array_equal(d["row"], row) and \
                np.array_equal(d["mask"], mask)
        notes.append({"view": int(v), "points": int(len(P)), "equal": bool(good)})
        ok = ok and good
    return ok, {"views": notes, "oracle_s": time.perf_counter() - t0,
                "what": "the last timed step's maps, mask, point count, xyz and BGR of views 0 and V-1 vs "
                        "oracle/sl_oracle.py on the same resident stacks: " +
                        ("xyz within 1.02e-5 rel (fast mode)" if fast else "xyz == float32(reference f64), bitwise")}


def path_bytes(H, W, read_planes, n_points, maps):
    """SURVEY.md §8(d), whole path per view: the stack planes the path reads
    (2 + 2(nc+nr) with maps; 2 + 2 nc for the cloud alone -- row planes are
    never read, sl_system.py:584-653 uses only col_map) + 3 B/px texture +
    15 B/point (f32 xyz + BGR) + 9 B/px col/row/mask maps when written."""
    px = H * W
    return read_planes * px + 3 * px + 15 * n_points + (9 * px if maps else 0)


def decode_bytes(H, W, read_planes, maps, decide):
    """Algorithmic bytes of one k_decode pass over a view: the stack planes it
    streams + the col/row int32 maps it writes (+ the mask map on the decide
    path, where k_decode applies the mask; else k_count writes it).  Its 2-byte
    per-pixel records and point bits for k_cloud are overhead, not counted."""
    return H * W * (read_planes + ((9 if decide else 8) if maps else 0))


def cpu_baseline(stack_h, tex_h, calib, budget_s):
    """Time the oracle (NumPy restatement of the reference path, 1 thread)."""
    from oracle import sl_oracle
    imgs = list(stack_h)
    px = stack_h.shape[1] * stack_h.shape[2]
    n, t0 = 0, time.perf_counter()
    while True:
        sl_oracle.decode_triangulate(imgs, tex_h, calib)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or el / n * (n + 1) > 1.5 * budget_s:
            break
    return n * px / el, n, el


_MP_VIEW = {}


def _mp_worker(args):
    """One process of the P-process CPU baseline: the oracle on the shared view
    until the deadline; -> views done."""
    deadline, = args
    from oracle import sl_oracle
    st, tx, calib = _MP_VIEW["st"], _MP_VIEW["tx"], _MP_VIEW["calib"]
    imgs = list(st)
    n = 0
    while time.time() < deadline or n == 0:
        sl_oracle.decode_triangulate(imgs, tx, calib)
        n += 1
    return n


def cpu_baseline_procs(stack_h, tex_h, calib, procs, budget_s):
    """The reference's parallelism for many views: one view
    per process, P processes (fork, before this process touches the GPU), each
    running the oracle until a common deadline -> (px/s, views, seconds)."""
    import multiprocessing as mp
    _MP_VIEW.update(st=stack_h, tx=tex_h, calib=calib)
    px = stack_h.shape[1] * stack_h.shape[2]
    ctx = mp.get_context("fork")
    with ctx.Pool(procs) as pool:
        t0 = time.time()
        counts = pool.map(_mp_worker, [(t0 + budget_s,)] * procs)
        el = time.time() - t0
    _MP_VIEW.clear()
    return sum(counts) * px / el, sum(counts), el


def host_info():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    share = os.environ.get("OMP_NUM_THREADS")
    return {"cpu_model": model, "host_cores": os.cpu_count(),
            "core_share": int(share) if share and share.isdigit() else None}


def cpu_view(cfg, cfg_idx, gv):
    """The CPU baseline's sample view (host arrays) and its calibration."""
    rig = synth.Rig(H=cfg["H"], W=cfg["W"], Wp=cfg["Wp"], Hp=cfg["Hp"])
    st, tx = synth.render_stack(rig, seed=1000 * cfg_idx + gv, include_rows=cfg["rows"],
                                view_deg=cfg["deg"] * gv, device="cpu")
    return st.numpy(), tx.numpy(), synth.make_calibration(rig, with_Nc=False)


def cpu_baseline_multi(a, cfg, cfg_idx):
    """Rank 0, N = 1, BEFORE the GPU is touched (the pool forks): the oracle on
    P processes, one view each, for the multi-view configs."""
    info = host_info()
    procs = a.cpu_procs if a.cpu_procs else (info["core_share"] or min(os.cpu_count() or 1, 16))
    if a.cpu_procs == 0 or procs <= 1 or not (cfg["views"] > 1 or a.cpu_procs):
        return None
    st, tx, calib = cpu_view(cfg, cfg_idx, 0)
    H, W = st.shape[1:]
    vp, np_, elp = cpu_baseline_procs(st, tx, calib, procs, a.cpu_seconds)
    return {"value": vp, "unit": "px/s", "cores": procs, "kind": "port",
            "sample": f"{np_} x {W}x{H} view(s) over {procs} processes (one view per process at a time), "
                      f"{elp:.1f} s"}


def cpu_baseline_single(a, cfg, cfg_idx, multi):
    """Rank 0, N = 1, AFTER the GPU measurement (so that ~12 s of CPU work and
    its garbage never sit in front of the timed window): the oracle (a NumPy
    restatement of the reference path, bit-exact to the fixtures the reference
    produced; oracle/sl_oracle.py) on one process."""
    st, tx, calib = cpu_view(cfg, cfg_idx, 0)
    H, W = st.shape[1:]
    v1, n1, el1 = cpu_baseline(st, tx, calib, a.cpu_seconds)
    out = {"value": v1, "unit": "px/s", "cores": 1, "kind": "port",
           "sample": f"{n1} x {W}x{H} view(s), {st.shape[0]} planes, oracle/sl_oracle.py "
                     f"(NumPy restatement, bit-exact to reference fixtures), 1 process, {el1:.1f} s",
           **host_info()}
    # the oracle / reference speed ratio measured on one host with identical
    # outputs (scripts/ref_vs_oracle_timing.py, build container): the
    # reference's own code would run at about value / ratio here
    ratio_f = os.path.join(REPO, "profiles", "r02_ref_vs_oracle_timing.json")
    if os.path.exists(ratio_f):
        try:
            case = {1: "c1", 2: "c2", 3: "c3", 4: "c2", 5: "c2"}[cfg_idx]
            r = next(x for x in json.load(open(ratio_f))["cases"] if x["case"].startswith(case))
            out["reference_estimate"] = {"value": v1 / r["oracle_over_reference_speed"], "unit": "px/s",
                                         "oracle_over_reference_speed": r["oracle_over_reference_speed"],
                                         "source": f"profiles/r02_ref_vs_oracle_timing.json ({r['case']})"}
        except (OSError, ValueError, KeyError, StopIteration):
            pass
    if multi is not None:
        out["multi_process"] = multi
    return out


def spread(us):
    """min / median / max (and the values, for short runs) of per-step µs."""
    if not us:
        return None
    d = {"min": min(us), "median": statistics.median(us), "max": max(us), "mean": sum(us) / len(us)}
    if len(us) <= 64:
        d["steps"] = [round(x, 1) for x in us]
    return d


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))  # this process never touches a GPU
    # launched by torch.distributed.run (any world size, 1 included): process
    # group, barrier + max-over-ranks timing and the gather all run
    world, rank, local, distributed = rank_env()
    if "WORLD_SIZE" in os.environ and world != a.gpus:
        sys.exit(f"bench.py: --gpus {a.gpus} disagrees with WORLD_SIZE={world}")
    if a.selftest:
        return selftest(a)
    if a.backend != "nccl":
        sys.exit("bench.py: --backend gloo is only for --selftest (the GPU bench gathers over RCCL)")
    cfg = CONFIGS[a.config]
    cfg_idx = int(a.config[1:])
    cpu_on = a.cpu_baseline and world == 1 and rank == 0
    cpu_multi = cpu_baseline_multi(a, cfg, cfg_idx) if cpu_on else None  # forks: before the GPU
    if distributed:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if distributed else 0)
    torch.cuda.set_device(dev)
    H, W, Wp, Hp, rows, maps = cfg["H"], cfg["W"], cfg["Wp"], cfg["Hp"], cfg["rows"], cfg["maps"]
    V_cfg = a.views or cfg["views"]
    if a.scaling == "strong" and V_cfg < world:
        sys.exit(f"bench.py: --scaling strong needs at least {world} views (got {V_cfg})")
    views = my_views(a.scaling, V_cfg, world, rank)
    V = len(views)
    V_total = V_cfg if a.scaling == "strong" else V_cfg * world
    rig = synth.Rig(H=H, W=W, Wp=Wp, Hp=Hp)
    calib = synth.make_calibration(rig, with_Nc=False)
    stack = None
    tex = torch.empty((V, H, W, 3), dtype=torch.uint8, device=dev)
    poses = torch.empty((V, 4, 4), dtype=torch.float64, device=dev) if cfg["pose"] else None
    for v in range(V):
        gv = views[v]  # global view index
        s, t = synth.render_stack(rig, seed=1000 * cfg_idx + gv, include_rows=rows,
                                  view_deg=cfg["deg"] * gv, device=dev)
        if stack is None:
            stack = torch.empty((V,) + tuple(s.shape), dtype=torch.uint8, device=dev)
        stack[v].copy_(s)
        tex[v].copy_(t)
        if poses is not None:
            poses[v].copy_(torch.from_numpy(synth.turntable_pose(cfg["deg"] * gv)))
        del s, t
    torch.cuda.empty_cache()
    n_planes = stack.shape[1]
    nc = synth.n_bits(Wp)
    read_planes = n_planes if maps else 2 + 2 * nc
    eng = core.Reconstructor(dev)
    eng.set_calibration(calib, H, W)
    eng.reserve(V, H * W)
    n_cols, n_rows = Wp, (Hp if rows else 1080)
    out = {}

    # the headline xyz mode: exact (the reference's f64 arithmetic) unless
    # --xyz fast; SL_XYZ_F32_FAST applies without a pose (include/slgpu.h)
    head_fast = a.xyz == "fast" and poses is None

    # --next-stats (default): the next step reads the same resident stack, and
    # each call names it (sl_stack_next), so a call's k_cloud also runs the next
    # call's histogram pass and every call but the first starts with k_decode
    nxt = stack if a.next_stats else None

    def step(o, maps=maps, fast=head_fast):
        eng.decode_triangulate(stack, n_cols, n_rows, texture=tex, maps=maps, cloud=True,
                               xyz_dtype=torch.float32, poses=poses, fast_f32=fast, out=o, next_stack=nxt)
        return None

    # --streams S: core.ReconstructorPool, S contexts (own scratch, own
    # outputs) on one HIP stream each; step i runs on lane i % S.  S = 1: the
    # plain engine on the current stream
    S = max(1, a.streams if a.streams is not None else cfg.get("streams", 1))
    lane_prio = a.lane_priority if a.lane_priority is not None else cfg.get("lane_priority", 0)  # (explicit: the
    # pool's own default would give configs 3 lanes or more high priority as well)
    pool = None
    if S > 1:
        pool = core.ReconstructorPool(dev, lanes=S, reuse_outputs=True, stream_priority=lane_prio)
        pool.set_calibration(calib, H, W)
        pool.reserve(V, H * W)
        eng = pool.engines[0]
        if V > 1:
            out = pool._outs[0]

    # a stream of the bench's own (a graph capture needs a non-default
    # stream): one lane runs every step on it, so calls captured on it follow
    # the eager ones with no cross-stream hand-off; with lanes it is the
    # capture's origin, which the lane streams fork from and join
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    cur = torch.cuda.current_stream(dev)

    def drop_next_all():
        """sl_stack_next(NULL) on every context (a failed capture's queued passes never ran)."""
        for e in (pool.engines if pool is not None else [eng]):
            e.drop_next()

    # one view per step (V == 1): the steps cycle through the resident views
    # of ring["slots"] (slot 0 = the view above; --ring / --ring-control add
    # distinct ones, each with its own stack, texture and outputs), every call
    # naming its context's next stack (sl_stack_next).  With S lanes, step i
    # runs on lane i % S and the ring holds a multiple of S views, so a view's
    # outputs are always written by one lane, in order.
    ring_req = max(1, a.ring if a.ring is not None else cfg.get("ring", 1)) if V == 1 else 1
    ctl_req = 0
    ring_ctl = a.ring_control if a.ring_control is not None else cfg.get("ring_control", 3)
    if V == 1 and ring_ctl > 0:
        ctl_req = 1 if ring_req > 1 else ring_ctl  # the control: one view, or distinct ones
    slots = [dict(stack=stack, tex=tex, out=out)]  # the distinct resident views

    def ring_of(n):
        """The slots of a window over n distinct views: n rounded up to a
        multiple of S; one view: slot 0's stack and texture on every lane, each
        lane with outputs of its own."""
        if n <= 1:
            return [slots[0]] + [dict(stack=stack, tex=tex, out={}) for _ in range(1, S)]
        while len(slots) < S * -(-n // S):
            k = len(slots)
            s_, t_ = synth.render_stack(rig, seed=1000 * cfg_idx + 500 + k, include_rows=rows,
                                        view_deg=cfg["deg"] * (views[0] + 7 * k), device=dev)
            slots.append(dict(stack=s_[None].contiguous(), tex=t_[None].contiguous(), out={}))
            del s_, t_
        return slots[:S * -(-n // S)]

    head_slots = ring_of(ring_req) if V == 1 else []
    ctl_slots = ring_of(ctl_req) if ctl_req else []
    ring_R = len({sl["stack"].data_ptr() for sl in head_slots}) if V == 1 else 1
    ring = {"slots": head_slots, "i": 0}

    def one(at=None):
        """One step (the next, or step number ``at``: ring slot at % R, lane
        at % S); -> the stream it ran on."""
        if at is None:
            at = ring["i"]
            ring["i"] += 1
        if V == 1:
            act = ring["slots"]
            sl, nx = act[at % len(act)], act[(at + S) % len(act)]  # nx: this context's next call
            st_, tx_, o_, nx_ = sl["stack"], sl["tex"], sl["out"], nx["stack"] if a.next_stats else None
        else:
            st_, tx_, o_, nx_ = stack, tex, out, nxt
        if pool is None:
            eng.decode_triangulate(st_, n_cols, n_rows, texture=tx_, maps=maps, cloud=True,
                                   xyz_dtype=torch.float32, poses=poses, fast_f32=head_fast, out=o_,
                                   next_stack=nx_)
            return cur
        # resident inputs (wait_inputs=False); one view: its own outputs, else
        # the lane's (never read while the window runs)
        res = pool.decode_triangulate(st_, n_cols, n_rows, texture=tx_, maps=maps, cloud=True,
                                      xyz_dtype=torch.float32, poses=poses, fast_f32=head_fast,
                                      wait_inputs=False, lane=at % S, next_stack=nx_, prepared=True,
                                      **({"out": o_} if V == 1 else {}))
        return res["stream"]

    def run_steps(k):
        for _ in range(k):
            one()

    def sync_all():
        torch.cuda.synchronize(dev)

    for act in ([ctl_slots] if ctl_slots else []) + [head_slots]:  # every slot's outputs allocated before any window
        ring["slots"], ring["i"] = act, 0
        run_steps(max(a.warmup, S, len(act)))
    sync_all()
    if V == 1:
        out = slots[0]["out"]
    # points per step: the mean over the views the headline cycles through
    n_pts = (sum(int(sl["out"]["view_offsets"][-1].item()) for sl in head_slots) / len(head_slots)
             if V == 1 else int(out["view_offsets"][-1].item()))

    def end_on_slot0(k):
        """The next k steps end on slot 0 (whose outputs the verified sample copies)."""
        if V == 1:
            ring["i"] = (1 - k) % len(ring["slots"])

    def timed(k, evs=None):
        """K steps between barrier + synchronize pairs; with ``evs`` (k+1
        HIP events), one event per step boundary on the step's stream ->
        (seconds, per-step µs or None)."""
        if distributed:
            dist.barrier()
        sync_all()
        t0 = time.perf_counter()
        if evs:
            evs[0].record(cur if pool is None else pool.streams[ring["i"] % S])
        for i in range(k):
            st = one()
            if evs:
                evs[i + 1].record(st)
        t_enq = time.perf_counter()
        sync_all()
        # this rank's K steps are complete here; the closing barrier's own
        # latency stays out of the interval (the max over ranks covers skew)
        el = time.perf_counter() - t0
        us = None
        if evs:
            # completion times from the window's first event; with several
            # lanes (--streams) steps complete on different streams, so the
            # per-step intervals are those of the sorted completion times
            tc = sorted(evs[0].elapsed_time(evs[i + 1]) for i in range(k))
            us = [1e3 * (b - a_) for a_, b in zip([0.0] + tc[:-1], tc)]
        host_enq_ms[0] = 1e3 * (t_enq - t0)
        return el, us

    host_enq_ms = [None]

    def timed_graph(k):
        """The headline window as one hipGraph launch (one lane): the K steps
        are captured first (untimed; the library's calls enqueue into the
        graph exactly as onto the stream, host-side state advancing as for K
        calls), then the graph is launched once between barrier + synchronize
        pairs.  -> (seconds, graph, capture ms)."""
        g = torch.cuda.CUDAGraph()
        t_c = time.perf_counter()
        # thread-local capture: other threads' calls (RCCL's proxy threads) are not disturbed
        with torch.cuda.graph(g, stream=cur, capture_error_mode="thread_local"):
            for _ in range(k):
                one()
        cap_ms = 1e3 * (time.perf_counter() - t_c)
        if distributed:
            dist.barrier()
        sync_all()
        t0 = time.perf_counter()
        g.replay()
        t_enq = time.perf_counter()
        sync_all()
        el = time.perf_counter() - t0
        host_enq_ms[0] = 1e3 * (t_enq - t0)
        return el, g, cap_ms

    def preroll(ms):
        """Back-to-back steps for ``ms`` of wall time (a sync every 16 steps)."""
        n, t_pr = 0, time.perf_counter()
        while (time.perf_counter() - t_pr) * 1e3 < ms:
            run_steps(16)
            sync_all()
            n += 16
        return {"ms": 1e3 * (time.perf_counter() - t_pr), "steps": n}

    # The timed window follows the declared pre-roll with no idle gap: the
    # garbage collection and the event objects come before it.  (Measured,
    # rocprofv3 kernel trace of this command: after ~37 ms of idle GPU the
    # latency-bound k_cloud runs 10-25 % slower for the next ~20-30 ms of
    # load -- the chip's clock ramp -- so a window that opens after an idle
    # gap times the ramp, which is what the round-2 driver line showed.)
    # Per-step HIP events cost ~5.7 us of GPU idle per step (same trace), so
    # the headline window has none; an identical window with one event per
    # step boundary follows immediately and gives the per-step spread.
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    snap = snap_alloc(out, V, maps) if a.verify else None
    gc.collect()
    gc.disable()
    try:
        pre = preroll(a.preroll_ms)
        window = {"mode": "eager: K calls enqueued inside the window"}
        graph_keep = None
        end_on_slot0(a.steps)
        # with lanes the window is eager: captured, the lanes ran 3-5 % slower
        # at c2 (one graph forked and joined over the lane streams: 115.2-115.5
        # vs 109.2-110.1 us; one graph per lane: 118.3-118.6 vs 113.4-114.1 us;
        # profiles/r05_ab/lanes_graph_lines.jsonl), and the host enqueues the K
        # prepared calls in ~11 us each, far ahead of the GPU
        if a.graph and pool is None:
            try:
                el_rank, graph_keep, cap_ms = timed_graph(a.steps)
                window = {"mode": "hipGraph: the K steps captured after the pre-roll (untimed), launched once "
                                  "inside the window; every kernel of every step runs",
                          "capture_ms": cap_ms}
            except Exception as e:  # noqa: BLE001 -- capture unsupported here: the eager window instead
                window = {"mode": "eager (graph capture failed: %s)" % (str(e)[:160],)}
                torch.cuda.synchronize(dev)
                drop_next_all()  # the captured calls' queued passes never ran
                el_rank, _ = timed(a.steps)
        else:
            el_rank, _ = timed(a.steps)
        enq_ms = host_enq_ms[0]
        lane_snaps = []
        if snap is not None:  # the headline window's last step (the next window's sync waits for the copies)
            snap_copy(snap, out, cur)
            if V == 1:
                # and every other lane's last step: the window ends on slot 0
                # (lane 0), so lane j's last step ran slot (R - S + j) % R
                R_h = len(head_slots)
                for j in range(1, S):
                    k_s = (R_h - S + j) % R_h
                    sj = snap_alloc(head_slots[k_s]["out"], V, maps)
                    snap_copy(sj, head_slots[k_s]["out"], cur)
                    lane_snaps.append((j, k_s, sj))
        el_ev, step_us = timed(a.steps, evs)
        # the control window: the same K steps over ctl_R distinct resident
        # views (or one, when the headline cycles several), after its own
        # pre-roll, captured and launched as the headline -- do the 256 MB
        # Infinity Cache's hits on one view's texture, records and outputs
        # from step to step make the one-view headline faster?
        distinct = None
        if ctl_slots:
            ring["slots"] = ctl_slots
            pre2 = preroll(a.preroll_ms)
            end_on_slot0(a.steps)
            mode2 = "eager"
            if a.graph and pool is None:
                try:
                    el_ctl, graph_keep2, _ = timed_graph(a.steps)
                    mode2 = "hipGraph, as the headline"
                except Exception as e:  # noqa: BLE001
                    torch.cuda.synchronize(dev)
                    drop_next_all()
                    el_ctl, _ = timed(a.steps)
                    mode2 = "eager (graph capture failed: %s)" % (str(e)[:120],)
            else:
                el_ctl, _ = timed(a.steps)
            snap2 = snap_alloc(out, V, maps) if snap is not None else None
            if snap2 is not None:
                snap_copy(snap2, out, cur)
            ctl_views = len({sl["stack"].data_ptr() for sl in ctl_slots})
            resident = sum(sl["stack"].numel() + sl["tex"].numel() for sl in ctl_slots[:ctl_views])
            distinct = {"views": ctl_views, "ms_per_step": 1e3 * el_ctl / a.steps, "window": mode2,
                        "preroll": pre2, "resident_input_bytes": int(resident), "snap": snap2}
            ring["slots"] = head_slots
    finally:
        gc.enable()
    t = torch.tensor([el_rank], dtype=torch.float64, device=dev)
    if distributed:
        dist.barrier()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())

    # multi-rank facts + the timed gather of the clouds to rank 0
    n_loc = int(out["view_offsets"][-1].item())
    if distributed and a.gather == "native":
        def gfn():
            _, _, counts = parallel.gather_cloud_native(eng, out["xyz"][:n_loc], out["bgr"][:n_loc], dst=0)
            return counts
    else:
        def gfn():
            _, _, counts = parallel.gather_cloud(out["xyz"][:n_loc], out["bgr"][:n_loc], dst=0)
            return counts
    multi = gather_report(el_rank, n_loc, 15, dev, gfn, distributed)
    if distributed:
        multi["gather_path"] = ("sl_gather (the library's RCCL communicator)" if a.gather == "native"
                                else "torch.distributed batch_isend_irecv (RCCL)")
    if distributed and a.strong_leg and not (a.config == "c3" and a.scaling == "strong"):
        multi["strong_c3"] = strong_leg_report(a, world, rank, distributed, dev, 1920 * 1080,
                                               lambda views3: run_c3_leg(a, dev, views3))

    # per-kernel time: HIP events recorded by the library on the launch stream
    # around k_stats / k_decode / k_cloud, in a separate pass (events between
    # kernels add gaps, so they stay out of the timed loop above)
    eng.profile_enable(a.steps)
    for _ in range(a.steps):
        step(out)
    decode_ms, count_ms, cloud_ms, nl = eng.profile_read()
    eng.sync()
    # k_decode's launch duration for the roofline: the last step's last launch
    # group re-run back to back between two HIP events on its stream (the
    # events' own cost amortised; the per-step events above include it).  Its
    # stack is larger than the 256 MB Infinity Cache, so the re-runs stream
    # from HBM like the steps (rocprofv3's per-dispatch average agrees)
    path_kind, n_groups, last_px = eng.last_launch_info()  # the launch group time_kernels re-runs
    decide = path_kind == 1  # [k_stats] + k_decode (mask + point decision) + k_cloud
    v_last = last_px // (H * W)                 # views in the timed (last) group
    t_dec, t_cnt, t_cld = eng.time_kernels(max(a.steps, 10))

    def loop_s(k, **kw):
        """A secondary window: its own short pre-roll (the same clock-ramp
        reason), then k steps."""
        o2 = {}
        t_pr = time.perf_counter()
        while (time.perf_counter() - t_pr) * 1e3 < min(a.preroll_ms, 100.0):
            for _ in range(16):
                step(o2, **kw)
            sync_all()
        t1 = time.perf_counter()
        for _ in range(k):
            step(o2, **kw)
        sync_all()
        return time.perf_counter() - t1, o2

    # secondary (maps configs): cloud-only mode (what generate_cloud runs: row planes unread)
    el_cloud = None
    if maps and a.secondary:
        el_cloud, o2 = loop_s(a.steps, maps=False)
        del o2

    # secondary: the other xyz mode (exact <-> fast), same workload
    alt = None
    if poses is None and a.secondary:
        el_alt, o3 = loop_s(a.steps, fast=not head_fast)
        eng.profile_enable(a.steps)
        for _ in range(a.steps):
            step(o3, fast=not head_fast)
        _, _, acloud_ms, anl = eng.profile_read()
        eng.sync()
        alt = {"xyz_mode": XYZ_MODES[not head_fast], "px_per_s": V_total * H * W * a.steps / el_alt,
               "ms_per_step": 1e3 * el_alt / a.steps, "k_cloud_ms": acloud_ms / max(anl, 1),
               "note": "secondary: never the headline" if not head_fast else "the reference's arithmetic"}
        del o3

    # one-shot latency: the config's call as the GUI makes it (unchained, one
    # at a time), and config 1's single view beside a config-2 run
    shots = None
    if a.single_shot > 0 and rank == 0:
        e1, s1 = (eng, cur) if pool is None else (pool.engines[0], pool.streams[0])
        o_ss = out  # (its verified sample was copied out after the headline window)

        def call_cfg():
            e1.decode_triangulate(stack, n_cols, n_rows, texture=tex, maps=maps, cloud=True,
                                  xyz_dtype=torch.float32, poses=poses, fast_f32=head_fast, out=o_ss, stream=s1)
        shots = {a.config: single_shot(e1, call_cfg, a.single_shot, s1)}
        if a.config == "c2":
            shots["c1"] = single_shot_c1(dev, a.single_shot, cur)
        shots["note"] = ("isolated calls (synchronize, one unchained call with its own k_stats, synchronize), "
                         "stacks resident; wall_us = host enqueue + GPU + sync latency, gpu_us = HIP events "
                         "around the call on its stream; the headline instead streams chained calls")
        del o_ss

    verified, verification = None, None
    if snap is not None:
        verified, verification = verify(snap, stack, tex, poses, calib, n_cols, n_rows, head_fast)
        if V == 1:
            # one ring slot per lane: lane 0's last step (slot 0, above) and
            # every other lane's, each against the oracle on its own resident view
            lanes_v = [{"lane": 0, "slot": 0, "views": verification["views"]}]
            for j, k_s, sj in lane_snaps:
                okj, verj = verify(sj, head_slots[k_s]["stack"], head_slots[k_s]["tex"], poses, calib, n_cols,
                                   n_rows, head_fast)
                lanes_v.append({"lane": j, "slot": k_s, "views": verj["views"]})
                verified = verified and okj
            verification["lane_slots"] = lanes_v
        if distinct is not None and distinct.get("snap") is not None:
            ok2, ver2 = verify(distinct["snap"], stack, tex, poses, calib, n_cols, n_rows, head_fast)
            verification["distinct_views_window"] = ver2
            verified = verified and ok2
        if distributed:
            f = torch.tensor([1 if verified else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(f, op=dist.ReduceOp.MIN)
            verified = bool(f.item())
            verification["ranks"] = world

    cpu = cpu_baseline_single(a, cfg, cfg_idx, cpu_multi) if cpu_on else None

    if rank == 0:
        px_step = V_total * H * W  # whole job: every rank's views
        value = px_step * a.steps / el
        # the re-run figure only where the group's stack exceeds the 256 MB
        # Infinity Cache (else the re-runs would read it warm): in-step events
        rerun_ok = H * W * read_planes * v_last > 256 * 2 ** 20
        dec_avg_ms = t_dec if rerun_ok else decode_ms / max(nl, 1)
        v_roof = v_last if rerun_ok else V
        ab = decode_bytes(H, W, read_planes, maps, decide) * v_roof
        achieved = ab / (dec_avg_ms * 1e-3) / 1e9
        path_b = path_bytes(H, W, read_planes, n_pts / V, maps) * V
        path_gbps = path_b / (el / a.steps) / 1e9
        # PMC bytes (rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md)
        # of the same command, from a committed profile -- not measured here
        traffic = traffic_k = None
        if a.traffic is None:
            a.traffic = os.path.join(REPO, TRAFFIC_DIR, f"traffic_{a.config}.json")
        if os.path.exists(a.traffic):
            try:
                tj = json.load(open(a.traffic))
                if tj.get("config") == a.config and tj.get("views") == V and tj.get("decide", False) == decide \
                        and tj.get("xyz") == ("fast" if head_fast else "exact") and tj.get("ring", 1) == ring_R:
                    traffic = tj.get("bytes_per_step")
                    traffic_k = tj.get("kernels", {}).get("k_decode")  # per step: all its launches
                    if traffic_k is not None:
                        traffic_k *= v_roof / V  # per launch, as achieved / algorithmic_bytes_per_launch
            except (OSError, ValueError):
                traffic = traffic_k = None
        slots = ("k_decode", "k_stats", "k_cloud") if decide else ("k_decode", "k_count", "k_cloud")
        res = {
            "metric": "decoded+triangulated px/s",
            "value": value,
            "unit": "px/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": 1e3 * el / a.steps,
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": None,
            "dtype": "u8+f32" if head_fast else "u8+f64",
            "data": "synthetic",
            "config": {"workload": f"BASELINE config {cfg_idx}: {V} x {W}x{H} view(s) per GPU per step ({a.scaling} scaling, {V_total} in all), "
                                   f"{n_planes}-plane stacks (Gray {nc}+{n_planes // 2 - 1 - nc} bits + inverses), "
                                   + ("col/row/mask maps + " if maps else "")
                                   + "fp32 xyz/BGR cloud" + (" with turntable pose" if poses is not None else "")
                                   + (f"; the steps cycle through {ring_R} distinct resident views (chained)"
                                      if ring_R > 1 else ""),
                       "views_per_gpu": V, "views_total": V_total, "H": H, "W": W, "projector": f"{Wp}x{Hp}",
                       "parallelism": f"views sharded over {world} GPU(s)", "streams_per_gpu": S,
                       "lane_stream_priority": lane_prio if S > 1 else None,
                       "next_stats": bool(a.next_stats)},
            "timing": {"preroll": pre,
                       "step_us": spread(step_us),
                       "step_us_note": "HIP events at every step boundary, on the step's stream; intervals "
                                       "between the sorted completion times (several lanes: steps complete on "
                                       "different streams), in an identical window right after the timed one "
                                       "(the events add ~5.7 us of idle per step: not in the headline window)",
                       "ms_per_step_with_events": 1e3 * el_ev / a.steps,
                       "window": window,
                       "host_enqueue_ms": enq_ms,
                       "host_enqueue_note": "host time to enqueue the headline window's K steps (of its wall "
                                            "time): close to the wall time = the host, not the GPU, set the pace",
                       "gc": "collected before the pre-roll, disabled through the windows",
                       "ring_views": ring_R,
                       "distinct_views": None if distinct is None else {
                           "views": distinct["views"], "ms_per_step": distinct["ms_per_step"],
                           "ratio_to_headline": distinct["ms_per_step"] / (1e3 * el / a.steps),
                           "window": distinct["window"], "preroll": distinct["preroll"],
                           "resident_input_bytes": distinct["resident_input_bytes"],
                           "note": "the same K chained steps cycling through this many distinct resident views "
                                   "(stack, texture and outputs each), after their own pre-roll"
                                   + ("; one view: what of its texture, records and outputs the 256 MiB "
                                      "Infinity Cache keeps may serve the next step" if distinct["views"] == 1
                                      else "; their inputs exceed the 256 MiB Infinity Cache, so no line of a "
                                           "view's inputs survives to its next step"
                                      if distinct["resident_input_bytes"] > 2 ** 28
                                      else "; their inputs fit the 256 MiB Infinity Cache, so the control does "
                                           "not exclude cache hits from step to step")
                                   + "; verified like the headline (verification.distinct_views_window)"}},
            "roofline": {"bound": "hbm", "scope": "whole path per step: every kernel of the step",
                         "achieved": path_gbps, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": path_gbps / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": (f"PMC, {os.path.relpath(a.traffic, REPO)} (committed rocprofv3 "
                                            "FETCH_SIZE / WRITE_SIZE passes of this step's kernels, per step, "
                                            "each counter calibrated on known byte counts of the kernels' "
                                            "access widths: scripts/micro/store_calib)")
                                           if traffic is not None else None,
                         "algorithmic_bytes_per_step": path_b,
                         "bytes_note": f"SURVEY.md 8(d): {read_planes} stack planes read + 3 B/px BGR texture + "
                                       "15 B/point (f32 xyz + BGR)" + (" + 9 B/px col/row/mask maps" if maps else "")
                                       + "; time: the step's wall time (barrier + synchronize on both sides)",
                         "dominant_kernel": {
                             "name": "k_decode", "achieved": achieved, "frac": achieved / HBM_PEAK_GBS,
                             "avg_ms": dec_avg_ms, "algorithmic_bytes_per_launch": ab, "traffic": traffic_k,
                             "bytes_note": f"{read_planes} stack planes read"
                                           + ((" + col/row int32" + (" + mask" if decide else "") + " maps written")
                                              if maps else "")
                                           + f", per launch over {v_roof} view(s) (records, point bits are "
                                             "overhead); duration: "
                                           + ("HIP events around back-to-back re-runs of the launch "
                                              "(sl_time_kernels)" if rerun_ok
                                              else "HIP events around the kernel inside the steps"),
                             "lanes": S,
                             "lanes_note": None if S == 1 else (
                                 f"the window keeps {S} calls in flight on {S} streams, and their kernels run "
                                 "side by side: a rocprofv3 per-dispatch average of this command spans the time a "
                                 "launch shares the chip with the other lanes' launches (up to "
                                 f"{S}x this figure); --streams 1 gives the isolated dispatch (DESIGN.md 6.2)")}},
            "path": {"kind": ("k_decode (mask, point decision) + k_cloud (+ the next call's histogram pass: "
                              "sl_stack_next; the first call alone runs k_stats)" if a.next_stats
                              else "k_stats + k_decode (mask, point decision) + k_cloud") if decide
                             else "k_decode + k_count + k_cloud",
                     "launch_groups": n_groups,
                     "kernel_avg_ms": {slots[0]: decode_ms / max(nl, 1), slots[1]: count_ms / max(nl, 1),
                                       slots[2]: cloud_ms / max(nl, 1)},
                     "kernel_avg_ms_note": "HIP events around each kernel inside the steps (each event adds ~2-5 us)",
                     "rerun_ms_last_group": {slots[0]: t_dec, slots[1]: t_cnt, slots[2]: t_cld,
                                             "views": v_last,
                                             "note": "back-to-back re-runs (sl_time_kernels); the inputs of the "
                                                     "kernels after k_decode fit the 256 MB Infinity Cache, so "
                                                     "theirs run warm"}},
            "cpu_baseline": cpu,
            "verified": verified,
            "verification": verification,
            "single_shot": shots,
            "points_per_view": n_pts / V,
            "cloud_only_px_per_s": None if el_cloud is None else px_step * a.steps / el_cloud,
            "multi_gpu": multi,
            "xyz_mode": XYZ_MODES[head_fast],
            "alt_xyz_mode": alt,
        }
        print(json.dumps(res))
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

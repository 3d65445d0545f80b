"""The bench's steady state for PMC passes: N chained c2 steps (maps + exact
cloud, each call naming the next call's stack, sl_stack_next) on one
synthetic 4K view, nothing else on the GPU after set-up except the torch
copies of the rendering.  scripts/traffic_from_pmc.py --per-step N then
divides every step kernel's summed bytes by N (the first call's k_stats,
which no earlier call computed, is 1/N of a k_stats per step).

    python scripts/steps_app.py [--steps 40] [--no-next-stats] [--ring R] [--lanes S] [--views V --cloud-only]
                                [--config c1|c3|c4|c5]

--ring R (config 2, default 3 as bench.py): the steps cycle through R distinct
resident views (own stack, texture and outputs; R rounded up to a multiple of
the lanes), each naming its context's next stack.

--lanes S (default 2, as bench.py's configs 2-5): step i runs on lane i % S of
a core.ReconstructorPool (S contexts, one HIP stream each), as the bench does.

--views V --cloud-only: the multi-view configs' kernel shape instead (V 4K
views per call, cloud only: k_decode<11, 0, ...> and the exact k_cloud).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from structured_light_for_3d_model_replication_amd import core, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--no-next-stats", dest="next_stats", action="store_false", default=True)
ap.add_argument("--views", type=int, default=1)
ap.add_argument("--cloud-only", dest="cloud_only", action="store_true")
ap.add_argument("--poses", action="store_true", help="turntable poses (config 5's epilogue)")
ap.add_argument("--ring", type=int, default=3, help="config 2: distinct resident views cycled (bench.py --ring)")
ap.add_argument("--lanes", type=int, default=2, help="views in flight (bench.py --streams)")
ap.add_argument("--config", default=None,
                help="c1 / c3 / c4 / c5: that bench config's call (frame, views, cloud only, pose) instead "
         "(c1: one 1280x720 view, 1024-column projector, 22 planes, maps + cloud)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
H, W, deg, Wp, Hp, rows = 2160, 3840, 1.0, 1920, 1080, True
if a.config == "c1":  # bench.py CONFIGS["c1"]: one view, maps + cloud, the chain over one resident view
    H, W, Wp, Hp, rows, a.ring = 720, 1280, 1024, 768, False, 1
elif a.config:  # bench.py CONFIGS: one call = the config's views of one GPU
    H, W, a.views, deg = {"c3": (1080, 1920, 36, 10.0), "c4": (3000, 4000, 45, 1.0), "c5": (2160, 3840, 45, 1.0)}[a.config]
    a.cloud_only, a.poses = True, a.config == "c5"
rig = synth.Rig(H=H, W=W, Wp=Wp, Hp=Hp)
cal = synth.make_calibration(rig, with_Nc=False)
S = max(1, a.lanes)
R = S * -(-max(1, a.ring) // S) if a.views == 1 and a.config in (None, "c1") and a.ring > 1 else 1
ring = [synth.render_stack(rig, seed=3000 + k, view_deg=7.0 * k, include_rows=rows, device=dev) for k in range(1, R)]
views = [synth.render_stack(rig, seed=2000 + v, view_deg=deg * v, include_rows=rows, device=dev)
         for v in range(a.views)]
st = torch.stack([s_ for s_, _ in views]) if a.views > 1 else views[0][0]
tx = torch.stack([t_ for _, t_ in views]) if a.views > 1 else views[0][1]
del views
poses = None
if a.poses:
    import numpy as np
    poses = torch.from_numpy(np.stack([synth.turntable_pose(deg * v) for v in range(a.views)])).to(dev)
pool = core.ReconstructorPool(dev, lanes=S, reuse_outputs=True)
pool.set_calibration(cal, rig.H, rig.W)
slots = [(st, tx, {})] + [(s_, t_, {}) for s_, t_ in ring]
if R == 1:  # one view (the multi-view configs): every lane on it, each with its own outputs
    slots = [(st, tx, {}) for _ in range(S)]
torch.cuda.synchronize(dev)
for i in range(a.steps):
    s_, t_, o_ = slots[i % len(slots)]
    nxt = slots[(i + S) % len(slots)][0] if a.next_stats else None
    pool.decode_triangulate(s_, Wp, Hp, texture=t_, maps=not a.cloud_only, cloud=True, xyz_dtype=torch.float32,
                            out=o_, next_stack=nxt, poses=poses, wait_inputs=False, lane=i % S,
                            prepared=True)
pool.sync()
print(f"steps {a.steps} ring {R} lanes {S} points {int(slots[0][2]['view_offsets'][-1].item())}")

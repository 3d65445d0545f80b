"""Synthetic rig, calibration and Gray-code capture stacks.

Used by the benchmark, the parity tests and the golden-fixture generator to
produce inputs of the exact shape the reference consumes:

* ``make_calibration`` restates the pinhole camera rays and projector
  column/row planes of ``SLSystem.calibrate_final`` (server/sl_system.py:348-403)
  for a known synthetic rig, returning the same ``calib.mat`` fields
  (sl_system.py:406-415).
* ``render_stack`` ray-casts a sphere + orbiting bump + back wall, projects the
  hit points into the projector and forms the white / black / pattern / inverse
  images that ``capture_scan`` would record (patterns as in
  ``generate_patterns``, sl_system.py:44-86: bit 0 is the MSB of the Gray code).

Rendering runs in torch so the same code produces 4K stacks directly in HBM for
the benchmark and small CPU stacks for tests.  It is an input generator only;
nothing on the decode/triangulate path depends on it.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

PROJ_VALUE = 200  # server/config.py:20


def n_bits(n: int) -> int:
    """Bits of the Gray code for ``n`` stripes (sl_system.py:52-54, :538-539)."""
    return int(np.ceil(np.log2(n)))


@dataclass
class Rig:
    H: int                 # camera rows
    W: int                 # camera cols
    Wp: int = 1920         # projector cols
    Hp: int = 1080         # projector rows
    rot_y_deg: float = 15.0
    baseline_mm: float = 200.0

    @property
    def cam_K(self) -> np.ndarray:
        f = 0.9 * self.W
        return np.array([[f, 0.0, (self.W - 1) / 2.0],
                         [0.0, f, (self.H - 1) / 2.0],
                         [0.0, 0.0, 1.0]])

    @property
    def proj_K(self) -> np.ndarray:
        f = 0.8 * self.Wp
        return np.array([[f, 0.0, (self.Wp - 1) / 2.0],
                         [0.0, f, (self.Hp - 1) / 2.0],
                         [0.0, 0.0, 1.0]])

    @property
    def R(self) -> np.ndarray:
        a = math.radians(self.rot_y_deg)
        return np.array([[math.cos(a), 0.0, math.sin(a)],
                         [0.0, 1.0, 0.0],
                         [-math.sin(a), 0.0, math.cos(a)]])

    @property
    def T(self) -> np.ndarray:
        return np.array([[-self.baseline_mm], [0.0], [0.0]])


def make_calibration(rig: Rig, with_Nc: bool = True) -> dict:
    """calib.mat fields for ``rig`` following sl_system.py:348-415.

    ``Nc`` is built exactly as calibrate_final builds it (meshgrid, normalise
    along the last axis), so it is bit-identical to the pinhole fallback of
    reconstruct_point_cloud.  ``with_Nc=False`` stores a 3x1 placeholder, which
    makes the reference take its K-regeneration branch (sl_system.py:607-621).
    """
    h, w = rig.H, rig.W
    K1, K2, R, T = rig.cam_K, rig.proj_K, rig.R, rig.T
    if with_Nc:
        u, v = np.meshgrid(np.arange(w), np.arange(h))
        fx, fy, cx, cy = K1[0, 0], K1[1, 1], K1[0, 2], K1[1, 2]
        rays = np.stack(((u - cx) / fx, (v - cy) / fy, np.ones((h, w))), axis=2)
        rays /= np.linalg.norm(rays, axis=2, keepdims=True)
        Nc = rays.reshape(-1, 3).T
    else:
        Nc = np.zeros((3, 1))
    fxp, fyp, cxp, cyp = K2[0, 0], K2[1, 1], K2[0, 2], K2[1, 2]
    R_inv = R.T
    C_p = (-R_inv @ T).flatten()

    def plane(a_n, b_n):
        r1 = R_inv @ a_n
        r2 = R_inv @ b_n
        n = np.cross(r1.T, r2.T)
        n /= np.linalg.norm(n, axis=1, keepdims=True)
        d = -(n @ C_p)
        return np.concatenate([n, d[:, None]], axis=1)

    c = np.arange(rig.Wp, dtype=np.float64)
    ones = np.ones_like(c)
    col = plane(np.stack([(c - cxp) / fxp, (0 - cyp) / fyp * ones, ones]),
                np.stack([(c - cxp) / fxp, (rig.Hp - cyp) / fyp * ones, ones]))
    r = np.arange(rig.Hp, dtype=np.float64)
    ones = np.ones_like(r)
    row = plane(np.stack([(0 - cxp) / fxp * ones, (r - cyp) / fyp, ones]),
                np.stack([(rig.Wp - cxp) / fxp * ones, (r - cyp) / fyp, ones]))
    return {"Nc": Nc, "Oc": np.zeros((3, 1)), "wPlaneCol": col.T.copy(),
            "wPlaneRow": row.T.copy(), "cam_K": K1, "proj_K": K2, "R": R, "T": T}


def turntable_pose(angle_deg: float, center=(0.0, 0.0, 600.0)) -> np.ndarray:
    """4x4 pose that undoes a turntable rotation of ``angle_deg`` about the
    vertical axis through ``center`` (used by the config-5 merge epilogue)."""
    a = math.radians(-angle_deg)
    Ry = np.array([[math.cos(a), 0.0, math.sin(a)], [0.0, 1.0, 0.0],
                   [-math.sin(a), 0.0, math.cos(a)]])
    c = np.asarray(center, dtype=np.float64)
    M = np.eye(4)
    M[:3, :3] = Ry
    M[:3, 3] = c - Ry @ c
    return M


def _sphere_hit(o, d, center, radius):
    """Smallest positive ray parameter of |o + t d - c| = r (inf if none)."""
    oc = o - center
    b = (oc * d).sum(-1)
    cc = (oc * oc).sum(-1) - radius * radius
    disc = b * b - cc
    sq = torch.sqrt(torch.clamp(disc, min=0))
    t0 = -b - sq
    t1 = -b + sq
    t = torch.where(t0 > 1e-6, t0, t1)
    inf = torch.full_like(t, float("inf"))
    return torch.where((disc >= 0) & (t > 1e-6), t, inf)


def render_stack(rig: Rig, n_cols: int | None = None, n_rows: int | None = None,
                 view_deg: float = 0.0, seed: int = 0, device="cpu",
                 include_rows: bool = True, shadow_frac_scale: float = 1.0, scene: str = "default"):
    """Render one view's capture stack.

    Returns ``(stack uint8 [n_img,H,W], texture uint8 [H,W,3] BGR)`` on
    ``device`` with ``n_img = 2 + 2*(nc + nr)`` (nr = 0 if not include_rows).
    ``scene``: "default" (the SURVEY §8(d) scene: a sphere with a bump in front
    of a wall); "turntable" (no wall; two bumps fixed to the sphere, the whole
    object turned by ``view_deg`` about the vertical axis through its centre,
    so that turntable_pose(view_deg) maps every view back onto view 0 exactly:
    the registration tests' rigid, asymmetric object).
    """
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(int(seed))
    nc = n_bits(n_cols or rig.Wp)
    nr = n_bits(n_rows or rig.Hp) if include_rows else 0
    H, W = rig.H, rig.W
    f32 = torch.float32
    K = torch.tensor(rig.cam_K, dtype=f32, device=dev)
    v, u = torch.meshgrid(torch.arange(H, device=dev, dtype=f32),
                          torch.arange(W, device=dev, dtype=f32), indexing="ij")
    d = torch.stack([(u - K[0, 2]) / K[0, 0], (v - K[1, 2]) / K[1, 1], torch.ones_like(u)], -1)
    d = d / d.norm(dim=-1, keepdim=True)
    o = torch.zeros(3, device=dev, dtype=f32)

    center = torch.tensor([0.0, 0.0, 600.0], device=dev, dtype=f32)
    a = math.radians(view_deg)
    if scene == "turntable":
        ca, sa = math.cos(a), math.sin(a)
        spheres = [(center, 150.0)] + [
            (center + torch.tensor([ox * ca + oz * sa, oy, -ox * sa + oz * ca], device=dev, dtype=f32), r_)
            for (ox, oy, oz), r_ in (((110.0, -70.0, -60.0), 45.0), ((-60.0, 90.0, -100.0), 35.0))]
        t = torch.full_like(u, float("inf"))
    elif scene == "default":
        off = torch.tensor([110.0 * math.cos(a) - 0.0, -70.0, -110.0 * math.sin(a) - 60.0],
                           device=dev, dtype=f32)
        spheres = [(center, 150.0), (center + off, 45.0)]
        t = torch.where(d[..., 2] > 1e-6, 900.0 / d[..., 2], torch.full_like(u, float("inf")))  # the wall
    else:
        raise ValueError("scene must be 'default' or 'turntable'")
    for c_, r_ in spheres:
        t = torch.minimum(t, _sphere_hit(o, d, c_, r_))
    X = d * t[..., None]

    R = torch.tensor(rig.R, dtype=f32, device=dev)
    T = torch.tensor(rig.T.flatten(), dtype=f32, device=dev)
    Kp = torch.tensor(rig.proj_K, dtype=f32, device=dev)
    Xp = X @ R.T + T
    zp = Xp[..., 2]
    up = Kp[0, 0] * Xp[..., 0] / zp + Kp[0, 2]
    vp = Kp[1, 1] * Xp[..., 1] / zp + Kp[1, 2]
    col = torch.round(up)
    row = torch.round(vp)
    lit = (zp > 0) & (col >= 0) & (col < rig.Wp) & (row >= 0) & (row < rig.Hp) & torch.isfinite(t)
    # occlusion from the projector: segment C_p -> X blocked by a sphere
    Cp = torch.tensor((-rig.R.T @ rig.T).flatten(), dtype=f32, device=dev)
    seg = X - Cp
    dist = seg.norm(dim=-1)
    dirp = seg / dist[..., None].clamp(min=1e-6)
    for c_, r_ in spheres:
        th = _sphere_hit(Cp, dirp, c_, r_)
        lit &= ~(th < dist * (1 - 1e-3) - 0.5)
    col = torch.where(lit, col, torch.zeros_like(col)).to(torch.int64)
    row = torch.where(lit, row, torch.zeros_like(row)).to(torch.int64)

    albedo = 0.3 + 0.7 * torch.rand((H, W), generator=g, device=dev)
    ambient = torch.randint(0, 16, (H, W), generator=g, device=dev).to(f32)
    # a sparse set of pixels with white ~= black (shadow speckle)
    speckle = torch.rand((H, W), generator=g, device=dev) < 0.02 * shadow_frac_scale
    lit = lit & ~speckle
    amp = albedo * PROJ_VALUE * lit.to(f32)

    def shot(level):
        noise = torch.randn((H, W), generator=g, device=dev) * 2.0
        return torch.clamp(torch.round(level + ambient + noise), 0, 255).to(torch.uint8)

    planes = [shot(amp), shot(torch.zeros_like(amp))]
    for code, nb in ((col, nc), (row, nr)):
        gray = code ^ (code >> 1)
        for b in range(nb):
            bit = ((gray >> (nb - 1 - b)) & 1).to(f32)
            planes.append(shot(amp * bit))
            planes.append(shot(amp * (1 - bit)))
    stack = torch.stack(planes)
    tint = torch.stack([0.55 + 0.45 * torch.sin(u / 97.0) ** 2,      # B
                        0.6 + 0.4 * torch.cos(v / 61.0) ** 2,       # G
                        torch.full_like(u, 0.95)], -1)              # R
    tex = torch.clamp(torch.round(stack[0].to(f32)[..., None] * tint + 8.0), 0, 255).to(torch.uint8)
    return stack, tex

"""Generate the golden fixtures in this directory by running the REFERENCE's own
code on synthetic inputs.  Run in the build container only (it reads
/root/reference, which does not exist on the GPU box):

    python tests/golden/make_golden.py

How the reference is executed: the reference modules import packages this image
lacks (cv2, tkinter, flask_cors, pyserial), so the functions on the hot path are
taken from the reference's source files with ``ast`` -- the nested
``gray_decode`` / ``reconstruct_point_cloud`` and the ``generate_cloud`` method
of server/sl_system.py, and the module-level functions of
multi_point_cloud_process.py -- compiled unmodified and executed against NumPy,
SciPy, ``glob``/``os`` and a ``cv2`` namespace whose only member, ``imread``,
is an image *reader* (PIL for .png/.bmp files written by this script).  All
arithmetic executed is the reference's; the reader is I/O only.  For the
single-channel files written here ``imread(f, 0)`` is the identity and
``imread(f)`` replicates the channel three times, which is what cv2 returns.

Only inputs and outputs are stored (``*.npz``: arrays; ``*.ply``: text written
by the reference's own PLY writer).  No reference source or bytecode is kept.
"""
from __future__ import annotations

import ast
import glob
import json
import os
import shutil
import sys
import tempfile
import types

import numpy as np
import scipy.io
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

from structured_light_for_3d_model_replication_amd import synth  # noqa: E402


def _imread(path, flag=1):
    im = Image.open(path)
    a = np.asarray(im)
    if flag == 0:
        if a.ndim != 2:
            raise ValueError("fixtures only use single-channel files")
        return a.copy()
    if a.ndim == 2:
        return np.repeat(a[:, :, None], 3, axis=2)
    return a[:, :, ::-1].copy()


def _ns():
    cv2 = types.SimpleNamespace(imread=_imread)
    return {"np": np, "os": os, "glob": glob, "cv2": cv2, "scipy": scipy, "__name__": "ref"}


def _compile_defs(path, defs):
    mod = ast.Module(body=list(defs), type_ignores=[])
    ns = _ns()
    exec(compile(mod, path, "exec"), ns)
    return ns


def load_reference():
    """-> dict of callables taken from the reference source files."""
    p = os.path.join(REF, "server", "sl_system.py")
    tree = ast.parse(open(p, encoding="utf-8").read())
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "SLSystem")
    gen = next(n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name == "generate_cloud")
    nested = [n for n in gen.body if isinstance(n, ast.FunctionDef)]
    sl = _compile_defs(p, nested + [gen])
    p2 = os.path.join(REF, "multi_point_cloud_process.py")
    tree2 = ast.parse(open(p2, encoding="utf-8").read())
    want = {"load_calibration", "gray_decode", "reconstruct_point_cloud", "save_ply"}
    mp = _compile_defs(p2, [n for n in tree2.body if isinstance(n, ast.FunctionDef) and n.name in want])
    p3 = os.path.join(REF, "Old", "process_cloud.py")
    tree3 = ast.parse(open(p3, encoding="utf-8").read())
    cli = _compile_defs(p3, [n for n in tree3.body if isinstance(n, ast.FunctionDef) and n.name in want])
    return {
        "cli_load_calibration": cli["load_calibration"],
        "cli_gray_decode": cli["gray_decode"],
        "cli_reconstruct": cli["reconstruct_point_cloud"],
        "cli_save_ply": cli["save_ply"],
        "sl_gray_decode": sl["gray_decode"],
        "sl_reconstruct": sl["reconstruct_point_cloud"],
        "sl_generate_cloud": sl["generate_cloud"],
        "mp_gray_decode": mp["gray_decode"],
        "mp_reconstruct": mp["reconstruct_point_cloud"],
        "mp_save_ply": mp["save_ply"],
    }


def write_stack(folder, stack, ext=".png"):
    os.makedirs(folder, exist_ok=True)
    for i, im in enumerate(stack):
        Image.fromarray(np.ascontiguousarray(im)).save(os.path.join(folder, f"{i + 1:02d}{ext}"))


def calib_arrays(cal):
    return {f"calib_{k}": np.asarray(v) for k, v in cal.items()}


def save_case(name, meta, **arrays):
    np.savez_compressed(os.path.join(HERE, name + ".npz"), meta=json.dumps(meta), **arrays)
    print(f"  {name}: " + ", ".join(f"{k}{tuple(np.shape(v))}" for k, v in arrays.items() if k != "meta"))


def render(H, W, Wp, Hp, seed, include_rows=True, view=0.0):
    rig = synth.Rig(H=H, W=W, Wp=Wp, Hp=Hp)
    st, tex = synth.render_stack(rig, seed=seed, include_rows=include_rows, view_deg=view)
    return rig, st.numpy(), tex.numpy()


def run_sl(ref, tmp, name, stack, cal, n_cols, n_rows, texture=None):
    """Reference gray_decode (+ reconstruct) from sl_system on files in tmp."""
    folder = os.path.join(tmp, name)
    write_stack(folder, stack)
    col, row, mask, tex_ref = ref["sl_gray_decode"](folder, n_cols=n_cols, n_rows=n_rows)
    tex = tex_ref if texture is None else texture
    P, C = ref["sl_reconstruct"](col, row, mask, tex, cal)
    return col, row, mask, tex, P, C


def nonzero_oc_case(ref, tmp):
    """Oc != 0 with a per-pixel Nc table: the numerator np.dot(N.T, Oc) + d
    (sl_system.py:639) then depends on the BLAS's rounding order; the
    calibration goes through savemat/loadmat so the arrays have the layout
    the reference sees (loadmat's Fortran-ordered wPlaneCol)."""
    rig, st, _ = render(48, 64, 1920, 1080, seed=23)
    cal = synth.make_calibration(rig)
    cal["Oc"] = np.array([[12.5], [-3.25], [40.0]])
    mat = os.path.join(tmp, "calib_oc.mat")
    scipy.io.savemat(mat, cal)
    cal = {k: v for k, v in scipy.io.loadmat(mat).items() if not k.startswith("__")}
    col, row, mask, tex, P, C = run_sl(ref, tmp, "oc", st, cal, 1920, 1080)
    save_case("sl_nonzero_oc", {"mask_mode": "adaptive", "n_cols": 1920, "n_rows": 1080, "func": "sl"},
              stack=st, texture=tex, col_map=col, row_map=row, mask=mask, P=P, C=C, **calib_arrays(cal))


def cli_cases(ref, tmp):
    """Old/process_cloud.py's CLI: its __main__ sequence (:221-236) --
    load_calibration, gray_decode (fixed mask, the "Warning: Expected N
    pattern files" print), reconstruct_point_cloud, save_ply, "Done!" / the
    printed error -- run on a full stack, a short stack (warning, fewer bits),
    an odd file count (IndexError) and a missing calib file.  Stored: the
    stdout (folder paths as {DIR}) and the PLY text."""
    import contextlib
    import io as _io
    rig, st, _ = render(40, 56, 1920, 1080, seed=24)
    cal = synth.make_calibration(rig)
    mat = os.path.join(tmp, "cli_calib.mat")
    scipy.io.savemat(mat, cal)
    cases = {"full": st, "short": st[:12], "odd": st[:9], "nocalib": st}
    meta = {}
    arrays = {"stack": st, **calib_arrays(cal)}
    for name, stack in cases.items():
        folder = os.path.join(tmp, f"cli_{name}")
        write_stack(folder, stack, ext=".bmp")
        out = os.path.join(tmp, f"cli_{name}.ply")
        buf = _io.StringIO()
        with contextlib.redirect_stdout(buf):
            try:  # the __main__ block of Old/process_cloud.py, with its arguments
                calib_data = ref["cli_load_calibration"](mat if name != "nocalib" else mat + ".missing")
                c_map, r_map, mask, texture = ref["cli_gray_decode"](folder)
                points, colors = ref["cli_reconstruct"](c_map, r_map, mask, texture, calib_data)
                ref["cli_save_ply"](points, colors, out)
                print("Done!")
            except Exception as e:  # noqa: BLE001 -- the reference prints every error
                print(f"Error: {e}")
        meta[name] = {"files": int(len(stack)), "stdout": buf.getvalue().replace(tmp, "{DIR}")}
        if os.path.exists(out):
            shutil.copy(out, os.path.join(HERE, f"cli_process_cloud_{name}.ply"))
            meta[name]["ply"] = f"cli_process_cloud_{name}.ply"
    save_case("cli_process_cloud", {"func": "cli", "cases": meta}, **arrays)
    print("cli:", {k: v["stdout"].splitlines()[-1] for k, v in meta.items()})


def gui_stdout_cases(ref, tmp):
    """SLSystem.generate_cloud (server/sl_system.py:483-694, the GUI's "Generate
    .PLY", gui.py:563) run end to end on calib.mat + an image folder, with its
    stdout captured (folder paths as {DIR}) and the exception it raises: a full
    46-file stack, a short 12-file stack (fewer bits), a dangling odd file in
    the column sequence (IndexError), one in the row sequence, fewer than 4
    files (ValueError), a missing calib file (FileNotFoundError) and a calib
    file without 'Oc' (ValueError).  Stored: the stack, the calibration, and
    per case the file count, stdout, exception type and message."""
    import contextlib
    import io as _io
    rig, st, _ = render(36, 48, 1920, 1080, seed=25)
    cal = synth.make_calibration(rig)
    mat = os.path.join(tmp, "gui_calib.mat")
    scipy.io.savemat(mat, cal)
    mat_no_oc = os.path.join(tmp, "gui_calib_no_oc.mat")
    scipy.io.savemat(mat_no_oc, {k: v for k, v in cal.items() if k != "Oc"})
    cases = {"full": (46, "calib.mat"), "short": (12, "calib.mat"), "odd_cols": (9, "calib.mat"),
             "odd_rows": (31, "calib.mat"), "three": (3, "calib.mat"), "nocalib": (46, "missing.mat"),
             "no_oc": (46, "calib_no_oc.mat")}
    mats = {"calib.mat": mat, "missing.mat": mat + ".missing", "calib_no_oc.mat": mat_no_oc}
    meta = {}
    for name, (n_files, which) in cases.items():
        folder = os.path.join(tmp, f"gui_{name}")
        write_stack(folder, st[:n_files], ext=".bmp")
        buf = _io.StringIO()
        exc = None
        with contextlib.redirect_stdout(buf):
            try:
                ref["sl_generate_cloud"](None, folder, mats[which])
            except Exception as e:  # noqa: BLE001 -- recording the reference's exception
                exc = (type(e).__name__, str(e).replace(tmp, "{DIR}"))
        rec = {"files": n_files, "calib": which, "stdout": buf.getvalue().replace(tmp, "{DIR}"),
               "exception": exc}
        ply = os.path.join(folder, os.path.basename(folder) + ".ply")
        if os.path.exists(ply):
            shutil.copy(ply, os.path.join(HERE, f"sl_gui_stdout_{name}.ply"))
            rec["ply"] = f"sl_gui_stdout_{name}.ply"
        meta[name] = rec
    save_case("sl_gui_stdout", {"func": "gui_stdout", "cases": meta}, stack=st, **calib_arrays(cal))
    print("gui stdout:", {k: (v["stdout"].splitlines() or [""])[-1][:60] for k, v in meta.items()})


def main():
    ref = load_reference()
    tmp = tempfile.mkdtemp(prefix="golden_")
    if "--only-gui-stdout" in sys.argv:
        try:
            gui_stdout_cases(ref, tmp)
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
        return
    if "--only-cli" in sys.argv:
        try:
            cli_cases(ref, tmp)
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
        return
    if "--only-nonzero-oc" in sys.argv:  # add the one case without rewriting the others
        try:
            nonzero_oc_case(ref, tmp)
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
        return
    for f in glob.glob(os.path.join(HERE, "*.npz")) + glob.glob(os.path.join(HERE, "*.ply")):
        os.remove(f)
    try:
        # 1. generate_cloud end to end (GUI path): calib.mat -> decode -> PLY text
        rig, st, _ = render(48, 64, 1920, 1080, seed=11)
        cal = synth.make_calibration(rig)
        folder = os.path.join(tmp, "scan_e2e")
        write_stack(folder, st, ext=".bmp")
        mat = os.path.join(tmp, "calib.mat")
        scipy.io.savemat(mat, cal)
        ref["sl_generate_cloud"](None, folder, mat)
        shutil.copy(os.path.join(folder, "scan_e2e.ply"), os.path.join(HERE, "sl_generate_cloud_e2e.ply"))
        col, row, mask, tex, P, C = run_sl(ref, tmp, "e2e_dec", st, scipy.io.loadmat(mat), 1920, 1080)
        save_case("sl_generate_cloud_e2e", {"mask_mode": "adaptive", "n_cols": 1920, "n_rows": 1080,
                                            "func": "generate_cloud", "ply": "sl_generate_cloud_e2e.ply"},
                  stack=st, texture=tex, col_map=col, row_map=row, mask=mask, P=P, C=C,
                  **calib_arrays(cal))

        # 2..: sl_system gray_decode + reconstruct on assorted rigs / edge cases
        cases = [
            ("sl_1920x1080_noNc", dict(H=40, W=56, Wp=1920, Hp=1080, seed=12), 1920, 1080, False, True),
            ("sl_1024x768", dict(H=48, W=64, Wp=1024, Hp=768, seed=13), 1024, 768, True, True),
            ("sl_800x600", dict(H=32, W=48, Wp=800, Hp=600, seed=14), 800, 600, True, True),
            ("sl_c1_gui_defaults", dict(H=36, W=64, Wp=1024, Hp=768, seed=15), 1920, 1080, True, False),
            ("sl_c1_cols_only", dict(H=36, W=64, Wp=1024, Hp=768, seed=16), 1024, 768, True, False),
            ("sl_ragged_37x23", dict(H=23, W=37, Wp=1920, Hp=1080, seed=17), 1920, 1080, True, True),
            ("sl_tiny_proj_16x8", dict(H=20, W=32, Wp=16, Hp=8, seed=18), 16, 8, True, True),
        ]
        for name, rk, n_cols, n_rows, with_nc, rows in cases:
            rig, st, _ = render(rk["H"], rk["W"], rk["Wp"], rk["Hp"], rk["seed"], include_rows=rows)
            cal = synth.make_calibration(rig, with_Nc=with_nc)
            col, row, mask, tex, P, C = run_sl(ref, tmp, name, st, cal, n_cols, n_rows)
            save_case(name, {"mask_mode": "adaptive", "n_cols": n_cols, "n_rows": n_rows, "func": "sl"},
                      stack=st, texture=tex, col_map=col, row_map=row, mask=mask, P=P, C=C,
                      **calib_arrays(cal))

        # ties: quantised images so that p == i often (strict '>' -> bit 0)
        rig, st, _ = render(32, 48, 1920, 1080, seed=19)
        stq = (st // 24) * 24
        cal = synth.make_calibration(rig)
        col, row, mask, tex, P, C = run_sl(ref, tmp, "ties", stq, cal, 1920, 1080)
        save_case("sl_ties", {"mask_mode": "adaptive", "n_cols": 1920, "n_rows": 1080, "func": "sl"},
                  stack=stq, texture=tex, col_map=col, row_map=row, mask=mask, P=P, C=C, **calib_arrays(cal))

        # all-shadow (white == black: max contrast 0 -> empty mask) and inverted
        # contrast (white < black everywhere: negative dynamic range)
        for name, fn in (("sl_all_shadow", lambda s: np.concatenate([s[1:2], s[1:]])),
                         ("sl_negative_contrast", lambda s: np.concatenate([s[1:2] // 4, s[1:2], s[2:]]))):
            rig, st, _ = render(24, 32, 1920, 1080, seed=20)
            st2 = fn(st)
            cal = synth.make_calibration(rig)
            col, row, mask, tex, P, C = run_sl(ref, tmp, name, st2, cal, 1920, 1080)
            save_case(name, {"mask_mode": "adaptive", "n_cols": 1920, "n_rows": 1080, "func": "sl"},
                      stack=st2, texture=tex, col_map=col, row_map=row, mask=mask, P=P, C=C,
                      **calib_arrays(cal))

        # |denominator| straddling 1e-6: tilt chosen column planes so that the
        # plane normal is (nearly) orthogonal to the camera ray of some pixels.
        rig, st, _ = render(32, 48, 1920, 1080, seed=21)
        cal = synth.make_calibration(rig)
        folder = os.path.join(tmp, "den")
        write_stack(folder, st)
        col, row, mask, tex = ref["sl_gray_decode"](folder, n_cols=1920, n_rows=1080)
        planes = cal["wPlaneCol"].T.copy()
        idx = np.where(mask.ravel())[0]
        rays = cal["Nc"][:, idx]
        cols = np.clip(col.ravel()[idx], 0, planes.shape[0] - 1)
        rng = np.random.default_rng(5)
        eps_list = [0.0, 5e-7, -5e-7, 1e-6, -1e-6, 2e-6, 9.99e-7, 1.0000001e-6]
        used = set()
        for k, j in enumerate(rng.permutation(len(idx))):
            c = int(cols[j])
            if c in used:
                continue
            used.add(c)
            r = rays[:, j]
            n = planes[c, :3].copy()
            n = n - (n @ r) * r           # orthogonal to this pixel's ray
            n /= np.linalg.norm(n)
            e = eps_list[len(used) % len(eps_list)]
            n = n + e * r                  # n . r ~= e
            planes[c, :3] = n
            if len(used) >= 40:
                break
        cal["wPlaneCol"] = planes.T.copy()
        P, C = ref["sl_reconstruct"](col, row, mask, tex, cal)
        save_case("sl_denominator_edge", {"mask_mode": "adaptive", "n_cols": 1920, "n_rows": 1080, "func": "sl"},
                  stack=st, texture=tex, col_map=col, row_map=row, mask=mask, P=P, C=C, **calib_arrays(cal))

        # fixed-mask variant (multi_point_cloud_process.py) incl. its save_ply
        rig, st, _ = render(48, 64, 1024, 768, seed=22)
        cal = synth.make_calibration(rig)
        folder = os.path.join(tmp, "multi")
        write_stack(folder, st)
        col, row, mask, tex = ref["mp_gray_decode"](folder, n_cols=1024, n_rows=768)
        P, C = ref["mp_reconstruct"](col, row, mask, tex, cal)
        ref["mp_save_ply"](P, C, os.path.join(HERE, "mp_fixed_mask.ply"))
        save_case("mp_fixed_mask", {"mask_mode": "fixed", "n_cols": 1024, "n_rows": 768, "func": "mp",
                                    "ply": "mp_fixed_mask.ply"},
                  stack=st, texture=tex, col_map=col, row_map=row, mask=mask, P=P, C=C, **calib_arrays(cal))

        # reconstruct_point_cloud alone: colour texture, col codes past Wp (clip),
        # random mask
        rng = np.random.default_rng(7)
        H, W, Wp = 24, 40, 300
        rig = synth.Rig(H=H, W=W, Wp=Wp, Hp=200)
        cal = synth.make_calibration(rig)
        colm = rng.integers(0, 512, (H, W)).astype(np.int32)
        rowm = rng.integers(0, 256, (H, W)).astype(np.int32)
        maskm = rng.random((H, W)) < 0.7
        texc = rng.integers(0, 256, (H, W, 3)).astype(np.uint8)
        P, C = ref["sl_reconstruct"](colm, rowm, maskm, texc, cal)
        save_case("sl_reconstruct_colour_clip", {"func": "reconstruct"}, col_map=colm, row_map=rowm,
                  mask=maskm, texture=texc, P=P, C=C, **calib_arrays(cal))

        # adaptive-threshold pins: np.percentile of awkward sizes / distributions
        masks = {}
        for k, (h, w, kind) in enumerate([(7, 13, "u"), (17, 33, "u"), (48, 64, "lowamb"),
                                          (61, 59, "spiky"), (101, 103, "const"), (5, 9, "u"),
                                          (128, 96, "u"), (3, 3, "u"), (40, 41, "bimodal")]):
            rng = np.random.default_rng(100 + k)
            if kind == "u":
                black = rng.integers(0, 256, (h, w))
            elif kind == "lowamb":
                black = rng.integers(0, 16, (h, w))
            elif kind == "spiky":
                black = np.where(rng.random((h, w)) < 0.06, 250, rng.integers(0, 8, (h, w)))
            elif kind == "const":
                black = np.full((h, w), 37)
            else:
                black = np.where(rng.random((h, w)) < 0.5, 10, 200)
            white = np.clip(black + rng.integers(-30, 220, (h, w)), 0, 255)
            black = black.astype(np.uint8)
            white = white.astype(np.uint8)
            stack = np.stack([white, black, white, black])     # 4 files (minimum)
            folder = os.path.join(tmp, f"pct{k}")
            write_stack(folder, stack)
            col, row, mask, _ = ref["sl_gray_decode"](folder, n_cols=2, n_rows=2)
            masks[f"white_{k}"] = white
            masks[f"black_{k}"] = black
            masks[f"mask_{k}"] = mask
            masks[f"nf_{k}"] = np.float32(np.percentile(black.astype(np.float32), 95))
        save_case("adaptive_threshold_pins", {"n": 9}, **masks)

        # error behaviour: < 4 files -> ValueError; odd file reached -> IndexError
        errs = {}
        rig, st, _ = render(8, 16, 16, 8, seed=30)
        for n_img, tag in ((3, "three"), (9, "odd9"), (15, "odd15")):
            folder = os.path.join(tmp, f"err_{tag}")
            write_stack(folder, st[:n_img])
            try:
                ref["sl_gray_decode"](folder, n_cols=16, n_rows=8)
                errs[tag] = "ok"
            except Exception as e:  # noqa: BLE001 -- recording the reference's exception type
                errs[tag] = type(e).__name__
        save_case("errors", {"errors": errs, "n_cols": 16, "n_rows": 8}, stack=st)
        print("errors:", errs)
        nonzero_oc_case(ref, tmp)
        cli_cases(ref, tmp)
        gui_stdout_cases(ref, tmp)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()

"""Capture-stack ingest: file discovery and image decoding on the host.

Mirrors the file handling of gray_decode (server/sl_system.py:510-520, 556-557,
580): ``sorted(glob('*.bmp'))``, falling back to ``*.png``; every image read as
8-bit gray (``cv2.imread(f, 0)``) and file 0 re-read in colour (BGR) for the
texture.

OpenCV is not available in this image, so decoding uses Pillow.  For
single-channel files (what the fixtures and the synthetic rig produce) gray is
the identity and colour is the channel replicated three times, exactly what
cv2 returns.  Colour files are converted with OpenCV's fixed-point BT.601
weights ``(1868 B + 9617 G + 4899 R + 8192) >> 14``.  JPEG payloads saved under a
.bmp name (server/server.py:70) decode through Pillow's libjpeg, whose output
is not pinned against OpenCV's: parity for such captures is unpinned.
"""
from __future__ import annotations

import glob
import os
import threading

import numpy as np
from PIL import Image


def list_stack_files(folder: str) -> list[str]:
    files = sorted(glob.glob(os.path.join(folder, "*.bmp")))
    if not files:
        files = sorted(glob.glob(os.path.join(folder, "*.png")))
    return files


def _rgb_to_gray_cv(rgb: np.ndarray) -> np.ndarray:
    r = rgb[..., 0].astype(np.int32)
    g = rgb[..., 1].astype(np.int32)
    b = rgb[..., 2].astype(np.int32)
    return ((1868 * b + 9617 * g + 4899 * r + 8192) >> 14).astype(np.uint8)


def imread_gray(path: str) -> np.ndarray:
    """cv2.imread(path, 0) equivalent (uint8 H x W)."""
    with Image.open(path) as im:
        if im.mode == "L":
            return np.asarray(im).copy()
        if im.mode in ("I;16", "I", "F"):
            raise ValueError(f"{path}: unsupported high bit-depth image")
        return _rgb_to_gray_cv(np.asarray(im.convert("RGB")))


def imread_bgr(path: str) -> np.ndarray:
    """cv2.imread(path) equivalent (uint8 H x W x 3, BGR)."""
    with Image.open(path) as im:
        if im.mode == "L":
            a = np.asarray(im)
            return np.repeat(a[:, :, None], 3, axis=2)
        return np.ascontiguousarray(np.asarray(im.convert("RGB"))[:, :, ::-1])


def frame_size(path: str) -> tuple[int, int]:
    """(H, W) of an image file, from its header only."""
    with Image.open(path) as im:
        return im.size[1], im.size[0]


_POOL = None
_POOL_LOCK = threading.Lock()


def _pool(workers: int):
    global _POOL
    from concurrent.futures import ThreadPoolExecutor
    with _POOL_LOCK:
        if _POOL is None or _POOL._max_workers < workers:
            _POOL = ThreadPoolExecutor(max_workers=workers, thread_name_prefix="sl-ingest")
        return _POOL


def fill_stack(files: list[str], stack_out, tex_out, workers: int = 8) -> bool:
    """Decode files[0 : len(stack_out)] as gray straight into ``stack_out``
    (uint8 [n, H, W], e.g. a pinned tensor's numpy view) and file 0 in colour
    into ``tex_out`` [H, W, 3] BGR -- unless file 0 is single-channel, whose
    colour read is the gray plane replicated (cv2.imread): then ``tex_out`` is
    left untouched and True is returned (the caller may pass no texture)."""
    n = len(stack_out)
    if len(files) < n:
        raise ValueError(f"{len(files)} files for {n} planes")
    shape = tuple(stack_out.shape[1:])

    def one(j):
        a = imread_gray(files[j])
        if a.shape != shape:
            raise ValueError(f"{files[j]}: size {a.shape} differs from {shape}")
        stack_out[j] = a

    if workers > 1 and n > 1:
        list(_pool(workers).map(one, range(n)))
    else:
        for j in range(n):
            one(j)
    with Image.open(files[0]) as im:
        gray = im.mode == "L"
    if not gray:
        tex_out[...] = imread_bgr(files[0])
    return gray


def read_stack(folder: str, workers: int = 8):
    """-> (stack uint8 [n_img, H, W], texture uint8 [H, W, 3] BGR, files)."""
    files = list_stack_files(folder)
    if len(files) < 4:
        raise ValueError("Not enough images in folder to decode.")
    if workers > 1 and len(files) > 8:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=workers) as ex:
            planes = list(ex.map(imread_gray, files))
    else:
        planes = [imread_gray(f) for f in files]
    shape = planes[0].shape
    for f, p in zip(files, planes):
        if p.shape != shape:
            raise ValueError(f"{f}: size {p.shape} differs from {shape}")
    return np.stack(planes), imread_bgr(files[0]), files

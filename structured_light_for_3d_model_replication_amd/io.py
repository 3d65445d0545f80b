"""Capture-stack ingest: file discovery and image decoding on the host.

Mirrors the file handling of gray_decode (server/sl_system.py:510-520, 556-557,
580): ``sorted(glob('*.bmp'))``, falling back to ``*.png``; every image read as
8-bit gray (``cv2.imread(f, 0)``) and file 0 re-read in colour (BGR) for the
texture.

Uncompressed BMP files (the capture format the GUI saves, sl_system.py:519)
are read by ``read_bmp_gray`` straight from the file's pixel array: header
parse, then one strided copy of the rows (bottom-up rows flipped, the 4-byte
row padding dropped) -- checked byte for byte against Pillow's decoder in
tests/test_ingest.py.  Anything else (PNG, JPEG bytes under a .bmp name, RLE
BMPs) goes through Pillow.

OpenCV is not available in this image, so the other decoding uses Pillow.  For
single-channel files (what the fixtures and the synthetic rig produce) gray is
the identity and colour is the channel replicated three times, exactly what
cv2 returns.  Colour files are converted with OpenCV's fixed-point BT.601
weights ``(1868 B + 9617 G + 4899 R + 8192) >> 14``.  JPEG payloads (also the
ones saved under a .bmp name, server/server.py:70) are read as gray the way
cv2.imread(f, 0) reads them: libjpeg asked for grayscale output, i.e. the
decoded luma (Y) channel (Pillow's ``draft("L")``), with no colour
conversion -- 2-3x faster than decoding RGB and converting.  Pillow's libjpeg
is not pinned against OpenCV's (no cv2 here): parity for such captures is
unpinned.
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


_BMP_INFO = (40, 52, 56, 108, 124)  # BITMAPINFOHEADER and its V2..V5 extensions


def _bmp_layout(head: bytes):
    """(offset, H, W, bpp, bottom_up, palette_bgr | None) of an uncompressed
    8/24/32-bit BMP, from its first bytes, or None when the raw path does not
    apply (not 'BM', RLE / bitfield compression, other depths)."""
    if len(head) < 54 or head[:2] != b"BM":
        return None
    off = int.from_bytes(head[10:14], "little")
    dib = int.from_bytes(head[14:18], "little")
    if dib not in _BMP_INFO:
        return None
    W = int.from_bytes(head[18:22], "little", signed=True)
    H = int.from_bytes(head[22:26], "little", signed=True)
    planes = int.from_bytes(head[26:28], "little")
    bpp = int.from_bytes(head[28:30], "little")
    comp = int.from_bytes(head[30:34], "little")
    if planes != 1 or W <= 0 or H == 0 or bpp not in (8, 24, 32):
        return None
    if comp != 0 and not (comp == 3 and bpp == 32 and dib >= 52 and
                          head[54:66] == bytes.fromhex("0000ff0000ff0000ff000000")):
        return None  # BI_RGB, or BI_BITFIELDS with the default BGRx masks only
    pal = None
    if bpp == 8:
        n = int.from_bytes(head[46:50], "little") or 256
        p0 = 14 + dib
        if len(head) < p0 + 4 * n:
            return None
        pal = np.frombuffer(head, np.uint8, 4 * n, p0).reshape(n, 4)[:, :3]
    return off, abs(H), W, bpp, H > 0, pal


_TLS = threading.local()  # per decoding thread: a reused read buffer


def read_bmp_gray(path: str, out: np.ndarray | None = None) -> np.ndarray | None:
    """cv2.imread(path, 0) of an uncompressed BMP without a full decode:
    8-bit (palette mapped; gray palettes are the identity), 24/32-bit BGR(x)
    through OpenCV's fixed-point gray weights.  Writes into ``out`` (uint8
    [H, W]) when given.  None when the file is not such a BMP (the caller
    then decodes it with Pillow)."""
    with open(path, "rb") as f:
        head = f.read(14 + 124 + 1024)  # file header, largest info header, 256-entry palette
        lay = _bmp_layout(head)
        if lay is None:
            return None
        off, H, W, bpp, bottom_up, pal = lay
        bpr = W * bpp // 8
        stride = (bpr + 3) & ~3
        f.seek(off)
        # into this thread's reused buffer: a fresh 8-MB bytes object per file would be
        # page-faulted in (and zeroed) by the kernel every time
        need = stride * H
        buf = getattr(_TLS, "buf", None)
        if buf is None or len(buf) < need:
            buf = _TLS.buf = bytearray(need)
        mv = memoryview(buf)[:need]
        got = 0
        while got < need:
            k = f.readinto(mv[got:])
            if not k:
                break
            got += k
    if got < need - (stride - bpr):
        raise ValueError(f"{path}: truncated BMP pixel array")
    if got < need:
        mv[got:] = bytes(need - got)
    rows = np.frombuffer(buf, np.uint8, need).reshape(H, stride)[:, :bpr]
    if bottom_up:
        rows = rows[::-1]
    if out is None:
        out = np.empty((H, W), np.uint8)
    elif out.shape != (H, W):
        raise ValueError(f"{path}: size {(H, W)} differs from {tuple(out.shape)}")
    if bpp == 8:
        gray = pal[:, 0] if np.all(pal == pal[:, :1]) else _rgb_to_gray_cv(pal[:, ::-1])
        if len(gray) == 256 and np.array_equal(gray, np.arange(256, dtype=np.uint8)):
            out[...] = rows
        else:
            lut = np.zeros(256, np.uint8)
            lut[: len(gray)] = gray[:256]
            np.take(lut, rows, out=out)
    else:
        px = rows.reshape(H, W, bpp // 8)
        out[...] = _rgb_to_gray_cv(px[:, :, 2::-1])
    return out


def is_raw_bmp(path: str) -> bool:
    """An uncompressed BMP that read_bmp_gray reads without a decoder (a
    copy-bound read), as opposed to PNG / JPEG / RLE payloads (decode-bound)."""
    with open(path, "rb") as f:
        return _bmp_layout(f.read(14 + 124 + 1024)) is not None


def imread_gray(path: str, out: np.ndarray | None = None) -> np.ndarray:
    """cv2.imread(path, 0) equivalent (uint8 H x W)."""
    a = read_bmp_gray(path, out)
    if a is not None:
        return a
    with Image.open(path) as im:
        if im.format == "JPEG" and im.mode in ("RGB", "YCbCr"):
            # OpenCV's JPEG decoder with IMREAD_GRAYSCALE sets libjpeg's
            # out_color_space = JCS_GRAYSCALE: the luma plane as decoded
            im.draft("L", im.size)
        if im.mode == "L":
            return np.asarray(im).copy()
        if im.mode in ("I;16", "I", "F"):
            raise ValueError(f"{path}: unsupported high bit-depth image")
        return _rgb_to_gray_cv(np.asarray(im.convert("RGB")))


def imread_bgr(path: str, out: np.ndarray | None = None) -> np.ndarray:
    """cv2.imread(path) equivalent (uint8 H x W x 3, BGR), into ``out`` when
    given.  A colour file is decoded to RGB and packed as BGR by Pillow's raw
    packer (one pass in C; the same bytes as reversing the RGB channels)."""
    with Image.open(path) as im:
        if im.mode == "L":
            a = np.asarray(im)
            res = np.empty(a.shape + (3,), np.uint8) if out is None else out
            if res.shape != a.shape + (3,):
                raise ValueError(f"{path}: size {a.shape} differs from {tuple(res.shape[:2])}")
            res[...] = a[:, :, None]
            return res
        rgb = im if im.mode == "RGB" else im.convert("RGB")
        W, H = rgb.size
        buf = rgb.tobytes("raw", "BGR")
    a = np.frombuffer(buf, np.uint8).reshape(H, W, 3)
    if out is None:
        return a.copy()
    if out.shape != (H, W, 3):
        raise ValueError(f"{path}: size {(H, W)} differs from {tuple(out.shape[:2])}")
    out[...] = a
    return out


def frame_size(path: str) -> tuple[int, int]:
    """(H, W) of an image file, from its header only."""
    with Image.open(path) as im:
        return im.size[1], im.size[0]


_POOLS: dict = {}
_POOL_LOCK = threading.Lock()


def default_workers() -> int:
    """Decoding threads: the process's core share (OMP_NUM_THREADS, which the
    GPU box sets to its 16-core share; os.cpu_count() there is the whole
    machine's), at most 16.  Pillow's PNG and JPEG decoders release the GIL:
    16 threads decode a 4K view's 24 PNG files in 91 ms against 121 ms with 8
    (profiles/r02_ingest_mi355x_box.jsonl)."""
    share = os.environ.get("OMP_NUM_THREADS", "")
    n = int(share) if share.isdigit() and int(share) > 0 else (os.cpu_count() or 1)
    return max(1, min(16, n))


def _pool(workers: int):
    """A persistent pool of exactly ``workers`` decoding threads."""
    from concurrent.futures import ThreadPoolExecutor
    with _POOL_LOCK:
        if workers not in _POOLS:
            _POOLS[workers] = ThreadPoolExecutor(max_workers=workers, thread_name_prefix="sl-ingest")
        return _POOLS[workers]


def fill_stack(files: list[str], stack_out, tex_out, workers: int | None = None, on_plane=None) -> bool:
    """Decode files[0 : len(stack_out)] as gray straight into ``stack_out``
    (uint8 [n, H, W], e.g. a pinned tensor's numpy view) and file 0 in colour
    into ``tex_out`` [H, W, 3] BGR -- unless file 0 is single-channel, whose
    colour read is the gray plane replicated (cv2.imread): then ``tex_out`` is
    left untouched and True is returned (the caller may pass no texture).
    The colour decode (the longest task: a colour JPEG's RGB decode) starts
    first, beside the gray ones.  ``on_plane(j)`` is called, on the decoding
    thread, as soon as plane j is in ``stack_out`` (e.g. to start its upload)."""
    n = len(stack_out)
    workers = default_workers() if workers is None else workers
    if len(files) < n:
        raise ValueError(f"{len(files)} files for {n} planes")
    shape = tuple(stack_out.shape[1:])

    def one(j):
        dst = stack_out[j]
        a = imread_gray(files[j], dst)  # an uncompressed BMP is read straight into dst
        if a is not dst:
            if a.shape != shape:
                raise ValueError(f"{files[j]}: size {a.shape} differs from {shape}")
            dst[...] = a
        if on_plane is not None:
            on_plane(j)

    def colour():
        with Image.open(files[0]) as im:
            if im.mode == "L":
                return True
        imread_bgr(files[0], tex_out)
        return False

    if workers > 1 and n > 1:
        pool = _pool(workers)
        fc = pool.submit(colour)
        try:
            list(pool.map(one, range(n)))
        except BaseException:
            fc.exception()  # waited for: nothing writes tex_out after the call returns
            raise
        return fc.result()
    for j in range(n):
        one(j)
    return colour()


def read_stack(folder: str, workers: int | None = None):
    """-> (stack uint8 [n_img, H, W], texture uint8 [H, W, 3] BGR, files)."""
    workers = default_workers() if workers is None else workers
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

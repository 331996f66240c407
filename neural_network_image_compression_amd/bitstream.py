"""Bitstream container and directory drivers around the device codec.

The reference's on-disk bitstream is a PNG: the 96-channel u8 latent is reinterpreted
(raw C-order reshape per plane) as a 3-channel ``(n, 4h, 8w, 3)`` image
(``ProClass._feed_batch``, utils.py:30-44) and saved by Pillow with ``optimize=True``
(``save_img``, utils.py:85-87).  ``compress``/``uncompress`` walk a directory with
``read_dataset`` (utils.py:89-120) in batches of 4 (utils.py:46-62).

The pack/unpack reshape runs on the GPU (``nic_pack_latent``/``nic_unpack_latent``); PNG
coding (zlib) stays on the host, outside the measured encode/decode surface.
"""
from __future__ import annotations

import io
import os
from typing import List, Sequence, Tuple

import numpy as np

IMAGE_EXTS = ("png", "jpg", "jpeg", "gif", "pgm", "ppm", "bmp", "jp2")  # utils.py:94


def read_dataset(dataset_path: str) -> Tuple[List[np.ndarray], List[str]]:
    """utils.py:89-120: sorted directory listing, colour (3-D) images only, u8 arrays.

    Returns a list (images may differ in size; the reference's object-array path breaks
    under NumPy 2) and the file stems."""
    from PIL import Image

    imgs, names = [], []
    for fn in sorted(os.listdir(dataset_path)):
        if fn.split(".")[-1] in IMAGE_EXTS:
            with Image.open(os.path.join(dataset_path, fn)) as im:
                a = np.array(im)
            if a.ndim == 3:
                imgs.append(a.astype(np.uint8))
                names.append(".".join(fn.split(".")[:-1]))
    return imgs, names


def png_bytes(img: np.ndarray, optimize: bool = True) -> bytes:
    """Pillow PNG encoding as save_img (utils.py:87)."""
    from PIL import Image

    buf = io.BytesIO()
    Image.fromarray(img).save(buf, format="PNG", optimize=optimize)
    return buf.getvalue()


def png_sizes(images: np.ndarray, threads: int = 16) -> np.ndarray:
    """len(png_bytes(a)) of every u8 image a of images (M, H, W) or (M, H, W, 3), computed
    natively (nic_png_sizes: Pillow's row filters + zlib level 9 on host threads, no Python
    per image) -- byte for byte the size Pillow writes."""
    import ctypes

    from . import _lib

    a = np.ascontiguousarray(images, dtype=np.uint8)
    if a.ndim not in (3, 4) or (a.ndim == 4 and a.shape[3] != 3):
        raise ValueError(f"png_sizes: expected (M, H, W) or (M, H, W, 3) images, got shape {a.shape}")
    m, h, w = a.shape[:3]
    ch = 3 if a.ndim == 4 else 1
    out = np.empty(m, np.int64)
    if m:
        _lib.check(_lib.lib().nic_png_sizes(a.ctypes.data_as(ctypes.c_void_p), m, h, w, ch,
                                            out.ctypes.data_as(ctypes.c_void_p), int(threads)), "nic_png_sizes")
    return out


def save_img(img: np.ndarray, output_dir: str, filename: str) -> str:
    """utils.py:85-87."""
    assert (np.round(img) - img).sum() == 0
    path = os.path.join(output_dir, filename + ".png")
    with open(path, "wb") as f:
        f.write(png_bytes(np.asarray(img, dtype=np.uint8)))
    return path


def png_bpp(packed: np.ndarray, pixels: int, optimize: bool = True) -> float:
    """training.py:12-21 / training.py:157-163: 8 * len(PNG) / pixels of the original image."""
    return 8.0 * len(png_bytes(packed, optimize)) / float(pixels)


def _batches(shapes: Sequence[tuple], batch_size: int):
    """Consecutive runs of equal-shaped images, at most batch_size long (utils.py:53-62)."""
    i = 0
    while i < len(shapes):
        j = i + 1
        while j < len(shapes) and j - i < batch_size and shapes[j] == shapes[i]:
            j += 1
        yield i, j
        i = j


def feed_batch(model, x: np.ndarray, filenames: Sequence[str], output_dir: str, in_cshape: int,
               pool=None) -> list:
    """utils.py:30-44 for one batch: unpack (decoder side), run the codec, pack (encoder side), save.

    With a thread pool the PNG writes (zlib, which runs without the GIL inside Pillow) are
    submitted to it and their futures returned, so the caller can run the next batch on the
    GPU while this one is being compressed on the host cores."""
    import torch

    codec = model.codec
    dev = torch.from_numpy(np.ascontiguousarray(x)).to(f"cuda:{codec.device}")
    n, h, w, c = dev.shape
    if in_cshape == 96 and c == 3:
        dev = codec.unpack(dev)
    out = model._device_call(dev)
    if out.shape[-1] == 96:
        out = codec.pack(out)
    host = out.cpu().numpy()
    if pool is None:
        for i in range(host.shape[0]):
            save_img(np.squeeze(host[i]), output_dir, filenames[i])
        return []
    return [pool.submit(save_img, np.squeeze(host[i]), output_dir, filenames[i]) for i in range(host.shape[0])]


def use_model(model, dataset_path: str, checkpoint_path: str, output_dir: str, in_cshape: int,
              batch_size: int = 4, workers: int = 0) -> None:
    """utils.py:46-62.  ``workers`` > 0: PNG encoding (``save_img``, ~74 ms per 256^2 latent
    with optimize=True on one core) runs on that many host threads, overlapped with the
    device work of the following batches; the files written are byte-identical."""
    os.makedirs(output_dir, exist_ok=True)
    model.load(checkpoint_path)
    imgs, names = read_dataset(dataset_path)
    if workers <= 0:
        for i, j in _batches([a.shape for a in imgs], batch_size):
            feed_batch(model, np.stack(imgs[i:j]), names[i:j], output_dir, in_cshape)
        return
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(max_workers=workers) as pool:
        futures = []
        for i, j in _batches([a.shape for a in imgs], batch_size):
            futures += feed_batch(model, np.stack(imgs[i:j]), names[i:j], output_dir, in_cshape, pool=pool)
        for f in futures:
            f.result()  # re-raise any write error

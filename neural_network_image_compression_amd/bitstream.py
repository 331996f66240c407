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


PNG_MODES = {"pillow": 0, "tf": 1}  # nic.h NIC_PNG_PILLOW / NIC_PNG_TF


def _png_shape(images: np.ndarray, fn: str):
    a = np.ascontiguousarray(images, dtype=np.uint8)
    if a.ndim not in (3, 4) or (a.ndim == 4 and a.shape[3] != 3):
        raise ValueError(f"{fn}: expected (M, H, W) or (M, H, W, 3) images, got shape {a.shape}")
    return a, a.shape[0], a.shape[1], a.shape[2], 3 if a.ndim == 4 else 1


def png_sizes(images: np.ndarray, threads: int = 16, mode: str = "pillow") -> np.ndarray:
    """PNG byte counts of every u8 image of images (M, H, W) or (M, H, W, 3), computed natively
    on host threads (nic_png_encode without output).  mode "pillow": len(png_bytes(a)) byte for
    byte (save_img, utils.py:85-87); mode "tf": tf.image.encode_png(compression=-1)'s settings,
    what get_bpp sizes (training.py:12-21; parity with TF itself unpinned, nic.h)."""
    import ctypes

    from . import _lib

    a, m, h, w, ch = _png_shape(images, "png_sizes")
    out = np.empty(m, np.int64)
    if m:
        _lib.check(_lib.lib().nic_png_encode(a.ctypes.data_as(ctypes.c_void_p), m, h, w, ch, PNG_MODES[mode], None, 0,
                                             out.ctypes.data_as(ctypes.c_void_p), int(threads)), "nic_png_encode")
    return out


def png_encode(images: np.ndarray, threads: int = 16, mode: str = "pillow") -> List[bytes]:
    """The PNG files of every u8 image of images (M, H, W) or (M, H, W, 3), encoded natively on
    host threads (nic_png_encode); mode "pillow" is byte for byte Pillow's optimize=True file."""
    import ctypes

    from . import _lib

    a, m, h, w, ch = _png_shape(images, "png_encode")
    if m == 0:
        return []
    L = _lib.lib()
    stride = ctypes.c_int64()
    _lib.check(L.nic_png_bound(h, w, ch, PNG_MODES[mode], ctypes.byref(stride)), "nic_png_bound")
    buf = np.empty((m, stride.value), np.uint8)
    sizes = np.empty(m, np.int64)
    _lib.check(L.nic_png_encode(a.ctypes.data_as(ctypes.c_void_p), m, h, w, ch, PNG_MODES[mode],
                                buf.ctypes.data_as(ctypes.c_void_p), stride.value,
                                sizes.ctypes.data_as(ctypes.c_void_p), int(threads)), "nic_png_encode")
    return [buf[i, :sizes[i]].tobytes() for i in range(m)]


def save_img(img: np.ndarray, output_dir: str, filename: str) -> str:
    """utils.py:85-87 (the file Pillow's optimize=True writes, encoded natively)."""
    return save_imgs(np.asarray(img)[None], output_dir, [filename], threads=1)[0]


def save_imgs(imgs: np.ndarray, output_dir: str, filenames: Sequence[str], threads: int = 16) -> List[str]:
    """save_img (utils.py:85-87) of a batch of equal-shaped images: the PNG files encoded on
    ``threads`` native host threads (nic_png_encode, byte-identical to Pillow), then written."""
    imgs = np.asarray(imgs)
    assert (np.round(imgs) - imgs).sum() == 0  # utils.py:86
    files = png_encode(imgs.astype(np.uint8), threads=threads)
    paths = []
    for data, name in zip(files, filenames):
        path = os.path.join(output_dir, name + ".png")
        with open(path, "wb") as f:
            f.write(data)
        paths.append(path)
    return paths


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
               pool=None, png_threads: int = 16) -> list:
    """utils.py:30-44 for one batch: unpack (decoder side), run the codec, pack (encoder side), save.

    The batch's PNG files are encoded natively on ``png_threads`` host threads (nic_png_encode,
    byte-identical to Pillow's optimize=True).  With a pool the encode + write is submitted to
    it and its future returned, so the caller runs the next batch on the GPU meanwhile."""
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
    if host.shape[1] == 1 or host.shape[2] == 1:  # np.squeeze (utils.py:44) changes the mode
        for i in range(host.shape[0]):
            a = np.squeeze(host[i])
            save_imgs(a[None], output_dir, [filenames[i]], threads=1)
        return []
    imgs = host
    if pool is None:
        save_imgs(imgs, output_dir, filenames, threads=png_threads)
        return []
    return [pool.submit(save_imgs, imgs, output_dir, list(filenames), png_threads)]


def list_dataset(dataset_path: str) -> List[str]:
    """utils.py:92-94: the sorted directory entries with an image extension."""
    return [fn for fn in sorted(os.listdir(dataset_path)) if fn.split(".")[-1] in IMAGE_EXTS]


def _read_one(path: str):
    from PIL import Image

    with Image.open(path) as im:
        return np.array(im)


def _host_threads() -> int:
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except AttributeError:  # pragma: no cover
        return max(1, os.cpu_count() or 1)


WRITES_IN_FLIGHT = 2  # batches handed to the PNG writer and not yet written (use_model)
BATCH_PIXELS = 64 * 512 * 768  # pixels staged per device batch (use_model): 64 Kodak-sized images, 3 4K frames


def use_model(model, dataset_path: str, checkpoint_path: str, output_dir: str, in_cshape: int,
              batch_size: int = 64, workers=None) -> None:
    """utils.py:46-62: every colour image of ``dataset_path`` (sorted; read_dataset's filter)
    through the codec into ``output_dir``, one PNG per image named after its source.

    ``workers=0`` is the reference's serial loop (read everything, then batches of
    ``batch_size`` -- the reference's 4 -- each run and saved inline).  Otherwise (default) a
    pipeline over the host cores: images are decoded by a reader pool in file order, consecutive
    equal-shaped images are fed to the device ``batch_size`` (64) at a time (at most
    ``BATCH_PIXELS`` pixels), and each batch's PNG files are encoded natively on ``workers``
    threads (default: every CPU this process may use, at most 16) while the next batches are
    read and run; at most ``WRITES_IN_FLIGHT`` batches wait for the writer, so host memory stays
    bounded however large the directory.  Every image's output depends on that
    image alone (the kernels are batch-invariant), so the files are byte-identical either way."""
    os.makedirs(output_dir, exist_ok=True)
    model.load(checkpoint_path)
    if workers is not None and workers <= 0:
        imgs, names = read_dataset(dataset_path)
        for i, j in _batches([a.shape for a in imgs], batch_size):
            feed_batch(model, np.stack(imgs[i:j]), names[i:j], output_dir, in_cshape)
        return
    from concurrent.futures import ThreadPoolExecutor

    threads = _host_threads()
    png_threads = int(workers) if workers else min(16, threads)
    files = list_dataset(dataset_path)
    with ThreadPoolExecutor(max_workers=min(8, threads)) as readers, ThreadPoolExecutor(max_workers=1) as writer:
        futures, batch, names, depth = [], [], [], 4 * max(1, batch_size)
        pending = [readers.submit(_read_one, os.path.join(dataset_path, fn)) for fn in files[:depth]]

        def flush():
            if batch:
                # bounded host memory: at most WRITES_IN_FLIGHT batches' outputs wait for the
                # (slower) PNG writer; the device pass of the next batch still overlaps them
                while len(futures) >= WRITES_IN_FLIGHT:
                    futures.pop(0).result()  # re-raises a write error
                futures.extend(feed_batch(model, np.stack(batch), list(names), output_dir, in_cshape, pool=writer,
                                          png_threads=png_threads))
                batch.clear()
                names.clear()
            while futures and futures[0].done():
                futures.pop(0).result()  # re-raise a write error early

        for k, fn in enumerate(files):
            a = pending[k].result()
            if k + depth < len(files):  # keep `depth` decodes in flight ahead of the device
                pending.append(readers.submit(_read_one, os.path.join(dataset_path, files[k + depth])))
            pending[k] = None
            if a.ndim != 3:  # read_dataset keeps colour (3-D) images only
                continue
            if batch and (a.shape != batch[0].shape or len(batch) >= batch_size
                          or (len(batch) + 1) * a.shape[0] * a.shape[1] > BATCH_PIXELS):
                flush()
            batch.append(a.astype(np.uint8, copy=False))
            names.append(".".join(fn.split(".")[:-1]))
        flush()
        for f in futures:
            f.result()  # re-raise any write error

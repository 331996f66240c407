"""Rate-distortion evaluation on the device (BASELINE config 4 harness).

The reference reports rate as PNG bytes of the packed latent (``get_bpp``,
tf1_13/src/training.py:12-21, used at :157-163) and as the histogram entropy of the codes
(``disc_entropy``, training.py:66-71), and distortion as PSNR and MS-SSIM
(tf2_0/tests/calc_ssim.py:13).  ``rd_point`` computes all four for a batch of images with
the device kernels (encode, ``nic_entropy_hist``, pack, decode, ``nic_ms_ssim``,
``nic_sq_err``); only zlib (PNG) runs on the host, in a thread pool.  ``tile`` runs the
same images as non-overlapping ``tile x tile`` patches (config 4's "tiled into patches");
``rd_sweep`` evaluates several weight sets (the reference's lambda sweep,
``entropy_loss_coef`` in training.py:54) whole-image and tiled.

No trained checkpoints ship with the reference, so with seeded weights these points are
plumbing, not the reference's RD curve.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from .bitstream import png_sizes
from .codec import Codec
from .quality import ms_ssim_supported


def tile_patches(x: np.ndarray, tile: int) -> np.ndarray:
    """(N,H,W,3) -> (N*(H/t)*(W/t), t, t, 3), row-major tiles per image."""
    n, h, w, c = x.shape
    if h % tile or w % tile:
        raise ValueError(f"tile_patches: {h}x{w} is not a multiple of {tile}")
    t = x.reshape(n, h // tile, tile, w // tile, tile, c).transpose(0, 1, 3, 2, 4, 5)
    return np.ascontiguousarray(t.reshape(-1, tile, tile, c))


def untile_patches(t: np.ndarray, n: int, h: int, w: int) -> np.ndarray:
    tile, c = t.shape[1], t.shape[3]
    x = t.reshape(n, h // tile, w // tile, tile, tile, c).transpose(0, 1, 3, 2, 4, 5)
    return np.ascontiguousarray(x.reshape(n, h, w, c))


def rd_point(codec: Codec, images: np.ndarray, tile: Optional[int] = None, png: bool = True,
             workers: int = 8) -> Dict[str, object]:
    """Rate and distortion of u8 images (N,H,W,3) through ``codec`` (weights already set).

    Returns per-image arrays and batch means: ``bpp_entropy`` (histogram entropy of every
    latent plane x its symbols / pixels), ``bpp_png`` (PNG of the packed latent, Pillow
    ``optimize=True`` as ``save_img``), ``psnr_db`` and ``ms_ssim`` (of the image
    reassembled from its tiles when ``tile`` is set)."""
    import torch

    x = np.ascontiguousarray(images, dtype=np.uint8)
    n, h, w, _ = x.shape
    units = tile_patches(x, tile) if tile else x
    dev = torch.from_numpy(units).to(f"cuda:{codec.device}")
    z = codec.encode(dev)
    bits = codec.entropy(z).view(3, -1)  # plane-major: row p = plane p / m of unit p % m
    m, h8, w8, _ = z.shape
    sym_bits = (bits.sum(dim=0) * (h8 * w8 * 32)).double().cpu().numpy()  # bits per unit
    rec = codec.decode(z)[:, :units.shape[1], :units.shape[2]].contiguous()
    packed = codec.pack(z).cpu().numpy() if png else None
    rec_h = rec.cpu().numpy()
    if tile:
        rec_h = untile_patches(rec_h, n, h, w)
        per = (h // tile) * (w // tile)
        sym_bits = sym_bits.reshape(n, per).sum(axis=1)
    rec_d = torch.from_numpy(rec_h).to(dev.device)
    x_d = torch.from_numpy(x).to(dev.device)
    out: Dict[str, object] = {"images": n, "size": [h, w], "tile": tile,
                              "bpp_entropy": sym_bits / (h * w),
                              "psnr_db": codec.psnr(x_d, rec_d, per_image=True)}
    if ms_ssim_supported(h, w):
        out["ms_ssim"] = codec.ms_ssim(x_d, rec_d).cpu().numpy().astype(np.float64)
    if png:  # Pillow's byte counts, computed natively on host threads (bitstream.png_sizes)
        sizes = png_sizes(packed, threads=max(1, workers)).astype(np.float64)
        if tile:
            sizes = sizes.reshape(n, -1).sum(axis=1)
        out["bpp_png"] = 8.0 * sizes / (h * w)
    for k in ("bpp_entropy", "bpp_png", "psnr_db", "ms_ssim"):
        if k in out:
            out[k + "_mean"] = float(np.mean(out[k]))
    return out


def rd_sweep(weight_sets: Dict[str, dict], images: np.ndarray, tile: Optional[int] = 256, device: int = 0,
             png: bool = True) -> Dict[str, Dict[str, Dict[str, object]]]:
    """One RD point per weight set, whole-image and (if ``tile``) tiled; the tiled point also
    carries ``tile_border_psnr_delta_db`` = PSNR(tiled) - PSNR(whole)."""
    codec = Codec(device)
    res: Dict[str, Dict[str, Dict[str, object]]] = {}
    for label, weights in weight_sets.items():
        codec.set_weights(weights)
        whole = rd_point(codec, images, None, png)
        res[label] = {"whole": whole}
        if tile and images.shape[1] % tile == 0 and images.shape[2] % tile == 0:
            tiled = rd_point(codec, images, tile, png)
            tiled["tile_border_psnr_delta_db"] = tiled["psnr_db_mean"] - whole["psnr_db_mean"]
            res[label]["tiled"] = tiled
    return res

"""Quality evaluation on the device: MS-SSIM and PSNR.

Mirrors the reference's evaluator ``tf2_0/tests/calc_ssim.py``: two directories are read
with ``read_dataset`` (utils.py:89-120), images with the same file stem are paired, and
``tf.image.ssim_multiscale(img1, img2, max_val=255)`` (calc_ssim.py:13) is printed per pair
and averaged (calc_ssim.py:24-34).  Here the metric is ``nic_ms_ssim`` (HIP kernels,
``csrc/nic_quality.hip``) on a ``Codec``'s device; PSNR comes from the exact device sum of
squared errors (``nic_sq_err``).
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from .bitstream import read_dataset
from .codec import Codec


MS_SSIM_SCALES = 5
SSIM_FILTER = 11


def ms_ssim_supported(h: int, w: int) -> bool:
    """tf.image.ssim_multiscale's shape rule: each of the 5 scales (odd sizes SYMMETRIC-padded,
    then halved: ceil(n / 2)) must hold the 11 x 11 window -- H, W >= 161."""
    for _ in range(MS_SSIM_SCALES - 1):
        if min(h, w) < SSIM_FILTER:
            return False
        h, w = -(-h // 2), -(-w // 2)
    return min(h, w) >= SSIM_FILTER


def _dev(codec: Codec, a: np.ndarray):
    import torch

    a = np.asarray(a, dtype=np.uint8)
    if a.ndim == 3:  # calc_ssim feeds np.squeeze(x) of one (H,W,3) image
        a = a[None]
    return torch.from_numpy(np.ascontiguousarray(a)).to(f"cuda:{codec.device}")


def ms_ssim(img1, img2, codec: Optional[Codec] = None) -> np.ndarray:
    """MS-SSIM of u8 images (H,W,3) or batches (N,H,W,3) -> (N,) float32 (NumPy in, NumPy out)."""
    codec = codec if codec is not None else Codec()
    return codec.ms_ssim(_dev(codec, img1), _dev(codec, img2)).cpu().numpy()


def psnr(img1, img2, codec: Optional[Codec] = None, max_val: float = 255.0) -> float:
    codec = codec if codec is not None else Codec()
    return codec.psnr(_dev(codec, img1), _dev(codec, img2), max_val=max_val)


def calc_ssim(dataset_path_1: str, dataset_path_2: str, codec: Optional[Codec] = None,
              verbose: bool = True) -> Dict[str, float]:
    """calc_ssim.py:19-34: MS-SSIM of every same-named image pair; returns {stem: ssim} and,
    under the key ``'average'``, their mean.  Raises if no names match (the reference would
    divide by zero)."""
    codec = codec if codec is not None else Codec()
    x1, names1 = read_dataset(dataset_path_1)
    x2, names2 = read_dataset(dataset_path_2)
    index2 = {n: i for i, n in enumerate(names2)}
    out: Dict[str, float] = {}
    for i, name in enumerate(names1):
        j = index2.get(name)
        if j is None:
            continue
        s = float(ms_ssim(np.squeeze(x1[i]), np.squeeze(x2[j]), codec)[0])
        out[name] = s
        if verbose:
            print("SSIM of {0}: {1}".format(name, s))
    if not out:
        raise ValueError(f"calc_ssim: no image names in common between {dataset_path_1} and {dataset_path_2}")
    out["average"] = float(np.mean(list(out.values())))
    if verbose:
        print("average SSIM: {}".format(out["average"]))
    return out

"""Host-side mirror of the reference codec surface, running on the HIP C-ABI.

Reference classes (AlexFuster/Neural_network_image_compression, tf2_0/src):

* ``ProClass`` (utils.py:15-62): owns the Y and CbCr models, ``load(path)`` reads
  ``path + 'Y'`` and ``path + 'CbCr'``, ``_use_model``/``_feed_batch`` drive directories.
* ``Encoder`` (encoder.py:34-51): ``__call__(x)`` u8 (N,H,W,3) -> u8 (N,h,w,96);
  ``compress(dataset_path, checkpoint_path)``.
* ``Decoder`` (decoder.py:35-52): ``__call__(z)`` u8 (N,h,w,96) -> u8 (N,8h,8w,3);
  ``uncompress(dataset_path, checkpoint_path)``.

Here the per-plane Keras models become one fused device pipeline over all 3N planes
(``libnic.so``).  ``__call__`` accepts NumPy arrays (copied to and from the device, like
the reference's ``.numpy()`` hand-offs) or ROCm ``torch.uint8`` tensors (no host copy;
work is queued on the current torch stream and a device tensor is returned).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import numpy as np

from . import _lib
from . import weights as W


def _torch():
    import torch

    return torch


def _stream_ptr(torch, device: int) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _as_u8_array(x, what: str) -> np.ndarray:
    a = np.asarray(x)
    if a.dtype == np.uint8:
        return a
    if a.dtype.kind in "iuf":
        # the reference computes x.astype(float32)/255 (encoder.py:39, decoder.py:40); the
        # device path is defined on u8 codes, so only exactly representable inputs are taken
        if a.size and (not np.all(np.isfinite(a)) or np.any(a != np.round(a)) or a.min() < 0 or a.max() > 255):
            raise ValueError(f"{what}: values must be integers in [0, 255], got dtype {a.dtype}")
        return a.astype(np.uint8)
    raise TypeError(f"{what}: unsupported dtype {a.dtype}")


class Codec:
    """One ``nic_ctx`` on one HIP device: weights + workspace for encode/decode/entropy."""

    def __init__(self, device: Optional[int] = None, precision: str = "f16x3"):
        torch = _torch()
        if not torch.cuda.is_available():
            raise RuntimeError("neural_network_image_compression_amd needs a ROCm GPU (no CPU fallback)")
        self.device = torch.cuda.current_device() if device is None else int(device)
        self._L = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(self._L.nic_create(self.device, ctypes.byref(h)), "nic_create")
        self._h = h
        self._keep: Dict[str, np.ndarray] = {}
        self.precision = precision

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.nic_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- weights ---------------------------------------------------------------------
    def set_tensor(self, model: str, layer: str, kind: str, value: np.ndarray) -> None:
        a = np.ascontiguousarray(value, dtype=np.float32)
        shape = (ctypes.c_int64 * a.ndim)(*a.shape)
        rc = self._L.nic_set_weights(self._h, W.MODEL_ID[model], f"{layer}/{kind}".encode(), a.ctypes.data,
                                     shape, a.ndim)
        _lib.check(rc, f"nic_set_weights({model}/{layer}/{kind})")

    def set_weights(self, weights: W.Weights) -> None:
        for key, value in weights.items():
            model, layer, kind = key.split("/")
            if model not in W.MODEL_ID:
                raise KeyError(f"unknown model {model!r} in key {key!r}")
            self.set_tensor(model, layer, kind, value)

    def ready(self):
        e, d = ctypes.c_int(), ctypes.c_int()
        _lib.check(self._L.nic_weights_ready(self._h, ctypes.byref(e), ctypes.byref(d)), "nic_weights_ready")
        return bool(e.value), bool(d.value)

    @property
    def precision(self) -> str:
        m = ctypes.c_int()
        _lib.check(self._L.nic_get_precision(self._h, ctypes.byref(m)), "nic_get_precision")
        return {v: k for k, v in _lib.PRECISIONS.items()}[m.value]

    @precision.setter
    def precision(self, mode: str) -> None:
        """'f16x3' (default: split-f16 MFMA) or 'fp32' (exact fp32 MFMA) for the Cin>=32 convs."""
        if mode not in _lib.PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(_lib.PRECISIONS)}, got {mode!r}")
        _lib.check(self._L.nic_set_precision(self._h, _lib.PRECISIONS[mode]), "nic_set_precision")

    def set_range_policy(self, policy: str) -> None:
        """f16 range guard of the split-f16 mode (include/nic.h NIC_RANGE_*): 'fallback'
        (default; a tripped pass is recomputed by the exact-fp32 kernels on the device) or
        'error' (the call synchronises and raises NicError(NIC_ERANGE))."""
        if policy not in _lib.RANGE_POLICIES:
            raise ValueError(f"range policy must be one of {sorted(_lib.RANGE_POLICIES)}, got {policy!r}")
        _lib.check(self._L.nic_set_range_policy(self._h, _lib.RANGE_POLICIES[policy]), "nic_set_range_policy")

    def range_trips(self) -> int:
        """Encode/decode passes whose split-f16 activations left the f16 range (synchronises)."""
        n = ctypes.c_int64()
        _lib.check(self._L.nic_range_trips(self._h, ctypes.byref(n)), "nic_range_trips")
        return int(n.value)

    def rerun_launch_info(self) -> dict:
        """How the chained exact-fp32 re-run launches here (nic_rerun_launch_info)."""
        v = [ctypes.c_int() for _ in range(3)]
        _lib.check(self._L.nic_rerun_launch_info(self._h, *[ctypes.byref(t) for t in v]), "nic_rerun_launch_info")
        return {"blocks_per_cu": v[0].value, "grid": v[1].value, "cooperative": bool(v[2].value)}

    def set_timing(self, enable: bool) -> None:
        """Bracket every layer launch with hipEvents on the launch stream (resets the sums)."""
        _lib.check(self._L.nic_set_timing(self._h, int(bool(enable))), "nic_set_timing")

    def layer_times(self):
        """{layer: (total_ms, launches)} accumulated since set_timing(True)."""
        ms = np.zeros(len(_lib.LAYER_NAMES), np.float64)
        cnt = np.zeros(len(_lib.LAYER_NAMES), np.int64)
        _lib.check(self._L.nic_layer_times(self._h, ms.ctypes.data, cnt.ctypes.data), "nic_layer_times")
        return {name: (float(ms[i]), int(cnt[i])) for i, name in enumerate(_lib.LAYER_NAMES)}

    def reserve(self, n: int, h: int, w: int) -> None:
        _lib.check(self._L.nic_reserve(self._h, n, h, w), "nic_reserve")

    # -- device entry points (torch uint8 tensors on this device) ----------------------
    def _check_dev(self, t, ndim: int, last: int, what: str):
        torch = _torch()
        if not isinstance(t, torch.Tensor) or t.dtype != torch.uint8 or t.device.type != "cuda":
            raise TypeError(f"{what}: expected a cuda torch.uint8 tensor")
        if t.device.index != self.device:
            raise ValueError(f"{what}: tensor on cuda:{t.device.index}, codec on cuda:{self.device}")
        if t.ndim != ndim or t.shape[-1] != last:
            raise ValueError(f"{what}: expected shape (N,H,W,{last}), got {tuple(t.shape)}")
        return t.contiguous()

    def encode(self, x, prequant: bool = False, out=None):
        """(N,H,W,3) u8 -> (N,ceil(H/8),ceil(W/8),96) u8 [, fp32 clipped pre-quant latent]."""
        torch = _torch()
        x = self._check_dev(x, 4, 3, "encode")
        n, h, w, _ = x.shape
        h8, w8 = _lib.latent_shape(h, w)
        z = out if out is not None else torch.empty((n, h8, w8, 96), dtype=torch.uint8, device=x.device)
        f = torch.empty((n, h8, w8, 96), dtype=torch.float32, device=x.device) if prequant else None
        rc = self._L.nic_encode(self._h, x.data_ptr(), n, h, w, z.data_ptr(), f.data_ptr() if f is not None else None,
                                _stream_ptr(torch, self.device))
        _lib.check(rc, "nic_encode")
        return (z, f) if prequant else z

    def encode_entropy(self, x, counts: bool = False, out=None):
        """encode(x) and entropy(latent) in one pass (nic_encode_entropy: the codes are counted
        in conv8's epilogue): (latent, (3N,) fp32 bits/symbol [, (3N,256) int32 counts])."""
        torch = _torch()
        x = self._check_dev(x, 4, 3, "encode_entropy")
        n, h, w, _ = x.shape
        h8, w8 = _lib.latent_shape(h, w)
        z = out if out is not None else torch.empty((n, h8, w8, 96), dtype=torch.uint8, device=x.device)
        bits = torch.empty((3 * n,), dtype=torch.float32, device=x.device)
        cnt = torch.empty((3 * n, 256), dtype=torch.int32, device=x.device) if counts else None
        rc = self._L.nic_encode_entropy(self._h, x.data_ptr(), n, h, w, z.data_ptr(),
                                        cnt.data_ptr() if cnt is not None else None, bits.data_ptr(),
                                        _stream_ptr(torch, self.device))
        _lib.check(rc, "nic_encode_entropy")
        return (z, bits, cnt) if counts else (z, bits)

    def encode_entropy_folds(self, n: int, h: int, w: int) -> bool:
        """True when encode_entropy on (n, h, w) images counts the codes inside conv8 (the fold),
        False when it runs encode + entropy (nic_encode_entropy_fold)."""
        import ctypes
        f = ctypes.c_int()
        _lib.check(self._L.nic_encode_entropy_fold(self._h, n, h, w, ctypes.byref(f)), "nic_encode_entropy_fold")
        return bool(f.value)

    def decode(self, z, rgb_f32: bool = False, out=None):
        """(N,h,w,96) u8 -> (N,8h,8w,3) u8 [, fp32 clipped RGB before quantisation]."""
        torch = _torch()
        z = self._check_dev(z, 4, 96, "decode")
        n, h8, w8, _ = z.shape
        x = out if out is not None else torch.empty((n, 8 * h8, 8 * w8, 3), dtype=torch.uint8, device=z.device)
        f = torch.empty((n, 8 * h8, 8 * w8, 3), dtype=torch.float32, device=z.device) if rgb_f32 else None
        rc = self._L.nic_decode(self._h, z.data_ptr(), n, h8, w8, x.data_ptr(), f.data_ptr() if f is not None else None,
                                _stream_ptr(torch, self.device))
        _lib.check(rc, "nic_decode")
        return (x, f) if rgb_f32 else x

    # -- host entry points (NumPy u8 arrays; nic_encode_host / nic_decode_host) ----------
    def _host_out(self, shape):
        """A u8 result array in page-locked memory (torch's caching host allocator): the D2H
        DMA lands in it directly, and a Decoder handed an Encoder result DMA's it directly."""
        torch = _torch()
        n = int(np.prod(shape))
        return torch.empty(max(n, 1), dtype=torch.uint8, pin_memory=True).numpy()[:n].reshape(shape)

    def encode_host(self, x: np.ndarray, chunks: int = 3) -> np.ndarray:
        """(N,H,W,3) u8 host array -> (N,ceil(H/8),ceil(W/8),96) u8 host array (synchronous)."""
        torch = _torch()
        x = np.ascontiguousarray(x, dtype=np.uint8)
        if x.ndim != 4 or x.shape[3] != 3:
            raise ValueError(f"encode_host: expected shape (N,H,W,3), got {x.shape}")
        n, h, w, _ = x.shape
        h8, w8 = _lib.latent_shape(h, w) if h > 0 and w > 0 else (0, 0)
        z = self._host_out((n, h8, w8, 96))
        rc = self._L.nic_encode_host(self._h, x.ctypes.data, n, h, w, z.ctypes.data, int(chunks),
                                     _stream_ptr(torch, self.device))
        _lib.check(rc, "nic_encode_host")
        return z

    def decode_host(self, z: np.ndarray, chunks: int = 3) -> np.ndarray:
        """(N,h,w,96) u8 host array -> (N,8h,8w,3) u8 host array (synchronous)."""
        torch = _torch()
        z = np.ascontiguousarray(z, dtype=np.uint8)
        if z.ndim != 4 or z.shape[3] != 96:
            raise ValueError(f"decode_host: expected shape (N,h,w,96), got {z.shape}")
        n, h8, w8, _ = z.shape
        x = self._host_out((n, 8 * h8, 8 * w8, 3))
        rc = self._L.nic_decode_host(self._h, z.ctypes.data, n, h8, w8, x.ctypes.data, int(chunks),
                                     _stream_ptr(torch, self.device))
        _lib.check(rc, "nic_decode_host")
        return x

    def entropy(self, z, counts: bool = False):
        """Histogram entropy per latent plane: (3N,) fp32 bits/symbol [, (3N,256) int32 counts]."""
        torch = _torch()
        z = self._check_dev(z, 4, 96, "entropy")
        n, h8, w8, _ = z.shape
        bits = torch.empty((3 * n,), dtype=torch.float32, device=z.device)
        cnt = torch.empty((3 * n, 256), dtype=torch.int32, device=z.device) if counts else None
        rc = self._L.nic_entropy_hist(self._h, z.data_ptr(), n, h8, w8, cnt.data_ptr() if cnt is not None else None,
                                      bits.data_ptr(), _stream_ptr(torch, self.device))
        _lib.check(rc, "nic_entropy_hist")
        return (bits, cnt) if counts else bits

    def ms_ssim(self, a, b, per_scale: bool = False):
        """tf.image.ssim_multiscale(a, b, max_val=255) per image (calc_ssim.py:13): (N,) fp32
        [, (N,3,5,2) mean SSIM / mean cs per channel and scale]."""
        torch = _torch()
        a = self._check_dev(a, 4, 3, "ms_ssim")
        b = self._check_dev(b, 4, 3, "ms_ssim")
        if a.shape != b.shape:
            raise ValueError(f"ms_ssim: shapes differ {tuple(a.shape)} vs {tuple(b.shape)}")
        n, h, w, _ = a.shape
        out = torch.empty((n,), dtype=torch.float32, device=a.device)
        ps = torch.empty((n, 3, 5, 2), dtype=torch.float32, device=a.device) if per_scale else None
        rc = self._L.nic_ms_ssim(self._h, a.data_ptr(), b.data_ptr(), n, h, w, out.data_ptr(),
                                 ps.data_ptr() if ps is not None else None, _stream_ptr(torch, self.device))
        _lib.check(rc, "nic_ms_ssim")
        return (out, ps) if per_scale else out

    def sq_err(self, a, b):
        """Exact per-image sum of squared differences of two u8 tensors (N,...): (N,) int64."""
        torch = _torch()
        for t in (a, b):
            if not isinstance(t, torch.Tensor) or t.dtype != torch.uint8 or t.device.type != "cuda":
                raise TypeError("sq_err: expected cuda torch.uint8 tensors")
            if t.device.index != self.device:  # nic_sq_err launches on this codec's stream
                raise ValueError(f"sq_err: tensor on cuda:{t.device.index}, codec on cuda:{self.device}")
        if a.shape != b.shape or a.ndim < 1:
            raise ValueError(f"sq_err: shapes differ {tuple(a.shape)} vs {tuple(b.shape)}")
        a, b = a.contiguous(), b.contiguous()
        n = a.shape[0]
        out = torch.empty((n,), dtype=torch.int64, device=a.device)
        per = a.numel() // n if n else 0
        _lib.check(self._L.nic_sq_err(a.data_ptr(), b.data_ptr(), n, per, out.data_ptr(),
                                      _stream_ptr(torch, self.device)), "nic_sq_err")
        return out

    def psnr(self, a, b, max_val: float = 255.0, per_image: bool = False):
        """PSNR in dB over the whole batch (as the oracle's psnr) or per image, from the exact
        device sum of squared errors."""
        import math

        sse = self.sq_err(a, b).cpu().numpy().astype(np.float64)
        n = a.shape[0]
        per = a.numel() // n if n else 0

        def db(s, count):
            return float("inf") if s == 0 else 10.0 * math.log10(max_val ** 2 * count / s)

        if per_image:
            return np.array([db(s, per) for s in sse])
        return db(float(sse.sum()), per * n)

    def pack(self, z):
        """(N,h,w,96) -> (N,4h,8w,3) bitstream image (utils.py:39-40)."""
        torch = _torch()
        z = self._check_dev(z, 4, 96, "pack")
        n, h8, w8, _ = z.shape
        out = torch.empty((n, 4 * h8, 8 * w8, 3), dtype=torch.uint8, device=z.device)
        _lib.check(self._L.nic_pack_latent(z.data_ptr(), n, h8, w8, out.data_ptr(), _stream_ptr(torch, self.device)),
                   "nic_pack_latent")
        return out

    def unpack(self, img):
        """(N,4h,8w,3) -> (N,h,w,96) (utils.py:35-36)."""
        torch = _torch()
        img = self._check_dev(img, 4, 3, "unpack")
        n, hh, ww, _ = img.shape
        if hh % 4 or ww % 8:
            raise ValueError(f"unpack: packed image {tuple(img.shape)} is not (N,4h,8w,3)")
        out = torch.empty((n, hh // 4, ww // 8, 96), dtype=torch.uint8, device=img.device)
        _lib.check(self._L.nic_unpack_latent(img.data_ptr(), n, hh // 4, ww // 8, out.data_ptr(),
                                             _stream_ptr(torch, self.device)), "nic_unpack_latent")
        return out


class ProClass:
    """utils.py:15-62: shared Y/CbCr model holder (kind 'encoder' or 'decoder')."""

    #: chunks of the native host-array pipeline per call (nic_encode_host / nic_decode_host):
    #: 3 ramped chunks measured fastest for the config-2 batch (2.00 vs 2.07 ms for 4, 2.08 for
    #: 2; descending / ascending chunk sizes no better, profiles/r3n_host_plan_sweep.txt)
    host_chunks = 3

    kind = ""

    def __init__(self, device: Optional[int] = None, codec: Optional[Codec] = None, precision: str = "f16x3"):
        self.codec = codec if codec is not None else Codec(device, precision=precision)

    def load(self, path: str) -> None:
        """utils.py:26-28: weights from ``path + 'Y'`` and ``path + 'CbCr'`` (safetensors)."""
        self.codec.set_weights(W.load(path, self.kind))

    def set_weights(self, weights: W.Weights) -> None:
        sub = {k: v for k, v in weights.items() if k.startswith(self.kind)}
        W.validate(sub, [self.kind + m for m in W.PLANE_MODELS])
        self.codec.set_weights(sub)

    def _device_call(self, x):
        raise NotImplementedError

    def _host_call(self, a: np.ndarray) -> np.ndarray:
        raise NotImplementedError

    def __call__(self, x):
        """Device tensors stay on the device; host arrays (NumPy, CPU tensors) go through the
        native chunked host pipeline and come back as NumPy (in page-locked memory)."""
        torch = _torch()
        if isinstance(x, torch.Tensor) and x.device.type == "cuda":
            return self._device_call(x)
        a = _as_u8_array(x.cpu().numpy() if isinstance(x, torch.Tensor) else x, type(self).__name__)
        if a.ndim != 4:
            raise ValueError(f"{type(self).__name__}: expected a 4-D NHWC batch, got shape {a.shape}")
        return self._host_call(a)


class Encoder(ProClass):
    """encoder.py:34-51."""

    kind = "encoder"

    def _device_call(self, x):
        return self.codec.encode(x)

    def _host_call(self, a):
        if a.shape[3] != 3:
            raise ValueError(f"Encoder: expected shape (N,H,W,3), got {a.shape}")
        return self.codec.encode_host(a, self.host_chunks)

    def compress(self, dataset_path: str, checkpoint_path: str, batch_size: int = 64, workers=None) -> None:
        """encoder.py:49-51: every image in ``dataset_path`` -> ``dataset_path + '_compressed'``.
        Pipelined over the host cores in batches of ``batch_size`` (bitstream.use_model);
        ``workers=0, batch_size=4`` is the reference's serial loop (same files)."""
        from .bitstream import use_model

        use_model(self, dataset_path, checkpoint_path, dataset_path + "_compressed", in_cshape=3,
                  batch_size=batch_size, workers=workers)


class Decoder(ProClass):
    """decoder.py:35-52."""

    kind = "decoder"

    def _device_call(self, z):
        return self.codec.decode(z)

    def _host_call(self, a):
        if a.shape[3] != 96:
            raise ValueError(f"Decoder: expected shape (N,h,w,96), got {a.shape}")
        return self.codec.decode_host(a, self.host_chunks)

    def uncompress(self, dataset_path: str, checkpoint_path: str, batch_size: int = 64, workers=None) -> None:
        """decoder.py:50-52: packed PNGs in ``dataset_path`` -> ``dataset_path.replace('compressed','uncompressed')``.
        Pipelined as compress (``workers=0, batch_size=4``: the reference's serial loop)."""
        from .bitstream import use_model

        use_model(self, dataset_path, checkpoint_path, dataset_path.replace("compressed", "uncompressed"),
                  in_cshape=96, batch_size=batch_size, workers=workers)

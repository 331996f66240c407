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


class _HostPipe:
    """Host-array surface of a device call: pinned staging buffers (grown on demand, reused)
    and the batch cut into chunks so that chunk k's host->pinned copy and H2D DMA (copy
    stream), chunk k-1's device pass (compute stream) and chunk k-2's D2H DMA overlap.
    The reference's surface moves NumPy in and out around every call (encoder.py:38-47,
    decoder.py:39-48); this is that hand-off, pipelined.  Every call synchronises before it
    returns (NumPy out), so the staging buffers are free again for the next call."""

    def __init__(self, device: int):
        torch = _torch()
        self.device = device
        self.copy = torch.cuda.Stream(device)
        self.comp = torch.cuda.Stream(device)
        self._pin = {}

    def _pinned(self, key: str, nbytes: int):
        torch = _torch()
        buf = self._pin.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, pin_memory=True)
            self._pin[key] = buf
        return buf

    def run(self, a: np.ndarray, fn, out_tail, chunks: int) -> np.ndarray:
        """fn: device u8 (n, *a.shape[1:]) -> device u8 (n, *out_tail); returns NumPy."""
        torch = _torch()
        n = a.shape[0]
        out = np.empty((n,) + tuple(out_tail), np.uint8)
        if n == 0:
            return out
        a = np.ascontiguousarray(a)
        in_row, out_row = a[0].nbytes, out[0].nbytes
        pin_in = self._pinned("in", n * in_row)
        pin_out = self._pinned("out", n * out_row)
        cur = torch.cuda.current_stream(self.device)
        self.copy.wait_stream(cur)  # the caller's earlier work on this device comes first
        self.comp.wait_stream(cur)
        bounds = np.linspace(0, n, min(chunks, n) + 1).astype(int)
        done = []
        keep = []
        for lo, hi in zip(bounds[:-1], bounds[1:]):
            if hi == lo:
                continue
            src = pin_in[lo * in_row:hi * in_row]
            src.numpy()[:] = a[lo:hi].reshape(-1)  # host copy into pinned memory
            with torch.cuda.stream(self.copy):
                x = torch.empty((hi - lo,) + a.shape[1:], dtype=torch.uint8, device=f"cuda:{self.device}")
                x.view(-1).copy_(src, non_blocking=True)
                ev_in = torch.cuda.Event()
                ev_in.record(self.copy)
            with torch.cuda.stream(self.comp):
                self.comp.wait_event(ev_in)
                y = fn(x)
                ev_y = torch.cuda.Event()
                ev_y.record(self.comp)
            with torch.cuda.stream(self.copy):
                self.copy.wait_event(ev_y)
                pin_out[lo * out_row:hi * out_row].copy_(y.reshape(-1), non_blocking=True)
                ev_out = torch.cuda.Event()
                ev_out.record(self.copy)
            keep.append((x, y))  # device buffers stay alive until their DMA is done
            done.append((lo, hi, ev_out))
        flat = out.reshape(-1)
        po = pin_out.numpy()
        for lo, hi, ev in done:  # chunk k's pinned -> NumPy copy overlaps chunk k+1's work
            ev.synchronize()
            flat[lo * out_row:hi * out_row] = po[lo * out_row:hi * out_row]
        cur.wait_stream(self.copy)
        return out


class ProClass:
    """utils.py:15-62: shared Y/CbCr model holder (kind 'encoder' or 'decoder')."""

    #: chunks of the host-array pipeline (``_HostPipe``) per call
    host_chunks = 4

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

    def __call__(self, x):
        torch = _torch()
        if isinstance(x, torch.Tensor) and x.device.type == "cuda":
            return self._device_call(x)
        a = _as_u8_array(x.cpu().numpy() if isinstance(x, torch.Tensor) else x, type(self).__name__)
        if a.ndim != 4:
            raise ValueError(f"{type(self).__name__}: expected a 4-D NHWC batch, got shape {a.shape}")
        self._check_host(a)
        if getattr(self, "_pipe", None) is None:
            self._pipe = _HostPipe(self.codec.device)
        return self._pipe.run(a, self._device_call, self._out_tail(a.shape), self.host_chunks)

    def _check_host(self, a: np.ndarray) -> None:
        pass

    def _out_tail(self, shape):
        raise NotImplementedError


class Encoder(ProClass):
    """encoder.py:34-51."""

    kind = "encoder"

    def _device_call(self, x):
        return self.codec.encode(x)

    def _check_host(self, a):
        if a.shape[3] != 3:
            raise ValueError(f"Encoder: expected shape (N,H,W,3), got {a.shape}")

    def _out_tail(self, shape):
        h8, w8 = _lib.latent_shape(shape[1], shape[2])
        return (h8, w8, 96)

    def compress(self, dataset_path: str, checkpoint_path: str, batch_size: int = 4, workers: int = 0) -> None:
        """encoder.py:49-51: every image in ``dataset_path`` -> ``dataset_path + '_compressed'``.
        ``workers``: host threads for the PNG writes (0 = inline, as the reference)."""
        from .bitstream import use_model

        use_model(self, dataset_path, checkpoint_path, dataset_path + "_compressed", in_cshape=3,
                  batch_size=batch_size, workers=workers)


class Decoder(ProClass):
    """decoder.py:35-52."""

    kind = "decoder"

    def _device_call(self, z):
        return self.codec.decode(z)

    def _check_host(self, a):
        if a.shape[3] != 96:
            raise ValueError(f"Decoder: expected shape (N,h,w,96), got {a.shape}")

    def _out_tail(self, shape):
        return (8 * shape[1], 8 * shape[2], 3)

    def uncompress(self, dataset_path: str, checkpoint_path: str, batch_size: int = 4, workers: int = 0) -> None:
        """decoder.py:50-52: packed PNGs in ``dataset_path`` -> ``dataset_path.replace('compressed','uncompressed')``."""
        from .bitstream import use_model

        use_model(self, dataset_path, checkpoint_path, dataset_path.replace("compressed", "uncompressed"),
                  in_cshape=96, batch_size=batch_size, workers=workers)

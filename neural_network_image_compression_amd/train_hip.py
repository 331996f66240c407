"""HIP convolutions for the training side path (tf2_0/src/training.py:74-151).

Keras ``Conv2D(padding='SAME')`` and ``Conv2DTranspose(padding='SAME')`` on NHWC fp32
tensors, forward and backward, on the split-f16x3 MFMA kernels of ``csrc/nic_train.hip``
through the C-ABI (``nic_conv_gather``, ``nic_conv_wgrad``, ``nic_absmax_scale``):

=====================  ==========================================================
Conv2D forward         gather, src = s*o + k - pad, kernel HWIO (layout 0)
Conv2D input grad      gather "transposed", src = (o + pad - k)/s, same kernel (layout 1)
Conv2D kernel grad     wgrad(gat = x, dir = dy) -> HWIO
Conv2DTranspose fwd    gather "transposed", kernel HWOI (layout 1)
Conv2DTranspose dx     gather, src = s*o + k - pad, same kernel (layout 0)
Conv2DTranspose dW     wgrad(gat = dy, dir = x) -> HWOI
=====================  ==========================================================

The SSIM loss's separable Gaussian (one-channel VALID correlation) runs on the same gather
kernel (``gauss_valid``).

Each operand gets a power-of-two scale (max |t| * scale in [2^13, 2^14)) computed on the
device, so the f16 hi/lo split keeps tiny gradients exact to ~2^-22.  Bias gradients are
plain reductions (torch), as are the leaky-ReLU / clip / SSIM elementwise parts.  There is
no fallback: without the built library these raise.
"""
from __future__ import annotations

from typing import Tuple

from . import _lib


def _torch():
    import torch

    return torch


def same_pad(n: int, k: int, s: int) -> Tuple[int, int]:
    out = -(-n // s)
    pad = max((out - 1) * s + k - n, 0)
    return pad // 2, pad - pad // 2


def _stream():
    return _torch().cuda.current_stream().cuda_stream


def _scales(*ts):
    """Device (len(ts),) fp32 tensor of power-of-two operand scales (nic_absmax_scale)."""
    torch = _torch()
    dev = ts[0].device
    out = torch.empty(len(ts), dtype=torch.float32, device=dev)
    work = torch.empty(512, dtype=torch.float32, device=dev)
    L = _lib.lib()
    for i, t in enumerate(ts):
        _lib.check(L.nic_absmax_scale(t.data_ptr(), t.numel(), out.data_ptr() + 4 * i, work.data_ptr(), _stream()),
                   "nic_absmax_scale")
    return out


def _check(t, name):
    torch = _torch()
    if not isinstance(t, torch.Tensor) or t.dtype != torch.float32 or t.device.type != "cuda":
        raise TypeError(f"{name}: expected a cuda float32 tensor")
    return t.contiguous()


def gather(x, wt, layout: int, stride: int, pad: Tuple[int, int], transposed: int, out_hw: Tuple[int, int],
           cout: int, bias=None):
    """nic_conv_gather on NHWC x: returns (n, oh, ow, cout)."""
    torch = _torch()
    x = _check(x, "gather x")
    wt = _check(wt, "gather wt")
    n, h, w, cin = x.shape
    kh, kw = wt.shape[0], wt.shape[1]
    y = torch.empty((n, out_hw[0], out_hw[1], cout), dtype=torch.float32, device=x.device)
    sc = _scales(x, wt)
    b = _check(bias, "gather bias").data_ptr() if bias is not None else None
    _lib.check(_lib.lib().nic_conv_gather(x.data_ptr(), n, h, w, cin, wt.data_ptr(), kh, kw, layout, stride, pad[0],
                                          pad[1], transposed, b, sc.data_ptr(), y.data_ptr(), out_hw[0], out_hw[1],
                                          cout, _stream()), "nic_conv_gather")
    return y


def wgrad(gat, dirt, kh: int, kw: int, stride: int, pad: Tuple[int, int]):
    """nic_conv_wgrad: (kh, kw, ca, cb) = sum_u gat[s*u + k - pad][a] * dir[u][b]."""
    torch = _torch()
    import ctypes

    gat = _check(gat, "wgrad gat")
    dirt = _check(dirt, "wgrad dir")
    n, gh, gw, ca = gat.shape
    _, uh, uw, cb = dirt.shape
    L = _lib.lib()
    need = ctypes.c_int64()
    _lib.check(L.nic_conv_wgrad_work(n, uh, uw, kh, kw, ca, cb, ctypes.byref(need)), "nic_conv_wgrad_work")
    work = torch.empty(max(int(need.value), 1), dtype=torch.float32, device=gat.device)
    dw = torch.empty((kh, kw, ca, cb), dtype=torch.float32, device=gat.device)
    sc = _scales(gat, dirt)
    _lib.check(L.nic_conv_wgrad(gat.data_ptr(), n, gh, gw, ca, dirt.data_ptr(), uh, uw, cb, kh, kw, stride, pad[0],
                                pad[1], sc.data_ptr(), dw.data_ptr(), work.data_ptr(), int(need.value), _stream()),
               "nic_conv_wgrad")
    return dw


def _conv_fn():
    torch = _torch()

    class Conv2DSame(torch.autograd.Function):
        """Keras Conv2D(padding='SAME') without activation, NHWC; kernel (kh, kw, Cin, Cout)."""

        @staticmethod
        def forward(ctx, x, kernel, bias, stride):
            n, h, w, _ = x.shape
            kh, kw, _, cout = kernel.shape
            pt, pl = same_pad(h, kh, stride)[0], same_pad(w, kw, stride)[0]
            oh, ow = -(-h // stride), -(-w // stride)
            ctx.save_for_backward(x, kernel)
            ctx.geo = (stride, pt, pl)
            return gather(x, kernel, 0, stride, (pt, pl), 0, (oh, ow), cout, bias)

        @staticmethod
        def backward(ctx, dy):
            x, kernel = ctx.saved_tensors
            stride, pt, pl = ctx.geo
            dy = dy.contiguous()
            kh, kw, cin, _ = kernel.shape
            dx = gather(dy, kernel, 1, stride, (pt, pl), 1, (x.shape[1], x.shape[2]), cin) \
                if ctx.needs_input_grad[0] else None
            dk = wgrad(x, dy, kh, kw, stride, (pt, pl)) if ctx.needs_input_grad[1] else None
            db = dy.sum(dim=(0, 1, 2)) if ctx.needs_input_grad[2] else None
            return dx, dk, db, None

    class Conv2DTransposeSame(torch.autograd.Function):
        """Keras Conv2DTranspose(padding='SAME') without activation, NHWC; kernel (kh, kw, Cout, Cin)."""

        @staticmethod
        def forward(ctx, x, kernel, bias, stride):
            n, h, w, _ = x.shape
            kh, kw, cout, _ = kernel.shape
            oh, ow = h * stride, w * stride
            pt, pl = same_pad(oh, kh, stride)[0], same_pad(ow, kw, stride)[0]
            ctx.save_for_backward(x, kernel)
            ctx.geo = (stride, pt, pl)
            return gather(x, kernel, 1, stride, (pt, pl), 1, (oh, ow), cout, bias)

        @staticmethod
        def backward(ctx, dy):
            x, kernel = ctx.saved_tensors
            stride, pt, pl = ctx.geo
            dy = dy.contiguous()
            kh, kw, _, cin = kernel.shape
            dx = gather(dy, kernel, 0, stride, (pt, pl), 0, (x.shape[1], x.shape[2]), cin) \
                if ctx.needs_input_grad[0] else None
            dk = wgrad(dy, x, kh, kw, stride, (pt, pl)) if ctx.needs_input_grad[1] else None
            db = dy.sum(dim=(0, 1, 2)) if ctx.needs_input_grad[2] else None
            return dx, dk, db, None

    class Conv2DValid1(torch.autograd.Function):
        """One-channel VALID correlation with a constant kernel (kh, kw, 1, 1), NHWC: the
        separable Gaussian of tf.image.ssim (the SSIM loss, training.py:119-121)."""

        @staticmethod
        def forward(ctx, x, kernel):
            n, h, w, _ = x.shape
            kh, kw = kernel.shape[0], kernel.shape[1]
            ctx.save_for_backward(kernel)
            ctx.hw = (h, w)
            return gather(x, kernel, 0, 1, (0, 0), 0, (h - kh + 1, w - kw + 1), 1)

        @staticmethod
        def backward(ctx, dy):
            (kernel,) = ctx.saved_tensors
            return gather(dy.contiguous(), kernel, 1, 1, (0, 0), 1, ctx.hw, 1), None

    return Conv2DSame, Conv2DTransposeSame, Conv2DValid1


_FNS = None


def _fns():
    global _FNS
    if _FNS is None:
        _FNS = _conv_fn()
    return _FNS


def conv_same(x, kernel_hwio, bias, stride: int, act: bool = True):
    """Keras Conv2D(padding='SAME') + leaky_relu(0.2) on NHWC (HIP)."""
    import torch.nn.functional as F

    y = _fns()[0].apply(x, kernel_hwio, bias, stride)
    return F.leaky_relu(y, 0.2) if act else y


def tconv_same(x, kernel_hwoi, bias, stride: int):
    """Keras Conv2DTranspose(padding='SAME') + leaky_relu(0.2) on NHWC (HIP)."""
    import torch.nn.functional as F

    return F.leaky_relu(_fns()[1].apply(x, kernel_hwoi, bias, stride), 0.2)


def gauss_valid(t, g1d):
    """Separable VALID Gaussian of NCHW one-channel planes (N,1,H,W) on the HIP gather GEMM
    (horizontal then vertical, as training.ssim's filt): returns (N,1,H-10,W-10)."""
    n, c, h, w = t.shape
    if c != 1:
        raise ValueError("gauss_valid: one-channel planes")
    k = g1d.numel()
    x = t.reshape(n, h, w, 1)
    x = _fns()[2].apply(x, g1d.reshape(1, k, 1, 1).contiguous())
    x = _fns()[2].apply(x, g1d.reshape(k, 1, 1, 1).contiguous())
    return x.reshape(n, 1, x.shape[1], x.shape[2])

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

The SSIM loss's separable Gaussian (one-channel VALID correlation) runs on a 1-D HIP
kernel and its adjoint (``gauss_valid``, ``nic_gauss_1d``).

Each operand gets a power-of-two scale (max |t| * scale in [2^13, 2^14)) computed on the
device once per tensor (x and the kernel in the forward, dy in the backward), so the f16 hi/lo split keeps tiny gradients exact to ~2^-22.  The layers' leaky-ReLU runs in
the gather's epilogue (``nic_conv_gather_act``), and its gradient with the bias gradient in
one deterministic pass (``nic_act_bias_grad``: dz = dy * leaky'(y), db = column sums of dz).
The clip, residual-add, noise and SSIM elementwise parts and the Entropynet's two dense layers
(plain library GEMMs) stay on torch.  There is no fallback: without the built library these
raise.
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


def _stream(device):
    """The current stream of the operands' device (not of the current device)."""
    return _torch().cuda.current_stream(device).cuda_stream


def _same_device(*ts):
    devs = {t.device for t in ts if t is not None}
    if len(devs) != 1:
        raise ValueError(f"operands on different devices: {sorted(map(str, devs))}")
    return devs.pop()


def scale(t):
    """Device (1,) fp32 power-of-two operand scale of t (nic_absmax_scale); computed once per
    tensor and passed to every GEMM that reads it.  Strided views are made contiguous first
    (the kernel reads t.numel() elements from t.data_ptr())."""
    torch = _torch()
    t = _check(t, "scale t")
    with torch.cuda.device(t.device):
        out = torch.empty(1, dtype=torch.float32, device=t.device)
        work = torch.empty(512, dtype=torch.float32, device=t.device)
        _lib.check(_lib.lib().nic_absmax_scale(t.data_ptr(), t.numel(), out.data_ptr(), work.data_ptr(),
                                               _stream(t.device)), "nic_absmax_scale")
    return out


def _check(t, name):
    torch = _torch()
    if not isinstance(t, torch.Tensor) or t.dtype != torch.float32 or t.device.type != "cuda":
        raise TypeError(f"{name}: expected a cuda float32 tensor")
    return t.contiguous()


def gather(x, wt, layout: int, stride: int, pad: Tuple[int, int], transposed: int, out_hw: Tuple[int, int],
           cout: int, bias=None, sx=None, sw=None, act: int = 0):
    """nic_conv_gather_act on NHWC x: returns (n, oh, ow, cout), leaky_relu(0.2)-activated
    when act.  sx / sw: operand scales (:func:`scale`), computed here when not given."""
    torch = _torch()
    import ctypes

    x = _check(x, "gather x")
    wt = _check(wt, "gather wt")
    dev = _same_device(x, wt, bias, sx, sw)
    n, h, w, cin = x.shape
    kh, kw = wt.shape[0], wt.shape[1]
    L = _lib.lib()
    need = ctypes.c_int64()
    _lib.check(L.nic_conv_gather_work(kh, kw, cin, cout, ctypes.byref(need)), "nic_conv_gather_work")
    work = torch.empty(int(need.value) // 4, dtype=torch.float32, device=x.device)
    y = torch.empty((n, out_hw[0], out_hw[1], cout), dtype=torch.float32, device=x.device)
    sx = scale(x) if sx is None else sx
    sw = scale(wt) if sw is None else sw
    bias = _check(bias, "gather bias") if bias is not None else None
    b = bias.data_ptr() if bias is not None else None
    with torch.cuda.device(dev):
        _lib.check(L.nic_conv_gather_act(x.data_ptr(), n, h, w, cin, wt.data_ptr(), kh, kw, layout, stride, pad[0],
                                         pad[1], transposed, b, sx.data_ptr(), sw.data_ptr(), y.data_ptr(), out_hw[0],
                                         out_hw[1], cout, int(act), work.data_ptr(), int(need.value), _stream(dev)),
                   "nic_conv_gather_act")
    return y


ABG_ROWS = 256  # rows per block of nic_act_bias_grad (its work: per block a row of sums and a max)


def act_bias_grad(y, dy, act: int, want_dz: bool = True, want_db: bool = True):
    """nic_act_bias_grad on NHWC tensors: (dz, db, dz_scale) with dz = dy * leaky'(y) (dy itself
    when not act), db its per-channel sums and dz_scale its operand scale (:func:`scale`), from
    one pass; dz / db are None when not wanted (dz_scale too, without dz)."""
    torch = _torch()
    dy = _check(dy, "act_bias_grad dy")
    if act:
        y = _check(y, "act_bias_grad y")
    dev = _same_device(y if act else None, dy)
    cols = dy.shape[-1]
    rows = dy.numel() // cols if cols else 0
    dz = (torch.empty_like(dy) if act else dy) if want_dz else None
    if not want_db and not want_dz:
        return None, None, None
    db = torch.empty((cols,), dtype=torch.float32, device=dy.device) if want_db else None
    sdz = torch.empty((1,), dtype=torch.float32, device=dy.device) if want_dz else None
    need = -(-rows // ABG_ROWS) * (cols + 1)  # nic_act_bias_grad_work (checked by the call)
    work = torch.empty(max(need, 1), dtype=torch.float32, device=dy.device)
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().nic_act_bias_grad(
            y.data_ptr() if act else None, dy.data_ptr(), rows, cols, int(act),
            dz.data_ptr() if (dz is not None and act) else None, db.data_ptr() if db is not None else None,
            sdz.data_ptr() if sdz is not None else None, work.data_ptr(), need, _stream(dev)), "nic_act_bias_grad")
    return dz, db, sdz


def wgrad(gat, dirt, kh: int, kw: int, stride: int, pad: Tuple[int, int], sg=None, sd=None):
    """nic_conv_wgrad: (kh, kw, ca, cb) = sum_u gat[s*u + k - pad][a] * dir[u][b]."""
    torch = _torch()
    import ctypes

    gat = _check(gat, "wgrad gat")
    dirt = _check(dirt, "wgrad dir")
    dev = _same_device(gat, dirt, sg, sd)
    n, gh, gw, ca = gat.shape
    _, uh, uw, cb = dirt.shape
    L = _lib.lib()
    need = ctypes.c_int64()
    _lib.check(L.nic_conv_wgrad_work(n, uh, uw, kh, kw, ca, cb, ctypes.byref(need)), "nic_conv_wgrad_work")
    work = torch.empty(max(int(need.value), 1), dtype=torch.float32, device=gat.device)
    dw = torch.empty((kh, kw, ca, cb), dtype=torch.float32, device=gat.device)
    sg = scale(gat) if sg is None else sg
    sd = scale(dirt) if sd is None else sd
    with torch.cuda.device(dev):
        _lib.check(L.nic_conv_wgrad(gat.data_ptr(), n, gh, gw, ca, dirt.data_ptr(), uh, uw, cb, kh, kw, stride,
                                    pad[0], pad[1], sg.data_ptr(), sd.data_ptr(), dw.data_ptr(), work.data_ptr(),
                                    int(need.value), _stream(dev)), "nic_conv_wgrad")
    return dw


def gauss_1d(t, taps, vertical: int, adjoint: int):
    """nic_gauss_1d on one-channel planes (n, h, w)."""
    torch = _torch()
    t = _check(t, "gauss t")
    taps = _check(taps, "gauss taps")
    dev = _same_device(t, taps)
    n, h, w = t.shape
    d = taps.numel() - 1
    sgn = 1 if adjoint else -1
    ho, wo = (h + sgn * d, w) if vertical else (h, w + sgn * d)
    out = torch.empty((n, ho, wo), dtype=torch.float32, device=t.device)
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().nic_gauss_1d(t.data_ptr(), n, h, w, taps.data_ptr(), taps.numel(), vertical, adjoint,
                                           out.data_ptr(), ho, wo, _stream(dev)), "nic_gauss_1d")
    return out


def _conv_fn():
    torch = _torch()

    class Conv2DSame(torch.autograd.Function):
        """Keras Conv2D(padding='SAME'), leaky_relu(0.2) when act, NHWC; kernel (kh, kw, Cin, Cout)."""

        @staticmethod
        def forward(ctx, x, kernel, bias, stride, act):
            x, kernel = _check(x, "Conv2DSame x"), _check(kernel, "Conv2DSame kernel")
            n, h, w, _ = x.shape
            kh, kw, _, cout = kernel.shape
            pt, pl = same_pad(h, kh, stride)[0], same_pad(w, kw, stride)[0]
            oh, ow = -(-h // stride), -(-w // stride)
            sx, sw = scale(x), scale(kernel)
            y = gather(x, kernel, 0, stride, (pt, pl), 0, (oh, ow), cout, bias, sx, sw, act=int(act))
            ctx.save_for_backward(x, kernel, sx, sw, y if act else None)
            ctx.geo = (stride, pt, pl, bool(act))
            return y

        @staticmethod
        def backward(ctx, dy):
            x, kernel, sx, sw, y = ctx.saved_tensors
            stride, pt, pl, act = ctx.geo
            dy = dy.contiguous()
            need_dz = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
            dy, db, sdy = act_bias_grad(y, dy, act, need_dz, ctx.needs_input_grad[2])
            if not need_dz:
                return None, None, db, None, None
            kh, kw, cin, _ = kernel.shape
            dx = gather(dy, kernel, 1, stride, (pt, pl), 1, (x.shape[1], x.shape[2]), cin, None, sdy, sw) \
                if ctx.needs_input_grad[0] else None
            dk = wgrad(x, dy, kh, kw, stride, (pt, pl), sx, sdy) if ctx.needs_input_grad[1] else None
            return dx, dk, db, None, None

    class Conv2DTransposeSame(torch.autograd.Function):
        """Keras Conv2DTranspose(padding='SAME'), leaky_relu(0.2) when act, NHWC; kernel (kh, kw, Cout, Cin)."""

        @staticmethod
        def forward(ctx, x, kernel, bias, stride, act):
            x, kernel = _check(x, "Conv2DTransposeSame x"), _check(kernel, "Conv2DTransposeSame kernel")
            n, h, w, _ = x.shape
            kh, kw, cout, _ = kernel.shape
            oh, ow = h * stride, w * stride
            pt, pl = same_pad(oh, kh, stride)[0], same_pad(ow, kw, stride)[0]
            sx, sw = scale(x), scale(kernel)
            y = gather(x, kernel, 1, stride, (pt, pl), 1, (oh, ow), cout, bias, sx, sw, act=int(act))
            ctx.save_for_backward(x, kernel, sx, sw, y if act else None)
            ctx.geo = (stride, pt, pl, bool(act))
            return y

        @staticmethod
        def backward(ctx, dy):
            x, kernel, sx, sw, y = ctx.saved_tensors
            stride, pt, pl, act = ctx.geo
            dy = dy.contiguous()
            need_dz = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
            dy, db, sdy = act_bias_grad(y, dy, act, need_dz, ctx.needs_input_grad[2])
            if not need_dz:
                return None, None, db, None, None
            kh, kw, _, cin = kernel.shape
            dx = gather(dy, kernel, 0, stride, (pt, pl), 0, (x.shape[1], x.shape[2]), cin, None, sdy, sw) \
                if ctx.needs_input_grad[0] else None
            dk = wgrad(dy, x, kh, kw, stride, (pt, pl), sdy, sx) if ctx.needs_input_grad[1] else None
            return dx, dk, db, None, None

    class Gauss1D(torch.autograd.Function):
        """One-channel VALID correlation along x or y with constant taps (nic_gauss_1d), the
        separable Gaussian of tf.image.ssim (the SSIM loss, training.py:119-121)."""

        @staticmethod
        def forward(ctx, t, taps, vertical):
            ctx.save_for_backward(taps)
            ctx.vertical = vertical
            return gauss_1d(t, taps, vertical, 0)

        @staticmethod
        def backward(ctx, dy):
            (taps,) = ctx.saved_tensors
            return gauss_1d(dy.contiguous(), taps, ctx.vertical, 1), None, None

    class SsimMap(torch.autograd.Function):
        """Per-plane mean of tf.image.ssim's map from its filtered terms (nic_ssim_map /
        nic_ssim_map_grad): mx, my, sxy = G*(x y), sxx = G*(x^2 + y^2), each (N, ...) planes."""

        @staticmethod
        def forward(ctx, mx, my, sxy, sxx, c1, c2):
            ts = [_check(t, "SsimMap term") for t in (mx, my, sxy, sxx)]
            dev = _same_device(*ts)
            n = ts[0].shape[0]
            hw = ts[0].numel() // max(n, 1)
            out = torch.empty((n,), dtype=torch.float32, device=ts[0].device)
            need = n * (-(-hw // SSIM_PIX))  # nic_ssim_map_work (checked by the call)
            work = torch.empty(max(need, 1), dtype=torch.float32, device=ts[0].device)
            with torch.cuda.device(dev):
                _lib.check(_lib.lib().nic_ssim_map(*(t.data_ptr() for t in ts), n, hw, c1, c2, out.data_ptr(),
                                                   work.data_ptr(), need, _stream(dev)), "nic_ssim_map")
            ctx.save_for_backward(*ts)
            ctx.consts = (c1, c2, n, hw)
            return out

        @staticmethod
        def backward(ctx, g):
            ts = ctx.saved_tensors
            c1, c2, n, hw = ctx.consts
            g = g.contiguous()
            grads = [torch.empty_like(t) for t in ts]
            dev = ts[0].device
            with torch.cuda.device(dev):
                _lib.check(_lib.lib().nic_ssim_map_grad(*(t.data_ptr() for t in ts), g.data_ptr(), n, hw, c1, c2,
                                                        *(t.data_ptr() for t in grads), _stream(dev)),
                           "nic_ssim_map_grad")
            return (*grads, None, None)

    return Conv2DSame, Conv2DTransposeSame, Gauss1D, SsimMap


_FNS = None


def _fns():
    global _FNS
    if _FNS is None:
        _FNS = _conv_fn()
    return _FNS


def conv_same(x, kernel_hwio, bias, stride: int, act: bool = True):
    """Keras Conv2D(padding='SAME') + leaky_relu(0.2) on NHWC (HIP, activation in the epilogue)."""
    return _fns()[0].apply(x, kernel_hwio, bias, stride, bool(act))


def tconv_same(x, kernel_hwoi, bias, stride: int):
    """Keras Conv2DTranspose(padding='SAME') + leaky_relu(0.2) on NHWC (HIP, activation in the epilogue)."""
    return _fns()[1].apply(x, kernel_hwoi, bias, stride, True)


SSIM_PIX = 1024  # map pixels per block of nic_ssim_map (its work: one partial sum per block)


def ssim_map_mean(mx, my, sxy, sxx, c1: float, c2: float):
    """(N,) per-plane mean of tf.image.ssim's map from its filtered terms (HIP, differentiable)."""
    return _fns()[3].apply(mx, my, sxy, sxx, float(c1), float(c2))


def gauss_valid(t, g1d):
    """Separable VALID Gaussian of NCHW one-channel planes (N,1,H,W) on the HIP 1-D kernel
    (horizontal then vertical, as training.ssim's filt): returns (N,1,H-10,W-10)."""
    n, c, h, w = t.shape
    if c != 1:
        raise ValueError("gauss_valid: one-channel planes")
    g1d = g1d.contiguous()
    x = _fns()[2].apply(t.reshape(n, h, w), g1d, 0)
    x = _fns()[2].apply(x, g1d, 1)
    return x.reshape(n, 1, x.shape[1], x.shape[2])


def keras_adam_alpha(step: int, lr: float = 1e-4, beta1: float = 0.9, beta2: float = 0.999) -> float:
    """alpha = lr * sqrt(1 - beta2^t) / (1 - beta1^t) in fp32, with Keras' fp32 iteration powers
    (``local_step = iterations + 1``; ``pow(beta, local_step)``) -- the scalar of TF's ApplyAdam."""
    import numpy as np

    f = np.float32
    b1p, b2p = np.power(f(beta1), f(step)), np.power(f(beta2), f(step))
    return float(f(f(lr) * np.sqrt(f(1) - b2p)) / (f(1) - b1p))


class KerasAdam:
    """tf.keras.optimizers.Adam(lr) (training.py:149) on HIP: one ``nic_adam_keras`` launch per
    step over every parameter of the model (m and v kept per parameter, zero-initialised like
    Keras' slots), the update in TF's ApplyAdam order in fp32.  ``step(grads)`` takes the
    gradients in the order of ``params``."""

    def __init__(self, params, lr: float = 1e-4, beta1: float = 0.9, beta2: float = 0.999, epsilon: float = 1e-7):
        torch = _torch()
        self.params = list(params)
        dev = _same_device(*self.params)
        for p in self.params:
            if p.dtype != torch.float32 or not p.is_contiguous():
                raise TypeError("KerasAdam: parameters must be contiguous float32 tensors")
        self.lr, self.beta1, self.beta2, self.epsilon = lr, beta1, beta2, epsilon
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.iterations = 0
        self.device = dev
        self.max_n = max((p.numel() for p in self.params), default=0)
        # the {var, m, v, grad, n} table: a pinned host copy (only the gradient pointers change
        # between steps) and its device twin, reused every step
        import numpy as np

        n = len(self.params)
        self._host = torch.empty((n, 5), dtype=torch.int64, pin_memory=True)
        self._hnp = self._host.numpy()
        self._fill_table()
        self._dev = torch.empty((n, 5), dtype=torch.int64, device=dev)
        self._copied = None  # event: the last table upload has read the pinned buffer

    def _fill_table(self) -> None:
        for i, (p, m, v) in enumerate(zip(self.params, self.m, self.v)):
            self._hnp[i] = (p.data_ptr(), m.data_ptr(), v.data_ptr(), 0, p.numel())
        self._ptrs = [p.data_ptr() for p in self.params]

    def _check_table(self) -> None:
        """A parameter rebound since the table was built (p.data = ..., a reload into new
        tensors) would leave the kernel writing through a stale pointer: re-point the table
        at the current storage (same shapes: the m / v slots still fit)."""
        torch = _torch()
        if all(p.data_ptr() == q for p, q in zip(self.params, self._ptrs)):
            return
        for p, m in zip(self.params, self.m):
            if p.shape != m.shape or p.dtype != torch.float32 or not p.is_contiguous() or p.device != m.device:
                raise TypeError("KerasAdam: a parameter was rebound to a tensor of another shape / dtype / "
                                "layout / device")
        self._fill_table()

    def step(self, grads) -> None:
        torch = _torch()
        grads = [g.detach().contiguous() for g in grads]
        if len(grads) != len(self.params):
            raise ValueError("KerasAdam.step: one gradient per parameter")
        for p, g in zip(self.params, grads):
            if g.shape != p.shape or g.dtype != torch.float32 or g.device != p.device:
                raise ValueError("KerasAdam.step: gradient shape / dtype / device differs from its parameter")
        self.iterations += 1
        alpha = keras_adam_alpha(self.iterations, self.lr, self.beta1, self.beta2)
        with torch.cuda.device(self.device):
            if self._copied is not None:
                self._copied.synchronize()  # the previous upload has read the pinned table
            self._check_table()
            for i, g in enumerate(grads):
                self._hnp[i, 3] = g.data_ptr()
            self._dev.copy_(self._host, non_blocking=True)
            self._copied = torch.cuda.Event()
            self._copied.record()
            _lib.check(_lib.lib().nic_adam_keras(self._dev.data_ptr(), len(grads), self.max_n, alpha, self.beta1,
                                                 self.beta2, self.epsilon, _stream(self.device)), "nic_adam_keras")
        self._keep = grads  # alive until the stream has run the launch

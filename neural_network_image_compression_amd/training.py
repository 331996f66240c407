"""Training side path: tf2_0/src/training.py:44-172 on PyTorch-ROCm autograd.

Not the hot path (the inference kernels are HIP, csrc/); this is the reference's trainer
restated so that trained weights exist for the codec and the config-4 RD sweep:

* ``Entropynet`` (training.py:25-42): conv 64 k5 s2 -> conv 64 k3 -> conv 64 k3 ->
  Flatten (NHWC order, as Keras) -> Dense 512 -> Dense 1 -> clip [0, 8], a learned bpp
  estimate of one latent plane.
* Convolutions (``backend="hip"``, the default): every conv of the step -- encoder,
  decoder, Entropynet; forward, input and kernel gradients -- runs on the HIP split-f16x3
  MFMA kernels of ``csrc/nic_train.hip`` (``train_hip``), NHWC; ``backend="torch"`` keeps
  the PyTorch-autograd restatement (MIOpen) the HIP path is tested against.
* ``Training.__call__`` (training.py:53-165): per batch, /255, random left-right and
  up-down flips per image, RGB -> YCbCr planes, the Y model on Y and the CbCr model on
  Cb||Cr, uniform noise U(-0.5, 0.5)/255 on the latent as the quantisation proxy, the PNG
  bpp of the rounded latent (``get_bpp``, training.py:14-21) as the entropy net's target,
  losses ``(1 - SSIM)/2 + coef * entropy`` (Y) and ``(1 - SSIM)/2 + 0.01 * entropy``
  (CbCr, the reference hard-codes 0.01 there), Adam(1e-4) per Y / CbCr / entropy net,
  ``entropy_loss_coef += 0.01`` per epoch, validation through the HIP codec's
  ``compress``/``uncompress`` every 10 steps.  TF's ``tape.gradient`` of a non-scalar
  loss sums its elements; the losses here are summed the same way.
* ``_save`` (training.py:167-172) writes the reference's own TF checkpoint format
  (``weights.save_tf``), which ``ProClass.load`` / the HIP codec read back.

Parameters are kept in the Keras layouts of ``weights.py`` so they move to and from the
codec unchanged.
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional

import numpy as np

from . import weights as W
from .bitstream import png_sizes

YCBCR = ((0.299, 0.587, 0.114), (-0.16874, -0.33126, 0.5), (0.5, -0.41869, -0.08131))  # utils.py:7
YCBCR_OFF = (0.0, 0.5, 0.5)  # utils.py:9


def _torch():
    import torch

    return torch


def same_pad(n: int, k: int, s: int):
    out = -(-n // s)
    pad = max((out - 1) * s + k - n, 0)
    return pad // 2, pad - pad // 2


def conv_same(x, kernel_hwio, bias, stride: int, act: bool = True):
    """Keras Conv2D(padding='SAME') + leaky_relu(0.2) on NCHW; kernel (kh,kw,Cin,Cout)."""
    import torch.nn.functional as F

    t, b = same_pad(x.shape[2], kernel_hwio.shape[0], stride)
    l, r = same_pad(x.shape[3], kernel_hwio.shape[1], stride)
    y = F.conv2d(F.pad(x, (l, r, t, b)), kernel_hwio.permute(3, 2, 0, 1), bias, stride=stride)
    return F.leaky_relu(y, 0.2) if act else y


def tconv_same(x, kernel_hwoi, bias, stride: int):
    """Keras Conv2DTranspose(padding='SAME') + leaky_relu(0.2); kernel (kh,kw,Cout,Cin)."""
    import torch.nn.functional as F

    n = (x.shape[2] * stride, x.shape[3] * stride)
    pt, _ = same_pad(n[0], kernel_hwoi.shape[0], stride)
    pl, _ = same_pad(n[1], kernel_hwoi.shape[1], stride)
    full = F.conv_transpose2d(x, kernel_hwoi.permute(3, 2, 0, 1), stride=stride)
    full = F.pad(full, (0, max(0, pl + n[1] - full.shape[3]), 0, max(0, pt + n[0] - full.shape[2])))
    y = full[:, :, pt:pt + n[0], pl:pl + n[1]] + bias.view(1, -1, 1, 1)
    return F.leaky_relu(y, 0.2)


def _convs(hip: bool):
    if hip:
        from . import train_hip

        return train_hip.conv_same, train_hip.tconv_same
    return conv_same, tconv_same


def base_encoder(p: Dict[str, object], x, hip: bool = False):
    """encoder.py:7-32 on planes (N,1,H,W) NCHW -> (N,32,h,w), or with ``hip`` on NHWC
    (N,H,W,1) -> (N,h,w,32) through the HIP training convolutions (train_hip)."""
    conv, _ = _convs(hip)
    x = conv(x, p["conv1/kernel"], p["conv1/bias"], 2)
    x = conv(x, p["conv2/kernel"], p["conv2/bias"], 2)
    res = x
    x = conv(x, p["conv3/kernel"], p["conv3/bias"], 1)
    x = conv(x, p["conv4/kernel"], p["conv4/bias"], 1)
    x = conv(x + res, p["conv8/kernel"], p["conv8/bias"], 2)
    return x.clamp(0, 1)


def base_decoder(p: Dict[str, object], x, hip: bool = False):
    """decoder.py:7-32 on latents (N,32,h,w) NCHW -> (N,1,8h,8w), or NHWC with ``hip``."""
    _, tconv = _convs(hip)
    x = tconv(x, p["dconv1/kernel"], p["dconv1/bias"], 2)
    res = x
    x = tconv(x, p["dconv5/kernel"], p["dconv5/bias"], 1)
    x = tconv(x, p["dconv6/kernel"], p["dconv6/bias"], 1)
    x = tconv(x + res, p["dconv7/kernel"], p["dconv7/bias"], 2)
    x = tconv(x, p["dconv8/kernel"], p["dconv8/bias"], 2)
    return x.clamp(0, 1)


def colour_planes(x_norm):
    """convert_to_colourspace (utils.py:64-68, 74-77): NHWC [0,1] -> 3 planes (N,1,H,W)."""
    r, g, b = x_norm[..., 0], x_norm[..., 1], x_norm[..., 2]
    return [(((r * k[0] + g * k[1]) + b * k[2]) + off)[:, None] for k, off in zip(YCBCR, YCBCR_OFF)]


def _gauss_window(torch, device, dtype, size: int = 11, sigma: float = 1.5):
    c = torch.arange(size, dtype=torch.float64) - (size - 1) / 2.0
    g = torch.exp(-0.5 * c * c / sigma ** 2)
    g = g / g.sum()
    return g.to(device=device, dtype=dtype)


def ssim(x, y, max_val: float = 1.0, hip: bool = False):
    """tf.image.ssim (11x11 Gaussian sigma 1.5, k1 0.01, k2 0.03, VALID) of NCHW planes ->
    (N,) mean over the valid map and channels; differentiable.  ``hip``: the Gaussian runs on
    the HIP 1-D kernel and the map's arithmetic with its mean on nic_ssim_map (one-channel planes)."""
    torch = _torch()
    import torch.nn.functional as F

    g = _gauss_window(torch, x.device, x.dtype)
    c = x.shape[1]

    def filt(t):
        if hip:
            from . import train_hip

            return train_hip.gauss_valid(t, g)
        t = F.conv2d(t, g.view(1, 1, 1, -1).expand(c, 1, 1, -1), groups=c)
        return F.conv2d(t, g.view(1, 1, -1, 1).expand(c, 1, -1, 1), groups=c)

    c1, c2 = (0.01 * max_val) ** 2, (0.03 * max_val) ** 2
    mx, my = filt(x), filt(y)
    if hip and c == 1:  # the map and its mean (and their gradients) in one HIP pass each
        from . import train_hip

        return train_hip.ssim_map_mean(mx, my, filt(x * y), filt(x * x + y * y), c1, c2)
    num0 = mx * my * 2.0
    den0 = mx * mx + my * my
    lum = (num0 + c1) / (den0 + c1)
    num1 = filt(x * y) * 2.0
    den1 = filt(x * x + y * y)
    cs = (num1 - num0 + c2) / (den1 - den0 + c2)
    return (lum * cs).mean(dim=(1, 2, 3))


def png_bpp_planes(encoded_u8: np.ndarray, tot_pixels: float, threads: int = 16, mode: str = "tf") -> np.ndarray:
    """get_bpp (training.py:14-21): latent planes (M,h,w,32) u8 -> (M,) 8*len(PNG((4h,8w)))/pixels.

    The PNG sizes are computed natively on ``threads`` host threads (bitstream.png_sizes /
    nic_png_encode).  mode "tf" (default): the settings of ``tf.image.encode_png`` that
    get_bpp calls (training.py:12: libpng defaults, zlib level 6; parity with TF itself
    unpinned, nic.h NIC_PNG_TF); mode "pillow": the bytes save_img writes (utils.py:85-87,
    optimize=True; tested equal to Pillow byte for byte) -- the validation bpp."""
    m, h, w, _ = encoded_u8.shape
    sizes = png_sizes(encoded_u8.reshape(m, 4 * h, 8 * w), threads, mode=mode)
    return (8.0 * sizes.astype(np.float64) / tot_pixels).astype(np.float32)


class Entropynet:
    """training.py:25-42 with Keras-style glorot-uniform kernels and zero biases."""

    def __init__(self, latent_hw, device, seed: int = 0):
        torch = _torch()
        gen = torch.Generator().manual_seed(seed)
        h2, w2 = -(-latent_hw[0] // 2), -(-latent_hw[1] // 2)

        def glorot(shape, fan_in, fan_out):
            lim = (6.0 / (fan_in + fan_out)) ** 0.5
            return ((torch.rand(shape, generator=gen) * 2 - 1) * lim).to(device).requires_grad_()

        self.p = {
            "conv1/kernel": glorot((5, 5, 32, 64), 25 * 32, 25 * 64),
            "conv2/kernel": glorot((3, 3, 64, 64), 9 * 64, 9 * 64),
            "conv3/kernel": glorot((3, 3, 64, 64), 9 * 64, 9 * 64),
            "dense1/kernel": glorot((h2 * w2 * 64, 512), h2 * w2 * 64, 512),
            "dense2/kernel": glorot((512, 1), 512, 1),
        }
        for name, n in (("conv1", 64), ("conv2", 64), ("conv3", 64), ("dense1", 512), ("dense2", 1)):
            self.p[name + "/bias"] = torch.zeros(n, device=device, requires_grad=True)

    def parameters(self) -> List[object]:
        return list(self.p.values())

    def __call__(self, z, hip: bool = False):
        """z: (M,32,h,w) NCHW, or (M,h,w,32) NHWC with ``hip`` (HIP convolutions)."""
        p = self.p
        conv, _ = _convs(hip)
        x = conv(z, p["conv1/kernel"], p["conv1/bias"], 2)
        x = conv(x, p["conv2/kernel"], p["conv2/bias"], 1)
        x = conv(x, p["conv3/kernel"], p["conv3/bias"], 1)
        x = (x if hip else x.permute(0, 2, 3, 1)).reshape(x.shape[0], -1)  # Keras Flatten of NHWC
        x = x @ p["dense1/kernel"] + p["dense1/bias"]
        x = x @ p["dense2/kernel"] + p["dense2/bias"]
        return x.clamp(0, 8)


KERAS_ADAM_EPS = 1e-7
ADAM_BETA2 = 0.999


def keras_adam_eps(step: int, eps: float = KERAS_ADAM_EPS, beta2: float = ADAM_BETA2) -> float:
    """torch.optim.Adam's eps that reproduces tf.keras Adam's update at (1-based) ``step``.

    Keras computes lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t) and theta -= lr_t * m / (sqrt(v) + eps)
    (epsilon-hat, added to the uncorrected sqrt(v)); torch adds eps to sqrt(v_hat) =
    sqrt(v) / sqrt(1 - b2^t).  The two agree when torch's eps = eps / sqrt(1 - b2^t)
    (about 32x the Keras value at step 1, tending to it)."""
    return eps / float(np.sqrt(1.0 - beta2 ** step))


class Training:
    """training.py:44-172.

    Parity notes (unpinned: no TF here): the optimiser follows Keras' Adam exactly
    (:func:`keras_adam_eps`); the entropy net's bpp target sizes the latent planes with
    ``tf.image.encode_png``'s settings as get_bpp does (training.py:12-21: libpng defaults,
    zlib level 6, 8 KiB IDATs; ``png_mode`` "tf", nic.h NIC_PNG_TF) -- a restatement of libpng /
    zlib, not TF's own bytes; validation's val_bpp sizes the files save_img writes (Pillow,
    optimize=True, byte-identical)."""

    def __init__(self, device: str = "cuda", weights: Optional[W.Weights] = None, seed: int = 0,
                 checkpoint_dir: str = "../checkpoints/", backend: Optional[str] = None,
                 png_threads: int = 16):
        """backend "hip" (default on a GPU): every convolution of the step, forward and
        backward, on the HIP split-f16x3 MFMA kernels (train_hip, NHWC); "torch" (default on
        the CPU): PyTorch autograd convolutions (MIOpen / oneDNN, NCHW) -- the restatement the
        HIP path is tested against."""
        torch = _torch()
        backend = backend or ("hip" if torch.device(device).type == "cuda" else "torch")
        if backend not in ("hip", "torch"):
            raise ValueError(f"backend must be 'hip' or 'torch', not {backend!r}")
        self.hip = backend == "hip"
        self.hip_adam = True  # HIP backend: the Keras Adam update on HIP (False: torch.optim.Adam)
        self.device = torch.device(device)
        w = weights if weights is not None else W.seeded_weights(seed, init="glorot")  # Keras defaults
        self.params = {k: torch.tensor(np.asarray(v, np.float32), device=self.device, requires_grad=True)
                       for k, v in w.items()}
        self.seed = seed
        self.epoch = 0
        self.checkpoint_dir = checkpoint_dir
        self.entropy_model: Optional[Entropynet] = None
        self._opt = None
        self._gen = torch.Generator(device=self.device).manual_seed(seed)
        # the PNG-size target (get_bpp, training.py:14-21: 3B PNG encodes per step) runs on
        # host threads (nic_png_encode) while the device runs the codec's backward: train_step
        # needs it only for the entropy net's own loss, after the codec gradients are queued
        self.png_threads = png_threads
        self.png_mode = "tf"  # get_bpp's encoder (training.py:12); "pillow": save_img's
        self._pool = ThreadPoolExecutor(max_workers=1)

    def _model(self, name: str) -> Dict[str, object]:
        pre = name + "/"
        return {k[len(pre):]: v for k, v in self.params.items() if k.startswith(pre)}

    def _variables(self, plane: str) -> List[object]:
        return [v for k, v in self.params.items() if k.startswith("encoder" + plane + "/") or
                k.startswith("decoder" + plane + "/")]

    def _setup(self, hw):
        torch = _torch()
        if self.entropy_model is None:
            self.entropy_model = Entropynet((-(-hw[0] // 8), -(-hw[1] // 8)), self.device, self.seed)
        if self._opt is None:
            # tf.keras.optimizers.Adam(1e-4): beta 0.9 / 0.999, epsilon 1e-7 -- on HIP, TF's
            # ApplyAdam update in fp32 (train_hip.KerasAdam, one launch per model); on the torch
            # backend torch.optim.Adam with Keras' epsilon-hat (see keras_adam_eps)
            if self.hip and self.hip_adam:
                from .train_hip import KerasAdam

                mk = lambda ps: KerasAdam(ps, lr=1e-4, beta1=0.9, beta2=ADAM_BETA2, epsilon=KERAS_ADAM_EPS)  # noqa: E731
            else:
                mk = lambda ps: torch.optim.Adam(ps, lr=1e-4, betas=(0.9, ADAM_BETA2), eps=KERAS_ADAM_EPS)  # noqa: E731
            self._opt = (mk(self._variables("Y")), mk(self._variables("CbCr")), mk(self.entropy_model.parameters()))

    def train_step(self, images, entropy_loss_coef: float, flip: bool = True) -> Dict[str, object]:
        """One batch (training.py:67-147): u8 NHWC images (B,H,W,3) -> metrics."""
        torch = _torch()
        f = self.losses(images, entropy_loss_coef, flip, defer_png=True)
        loss0, loss1 = f["loss0"], f["loss1"]
        opt_y, opt_c, opt_e = self._opt
        ent_params = self.entropy_model.parameters()
        # three tapes: main losses update the codec models only, the entropy loss the net only;
        # the codec gradients are queued while the host threads size the PNG target
        gy = torch.autograd.grad(loss0, self._variables("Y"), retain_graph=True)
        gc = torch.autograd.grad(loss1, self._variables("CbCr"), retain_graph=True)
        aprox_entropy_loss = self.finish_entropy_loss(f)
        ge = torch.autograd.grad(aprox_entropy_loss, ent_params)
        for opt, params, grads in ((opt_y, self._variables("Y"), gy), (opt_c, self._variables("CbCr"), gc),
                                   (opt_e, ent_params, ge)):
            if not isinstance(opt, torch.optim.Optimizer):  # train_hip.KerasAdam
                opt.step(grads)
                continue
            for prm, g in zip(params, grads):
                prm.grad = g
            for group in opt.param_groups:  # Keras' epsilon-hat at this step (keras_adam_eps)
                st = opt.state.get(group["params"][0], {}).get("step", 0)
                group["eps"] = keras_adam_eps(int(st) + 1)
            opt.step()
            opt.zero_grad(set_to_none=True)
        b = images.shape[0]
        cb, cr = torch.split(f["ssim1_each"].detach(), b)
        bpp = f["bpp"]
        return {"ssim": [float(f["ssim0"].detach()), float(cb.mean()), float(cr.mean())],
                "bpp": [float(v.mean()) for v in np.split(bpp, 3)],
                "entropy_loss": float(aprox_entropy_loss.detach()), "loss": [float(loss0.detach()), float(loss1.detach())]}

    def _png_target(self, codes, pixels: float):
        """Start get_bpp of the step's u8 codes (M,h,w,32) on a host thread: an async copy to
        page-locked memory, then the native PNG sizes once it has landed.  Returns a future."""
        torch = _torch()
        threads, mode = self.png_threads, self.png_mode
        if codes.is_cuda:
            host = torch.empty(codes.shape, dtype=torch.uint8, pin_memory=True)
            host.copy_(codes, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()

            def job():
                ev.synchronize()
                return png_bpp_planes(host.numpy(), pixels, threads, mode)
        else:
            arr = codes.numpy().copy()

            def job():
                return png_bpp_planes(arr, pixels, threads, mode)
        return self._pool.submit(job)

    def finish_entropy_loss(self, f: Dict[str, object]):
        """The entropy net's loss (training.py:93-101) once the PNG target is in: MSE between
        its estimate and get_bpp of the codes.  Sets f["bpp"] and f["entropy_loss"]."""
        torch = _torch()
        if "entropy_loss" not in f:
            bpp = f.pop("bpp_future").result()
            bpp_t = torch.from_numpy(bpp).to(self.device).view(-1, 1)
            f["bpp"] = bpp
            f["entropy_loss"] = ((bpp_t - f["aprox"]) ** 2).mean()
        return f["entropy_loss"]

    def losses(self, images, entropy_loss_coef: float, flip: bool = True, defer_png: bool = False) -> Dict[str, object]:
        """The step's forward pass (training.py:67-126): the two codec losses, the entropy
        net's loss and the tensors the metrics read (differentiable w.r.t. the parameters).
        defer_png: leave the PNG target running (f["bpp_future"]); finish_entropy_loss
        completes f["entropy_loss"] / f["bpp"] later."""
        torch = _torch()
        x = images.to(self.device)
        b = x.shape[0]
        self._setup(x.shape[1:3])
        img = x.float() / 255
        if flip:  # random_flip_left_right / random_flip_up_down, per image
            lr = torch.rand(b, generator=self._gen, device=self.device) < 0.5
            ud = torch.rand(b, generator=self._gen, device=self.device) < 0.5
            img = torch.where(lr.view(-1, 1, 1, 1), img.flip(2), img)
            img = torch.where(ud.view(-1, 1, 1, 1), img.flip(1), img)
        planes = colour_planes(img)
        p0, p1 = planes[0], torch.cat(planes[1:], dim=0)
        hip = self.hip
        if hip:  # one channel: (N,1,H,W) and (N,H,W,1) share their memory layout
            p0, p1 = p0.reshape(p0.shape[0], *p0.shape[2:], 1), p1.reshape(p1.shape[0], *p1.shape[2:], 1)
        enc0 = base_encoder(self._model("encoderY"), p0, hip)
        enc1 = base_encoder(self._model("encoderCbCr"), p1, hip)

        def noise(t):  # drawn in NCHW order in both layouts (same stream of numbers)
            shape = (t.shape[0], t.shape[3], t.shape[1], t.shape[2]) if hip else t.shape
            u = torch.rand(shape, generator=self._gen, device=self.device) - 0.5
            return u.permute(0, 2, 3, 1) if hip else u

        noisy0 = (enc0 + noise(enc0) / 255).clamp(0, 1)
        noisy1 = (enc1 + noise(enc1) / 255).clamp(0, 1)
        batch_enc = torch.cat([enc0, enc1], dim=0)
        aprox = self.entropy_model(batch_enc, hip)  # (3B, 1)
        codes = torch.round(batch_enc.detach() * 255).clamp(0, 255).to(torch.uint8)
        codes = codes if hip else codes.permute(0, 2, 3, 1)
        bpp_future = self._png_target(codes.contiguous(), float(x.shape[1] * x.shape[2]))
        ent = torch.split(aprox, b, dim=0)
        dec0 = base_decoder(self._model("decoderY"), noisy0, hip)
        dec1 = base_decoder(self._model("decoderCbCr"), noisy1, hip)
        if hip:  # back to (N,1,H,W) views for the SSIM filter
            p0, p1, dec0, dec1 = (t.reshape(t.shape[0], 1, *t.shape[1:3]) for t in (p0, p1, dec0, dec1))
        ssim0 = ssim(p0, dec0, hip=hip).mean()
        ssim1_each = ssim(p1, dec1, hip=hip)
        ssim1 = ssim1_each.mean()
        loss0 = ((1 - ssim0) / 2 + entropy_loss_coef * ent[0]).sum()
        loss1 = ((1 - ssim1) / 2 + 0.01 * torch.cat(ent[1:], dim=0)).sum()  # reference: 0.01 (training.py:124)
        f = {"loss0": loss0, "loss1": loss1, "ssim0": ssim0, "ssim1_each": ssim1_each, "aprox": aprox,
             "bpp_future": bpp_future}
        if not defer_png:
            self.finish_entropy_loss(f)
        return f

    def weights(self) -> W.Weights:
        return {k: v.detach().float().cpu().numpy().copy() for k, v in self.params.items()}

    def _save(self) -> None:
        """training.py:167-172, in the reference's TF checkpoint format."""
        w = self.weights()
        W.save_tf(w, os.path.join(self.checkpoint_dir, "encoder"), "encoder")
        W.save_tf(w, os.path.join(self.checkpoint_dir, "decoder"), "decoder")

    def __call__(self, x: np.ndarray, x_val_path: Optional[str], max_epochs: int, batch_size: int,
                 entropy_loss_coef: float, verbose: bool = True,
                 epoch_samples: Optional[int] = None, coef_step: float = 0.01) -> List[Dict[str, object]]:
        """training.py:53-165: epochs over shuffled batches of the u8 array x (N,H,W,3).
        ``epoch_samples``: the epoch length in images when x is a subset of the reference's
        training set (each epoch then walks that many images over reshuffled passes of x, so
        the per-epoch coefficient schedule keeps the reference's pace); None = one pass.
        ``coef_step``: the coefficient's increment after every epoch (training.py:165: 0.01;
        0 trains at a fixed coefficient, an RD-sweep option the reference does not have)."""
        torch = _torch()
        rng = np.random.default_rng(self.seed)
        log = []
        step = 0
        per_epoch = epoch_samples or len(x)
        for epoch in range(self.epoch, max_epochs):
            self.epoch = epoch
            order = np.concatenate([rng.permutation(len(x)) for _ in range(-(-per_epoch // len(x)))])[:per_epoch]
            for i in range(0, per_epoch, batch_size):
                m = self.train_step(torch.from_numpy(np.ascontiguousarray(x[order[i:i + batch_size]])),
                                    entropy_loss_coef)
                m["epoch"] = epoch
                log.append(m)
                if verbose:
                    print("EPOCH:", epoch, "SSIM:", m["ssim"], "BPP:", m["bpp"], "Entropy loss:", m["entropy_loss"])
                step += 1
                if x_val_path is not None and step % 10 == 0:
                    self._validate(x_val_path)
            entropy_loss_coef += coef_step
        return log

    def _validate(self, x_val_path: str) -> None:
        """training.py:152-163: save, compress / uncompress the validation set with the HIP
        codec, write per-image PNG bpp to <val>_compressed/val_bpp.txt."""
        from .bitstream import read_dataset
        from .codec import Decoder, Encoder

        self._save()
        enc, dec = Encoder(), Decoder()
        enc.compress(x_val_path, os.path.join(self.checkpoint_dir, "encoder"), workers=8)
        comp = x_val_path + "_compressed"
        dec.uncompress(comp, os.path.join(self.checkpoint_dir, "decoder"), workers=8)
        imgs, names = read_dataset(x_val_path)
        pixels = {n: a.shape[0] * a.shape[1] for a, n in zip(imgs, names)}
        with open(os.path.join(comp, "val_bpp.txt"), "w") as f:
            for fn in sorted(os.listdir(comp)):
                if fn.endswith(".png"):
                    stem = fn[:-4]
                    f.write(f"{fn}\t{8 * os.path.getsize(os.path.join(comp, fn)) / pixels[stem]}\n")

"""CPU ORACLE — test infrastructure only, never the product path.

A NumPy restatement of the reference's TF2 encode -> decode hot path
(AlexFuster/Neural_network_image_compression, ``tf2_0/src``) and of its entropy
estimator (``tf1_13/src/training.py:66-71``).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it,
and only as the checker / the timed CPU baseline.

PARITY UNPINNED at the TensorFlow boundary: TensorFlow is not installed in this
container (``import tensorflow`` -> ModuleNotFoundError), the reference ships no
checkpoints, golden vectors or known-answer tests, so nothing
produced by the reference itself can pin this restatement.  It is instead
(1) derived line by line from the cited reference code plus TF's documented op
semantics (SAME padding, Conv2DTranspose as the conv adjoint, half-to-even
rounding), (2) cross-checked against an independent PyTorch-CPU restatement
(tests/test_oracle.py), and (3) frozen as golden fixtures under tests/golden/.

Numerics.  TF runs every op in fp32.  Elementwise ops here are evaluated in fp32 in
the reference's operation order (each product and sum rounded separately, no FMA).
Convolutions accumulate in float64 (``acc=np.float64``, the reference of record: the
correctly rounded fp32 result TF's fp32 kernels approximate) or in fp32
(``acc=np.float32``, BLAS sgemm; the timed CPU baseline), then round to fp32 before the
bias add, exactly as Keras' Conv -> BiasAdd -> activation sequence.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

F32 = np.float32

# --- colour constants -------------------------------------------------------------
# utils.py:7-9.  The kernel is float64; TF converts each scalar to fp32 when it meets
# an fp32 tensor (utils.py:64-68), so the arithmetic uses fp32(k).
YCBCR_KERNEL_F64 = np.array([[0.299, 0.587, 0.114],
                             [-0.16874, -0.33126, 0.5],
                             [0.5, -0.41869, -0.08131]])
YCBCR_INV_KERNEL_F64 = np.linalg.inv(YCBCR_KERNEL_F64)  # utils.py:8
YCBCR_OFF_F64 = np.array([0, 0.5, 0.5])                  # utils.py:9
YCBCR_KERNEL = YCBCR_KERNEL_F64.astype(F32)
YCBCR_INV_KERNEL = YCBCR_INV_KERNEL_F64.astype(F32)
YCBCR_OFF = YCBCR_OFF_F64.astype(F32)

LEAKY_ALPHA = F32(0.2)  # tf.nn.leaky_relu default (encoder.py:10, decoder.py:10)
LOG2_F32 = F32(np.log(np.float32(2)))  # tf1_13/src/training.py:28 logof2


def normalise_u8(x: np.ndarray) -> np.ndarray:
    """``x.astype(np.float32) / 255`` (encoder.py:39, decoder.py:40): correctly rounded fp32."""
    return x.astype(F32) / F32(255)


def _project(k: np.ndarray, t0, t1, t2):
    """utils.py:64-68, fp32, ((t0*k0 + t1*k1) + t2*k2), every op rounded."""
    outs = []
    for r in range(3):
        a = t0 * k[r, 0]
        b = t1 * k[r, 1]
        c = t2 * k[r, 2]
        outs.append((a + b) + c)
    return outs


def convert_to_colourspace(x_norm: np.ndarray) -> List[np.ndarray]:
    """utils.py:74-77: split RGB, project, add offsets.  Returns [Y, Cb, Cr], each (N,H,W,1) fp32."""
    t0, t1, t2 = (x_norm[..., i:i + 1] for i in range(3))
    o = _project(YCBCR_KERNEL, t0, t1, t2)
    return [o[i] + YCBCR_OFF[i] for i in range(3)]


def convert_to_rgb(y: np.ndarray, cb: np.ndarray, cr: np.ndarray) -> np.ndarray:
    """utils.py:70-72 on NumPy-1.x fp32 arrays (decoder.py:45-46): subtract offsets, project, concat."""
    o = _project(YCBCR_INV_KERNEL, y - YCBCR_OFF[0], cb - YCBCR_OFF[1], cr - YCBCR_OFF[2])
    return np.concatenate(o, axis=3)


def quantise_u8(v: np.ndarray) -> np.ndarray:
    """``np.round(v * 255).astype(np.uint8)`` (encoder.py:47, decoder.py:48): fp32 multiply,
    round half to even.  ``v`` is already clipped to [0, 1]."""
    return np.round(v.astype(F32) * F32(255)).astype(np.uint8)


# --- TF 'SAME' convolutions ---------------------------------------------------------

def same_pads(n: int, k: int, s: int) -> Tuple[int, int, int]:
    """TF SAME geometry for one spatial dim: (out, pad_lo, pad_hi)."""
    out = -(-n // s)
    pad = max((out - 1) * s + k - n, 0)
    return out, pad // 2, pad - pad // 2


def leaky(z: np.ndarray) -> np.ndarray:
    """tf.nn.leaky_relu(z, 0.2) = max(0.2*z, z) in fp32."""
    return np.maximum(z * LEAKY_ALPHA, z)


def conv2d_same(x: np.ndarray, kernel: np.ndarray, stride: int, acc=np.float64) -> np.ndarray:
    """Keras Conv2D(padding='SAME') without bias: x (N,H,W,Cin) fp32, kernel HWIO.

    Cross-correlation, asymmetric TF padding (pad_lo = floor(pad/2)).  Accumulates in
    ``acc`` and rounds the sum to fp32.
    """
    n, h, w, cin = x.shape
    kh, kw, kcin, cout = kernel.shape
    assert kcin == cin, (kernel.shape, x.shape)
    oh, ph0, ph1 = same_pads(h, kh, stride)
    ow, pw0, pw1 = same_pads(w, kw, stride)
    xp = np.pad(x.astype(acc), ((0, 0), (ph0, ph1), (pw0, pw1), (0, 0)))
    kern = kernel.astype(acc)
    out = np.zeros((n * oh * ow, cout), dtype=acc)
    for i in range(kh):
        for j in range(kw):
            patch = xp[:, i:i + stride * (oh - 1) + 1:stride, j:j + stride * (ow - 1) + 1:stride, :]
            out += patch.reshape(-1, cin) @ kern[i, j]
    return out.reshape(n, oh, ow, cout).astype(F32)


def conv2d_transpose_same(x: np.ndarray, kernel: np.ndarray, stride: int, acc=np.float64) -> np.ndarray:
    """Keras Conv2DTranspose(padding='SAME') without bias: x (N,h,w,Cin), kernel (kh,kw,Cout,Cin).

    Output size n*s per dim.  Defined as the adjoint of the SAME conv mapping n*s -> n:
    ``y[j] = sum_i x[i] * w[j - s*i + pad_lo]`` with pad_lo of that forward conv; computed
    here by scattering each tap and cropping (independent of the phase decomposition the
    GPU kernels use).
    """
    n, h, w, cin = x.shape
    kh, kw, cout, kcin = kernel.shape
    assert kcin == cin, (kernel.shape, x.shape)
    oh, ow = h * stride, w * stride
    _, ph0, _ = same_pads(oh, kh, stride)
    _, pw0, _ = same_pads(ow, kw, stride)
    full_h = (h - 1) * stride + kh
    full_w = (w - 1) * stride + kw
    full = np.zeros((n, full_h, full_w, cout), dtype=acc)
    xf = x.astype(acc).reshape(-1, cin)
    kern = kernel.astype(acc)
    for i in range(kh):
        for j in range(kw):
            contrib = (xf @ kern[i, j].T).reshape(n, h, w, cout)
            full[:, i:i + stride * (h - 1) + 1:stride, j:j + stride * (w - 1) + 1:stride, :] += contrib
    need_h = ph0 + oh - full_h
    need_w = pw0 + ow - full_w
    if need_h > 0 or need_w > 0:
        full = np.pad(full, ((0, 0), (0, max(need_h, 0)), (0, max(need_w, 0)), (0, 0)))
    return full[:, ph0:ph0 + oh, pw0:pw0 + ow, :].astype(F32)


def _layer(x, params: Dict[str, np.ndarray], name: str, stride: int, transposed: bool, acc):
    k = params[name + "/kernel"]
    b = params[name + "/bias"]
    z = (conv2d_transpose_same if transposed else conv2d_same)(x, k, stride, acc)
    return leaky(z + b)  # Keras: conv -> BiasAdd -> activation, fp32


def base_encoder(params: Dict[str, np.ndarray], x: np.ndarray, acc=np.float64) -> np.ndarray:
    """BaseEncoder.call (encoder.py:19-32).  params keyed '<layer>/<kernel|bias>'."""
    x = _layer(x, params, "conv1", 2, False, acc)
    x = _layer(x, params, "conv2", 2, False, acc)
    res = x
    x = _layer(x, params, "conv3", 1, False, acc)
    x = _layer(x, params, "conv4", 1, False, acc)
    x = x + res
    x = _layer(x, params, "conv8", 2, False, acc)
    return np.clip(x, F32(0), F32(1))


def base_decoder(params: Dict[str, np.ndarray], x: np.ndarray, acc=np.float64) -> np.ndarray:
    """BaseDecoder.call (decoder.py:19-32)."""
    x = _layer(x, params, "dconv1", 2, True, acc)
    res = x
    x = _layer(x, params, "dconv5", 1, True, acc)
    x = _layer(x, params, "dconv6", 1, True, acc)
    x = x + res
    x = _layer(x, params, "dconv7", 2, True, acc)
    x = _layer(x, params, "dconv8", 2, True, acc)
    return np.clip(x, F32(0), F32(1))


def _model_params(weights: Dict[str, np.ndarray], model: str) -> Dict[str, np.ndarray]:
    pre = model + "/"
    return {k[len(pre):]: v for k, v in weights.items() if k.startswith(pre)}


def run_model(weights, kind: str, planes: Sequence[np.ndarray], acc=np.float64) -> List[np.ndarray]:
    """ProClass.run_model (utils.py:19-24): model 0 (Y) on plane 0, shared model 1 (CbCr) on 1 and 2."""
    fn = base_encoder if kind == "encoder" else base_decoder
    py = _model_params(weights, kind + "Y")
    pc = _model_params(weights, kind + "CbCr")
    return [fn(py, planes[0], acc), fn(pc, planes[1], acc), fn(pc, planes[2], acc)]


def encode_f32(weights, x_u8: np.ndarray, acc=np.float64) -> np.ndarray:
    """Encoder.__call__ up to the quantiser (encoder.py:38-45): (N,H,W,3) u8 -> (N,h,w,96) fp32 in [0,1]."""
    assert x_u8.dtype == np.uint8 and x_u8.ndim == 4 and x_u8.shape[3] == 3
    planes = convert_to_colourspace(normalise_u8(x_u8))
    return np.concatenate(run_model(weights, "encoder", planes, acc), axis=3)


def encode(weights, x_u8: np.ndarray, acc=np.float64) -> np.ndarray:
    """Encoder.__call__ (encoder.py:38-47): u8 RGB -> u8 latent (N, ceil(H/8), ceil(W/8), 96)."""
    return quantise_u8(encode_f32(weights, x_u8, acc))


def decode_f32(weights, z_u8: np.ndarray, acc=np.float64) -> np.ndarray:
    """Decoder.__call__ up to the output quantiser (decoder.py:39-46): clipped fp32 RGB."""
    assert z_u8.dtype == np.uint8 and z_u8.ndim == 4 and z_u8.shape[3] == 96
    zn = normalise_u8(z_u8)
    planes = [zn[..., 32 * i:32 * (i + 1)] for i in range(3)]  # tf.split(., 3, axis=3)
    y, cb, cr = run_model(weights, "decoder", planes, acc)
    return np.clip(convert_to_rgb(y, cb, cr), F32(0), F32(1))


def decode(weights, z_u8: np.ndarray, acc=np.float64) -> np.ndarray:
    """Decoder.__call__ (decoder.py:39-48): u8 latent -> u8 RGB (N, 8h, 8w, 3)."""
    return quantise_u8(decode_f32(weights, z_u8, acc))


# --- bitstream layout (utils.py:30-44) ------------------------------------------------

def pack_latent(z: np.ndarray) -> np.ndarray:
    """utils.py:39-40: (n,h,w,96) -> (n,4h,8w,3), plane p = raw C-order reshape of channels 32p..32p+31."""
    n, h, w, c = z.shape
    assert c == 96
    return np.concatenate([z[..., 32 * i:32 * (i + 1)].reshape((n, h * 4, w * 8, 1)) for i in range(3)], axis=3)


def unpack_latent(img: np.ndarray) -> np.ndarray:
    """utils.py:35-36: (n,4h,8w,3) -> (n,h,w,96)."""
    n, h, w, c = img.shape
    assert c == 3
    return np.concatenate([img[..., i].reshape((n, h // 4, w // 8, 32)) for i in range(3)], axis=3)


# --- entropy estimation -------------------------------------------------------------

def latent_planes(z: np.ndarray) -> np.ndarray:
    """Plane-major stack as tf1_13/src/training.py:62 (concat of Y, Cb, Cr along the batch):
    (3N, h*w*32) codes; row p = plane p//N of image p%N."""
    n = z.shape[0]
    return np.concatenate([z[..., 32 * i:32 * (i + 1)].reshape(n, -1) for i in range(3)], axis=0)


def histograms(z: np.ndarray) -> np.ndarray:
    """(3N, 256) int64 code counts (training.py:68's per-bin tf.equal + reduce_sum)."""
    flat = latent_planes(z)
    return np.stack([np.bincount(r, minlength=256) for r in flat]).astype(np.int64)


def hist_entropy(z: np.ndarray) -> np.ndarray:
    """tf1_13/src/training.py:66-71: per plane-image H = sum_i p_i * (-log(clip(p_i,1e-5,1)) / log 2).

    Terms in fp32 exactly as TF; summed in float64 and rounded to fp32 (TF's reduce order is
    unspecified).  Returns (3N, 1) fp32 bits/symbol.
    """
    counts = histograms(z)
    n_sym = F32(latent_planes(z).shape[1])
    p = counts.astype(F32) / n_sym
    logp = np.log(np.clip(p, F32(1e-5), F32(1.0)))
    terms = p * (-logp / LOG2_F32)
    return terms.astype(np.float64).sum(axis=1).astype(F32).reshape(-1, 1)


# --- quality metrics ----------------------------------------------------------------

def psnr(a: np.ndarray, b: np.ndarray, max_val: float = 255.0) -> float:
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    if mse == 0:
        return float("inf")
    return float(10 * np.log10(max_val ** 2 / mse))


# --- MS-SSIM (tf2_0/tests/calc_ssim.py:13: tf.image.ssim_multiscale(img1, img2, max_val=255)) ---
# Restated from TensorFlow's documented algorithm (tf.image.ssim_multiscale, TF 1.13/2.0):
# uint8 -> float32 by x * (1/255) (convert_image_dtype), max_val -> 1.0; 11x11 Gaussian
# (sigma 1.5, softmax-normalised), VALID depthwise filtering, k1 = 0.01, k2 = 0.03;
# 5 scales with power factors (0.0448, 0.2856, 0.3001, 0.2363, 0.1333); between scales a
# 2x2 VALID average pool after SYMMETRIC padding of odd sizes; cs (contrast-structure) of
# scales 0..3 and SSIM of scale 4, each relu'd, combined as a weighted geometric mean,
# then averaged over colour channels.  Evaluated in float64 here.
MSSSIM_WEIGHTS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)


def _fspecial_gauss(size: int = 11, sigma: float = 1.5) -> np.ndarray:
    coords = np.arange(size, dtype=np.float64) - (size - 1) / 2.0
    g = coords ** 2 * (-0.5 / sigma ** 2)
    g = g[None, :] + g[:, None]
    g = np.exp(g - g.max())
    return g / g.sum()


def _filter_valid(x: np.ndarray, k: np.ndarray) -> np.ndarray:
    """Depthwise 'VALID' correlation of (N,H,W,C) with a separable-free (s,s) kernel."""
    s = k.shape[0]
    n, h, w, c = x.shape
    out = np.zeros((n, h - s + 1, w - s + 1, c))
    for i in range(s):
        for j in range(s):
            out += k[i, j] * x[:, i:i + h - s + 1, j:j + w - s + 1, :]
    return out


def _ssim_per_channel(x, y, max_val=1.0, k1=0.01, k2=0.03, kernel=None):
    kernel = _fspecial_gauss() if kernel is None else kernel
    c1, c2 = (k1 * max_val) ** 2, (k2 * max_val) ** 2
    mean0, mean1 = _filter_valid(x, kernel), _filter_valid(y, kernel)
    num0 = mean0 * mean1 * 2.0
    den0 = mean0 ** 2 + mean1 ** 2
    luminance = (num0 + c1) / (den0 + c1)
    num1 = _filter_valid(x * y, kernel) * 2.0
    den1 = _filter_valid(x ** 2 + y ** 2, kernel)
    cs = (num1 - num0 + c2) / (den1 - den0 + c2)
    return (luminance * cs).mean(axis=(1, 2)), cs.mean(axis=(1, 2))


def ms_ssim_scale_sizes(h: int, w: int) -> List[Tuple[int, int]]:
    """Image size at each of the 5 scales: odd sizes are SYMMETRIC-padded by one, then 2x2
    pooled, so every scale is ceil(previous / 2)."""
    sizes = [(h, w)]
    for _ in range(len(MSSSIM_WEIGHTS) - 1):
        h, w = -(-h // 2), -(-w // 2)
        sizes.append((h, w))
    return sizes


def ms_ssim_supported(h: int, w: int, filter_size: int = 11) -> bool:
    """TF's _ssim_per_channel asserts every scale's H, W >= filter_size: 161 px and up."""
    return all(min(s) >= filter_size for s in ms_ssim_scale_sizes(h, w))


def ms_ssim_terms(img1: np.ndarray, img2: np.ndarray) -> np.ndarray:
    """Per-scale terms of ms_ssim: (N,C,5,2) float64 = (mean SSIM, mean cs) per channel and
    scale, before the relu and the weighted geometric mean."""
    if not ms_ssim_supported(img1.shape[1], img1.shape[2]):
        raise ValueError(f"MS-SSIM needs every one of the 5 scales to hold the 11x11 window "
                         f"(H, W >= 161), got {img1.shape[1:3]}")
    x = img1.astype(np.float64) * np.float32(1.0 / 255)
    y = img2.astype(np.float64) * np.float32(1.0 / 255)
    terms = []
    for k in range(len(MSSSIM_WEIGHTS)):
        if k > 0:
            h, w = x.shape[1], x.shape[2]
            if h % 2 or w % 2:
                pad = ((0, 0), (0, h % 2), (0, w % 2), (0, 0))
                x, y = np.pad(x, pad, mode="symmetric"), np.pad(y, pad, mode="symmetric")
            x = 0.25 * (x[:, 0::2, 0::2] + x[:, 1::2, 0::2] + x[:, 0::2, 1::2] + x[:, 1::2, 1::2])
            y = 0.25 * (y[:, 0::2, 0::2] + y[:, 1::2, 0::2] + y[:, 0::2, 1::2] + y[:, 1::2, 1::2])
        terms.append(np.stack(_ssim_per_channel(x, y), axis=-1))
    return np.stack(terms, axis=2)


def ms_ssim(img1: np.ndarray, img2: np.ndarray) -> np.ndarray:
    """tf.image.ssim_multiscale(img1, img2, max_val=255) for u8 (N,H,W,C) -> (N,).

    Like TF, every one of the 5 scales must still hold the 11x11 window: H, W >= 161."""
    t = ms_ssim_terms(img1, img2)
    # cs of scales 0..3 and SSIM of the last scale, each relu'd
    mcs = np.concatenate([t[:, :, :-1, 1], t[:, :, -1:, 0]], axis=-1)
    return np.prod(np.maximum(mcs, 0) ** np.asarray(MSSSIM_WEIGHTS), axis=-1).mean(axis=-1)

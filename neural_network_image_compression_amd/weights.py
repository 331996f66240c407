"""Codec parameter table, seeded initialisation and on-disk weight format.

The four Keras models of the reference and their layer stacks:

* ``BaseEncoder`` (tf2_0/src/encoder.py:7-17): conv1 1->32 k5 s2, conv2 32->64 k5 s2,
  conv3 64->64 k3 s1, conv4 64->64 k3 s1, conv8 64->32 k5 s2.  Keras ``Conv2D``
  kernels are HWIO ``(kh, kw, Cin, Cout)``.
* ``BaseDecoder`` (tf2_0/src/decoder.py:7-17): dconv1 32->64 k5 s2, dconv5 / dconv6
  64->64 k3 s1, dconv7 64->64 k5 s2, dconv8 64->1 k5 s2.  Keras ``Conv2DTranspose``
  kernels are ``(kh, kw, Cout, Cin)``.

``ProClass`` (tf2_0/src/utils.py:15-28) holds two instances of each: model 0 runs the
Y plane, model 1 (shared) runs Cb and Cr.  Checkpoints are written per model as
``'../checkpoints/encoder' + name`` with name in ``['Y', 'CbCr']``
(training.py:167-172; loaded by utils.py:26-28).

No trained checkpoint ships with the reference, so parity work uses *seeded* weights
from a NumPy PCG64 stream (:func:`seeded_weights`): either Keras' own defaults
(glorot_uniform, zero bias) or a variance-preserving "spread" init whose latents and
reconstructions are not collapsed by the clips.

The on-disk format is safetensors keyed ``<model>/<layer>/{kernel,bias}`` in the Keras
layouts above, one file per model (``<prefix>Y.safetensors``, ``<prefix>CbCr.safetensors``),
mirroring ``ProClass.load(path)``'s ``path + 'Y'`` / ``path + 'CbCr'`` convention.
"""
from __future__ import annotations

import hashlib
import os
from dataclasses import dataclass
from typing import Dict, Iterable, List, Tuple

import numpy as np

#: checkpoint suffixes, utils.py:5
PLANE_MODELS = ("Y", "CbCr")


@dataclass(frozen=True)
class LayerSpec:
    name: str
    k: int
    stride: int
    cin: int
    cout: int
    transposed: bool

    @property
    def kernel_shape(self) -> Tuple[int, int, int, int]:
        if self.transposed:  # Conv2DTranspose: (kh, kw, Cout, Cin)
            return (self.k, self.k, self.cout, self.cin)
        return (self.k, self.k, self.cin, self.cout)  # Conv2D: HWIO


#: encoder.py:10-17 (conv5..7 are commented out in the reference)
ENCODER_LAYERS: Tuple[LayerSpec, ...] = (
    LayerSpec("conv1", 5, 2, 1, 32, False),
    LayerSpec("conv2", 5, 2, 32, 64, False),
    LayerSpec("conv3", 3, 1, 64, 64, False),
    LayerSpec("conv4", 3, 1, 64, 64, False),
    LayerSpec("conv8", 5, 2, 64, 32, False),
)

#: decoder.py:10-17 (dconv2..4 are commented out in the reference)
DECODER_LAYERS: Tuple[LayerSpec, ...] = (
    LayerSpec("dconv1", 5, 2, 32, 64, True),
    LayerSpec("dconv5", 3, 1, 64, 64, True),
    LayerSpec("dconv6", 3, 1, 64, 64, True),
    LayerSpec("dconv7", 5, 2, 64, 64, True),
    LayerSpec("dconv8", 5, 2, 64, 1, True),
)

#: model id -> (model name, layer table).  Ids are the C-ABI's ``model_id``.
MODELS: Tuple[Tuple[str, Tuple[LayerSpec, ...]], ...] = (
    ("encoderY", ENCODER_LAYERS),
    ("encoderCbCr", ENCODER_LAYERS),
    ("decoderY", DECODER_LAYERS),
    ("decoderCbCr", DECODER_LAYERS),
)
MODEL_NAMES = tuple(m for m, _ in MODELS)
MODEL_ID = {m: i for i, m in enumerate(MODEL_NAMES)}

Weights = Dict[str, np.ndarray]


def layer_table(model: str) -> Tuple[LayerSpec, ...]:
    return dict(MODELS)[model]


def keys(models: Iterable[str] = MODEL_NAMES) -> List[str]:
    out = []
    for m in models:
        for spec in layer_table(m):
            out += [f"{m}/{spec.name}/kernel", f"{m}/{spec.name}/bias"]
    return out


def expected_shape(key: str) -> Tuple[int, ...]:
    model, layer, kind = key.split("/")
    spec = {s.name: s for s in layer_table(model)}[layer]
    return spec.kernel_shape if kind == "kernel" else (spec.cout,)


def glorot_limit(shape: Tuple[int, ...]) -> float:
    """keras.initializers.glorot_uniform: fans from kernel shape (receptive field x dims[-2:])."""
    receptive = int(np.prod(shape[:-2]))
    fan_in, fan_out = shape[-2] * receptive, shape[-1] * receptive
    return float(np.sqrt(6.0 / (fan_in + fan_out)))


def fan_in(spec: LayerSpec) -> float:
    """Inputs feeding one output: k*k*Cin, divided by s*s for a strided transposed conv."""
    f = spec.k * spec.k * spec.cin
    return f / (spec.stride ** 2) if spec.transposed else float(f)


#: 'spread' init gains (see seeded_weights)
SPREAD_GAIN_HIDDEN = 1.2
SPREAD_GAIN_LAST = 0.4
SPREAD_LAST_BIAS = 0.45


def seeded_weights(seed: int = 0, init: str = "spread", bias_range: float = 0.02) -> Weights:
    """Deterministic codec weights from a NumPy PCG64 stream.

    ``init='glorot'``: Keras' defaults (glorot_uniform kernels, zero biases).  With these
    the activations shrink layer by layer and the decoder output collapses to a constant
    that the [0,1] clip then hides, which makes a weak parity fixture.

    ``init='spread'`` (default for fixtures and benches): variance-preserving uniform
    kernels, limit = gain*sqrt(3/fan_in) (gain 1.2 hidden, 0.4 on the last layer of each
    model), biases U(-bias_range, bias_range) and +0.45 on the last layer, so latent codes
    and reconstructions spread over most of [0, 255] (kodim21 crop: ~0.3 % zero codes,
    ~7.2 bits/symbol, ~12 % clipped recon samples).

    Draw order: models in MODEL_NAMES order, layers in table order, kernel then bias.
    """
    if init not in ("spread", "glorot"):
        raise ValueError(f"unknown init {init!r}")
    rng = np.random.Generator(np.random.PCG64(seed))
    w: Weights = {}
    for model, layers in MODELS:
        for i, spec in enumerate(layers):
            shape = spec.kernel_shape
            last = i == len(layers) - 1
            if init == "glorot":
                lim = glorot_limit(shape)
            else:
                g = SPREAD_GAIN_LAST if last else SPREAD_GAIN_HIDDEN
                lim = float(np.sqrt(3.0 * g * g / fan_in(spec)))
            w[f"{model}/{spec.name}/kernel"] = rng.uniform(-lim, lim, size=shape).astype(np.float32)
            if init == "glorot":
                b = np.zeros((spec.cout,))
            else:
                b = rng.uniform(-bias_range, bias_range, size=(spec.cout,))
                if last:
                    b = b + SPREAD_LAST_BIAS
            w[f"{model}/{spec.name}/bias"] = b.astype(np.float32)
    return w


def validate(w: Weights, models: Iterable[str] = MODEL_NAMES) -> None:
    for k in keys(models):
        if k not in w:
            raise KeyError(f"missing weight tensor {k!r}")
        a = w[k]
        if tuple(a.shape) != expected_shape(k):
            raise ValueError(f"{k}: shape {tuple(a.shape)} != Keras shape {expected_shape(k)}")
        if a.dtype != np.float32:
            raise TypeError(f"{k}: dtype {a.dtype} != float32")


def digest(w: Weights) -> str:
    """SHA-256 over the tensors in key order (raw little-endian fp32 bytes)."""
    h = hashlib.sha256()
    for k in sorted(w):
        h.update(k.encode())
        h.update(np.ascontiguousarray(w[k], dtype="<f4").tobytes())
    return h.hexdigest()


def split_models(w: Weights, prefix: str) -> Dict[str, Weights]:
    """{'Y': {...}, 'CbCr': {...}} for prefix 'encoder' or 'decoder'."""
    out = {}
    for name in PLANE_MODELS:
        m = prefix + name
        out[name] = {k: v for k, v in w.items() if k.startswith(m + "/")}
    return out


def save(w: Weights, path_prefix: str, kind: str) -> List[str]:
    """Write ``path_prefix + 'Y' + '.safetensors'`` and ``... + 'CbCr' ...`` for kind encoder|decoder.

    Mirrors Training._save (training.py:167-172): one file per plane model.
    """
    from safetensors.numpy import save_file

    paths = []
    for name, sub in split_models(w, kind).items():
        p = path_prefix + name + ".safetensors"
        d = os.path.dirname(p)
        if d:
            os.makedirs(d, exist_ok=True)
        save_file({k: np.ascontiguousarray(v) for k, v in sub.items()}, p)
        paths.append(p)
    return paths


def save_tf(w: Weights, path_prefix: str, kind: str) -> List[str]:
    """The reference's own format: ``Model.save_weights(path_prefix + name)`` for name in
    Y, CbCr (training.py:167-170), i.e. TF object-based tensor bundles keyed
    ``<layer>/<kernel|bias>/.ATTRIBUTES/VARIABLE_VALUE`` plus the TrackableObjectGraph that
    object-based restore walks (see tfckpt.py; loading these files with TF's own
    ``load_weights`` is unpinned: TF is not available here)."""
    from . import tfckpt

    paths = []
    for i, (name, sub) in enumerate(split_models(w, kind).items()):
        m = kind + name + "/"
        tensors = {k[len(m):] + tfckpt.VARIABLE_SUFFIX: np.asarray(v, np.float32) for k, v in sub.items()}
        # Keras names the two instances of BaseEncoder 'base_encoder', 'base_encoder_1'
        scope = "base_" + kind + ("" if i == 0 else f"_{i}")
        paths += tfckpt.write_bundle(path_prefix + name, tensors, tfckpt.encode_object_graph(tensors, scope))
    return paths


def load(path_prefix: str, kind: str) -> Weights:
    """Inverse of :func:`save`; mirrors ProClass.load (utils.py:26-28).

    ``path_prefix + name`` may also be a TF checkpoint written by the reference's
    ``save_weights`` (``<prefix><name>.index`` + ``.data-*``), read without TensorFlow."""
    from safetensors.numpy import load_file

    from . import tfckpt

    w: Weights = {}
    for name in PLANE_MODELS:
        p = path_prefix + name
        if not p.endswith(".safetensors") and os.path.exists(p + ".index"):
            layers = tfckpt.keras_layer_tensors(tfckpt.read_bundle(p))
            order = [spec.name for spec in (ENCODER_LAYERS if kind == "encoder" else DECODER_LAYERS)]
            for k, v in layers.items():
                lname, var = k.split("/")
                # subclassed models key by attribute (conv1/...); functional / Sequential
                # saves key by position (layer_with_weights-0/...)
                if lname.startswith("layer_with_weights-") and lname[19:].isdigit() and int(lname[19:]) < len(order):
                    lname = order[int(lname[19:])]
                if lname in order:
                    w[kind + name + "/" + lname + "/" + var] = np.asarray(v, np.float32)
            continue
        if not p.endswith(".safetensors"):
            p += ".safetensors"
        sub = load_file(p)
        for k, v in sub.items():
            if not k.startswith(kind + name + "/"):
                raise KeyError(f"{p}: unexpected tensor {k!r} for model {kind + name}")
            w[k] = v.astype(np.float32, copy=False)
    validate(w, [kind + n for n in PLANE_MODELS])
    return w

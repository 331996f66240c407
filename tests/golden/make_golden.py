"""Regenerate the golden fixtures in tests/golden/ from the CPU oracle.

    python tests/golden/make_golden.py [--ref-data /root/reference/data]

Inputs come from the reference's own data files (read here as pixel data only):
  * kodim21.png crop [0:256, 0:256]          -> case 'kodim21_256'  (BASELINE config 1)
  * imagenet_patches/00000..00003.jpg (128^2) -> case 'imagenet4'
  * kodim21.png crop [100:137, 200:253]      -> case 'odd37x53'   (TF-SAME odd sizes)
  * kodim21.png crop [0:256, 0:256] with Keras glorot/zero-bias weights -> 'kodim21_glorot'
The decoded pixels are stored, so the GPU box never decodes JPEG/PNG.

Outputs (oracle, float64-accumulated convolutions): u8 latent, fp32 clipped pre-quant
latent, u8 reconstruction of that latent, per-plane histograms and entropy, PSNR.
Weights are regenerated from seeds by neural_network_image_compression_amd.weights; their
SHA-256 is recorded so generator drift is caught.  Parity vs TensorFlow itself is
UNPINNED (no TF here, no reference fixtures): see oracle/nic_oracle.py.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from neural_network_image_compression_amd import weights as W  # noqa: E402
from oracle import nic_oracle as O  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def load_inputs(ref_data: str):
    from PIL import Image

    kod = np.array(Image.open(os.path.join(ref_data, "kodak_img", "kodim21.png")).convert("RGB"))
    patches = [np.array(Image.open(os.path.join(ref_data, "imagenet_patches", f"{i:05d}.jpg")).convert("RGB"))
               for i in range(4)]
    return {
        "kodim21_256": (kod[None, 0:256, 0:256], "spread"),
        "imagenet4": (np.stack(patches), "spread"),
        "odd37x53": (kod[None, 100:137, 200:253], "spread"),
        "kodim21_glorot": (kod[None, 0:256, 0:256], "glorot"),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref-data", default="/root/reference/data")
    args = ap.parse_args()
    manifest = {"seed": 0, "oracle_acc": "float64", "weights": {}, "cases": {}}
    wsets = {init: W.seeded_weights(0, init=init) for init in ("spread", "glorot")}
    for init, w in wsets.items():
        manifest["weights"][init] = W.digest(w)
    for name, (x, init) in load_inputs(args.ref_data).items():
        w = wsets[init]
        x = np.ascontiguousarray(x, dtype=np.uint8)
        f = O.encode_f32(w, x)
        z = O.quantise_u8(f)
        rf = O.decode_f32(w, z)
        r = O.quantise_u8(rf)
        counts = O.histograms(z)
        bits = O.hist_entropy(z)
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), x=x, latent=z, prequant=f, recon=r,
                            counts=counts.astype(np.int32), bits=bits)
        # distance of x*255 to the nearest .5 rounding boundary (codes that may flip)
        v = f.astype(np.float64) * 255
        near = int(np.sum(np.abs(v - np.floor(v) - 0.5) < 1e-3))
        manifest["cases"][name] = {
            "init": init, "x_shape": list(x.shape), "latent_shape": list(z.shape), "recon_shape": list(r.shape),
            "psnr_db": O.psnr(x, r[:, :x.shape[1], :x.shape[2]]),
            "zero_codes": float(np.mean(z == 0)), "bits_mean": float(bits.mean()),
            "codes_near_half": near, "recon_clipped": float(np.mean((rf == 0) | (rf == 1))),
        }
        print(name, manifest["cases"][name])
    with open(os.path.join(OUT, "manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()

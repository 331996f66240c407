"""Regenerate the golden fixtures in tests/golden/ from the CPU oracle.

    python tests/golden/make_golden.py [--ref-data /root/reference/data]

Inputs come from the reference's own data files (read here as pixel data only):
  * kodim21.png crop [0:256, 0:256]          -> case 'kodim21_256'  (BASELINE config 1)
  * imagenet_patches/00000..00003.jpg (128^2) -> case 'imagenet4'
  * kodim21.png crop [100:137, 200:253]      -> case 'odd37x53'   (TF-SAME odd sizes)
  * kodim21.png crop [0:256, 0:256] with Keras glorot/zero-bias weights -> 'kodim21_glorot'
  * the whole kodim21.png (512 x 768)          -> case 'kodim21_full'  (BASELINE config 4, whole)
  * its six 256^2 tiles (2 rows x 3 columns)  -> case 'kodim21_tiles' (config 4, tiled)
  * kodim21_256 and imagenet4 with the TRAINED codecs of coefficients 0.01 / 0.02 / 0.03
    (tests/golden/trained, tools/train_rd.py) -> cases '*_trained', '*_trained_c0.02',
    '*_trained_c0.03'   (--only-trained)
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


SAMPLE_STRIDE = 37  # full-resolution cases keep every 37th pre-quant value (size budget)


def near_half(f: np.ndarray) -> np.ndarray:
    """Codes whose oracle x*255 lies within 1e-3 of a .5 rounding boundary (may flip +-1)."""
    v = f.astype(np.float64) * 255
    return np.abs(v - np.floor(v) - 0.5) < 1e-3


def full_resolution_cases(ref_data: str, w, manifest):
    """SURVEY §8c golden vectors (3): the whole kodim21 (512 x 768, run as one image like
    utils.py:46-62) and its six non-overlapping 256^2 tiles (config 4's tiled form).  The
    pre-quant latent is kept only at every SAMPLE_STRIDE-th value plus a packed bitmask of
    the near-.5 codes; latents and reconstructions are stored whole."""
    from PIL import Image

    kod = np.array(Image.open(os.path.join(ref_data, "kodak_img", "kodim21.png")).convert("RGB"))
    assert kod.shape == (512, 768, 3), kod.shape
    x = np.ascontiguousarray(kod[None])
    tiles = np.stack([kod[256 * ty:256 * ty + 256, 256 * tx:256 * tx + 256] for ty in range(2) for tx in range(3)])
    for name, xi in (("kodim21_full", x), ("kodim21_tiles", tiles)):
        f = O.encode_f32(w, xi)
        z = O.quantise_u8(f)
        r = O.quantise_u8(O.decode_f32(w, z))
        near = near_half(f)
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), latent=z, recon=r,
                            prequant_sample=f.ravel()[::SAMPLE_STRIDE], near_half=np.packbits(near.ravel()),
                            counts=O.histograms(z).astype(np.int32), bits=O.hist_entropy(z),
                            **({"x": x} if name == "kodim21_full" else {}))
        manifest["cases"][name] = {
            "init": "spread", "x_shape": list(xi.shape), "latent_shape": list(z.shape),
            "recon_shape": list(r.shape), "psnr_db": O.psnr(xi, r), "zero_codes": float(np.mean(z == 0)),
            "codes_near_half": int(near.sum()), "sample_stride": SAMPLE_STRIDE,
            "ms_ssim": [float(v) for v in O.ms_ssim(xi, r)],
        }
        print(name, manifest["cases"][name])


TRAINED = os.path.join(OUT, "trained")  # coef<c>_{encoder,decoder}{Y,CbCr}.safetensors
TRAINED_COEFS = ("0.01", "0.02", "0.03")


def trained_weights(coef="0.01"):
    """A codec trained by tools/train_rd.py with entropy_loss_coef `coef` (30 epochs over the
    reference's 19,000 patches, the TF encode_png target, seed 0; round 4,
    profiles/r4t0_train_rd.json), committed as safetensors."""
    pre = os.path.join(TRAINED, f"coef{coef}_")
    w = W.load(pre + "encoder", "encoder")
    w.update(W.load(pre + "decoder", "decoder"))
    return w


def trained_case_name(base, coef):
    return f"{base}_trained" + ("" if coef == "0.01" else f"_c{coef}")


def trained_cases(ref_data: str, manifest):
    """Golden vectors with trained weights (realistic activation ranges and latent statistics):
    the kodim21 crop [0:256, 0:256] and the four ImageNet patches, per trained coefficient."""
    for coef in TRAINED_COEFS:
        w = trained_weights(coef)
        manifest["weights"][f"trained_coef{coef}"] = W.digest(w)
        for name, (x, _) in load_inputs(ref_data).items():
            if name not in ("kodim21_256", "imagenet4"):
                continue
            x = np.ascontiguousarray(x, dtype=np.uint8)
            f = O.encode_f32(w, x)
            z = O.quantise_u8(f)
            rf = O.decode_f32(w, z)
            r = O.quantise_u8(rf)
            case = trained_case_name(name, coef)
            np.savez_compressed(os.path.join(OUT, f"{case}.npz"), x=x, latent=z, prequant=f, recon=r,
                                counts=O.histograms(z).astype(np.int32), bits=O.hist_entropy(z))
            manifest["cases"][case] = {
                "init": f"trained_coef{coef}", "x_shape": list(x.shape), "latent_shape": list(z.shape),
                "recon_shape": list(r.shape), "psnr_db": O.psnr(x, r), "zero_codes": float(np.mean(z == 0)),
                "bits_mean": float(O.hist_entropy(z).mean()), "codes_near_half": int(near_half(f).sum()),
                "prequant_absmax": float(np.abs(f).max()),
            }
            print(case, manifest["cases"][case])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref-data", default="/root/reference/data")
    ap.add_argument("--only-full", action="store_true", help="regenerate only the full-resolution kodim21 cases")
    ap.add_argument("--only-trained", action="store_true", help="regenerate only the trained-weight cases")
    args = ap.parse_args()
    if args.only_trained:
        with open(os.path.join(OUT, "manifest.json")) as fh:
            manifest = json.load(fh)
        trained_cases(args.ref_data, manifest)
        with open(os.path.join(OUT, "manifest.json"), "w") as fh:
            json.dump(manifest, fh, indent=1, sort_keys=True)
        return
    manifest = {"seed": 0, "oracle_acc": "float64", "weights": {}, "cases": {}}
    if args.only_full:
        with open(os.path.join(OUT, "manifest.json")) as fh:
            manifest = json.load(fh)
    wsets = {init: W.seeded_weights(0, init=init) for init in ("spread", "glorot")}
    for init, w in wsets.items():
        assert manifest["weights"].get(init, W.digest(w)) == W.digest(w), "weight generator drifted"
        manifest["weights"][init] = W.digest(w)
    full_resolution_cases(args.ref_data, wsets["spread"], manifest)
    if args.only_full:
        with open(os.path.join(OUT, "manifest.json"), "w") as fh:
            json.dump(manifest, fh, indent=1, sort_keys=True)
        return
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
        near = int(near_half(f).sum())
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

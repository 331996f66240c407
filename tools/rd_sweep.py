"""Config-4 harness run: RD points (entropy bpp, PNG bpp, PSNR, MS-SSIM) for three weight
sets on Kodak-sized (512x768) synthetic smooth images, whole-image and as 256^2 tiles.

The reference's sweep is over three *trained* models (entropy_loss_coef 0.01/0.02/0.03,
tf1_13/src/training.py:54); none ship, so the three sets here are seeded (seeds 0, 1, 2)
and the points are plumbing.  Prints one JSON line (means per set and mode, plus timing).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from neural_network_image_compression_amd import weights as W  # noqa: E402
from neural_network_image_compression_amd.rd import rd_sweep  # noqa: E402


def smooth_images(n, h, w, seed):
    rng = np.random.default_rng(seed)
    a = np.cumsum(np.cumsum(rng.integers(-2, 3, (n, h, w, 3)), axis=1), axis=2).astype(np.float64)
    a -= a.min(axis=(1, 2, 3), keepdims=True)
    a *= 255.0 / np.maximum(a.max(axis=(1, 2, 3), keepdims=True), 1)
    return a.astype(np.uint8)


def main():
    n = int(os.environ.get("RD_IMAGES", "8"))
    x = smooth_images(n, 512, 768, 0)
    sets = {f"seed{s}": W.seeded_weights(s) for s in (0, 1, 2)}
    t0 = time.perf_counter()
    res = rd_sweep(sets, x, tile=256)
    el = time.perf_counter() - t0
    out = {"config": f"config4 harness: {n} synthetic smooth 512x768 images, 3 seeded weight sets "
                     "(untrained: plumbing, not the reference's lambda sweep)", "seconds": round(el, 2), "points": {}}
    for label, modes in res.items():
        out["points"][label] = {
            mode: {k: (round(v, 6) if isinstance(v, float) else v) for k, v in d.items()
                   if k.endswith("_mean") or k in ("tile", "tile_border_psnr_delta_db")}
            for mode, d in modes.items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

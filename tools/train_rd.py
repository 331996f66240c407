"""Config-4 RD sweep with trained models: train the codec (training.py, the reference's
loss) at entropy_loss_coef 0.01 / 0.02 / 0.03 (training.py:54), then evaluate each trained
set with the device RD harness (rd.py) whole-image and as 256^2 tiles.

Data: no dataset travels to the GPU box, so training uses synthetic smooth 128^2 patches
and the evaluation synthetic smooth 512x768 images (Kodak size).  Short runs: the curve
shows the harness end to end, not the reference's converged RD numbers.

    python tools/train_rd.py [steps]
"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from neural_network_image_compression_amd import training as T  # noqa: E402
from neural_network_image_compression_amd import weights as W  # noqa: E402
from neural_network_image_compression_amd.rd import rd_sweep  # noqa: E402


def smooth_images(n, h, w, seed):
    rng = np.random.default_rng(seed)
    a = np.cumsum(np.cumsum(rng.integers(-2, 3, (n, h, w, 3)), axis=1), axis=2).astype(np.float64)
    a -= a.min(axis=(1, 2, 3), keepdims=True)
    a *= 255.0 / np.maximum(a.max(axis=(1, 2, 3), keepdims=True), 1)
    return a.astype(np.uint8)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    batch = 16
    x = smooth_images(batch * 8, 128, 128, 0)
    sets, train_log = {}, {}
    for coef in (0.01, 0.02, 0.03):
        t0 = time.perf_counter()
        with tempfile.TemporaryDirectory() as d:
            tr = T.Training(device="cuda", weights=W.seeded_weights(0), seed=0, checkpoint_dir=d + "/")
            log = []
            epochs = max(1, -(-steps * batch // len(x)))
            log = tr(x, None, max_epochs=epochs, batch_size=batch, entropy_loss_coef=coef, verbose=False)[:steps]
            tr._save()
            w = W.load(os.path.join(d, "encoder"), "encoder")
            w.update(W.load(os.path.join(d, "decoder"), "decoder"))
        label = f"coef{coef:.2f}"
        sets[label] = w
        train_log[label] = {"steps": len(log), "seconds": round(time.perf_counter() - t0, 2),
                            "first": {k: log[0][k] for k in ("ssim", "bpp", "entropy_loss")},
                            "last": {k: log[-1][k] for k in ("ssim", "bpp", "entropy_loss")}}
        print(label, json.dumps(train_log[label]), flush=True)
    ev = smooth_images(4, 512, 768, 1)
    res = rd_sweep(sets, ev, tile=256)
    out = {"config": "config4: trained at entropy_loss_coef 0.01/0.02/0.03 (short runs on synthetic 128^2 "
                     "patches), evaluated on 4 synthetic 512x768 images, whole and 256^2 tiles",
           "train": train_log, "points": {}}
    for label, modes in res.items():
        out["points"][label] = {mode: {k: (round(v, 6) if isinstance(v, float) else v) for k, v in d.items()
                                       if k.endswith("_mean") or k in ("tile", "tile_border_psnr_delta_db")}
                                for mode, d in modes.items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

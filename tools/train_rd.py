"""Config-4 RD sweep with trained models: train the codec (training.py, the reference's
Training with its loss, optimisers and per-epoch coefficient schedule) from each initial
entropy_loss_coef (SURVEY config 4: 0.01 / 0.02 / 0.03; the reference's main uses 0.01,
tf2_0/src/training.py:179), then evaluate each trained set with the device RD harness
(rd.py) on the reference's Kodak image kodim21 (768x512), whole-image and as 256^2 tiles.

Data: the reference's own training patches.  data/imagenet_patches_full (all 19,000, copied
by tools/make_train_subset.py --full; git- and gpurun-ignored except for the training call)
is used when present, one epoch = one pass, as training.py:175-179; otherwise the committed
1,000-patch subset data/imagenet_patches_1k with --epoch-samples images (default 19,000)
per epoch drawn from reshuffled passes, so the coefficient schedule keeps the reference's pace.

    python tools/train_rd.py [--epochs 30] [--batch 64] [--steps N] [--out FILE] [--save-dir DIR]
"""
import argparse
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


def load_patches(d):
    from PIL import Image
    names = sorted(f for f in os.listdir(d) if f.endswith(".jpg"))
    return np.stack([np.asarray(Image.open(os.path.join(d, f)).convert("RGB")) for f in names])


def main():
    ap = argparse.ArgumentParser()
    full = os.path.join(ROOT, "data", "imagenet_patches_full")
    ap.add_argument("--data", default=full if os.path.isdir(full) else os.path.join(ROOT, "data", "imagenet_patches_1k"))
    ap.add_argument("--epochs", type=int, default=30)  # training.py:179
    ap.add_argument("--epoch-samples", type=int, default=None,
                    help="images per epoch (default: one pass of the full set, 19,000 for the subset)")
    ap.add_argument("--save-dir", default=None, help="write each trained set as <dir>/coefX.XX_{encoder,decoder}{Y,CbCr}.safetensors")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=0, help="stop each run after this many steps (0: all epochs)")
    ap.add_argument("--coefs", default="0.01,0.02,0.03")
    ap.add_argument("--coef-step", type=float, default=0.01,
                    help="coefficient increment per epoch (training.py:165: 0.01; 0 = fixed coefficient)")
    ap.add_argument("--seeds", default="0", help="weight-init / shuffling seeds per coefficient (label suffix _sN for N > 0)")
    ap.add_argument("--png-mode", default="tf", choices=("tf", "pillow"),
                    help="the PNG encoder of the entropy net's target (get_bpp: tf.image.encode_png settings)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    x = load_patches(args.data)
    if args.epoch_samples is None:
        args.epoch_samples = len(x) if len(x) >= 19000 else 19000
    print(f"data: {len(x)} patches from {args.data}, {args.epoch_samples} images per epoch", flush=True)
    with np.load(os.path.join(ROOT, "tests", "golden", "kodim21_full.npz"), allow_pickle=False) as g:
        ev = g["x"]  # the reference's data/kodak_img/kodim21.png, (1, 512, 768, 3)
    sets, train_log = {}, {}
    runs = [(float(c), int(sd)) for c in args.coefs.split(",") for sd in args.seeds.split(",")]
    for coef, seed in runs:
        t0 = time.perf_counter()
        with tempfile.TemporaryDirectory() as d:
            tr = T.Training(device="cuda", weights=W.seeded_weights(seed, init="glorot"), seed=seed, checkpoint_dir=d + "/")
            tr.png_mode = args.png_mode
            epochs = args.epochs
            if args.steps:
                epochs = min(epochs, -(-args.steps * args.batch // args.epoch_samples))
            t1 = time.perf_counter()
            log = tr(x, None, max_epochs=epochs, batch_size=args.batch, entropy_loss_coef=coef, verbose=True,
                     epoch_samples=args.epoch_samples, coef_step=args.coef_step)
            t_train = time.perf_counter() - t1
            if args.steps:
                log = log[:args.steps]
            tr._save()
            w = W.load(os.path.join(d, "encoder"), "encoder")
            w.update(W.load(os.path.join(d, "decoder"), "decoder"))
        label = f"coef{coef:.2f}" + ("" if args.coef_step == 0.01 else f"_step{args.coef_step:g}") + (f"_s{seed}" if seed else "")
        sets[label] = w
        if args.save_dir:
            os.makedirs(args.save_dir, exist_ok=True)
            for kind in ("encoder", "decoder"):  # <dir>/<label>_encoderY.safetensors, ...
                W.save(w, os.path.join(args.save_dir, f"{label}_{kind}"), kind)
        tail = log[-20:]
        train_log[label] = {"steps": len(log), "epochs": epochs, "seed": seed, "png_mode": args.png_mode, "seconds": round(time.perf_counter() - t0, 1),
                            "train_seconds": round(t_train, 1),
                            "first": {k: log[0][k] for k in ("ssim", "bpp", "entropy_loss")},
                            "last20_mean": {k: [float(np.mean([m[k][j] for m in tail])) for j in range(3)]
                                            for k in ("ssim", "bpp")}}
        print(label, json.dumps(train_log[label]), flush=True)
    res = rd_sweep(sets, ev, tile=256)
    sched = "+0.01 per epoch, training.py:165" if args.coef_step == 0.01 else f"+{args.coef_step:g} per epoch, not the reference's +0.01"
    out = {"config": f"config4: trained from entropy_loss_coef {args.coefs} ({sched}), "
                     f"{args.epochs} epochs of {args.epoch_samples} images, batch {args.batch}, on the reference's "
                     f"ImageNet patches ({len(x)} of them); evaluated on kodim21 768x512, whole and 256^2 tiles",
           "train": train_log, "points": {}}
    for label, modes in res.items():
        out["points"][label] = {mode: {k: (round(v, 6) if isinstance(v, float) else v) for k, v in d.items()
                                       if k.endswith("_mean") or k in ("tile", "tile_border_psnr_delta_db")}
                                for mode, d in modes.items()}
    print(json.dumps(out), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

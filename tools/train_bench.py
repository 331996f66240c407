#!/usr/bin/env python
"""Training-step timing: HIP convolutions (train_hip, NHWC) vs PyTorch autograd (MIOpen).

One step = Training.losses() forward + the three autograd.grad calls of train_step
(tf2_0/src/training.py:74-151) on a batch of B synthetic 128x128 patches, Adam excluded.
The PNG-size bpp target (host threads, nic_png_sizes, training.py:12-21) is replaced by zeros
unless --png, so the device work is what is timed (it is the same host work for both backends);
with --png it overlaps the codec's backward as in Training.train_step.

    python tools/train_bench.py [--batch 64] [--size 128] [--steps 10] [--out gpurun_out/train_bench.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def conv_gflop(b, s):
    # encoder + decoder per plane at s x s (SURVEY §8d per-256^2 figures scale with area),
    # 3 planes per image; Entropynet on the 3 latents: conv 32->64 k5 s2 + 2 x conv 64->64 k3
    codec = (1.1545 + 1.6001) * (s / 256.0) ** 2 * 3 * b
    h8 = s // 8
    h16 = -(-h8 // 2)
    ent = 3 * b * 2 * h16 * h16 * 64 * (25 * 32 + 2 * 9 * 64) / 1e9
    return codec + ent  # forward; backward = 2x (input + kernel gradients)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--backends", default="hip,torch")
    ap.add_argument("--png", action="store_true", help="keep the host PNG-size target (the full step)")
    ap.add_argument("--png-threads", type=int, default=16)
    args = ap.parse_args()
    import torch

    from neural_network_image_compression_amd import training as T
    from neural_network_image_compression_amd import weights as W

    if not args.png:
        T.png_bpp_planes = lambda enc, tot, threads=None, mode=None: np.zeros(enc.shape[0], np.float32)  # device work only
    g = torch.Generator().manual_seed(0)
    imgs = torch.randint(0, 256, (args.batch, args.size, args.size, 3), generator=g, dtype=torch.uint8).cuda()
    w0 = W.seeded_weights(0, init="glorot")
    res = {"batch": args.batch, "size": args.size, "steps": args.steps,
           "conv_gflop_fwd": round(conv_gflop(args.batch, args.size), 2),
           "step": "Training.losses + autograd.grad of the three losses (no Adam"
                   + (", host PNG target)" if args.png else ", PNG target zeroed)")}
    for be in args.backends.split(","):
        tr = T.Training(device="cuda", weights=w0, seed=0, checkpoint_dir="/tmp/nic_tb/", backend=be,
                        png_threads=args.png_threads)

        def step():
            f = tr.losses(imgs, 0.01, flip=True, defer_png=True)
            torch.autograd.grad(f["loss0"], tr._variables("Y"), retain_graph=True)
            torch.autograd.grad(f["loss1"], tr._variables("CbCr"), retain_graph=True)
            torch.autograd.grad(tr.finish_entropy_loss(f), tr.entropy_model.parameters())

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        res[be] = {"ms_per_step": round(ms, 2),
                   "conv_tflops_equiv": round(3 * res["conv_gflop_fwd"] / ms, 2)}
        print(be, res[be], flush=True)
    if "hip" in res and "torch" in res:
        res["speedup_hip_vs_torch"] = round(res["torch"]["ms_per_step"] / res["hip"]["ms_per_step"], 2)
    print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

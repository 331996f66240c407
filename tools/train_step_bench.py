"""Full Training.train_step timing on the HIP backend (training.py:67-149: forward, the three
gradient tapes, the PNG-size target on host threads, and the optimiser update), with the Keras
Adam update on HIP (nic_adam_keras, default) and with torch.optim.Adam, alternately.
    python tools/train_step_bench.py [--batch 64] [--size 128] [--steps 20]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import torch

    from neural_network_image_compression_amd import training as T

    g = torch.Generator().manual_seed(3)
    imgs = torch.randint(0, 256, (args.batch, args.size, args.size, 3), generator=g, dtype=torch.uint8)
    res = {"batch": args.batch, "size": args.size, "steps": args.steps,
           "step": "Training.train_step (losses, 3 gradient tapes, PNG target on host threads, Adam)"}
    for rnd in range(2):
        for hip_adam in (True, False):
            tr = T.Training(device="cuda", seed=0, checkpoint_dir="/tmp/", backend="hip")
            tr.hip_adam = hip_adam
            tr._setup(imgs.shape[1:3])
            for _ in range(3):
                tr.train_step(imgs, 0.01)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                tr.train_step(imgs, 0.01)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / args.steps * 1e3
            res.setdefault("hip_adam" if hip_adam else "torch_adam", []).append(round(ms, 2))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

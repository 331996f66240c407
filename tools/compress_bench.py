"""Directory throughput of the reference's file-level API: Encoder.compress /
Decoder.uncompress (encoder.py:49-51, decoder.py:50-52, utils.py:30-62, 85-87) on a directory of
256^2 RGB PNG tiles cut from kodim21 (the reference's validation image; 6 tiles, flipped and
shifted into `--images` distinct ones).  Reports images/s and MP/s per driver mode (the reference's serial loop, round 4's threaded
writes, round 5's pipeline) on the kodim21 tiles and on data/imagenet_patches_1k, and whether
every mode wrote the same bytes.

Output: one JSON line.  Needs the GPU (the codec) and the built library."""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def tiles(n):
    with np.load(os.path.join(ROOT, "tests", "golden", "kodim21_full.npz"), allow_pickle=False) as g:
        x = g["x"][0]
    base = [x[y:y + 256, xx:xx + 256] for y in (0, 256) for xx in (0, 256, 512)] if x.shape[0] >= 512 else []
    if not base:
        base = [x[y:y + 256, xx:xx + 256] for y in (0, 256, 512) for xx in (0, 256)]
    out = []
    k = 0
    while len(out) < n:
        t = base[k % len(base)]
        v = k // len(base)
        t = np.roll(t, (3 * v) % 256, axis=1)
        if v & 1:
            t = t[:, ::-1]
        if v & 2:
            t = t[::-1]
        out.append(np.ascontiguousarray(t))
        k += 1
    return out


def run_modes(enc, dec, tmp, ds, ck, n, px, modes, repeat):
    """Best-of-`repeat` compress / uncompress wall time per driver mode (after a warm-up round)."""
    res, files = {}, {}
    for name, kw in modes:
        best = {}
        for r in range(repeat + 1):  # the first round warms up (HIP modules, page cache)
            for d in (os.path.basename(ds) + "_compressed", os.path.basename(ds) + "_uncompressed"):
                shutil.rmtree(os.path.join(tmp, d), ignore_errors=True)
            t0 = time.perf_counter()
            enc.compress(ds, os.path.join(ck, "encoder"), **kw)
            t1 = time.perf_counter()
            dec.uncompress(ds + "_compressed", os.path.join(ck, "decoder"), **kw)
            t2 = time.perf_counter()
            if r:
                best["compress_s"] = min(best.get("compress_s", 1e9), t1 - t0)
                best["uncompress_s"] = min(best.get("uncompress_s", 1e9), t2 - t1)
        out = {k: round(v, 4) for k, v in best.items()}
        out.update({"compress_img_s": round(n / best["compress_s"], 1), "uncompress_img_s": round(n / best["uncompress_s"], 1),
                    "compress_MP_s": round(n * px / 1e6 / best["compress_s"], 2),
                    "uncompress_MP_s": round(n * px / 1e6 / best["uncompress_s"], 2), "args": kw})
        res[name] = out
        files[name] = {d: {f: open(os.path.join(ds + d, f), "rb").read() for f in sorted(os.listdir(ds + d))}
                       for d in ("_compressed", "_uncompressed")}
    same = all(files[k] == files[modes[0][0]] for k in files)
    return res, same


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=192)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--imagenet", default=os.path.join(ROOT, "data", "imagenet_patches_1k"))
    args = ap.parse_args()
    from PIL import Image

    from neural_network_image_compression_amd import weights as W
    from neural_network_image_compression_amd.codec import Decoder, Encoder

    tmp = tempfile.mkdtemp(prefix="nic_compress_")
    try:
        ds = os.path.join(tmp, "tiles")
        os.makedirs(ds)
        for i, t in enumerate(tiles(args.images)):
            Image.fromarray(t).save(os.path.join(ds, f"t{i:05d}.png"))
        ck = os.path.join(tmp, "ck")
        w = W.seeded_weights(0, init="spread")
        W.save(w, os.path.join(ck, "encoder"), "encoder")
        W.save(w, os.path.join(ck, "decoder"), "decoder")
        enc, dec = Encoder(0), Decoder(0)
        # the reference's serial loop (utils.py:46-62: batches of 4, each saved inline), round 4's
        # default (batches of 4, PNG writes on 8 threads behind the device), round 5's pipeline
        modes = [("serial_b4", {"batch_size": 4, "workers": 0}), ("r4_b4_w8", {"batch_size": 4, "workers": 8}),
                 ("pipeline_b64", {})]
        out = {"tool": "compress_bench", "host_cpus": len(os.sched_getaffinity(0))}
        res, same = run_modes(enc, dec, tmp, ds, ck, args.images, 65536, modes, args.repeat)
        out["kodim21_tiles"] = {"images": args.images, "tile": "256x256x3 kodim21 tiles", "modes": res,
                                "files_identical_across_modes": same}
        if os.path.isdir(args.imagenet):
            inet = os.path.join(tmp, "inet")
            shutil.copytree(args.imagenet, inet)
            n = len([f for f in os.listdir(inet) if f.endswith(".jpg")])
            res, same = run_modes(enc, dec, tmp, inet, ck, n, 128 * 128, modes, args.repeat)
            out["imagenet_patches_1k"] = {"images": n, "tile": "128x128x3 JPEG patches", "modes": res,
                                          "files_identical_across_modes": same}
        print(json.dumps(out), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()

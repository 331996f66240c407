"""Directory throughput of the reference's file-level API: Encoder.compress /
Decoder.uncompress (encoder.py:49-51, decoder.py:50-52, utils.py:30-62, 85-87) on a directory of
256^2 RGB PNG tiles cut from kodim21 (the reference's validation image; 6 tiles, flipped and
shifted into `--images` distinct ones).  Reports images/s and MP/s per surface and PNG writer:

  native  -- bitstream.save_imgs: nic_png_encode on 16 host threads (Pillow-identical bytes)
  pillow  -- Pillow optimize=True per image on `--workers` Python threads (round 3's writer)

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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=192)
    ap.add_argument("--batch", type=int, default=4, help="utils.py:53 batches of 4")
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--repeat", type=int, default=2)
    args = ap.parse_args()
    from PIL import Image

    from neural_network_image_compression_amd import bitstream as B
    from neural_network_image_compression_amd import weights as W
    from neural_network_image_compression_amd.codec import Decoder, Encoder

    tmp = tempfile.mkdtemp(prefix="nic_compress_")
    try:
        ds = os.path.join(tmp, "tiles")
        os.makedirs(ds)
        for i, t in enumerate(tiles(args.images)):
            Image.fromarray(t).save(os.path.join(ds, f"t{i:05d}.png"))
        w = W.seeded_weights(0, init="spread")
        W.save(w, os.path.join(tmp, "ck", "encoder"), "encoder")
        W.save(w, os.path.join(tmp, "ck", "decoder"), "decoder")
        enc, dec = Encoder(0), Decoder(0)
        native_save = B.save_imgs

        def pillow_save(imgs, output_dir, filenames, threads=16):  # round 3's per-image Pillow writer
            paths = []
            for a, name in zip(imgs, filenames):
                p = os.path.join(output_dir, name + ".png")
                with open(p, "wb") as f:
                    f.write(B.png_bytes(np.asarray(a, np.uint8)))
                paths.append(p)
            return paths

        res = {}
        for writer, fn in (("native", native_save), ("pillow", pillow_save)):
            B.save_imgs = fn
            best = {}
            for r in range(args.repeat + 1):  # first round warms up (HIP modules, page cache)
                for d in ("tiles_compressed", "tiles_uncompressed"):
                    shutil.rmtree(os.path.join(tmp, d), ignore_errors=True)
                t0 = time.perf_counter()
                enc.compress(ds, os.path.join(tmp, "ck", "encoder"), batch_size=args.batch, workers=args.workers)
                t1 = time.perf_counter()
                dec.uncompress(os.path.join(tmp, "tiles_compressed"), os.path.join(tmp, "ck", "decoder"),
                               batch_size=args.batch, workers=args.workers)
                t2 = time.perf_counter()
                if r:
                    best["compress_s"] = min(best.get("compress_s", 1e9), t1 - t0)
                    best["uncompress_s"] = min(best.get("uncompress_s", 1e9), t2 - t1)
            n = args.images
            res[writer] = {k: round(v, 4) for k, v in best.items()}
            res[writer].update({"compress_img_s": round(n / best["compress_s"], 1),
                                "uncompress_img_s": round(n / best["uncompress_s"], 1),
                                "compress_MP_s": round(n * 65536 / 1e6 / best["compress_s"], 2),
                                "uncompress_MP_s": round(n * 65536 / 1e6 / best["uncompress_s"], 2)})
            if writer == "native":
                files = {f: open(os.path.join(tmp, "tiles_compressed", f), "rb").read()
                         for f in sorted(os.listdir(os.path.join(tmp, "tiles_compressed")))[:8]}
        B.save_imgs = native_save
        same = all(open(os.path.join(tmp, "tiles_compressed", f), "rb").read() == b for f, b in files.items())
        print(json.dumps({"tool": "compress_bench", "images": args.images, "tile": "256x256x3 kodim21 tiles",
                          "batch": args.batch, "workers": args.workers, "writers": res,
                          "native_equals_pillow_files": same}), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()

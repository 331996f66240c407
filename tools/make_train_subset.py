"""Training-data fixture for the config-4 RD sweep (tools/train_rd.py): a deterministic
subset of the reference's own training patches, data/imagenet_patches (128x128 RGB JPEGs,
the set tf2_0/src/training.py:175-177 trains on), copied byte for byte so that the
subset travels to the GPU box (the reference tree does not).  Every 19th file of the 19,000
-> 1,000 patches.

    python tools/make_train_subset.py [--full] [/root/reference/data/imagenet_patches]
"""
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DST = os.path.join(ROOT, "data", "imagenet_patches_1k")


def main():
    args = [a for a in sys.argv[1:] if a != "--full"]
    full = "--full" in sys.argv[1:]
    src = args[0] if args else "/root/reference/data/imagenet_patches"
    names = sorted(f for f in os.listdir(src) if f.endswith(".jpg"))
    # --full: all 19,000 patches into data/imagenet_patches_full (git-ignored and gpurun-ignored
    # except for the training call that reads it: 112 MB would ride along with every GPU call)
    dst = os.path.join(ROOT, "data", "imagenet_patches_full") if full else DST
    names = names if full else names[::19][:1000]
    os.makedirs(dst, exist_ok=True)
    manifest = {}
    for f in names:
        shutil.copyfile(os.path.join(src, f), os.path.join(dst, f))
        with open(os.path.join(dst, f), "rb") as fh:
            manifest[f] = hashlib.sha256(fh.read()).hexdigest()[:16]
    with open(os.path.join(dst, "manifest.json"), "w") as fh:
        json.dump({"source": "reference data/imagenet_patches, " + ("all files" if full else "every 19th file (sorted)"),
                   "files": manifest}, fh,
                  indent=0)
    print(len(names), "patches ->", dst)


if __name__ == "__main__":
    main()

"""Training-data fixture for the config-4 RD sweep (tools/train_rd.py): a deterministic
subset of the reference's own training patches, data/imagenet_patches (128x128 RGB JPEGs,
the set tf2_0/src/training.py:175-177 trains on), copied byte for byte so that the
subset travels to the GPU box (the reference tree does not).  Every 19th file of the 19,000
-> 1,000 patches.

    python tools/make_train_subset.py [/root/reference/data/imagenet_patches]
"""
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DST = os.path.join(ROOT, "data", "imagenet_patches_1k")


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/data/imagenet_patches"
    names = sorted(f for f in os.listdir(src) if f.endswith(".jpg"))[::19][:1000]
    os.makedirs(DST, exist_ok=True)
    manifest = {}
    for f in names:
        shutil.copyfile(os.path.join(src, f), os.path.join(DST, f))
        with open(os.path.join(DST, f), "rb") as fh:
            manifest[f] = hashlib.sha256(fh.read()).hexdigest()[:16]
    with open(os.path.join(DST, "manifest.json"), "w") as fh:
        json.dump({"source": "reference data/imagenet_patches, every 19th file (sorted)", "files": manifest}, fh,
                  indent=0)
    print(len(names), "patches ->", DST)


if __name__ == "__main__":
    main()

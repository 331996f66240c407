#!/bin/bash
# config-4 training sweeps on the full patch set (needs data/imagenet_patches_full in
# the upload, or data/imagenet_patches_full.tar): COEFS, SEEDS, STEP (coefficient increment per epoch), TAG
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
# the 19,000 patches travel as one tar (a directory of them overflows the upload's entry limit;
# .gpurunignore lists the tar: drop that line for a training call)
if [ ! -d data/imagenet_patches_full ] && [ -f data/imagenet_patches_full.tar ]; then
  tar xf data/imagenet_patches_full.tar -C data || exit 1
fi
timeout -k 10 ${LIMIT:-1100} python -u tools/train_rd.py --coefs "$COEFS" --seeds "$SEEDS" --coef-step "${STEP:-0.01}" \
  --out $O/${TAG}_train_rd.json > $O/${TAG}_train.log 2>&1
rc=$?; grep -v "^EPOCH" $O/${TAG}_train.log | tail -12; exit $rc

#!/bin/bash
# round 5: config-4 training sweeps on the full patch set (needs data/imagenet_patches_full in
# the upload): COEFS, SEEDS, STEP (coefficient increment per epoch), TAG
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
timeout -k 10 ${LIMIT:-1100} python -u tools/train_rd.py --coefs "$COEFS" --seeds "$SEEDS" --coef-step "${STEP:-0.01}" \
  --out $O/${TAG}_train_rd.json > $O/${TAG}_train.log 2>&1
rc=$?; grep -v "^EPOCH" $O/${TAG}_train.log | tail -12; exit $rc

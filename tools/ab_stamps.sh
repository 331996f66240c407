#!/bin/bash
# Build the stamp harness for each NIC_PIN variant and run them alternately (2 rounds).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-ab}"; mkdir -p "$OUT"
for v in ${VARIANTS:-0 1}; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNIC_STAMPS -DNIC_PIN=$v \
    -I "$ROOT/neural_network_image_compression_amd/csrc" "$ROOT/tools/stamps.cpp" -o /tmp/stamps_$v || exit 1
done
for round in 1 2; do
  for v in ${VARIANTS:-0 1}; do
    echo "== NIC_PIN=$v round $round" >> "$OUT/${TAG}_stamps.txt"
    timeout -k 10 120 /tmp/stamps_$v >> "$OUT/${TAG}_stamps.txt" 2>&1 || { echo "stamps rc=$?"; exit 1; }
  done
done
cat "$OUT/${TAG}_stamps.txt"

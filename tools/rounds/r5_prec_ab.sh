#!/bin/bash
# A/B of the split-f16 operand significands (diagnostic): the same build with weights' hi
# rounded to fewer bits (NIC_W_HI_BITS / NIC_W_LO_BITS, host repack) and a build whose
# activation hi is rounded (libnic_a8.so, -DNIC_A_HI_BITS=8), alternating on one box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r5b
mkdir -p $OUT
B="python bench.py --steps 30 --warmup 20 --no-cpu-baseline --no-host-path --no-quality --no-power-probe"
for r in 1 2; do
  for cfg in base w8 a8 aw8 w8l8; do
    case $cfg in
      base) env="" ;;
      w8) env="NIC_W_HI_BITS=8" ;;
      a8) env="NIC_LIB=$PWD/neural_network_image_compression_amd/libnic_a8.so" ;;
      aw8) env="NIC_W_HI_BITS=8 NIC_LIB=$PWD/neural_network_image_compression_amd/libnic_a8.so" ;;
      w8l8) env="NIC_W_HI_BITS=8 NIC_W_LO_BITS=8" ;;
    esac
    env $env timeout -k 10 120 $B > $OUT/${cfg}_$r.json 2> $OUT/${cfg}_$r.err || { echo "$cfg rc=$?"; exit 1; }
    python - "$OUT/${cfg}_$r.json" "$cfg" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
L = d["layers"]
print(sys.argv[2], d["value"], d["ms_per_step"], " ".join(f"{k}={v['avg_ms']}" for k, v in L.items()),
      "psnr_vs_oracle", d.get("parity", {}).get("psnr_gpu_vs_oracle_db"))
PY
  done
done

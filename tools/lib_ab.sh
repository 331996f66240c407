#!/bin/bash
# A/B of compile-time variants (libnic_*.so via NIC_LIB), alternating on one box
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r5g}
mkdir -p $OUT
B="python bench.py --steps 30 --warmup 20 --no-cpu-baseline --no-host-path --no-quality --no-power-probe --no-parity"
for r in 1 2; do
  for v in "$@"; do
    lib=$PWD/neural_network_image_compression_amd/libnic${v:+_$v}.so
    [ "$v" = base ] && lib=$PWD/neural_network_image_compression_amd/libnic.so
    NIC_LIB=$lib timeout -k 10 120 $B > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { echo "$v rc=$?"; tail -3 $OUT/${v}_$r.err; exit 1; }
    python - "$OUT/${v}_$r.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], d["value"], d["ms_per_step"], " ".join(f"{k}={v['avg_ms']}" for k, v in d["layers"].items()))
PY
  done
done

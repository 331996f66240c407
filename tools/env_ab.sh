#!/bin/bash
# A/B of env-var variants of one build, alternating on one box: each argument is
# NAME=VALUE (or "base" for no setting), e.g. TAG=x bash tools/env_ab.sh base NIC_K3P=0
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r5j}
mkdir -p $OUT
B="python bench.py --steps 30 --warmup 20 --no-cpu-baseline --no-host-path --no-quality --no-power-probe --no-parity"
for r in 1 2; do
  for v in "$@"; do
    f=$(echo "$v" | tr '=-' '_m')
    if [ "$v" = base ]; then
      timeout -k 10 120 $B > $OUT/${f}_$r.json 2> $OUT/${f}_$r.err || { echo "$v rc=$?"; tail -3 $OUT/${f}_$r.err; exit 1; }
    else
      env "$v" timeout -k 10 120 $B > $OUT/${f}_$r.json 2> $OUT/${f}_$r.err || { echo "$v rc=$?"; tail -3 $OUT/${f}_$r.err; exit 1; }
    fi
    python - "$OUT/${f}_$r.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], d["value"], d["ms_per_step"], " ".join(f"{k}={v['avg_ms']}" for k, v in d["layers"].items()))
PY
  done
done

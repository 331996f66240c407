#!/bin/bash
# round 4: the driver's bench command (--steps 20 --warmup 5) vs longer warmups, 2 rounds
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
B="--steps 20 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
for r in 1 2; do
  for w in 5 10 50; do
    timeout -k 10 200 python bench.py $B --warmup $w > $OUT/r4y_w${w}_$r.json 2>/dev/null || { echo "w$w $r failed"; exit 1; }
  done
done
python3 - <<'PY'
import json
for r in (1, 2):
    for w in (5, 10, 50):
        d=json.loads(open(f"gpurun_out/r4y_w{w}_{r}.json").read().strip().splitlines()[-1])
        L=d["layers"]
        print(f"w{w}_{r}", d["value"], d["ms_per_step"], {k: L[k].get("avg_ms") for k in ("conv2","conv4","dconv7")})
PY
echo "[done]"

#!/bin/bash
# round 4: k3 balance charge 1 vs 2 (3 alternating rounds), then the full GPU suite + smoke
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
B="--steps 30 --warmup 20 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
for r in 1 2 3; do
  for f in 2 1; do
    NIC_K3P_BAL=$f timeout -k 10 200 python bench.py $B > $OUT/r4z6_f${f}_$r.json 2>/dev/null || { echo "f$f $r failed"; exit 1; }
  done
done
python3 - <<'PY'
import json
for r in (1, 2, 3):
    for f in (2, 1):
        d=json.loads(open(f"gpurun_out/r4z6_f{f}_{r}.json").read().strip().splitlines()[-1])
        L=d["layers"]
        print(f"f{f}_{r}", d["value"], d["ms_per_step"], {k: L[k].get("avg_ms") for k in ("conv4","dconv6")})
PY
STEPS=tests,smoke bash tools/gpu_check.sh r4f6 || exit $?
echo "[done]"

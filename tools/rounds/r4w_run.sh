#!/bin/bash
# round 4: k3 pair range balancing -- host-array surface A/B (fresh process per setting) and the
# per-segment cost of the balance (NIC_K3P_BAL 2 / 3 / 4 / 0) on the bench's pair timing
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 800 python tools/host_plan_sweep.py k3bal > $OUT/r4w_host_k3bal.jsonl 2>&1 || { echo "sweep failed"; cat $OUT/r4w_host_k3bal.jsonl; exit 1; }
cat $OUT/r4w_host_k3bal.jsonl
B="--steps 30 --warmup 10 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
for r in 1 2; do
  for f in 3 2 4 0; do
    NIC_K3P_BAL=$f timeout -k 10 200 python bench.py $B > $OUT/r4w_f${f}_$r.json 2>/dev/null || { echo "f$f $r failed"; exit 1; }
  done
done
python3 - <<'PY'
import json
for r in (1, 2):
    for f in (3, 2, 4, 0):
        d=json.loads(open(f"gpurun_out/r4w_f{f}_{r}.json").read().strip().splitlines()[-1])
        L=d["layers"]
        print(f"f{f}_{r}", d["value"], d["ms_per_step"], {k: L[k].get("avg_ms") for k in ("conv4","dconv6")})
PY
echo "[done]"

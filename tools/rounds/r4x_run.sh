#!/bin/bash
# round 4: the operand dependence of the step (power-limited clock): seeded weights + random
# images (the headline workload) vs the trained codec and / or natural kodim21 crops, 2 rounds
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
B="--steps 30 --warmup 10 --no-cpu-baseline --no-power-probe --no-host-path --no-quality"
for r in 1 2; do
  for v in sr tr sn tn; do
    case $v in sr) E="";; tr) E="--weights trained";; sn) E="--images natural";; tn) E="--weights trained --images natural";; esac
    timeout -k 10 200 python bench.py $B $E > $OUT/r4x_${v}_$r.json 2> $OUT/r4x_${v}_$r.err || { echo "$v $r failed"; tail -5 $OUT/r4x_${v}_$r.err; exit 1; }
  done
done
python3 - <<'PY'
import json
for r in (1, 2):
    for v in ("sr", "tr", "sn", "tn"):
        d=json.loads(open(f"gpurun_out/r4x_{v}_{r}.json").read().strip().splitlines()[-1])
        L=d["layers"]
        print(f"{v}_{r}", d["value"], d["ms_per_step"], d["data"], d["config"]["weights"][:20], d.get("parity"), {k: L[k].get("avg_ms") for k in L})
PY
echo "[done]"

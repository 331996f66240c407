#!/bin/bash
# round 4: dconv1_all with one block group over both models (default) vs per-model groups
# (NIC_D1M=0) -- decode / dconv1 / surface tests, then 3 alternating bench rounds
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "golden or alternative or decode or surface or trip or trained" > $OUT/r4z7_tests.log 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -3 $OUT/r4z7_tests.log
[ $rc -eq 0 ] || exit $rc
B="--steps 30 --warmup 20 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
for r in 1 2 3; do
  for m in 1 0; do
    NIC_D1M=$m timeout -k 10 200 python bench.py $B > $OUT/r4z7_m${m}_$r.json 2>/dev/null || { echo "m$m $r failed"; exit 1; }
  done
done
python3 - <<'PY'
import json
for r in (1, 2, 3):
    for m in (1, 0):
        d=json.loads(open(f"gpurun_out/r4z7_m{m}_{r}.json").read().strip().splitlines()[-1])
        L=d["layers"]
        print(f"m{m}_{r}", d["value"], d["ms_per_step"], {k: L[k].get("avg_ms") for k in ("dconv1",)})
PY
echo "[done]"

#!/bin/bash
# round 4: fused k3 pair with step-balanced block row ranges (default, NIC_K3P_BAL=3) vs the
# equal-rows split (NIC_K3P_BAL=0) -- tests, interleaved bench A/B with the host-array path, 4K
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "golden or alternative or k3 or encode or decode or surface or trip or trained" > $OUT/r4v_tests.log 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -3 $OUT/r4v_tests.log
[ $rc -eq 0 ] || exit $rc
B="--steps 30 --warmup 10 --no-cpu-baseline --no-parity --no-power-probe --no-quality"
for r in 1 2 3; do
  timeout -k 10 200 python bench.py $B > $OUT/r4v_b3_$r.json 2>/dev/null || { echo "b3 $r failed"; exit 1; }
  NIC_K3P_BAL=0 timeout -k 10 200 python bench.py $B > $OUT/r4v_b0_$r.json 2>/dev/null || { echo "b0 $r failed"; exit 1; }
done
B4="--workload 4k --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
timeout -k 10 300 python bench.py $B4 > $OUT/r4v_4k_b3.json 2>/dev/null || exit 1
NIC_K3P_BAL=0 timeout -k 10 300 python bench.py $B4 > $OUT/r4v_4k_b0.json 2>/dev/null || exit 1
python3 - <<'PY'
import json
for t in ("b3_1","b0_1","b3_2","b0_2","b3_3","b0_3","4k_b3","4k_b0"):
    d=json.loads(open(f"gpurun_out/r4v_{t}.json").read().strip().splitlines()[-1])
    L=d["layers"]; hp=d.get("pcie_inclusive") or {}
    print(t, d["value"], d["ms_per_step"], {k: L[k].get("avg_ms") for k in ("conv4","dconv6") if k in L}, hp.get("mp_per_s"), hp.get("ms_per_batch"))
PY
echo "[done]"

#!/bin/bash
# round 4: k3 pair with conv_b's MFMA stream at priority 2 (NIC_K3P_PRIO=1) vs both at 1 -- tests + A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "golden or alternative or k3 or encode" > gpurun_out/r4r_tests.log 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -3 gpurun_out/r4r_tests.log
[ $rc -eq 0 ] || exit $rc
B="--steps 30 --warmup 10 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
for r in 1 2 3; do
  timeout -k 10 200 python bench.py $B > gpurun_out/r4r_p1_$r.json 2>/dev/null || { echo "p1 $r failed"; exit 1; }
  NIC_LIB=$PWD/ab/libnic_prio0.so timeout -k 10 200 python bench.py $B > gpurun_out/r4r_p0_$r.json 2>/dev/null || { echo "p0 $r failed"; exit 1; }
done
python3 - <<'PY'
import json
for t in ("p1_1","p0_1","p1_2","p0_2","p1_3","p0_3"):
    d=json.loads(open(f"gpurun_out/r4r_{t}.json").read().strip().splitlines()[-1])
    L=d["layers"]
    print(t, d["value"], d["ms_per_step"], {k: L[k].get("avg_ms") for k in ("conv2","conv4","dconv6","dconv7") if k in L})
PY

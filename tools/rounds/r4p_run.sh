#!/bin/bash
# round 4: conv12 with conv1 shares in half-tile units (NIC_C12_U0=5) vs whole tiles (U0=0 build) -- tests + A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "encode or golden or range_guard or kodim21 or alternative" > gpurun_out/r4p_tests.log 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -3 gpurun_out/r4p_tests.log
[ $rc -eq 0 ] || exit $rc
B="--steps 30 --warmup 10 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
for r in 1 2 3; do
  timeout -k 10 200 python bench.py $B > gpurun_out/r4p_u5_$r.json 2>/dev/null || { echo "u5 $r failed"; exit 1; }
  NIC_LIB=$PWD/ab/libnic_c12u0.so timeout -k 10 200 python bench.py $B > gpurun_out/r4p_u0_$r.json 2>/dev/null || { echo "u0 $r failed"; exit 1; }
done
B4="--workload 4k --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
timeout -k 10 300 python bench.py $B4 > gpurun_out/r4p_4k_u5.json 2>/dev/null || { echo "4k e3 failed"; exit 1; }
NIC_LIB=$PWD/ab/libnic_c12u0.so timeout -k 10 300 python bench.py $B4 > gpurun_out/r4p_4k_u0.json 2>/dev/null || { echo "4k e0 failed"; exit 1; }
python3 - <<'PY'
import json
for t in ("u5_1","u0_1","u5_2","u0_2","u5_3","u0_3","4k_u5","4k_u0"):
    d=json.loads(open(f"gpurun_out/r4p_{t}.json").read().strip().splitlines()[-1])
    L=d["layers"]
    print(t, d["value"], d["ms_per_step"], {k: L[k].get("avg_ms") for k in ("conv2","conv8") if k in L})
PY

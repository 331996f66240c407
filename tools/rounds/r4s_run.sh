#!/bin/bash
# round 4: conv8 (tap-split) stream priorities, last tap group at 2 (NIC_WS2_PRIO=1) vs none -- tests + A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "golden or encode or entropy" > gpurun_out/r4s_tests.log 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -3 gpurun_out/r4s_tests.log
[ $rc -eq 0 ] || exit $rc
B="--steps 30 --warmup 10 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
for r in 1 2 3; do
  timeout -k 10 200 python bench.py $B > gpurun_out/r4s_w1_$r.json 2>/dev/null || { echo "w1 $r failed"; exit 1; }
  NIC_LIB=$PWD/ab/libnic_ws2p0.so timeout -k 10 200 python bench.py $B > gpurun_out/r4s_w0_$r.json 2>/dev/null || { echo "w0 $r failed"; exit 1; }
done
python3 - <<'PY'
import json
for t in ("w1_1","w0_1","w1_2","w0_2","w1_3","w0_3"):
    d=json.loads(open(f"gpurun_out/r4s_{t}.json").read().strip().splitlines()[-1])
    L=d["layers"]
    print(t, d["value"], d["ms_per_step"], {k: L[k].get("avg_ms") for k in ("conv2","conv8","conv4","dconv7") if k in L})
PY
B4="--workload 4k --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
timeout -k 10 300 python bench.py $B4 > gpurun_out/r4s_4k_w1.json 2>/dev/null || exit 1
NIC_LIB=$PWD/ab/libnic_ws2p0.so timeout -k 10 300 python bench.py $B4 > gpurun_out/r4s_4k_w0.json 2>/dev/null || exit 1
python3 - <<'PY'
import json
for t in ("4k_w1","4k_w0"):
    d=json.loads(open(f"gpurun_out/r4s_{t}.json").read().strip().splitlines()[-1])
    print(t, d["value"], d["ms_per_step"], {k: v.get("avg_ms") for k, v in d["layers"].items()})
PY

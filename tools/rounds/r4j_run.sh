#!/bin/bash
# round 4: dconv1 code prefetch depth A/B (config 2), conv8 XCD-range walk A/B (4K, no fold)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "decode or dconv1 or encode_entropy" > gpurun_out/r4j_tests.log 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -3 gpurun_out/r4j_tests.log
[ $rc -eq 0 ] || exit $rc
B="--steps 30 --warmup 10 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
for r in 1 2 3; do
  timeout -k 10 200 python bench.py $B > gpurun_out/r4j_pf2_$r.json 2>/dev/null || { echo "pf2 $r failed"; exit 1; }
  NIC_LIB=$PWD/ab/libnic_d1pf1.so timeout -k 10 200 python bench.py $B > gpurun_out/r4j_pf1_$r.json 2>/dev/null || { echo "pf1 $r failed"; exit 1; }
done
B4="--workload 4k --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
for r in 1 2; do
  NIC_BENCH_HIST=sep timeout -k 10 300 python bench.py $B4 > gpurun_out/r4j_4k_def_$r.json 2>/dev/null || { echo "4k def failed"; exit 1; }
  NIC_BENCH_HIST=sep NIC_C8W=x timeout -k 10 300 python bench.py $B4 > gpurun_out/r4j_4k_xr_$r.json 2>/dev/null || { echo "4k xr failed"; exit 1; }
done
python3 - <<'PY'
import json
for t in ("pf2_1","pf1_1","pf2_2","pf1_2","pf2_3","pf1_3","4k_def_1","4k_xr_1","4k_def_2","4k_xr_2"):
    d=json.loads(open(f"gpurun_out/r4j_{t}.json").read().strip().splitlines()[-1])
    L=d["layers"]
    print(t, d["value"], d["ms_per_step"], {k: L[k].get("avg_ms") for k in ("conv8","dconv1") if k in L})
PY

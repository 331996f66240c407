#!/bin/bash
# round 4: fold with device-scope atomics into per-plane counts -- tests, 4K A/B, 4K kernel summary
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "encode_entropy or entropy or range_guard" > gpurun_out/r4q_tests.log 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -3 gpurun_out/r4q_tests.log
[ $rc -eq 0 ] || exit $rc
B="--workload 4k --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
for r in 1 2 3; do
  timeout -k 10 300 python bench.py $B > gpurun_out/r4q_4k_fold_$r.json 2>/dev/null || { echo "fold $r failed"; exit 1; }
  NIC_BENCH_HIST=sep timeout -k 10 300 python bench.py $B > gpurun_out/r4q_4k_sep_$r.json 2>/dev/null || { echo "sep $r failed"; exit 1; }
done
python3 - <<'PY'
import json
for t in ("fold_1","sep_1","fold_2","sep_2","fold_3","sep_3"):
    d=json.loads(open(f"gpurun_out/r4q_4k_{t}.json").read().strip().splitlines()[-1])
    print(t, d["value"], d["ms_per_step"], {k: v.get("avg_ms") for k, v in d["layers"].items()})
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4q_4kprof -o k \
  -- python3 bench.py $B > gpurun_out/r4q_4kprof.log 2>&1; echo "[prof] rc=$?"
find gpurun_out/r4q_4kprof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150 | head -8

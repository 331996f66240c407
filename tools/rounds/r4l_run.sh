#!/bin/bash
# round 4: histogram fold (counting on the ts = 1 waves): tests + 4K A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "encode_entropy or entropy" > gpurun_out/r4l_tests.log 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -4 gpurun_out/r4l_tests.log
[ $rc -eq 0 ] || exit $rc
B="--workload 4k --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
for r in 1 2 3; do
  timeout -k 10 300 python bench.py $B > gpurun_out/r4l_4k_fold_$r.json 2> gpurun_out/r4l_4k_fold_$r.err || { echo "fold $r failed"; tail -3 gpurun_out/r4l_4k_fold_$r.err; exit 1; }
  NIC_BENCH_HIST=sep timeout -k 10 300 python bench.py $B > gpurun_out/r4l_4k_sep_$r.json 2> gpurun_out/r4l_4k_sep_$r.err || { echo "sep $r failed"; exit 1; }
done
python3 - <<'PY'
import json
for t in ("fold_1","sep_1","fold_2","sep_2","fold_3","sep_3"):
    d=json.loads(open(f"gpurun_out/r4l_4k_{t}.json").read().strip().splitlines()[-1])
    print(t, d["value"], d["ms_per_step"], {k: v.get("avg_ms") for k, v in d["layers"].items()})
PY

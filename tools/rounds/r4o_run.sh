#!/bin/bash
# round 4: host pipeline with two compute streams / pass slots -- tests + A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "numpy_surface or range_guard or barrier_timeout or compress" > gpurun_out/r4o_tests.log 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -3 gpurun_out/r4o_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python tools/host_plan_sweep.py 1 > gpurun_out/r4o_two_$r.jsonl 2>&1 || { echo "two failed"; exit 1; }
  NIC_HOST_SLOTS=1 timeout -k 10 200 python tools/host_plan_sweep.py 1 > gpurun_out/r4o_one_$r.jsonl 2>&1 || { echo "one failed"; exit 1; }
done
for f in two_1 one_1 two_2 one_2; do echo "$f $(cat gpurun_out/r4o_$f.jsonl)"; done

#!/bin/bash
# round 4: full GPU suite + default bench on the new defaults
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r4e_tests.log 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -3 gpurun_out/r4e_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r4e_bench.json 2> gpurun_out/r4e_bench.err; rc=$?
echo "[bench] rc=$rc"; cat gpurun_out/r4e_bench.json
exit $rc

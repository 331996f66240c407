#!/bin/bash
# round 4 final build: full GPU suite, smoke, headline bench, kernel summary
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
STEPS=tests,smoke,bench,prof bash tools/gpu_check.sh r4f7 || exit $?
timeout -k 10 300 python bench.py --workload 4k --steps 20 --warmup 10 > gpurun_out/r4f7_4k_bench.json 2> gpurun_out/r4f7_4k.err; echo "[4k] rc=$?"

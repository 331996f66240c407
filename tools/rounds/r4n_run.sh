#!/bin/bash
# round 4: stamp harnesses of the k3 pair (random / zero weights) and conv12 on the current build
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 120 ./ab/k3p_stamps > gpurun_out/r4n_k3p_stamps.txt 2>&1; echo "[k3p] rc=$?"; cat gpurun_out/r4n_k3p_stamps.txt
timeout -k 10 120 ./ab/k3p_stamps zero > gpurun_out/r4n_k3p_stamps_zero.txt 2>&1; echo "[k3p zero] rc=$?"; cat gpurun_out/r4n_k3p_stamps_zero.txt
timeout -k 10 120 ./ab/c12_stamps > gpurun_out/r4n_c12_stamps.txt 2>&1; echo "[c12] rc=$?"; cat gpurun_out/r4n_c12_stamps.txt
bash tools/r4o_run.sh

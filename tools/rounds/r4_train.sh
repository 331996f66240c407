# round 4: config-4 training runs on the GPU box (TF encode_png target, seeds), RD-evaluated
# usage: bash tools/r4_train.sh <coefs> <seeds> <tag>
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1150 python -u tools/train_rd.py --coefs "$1" --seeds "$2" --png-mode tf \
  --save-dir gpurun_out/trained_$3 --out gpurun_out/$3_train_rd.json > gpurun_out/$3_train.log 2>&1
rc=$?; tail -4 gpurun_out/$3_train.log | cut -c1-2000; echo "[train] rc=$rc"; exit $rc

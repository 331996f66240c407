set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
STEPS=tests,smoke,bench,prof bash tools/gpu_check.sh r4b || exit $?
timeout -k 10 300 python tools/compress_bench.py --images 192 > gpurun_out/r4b_compress.json 2> gpurun_out/r4b_compress.err
echo "[compress] rc=$?"; cat gpurun_out/r4b_compress.json; tail -3 gpurun_out/r4b_compress.err

# round 4: first GPU run of the Winograd k3 pair -- focused parity, then the bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "golden or wino or k3 or full_size or random_shapes or batch_inv or barrier or range_guard" > gpurun_out/r4c_pytest.log 2>&1
rc=$?; tail -30 gpurun_out/r4c_pytest.log; echo "[pytest] rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-power-probe > gpurun_out/r4c_bench.json 2> gpurun_out/r4c_bench.err
rc=$?; cat gpurun_out/r4c_bench.json; tail -5 gpurun_out/r4c_bench.err; echo "[bench] rc=$rc"
[ $rc -ne 0 ] && exit $rc
NIC_K3P=d timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-power-probe --no-parity > gpurun_out/r4c_bench_direct.json 2> gpurun_out/r4c_bench_direct.err
rc=$?; cat gpurun_out/r4c_bench_direct.json; echo "[bench-direct] rc=$rc"
exit 0

# round 4: Winograd k3 pair + all-phase dconv1 -- focused parity, then benches (A/B)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "golden or wino or k3 or full_size or random_shapes or batch_inv or barrier or dconv1" > gpurun_out/r4c_pytest.log 2>&1
rc=$?; tail -15 gpurun_out/r4c_pytest.log; echo "[pytest] rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="--steps 20 --warmup 10 --no-cpu-baseline --no-power-probe --no-parity --no-host-path --no-quality"
timeout -k 10 200 python bench.py $B > gpurun_out/r4c_bench.json 2> gpurun_out/r4c_bench.err
rc=$?; echo "[bench] rc=$rc"; [ $rc -ne 0 ] && exit $rc
NIC_K3P=d timeout -k 10 200 python bench.py $B > gpurun_out/r4c_bench_direct.json 2> gpurun_out/r4c_bench_direct.err; echo "[direct] rc=$?"
NIC_LIB=$PWD/ab/libnic_il0.so timeout -k 10 200 python bench.py $B > gpurun_out/r4c_bench_il0.json 2> gpurun_out/r4c_bench_il0.err; echo "[il0] rc=$?"
NIC_D1=a timeout -k 10 200 python bench.py $B > gpurun_out/r4c_bench_d1a.json 2> gpurun_out/r4c_bench_d1a.err; echo "[d1a] rc=$?"
timeout -k 10 200 python bench.py $B > gpurun_out/r4c_bench2.json 2> gpurun_out/r4c_bench2.err; echo "[bench2] rc=$?"
python3 - <<'PY'
import json
for f in ("r4c_bench","r4c_bench_direct","r4c_bench_il0","r4c_bench_d1a","r4c_bench2"):
    try:
        d=json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
        print(f, d["value"], d["ms_per_step"], {k: v.get("avg_ms") for k, v in d["layers"].items()})
    except Exception as e:
        print(f, "ERR", e)
PY

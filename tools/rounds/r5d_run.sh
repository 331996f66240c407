#!/bin/bash
# round 5: directory-driver pipeline (test + throughput) and the host-surface box rates
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "compress" -p no:cacheprovider > $O/r5d_pytest.log 2>&1
rc=$?; tail -3 $O/r5d_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/compress_bench.py > $O/r5d_compress_bench.json 2> $O/r5d_compress_bench.err
rc=$?; cat $O/r5d_compress_bench.json; [ $rc -eq 0 ] || { tail -5 $O/r5d_compress_bench.err; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/r5d_bench.json 2> $O/r5d_bench.err
rc=$?; python -c "import json; d=json.load(open('$O/r5d_bench.json')); print(d['value'], d['pcie_inclusive'])"; exit $rc

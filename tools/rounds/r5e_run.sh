#!/bin/bash
# round 5: pre-summed dconv8 projections (GPU suite), directory-driver pipeline, bench + host box rates
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r5e_pytest_gpu.log 2>&1
rc=$?; tail -4 $O/r5e_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 10 > $O/r5e_bench.json 2> $O/r5e_bench.err
rc=$?; python -c "
import json; d=json.load(open('$O/r5e_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])
print({k: v['avg_ms'] for k, v in d['layers'].items()}); print(d['pcie_inclusive']); print(d['parity'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python tools/compress_bench.py > $O/r5e_compress_bench.json 2> $O/r5e_compress_bench.err
rc=$?; cat $O/r5e_compress_bench.json; [ $rc -eq 0 ] || { tail -5 $O/r5e_compress_bench.err; exit $rc; }

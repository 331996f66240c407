#!/bin/bash
# round 5: pre-summed projections, structured form (GPU suite + bench)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
T=${1:-r5f}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/${T}_pytest_gpu.log 2>&1
rc=$?; tail -4 $O/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-host-path --no-quality > $O/${T}_bench_$k.json 2> $O/${T}_bench_$k.err
rc=$?; python -c "
import json; d=json.load(open('$O/${T}_bench_$k.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])
print({k: v['avg_ms'] for k, v in d['layers'].items()}); print(d['parity'])"; [ $rc -eq 0 ] || exit $rc
done

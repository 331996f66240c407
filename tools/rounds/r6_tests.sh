#!/bin/bash
# round 6: a subset of the GPU tests (pytest -k expression $2), then optionally the bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=$1; K=$2
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -k "$K" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/${T}_pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/${T}_pytest.log | tail -40; [ $rc -eq 0 ] || exit $rc
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-host-path --no-quality > $O/${T}_bench.json 2> $O/${T}_bench.err
  rc=$?; python3 -c "
import json; d=json.load(open('$O/${T}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])
print({k: v['avg_ms'] for k, v in d['layers'].items()}); print(d.get('parity'))"; exit $rc
fi

#!/bin/bash
# round 6: rocprofv3 kernel stats of the training step, current tree vs r6_old/ (the tree before
# the fused activation), one process each
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r6y_tp_new -o k -- \
  python3 tools/train_step_bench.py --steps 10 > $O/r6y_tp_new.log 2>&1 || { echo "new rc=$?"; exit 1; }
cd r6_old
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r6y_tp_old -o k -- \
  python3 tools/train_step_bench.py --steps 10 > $O/r6y_tp_old.log 2>&1 || { echo "old rc=$?"; exit 1; }
cd ..
for v in new old; do
  echo "== $v"
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print('total ms', round(tot/1e6,2), 'calls', sum(int(r['Calls']) for r in rows))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print(f\"  {r['Name'][:70]:70s} {int(r['Calls']):6d} {float(r['TotalDurationNs'])/1e6:8.2f} ms\")" $O/r6y_tp_$v/k_kernel_stats.csv
done

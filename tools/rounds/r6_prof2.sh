#!/bin/bash
# round 6: rocprofv3 kernel stats of a short config-2 bench under each library build
# usage: bash tools/rounds/r6_prof2.sh TAG v1 v2 ...   (v = base | suffix of libnic_<v>.so)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
export TMPDIR=/tmp
for v in "$@"; do
  lib=$PWD/neural_network_image_compression_amd/libnic_$v.so
  [ "$v" = base ] && lib=$PWD/neural_network_image_compression_amd/libnic.so
  NIC_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_$v -o run -- \
    python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-host-path --no-quality --no-power-probe --no-parity \
    > gpurun_out/${TAG}_prof_$v.log 2>&1 || { echo "$v rc=$?"; tail -5 gpurun_out/${TAG}_prof_$v.log; exit 1; }
  f=$(ls gpurun_out/${TAG}_prof_$v/*/run_kernel_stats.csv 2>/dev/null | head -n 1)
  [ -n "$f" ] || f=$(ls gpurun_out/${TAG}_prof_$v/run_kernel_stats.csv)
  echo "== $v"; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f\"{r['Name'][:60]:60s} {int(r['Calls']):6d} {float(r['AverageNs'])/1000:9.2f} us\")" "$f"
done

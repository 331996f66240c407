#!/bin/bash
# round 4: host-surface plan sweep (copy pool), compress()/uncompress() throughput + rocprof stats
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python tools/host_plan_sweep.py > gpurun_out/r4g_host_sweep.jsonl 2> gpurun_out/r4g_host_sweep.err || { echo "sweep failed"; tail -5 gpurun_out/r4g_host_sweep.err; exit 1; }
cat gpurun_out/r4g_host_sweep.jsonl
timeout -k 10 300 python tools/compress_bench.py --images 192 > gpurun_out/r4g_compress.json 2> gpurun_out/r4g_compress.err || { echo "compress failed"; tail -5 gpurun_out/r4g_compress.err; exit 1; }
cat gpurun_out/r4g_compress.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4g_cprof -o cp -- python3 tools/compress_bench.py --images 96 --repeat 1 > gpurun_out/r4g_cprof.log 2>&1 || { echo "compress prof failed"; tail -5 gpurun_out/r4g_cprof.log; exit 1; }
find gpurun_out/r4g_cprof -name "*kernel_stats.csv" | head -3

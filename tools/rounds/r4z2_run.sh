#!/bin/bash
# round 4 evidence, part 2: PMC passes (traffic, instruction mix), config 4 / config 5 benches,
# the 4K kernel summary, compress()/uncompress() throughput + its kernel summary
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=r4z
stop_on() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "[$2] stopping"; exit "$1"; fi; }
bash tools/pmc.sh "$TAG" || exit $?
python3 tools/pmc_summary.py "$OUT/${TAG}_pmc" > "$OUT/${TAG}_traffic.json" 2> /dev/null
timeout -k 10 300 python bench.py --workload kodak --steps 20 --warmup 10 --no-power-probe > "$OUT/${TAG}_kodak_bench.json" 2> "$OUT/${TAG}_kodak.err"
stop_on $? kodak
timeout -k 10 300 python bench.py --workload 4k --steps 20 --warmup 10 > "$OUT/${TAG}_4k_bench.json" 2> "$OUT/${TAG}_4k.err"
stop_on $? 4k
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_4kprof" -o k \
  -- python3 "$ROOT/bench.py" --workload 4k --steps 20 --warmup 10 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality > "$OUT/${TAG}_4kprof.log" 2>&1
stop_on $? 4kprof
timeout -k 10 300 python tools/compress_bench.py --images 192 > "$OUT/${TAG}_compress.json" 2> "$OUT/${TAG}_compress.err"
stop_on $? compress
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_cprof" -o c \
  -- python3 "$ROOT/tools/compress_bench.py" --images 96 --repeat 1 > "$OUT/${TAG}_cprof.log" 2>&1
stop_on $? cprof
cat "$OUT/${TAG}_kodak_bench.json" | cut -c1-300; cat "$OUT/${TAG}_4k_bench.json" | cut -c1-300; cat "$OUT/${TAG}_compress.json"
B="--steps 20 --warmup 10 --no-cpu-baseline --no-parity --no-power-probe --no-quality"
for r in 1 2; do
  timeout -k 10 200 python bench.py $B > "$OUT/${TAG}_host_pool_$r.json" 2>/dev/null || exit 1
  NIC_HOST_COPY_THREADS=0 timeout -k 10 200 python bench.py $B > "$OUT/${TAG}_host_nopool_$r.json" 2>/dev/null || exit 1
done
python3 - <<'PY'
import json
for t in ("pool_1","nopool_1","pool_2","nopool_2"):
    d=json.loads(open(f"gpurun_out/r4z_host_{t}.json").read().strip().splitlines()[-1])
    print(t, d["value"], d["pcie_inclusive"]["mp_per_s"], d["pcie_inclusive"]["ms_per_batch"])
PY
echo "[done]"

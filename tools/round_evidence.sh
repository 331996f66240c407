#!/bin/bash
# Evidence for one build on one GPU box: GPU tests, smoke, the headline bench (with CPU
# baseline), a rocprofv3 kernel-trace summary of the same command, PMC passes (HBM bytes,
# instruction mix, MFMA busy), and the config-4 / config-5 benches (+ the 4K kernel summary).
# Every GPU step has its own time limit; an abnormal exit ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="${1:-ev}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_on() {
  echo "[$2] rc=$1"
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "[$2] abnormal exit: stopping"; exit "$1"; fi
}
STEPS=tests,smoke,bench,prof bash tools/gpu_check.sh "$TAG" || exit $?
bash tools/pmc.sh "$TAG" || exit $?
timeout -k 10 300 python bench.py --workload kodak --steps 20 --warmup 10 --no-power-probe > "$OUT/${TAG}_kodak_bench.json" 2> "$OUT/${TAG}_kodak.err"
stop_on $? kodak
timeout -k 10 300 python bench.py --workload 4k --steps 20 --warmup 10 > "$OUT/${TAG}_4k_bench.json" 2> "$OUT/${TAG}_4k.err"
stop_on $? 4k
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_4kprof" -o k \
  -- python3 "$ROOT/bench.py" --workload 4k --steps 20 --warmup 10 > "$OUT/${TAG}_4kprof.log" 2>&1
stop_on $? 4kprof
python3 tools/pmc_summary.py "$OUT/${TAG}_pmc" > "$OUT/${TAG}_traffic.json" 2> /dev/null
echo "[done]"

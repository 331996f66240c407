#!/bin/bash
# One GPU-box session: gpu tests -> smoke -> bench -> rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash / fault / timeout ends the script
# (pytest rc 1 = failed assertions only, which still lets the bench run).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
TAG="${1:-run}"
STEPS="${STEPS:-all}"

stop_on() {  # $1 = rc, $2 = step name
  local rc=$1
  echo "[$2] rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "[$2] abnormal exit: stopping"; exit "$rc"; fi
}

if [[ "$STEPS" == all || "$STEPS" == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 --timeout-method thread > "$OUT/${TAG}_pytest_gpu.log" 2>&1
  rc=$?; tail -40 "$OUT/${TAG}_pytest_gpu.log"; stop_on $rc pytest
fi
if [[ "$STEPS" == all || "$STEPS" == *smoke* ]]; then
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1
  rc=$?; tail -5 "$OUT/${TAG}_smoke.log"; stop_on $rc smoke
fi
if [[ "$STEPS" == all || "$STEPS" == *bench* ]]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 10 > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
  rc=$?; cat "$OUT/${TAG}_bench.json"; tail -5 "$OUT/${TAG}_bench.err"; stop_on $rc bench
fi
if [[ "$STEPS" == all || "$STEPS" == *prof* ]]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof" -o kt \
    -- python3 "$ROOT/bench.py" --steps 20 --warmup 10 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality > "$OUT/${TAG}_prof.log" 2>&1
  rc=$?; tail -3 "$OUT/${TAG}_prof.log"; stop_on $rc rocprof
  find "$OUT/${TAG}_prof" -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-220
fi
exit 0

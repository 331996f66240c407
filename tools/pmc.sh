#!/bin/bash
# rocprofv3 PMC passes over a short bench run (one counter group per pass, --kernel-trace
# only beside --pmc, as the pool requires).  Output CSVs land in gpurun_out/<tag>_pmc/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
TAG="${1:-pmc}"
mkdir -p "$OUT/${TAG}_pmc"
export TMPDIR=/tmp
BENCH=(python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality)
if [ "${LIST:-0}" = 1 ]; then
  timeout -k 10 120 rocprofv3 -L > "$OUT/${TAG}_pmc/counters.txt" 2>&1
  echo "[list] rc=$?"
fi
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/${TAG}_pmc/p$i" -o pmc -- "${BENCH[@]}" \
    > "$OUT/${TAG}_pmc/p$i.log" 2>&1
  rc=$?
  echo "[pass $i: $group] rc=$rc"
  if [ $rc -ge 124 ]; then echo "abnormal exit: stopping"; exit $rc; fi
done <<GROUPS
${PMC_GROUPS:-FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
TCC_HIT_sum TCC_MISS_sum}
GROUPS
exit 0

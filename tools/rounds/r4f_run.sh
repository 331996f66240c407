#!/bin/bash
# round 4: XCD-remap A/B (NIC_WSX), PMC traffic, host-surface probe + timeline
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 30 --warmup 10 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
for r in 1 2; do
  timeout -k 10 200 python bench.py $B > gpurun_out/r4f_x1_$r.json 2> gpurun_out/r4f_x1_$r.err || { echo "x1 $r failed"; exit 1; }
  NIC_WSX=0 timeout -k 10 200 python bench.py $B > gpurun_out/r4f_x0_$r.json 2> gpurun_out/r4f_x0_$r.err || { echo "x0 $r failed"; exit 1; }
done
python3 - <<'PY'
import json
for t in ("x1_1","x0_1","x1_2","x0_2"):
    d=json.loads(open(f"gpurun_out/r4f_{t}.json").read().strip().splitlines()[-1])
    print(t, d["value"], {k: v["avg_ms"] for k, v in d["layers"].items()})
PY
PMC_GROUPS="FETCH_SIZE
WRITE_SIZE" bash tools/pmc.sh r4f || exit $?
python3 tools/pmc_summary.py gpurun_out/r4f_pmc > gpurun_out/r4f_summary.json 2>&1
python3 - <<'PY'
import json
d=json.load(open("gpurun_out/r4f_summary.json"))
print({k: v.get("hbm_bytes_per_launch") for k, v in d["layers"].items()})
PY
timeout -k 10 300 python tools/pcie_probe.py > gpurun_out/r4f_pcie_probe.json 2> gpurun_out/r4f_pcie_probe.err || { echo "probe failed"; exit 1; }
cat gpurun_out/r4f_pcie_probe.json
timeout -k 10 300 rocprofv3 --sys-trace -d gpurun_out/r4f_trace -o ht -- python3 tools/host_trace.py > gpurun_out/r4f_trace.log 2>&1 || { echo "trace failed"; exit 1; }
python3 tools/host_timeline.py gpurun_out/r4f_trace > gpurun_out/r4f_timeline.txt 2>&1
tail -60 gpurun_out/r4f_timeline.txt
